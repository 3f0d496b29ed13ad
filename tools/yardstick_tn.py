"""Yardstick for the weight-gradient (TN) GEMMs: mmseq_gemm_wgrad (fp32 accumulate + fused bias
gradient) vs torch.matmul(dY^T, X) (hipBLASLt, bf16 out) at the config-3 joint shapes (K = R rows).
HIP-event time per call; one JSON line per shape. Measurement only."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_sequencing_amd import _native as N  # noqa: E402
from yardstick import timed  # noqa: E402
if os.environ.get("MMSEQ_BENCH_LIB"):  # A/B of library builds (tools/gpu_run.sh lib-ab)
    N.LIB_PATH = os.environ["MMSEQ_BENCH_LIB"]

R = int(sys.argv[1]) if len(sys.argv) > 1 else 640 * 513
g = torch.Generator(device="cuda").manual_seed(0)
for M, Nn in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
    dy = torch.randn(R, M, device="cuda", generator=g).bfloat16()
    x = torch.randn(R, Nn, device="cuda", generator=g).bfloat16()
    gW = torch.zeros(M, Nn, device="cuda")
    gb = torch.zeros(M, device="cuda")
    f = 2.0 * R * M * Nn
    t_ours = timed(lambda: N.gemm_wgrad(dy, x, gW, gb), 10)
    t_ours_nb = timed(lambda: N.gemm_wgrad(dy, x, gW), 10)
    dyt = dy.t()
    t_lib = timed(lambda: torch.matmul(dyt, x), 10)
    print(json.dumps({"M": M, "N": Nn, "K": R, "mmseq_tflops": round(f / t_ours / 1e12, 1),
                      "mmseq_no_bias_tflops": round(f / t_ours_nb / 1e12, 1),
                      "hipblaslt_bf16_out_tflops": round(f / t_lib / 1e12, 1)}), flush=True)
    del dy, x
