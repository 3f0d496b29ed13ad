"""MX-fp8 NT GEMM (mmseq_gemm_mxfp8) vs the bf16 NT GEMM (mmseq_gemm) on the config-5 forward
shapes (72 pair rows x 769 tokens: joint RoBERTa-large layer QKV / O / FC1 / FC2), plus the
quantiser's cost. HIP-event timing on the torch stream, 3 warm-up + 10 timed launches each.
usage: python tools/fp8_bench.py [rows]"""
import json
import sys

import torch

sys.path.insert(0, ".")
from multimodal_sequencing_amd import _native as N  # noqa: E402
import os  # noqa: E402
if os.environ.get("MMSEQ_BENCH_LIB"):  # A/B runs on one box: another build of the library
    N.LIB_PATH = os.environ["MMSEQ_BENCH_LIB"]


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 72 * 769
    dev = "cuda"
    out = {"rows": M, "shapes": []}
    for name, Nn, K, act in [("qkv", 3072, 1024, 0), ("o", 1024, 1024, 0), ("fc1", 4096, 1024, 0),
                             ("fc1_gelu", 4096, 1024, 1), ("fc2", 1024, 4096, 0)]:
        A = torch.randn(M, K, device=dev).bfloat16()
        W = (torch.randn(Nn, K, device=dev) * 0.02).bfloat16()
        bias = torch.zeros(Nn, device=dev)
        C = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
        t_bf16 = timeit(lambda: N.gemm(A, W, C, M, Nn, K, bias=bias, act=act))
        qa, qw = N.quant_mxfp8(A), N.quant_mxfp8(W)
        t_q = timeit(lambda: N.quant_mxfp8(A, out=qa))
        t_fp8 = timeit(lambda: N.gemm_mxfp8(qa, qw, C, bias=bias, act=act))
        fl = 2.0 * M * Nn * K
        t_q8 = timeit(lambda: N.gemm_mxfp8_q8(qa, qw, bias=bias, act=act)) if Nn >= 3072 else None
        out["shapes"].append({"gemm": name, "N": Nn, "K": K,
                              "mxfp8_q8out_us": t_q8 * 1e6 if t_q8 else None,
                              "bf16_us": t_bf16 * 1e6, "bf16_tflops": fl / t_bf16 / 1e12,
                              "mxfp8_us": t_fp8 * 1e6, "mxfp8_tflops": fl / t_fp8 / 1e12,
                              "quant_act_us": t_q * 1e6,
                              "quant_gbps": (M * K * 2 + M * K + M * K / 32) / t_q / 1e9})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
