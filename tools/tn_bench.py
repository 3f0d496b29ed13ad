"""Weight-gradient (TN, fp32 accumulate) GEMMs of the joint encoder at the path's shapes: TFLOP/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_sequencing_amd import _native as N  # noqa: E402

R = 164160
for M, Nn in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
    A = torch.randn(R, M, device="cuda").bfloat16()
    B = torch.randn(R, Nn, device="cuda").bfloat16()
    C = torch.zeros(M, Nn, device="cuda")
    for _ in range(3):
        N.gemm(A, B, C, M, Nn, R, trans=True, accumulate=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(20):
        N.gemm(A, B, C, M, Nn, R, trans=True, accumulate=True)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 20 * 1e-3
    print(json.dumps({"M": M, "N": Nn, "K": R, "us": round(t * 1e6, 1),
                      "tflops": round(2.0 * M * Nn * R / t / 1e12, 1)}), flush=True)
