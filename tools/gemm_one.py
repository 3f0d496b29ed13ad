"""One bf16 NT GEMM shape of the path, repeated (for PMC passes and A/B timing of library builds:
MMSEQ_BENCH_LIB). usage: gemm_one.py N K [epi] [iters]; prints HIP-event TFLOP/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_sequencing_amd import _native as N  # noqa: E402
if os.environ.get("MMSEQ_BENCH_LIB"):
    N.LIB_PATH = os.environ["MMSEQ_BENCH_LIB"]

R = 328320
Nn, K = int(sys.argv[1]), int(sys.argv[2])
epi = sys.argv[3] if len(sys.argv) > 3 else "plain"
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 10
g = torch.Generator(device="cuda").manual_seed(0)
A = torch.randn(R, K, device="cuda", generator=g).bfloat16()
W = (torch.randn(Nn, K, device="cuda", generator=g) * 0.05).bfloat16()
C = torch.empty(R, Nn, device="cuda", dtype=torch.bfloat16)
bias = torch.randn(Nn, device="cuda", generator=g)
res = torch.randn(R, Nn, device="cuda", generator=g).bfloat16()
kw = {"plain": {}, "res": {"bias": bias, "resid": res}, "gelu": {"bias": bias, "act": 1, "aux": res}}[epi]
f = lambda: N.gemm(A, W, C, R, Nn, K, **kw)
f()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    f()
e1.record()
torch.cuda.synchronize()
t = e0.elapsed_time(e1) / iters * 1e-3
print(json.dumps({"N": Nn, "K": K, "epi": epi, "lib": os.environ.get("MMSEQ_BENCH_LIB", "tree"),
                  "tflops": round(2.0 * R * Nn * K / t / 1e12, 1)}), flush=True)
