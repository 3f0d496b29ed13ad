"""Microbenchmark of mmseq_gemm on the path's shapes (bf16), fast vs generic kernel."""
import sys, os, json
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_sequencing_amd import _native as N

def bench(M, Nn, K, trans, fast, iters=20):
    N.gemm_set_fast(fast)
    if trans:
        A = torch.randn(K, M, device="cuda").bfloat16(); B = torch.randn(K, Nn, device="cuda").bfloat16()
        C = torch.zeros(M, Nn, device="cuda")
    else:
        A = torch.randn(M, K, device="cuda").bfloat16(); B = torch.randn(Nn, K, device="cuda").bfloat16()
        C = torch.empty(M, Nn, device="cuda", dtype=torch.bfloat16)
    kw = dict(trans=trans, accumulate=bool(trans))
    for _ in range(3): N.gemm(A, B, C, M, Nn, K, **kw)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record()
    for _ in range(iters): N.gemm(A, B, C, M, Nn, K, **kw)
    e1.record(); torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / iters * 1e-3
    return 2.0 * M * Nn * K / t / 1e12

R = 164160  # joint rows at 16 stories (320 pairs x 513)
shapes = [(R, 2304, 768, 0), (R, 768, 768, 0), (R, 3072, 768, 0), (R, 768, 3072, 0),
          (768, 3072, R, 1), (3072, 768, R, 1), (2304, 768, R, 1), (768, 768, R, 1), (4096, 4096, 4096, 0), (4096, 4096, 4096, 1)]
for M, Nn, K, tr in shapes:
    modes = (("default", 1), ("big", 4), ("dbuf", 2), ("ring", 3)) if not tr else \
        (("default", 1), ("dbuf", 2), ("ring", 3))
    r = {k: round(bench(M, Nn, K, tr, v), 1) for k, v in modes}
    if tr == 0:  # hipBLASLt through torch, as a yardstick only
        A = torch.randn(M, K, device="cuda").bfloat16(); B = torch.randn(Nn, K, device="cuda").bfloat16()
        for _ in range(3): torch.matmul(A, B.t())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10): torch.matmul(A, B.t())
        e1.record(); torch.cuda.synchronize()
        r["torch"] = round(2.0 * M * Nn * K / (e0.elapsed_time(e1) / 10 * 1e-3) / 1e12, 1)
    print(json.dumps({"M": M, "N": Nn, "K": K, "trans": tr, **r}), flush=True)
