"""Microbenchmark of the ViT embedding kernels (mmseq_vit_embed_fwd / _bwd) at config 3's shape
(P = 640 pairs, 1 + 2 x 196 tokens, W = 768, bf16). MMSEQ_BENCH_LIB: an A/B build of the library."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_sequencing_amd import _native as N  # noqa: E402
if os.environ.get("MMSEQ_BENCH_LIB"):
    N.LIB_PATH = os.environ["MMSEQ_BENCH_LIB"]

P, gg, W = 640, 196, 768
ntok = 1 + 2 * gg
g = torch.Generator(device="cpu").manual_seed(0)
po = torch.randn(P * 2 * gg, W, generator=g).to("cuda", torch.bfloat16)
cls, pos = torch.randn(W, device="cuda"), torch.randn(gg + 1, W, device="cuda")
gam, bet = torch.ones(W, device="cuda"), torch.zeros(W, device="cuda")
x = torch.empty(P * ntok, W, device="cuda", dtype=torch.bfloat16)
y, mean, rstd = torch.empty_like(x), torch.empty(P * ntok, device="cuda"), torch.empty(P * ntok, device="cuda")
dy = torch.randn(P * ntok, W, generator=g).to("cuda", torch.bfloat16)
dpo = torch.empty_like(po)
dcls, dpos, dg, db = torch.zeros_like(cls), torch.zeros_like(pos), torch.zeros_like(gam), torch.zeros_like(bet)
fwd = lambda: N.vit_embed_fwd(P, ntok, W, gg, po, cls, pos, gam, bet, 1e-5, x, y, mean, rstd)
bwd = lambda: N.vit_embed_bwd(P, ntok, W, gg, dy, x, mean, rstd, gam, dpo, dcls, dpos, dg, db)
for name, f, gb in (("fwd", fwd, 3 * P * ntok * W * 2), ("bwd", bwd, 3 * P * ntok * W * 2)):
    f(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        f()
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 10 * 1e3
    print(f"vit_embed_{name}: {us:.1f} us per call, {gb / us / 1e3:.0f} GB/s of the 3 row tensors", flush=True)
