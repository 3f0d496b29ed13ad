"""Run the bf16 attention forward (and optionally backward) for given T values, a few times each:
a small target for rocprofv3 --pmc passes.  usage: python tools/attn_one.py T [T ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_sequencing_amd import _native as N  # noqa: E402

P, heads = 320, 12
N.attn_set_fast(int(os.environ.get("ATTN_VARIANT", "2")))
H = heads * 64
for T in [int(x) for x in sys.argv[1:]]:
    g = torch.Generator(device="cpu").manual_seed(0)
    qkv = (torch.randn(P * T, 3 * H, generator=g) * 0.5).to("cuda", torch.bfloat16)
    bias = torch.zeros(P, T, device="cuda")
    out = torch.empty(P * T, H, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(P, heads, T, device="cuda")
    for _ in range(3):
        N.attn_fwd(P, T, heads, qkv, 3 * H, 0, H, 2 * H, bias, 0.125, out, H, lse)
    torch.cuda.synchronize()
    print("T", T, "done", flush=True)
