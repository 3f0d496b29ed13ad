"""Microbenchmark of the fused attention kernels on the path's shapes (bf16), with/without dropout."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_sequencing_amd import _native as N
if os.environ.get("MMSEQ_BENCH_LIB"):  # A/B runs: another build of the library, same process layout
    N.LIB_PATH = os.environ["MMSEQ_BENCH_LIB"]


def run(P, T, heads, drop, iters=5, bits=False, variant=1):
    H = heads * 64
    g = torch.Generator(device="cpu").manual_seed(0)
    qkv = (torch.randn(P * T, 3 * H, generator=g) * 0.5).to("cuda", torch.bfloat16)
    bias = torch.zeros(P, T, device="cuda")
    out = torch.empty(P * T, H, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(P, heads, T, device="cuda")
    dout = torch.randn(P * T, H, generator=g).to("cuda", torch.bfloat16)
    delta = torch.empty_like(lse)
    dqkv = torch.empty_like(qkv)
    d = N.drop(0.1, 5, 99) if drop else None
    kb = N.attn_keep_bits(P, T, heads, "cuda") if bits else None
    fwd = lambda: N.attn_fwd(P, T, heads, qkv, 3 * H, 0, H, 2 * H, bias, 0.125, out, H, lse, drop=d,
                             keep_bits=kb)
    bwd = lambda: N.attn_bwd(P, T, heads, qkv, 3 * H, 0, H, 2 * H, bias, 0.125, out, H, dout, H,
                             lse, delta, dqkv, 3 * H, drop=d, keep_bits=kb)
    res = {}
    N.attn_set_fast(variant)
    for name, f in (("fwd", fwd), ("bwd", bwd)):
        f(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters): f()
        e1.record(); torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / iters * 1e-3
        fl = 4.0 * P * heads * T * T * 64 * (1 if name == "fwd" else 2.5)
        res[name + "_us"] = round(t * 1e6, 1)
        res[name + "_tflops"] = round(fl / t / 1e12, 1)
    return res


variants = [int(v) for v in sys.argv[1:]] or [1, 2]
Ts = [int(t) for t in os.environ.get("ATTN_SHAPES", "513,393").split(",")]  # e.g. 513,512,393,384
for P, T in [(640, t) for t in Ts]:
    for drop, bits in ((False, False), (True, True)):
        for var in variants:
            print(json.dumps({"P": P, "T": T, "drop": drop, "bits": bits, "variant": var,
                              **run(P, T, 12, drop, bits=bits, variant=var)}), flush=True)
