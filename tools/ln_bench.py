"""LayerNorm forward (bf16, fp32 statistics) at the path's shapes, HIP-event timed on the torch
stream; prints GB/s of the algorithmic bytes (x read + y written). A/B via MMSEQ_BENCH_LIB.
    python tools/ln_bench.py"""
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from multimodal_sequencing_amd import _native as N  # noqa: E402
from multimodal_sequencing_amd import kernels as K  # noqa: E402
if os.environ.get("MMSEQ_BENCH_LIB"):
    N.LIB_PATH = os.environ["MMSEQ_BENCH_LIB"]

out = []
for rows, H in [(164160, 768), (20 * 32 * 393 // 2, 768), (55368, 1024)]:
    x = torch.randn(rows, H, device="cuda").bfloat16()
    y = torch.empty_like(x)
    g = torch.randn(H, device="cuda")
    b = torch.randn(H, device="cuda")
    mean = torch.empty(rows, device="cuda")
    rstd = torch.empty(rows, device="cuda")
    f = lambda: N.layernorm_fwd(rows, H, x, K._rows(H), g, b, 1e-5, y, K._rows(H), mean, rstd)  # noqa
    for _ in range(3):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        f()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    ref = torch.nn.functional.layer_norm(x.float(), (H,), g, b, 1e-5)
    err = float((y.float() - ref).abs().max())
    out.append({"rows": rows, "H": H, "us": round(us, 1), "GBps": round(rows * H * 4 / us / 1e3, 1),
                "max_abs_err": err})
print(json.dumps(out))

# backward (python tools/ln_bench.py bwd): dy, x read, dx (+ the dropout-masked dx_drop) written,
# dgamma / dbeta partials reduced; the joint encoder's rows at config 3
if len(sys.argv) > 1 and sys.argv[1] == "bwd":
    res = []
    for rows, H, drop in [(640 * 513, 768, False), (640 * 513, 768, True), (640 * 393, 768, False)]:
        x = torch.randn(rows, H, device="cuda").bfloat16()
        dy = torch.randn(rows, H, device="cuda").bfloat16()
        g = torch.randn(H, device="cuda")
        mean, rstd = torch.zeros(rows, device="cuda"), torch.ones(rows, device="cuda")
        dx, dxd = torch.empty_like(x), torch.empty_like(x) if drop else None
        dg, db = torch.zeros(H, device="cuda"), torch.zeros(H, device="cuda")
        d = N.drop(0.1, 3, 4) if drop else None
        f = lambda: N.layernorm_bwd(rows, H, dy, K._rows(H), x, K._rows(H), mean, rstd, g, dx, K._rows(H),  # noqa
                                    None, K._rows(H), dg, db, dx_drop=dxd, drop_dx=d)
        for _ in range(3):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            f()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        nbytes = rows * H * 2 * (4 if drop else 3)
        res.append({"rows": rows, "H": H, "dx_drop": drop, "us": round(us, 1), "GBps": round(nbytes / us / 1e3, 1)})
    print(json.dumps(res))
