"""HIP-event time of the BERSON head's small fp32 GEMMs (the split-K path of mmseq_gemm for
outputs with < 128 tiles of 128 x 128): forward shapes from profiles/r5_v23_gemm_census.log and
the weight-gradient form (trans = 1, K = rows). Measurement only.
    python tools/gemm_f32_small.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_sequencing_amd import _native as N  # noqa: E402

if os.environ.get("MMSEQ_BENCH_LIB"):
    N.LIB_PATH = os.environ["MMSEQ_BENCH_LIB"]


def timed(fn, iters=50):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    tot = 0.0
    for trans, M, Nn, K in ((0, 160, 768, 768), (0, 32, 768, 3072), (0, 32, 3072, 768),
                            (0, 160, 768, 3072), (0, 160, 3072, 768), (1, 768, 768, 160),
                            (1, 768, 3072, 160), (1, 3072, 768, 160), (1, 768, 768, 32)):
        if trans:  # C[M][N] += A^T B with A [K][M], B [K][N]
            A = torch.randn(K, M, device="cuda", generator=g)
            B = torch.randn(K, Nn, device="cuda", generator=g)
        else:
            A = torch.randn(M, K, device="cuda", generator=g)
            B = torch.randn(Nn, K, device="cuda", generator=g)
        C = torch.zeros(M, Nn, device="cuda")
        us = timed(lambda: N.gemm(A, B, C, M, Nn, K, trans=trans, accumulate=bool(trans)))
        tot += us
        print(json.dumps({"trans": trans, "M": M, "N": Nn, "K": K, "us": round(us, 1)}), flush=True)
    print(json.dumps({"total_us": round(tot, 1)}), flush=True)


if __name__ == "__main__":
    main()
