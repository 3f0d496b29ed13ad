"""Yardstick: mmseq's bf16 NT GEMM (product default) vs torch.matmul (hipBLASLt) on the
config-3 joint-encoder shapes at B = 32 stories (R = 640 pairs x 513 rows), plain output.
HIP-event time per call; prints one JSON line per shape. Measurement only."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_sequencing_amd import _native as N  # noqa: E402


def timed(fn, iters):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 640 * 513
    g = torch.Generator(device="cuda").manual_seed(0)
    for Nn, K in ((2304, 768), (768, 768), (3072, 768), (768, 3072), (768, 2304)):
        A = torch.randn(R, K, device="cuda", generator=g).bfloat16()
        B = torch.randn(Nn, K, device="cuda", generator=g).bfloat16()
        C = torch.empty(R, Nn, device="cuda", dtype=torch.bfloat16)
        f = 2.0 * R * Nn * K
        t_ours = timed(lambda: N.gemm(A, B, C, R, Nn, K), 10)
        Bt = B.t()
        t_lib = timed(lambda: torch.matmul(A, Bt), 10)
        ref = torch.matmul(A[:4096], Bt).float()
        err = float((C[:4096].float() - ref).abs().max() / ref.abs().max())
        print(json.dumps({"M": R, "N": Nn, "K": K, "mmseq_tflops": round(f / t_ours / 1e12, 1),
                          "hipblaslt_tflops": round(f / t_lib / 1e12, 1),
                          "rel_err": err}), flush=True)
        del A, B, C


if __name__ == "__main__":
    main()
