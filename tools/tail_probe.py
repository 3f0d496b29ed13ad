"""What the persistent NT kernel's partial last round costs on the N = 768 shapes: the product
GEMM at R = 640 x 513 rows (3 849 tiles = 15 rounds + 9 tiles on 256 CUs) against R = 327 680
(exactly 15 rounds) and the 640-row remainder alone (the generic 128 x 128 kernel). HIP-event
time per call, plain bf16 output with bias. Measurement only.
    python tools/tail_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_sequencing_amd import _native as N  # noqa: E402


def timed(fn, iters=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    R = 640 * 513
    for Nn, K in ((768, 768), (768, 2304), (768, 3072)):
        A = torch.randn(R, K, device="cuda", generator=g).bfloat16()
        B = torch.randn(Nn, K, device="cuda", generator=g).bfloat16()
        C = torch.empty(R, Nn, device="cuda", dtype=torch.bfloat16)
        bias = torch.randn(Nn, device="cuda", generator=g)
        row = {"N": Nn, "K": K}
        for M in (R, 327680, 640, 11520, 251520, 250112):
            us = timed(lambda: N.gemm(A, B, C, M, Nn, K, bias=bias))
            row[f"M{M}_us"] = round(us, 1)
            row[f"M{M}_tflops"] = round(2.0 * M * Nn * K / us / 1e6, 1)
        print(json.dumps(row), flush=True)
        del A, B, C


if __name__ == "__main__":
    main()
