"""What the TN weight-gradient kernel's fused bias gradient costs on the GEMMs whose dY a LayerNorm
backward writes (the attention output projection and FC2 / c_proj: out = 768): mmseq_gemm_wgrad
with and without gb, HIP-event time per call, joint-encoder and ViT row counts. Measurement only.
    python tools/tn_bias_probe.py"""
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
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    for R in (640 * 513, 640 * 393):
        for out, inp in ((768, 768), (768, 3072), (3072, 768), (2304, 768)):
            dy = torch.randn(R, out, device="cuda", generator=g).bfloat16()
            x = torch.randn(R, inp, device="cuda", generator=g).bfloat16()
            gW = torch.zeros(out, inp, device="cuda")
            gb = torch.zeros(out, device="cuda")
            t_b = timed(lambda: N.gemm_wgrad(dy, x, gW, gb))
            t_n = timed(lambda: N.gemm_wgrad(dy, x, gW))
            f = 2.0 * R * out * inp
            print(json.dumps({"R": R, "out": out, "in": inp, "with_bias_us": round(t_b, 1),
                              "no_bias_us": round(t_n, 1), "bias_cost": round(t_b / t_n - 1, 3),
                              "tflops_no_bias": round(f / t_n / 1e6, 1)}), flush=True)
            del dy, x


if __name__ == "__main__":
    main()
