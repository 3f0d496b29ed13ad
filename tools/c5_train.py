"""Config-5 training steps (ViT-L/14 + 24 x 1024, N = 9, T = 769; 4 stories in micro-batches of 2),
bf16 or with the fp8 forward GEMMs: a rocprofv3 target for the bench's config-5 training leg.
usage: python tools/c5_train.py [bf16|fp8|fp8dg] [steps]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import synthetic_batch  # noqa: E402
from multimodal_sequencing_amd import kernels as K  # noqa: E402
from multimodal_sequencing_amd import model_zoo  # noqa: E402
from multimodal_sequencing_amd.trainer import FusedAdamW, train_step  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "fp8"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
preset = model_zoo.PRESETS["config5"]
m = model_zoo.build_preset("config5", device="cuda", dtype=torch.bfloat16, seed=0)
m.train()
opt = FusedAdamW(m.stores(), lr=5e-6, warmup=100, total_steps=100)
data = synthetic_batch(4, preset["N"], preset["per_seq"], 50265, 224, "cuda", seed=3000)
mbs = [{k: v[o:o + 2] for k, v in data.items()} for o in (0, 2)]
with K.fp8_forward(mode != "bf16", training=True, dgrad=mode == "fp8dg"):
    train_step(m, opt, mbs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = train_step(m, opt, mbs)
    torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / steps
print(f"config5 train ({mode}): {dt * 1e3:.1f} ms/step, loss {float(loss):.4f}", flush=True)
