"""Headline benchmark: multimodal fine-tuning steps/sec (fwd+bwd+optimizer) at N = 5 story steps,
pair sequence 512 (120 text + 393 ViT-B/16 tokens), BASELINE config 3 (1 GPU) / config 4 (DP).

One "step" = one optimizer step of the reference train loop (trainers/train.py:275-363) over a
per-GPU batch of B stories (B = 32, config 3), all 20 ordered pairs per story, bf16 compute with
fp32 master weights; synthetic seeded inputs already resident in HBM; random-init weights of the
exact architecture. Launch (multi-GPU):
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import re
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from multimodal_sequencing_amd import _native as N  # noqa: E402
from multimodal_sequencing_amd import model_zoo  # noqa: E402
from multimodal_sequencing_amd.trainer import FusedAdamW, GradAllReduce, train_step  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md chip table)


def story_flops(Pst, Lt, Tv, H, Lj, W, Lv, patch, E, ff=4):
    """SURVEY §8(d) algorithmic fwd FLOPs per story (2 FLOP / MAC)."""
    npatch = Tv - 1
    T = Lt + Tv
    vit = 2 * (npatch * 3 * patch * patch * W + Lv * (12 * Tv * W * W + 2 * Tv * Tv * W) + Tv * W * E)
    joint = 2 * Lj * (12 * T * H * H + 2 * T * T * H)
    visn = 2 * Tv * E * H
    head = 2 * Pst * Lt * H * H + 2 * Pst * Lt * H
    return Pst * (vit + visn + joint) + head


def synthetic_batch(B, Nst, per_seq, vocab, res, device, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    k = per_seq - 2
    content = torch.randint(3, vocab, (B, Nst, k), generator=g)
    steps = torch.cat([torch.zeros(B, Nst, 1, dtype=torch.long), content,
                       torch.full((B, Nst, 1), 2, dtype=torch.long)], -1)
    ids = steps.view(B, Nst * per_seq)
    labels = torch.stack([torch.argsort(torch.randperm(Nst, generator=g)) for _ in range(B)])
    images = torch.randn(B, Nst, 3, res, res, generator=g).to(device)
    return {"input_ids": ids, "labels": labels, "images": images}


class GemmTimer:
    """Records HIP events around every bf16 NT GEMM launch (the dominant kernel) on the stream it
    is launched on, to report achieved TFLOP/s per launch live from the timed region."""

    def __init__(self):
        self.recs = []
        self.on = False
        self._orig = N.gemm

    def install(self):
        orig = self._orig
        timer = self

        def wrapped(A, B, C, M, Nn, K, **kw):
            if timer.on and kw.get("trans", 0) == 0 and A.dtype == torch.bfloat16:
                s = torch.cuda.current_stream()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(s)
                orig(A, B, C, M, Nn, K, **kw)
                e1.record(s)
                bt = kw.get("batch", 1)
                # algorithmic HBM bytes: A, B, C once (+ residual / dact / aux tensors), bf16
                extra = sum(1 for k in ("resid", "dact", "aux") if kw.get(k) is not None)
                if kw.get("accumulate"):
                    extra += 1
                byts = 2.0 * bt * (M * K + Nn * K + M * Nn * (1 + extra))
                timer.recs.append((e0, e1, 2.0 * M * Nn * K * bt, byts))
            else:
                orig(A, B, C, M, Nn, K, **kw)

        N.gemm = wrapped
        import multimodal_sequencing_amd.kernels as Kmod
        Kmod.N.gemm = wrapped

    def summary(self):
        if not self.recs:
            return None
        t = sum(r[0].elapsed_time(r[1]) for r in self.recs) * 1e-3
        f = sum(r[2] for r in self.recs)
        b = sum(r[3] for r in self.recs)
        n = len(self.recs)
        return {"launches": n, "avg_us": t / n * 1e6, "avg_gflop": f / n / 1e9,
                "achieved_tflops": f / t / 1e12, "avg_alg_bytes": b / n}


def pmc_traffic(group="gemm256_nt"):
    """Per-launch HBM traffic of the roofline kernel from the newest committed rocprofv3 --pmc
    summary (profiles/r*_pmc_traffic.json, made by tools/pmc_traffic.py: FETCH_SIZE x 2 +
    WRITE_SIZE, the gfx950 corrections of MI355X_MICROARCH.md), or None."""
    import glob
    def order(f):  # r<round>_v<version>: numeric, so v10 sorts after v9
        m = re.match(r"r(\d+)_v(\d+)_", os.path.basename(f))
        return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")), key=order)
    if not files:
        return None, None
    try:
        d = json.load(open(files[-1]))
        return d[group]["traffic_bytes"], os.path.relpath(files[-1], ROOT)
    except (OSError, KeyError, ValueError):
        return None, None


def cpu_baseline(preset, seconds_hint=30):
    """The CPU oracle (fp32 PyTorch restatement, oracle/berson_oracle.py) timed on host cores:
    one fwd+bwd of ONE story of the same config (bounded sample)."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from oracle import berson_oracle as O
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    m = model_zoo.build_preset(preset, device="cpu", dtype=torch.float32)
    params = {k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    p = model_zoo.PRESETS[preset]
    data = synthetic_batch(1, p["N"], p["per_seq"], 50265, 224, "cpu", seed=7)
    cfg = {"N": p["N"], "heads": p["joint"]["num_attention_heads"], "inter_heads": 8,
           "text_only": p["vision"] is None, "vit_heads": None}
    t0 = time.perf_counter()
    loss, _, _ = O.forward_loss(params, data["input_ids"].numpy(), data["labels"].numpy(),
                                data["images"], cfg)
    loss.backward()
    dt = time.perf_counter() - t0
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": 1.0 / dt, "unit": "stories/s (fwd+bwd, fp32)", "cores": threads,
            "kind": "port", "sample": f"1 story ({p['N']} steps, {p['N'] * (p['N'] - 1)} pairs) "
            f"fwd+bwd of the oracle on {threads} threads of {cpu}; {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="config3")
    ap.add_argument("--batch", type=int, default=32, help="stories per GPU per step")
    ap.add_argument("--micro", type=int, default=16, help="stories per micro-batch")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gemm-timer", action="store_true")
    ap.add_argument("--fwd-steps", type=int, default=3,
                    help="forward-only passes timed after the training steps (north-star check)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    preset = model_zoo.PRESETS[args.config]
    model = model_zoo.build_preset(args.config, device=dev, dtype=torch.bfloat16, seed=0)
    model.train()  # dropout p = 0.1 at every reference site, counter-based masks
    model.bert.dropout_seed = 1 + rank
    stores = model.stores()
    opt = FusedAdamW(stores, lr=5e-6, warmup=100)
    reducer = GradAllReduce(stores) if world > 1 else None
    data = synthetic_batch(args.batch, preset["N"], preset["per_seq"], 50265, 224, dev,
                           seed=1000 + rank)
    mbs = []
    for o in range(0, args.batch, args.micro):
        mbs.append({k: v[o:o + args.micro] for k, v in data.items()})

    timer = GemmTimer()
    if not args.no_gemm_timer:
        timer.install()
    for _ in range(args.warmup):
        train_step(model, opt, mbs, reducer)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timer.on = True
    t0 = time.perf_counter()
    loss = None
    for _ in range(args.steps):
        loss = train_step(model, opt, mbs, reducer)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    timer.on = False
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()

    # North-star forward check (stories/s_fwd x fwd FLOP/story / peak): the same
    # batch, eval mode (no dropout), no autograd graph, timed like the training steps.
    fwd_dt = None
    if args.fwd_steps > 0:
        model.eval()
        with torch.no_grad():
            for b in mbs:
                model(b)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            f0 = time.perf_counter()
            for _ in range(args.fwd_steps):
                for b in mbs:
                    model(b)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            fwd_dt = time.perf_counter() - f0
        model.train()
        if world > 1:
            t = torch.tensor([fwd_dt], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            fwd_dt = t.item()

    Nst, per = preset["N"], preset["per_seq"]
    Pst = Nst * (Nst - 1)
    J = preset["joint"]
    V = model.bert.vision
    g = 224 // V["patch"]
    Tv = 1 + 2 * g * g
    Lt = 2 * per
    fwd = story_flops(Pst, Lt, Tv, J["hidden_size"], J["num_hidden_layers"], V["width"],
                      V["layers"], V["patch"], V["embed"])
    stories = args.batch * args.steps * world
    steps_s = args.steps * world / dt
    out = {
        "metric": "multimodal steps/sec (fwd+bwd) at N=5 steps, seq=512, ViT-B/16; 1/2/4/8 GPU",
        "value": steps_s, "unit": "steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (seeded token ids U[3,50265), N(0,1) 224x224 images), random-init "
                "weights, train mode (dropout 0.1)",
        "config": {"workload": f"{args.config}: ViT-B/16 + 12x768 joint encoder + BERSON, "
                               f"N={Nst} steps, {Pst} pairs/story, pair seq {Lt}+{Tv}={Lt + Tv}",
                   "global_batch": args.batch * world, "stories_per_gpu": args.batch,
                   "micro_batch": args.micro, "seq_len": Lt + Tv, "parallelism": f"dp{world}"},
        "stories_per_s": stories / dt,
        "model_tflops": stories / dt * 3 * fwd / 1e12,
        "model_flops_util": stories / dt * 3 * fwd / 1e12 / PEAK_BF16_TFLOPS,
        "loss": float(loss.item()) if loss is not None else None,
    }
    if fwd_dt is not None:
        fst = args.batch * args.fwd_steps * world / fwd_dt
        out["forward"] = {"stories_per_s": fst, "ms_per_batch": fwd_dt / args.fwd_steps * 1e3,
                          "tflops": fst * fwd / 1e12,
                          "mfma_frac": fst * fwd / 1e12 / PEAK_BF16_TFLOPS,
                          "mode": "eval (no dropout), torch.no_grad, full model forward incl. "
                                  "BERSON head + loss; ViT + joint encoder are >99.9% of FLOPs"}
    gs = timer.summary()
    if gs:
        traffic, tsrc = pmc_traffic()
        out["roofline"] = {"bound": "mfma", "kernel": "gemm256_nt_kernel (bf16 NT: fwd + dgrad)",
                           "achieved": gs["achieved_tflops"], "peak": PEAK_BF16_TFLOPS,
                           "unit": "TFLOP/s", "frac": gs["achieved_tflops"] / PEAK_BF16_TFLOPS,
                           "traffic": traffic, "traffic_unit": "bytes per launch (PMC)",
                           "traffic_source": tsrc,
                           "algorithmic_bytes_per_launch": gs["avg_alg_bytes"],
                           "launches": gs["launches"],
                           "avg_launch_us": gs["avg_us"], "avg_gflop_per_launch": gs["avg_gflop"]}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(args.config)
        except Exception as e:  # the baseline is reported, never required for the GPU number
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
