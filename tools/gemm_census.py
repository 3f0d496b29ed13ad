"""Every mmseq_gemm call of one config-3 training step, grouped by (dtype, trans, M, N, K) with
HIP-event time per group: which GEMMs cost what (bench.py's model and batch)."""
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from multimodal_sequencing_amd import _native as N  # noqa: E402
from multimodal_sequencing_amd import model_zoo  # noqa: E402
from multimodal_sequencing_amd import kernels as Kmod  # noqa: E402
from multimodal_sequencing_amd.trainer import FusedAdamW, train_step  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    preset = model_zoo.PRESETS["config3"]
    model = model_zoo.build_preset("config3", device=dev, dtype=torch.bfloat16, seed=0)
    model.train()
    opt = FusedAdamW(model.stores(), lr=5e-6, warmup=100)
    data = bench.synthetic_batch(32, preset["N"], preset["per_seq"], 50265, 224, dev, seed=1000)
    mbs = [data]  # bench.py's default: the whole 32-story batch in one micro-batch
    train_step(model, opt, mbs, None)
    torch.cuda.synchronize()
    recs = []
    orig = N.gemm

    def wrapped(A, B, C, M, Nn, K, **kw):
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        orig(A, B, C, M, Nn, K, **kw)
        e1.record(s)
        epi = "".join(t for t, on in (("acc+", kw.get("accumulate")), ("res+", kw.get("resid") is not None),
                                      ("drop+", kw.get("drop") is not None), (f"act{kw.get('act', 0)}+", kw.get("act")),
                                      ("dact+", kw.get("dact") is not None), ("aux+", kw.get("aux") is not None),
                                      ("bias+", kw.get("bias") is not None)) if on)
        key = (str(A.dtype).replace("torch.", ""), kw.get("trans", 0), M, Nn, K, epi or "plain")
        recs.append((key, e0, e1))

    N.gemm = wrapped
    Kmod.N.gemm = wrapped
    train_step(model, opt, mbs, None)
    torch.cuda.synchronize()
    agg = collections.defaultdict(lambda: [0, 0.0])
    for key, e0, e1 in recs:
        agg[key][0] += 1
        agg[key][1] += e0.elapsed_time(e1)
    tot = sum(v[1] for v in agg.values())
    print(f"total {tot:.1f} ms over {len(recs)} calls")
    for key, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        dt, tr, M, Nn, K, acc = key
        tf = 2.0 * M * Nn * K * n / (ms * 1e-3) / 1e12
        print(f"{dt:9s} tr={tr} M={M:7d} N={Nn:5d} K={K:7d} {acc:18s} calls={n:4d} {ms:8.2f} ms "
              f"{tf:7.1f} TF/s")


if __name__ == "__main__":
    main()
