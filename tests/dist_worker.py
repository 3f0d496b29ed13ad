"""Worker for tests/test_distributed_cpu.py (launched by torch.distributed.run, gloo backend).

mode "flat":    bucketed mean all-reduce of a small store issued by finish() alone.
mode "overlap": the product model's real grad layout (tiny golden config on CPU); a simulated
                backward writes each unit's gradient and reports it in backward order, exactly
                as the layer Functions do, with the reducer armed; buckets must be issued
                during the "backward" and the result must equal one flat all-reduce.
"""
import json
import os
import sys

import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "golden"))
from multimodal_sequencing_amd.params import ParamStore, Spec, normal  # noqa: E402
from multimodal_sequencing_amd.trainer import GradAllReduce  # noqa: E402


def flat(out, rank):
    specs = [Spec("a.weight", (300, 7), normal(1.0)), Spec("b.bias", (5,), normal(1.0))]
    st = ParamStore(specs, "cpu", torch.float32)
    g = torch.Generator().manual_seed(rank)
    st.grad.copy_(torch.randn(st.grad.shape, generator=g))
    GradAllReduce([st], bucket_mb=0.001)()  # tiny buckets: many chunks in flight
    torch.save(st.grad.clone(), os.path.join(out, f"grad{rank}.pt"))


def overlap(out, rank):
    from golden_util import load_fixture
    from multimodal_sequencing_amd import model_zoo
    meta, _, _ = load_fixture("tiny")
    m = model_zoo.build_from_golden(meta["config"], device="cpu")
    stores = m.stores()
    units, begin = m.ddp_units()
    red = GradAllReduce(stores, bucket_mb=0.25, units=units, begin_units=begin)
    g = torch.Generator().manual_seed(100 + rank)
    full = {id(s): torch.randn(s.numel, generator=g) for s in stores}
    for s in stores:
        s.grad.zero_()
    red.arm(True)
    # the head's backward runs first (it writes its whole store), then the inner model's units
    # in backward order: joint layers top-down, joint input, ViT blocks top-down, stem
    head = m.store
    head.grad.copy_(full[id(head)])
    inner = m.bert.store
    fired = []
    for span in ([L.span for L in reversed(m.bert.layer_refs)] + [m.bert.input_refs.span]
                 + [L.span for L in reversed(m.bert.block_refs)] + [m.bert.grad_units()[-1]]):
        inner.grad_begin()
        lo, hi = span
        inner.grad[lo:hi].copy_(full[id(inner)][lo:hi])
        inner.grad_ready(span)
        fired.append(len(red.works))
    # parameters that no unit covers (pooler, box_fc, ln_post, ...) get their grads last
    covered = torch.zeros(inner.numel, dtype=torch.bool)
    for lo, hi in m.bert.grad_units():
        covered[lo:hi] = True
    inner.grad[~covered] = full[id(inner)][~covered]
    red.finish()
    expect = {}
    for s in stores:
        ref = full[id(s)].clone()
        dist.all_reduce(ref, op=dist.ReduceOp.SUM)
        expect[id(s)] = ref / dist.get_world_size()
    for i, s in enumerate(stores):
        torch.save({"got": s.grad.clone(), "expect": expect[id(s)]},
                   os.path.join(out, f"ov{rank}_{i}.pt"))
    with open(os.path.join(out, f"fired{rank}.json"), "w") as f:
        json.dump({"fired_during_backward": fired,
                   "buckets": [len(red.plan[id(s)]["buckets"]) for s in stores]}, f)


def main():
    out, mode = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "flat")
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    {"flat": flat, "overlap": overlap}[mode](out, rank)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
