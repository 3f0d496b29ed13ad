"""Worker for tests/test_distributed_cpu.py (launched by torch.distributed.run, gloo backend).

mode "flat":    bucketed mean all-reduce of a small store issued by finish() alone.
mode "overlap": the product model's real grad layout (tiny golden config on CPU); a simulated
                backward writes each unit's gradient and reports it in backward order, exactly
                as the layer Functions do, with the reducer armed; buckets must be issued
                during the "backward" and the result must equal one flat all-reduce.
mode "real":    GPU (every rank on cuda:0, gloo): the product model (fp32, eval) under a REAL
                loss.backward() with the reducer armed; one story per rank. Every bucket's
                chunk is snapshotted at the moment it is issued and compared with the rank's
                final local gradient from an unarmed backward of the same story (a bucket that
                fired before its gradients were final differs); rank 0 also runs the
                single-process step over all the ranks' stories for the parent to compare.
mode "rccl":    GPU, backend "nccl" (= RCCL) at world size 1 on the box's one GPU: a bucket-sized
                all_reduce(AVG), then the product model's real backward with the reducer forced
                on (GradAllReduce(force=True)), so _fire / finish run their RCCL branch
                (ReduceOp.AVG, no host-side division) end to end.
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


REAL_CFG = {"B": 2, "N": 5, "per_seq": 8, "ragged": False, "text_only": False,
            "vit": {"embed": 96, "res": 32, "layers": 5, "width": 128, "patch": 8},
            "joint": {"vocab": 300, "hidden": 128, "layers": 6, "heads": 2, "inter": 512,
                      "max_pos": 514},
            "head": {"ff": 256, "heads": 8, "layers": 2}}


def real_inputs(world, seed=7):
    """`world` equal-length stories (make_golden.make_inputs layout), one per rank."""
    import numpy as np
    c = REAL_CFG
    g = np.random.RandomState(seed)
    B, N, k = world, c["N"], c["per_seq"] - 2
    ids = np.ones((B, N * c["per_seq"]), dtype=np.int64)
    for b in range(B):
        ids[b] = np.concatenate([[0] + list(g.randint(3, c["joint"]["vocab"], size=k)) + [2]
                                 for _ in range(N)])
    labels = np.stack([np.argsort(g.permutation(N)) for _ in range(B)]).astype(np.int64)
    R = c["vit"]["res"]
    images = g.standard_normal((B, N, 3, R, R)).astype(np.float32)
    return {"input_ids": torch.from_numpy(ids), "labels": torch.from_numpy(labels),
            "images": torch.from_numpy(images)}


def real(out, rank):
    from multimodal_sequencing_amd import model_zoo
    world = dist.get_world_size()
    dev = "cuda:0"  # every rank shares the box's one GPU
    m = model_zoo.build_from_golden(REAL_CFG, device=dev)
    m.eval()
    stores = m.stores()
    allin = real_inputs(world)
    mine = {k: v[rank:rank + 1] for k, v in allin.items()}
    # (1) unarmed backward of this rank's story: the final local gradient
    local = None
    for rep in range(2):  # twice: the unarmed backward must itself be bitwise reproducible
        m.zero_grad()
        m(mine)[0].backward()
        torch.cuda.synchronize()
        again = [s.grad.clone() for s in stores]
        if local is None:
            local = again
    nondet = [(i, float((a - b).abs().max()), float(a.abs().max()))
              for i, (a, b) in enumerate(zip(local, again)) if not torch.equal(a, b)]
    # (2) the same backward with the reducer armed; snapshot each chunk when it is issued
    units, begin = m.ddp_units()
    red = GradAllReduce(stores, bucket_mb=0.05, units=units, begin_units=begin)
    snaps, phase = [], ["backward"]
    fire = red._fire

    def spy(store, j):
        pl = red.plan[id(store)]
        if not pl["fired"][j]:
            lo, hi = pl["buckets"][j][:2]
            snaps.append((stores.index(store), lo, hi, store.grad[lo:hi].clone(), phase[0]))
        fire(store, j)

    red._fire = spy
    m.zero_grad()
    red.arm(True)
    loss = m(mine)[0]
    loss.backward()
    in_backward = len(red.works)
    phase[0] = "finish"
    red.finish()
    torch.cuda.synchronize()
    # the backward is bit-stable (fixed-order sums everywhere, `nondeterministic` must be empty),
    # so every bucket's chunk at issue time must equal the final local gradient bit for bit; a
    # bucket issued before its gradients were final would miss whole contributions
    bad = []
    for i, lo, hi, snap, _ in snaps:
        ref = local[i][lo:hi]
        if not torch.equal(snap, ref):
            bad.append((i, lo, hi, float((snap - ref).abs().max()), float(ref.abs().max())))
    total = sum(len(red.plan[id(s)]["buckets"]) for s in stores)
    res = {"fired_in_backward": in_backward, "buckets": total, "snapshots": len(snaps),
           "early": bad, "loss": float(loss.detach()), "nondeterministic": nondet,
           "fired": [(i, lo, hi, ph) for i, lo, hi, _, ph in snaps],
           "unit_buckets_in_finish": sum(1 for i, lo, hi, _, ph in snaps if ph == "finish" and
                                         any(b[:2] == [lo, hi] and b[2] for b in
                                             red.plan[id(stores[i])]["buckets"]))}
    torch.save({"grad": [s.grad.cpu() for s in stores], "local": [x.cpu() for x in local]},
               os.path.join(out, f"real{rank}.pt"))
    if rank == 0:  # (3) one process, all stories in one batch (the DP mean's target)
        m.zero_grad()
        full = m(allin)[0]
        full.backward()
        torch.cuda.synchronize()
        torch.save([s.grad.cpu() for s in stores], os.path.join(out, "single.pt"))
        res["single_loss"] = float(full)
    with open(os.path.join(out, f"real{rank}.json"), "w") as f:
        json.dump(res, f)


def rccl(out, rank):
    from multimodal_sequencing_amd import model_zoo
    dev = torch.device("cuda", 0)
    res = {"backend": dist.get_backend(), "world": dist.get_world_size(),
           "rccl_version": ".".join(str(v) for v in torch.cuda.nccl.version())}
    # a 64 MB bucket (the reducer's default cap) through all_reduce(AVG)
    x = torch.randn(16 << 20, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
    want = x.clone()
    dist.all_reduce(x, op=dist.ReduceOp.AVG)
    torch.cuda.synchronize()
    res["avg_bucket_equal"] = bool(torch.equal(x, want))
    # the product model's backward with the RCCL reducer armed at world 1
    m = model_zoo.build_from_golden(REAL_CFG, device=dev)
    m.eval()
    stores = m.stores()
    mine = {k: v[:1] for k, v in real_inputs(1).items()}
    m.zero_grad()
    m(mine)[0].backward()
    torch.cuda.synchronize()
    local = [s.grad.clone() for s in stores]
    units, begin = m.ddp_units()
    red = GradAllReduce(stores, bucket_mb=0.05, units=units, begin_units=begin, force=True)
    m.zero_grad()
    red.arm(True)
    res["armed"] = red.armed
    m(mine)[0].backward()
    res["fired_in_backward"] = len(red.works)
    res["avg_ops"] = sum(1 for _, _, avg in red.works if avg)
    red.finish()
    torch.cuda.synchronize()
    res["buckets"] = sum(len(red.plan[id(s)]["buckets"]) for s in stores)
    res["max_rel_diff"] = max(float((s.grad - g).abs().max()) / (float(g.abs().max()) + 1e-30)
                              for s, g in zip(stores, local))
    with open(os.path.join(out, f"rccl{rank}.json"), "w") as f:
        json.dump(res, f)


def main():
    out, mode = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "flat")
    if mode == "rccl":
        torch.cuda.set_device(0)
    dist.init_process_group("nccl" if mode == "rccl" else "gloo")
    rank = dist.get_rank()
    {"flat": flat, "overlap": overlap, "real": real, "rccl": rccl}[mode](out, rank)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
