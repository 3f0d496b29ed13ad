"""Data-parallel logic on CPU: world_size-2 gloo process groups running the same reducer code
RCCL runs on the GPU box (bucketed mean all-reduce of the flat grad buffers, issued from the
layer backwards), DistributedSampler story sharding, and the reference's LR schedule."""
import json
import os
import subprocess
import sys

import pytest
import torch

from multimodal_sequencing_amd.trainer import FusedAdamW, distributed_indices, linear_warmup_lr

HERE = os.path.dirname(os.path.abspath(__file__))


def _launch(tmp_path, mode, world=2):
    port = 29500 + (os.getpid() * 7 + len(mode)) % 2000
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                    f"--nproc-per-node={world}", "--master-addr", "127.0.0.1", "--master-port",
                    str(port), os.path.join(HERE, "dist_worker.py"), str(tmp_path), mode],
                   check=True, timeout=300, env=dict(os.environ, OMP_NUM_THREADS="1"))


@pytest.mark.parametrize("world", [2, 4])
def test_bucketed_allreduce_mean_gloo(tmp_path, world):
    _launch(tmp_path, "flat", world)
    res = [torch.load(tmp_path / f"grad{r}.pt") for r in range(world)]
    expect = sum(torch.randn(res[0].shape, generator=torch.Generator().manual_seed(r))
                 for r in range(world)) / world
    for r in range(world):
        torch.testing.assert_close(res[r], expect)
        assert torch.equal(res[0], res[r])  # bitwise identical across ranks


@pytest.mark.parametrize("world", [2, 4])
def test_overlapped_backward_allreduce_gloo(tmp_path, world):
    """Buckets issued from the unit reports during the (simulated) backward give the same mean
    as one all-reduce of the whole buffer (bitwise at 2 ranks), bitwise identical on every rank,
    and most of them are in flight before the backward ends (2 ranks, and 4 as a rehearsal of
    the wider node)."""
    _launch(tmp_path, "overlap", world)
    for r in range(world):
        for i in range(2):
            d = torch.load(tmp_path / f"ov{r}_{i}.pt")
            if world == 2:  # a sum of two is order-free: bitwise equal to the flat all-reduce
                assert torch.equal(d["got"], d["expect"]), (r, i)
            else:  # more ranks: the collective's summation order depends on the bucket size
                torch.testing.assert_close(d["got"], d["expect"], rtol=1e-6, atol=1e-7)
        if r:
            for i in range(2):
                assert torch.equal(torch.load(tmp_path / f"ov0_{i}.pt")["got"],
                                   torch.load(tmp_path / f"ov{r}_{i}.pt")["got"])
    info = json.load(open(tmp_path / "fired0.json"))
    fired = info["fired_during_backward"]
    assert fired == sorted(fired) and fired[0] >= 1  # the head's buckets go at the first begin
    total = sum(info["buckets"])
    assert fired[-1] >= total // 2, (fired, total)  # overlap: issued before finish()


@pytest.mark.parametrize("n,world", [(64, 2), (64, 8), (10, 4), (7, 3)])
@pytest.mark.parametrize("shuffle", [True, False])
def test_distributed_indices_match_sampler(n, world, shuffle):
    from torch.utils.data import DistributedSampler
    data = list(range(n))
    for rank in range(world):
        ref = list(DistributedSampler(data, num_replicas=world, rank=rank, shuffle=shuffle))
        assert distributed_indices(n, world, rank, shuffle=shuffle) == ref


def test_warmup_schedule():
    assert linear_warmup_lr(0, 1.0, 100, 1000) == 0.0
    assert linear_warmup_lr(50, 1.0, 100, 1000) == 0.5
    assert linear_warmup_lr(100, 1.0, 100, 1000) == 1.0
    assert abs(linear_warmup_lr(550, 1.0, 100, 1000) - 0.5) < 1e-12


def test_lr_sequence_matches_lambdalr():
    """The k-th update uses lambda(k - 1): LambdaLR evaluates lambda(0) at construction and the
    reference calls scheduler.step() after optimizer.step() (train.py:185-190, 361-362)."""
    warm, total, base = 4, 10, 5e-6
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=base)
    sched = torch.optim.lr_scheduler.LambdaLR(
        opt, lambda s: s / max(1, warm) if s < warm else max(0.0, (total - s) / max(1, total - warm)))
    store = type("S", (), {"master": torch.zeros(4)})()
    ours = FusedAdamW([store], lr=base, warmup=warm, total_steps=total)
    for _ in range(total + 2):
        ref_lr = opt.param_groups[0]["lr"]  # the lr optimizer.step() applies now
        assert abs(ours.current_lr() - ref_lr) < 1e-18, (ours.step_count, ours.current_lr(), ref_lr)
        opt.step()
        sched.step()
        ours.step_count += 1
