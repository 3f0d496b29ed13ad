"""Data-parallel logic on CPU: world_size-2 gloo process group, bucketed mean all-reduce of the
flat grad buffers (the same code path RCCL runs on the GPU box), and DistributedSampler-style
story sharding with no data-path collective."""
import os

import subprocess
import sys

import torch

from multimodal_sequencing_amd.trainer import linear_warmup_lr


def test_bucketed_allreduce_mean_gloo(tmp_path):
    world = 2
    port = 29500 + os.getpid() % 1000
    here = os.path.dirname(os.path.abspath(__file__))
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                    f"--nproc-per-node={world}", "--master-addr", "127.0.0.1", "--master-port",
                    str(port), os.path.join(here, "dist_worker.py"), str(tmp_path)],
                   check=True, timeout=240, env=dict(os.environ, OMP_NUM_THREADS="1"))
    res = [torch.load(tmp_path / f"grad{r}.pt") for r in range(world)]
    expect = sum(torch.randn(res[0].shape, generator=torch.Generator().manual_seed(r))
                 for r in range(world)) / world
    for r in range(world):
        torch.testing.assert_close(res[r], expect)
    assert torch.equal(res[0], res[1])  # bitwise identical across ranks


def test_warmup_schedule():
    assert linear_warmup_lr(0, 1.0, 100, 1000) == 0.0
    assert linear_warmup_lr(50, 1.0, 100, 1000) == 0.5
    assert linear_warmup_lr(100, 1.0, 100, 1000) == 1.0
    assert abs(linear_warmup_lr(550, 1.0, 100, 1000) - 0.5) < 1e-12
