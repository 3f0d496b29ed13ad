"""Config 4's data-parallel reducer under a REAL autograd backward (trainers/train.py:217-221
wraps the model in DDP; here trainer.GradAllReduce fires bucketed all-reduces from the layer
backwards). Two ranks share the box's one GPU over gloo (tests/dist_worker.py mode "real"),
launched as a child process of this test by torch.distributed.run.

Checked: (1) every bucket's chunk, snapshotted at the instant its all-reduce is issued, equals
the rank's final local gradient of an unarmed backward of the same story bit for bit (the backward
is bit-stable: two unarmed backwards are compared first; a bucket issued early would miss whole
contributions) — no bucket fires before its gradients are final, including the BERSON head
store that counts as complete at the inner model's first backward begin (trainer.py
GradAllReduce._begin); (2) >= 10 buckets are issued during the backward itself, and every
unit-covered bucket is; (3) the averaged gradients are bitwise equal across ranks and equal
(local0 + local1) / 2 to rounding; (4) they match the single-process step over both stories (rtol 1e-5).
"""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_dp_reducer_real_backward_two_ranks(tmp_path):
    port = 29500 + (os.getpid() * 13) % 2000
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                    "--nproc-per-node=2", "--master-addr", "127.0.0.1", "--master-port",
                    str(port), os.path.join(HERE, "dist_worker.py"), str(tmp_path), "real"],
                   check=True, timeout=240, env=dict(os.environ, OMP_NUM_THREADS="4"))
    info = [json.load(open(tmp_path / f"real{r}.json")) for r in range(2)]
    res = [torch.load(tmp_path / f"real{r}.pt") for r in range(2)]
    single = torch.load(tmp_path / "single.pt")
    for r, it in enumerate(info):
        print(f"rank {r}: {it['buckets']} buckets, {it['fired_in_backward']} issued during the "
              f"backward, run-to-run differences {it['nondeterministic']}")
    for r, it in enumerate(info):
        assert it["nondeterministic"] == [], (r, it["nondeterministic"])  # bit-stable backward
        assert it["early"] == [], (r, it["early"], it["fired"])  # no chunk changed after it fired
        assert it["snapshots"] == it["buckets"]
        assert it["fired_in_backward"] >= 10, it
        assert it["unit_buckets_in_finish"] == 0, it  # only orphan spans wait for finish()
    assert abs((info[0]["loss"] + info[1]["loss"]) / 2 - info[0]["single_loss"]) < 1e-5
    for i in range(len(single)):
        g0, g1 = res[0]["grad"][i], res[1]["grad"][i]
        assert torch.equal(g0, g1), i  # bitwise identical on both ranks
        scale = float(single[i].abs().max())
        torch.testing.assert_close(g0, (res[0]["local"][i] + res[1]["local"][i]) / 2,
                                   rtol=1e-5, atol=1e-6 * scale)
        torch.testing.assert_close(g0, single[i], rtol=1e-5, atol=1e-6 * scale)


def test_rccl_reducer_world1(tmp_path):
    """The reducer's RCCL branch (ReduceOp.AVG, trainer.py GradAllReduce._fire) executed on the
    box's GPU: backend "nccl" at world size 1 (RCCL refuses two ranks on one GPU), the reducer
    forced on, buckets issued during the real backward and finished; at world 1 the mean is the
    local gradient bit for bit."""
    port = 29500 + (os.getpid() * 17 + 7) % 2000
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                    "--nproc-per-node=1", "--master-addr", "127.0.0.1", "--master-port",
                    str(port), os.path.join(HERE, "dist_worker.py"), str(tmp_path), "rccl"],
                   check=True, timeout=240, env=dict(os.environ, OMP_NUM_THREADS="4"))
    it = json.load(open(tmp_path / "rccl0.json"))
    print(f"RCCL {it['rccl_version']}: backend {it['backend']}, {it['buckets']} buckets, "
          f"{it['fired_in_backward']} issued during the backward ({it['avg_ops']} AVG)")
    assert it["backend"] == "nccl" and it["world"] == 1
    assert it["avg_bucket_equal"]
    assert it["armed"] and it["fired_in_backward"] >= 10
    assert it["avg_ops"] == it["fired_in_backward"]  # the RCCL AVG branch, not gloo's SUM + div
    assert it["max_rel_diff"] == 0.0, it
