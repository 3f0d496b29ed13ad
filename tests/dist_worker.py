"""Worker for tests/test_distributed_cpu.py (launched by torch.distributed.run, gloo backend)."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_sequencing_amd.params import ParamStore, Spec, normal  # noqa: E402
from multimodal_sequencing_amd.trainer import GradAllReduce  # noqa: E402


def main():
    out = sys.argv[1]
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    specs = [Spec("a.weight", (300, 7), normal(1.0)), Spec("b.bias", (5,), normal(1.0))]
    st = ParamStore(specs, "cpu", torch.float32)
    g = torch.Generator().manual_seed(rank)
    st.grad.copy_(torch.randn(st.grad.shape, generator=g))
    GradAllReduce([st], bucket_mb=0.001)()  # tiny buckets: many chunks in flight
    torch.save(st.grad.clone(), os.path.join(out, f"grad{rank}.pt"))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
