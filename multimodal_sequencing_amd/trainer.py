"""Training step with the reference's semantics (trainers/train.py:147-465, hot loop 275-363):
  loss = model(inputs)[0]; loss.backward()        (gradient accumulation over micro-batches)
  clip_grad_norm_(params, max_grad_norm = 1.0)     (:358-360)
  AdamW(lr, eps=1e-8, weight_decay, transformers-3.4 semantics) + linear warmup (:172-190)
  model.zero_grad()                                 (:363)
MI355X-first: the optimizer is ONE fused kernel per flat parameter store (clip factor read on
device from the fused sum-of-squares, no host sync), and the bf16 weight shadows are refreshed
in the same pass. Data parallelism: one process per GPU; the flat fp32 grad buffers are
all-reduced (mean) with RCCL in fixed-size buckets, launched asynchronously.
"""
import math

import torch
import torch.distributed as dist

from . import _native as N


def linear_warmup_lr(step, base_lr, warmup, total):
    """transformers get_linear_schedule_with_warmup (train.py:186-190)."""
    if step < warmup:
        return base_lr * step / max(1, warmup)
    return base_lr * max(0.0, (total - step) / max(1, total - warmup))


class FusedAdamW:
    def __init__(self, stores, lr=5e-6, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 max_grad_norm=1.0, warmup=100, total_steps=10 ** 9):
        self.stores = stores
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.max_grad_norm = max_grad_norm
        self.warmup, self.total = warmup, total_steps
        self.step_count = 0
        self.m = [torch.zeros_like(s.master) for s in stores]
        self.v = [torch.zeros_like(s.master) for s in stores]
        dev = stores[0].master.device
        self._ss = torch.zeros(len(stores) + 1, device=dev)

    def step(self):
        self.step_count += 1
        lr = linear_warmup_lr(self.step_count, self.lr, self.warmup, self.total)
        # global grad norm over all stores (clip_grad_norm_ over model.parameters())
        for i, s in enumerate(self.stores):
            N.sumsq(s.grad, self._ss[i:i + 1])
        total = self._ss[-1:]
        torch.sum(self._ss[:-1], dim=0, keepdim=True, out=total)
        for i, s in enumerate(self.stores):
            shadow = s.shadow if s.compute_dtype == torch.bfloat16 else None
            N.adamw(s.master, s.grad, self.m[i], self.v[i], s.decay_mask, lr, self.betas[0],
                    self.betas[1], self.eps, self.wd, self.step_count, self.max_grad_norm, total,
                    shadow)
            # transposed shadows (dgrad operands) from the updated master weights
            if s.compute_dtype == torch.bfloat16:
                s.shadow_stale = False
                for first, (t, names) in s.t_offsets.items():
                    src = s.packed(names, "f32")
                    N.transpose_cast(src, s.shadow_t[t:t + src.numel()])
            else:
                s.refresh_shadows()
        return lr


class GradAllReduce:
    """Bucketed mean all-reduce of the flat grad buffers over RCCL (backend "nccl" on ROCm)."""

    def __init__(self, stores, bucket_mb=64):
        self.stores = stores
        self.bucket = max(1, int(bucket_mb * (1 << 20)) // 4)

    def __call__(self):
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            return
        world = dist.get_world_size()
        avg = dist.get_backend() == "nccl"  # RCCL has ReduceOp.AVG; gloo (CPU tests) does not
        works = []
        for s in self.stores:
            g = s.grad
            for o in range(0, g.numel(), self.bucket):
                op = dist.ReduceOp.AVG if avg else dist.ReduceOp.SUM
                works.append((dist.all_reduce(g[o:o + self.bucket], op=op, async_op=True),
                              g[o:o + self.bucket]))
        for w, chunk in works:
            w.wait()
            if not avg:
                chunk.div_(world)


def train_step(model, optimizer, batches, reducer=None):
    """One optimizer step over `batches` (micro-batches of one per-rank batch).
    Returns the (device) mean loss."""
    total = sum(b["input_ids"].shape[0] for b in batches)
    loss_sum = None
    for b in batches:
        loss = model(b)[0] * (b["input_ids"].shape[0] / total)
        loss.backward()
        loss_sum = loss.detach() if loss_sum is None else loss_sum + loss.detach()
    if reducer is not None:
        reducer()
    optimizer.step()
    model.zero_grad()
    return loss_sum
