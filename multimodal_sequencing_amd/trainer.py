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
    """transformers get_linear_schedule_with_warmup lambda (train.py:186-190) at scheduler step
    `step` (0-based: LambdaLR evaluates lambda(0) at construction)."""
    if step < warmup:
        return base_lr * step / max(1, warmup)
    return base_lr * max(0.0, (total - step) / max(1, total - warmup))


def distributed_indices(n, world, rank, shuffle=True, seed=0, epoch=0):
    """torch.utils.data.DistributedSampler's index rule (train.py:158-161: the sampler is built
    with its defaults and never gets set_epoch, so epoch stays 0): a seeded permutation (or
    arange), padded by wrapping to a multiple of `world`, then every world-th index from `rank`."""
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        idx = torch.randperm(n, generator=g).tolist()
    else:
        idx = list(range(n))
    per = math.ceil(n / world)
    total = per * world
    pad = total - len(idx)
    if pad > 0:
        idx += (idx * math.ceil(pad / len(idx)))[:pad]
    return idx[rank:total:world]


class FusedAdamW:
    """transformers-3.4 AdamW + get_linear_schedule_with_warmup + clip_grad_norm_, one fused
    kernel per flat store. The k-th update (1-based) uses lr = lambda(k - 1), because the
    reference builds LambdaLR (lambda(0) at construction) and calls scheduler.step() after
    optimizer.step() (train.py:185-190, 361-362); Adam's bias correction uses k."""

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

    def current_lr(self):
        """lr the next step() applies (scheduler.get_last_lr() before that step)."""
        return linear_warmup_lr(self.step_count, self.lr, self.warmup, self.total)

    def step(self):
        lr = self.current_lr()
        self.step_count += 1
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
            s.version += 1
            if s.compute_dtype == torch.bfloat16:
                s.shadow_stale = False
                s.refresh_transposes()
            else:
                s.refresh_shadows()
        return lr

    # -- checkpoint/resume (trainers/train.py:193-201, 411-413) ---------------------------------
    def _param_slots(self, model):
        """[(name, store index, offset, numel)] in model.named_parameters() order (tied
        parameters once), split into the reference's two groups (train.py:172-183): decay
        first, then bias / LayerNorm.weight."""
        where = {}
        for i, s in enumerate(self.stores):
            base = s.master.data_ptr()
            for name, p in s.params.items():
                where[p.data_ptr()] = (i, (p.data_ptr() - base) // 4, p.numel())
        from .params import NO_DECAY
        groups = ([], [])
        for name, p in model.named_parameters():
            if p.data_ptr() not in where:
                raise ValueError(f"parameter {name} is not in the optimizer's stores")
            i, off, n = where[p.data_ptr()]
            groups[1 if any(nd in name for nd in NO_DECAY) else 0].append((name, i, off, n))
        return groups

    def state_dict(self, model):
        """transformers AdamW.state_dict() layout: {'state': {index: {'step', 'exp_avg',
        'exp_avg_sq'}}, 'param_groups': [decay group, no-decay group]}, indices running over
        the groups in model.named_parameters() order. Each group also carries 'param_names'
        (ignored by torch's loader) so a resume can match by name."""
        state, groups, idx = {}, [], 0
        for gi, slots in enumerate(self._param_slots(model)):
            ids = []
            for name, i, off, n in slots:
                shape = model.get_parameter(name).shape
                if self.step_count > 0:
                    state[idx] = {"step": self.step_count,
                                  "exp_avg": self.m[i][off:off + n].view(shape).cpu().clone(),
                                  "exp_avg_sq": self.v[i][off:off + n].view(shape).cpu().clone()}
                ids.append(idx)
                idx += 1
            groups.append({"lr": self.current_lr(), "betas": tuple(self.betas), "eps": self.eps,
                           "weight_decay": self.wd if gi == 0 else 0.0, "correct_bias": True,
                           "initial_lr": self.lr, "params": ids,
                           "param_names": [s[0] for s in slots]})
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, model, sd):
        """Restore moments and step from an AdamW state dict written by state_dict() or by the
        reference's torch.save(optimizer.state_dict()). Parameters are matched by 'param_names'
        when present, else by position in the reference's group order."""
        slots = self._param_slots(model)
        by_name = {s[0]: s for g in slots for s in g}
        saved = sd["param_groups"]
        if len(saved) != len(slots):
            raise ValueError(f"optimizer state has {len(saved)} groups, expected {len(slots)}")
        steps = set()
        for gi, g in enumerate(saved):
            names = g.get("param_names")
            if names is None:
                if len(g["params"]) != len(slots[gi]):
                    raise ValueError(f"group {gi}: {len(g['params'])} params in the state, "
                                     f"{len(slots[gi])} in the model")
                targets = slots[gi]
            else:
                targets = [by_name[n] for n in names]
            for pid, (name, i, off, n) in zip(g["params"], targets):
                st = sd["state"].get(pid, sd["state"].get(str(pid)))
                if st is None:
                    continue
                self.m[i][off:off + n].copy_(st["exp_avg"].reshape(-1).to(self.m[i].device))
                self.v[i][off:off + n].copy_(st["exp_avg_sq"].reshape(-1).to(self.v[i].device))
                steps.add(int(st["step"]))
        if len(steps) > 1:
            raise ValueError(f"parameters were saved at different steps {sorted(steps)}")
        self.step_count = steps.pop() if steps else 0

    def scheduler_state_dict(self):
        """torch LambdaLR.state_dict() of get_linear_schedule_with_warmup after `step_count`
        scheduler.step() calls (train.py:361-362), for scheduler.pt."""
        lr = self.current_lr()
        return {"base_lrs": [self.lr, self.lr], "last_epoch": self.step_count,
                "_step_count": self.step_count + 1, "verbose": False,
                "_get_lr_called_within_step": False, "_last_lr": [lr, lr],
                "lr_lambdas": [None, None]}

    def load_scheduler_state_dict(self, sd):
        self.step_count = int(sd["last_epoch"])

    def save(self, model, directory):
        """optimizer.pt + scheduler.pt next to a save_pretrained checkpoint."""
        from .checkpoint import OPTIMIZER_NAME, SCHEDULER_NAME
        torch.save(self.state_dict(model), f"{directory}/{OPTIMIZER_NAME}")
        torch.save(self.scheduler_state_dict(), f"{directory}/{SCHEDULER_NAME}")

    def load(self, model, directory):
        """train.py:193-201: resume both when both files exist; returns whether it did."""
        import os
        from .checkpoint import OPTIMIZER_NAME, SCHEDULER_NAME, load_weights_file
        o, s = os.path.join(directory, OPTIMIZER_NAME), os.path.join(directory, SCHEDULER_NAME)
        if not (os.path.isfile(o) and os.path.isfile(s)):
            return False
        self.load_state_dict(model, load_weights_file(o))
        self.load_scheduler_state_dict(load_weights_file(s))
        return True


class GradAllReduce:
    """Data-parallel gradient mean over RCCL (backend "nccl" on ROCm), overlapped with backward.

    The reference wraps the model in DDP (train.py:217-221), whose reducer all-reduces 25 MB
    buckets from autograd hooks. Here every store's flat grad buffer is cut into contiguous
    buckets (<= bucket_mb) at the boundaries of its backward units — one unit per layer-level
    autograd Function (a BERT layer, a ViT block, the stem, the projection, the joint input),
    each a contiguous span of the buffer. The Functions report their unit at the end of their
    backward (ParamStore.grad_ready); a bucket's async all-reduce is issued as soon as every unit
    overlapping it has reported, so RCCL runs on its own stream beside the remaining backward.
    Spans no unit covers (parameters without a gradient on this path, or written by ops that
    do not report) form their own buckets, issued by finish(). Stores listed in `begin_units`
    count as complete when the first unit of another store reports a backward begin (the BERSON
    head: autograd runs all of its nodes before the inner model's last layer). Only the last
    micro-batch's backward is armed; finish() issues what is left and waits for every bucket.
    `force=True` arms the reducer at world size 1 as well (an initialised group is required), so
    that the RCCL path runs end to end on a one-GPU box.
    """

    def __init__(self, stores, bucket_mb=64, units=None, begin_units=(), group=None, force=False):
        self.stores = list(stores)
        self.force = bool(force)
        # diagnostics (bench.py at N > 1): per finish(), the buckets issued during the backward
        # and the exposed all-reduce time = GPU time the compute stream waits in finish() after
        # the last backward kernel (events on the compute stream around the waits)
        self.timing = False
        self.records = []
        self.cap = max(1, int(bucket_mb * (1 << 20)) // 4)
        self.group = group
        self.armed = False
        self.works = []
        self.begin_units = set(id(s) for s in begin_units)
        units = units or {}
        self.plan = {}
        for s in self.stores:
            spans = list(units.get(id(s), []))
            if id(s) in self.begin_units:
                spans = [(0, s.numel)]
            self.plan[id(s)] = self._make_buckets(s, spans)
            s.grad_hook = self._ready
            s.begin_hook = self._begin

    @staticmethod
    def _pieces(numel, spans):
        """Partition [0, numel) into (lo, hi, unit index or -1) pieces in memory order."""
        cover = sorted((lo, hi, u) for u, (lo, hi) in enumerate(spans))
        out, pos = [], 0
        for lo, hi, u in cover:
            if lo < pos:
                raise ValueError("grad units overlap")
            if lo > pos:
                out.append((pos, lo, -1))
            out.append((lo, hi, u))
            pos = hi
        if pos < numel:
            out.append((pos, numel, -1))
        return out

    def _make_buckets(self, store, spans):
        """Buckets = contiguous [lo, hi) ranges: runs of whole units up to the cap (a unit larger
        than the cap is one bucket), and cap-sized pieces of the uncovered ranges."""
        buckets, cur = [], None  # bucket = [lo, hi, unit set, orphan]
        for lo, hi, u in self._pieces(store.numel, spans):
            if u < 0:
                while lo < hi:
                    take = min(hi - lo, self.cap)
                    buckets.append([lo, lo + take, set(), True])
                    lo += take
                cur = None
                continue
            if cur is None or cur[1] - cur[0] + (hi - lo) > self.cap:
                cur = [lo, lo, set(), False]
                buckets.append(cur)
            cur[1] = hi
            cur[2].add(u)
        span2unit = {tuple(sp): i for i, sp in enumerate(spans)}
        unit2b = {u: [j for j, bk in enumerate(buckets) if u in bk[2]] for u in range(len(spans))}
        return {"buckets": buckets, "span2unit": span2unit, "unit2b": unit2b}

    def _world(self):
        if not (dist.is_available() and dist.is_initialized()):
            return 1
        return dist.get_world_size(self.group)

    def arm(self, on):
        """Arm (last micro-batch) or disarm the backward-driven all-reduce."""
        self.armed = bool(on) and (self._world() > 1 or self.force)
        if self.armed:
            self.works = []
            for s in self.stores:
                pl = self.plan[id(s)]
                pl["pending"] = [set(b[2]) for b in pl["buckets"]]
                pl["fired"] = [False] * len(pl["buckets"])

    def _fire(self, store, j):
        pl = self.plan[id(store)]
        if pl["fired"][j]:
            return
        pl["fired"][j] = True
        lo, hi = pl["buckets"][j][:2]
        chunk = store.grad[lo:hi]
        avg = dist.get_backend(self.group) == "nccl"  # RCCL has ReduceOp.AVG; gloo does not
        op = dist.ReduceOp.AVG if avg else dist.ReduceOp.SUM
        self.works.append((dist.all_reduce(chunk, op=op, group=self.group, async_op=True),
                           chunk, avg))

    def _ready(self, store, span):
        if not self.armed:
            return
        pl = self.plan[id(store)]
        u = pl["span2unit"].get(tuple(span))
        if u is None:
            return
        for j in pl["unit2b"][u]:
            pl["pending"][j].discard(u)
            if not pl["pending"][j] and not pl["buckets"][j][3]:
                self._fire(store, j)

    def _begin(self, store):
        if not self.armed:
            return
        for s in self.stores:
            if id(s) in self.begin_units and s is not store:
                self._ready(s, (0, s.numel))

    def finish(self):
        """Issue every bucket not yet issued and wait for all (grads are the mean afterwards)."""
        world = self._world()
        if world == 1 and not self.force:
            return
        if not self.armed:
            self.arm(True)
        in_backward = len(self.works)
        e0 = None
        if self.timing and torch.cuda.is_available() and self.stores[0].grad.is_cuda:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        for s in self.stores:
            for j in range(len(self.plan[id(s)]["buckets"])):
                self._fire(s, j)
        total = len(self.works)
        for w, chunk, avg in self.works:
            w.wait()
            if not avg:
                chunk.div_(world)
        if e0 is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self.records.append((e0, e1, total, in_backward))
        self.works = []
        self.armed = False

    def timing_summary(self):
        """Mean exposed all-reduce ms per finish() and the bucket counts (after a synchronize)."""
        if not self.records:
            return None
        ms = [a.elapsed_time(b) for a, b, _, _ in self.records]
        return {"exposed_ms_mean": sum(ms) / len(ms), "exposed_ms_max": max(ms),
                "buckets": self.records[-1][2], "issued_in_backward": self.records[-1][3],
                "steps": len(ms)}

    __call__ = finish


def train_step(model, optimizer, batches, reducer=None):
    """One optimizer step over `batches` (micro-batches of one per-rank batch).
    Returns the (device) mean loss."""
    total = sum(b["input_ids"].shape[0] for b in batches)
    loss_sum = None
    for i, b in enumerate(batches):
        if reducer is not None:
            reducer.arm(i == len(batches) - 1)
        loss = model(b)[0] * (b["input_ids"].shape[0] / total)
        loss.backward()
        loss_sum = loss.detach() if loss_sum is None else loss_sum + loss.detach()
    if reducer is not None:
        reducer.finish()
    optimizer.step()
    model.zero_grad()
    return loss_sum
