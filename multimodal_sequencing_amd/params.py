"""Flat parameter store: every parameter of a component lives in ONE fp32 master buffer, its
gradient in ONE fp32 grad buffer, and its compute-dtype shadow (plus transposed shadows of the
matrices whose dgrad needs W^T as a K-contiguous operand) in compute-dtype buffers.

Why (MI355X-first): the optimizer is a single fused AdamW launch over the whole buffer, the
gradient norm one reduction, the data-parallel all-reduce runs on contiguous slices of the grad
buffer with no packing copies, and packed operands (Q|K|V weights of a BERT layer) are plain
views because the registration order places them back to back.

Drop-in surface: `named_parameters()` / `state_dict()` expose the reference's key names
 as nn.Parameter views sharing storage with the master buffer; `.grad` of each
view is the matching slice of the grad buffer.
"""
import math
import os
from collections import OrderedDict

import torch
from torch import nn

from . import _native as N

ALIGN = 64  # elements; keeps every tensor 256-B aligned in fp32 / 128-B in bf16


class Spec:
    __slots__ = ("name", "shape", "init", "decay", "transpose", "pack")

    def __init__(self, name, shape, init, decay=True, transpose=False, pack=None):
        self.name, self.shape, self.init = name, tuple(shape), init
        self.decay, self.transpose, self.pack = decay, transpose, pack


def _numel(shape):
    n = 1
    for s in shape:
        n *= s
    return n


class ParamStore:
    """Owns master / grad / shadow buffers for an ordered list of Specs.

    Specs with the same `pack` tag are laid out contiguously with no alignment padding between
    them so that the group is addressable as one matrix (e.g. packed QKV).
    """

    def __init__(self, specs, device, compute_dtype=torch.bfloat16):
        self.specs = list(specs)
        self.device = torch.device(device)
        self.compute_dtype = compute_dtype
        off = 0
        self.offsets = OrderedDict()
        prev_pack = None
        for s in self.specs:
            if s.pack is None or s.pack != prev_pack:
                off = (off + ALIGN - 1) // ALIGN * ALIGN
            self.offsets[s.name] = off
            off += _numel(s.shape)
            prev_pack = s.pack
        self.numel = (off + ALIGN - 1) // ALIGN * ALIGN
        # transposed shadows: one per transposed spec, or one per pack group of transposed specs
        self.tgroups = []
        for s in self.specs:
            if not s.transpose:
                continue
            if (s.pack is not None and self.tgroups and self.tgroups[-1][0] == s.pack):
                self.tgroups[-1][1].append(s.name)
            else:
                self.tgroups.append((s.pack, [s.name]))
        t_off = 0
        self.t_offsets = OrderedDict()
        for _, names in self.tgroups:
            self.t_offsets[names[0]] = (t_off, names)
            n = sum(_numel(self._spec(x).shape) for x in names)
            t_off += (n + ALIGN - 1) // ALIGN * ALIGN
        self.t_numel = t_off
        self.master = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        mask = torch.zeros(self.numel, dtype=torch.uint8)
        for s in self.specs:
            o = self.offsets[s.name]
            mask[o:o + _numel(s.shape)] = 0 if any(nd in s.name for nd in NO_DECAY) else 1
        self.decay_mask = mask.to(self.device)
        self._alloc_shadows()
        self.params = OrderedDict()
        for s in self.specs:
            o = self.offsets[s.name]
            p = nn.Parameter(self.master[o:o + _numel(s.shape)].view(s.shape))
            p.grad = self.grad[o:o + _numel(s.shape)].view(s.shape)
            self.params[s.name] = p
        self.shadow_stale = True
        self.version = 0  # bumped whenever the compute-dtype weights change (fp8 weight cache)
        # data-parallel hooks (trainer.GradAllReduce): a layer-level autograd Function reports
        # its grad span at the end of its backward (grad_ready) and its start (grad_begin)
        self.grad_hook = None
        self.begin_hook = None

    def span(self, names):
        """[lo, hi) of the buffer holding `names` (present ones), hi rounded up to the alignment
        so the dead padding after a unit belongs to it."""
        lo, hi = None, None
        for n in names:
            if n not in self.offsets:
                continue
            o = self.offsets[n]
            e = o + _numel(self._spec(n).shape)
            lo = o if lo is None else min(lo, o)
            hi = e if hi is None else max(hi, e)
        if lo is None:
            return None
        return (lo, min(self.numel, (hi + ALIGN - 1) // ALIGN * ALIGN))

    def grad_ready(self, span):
        if self.grad_hook is not None and span is not None:
            self.grad_hook(self, span)

    def grad_begin(self):
        if self.begin_hook is not None:
            self.begin_hook(self)

    def _alloc_shadows(self):
        if self.compute_dtype == torch.float32:
            self.shadow = self.master
        else:
            self.shadow = torch.zeros(self.numel, dtype=self.compute_dtype, device=self.device)
        self.shadow_t = torch.zeros(max(self.t_numel, 1), dtype=self.compute_dtype,
                                    device=self.device)

    def set_compute_dtype(self, dtype):
        if dtype != self.compute_dtype:
            self.compute_dtype = dtype
            self._alloc_shadows()
            self.shadow_stale = True

    # ---------------------------------------------------------------------------------------
    def init_weights(self, seed=0):
        g = torch.Generator(device="cpu").manual_seed(seed)
        host = torch.empty(self.numel, dtype=torch.float32)
        host.zero_()
        for s in self.specs:
            o, n = self.offsets[s.name], _numel(s.shape)
            host[o:o + n] = s.init(g, s.shape).reshape(-1)
        self.master.copy_(host.to(self.device))
        self.shadow_stale = True

    def load(self, state):
        """Copy a {name: tensor} mapping into the master buffer (missing names are an error)."""
        for s in self.specs:
            if s.name not in state:
                raise KeyError(f"missing parameter {s.name}")
            v = torch.as_tensor(state[s.name])
            if tuple(v.shape) != s.shape:
                raise ValueError(f"{s.name}: shape {tuple(v.shape)} != {s.shape}")
            self.params[s.name].data.copy_(v.to(self.device, torch.float32))
        self.shadow_stale = True

    def zero_grad(self):
        self.grad.zero_()

    def refresh_transposes(self):
        """Every transposed shadow from the master weights in one launch
        (mmseq_transpose_cast_batch; the descriptor table is built once)."""
        if not self.t_offsets:
            return
        if os.environ.get("MMSEQ_TBATCH", "1") == "0":  # A/B: one launch per matrix
            for first, (t, names) in self.t_offsets.items():
                src = self.packed(names, "f32")
                N.transpose_cast(src, self.shadow_t[t:t + src.numel()])
            return
        if getattr(self, "_tdesc", None) is None:
            rows_desc, tiles = [], 0
            for first, (t, names) in self.t_offsets.items():
                rows = sum(self._spec(x).shape[0] for x in names)
                cols = _numel(self._spec(first).shape) // self._spec(first).shape[0]
                rows_desc.append([rows, cols, self.offsets[first], t, tiles])
                tiles += ((rows + 63) // 64) * ((cols + 63) // 64)
            self._tdesc = torch.tensor(rows_desc, dtype=torch.int64, device=self.device)
            self._ttiles = tiles
        N.transpose_cast_batch(self._tdesc, self._ttiles, self.master, self.shadow_t)

    def refresh_shadows(self):
        """Re-derive the compute-dtype shadows from the master weights (after every update)."""
        if self.compute_dtype != torch.float32:
            N.cast(self.master, self.shadow)
        self.refresh_transposes()
        self.shadow_stale = False
        self.version += 1

    # ---------------------------------------------------------------------------------------
    def w(self, name):
        """compute-dtype shadow view."""
        s = self._spec(name)
        o = self.offsets[name]
        return self.shadow[o:o + _numel(s.shape)].view(s.shape)

    def wt(self, name):
        """compute-dtype transposed shadow [in][out] of the weight (or pack group) starting at
        `name`."""
        t, names = self.t_offsets[name]
        rows = sum(self._spec(x).shape[0] for x in names)
        cols = _numel(self._spec(names[0]).shape) // self._spec(names[0]).shape[0]
        return self.shadow_t[t:t + rows * cols].view(cols, rows)

    def f32(self, name):
        return self.params[name].data

    def g(self, name):
        return self.params[name].grad

    def packed(self, names, which="w"):
        """Contiguous view over a pack group (names in registration order)."""
        first, last = names[0], names[-1]
        o0 = self.offsets[first]
        o1 = self.offsets[last] + _numel(self._spec(last).shape)
        buf = {"w": self.shadow, "f32": self.master, "g": self.grad}[which]
        rows = sum(self._spec(n).shape[0] for n in names)
        return buf[o0:o1].view(rows, -1)

    def _spec(self, name):
        if not hasattr(self, "_spec_map"):
            self._spec_map = {s.name: s for s in self.specs}
        return self._spec_map[name]


# ------------------------------------------------------------------------------------------------
# init rules (reference): normal(0, 0.02) Linear/Embedding, zero bias, LN 1/0
# (lxrt/modeling.py:1244-1255, berson/modeling_bert.py:464-474); CLIP class/pos/proj
# scale*randn (clip/model.py:250-258); nn.LSTM U(-1/sqrt(H), 1/sqrt(H)).
def normal(std):
    return lambda g, shape: torch.randn(shape, generator=g) * std


def zeros(g, shape):
    return torch.zeros(shape)


def ones(g, shape):
    return torch.ones(shape)


def uniform(bound):
    return lambda g, shape: (torch.rand(shape, generator=g) * 2 - 1) * bound


def attach_tree(root: nn.Module, params, order=None):
    """Register each named nn.Parameter under nested container modules so that
    root.state_dict() / named_parameters() reproduce the reference's dotted key names. `order`
    (names -> names) sets the registration order where the reference's module order differs
    from the buffer layout (the submodules are created in first-seen order)."""
    names = list(params) if order is None else order(list(params))
    for name in names:
        p = params[name]
        parts = name.split(".")
        mod = root
        for part in parts[:-1]:
            if part not in mod._modules:
                mod.add_module(part, nn.Module())
            mod = mod._modules[part]
        mod.register_parameter(parts[-1], p)


def attach_buffers(root: nn.Module, buffers):
    """Register named tensors as module buffers under the dotted names (state_dict entries that
    are not parameters, e.g. BatchNorm running statistics)."""
    for name, t in buffers.items():
        parts = name.split(".")
        mod = root
        for part in parts[:-1]:
            if part not in mod._modules:
                mod.add_module(part, nn.Module())
            mod = mod._modules[part]
        mod.register_buffer(parts[-1], t)


def linear_specs(prefix, n_in, n_out, bias=True, std=0.02, transpose=True):
    out = [Spec(prefix + ".weight", (n_out, n_in), normal(std), transpose=transpose)]
    if bias:
        out.append(Spec(prefix + ".bias", (n_out,), zeros))
    return out


def ln_specs(prefix, width):
    return [Spec(prefix + ".weight", (width,), ones), Spec(prefix + ".bias", (width,), zeros)]


NO_DECAY = ("bias", "LayerNorm.weight")  # transformers AdamW grouping, trainers/train.py:172-183
