"""Pair expansion for BERSON (models/berson/process_inputs_for_berson.py:13-368).

On a GPU device the expansion runs as two HIP kernels (csrc/pairs.hip): a
per-story scan (step boundaries, gold ranks, pairwise labels, </s> positions, the batch's
longest pair) and the pair-row expansion. The pair length is the data-dependent max over the
batch (the reference pads to it, and — quirk App. C.7 — pads are ATTENDED because the pair mask
is padded with pad_id = 1), so it sizes the outputs: ONE int32 pair is read back per batch.
`prepare_berson_inputs_host` is the same computation in numpy (CPU tensors / CPU models).
Images are NOT duplicated per pair here (the reference's process_images copies each image into
8 pairs): the device kernels gather them by `pairs_list` (mmseq_vit_im2col).
"""
import itertools

import numpy as np
import torch

CLS_ID, PAD_ID, SEP_ID = 0, 1, 2


def pairs_generator(n):
    """:246-261 — combinations(i<j) followed by the reversed pairs."""
    one = [[a, b] for a, b in itertools.combinations(range(n), 2)]
    return one + [[b, a] for a, b in one], n * (n - 1)


def _split_steps(row, n_steps, cls_id, sep_id):
    """parse_input_ids (:100-110): step i = row[start_i : end_i + 1]."""
    starts = np.flatnonzero(row == cls_id)
    ends = np.flatnonzero(row == sep_id)
    if len(starts) != len(ends) or len(starts) != n_steps:
        raise ValueError(f"story has {len(starts)} <s> / {len(ends)} </s> markers, "
                         f"expected {n_steps} steps (process_inputs_for_berson.py:104,136)")
    return starts, ends


def prepare_berson_inputs(input_ids, labels, n_steps, cls_id=CLS_ID, sep_id=SEP_ID, pad_id=PAD_ID,
                          device=None):
    """Returns the reference's berson_inputs dict (:47-60) as int64 tensors (on `device`): by the
    device kernels when `device` is a GPU, else on the host."""
    if device is not None and torch.device(device).type == "cuda":
        return prepare_berson_inputs_device(input_ids, labels, n_steps, cls_id, sep_id, pad_id,
                                            device)
    return prepare_berson_inputs_host(input_ids, labels, n_steps, cls_id, sep_id, pad_id, device)


_PAIRS_CACHE = {}


def _pairs_on(device, n_steps):
    key = (str(device), n_steps)
    if key not in _PAIRS_CACHE:
        _PAIRS_CACHE[key] = torch.tensor(pairs_generator(n_steps)[0], dtype=torch.int64,
                                         device=device)
    return _PAIRS_CACHE[key]


def prepare_berson_inputs_device(input_ids, labels, n_steps, cls_id=CLS_ID, sep_id=SEP_ID,
                                 pad_id=PAD_ID, device="cuda"):
    """mmseq_pair_scan + mmseq_pair_expand; host ids are copied to the device first."""
    from . import _native as NT
    dev = torch.device(device)
    ids = torch.as_tensor(input_ids).to(dev, torch.int64, non_blocking=True).contiguous()
    lab = torch.as_tensor(labels).to(dev, torch.int64, non_blocking=True).contiguous()
    B, L = ids.shape
    N = n_steps
    npair = N * (N - 1)
    if tuple(lab.shape) != (B, N):
        raise ValueError(f"labels shape {tuple(lab.shape)} != ({B}, {N})")
    i64 = dict(dtype=torch.int64, device=dev)
    starts, lens = torch.empty(B, N, **i64), torch.empty(B, N, **i64)
    plab, sep = torch.empty(B, npair, **i64), torch.empty(B, npair, 2, **i64)
    status = torch.zeros(2, dtype=torch.int32, device=dev)
    NT.pair_scan(ids, lab, cls_id, sep_id, starts, lens, plab, sep, status)
    Lp, bad = status.tolist()  # the one read-back: the pair length sizes every later tensor
    if bad:
        raise ValueError(f"{bad} stor{'y' if bad == 1 else 'ies'} without exactly {N} "
                         "<s> ... </s> steps (process_inputs_for_berson.py:104,136)")
    out_ids, mask, tt = (torch.empty(B * npair, Lp, **i64) for _ in range(3))
    NT.pair_expand(ids, starts, lens, N, Lp, pad_id, cls_id != 0, out_ids, mask, tt)
    return {
        "input_ids": out_ids.view(B, npair, Lp), "attention_mask": mask.view(B, npair, Lp),
        "token_type_ids": tt.view(B, npair, Lp),
        "pairs_list": _pairs_on(dev, N)[None].expand(B, npair, 2).contiguous(),
        "passage_length": torch.full((B,), N, **i64), "pairs_num": torch.full((B,), npair, **i64),
        "sep_positions": sep, "ground_truth": lab, "mask_cls": torch.ones(B, N, **i64),
        "pairwise_labels": plab,
    }


def prepare_berson_inputs_host(input_ids, labels, n_steps, cls_id=CLS_ID, sep_id=SEP_ID,
                               pad_id=PAD_ID, device=None):
    """Host (numpy) restatement of the same expansion."""
    ids = input_ids.detach().cpu().numpy() if torch.is_tensor(input_ids) else np.asarray(input_ids)
    lab = labels.detach().cpu().numpy() if torch.is_tensor(labels) else np.asarray(labels)
    B = ids.shape[0]
    pairs, npair = pairs_generator(n_steps)
    pa = np.asarray(pairs, dtype=np.int64)
    starts = np.empty((B, n_steps), np.int64)
    lens = np.empty((B, n_steps), np.int64)
    for b in range(B):
        s, e = _split_steps(ids[b], n_steps, cls_id, sep_id)
        starts[b], lens[b] = s, e - s + 1
    l1 = lens[:, pa[:, 0]]  # [B, npair]
    l2 = lens[:, pa[:, 1]]
    plen = l1 + l2
    Lp = int(plen.max())
    col = np.arange(Lp)[None, None, :]
    in1 = col < l1[..., None]
    in2 = (col >= l1[..., None]) & (col < plen[..., None])
    src1 = starts[:, pa[:, 0]][..., None] + col
    src2 = starts[:, pa[:, 1]][..., None] + (col - l1[..., None])
    src = np.where(in1, src1, np.where(in2, src2, 0))
    gathered = np.take_along_axis(ids[:, None, :].repeat(npair, 1), np.clip(src, 0, ids.shape[1] - 1),
                                  axis=2)
    valid = in1 | in2
    out_ids = np.where(valid, gathered, pad_id)
    mask = np.where(valid, 1, pad_id)  # quirk C.7: padded with pad_id (=1 for RoBERTa)
    if cls_id == 0:
        tt = np.zeros_like(out_ids)
    else:
        tt = np.where(in2, 1, 0)
    sep = np.stack([l1 - 1, plen - 1], -1)
    # pairwise label = 1 iff sentence a comes before sentence c in the ground-truth order (:162-174)
    rank = np.argsort(lab, axis=1)  # rank[b][s] = position of sentence s in the gold order
    ra = np.take_along_axis(rank, np.broadcast_to(pa[None, :, 0], (B, npair)), 1)
    rc = np.take_along_axis(rank, np.broadcast_to(pa[None, :, 1], (B, npair)), 1)
    plab = (ra < rc).astype(np.int64)
    out = {
        "input_ids": out_ids, "attention_mask": mask, "token_type_ids": tt,
        "pairs_list": np.broadcast_to(pa[None], (B, npair, 2)).copy(),
        "passage_length": np.full((B,), n_steps, np.int64),
        "pairs_num": np.full((B,), npair, np.int64), "sep_positions": sep,
        "ground_truth": lab.astype(np.int64), "mask_cls": np.ones((B, n_steps), np.int64),
        "pairwise_labels": plab,
    }
    res = {k: torch.from_numpy(np.ascontiguousarray(v, dtype=np.int64)) for k, v in out.items()}
    if device is not None:
        res = {k: v.pin_memory().to(device, non_blocking=True) if torch.device(device).type == "cuda"
               else v.to(device) for k, v in res.items()}
    return res
