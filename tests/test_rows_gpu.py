"""The last joint layer on the text rows only (kernels.BertLayerFn Tq; mmseq_attn_fwd_rows /
_bwd_rows).

BertForOrdering.encode keeps only the text rows of the joint encoder's output (lang_feats,
berson/modeling_bert.py:1289-1290; lxrt/modeling.py:611-618 splits off the visual rows), so the last
layer's attention queries, output projection, LayerNorms and FFN run on those rows only. The claim
is exactness, not closeness: every kept row and the loss equal the full-size layer's (with the
attention-probability dropout on: its mask is drawn by the full-size index), and the gradients
differ only by the summation grouping of the weight-gradient GEMMs (the dropped rows contributed
exact zeros). The two hidden-dropout sites after the attention index their masks by the compacted
rows, so with those on the loss is a different (equally distributed) draw.
"""
import json
import os

import pytest
import torch

from counter_init import counter_state_dict
from golden_util import GOLDEN

pytestmark = pytest.mark.gpu
DEV = "cuda"
# relative gradient difference, text-rows vs full-size last layer (bf16, real_config5_l2 shape)
ROWS_GRAD_BOUND = 1e-5


def _qkv(P, T, heads, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    H = heads * 64
    qkv = (torch.randn(P * T, 3 * H, generator=g) * 0.5).to(DEV, torch.bfloat16)
    bias = ((torch.rand(P, T, generator=g) > 0.2).float() - 1).mul(10000.0).to(DEV)
    return qkv, bias


@pytest.mark.parametrize("P,T,Tq,heads,mode", [(3, 513, 120, 2, "bits"), (2, 393, 200, 4, "none"),
                                               (2, 769, 257, 2, "hash"), (1, 300, 1, 2, "bits"),
                                               (2, 160, 160, 2, "bits"),
                                               # Tq inside the forward's tail block of T (rows 256-271)
                                               (2, 272, 270, 2, "bits"), (1, 513, 513, 2, "none")])
def test_attention_rows_equal_full(P, T, Tq, heads, mode):
    """mmseq_attn_fwd_rows / _bwd_rows against mmseq_attn_fwd / _bwd (variant 1) with the dO rows
    past Tq zero: O, LSE and keep bits of rows < Tq, and the whole dQ|dK|dV (dQ = 0 past Tq),
    bit for bit."""
    from multimodal_sequencing_amd import _native as N
    N.attn_set_fast(1)
    H = heads * 64
    qkv, bias = _qkv(P, T, heads, P * T + Tq)
    d = N.drop(0.1, 21, 5) if mode != "none" else None
    bits = mode == "bits"
    kb_full = N.attn_keep_bits(P, T, heads, DEV).zero_() if bits else None
    kb_rows = N.attn_keep_bits(P, T, heads, DEV).zero_() if bits else None
    out = torch.empty(P * T, H, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(P, heads, T, device=DEV)
    N.attn_fwd(P, T, heads, qkv, 3 * H, 0, H, 2 * H, bias, 0.125, out, H, lse, drop=d, keep_bits=kb_full)
    out_r = torch.full((P * Tq, H), 7.0, device=DEV, dtype=torch.bfloat16)
    lse_r = torch.full((P, heads, T), 7.0, device=DEV)
    N.attn_fwd_rows(P, T, Tq, heads, qkv, bias, 0.125, out_r, lse_r, drop=d, keep_bits=kb_rows)
    assert torch.equal(out_r.view(P, Tq, H), out.view(P, T, H)[:, :Tq])
    assert torch.equal(lse_r[:, :, :Tq], lse[:, :, :Tq])
    if bits:
        nw = kb_full.numel() // (P * heads * T)
        assert torch.equal(kb_rows.view(P, heads, T, nw)[:, :, :Tq], kb_full.view(P, heads, T, nw)[:, :, :Tq])
    g = torch.Generator(device="cpu").manual_seed(Tq)
    dout = torch.randn(P, T, H, generator=g).to(DEV, torch.bfloat16)
    dout[:, Tq:] = 0
    ref = torch.empty_like(qkv)
    N.attn_bwd(P, T, heads, qkv, 3 * H, 0, H, 2 * H, bias, 0.125, out, H, dout.view(P * T, H), H, lse,
               torch.empty_like(lse), ref, 3 * H, drop=d, keep_bits=kb_full)
    got = torch.full_like(qkv, 3.0)
    N.attn_bwd_rows(P, T, Tq, heads, qkv, bias, 0.125, out_r, dout[:, :Tq].contiguous().view(P * Tq, H),
                    lse_r, torch.empty_like(lse), got, drop=d, keep_bits=kb_rows)
    assert torch.equal(got, ref)
    assert not got.view(P, T, 3 * H)[:, Tq:, :H].any()


def test_attention_rows_rejects_other_kernels():
    from multimodal_sequencing_amd import _native as N
    qkv, bias = _qkv(1, 128, 2, 0)
    lse = torch.empty(1, 2, 128, device=DEV)
    with pytest.raises(N.NativeError):
        N.attn_fwd_rows(1, 128, 129, 2, qkv, bias, 0.125, torch.empty(129, 128, device=DEV,
                        dtype=torch.bfloat16), lse)


def _c3_model():
    from make_golden_real import real_inputs
    from multimodal_sequencing_amd import model_zoo
    meta = json.load(open(os.path.join(GOLDEN, "real_config5_l2.json")))
    m = model_zoo.build_from_golden(meta["config"], device=DEV, dtype=torch.bfloat16)
    sd = counter_state_dict({k: tuple(v.shape) for k, v in m.state_dict().items()})
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    ids, labels, images = real_inputs(meta["input_seed"], meta["config"])
    inputs = {"input_ids": torch.from_numpy(ids), "labels": torch.from_numpy(labels),
              "images": torch.from_numpy(images).to(DEV)}
    return m, inputs


def test_text_rows_last_layer_equals_full_layer_in_training():
    """real_config5_l2 (72 pairs, T = 769, Lt = 255) in train mode with the attention-probability
    dropout on (hidden dropout off): the loss with the last joint layer on the text rows equals the
    full-size run's bit for bit, the gradients as close as two full-size backwards are to each
    other, and the beam-search ordering in eval is the same. With every dropout on: repeatable
    (the backward regenerates the forward's compacted masks)."""
    from multimodal_sequencing_amd import kernels as K
    from multimodal_sequencing_amd.berson import berson_pointer_network
    m, inputs = _c3_model()
    m.train()
    ph = m.bert.config.hidden_dropout_prob
    assert m.bert.config.attention_probs_dropout_prob > 0 and ph > 0

    def run(on):
        K.ROWS["on"] = on
        try:
            m.zero_grad()
            m.bert._n_fwd = 0  # the same dropout seeds in every run
            loss = m(inputs)[0]
            loss.backward()
            torch.cuda.synchronize()
            return float(loss), torch.cat([s.grad.clone() for s in m.stores()]).double()
        finally:
            K.ROWS["on"] = True

    m.bert.config.hidden_dropout_prob = 0.0
    try:
        (l0, g0), (l0b, g0b), (l1, g1) = run(False), run(False), run(True)
    finally:
        m.bert.config.hidden_dropout_prob = ph
    d_self, d_rows = (float((b - g0).norm() / g0.norm()) for b in (g0b, g1))
    print(f"attention dropout only: loss full {l0!r} text rows {l1!r}; gradient rel diff to a second "
          f"full run {d_self:.3e}, to the text-rows run {d_rows:.3e}")
    assert l1 == l0 == l0b
    # the backward is bit-stable (fixed-order table and pointer-head sums, test_determinism_gpu);
    # the text-rows run differs from the full one only by the last layer's fp32 weight-gradient
    # regrouping (its split-K slabs cover fewer rows)
    assert d_self == 0.0, d_self
    assert d_rows <= ROWS_GRAD_BOUND, d_rows
    (l0, g0), (l1, g1), (l2, g2) = run(False), run(True), run(True)
    cos = float(g1 @ g0 / (g1.norm() * g0.norm()))
    print(f"all dropout: loss full {l0!r} text rows {l1!r}; gradient cosine {cos:.5f}")
    # a different draw of two of the layer's masks: as different from the full run as any other
    # dropout sample (this 4-layer model's loss moves ~1 % between samples), so only repeatability
    # and finiteness are asserted here
    assert l2 == l1 and torch.equal(g2, g1)
    assert torch.isfinite(g1).all() and abs(l1 - l0) < 0.1 * abs(l0)
    m.eval()
    orders = []
    for on in (False, True):
        K.ROWS["on"] = on
        try:
            with torch.no_grad():
                orders.append(berson_pointer_network(m.args, m, None, inputs))
        finally:
            K.ROWS["on"] = True
    assert orders[0] == orders[1]
