"""Parity at the benchmark's real shapes against fixtures produced by running
the reference itself (tests/golden/make_golden_real.py, counter-based weights, seeded inputs):

  * one full config-3 story: ViT-B/16 + 12 x 768 joint encoder at T = 120 + 393 = 513 + the
    BERSON head, fwd + bwd + beam search — fp32 parity mode: loss within 1e-4 (north_star),
    total gradient norm within 1e-4 relative, every parameter's gradient norm within 2e-3
    relative, gradient samples within rtol 2e-3 / atol 1e-5, orderings identical; bf16 perf
    mode: loss within 2e-2 relative, identical ordering (or a reported near-tie);
  * single ops at real shape: a ViT ResidualAttentionBlock (T = 393), a BertLayer (T = 513, text
    key mask) and BertEmbeddings (padding_idx 0 rows), fwd + bwd through the HIP kernels.
"""
import json
import os

import numpy as np
import pytest
import torch

from counter_init import counter_state_dict
from golden_util import GOLDEN
from make_golden_real import op_inputs, real_inputs

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from multimodal_sequencing_amd import kernels as K
    from multimodal_sequencing_amd import model_zoo
    from multimodal_sequencing_amd.berson import berson_pointer_network
    from multimodal_sequencing_amd.params import (ParamStore, Spec, linear_specs, ln_specs, normal,
                                                  zeros)

DEV = "cuda"


def _fixture(name):
    path = os.path.join(GOLDEN, name + ".npz")
    if not os.path.exists(path):
        pytest.skip(f"{name}.npz not generated")
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        meta = json.load(f)
    return meta, dict(np.load(path))


def _check_grads(d, grads, rel_norm=2e-3, rtol=2e-3, atol=1e-5, cos_min=None):
    """grads: {name: tensor}. Norms, first-1024 and strided samples against the fixture."""
    n = 0
    for k in d:
        if not k.startswith("gn::"):
            continue
        name = k[4:]
        g = grads[name].detach().double().cpu().reshape(-1)
        ref_n = float(d[k])
        if cos_min is None:
            assert abs(float(g.norm()) - ref_n) <= rel_norm * ref_n + 1e-6, (name, float(g.norm()), ref_n)
        if "gh::" + name in d:
            step = max(1, g.numel() // 1024)
            got_h, got_s = g[:1024].numpy(), g[::step][:1024].numpy()
            ref_h, ref_s = d["gh::" + name], d["gs::" + name]
            if cos_min is None:
                np.testing.assert_allclose(got_h, ref_h, rtol=rtol, atol=atol, err_msg=name)
                np.testing.assert_allclose(got_s, ref_s, rtol=rtol, atol=atol, err_msg=name)
            else:
                a = np.concatenate([got_h, got_s])
                b = np.concatenate([ref_h, ref_s]).astype(np.float64)
                # skip analytically-zero gradients (e.g. tanh_linear.bias under the softmax)
                if np.linalg.norm(b) > 1e-6 * float(d["grad_norm"]) + 1e-8:
                    cos = float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b)))
                    assert cos > cos_min, (name, cos)
        if "g::" + name in d and cos_min is None:
            np.testing.assert_allclose(g.numpy(), d["g::" + name].reshape(-1), rtol=rtol, atol=atol,
                                       err_msg=name)
        n += 1
    assert n > 0


# ------------------------------------------------------------------------------------------
# full config-3 story
# ------------------------------------------------------------------------------------------
def _config3(dtype):
    meta, d = _fixture("real_config3")
    m = model_zoo.build_preset("config3", device=DEV, dtype=dtype)
    sd = m.state_dict()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in
                       counter_state_dict({k: tuple(v.shape) for k, v in sd.items()}).items()})
    m.eval()
    m.zero_grad()
    ids, labels, images = real_inputs(meta["input_seed"])
    inputs = {"input_ids": torch.from_numpy(ids), "labels": torch.from_numpy(labels),
              "images": torch.from_numpy(images).to(DEV)}
    return meta, d, m, inputs


def test_config3_story_fp32_matches_reference():
    meta, d, m, inputs = _config3(torch.float32)
    loss = m(inputs)[0]
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - float(d["loss"])) < 1e-4, (loss.item(), float(d["loss"]))
    grads = {k: p.grad for k, p in m.named_parameters()}
    gn = sum(float((g.double() ** 2).sum()) for g in grads.values()) ** 0.5
    assert abs(gn - float(d["grad_norm"])) < 1e-4 * float(d["grad_norm"]), (gn, float(d["grad_norm"]))
    _check_grads(d, grads)
    order = berson_pointer_network(m.args, m, None, inputs)
    assert order == [int(x) for x in d["order"][0]], (order, d["order"])


def test_config3_story_fp32_intermediates():
    meta, d, m, inputs = _config3(torch.float32)
    from multimodal_sequencing_amd.process_inputs import prepare_berson_inputs
    bi = prepare_berson_inputs(inputs["input_ids"], inputs["labels"], 5, device=DEV)
    P, Lt = 20, bi["input_ids"].shape[2]
    with torch.no_grad():
        joint, Lt = m.bert.encode_joint(bi["input_ids"].view(P, Lt), bi["attention_mask"].view(P, Lt),
                                        bi["token_type_ids"].view(P, Lt), inputs["images"],
                                        bi["pairs_list"])
        enc = m.encode(**bi, images=inputs["images"])
    lang = joint[:, :Lt].float().cpu().numpy()
    np.testing.assert_allclose(lang[0], d["i::lang_feats_p0"], rtol=1e-4, atol=2e-4)
    np.testing.assert_allclose(lang[19], d["i::lang_feats_p19"], rtol=1e-4, atol=2e-4)
    clean, para, _hcn, okey, _cls, _cm, cls_score = enc[:7]
    np.testing.assert_allclose(clean.cpu().numpy(), d["i::final_seq"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(cls_score.cpu().numpy(), d["i::cls_score"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(para.cpu().numpy(), d["i::para_matrix"], rtol=1e-4, atol=2e-4)
    np.testing.assert_allclose(okey.cpu().numpy(), d["i::original_key"], rtol=1e-4, atol=2e-4)


def test_config3_story_bf16_close_to_reference():
    meta, d, m, inputs = _config3(torch.bfloat16)
    loss = m(inputs)[0]
    loss.backward()
    torch.cuda.synchronize()
    ref = float(d["loss"])
    assert abs(loss.item() - ref) < 2e-2 * abs(ref), (loss.item(), ref)
    _check_grads(d, {k: p.grad for k, p in m.named_parameters()}, cos_min=0.95)
    order = berson_pointer_network(m.args, m, None, inputs)
    ref_order = [int(x) for x in d["order"][0]]
    if order != ref_order:  # report a near-tie instead of accepting it silently
        m32 = _config3(torch.float32)[2]

        def nll(o):
            with torch.no_grad():
                m32({**inputs, "labels": torch.tensor([o])})
            return float(m32.last_loss_terms[0]) * 4
        gap = nll(order) - nll(ref_order)
        print(f"NEAR-TIE config3: bf16 order {order} vs reference {ref_order}, fp32 gap {gap:.3e}")
        assert abs(gap) < 5e-3, (order, ref_order, gap)


# full-depth (12 ViT blocks + 12 joint layers) encoder output of the config-3 story against the
# reference: relative L2 of lang_feats (pair 0 and pair 19), the tensor the BERSON head reads
C3_BOUND = {"f32": 1e-4, "bf16": 1.5e-2}  # measured 1.5e-6 / 1.17e-2 (24 layers)


@pytest.mark.parametrize("mode", ["f32", "bf16"])
def test_config3_encoder_output_bounds(mode):
    meta, d, m, inputs = _config3(torch.float32 if mode == "f32" else torch.bfloat16)
    lang = _lang_feats(m, inputs).cpu().numpy()
    errs = [_rel_l2(lang[0], d["i::lang_feats_p0"]), _rel_l2(lang[19], d["i::lang_feats_p19"])]
    print(f"config3 lang_feats rel L2 ({mode}): {errs}")
    assert max(errs) <= C3_BOUND[mode], (mode, errs)


# ------------------------------------------------------------------------------------------
# config-5 shape (ViT-L/14 patch 14 -> K 588 padded to 640, width 1024, 16 heads, T = 769,
# RoBERTa-large width, N = 9 -> 72 pairs) with 2 + 2 layers
# ------------------------------------------------------------------------------------------
def _config5_l2(dtype):
    meta, d = _fixture("real_config5_l2")
    m = model_zoo.build_from_golden(meta["config"], device=DEV, dtype=dtype)
    sd = m.state_dict()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in
                       counter_state_dict({k: tuple(v.shape) for k, v in sd.items()}).items()})
    m.eval()
    m.zero_grad()
    ids, labels, images = real_inputs(meta["input_seed"], meta["config"])
    inputs = {"input_ids": torch.from_numpy(ids), "labels": torch.from_numpy(labels),
              "images": torch.from_numpy(images).to(DEV)}
    return meta, d, m, inputs


def test_config5_shape_fp32_matches_reference():
    meta, d, m, inputs = _config5_l2(torch.float32)
    loss = m(inputs)[0]
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - float(d["loss"])) < 1e-4, (loss.item(), float(d["loss"]))
    grads = {k: p.grad for k, p in m.named_parameters()}
    gn = sum(float((g.double() ** 2).sum()) for g in grads.values()) ** 0.5
    assert abs(gn - float(d["grad_norm"])) < 2e-4 * float(d["grad_norm"]), (gn, float(d["grad_norm"]))
    _check_grads(d, grads)
    order = berson_pointer_network(m.args, m, None, inputs)
    assert order == [int(x) for x in d["order"][0]], (order, d["order"])


def test_config5_shape_bf16_close_to_reference():
    meta, d, m, inputs = _config5_l2(torch.bfloat16)
    loss = m(inputs)[0]
    loss.backward()
    torch.cuda.synchronize()
    ref = float(d["loss"])
    assert abs(loss.item() - ref) < 2e-2 * abs(ref), (loss.item(), ref)
    _check_grads(d, {k: p.grad for k, p in m.named_parameters()}, cos_min=0.95)


# ------------------------------------------------------------------------------------------
# single ops at real shape
# ------------------------------------------------------------------------------------------
def _store(specs, prefix, dtype):
    st = ParamStore(specs, DEV, dtype)
    cw = counter_state_dict({prefix + s.name: s.shape for s in specs})
    st.load({s.name: torch.from_numpy(cw[prefix + s.name]) for s in specs})
    st.refresh_shadows()
    return st


def _grads_by_ref_name(st, prefix):
    return {prefix + n: p.grad for n, p in st.params.items()}


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_vit_block_T393(dtype):
    meta, d = _fixture("op_vit_block")
    W = 768
    specs = [Spec("attn.in_proj_weight", (3 * W, W), normal(0.02), transpose=True),
             Spec("attn.in_proj_bias", (3 * W,), zeros)]
    specs += linear_specs("attn.out_proj", W, W) + ln_specs("ln_1", W)
    specs += linear_specs("mlp.c_fc", W, 4 * W) + linear_specs("mlp.c_proj", 4 * W, W)
    specs += ln_specs("ln_2", W)
    st = _store(specs, meta["prefix"], dtype)
    L = K.LayerRefs(st, in_w="attn.in_proj_weight", in_b="attn.in_proj_bias",
                    out_w="attn.out_proj.weight", out_b="attn.out_proj.bias", ln1_w="ln_1.weight",
                    ln1_b="ln_1.bias", fc_w="mlp.c_fc.weight", fc_b="mlp.c_fc.bias",
                    proj_w="mlp.c_proj.weight", proj_b="mlp.c_proj.bias", ln2_w="ln_2.weight",
                    ln2_b="ln_2.bias")
    inp = op_inputs("vit_block", meta["seed"])
    P, T = 2, 393
    x = torch.from_numpy(inp["x"]).view(P * T, W).to(DEV, dtype).requires_grad_(True)
    anchor = torch.zeros((), device=DEV, requires_grad=True)
    y = K.VitBlockFn.apply(x, anchor, L, P, T, 12, 1e-5)
    y.backward(torch.from_numpy(inp["dy"]).view(P * T, W).to(DEV, dtype))
    torch.cuda.synchronize()
    got_y = y.detach().float().view(P, T, W).cpu().numpy()
    got_dx = x.grad.float().view(P, T, W).cpu().numpy()
    grads = _grads_by_ref_name(st, meta["prefix"])
    if dtype == torch.float32:
        np.testing.assert_allclose(got_y, d["y"], rtol=1e-4, atol=2e-4)
        np.testing.assert_allclose(got_dx, d["dx"], rtol=1e-3, atol=2e-5)
        _check_grads(d, grads)
    else:
        for a, b in ((got_y, d["y"]), (got_dx, d["dx"])):
            cos = float((a.ravel() @ b.ravel()) / (np.linalg.norm(a) * np.linalg.norm(b)))
            assert cos > 0.999, cos
        _check_grads(d, grads, cos_min=0.99)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bert_layer_T513_masked(dtype):
    meta, d = _fixture("op_bert_layer")
    H, I = 768, 3072
    a = "attention.self."
    specs = [Spec(a + "query.weight", (H, H), normal(0.02), transpose=True, pack="w"),
             Spec(a + "key.weight", (H, H), normal(0.02), transpose=True, pack="w"),
             Spec(a + "value.weight", (H, H), normal(0.02), transpose=True, pack="w"),
             Spec(a + "query.bias", (H,), zeros, pack="b"), Spec(a + "key.bias", (H,), zeros, pack="b"),
             Spec(a + "value.bias", (H,), zeros, pack="b")]
    specs += linear_specs("attention.output.dense", H, H) + ln_specs("attention.output.LayerNorm", H)
    specs += linear_specs("intermediate.dense", H, I) + linear_specs("output.dense", I, H)
    specs += ln_specs("output.LayerNorm", H)
    st = _store(specs, meta["prefix"], dtype)
    L = K.LayerRefs(st, qkv_w=[a + "query.weight", a + "key.weight", a + "value.weight"],
                    qkv_b=[a + "query.bias", a + "key.bias", a + "value.bias"],
                    o_w="attention.output.dense.weight", o_b="attention.output.dense.bias",
                    ln1_w="attention.output.LayerNorm.weight", ln1_b="attention.output.LayerNorm.bias",
                    i_w="intermediate.dense.weight", i_b="intermediate.dense.bias",
                    out_w="output.dense.weight", out_b="output.dense.bias",
                    ln2_w="output.LayerNorm.weight", ln2_b="output.LayerNorm.bias")
    inp = op_inputs("bert_layer", meta["seed"])
    P, T = 2, 513
    x = torch.from_numpy(inp["x"]).view(P * T, H).to(DEV, dtype).requires_grad_(True)
    key_bias = ((1.0 - torch.from_numpy(inp["mask"]).float()) * -10000.0).to(DEV)
    anchor = torch.zeros((), device=DEV, requires_grad=True)
    y = K.BertLayerFn.apply(x, key_bias, anchor, L, P, T, 12, 1e-12)
    y.backward(torch.from_numpy(inp["dy"]).view(P * T, H).to(DEV, dtype))
    torch.cuda.synchronize()
    got_y = y.detach().float().view(P, T, H).cpu().numpy()
    got_dx = x.grad.float().view(P, T, H).cpu().numpy()
    grads = _grads_by_ref_name(st, meta["prefix"])
    if dtype == torch.float32:
        np.testing.assert_allclose(got_y, d["y"], rtol=1e-4, atol=2e-4)
        np.testing.assert_allclose(got_dx, d["dx"], rtol=1e-3, atol=2e-5)
        _check_grads(d, grads)
    else:
        for a_, b_ in ((got_y, d["y"]), (got_dx, d["dx"])):
            cos = float((a_.ravel() @ b_.ravel()) / (np.linalg.norm(a_) * np.linalg.norm(b_)))
            assert cos > 0.999, cos
        _check_grads(d, grads, cos_min=0.99)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_embeddings_padding_idx(dtype):
    meta, d = _fixture("op_embeddings")
    H = 768
    specs = [Spec("word_embeddings.weight", (50265, H), normal(0.02)),
             Spec("position_embeddings.weight", (514, H), normal(0.02)),
             Spec("token_type_embeddings.weight", (1, H), normal(0.02))]
    specs += ln_specs("LayerNorm", H)
    st = _store(specs, meta["prefix"], dtype)
    L = K.LayerRefs(st, word="word_embeddings.weight", pos="position_embeddings.weight",
                    type="token_type_embeddings.weight", eln_w="LayerNorm.weight",
                    eln_b="LayerNorm.bias", v_w="-", v_b="-", vln_w="-", vln_b="-")
    inp = op_inputs("embeddings", meta["seed"])
    P, Lt = inp["ids"].shape
    ids = torch.from_numpy(inp["ids"]).to(DEV)
    anchor = torch.zeros((), device=DEV, requires_grad=True)
    joint, _kb = K.JointInputFn.apply(None, ids, torch.zeros_like(ids), torch.ones_like(ids), anchor,
                                      L, P, Lt, 0, 1e-12, dtype)
    joint.backward(torch.from_numpy(inp["dy"]).view(P * Lt, H).to(DEV, dtype))
    torch.cuda.synchronize()
    y = joint.detach().float().view(P, Lt, H).cpu().numpy()
    gw = st.params["word_embeddings.weight"].grad
    rows = torch.from_numpy(d["word_rows"]).to(DEV)
    if dtype == torch.float32:
        np.testing.assert_allclose(y, d["y"], rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(gw[rows].cpu().numpy(), d["g_word_rows"], rtol=1e-3, atol=1e-5)
        _check_grads(d, _grads_by_ref_name(st, meta["prefix"]))
    else:
        cos = float((y.ravel() @ d["y"].ravel()) / (np.linalg.norm(y) * np.linalg.norm(d["y"])))
        assert cos > 0.999, cos
        # bf16 dy: a row summed over many tokens (id 1 pads 70 positions) cancels, so compare
        # each row's direction
        a, b = gw[rows].cpu().double().numpy(), d["g_word_rows"].astype(np.float64)
        nb = np.linalg.norm(b, axis=1)
        live = nb > 0
        cos = (a[live] * b[live]).sum(1) / (np.linalg.norm(a[live], axis=1) * nb[live])
        assert cos.min() > 0.999, cos.min()
        assert np.abs(a[~live]).max(initial=0.0) == 0.0
    assert float(gw[0].abs().max()) == 0.0  # padding_idx 0 row never receives a gradient
    assert float(st.params["position_embeddings.weight"].grad[0].abs().max()) == 0.0


def _lang_feats(m, inputs):
    """lang_feats = joint[:, :Lt] (the text rows the BERSON head reads, modeling_bert.py:1289)."""
    from multimodal_sequencing_amd.process_inputs import prepare_berson_inputs
    N = m.n_steps
    bi = prepare_berson_inputs(inputs["input_ids"], inputs["labels"], N, device=DEV)
    P, Lt = bi["input_ids"].shape[0] * bi["input_ids"].shape[1], bi["input_ids"].shape[2]
    with torch.no_grad():
        joint, Lt = m.bert.encode_joint(bi["input_ids"].view(P, Lt), bi["attention_mask"].view(P, Lt),
                                        bi["token_type_ids"].view(P, Lt), inputs["images"],
                                        bi["pairs_list"])
    return joint[:, :Lt].float()


def _rel_l2(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


# encoder-output bounds at the config-5 shape (ViT-L/14 + 1024-wide joint, 2 + 2 layers), relative
# L2 of lang_feats (pair 0 and the last pair) against the reference's fp32 values. Measured: fp32
# 9e-7, bf16 5.4e-3, MX-fp8 3.9e-2 with all four encoder GEMMs of every layer on the fp8 MFMA
# (round 2, FC2 only: 2.7e-2); e4m3 keeps 3 mantissa bits (2^-4 relative rounding per operand)
C5_BOUND = {"f32": 1e-4, "bf16": 1e-2, "mxfp8": 5e-2}


@pytest.mark.parametrize("mode", ["f32", "bf16", "mxfp8"])
def test_config5_encoder_output_bounds(mode):
    """The benchmarked dtypes' encoder output against the reference: lang_feats relative L2 <= the
    bound of C5_BOUND (fp32 parity 1e-4, bf16 1e-2, MX-fp8 encoder GEMMs in eval 5e-2). A broken
    fp8 GEMM or quantiser moves it to O(1)."""
    from multimodal_sequencing_amd import kernels as K
    meta, d, m, inputs = _config5_l2(torch.float32 if mode == "f32" else torch.bfloat16)
    if mode == "mxfp8":
        with K.fp8_forward():
            lang = _lang_feats(m, inputs)
            assert len(K._FP8["cache"]) >= 4  # the fp8 GEMMs really ran
    else:
        lang = _lang_feats(m, inputs)
    lang = lang.cpu().numpy()
    errs = [_rel_l2(lang[0], d["i::lang_feats_p0"]), _rel_l2(lang[-1], d["i::lang_feats_p19"])]
    print(f"config5 lang_feats rel L2 ({mode}): {errs}")
    assert max(errs) <= C5_BOUND[mode], (mode, errs)


def test_config5_shape_fp8_forward_close_to_reference():
    """MX-fp8 encoder GEMMs (kernels.fp8_forward) in the eval no-grad forward of the config-5
    shape: loss within 1 % relative of the reference, and the fp8 GEMMs really run."""
    from multimodal_sequencing_amd import kernels as K
    meta, d, m, inputs = _config5_l2(torch.bfloat16)
    with torch.no_grad():
        base = m(inputs)[0].item()
        with K.fp8_forward():
            loss = m(inputs)[0].item()
            assert len(K._FP8["cache"]) >= 4  # the FC2 weight of 2 ViT blocks + 2 joint layers
    ref = float(d["loss"])
    print(f"config5 loss: reference {ref}, bf16 {base}, mxfp8 {loss}")
    assert abs(loss - ref) < 1e-2 * abs(ref), (loss, base, ref)
