"""Training-step semantics on the GPU: the identity data-parallel averaging relies on (a step
over B stories == the accumulation of two B/2 micro-steps), the optimizer against an fp64
restatement of the reference's AdamW + schedule + clipping, the boundary's reentrancy
(concurrent split-K GEMMs on two streams), the pooled output and checkpoint reloads."""
import math

import numpy as np
import pytest
import torch

from golden_util import load_fixture

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from multimodal_sequencing_amd import _native as nat
    from multimodal_sequencing_amd import model_zoo
    from multimodal_sequencing_amd.trainer import FusedAdamW, train_step

DEV = "cuda"


def _fixture_model(name="tiny", dtype=None):
    meta, d, params = load_fixture(name)
    m = model_zoo.build_from_golden(meta["config"], device=DEV, dtype=dtype or torch.float32)
    m.load_state_dict(params)
    m.eval()
    m.zero_grad()
    inputs = {"input_ids": torch.from_numpy(d["input_ids"]), "labels": torch.from_numpy(d["labels"]),
              "images": torch.from_numpy(d["images"]).to(DEV)}
    return meta, d, params, m, inputs


def test_micro_batch_accumulation_equals_full_batch():
    """loss and gradients of one B-story step == 2 accumulated B/2 micro-steps (the reference's
    per-rank loss is the mean over its stories, modeling_bert.py:1142,1172), and so are the
    parameters after the AdamW update. (Equal-length stories: with ragged ones the reference
    pads each batch to its own longest pair and ATTENDS the pads, App. C.7, so a split batch
    is a different computation there.)"""
    meta, d, params, m, inputs = _fixture_model("tiny")  # B = 2: micro-batches 1 + 1
    halves = [{k: v[:1] for k, v in inputs.items()}, {k: v[1:] for k, v in inputs.items()}]
    results = []
    for batches in ([inputs], halves):
        m.load_state_dict(params)
        m.zero_grad()
        opt = FusedAdamW(m.stores(), lr=1e-3, warmup=0, total_steps=10)
        total = sum(b["input_ids"].shape[0] for b in batches)
        loss_sum = 0.0
        for b in batches:  # train_step without the update, to look at the gradients
            loss = m(b)[0] * (b["input_ids"].shape[0] / total)
            loss.backward()
            loss_sum += loss.item()
        grads = [s.grad.clone() for s in m.stores()]
        opt.step()
        torch.cuda.synchronize()
        results.append((loss_sum, grads, [s.master.clone() for s in m.stores()]))
    (l1, g1, p1), (l2, g2, p2) = results
    assert abs(l1 - l2) < 1e-5 * max(1.0, abs(l1)), (l1, l2)
    assert abs(l1 - float(d["loss"])) < 1e-4
    for a, b in zip(g1, g2):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=2e-6)
    for a, b in zip(p1, p2):
        diff = (a - b).abs()
        # Adam normalises: an element whose two gradients differ only by rounding near 0 can
        # move by up to 2 lr; everything else agrees to far less than lr
        assert diff.max().item() <= 2e-3 + 1e-6
        assert (diff > 1e-5).float().mean().item() < 1e-3
    m.load_state_dict(params)
    m.zero_grad()
    loss = train_step(m, FusedAdamW(m.stores(), lr=1e-3, warmup=0, total_steps=10), halves)
    assert abs(loss.item() - l1) < 1e-5 * max(1.0, abs(l1))


def test_fused_adamw_schedule_clip_matches_fp64_reference():
    """3 FusedAdamW steps over two stores with warmup, clipping (global norm over both) and
    weight decay vs transformers-3.4 AdamW + get_linear_schedule_with_warmup + clip_grad_norm_
    restated in fp64 (trainers/train.py:172-190, 353-363)."""
    meta, d, params, m, inputs = _fixture_model("tiny")
    stores = m.stores()
    lr, wd, warm, total = 1e-3, 0.01, 2, 6
    opt = FusedAdamW(stores, lr=lr, warmup=warm, total_steps=total, weight_decay=wd)
    ref_p = [s.master.double().clone() for s in stores]
    ref_m = [torch.zeros_like(p) for p in ref_p]
    ref_v = [torch.zeros_like(p) for p in ref_p]
    masks = [s.decay_mask.double() for s in stores]
    g = torch.Generator(device="cpu").manual_seed(11)
    lam = (lambda k: k / warm if k < warm else max(0.0, (total - k) / (total - warm)))
    for k in range(1, 4):
        for s in stores:
            s.grad.copy_(torch.randn(s.numel, generator=g).to(DEV) * 0.05)
        grads = [s.grad.double().clone() for s in stores]
        norm = math.sqrt(sum(float((x ** 2).sum()) for x in grads))
        assert norm > 1.0  # clipping is active
        coef = min(1.0, 1.0 / (norm + 1e-6))
        step_lr = lr * lam(k - 1)
        used = opt.step()
        assert abs(used - step_lr) < 1e-15
        for i in range(len(stores)):
            gr = grads[i] * coef
            ref_m[i] = 0.9 * ref_m[i] + 0.1 * gr
            ref_v[i] = 0.999 * ref_v[i] + 0.001 * gr * gr
            st = step_lr * math.sqrt(1 - 0.999 ** k) / (1 - 0.9 ** k)
            ref_p[i] = ref_p[i] - st * ref_m[i] / (ref_v[i].sqrt() + 1e-8)
            ref_p[i] = ref_p[i] - step_lr * wd * ref_p[i] * masks[i]
    torch.cuda.synchronize()
    for s, rp in zip(stores, ref_p):
        torch.testing.assert_close(s.master.double(), rp, rtol=1e-5, atol=1e-6)


def test_concurrent_split_k_on_two_streams():
    """Two wgrad-shaped (split-K) GEMMs running concurrently on two streams give the same
    results as when run alone: the workspace is per call / per stream, not process-global."""
    g = torch.Generator(device="cpu").manual_seed(5)
    jobs = []
    for M, N, K in ((768, 768, 16384), (768, 3072, 8192)):
        dY = torch.randn(K, M, generator=g).to(DEV, torch.bfloat16)
        X = torch.randn(K, N, generator=g).to(DEV, torch.bfloat16)
        gb = torch.zeros(M, device=DEV)
        jobs.append((M, N, K, dY, X, gb))
    ref = []
    for M, N, K, dY, X, _ in jobs:
        C = torch.zeros(M, N, device=DEV)
        gb = torch.zeros(M, device=DEV)
        nat.gemm_wgrad(dY, X, C, gb)
        ref.append((C, gb))
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for rep in range(3):
        outs = []
        for (M, N, K, dY, X, _), s in zip(jobs, streams):
            C = torch.zeros(M, N, device=DEV)
            gb = torch.zeros(M, device=DEV)
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(4):  # keep both streams busy at once
                    C.zero_()
                    gb.zero_()
                    nat.gemm_wgrad(dY, X, C, gb)
            outs.append((C, gb))
        torch.cuda.synchronize()
        for (C, gb), (Cr, gbr) in zip(outs, ref):
            assert torch.equal(C, Cr)  # fixed-order split-K: bitwise reproducible
            assert torch.equal(gb, gbr)
    assert len(nat._ws) >= 3  # default stream + the two side streams


def test_pooled_output_is_pooler_dense():
    """LXRTModel.forward returns pooler.dense(lang_feats[:, 0]) (no tanh: lxrt/modeling.py:
    1125-1137, 1584) as the reference does."""
    meta, d, params, m, inputs = _fixture_model("tiny_textonly")
    inner = m.bert
    P, Lt = d["pair::input_ids"].shape[0] * d["pair::input_ids"].shape[1], d["pair::input_ids"].shape[2]
    ids = torch.from_numpy(d["pair::input_ids"]).view(P, Lt).to(DEV)
    msk = torch.from_numpy(d["pair::attention_mask"]).view(P, Lt).to(DEV)
    tt = torch.from_numpy(d["pair::token_type_ids"]).view(P, Lt).to(DEV)
    with torch.no_grad():
        (lang, visn), pooled = inner(ids, tt, msk)
    assert visn is None
    W = params["bert.pooler.dense.weight"].to(DEV)
    b = params["bert.pooler.dense.bias"].to(DEV)
    torch.testing.assert_close(pooled.float(), lang[:, 0].float() @ W.t() + b, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(lang.cpu().numpy(), d["i::lang_feats"], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_load_state_dict_after_forward_refreshes_shadows(dtype):
    """A forward builds the compute-dtype / transposed shadows; a later load_state_dict must
    invalidate them (the parameters are views of the master buffer)."""
    meta, d, params, m, inputs = _fixture_model(
        "tiny", torch.float32 if dtype == "f32" else torch.bfloat16)
    scrambled = {k: (v * 0.5 + 0.01) for k, v in params.items()}
    m.load_state_dict(scrambled)
    m(inputs)[0].backward()  # shadows now hold the scrambled weights
    m.zero_grad()
    m.load_state_dict(params)
    loss = m(inputs)[0]
    loss.backward()
    torch.cuda.synchronize()
    ref = float(d["loss"])
    tol = 1e-4 if dtype == "f32" else 2e-2 * abs(ref)
    assert abs(loss.item() - ref) < tol, (loss.item(), ref)
    grads = dict(m.named_parameters())
    for k in d:
        if k.startswith("g::bert.encoder.layer.0."):
            a = torch.from_numpy(d[k]).double().flatten()
            b = grads[k[3:]].grad.detach().cpu().double().flatten()
            if a.norm() < 1e-6:
                continue
            if dtype == "f32":
                np.testing.assert_allclose(b.numpy(), a.numpy(), rtol=2e-3, atol=1e-5, err_msg=k)
            else:
                assert float(a @ b / (a.norm() * b.norm())) > 0.98, k
