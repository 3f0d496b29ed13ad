"""Config-2 image-only MRM pretraining against the reference-generated
fixture (tests/golden/make_golden_pretrain.py: LXRTPretraining run in-process, eval mode, every
np.random draw recorded and replayed here as explicit inputs).

CPU: state-dict names/shapes (including the tied LM decoder) and the draw structure.
GPU (fp32 parity mode): total loss within 1e-4, the answer head, pooled output, visn_fc output,
MRM targets and LM-head prediction scores, and every parameter gradient (the ViT's are exactly
zero in the reference too); bf16 perf mode within 2e-2.
"""
import json
import os

import numpy as np
import pytest
import torch

from counter_init import counter_state_dict
from golden_util import GOLDEN
from multimodal_sequencing_amd.lxrt import LXRTConfig
from multimodal_sequencing_amd.pretraining import LXRTPretraining


def _load():
    meta = json.load(open(os.path.join(GOLDEN, "pretrain_tiny.json")))
    d = dict(np.load(os.path.join(GOLDEN, "pretrain_tiny.npz")))
    return meta, d


def _build(meta, device, dtype):
    c = meta["config"]
    J, V = c["joint"], c["vit"]
    cfg = LXRTConfig(vocab_size=J["vocab"], hidden_size=J["hidden"], num_hidden_layers=J["layers"],
                     num_attention_heads=J["heads"], intermediate_size=J["inter"],
                     max_position_embeddings=J["max_pos"], type_vocab_size=2)
    m = LXRTPretraining(cfg, visual_losses="obj", multimodal_text_part=False,
                        multimodal_img_part=True, cls_id=0, sep_id=2, pad_id=1,
                        max_story_length=c["N"], mlm_ignore_index=-1,
                        multimodal_pretrain_objectives=["patch_based_mrm_classification"],
                        clip_model_name="ViT-B/16", pretraining=True, device=device,
                        compute_dtype=dtype, vision=dict(V))
    params = counter_state_dict({k: tuple(v) for k, v in meta["shapes"].items()})
    params["cls.predictions.decoder.weight"] = params["bert.embeddings.word_embeddings.weight"]
    m.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    return m


def test_pretrain_state_dict_matches_reference():
    meta, _ = _load()
    m = _build(meta, "cpu", torch.float32)
    ours = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    ref = {k: tuple(v) for k, v in meta["shapes"].items()}
    assert set(ours) == set(ref), (sorted(set(ours) - set(ref)), sorted(set(ref) - set(ours)))
    for k in ref:
        assert ours[k] == ref[k], k
    sd = m.state_dict()
    assert sd["cls.predictions.decoder.weight"].data_ptr() == \
        sd["bert.embeddings.word_embeddings.weight"].data_ptr()  # tied (:1164-1167)


def test_pretrain_parameter_order_is_the_references():
    """named_parameters() order equals the reference's (the MRM head is built before
    BertPreTrainingHeads, lxrt/modeling.py:1713,1724-1728): positional optimizer.pt resume."""
    meta, _ = _load()
    m = _build(meta, "cpu", torch.float32)
    ours = [n for n, _ in m.named_parameters()]
    assert [k for k in meta["shapes"] if k in set(ours)] == ours


def test_pretrain_draw_structure():
    meta, d = _load()
    m = _build(meta, "cpu", torch.float32)
    B, Nimg = 4, 5
    Tv = 1 + 2 * 16
    dr = m.draw(B, Nimg, Tv)
    assert dr["sub_idx"].shape == (B, 2) and (np.diff(dr["sub_idx"], axis=1) > 0).all()
    per = Tv // 2
    mi = dr["mask_idx"]
    assert mi.shape == (B, 10)
    assert ((mi[:, :5] >= 1) & (mi[:, :5] < 1 + per)).all()
    assert ((mi[:, 5:] >= 1 + per) & (mi[:, 5:] < 1 + 2 * per)).all()
    for row in dr["shuffle"]:
        assert sorted(row) == list(range(10))
    # the fixture's recorded draws have the same structure
    assert d["mask_idx"].shape == (meta["config"]["B"], 10)


def _run(dtype):
    meta, d = _load()
    m = _build(meta, "cuda", dtype)
    m.eval()
    m.zero_grad()
    batch = {"input_ids": torch.from_numpy(d["input_ids"]), "images": torch.from_numpy(d["images"]),
             "draws": {"sub_idx": d["sub_idx"], "mask_idx": d["mask_idx"], "shuffle": d["shuffle"]}}
    loss, losses, answer = m(batch)
    loss.backward()
    torch.cuda.synchronize()
    return meta, d, m, loss, losses, answer


@pytest.mark.gpu
def test_pretrain_fp32_matches_reference():
    meta, d, m, loss, losses, answer = _run(torch.float32)
    assert abs(loss.item() - float(d["loss"])) < 1e-4, (loss.item(), float(d["loss"]))
    np.testing.assert_allclose(losses.cpu().numpy(), d["losses"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(answer.cpu().numpy(), d["answer_score"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(m.last_prediction_scores.float().cpu().numpy(),
                               d["i::prediction_scores"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(m.last_seq_relationship.detach().cpu().numpy(),
                               d["i::seq_relationship"], rtol=1e-4, atol=1e-5)
    grads = {k: p.grad for k, p in m.named_parameters()}
    checked = 0
    for k in d:
        if k.startswith("g::"):
            name = k[3:]
            if name == "cls.predictions.decoder.weight":
                continue  # tied: named_parameters lists the word table once
            np.testing.assert_allclose(grads[name].detach().cpu().numpy(), d[k], rtol=2e-3,
                                       atol=1e-6, err_msg=name)
            checked += 1
    assert checked > 20
    gn = sum(float((g.double() ** 2).sum()) for g in grads.values()) ** 0.5
    assert abs(gn - float(d["grad_norm"])) < 1e-3 * float(d["grad_norm"])


@pytest.mark.gpu
def test_pretrain_bf16_close_to_reference():
    meta, d, m, loss, losses, answer = _run(torch.bfloat16)
    ref = float(d["loss"])
    assert abs(loss.item() - ref) < 2e-2 * abs(ref), (loss.item(), ref)
    grads = {k: p.grad for k, p in m.named_parameters()}
    for k in d:
        if not k.startswith("g::") or k[3:] == "cls.predictions.decoder.weight":
            continue
        a = torch.from_numpy(d[k]).double().flatten()
        if a.norm() < 1e-8:  # exactly zero in the reference (the ViT) or analytically zero
            assert float(grads[k[3:]].abs().max()) < 1e-3 * float(d["grad_norm"]), k
            continue
        b = grads[k[3:]].detach().cpu().double().flatten()
        cos = float(a @ b / (a.norm() * b.norm() + 1e-30))
        assert cos > 0.98, (k, cos)
