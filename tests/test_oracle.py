"""Pin the CPU oracle against the reference's own outputs (golden fixtures)."""
import numpy as np
import pytest
import torch

from golden_util import FIXTURES, load_fixture, oracle_cfg
from oracle import berson_oracle as O


@pytest.mark.parametrize("name", FIXTURES)
def test_pairs_match_reference(name):
    meta, d, _ = load_fixture(name)
    pair = O.prepare_berson_inputs(d["input_ids"], d["labels"], meta["config"]["N"])
    for k, v in pair.items():
        np.testing.assert_array_equal(v, d["pair::" + k], err_msg=k)


@pytest.mark.parametrize("name", FIXTURES)
def test_loss_and_grads_match_reference(name):
    meta, d, params = load_fixture(name)
    cfg = oracle_cfg(meta)
    p = {k: v.clone().requires_grad_(v.dtype.is_floating_point) for k, v in params.items()}
    images = torch.from_numpy(d["images"])
    loss, pair, enc = O.forward_loss(p, d["input_ids"], d["labels"], images, cfg)
    assert abs(loss.item() - float(d["loss"])) < 1e-5, (loss.item(), float(d["loss"]))
    loss.backward()
    gsq = 0.0
    for k, v in p.items():
        if v.grad is not None:
            gsq += float((v.grad.double() ** 2).sum())
    assert abs(gsq ** 0.5 - float(d["grad_norm"])) < 1e-4 * float(d["grad_norm"])
    n = 0
    for k in d:
        if k.startswith("g::"):
            g = p[k[3:]].grad
            ref = d[k]
            if g is None:
                assert np.abs(ref).max() == 0, k
                continue
            np.testing.assert_allclose(g.numpy(), ref, rtol=2e-3, atol=2e-6, err_msg=k)
            n += 1
    assert n > 10
    np.testing.assert_allclose(enc["lang"].detach().numpy(), d["i::lang_feats"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(enc["okey"].detach().numpy(), d["i::original_key"], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("name", FIXTURES)
def test_beam_order_matches_reference(name):
    meta, d, params = load_fixture(name)
    cfg = oracle_cfg(meta)
    images = torch.from_numpy(d["images"])
    with torch.no_grad():
        for b in range(d["input_ids"].shape[0]):
            pair = O.prepare_berson_inputs(d["input_ids"][b:b + 1], d["labels"][b:b + 1], cfg["N"])
            enc = O.encode(params, pair, images[b:b + 1], cfg)
            assert O.beam_order(params, enc) == list(d["order"][b])


@pytest.mark.parametrize("name", FIXTURES)
def test_product_pair_expansion_bit_exact(name):
    """The product's vectorised pair expansion (multimodal_sequencing_amd/process_inputs.py)
    reproduces the reference's prepare_berson_inputs tensors bit for bit (pair:: fixtures)."""
    from multimodal_sequencing_amd.process_inputs import prepare_berson_inputs
    meta, d, _ = load_fixture(name)
    out = prepare_berson_inputs(d["input_ids"], d["labels"], meta["config"]["N"])
    for k in ["input_ids", "attention_mask", "token_type_ids", "pairs_list", "passage_length",
              "pairs_num", "sep_positions", "ground_truth", "mask_cls", "pairwise_labels"]:
        ref = d["pair::" + k]
        got = out[k].numpy()
        assert got.dtype == np.int64 and got.shape == ref.shape, (k, got.shape, ref.shape)
        assert np.array_equal(got, ref), k


def test_oracle_real_config3_story():
    """The oracle (also the bench's cpu_baseline) reproduces the reference at the benchmark's
    real shape: one config-3 story (ViT-B/16 + 12 x 768, T = 513), loss and gradient norms."""
    import json
    import os
    from counter_init import counter_state_dict
    from golden_util import GOLDEN
    from make_golden_real import real_inputs
    from multimodal_sequencing_amd import model_zoo
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    meta = json.load(open(os.path.join(GOLDEN, "real_config3.json")))
    d = dict(np.load(os.path.join(GOLDEN, "real_config3.npz")))
    shapes = {k: tuple(v.shape) for k, v in
              model_zoo.build_preset("config3", device="cpu", dtype=torch.float32).state_dict().items()}
    params = {k: torch.from_numpy(v).requires_grad_(True) for k, v in counter_state_dict(shapes).items()}
    ids, labels, images = real_inputs(meta["input_seed"])
    cfg = {"N": 5, "heads": 12, "inter_heads": 8, "text_only": False, "vit_heads": None}
    loss, _, _ = O.forward_loss(params, ids, labels, torch.from_numpy(images), cfg)
    loss.backward()
    assert abs(loss.item() - float(d["loss"])) < 1e-5, (loss.item(), float(d["loss"]))
    gn = sum(float((p.grad.double() ** 2).sum()) for p in params.values() if p.grad is not None) ** 0.5
    assert abs(gn - float(d["grad_norm"])) < 1e-5 * float(d["grad_norm"])
    for k in d:
        if k.startswith("gn::"):
            g = params[k[4:]].grad
            assert abs(float(g.double().norm()) - float(d[k])) <= 1e-4 * float(d[k]) + 1e-6, k


def test_bf16_emulation_without_rounding_is_the_oracle():
    """tests/bf16_emulation.py (the checker of tests/test_bf16_drift_gpu.py) restates the oracle's
    encoder: with no rounding site it reproduces the oracle bit for bit, and with every site its
    drift is of bf16's size."""
    import bf16_emulation as E
    meta, d, p = load_fixture("tiny")
    cfg = oracle_cfg(meta)
    pair = O.prepare_berson_inputs(d["input_ids"], d["labels"], cfg["N"])
    img = torch.from_numpy(d["images"])
    with torch.no_grad():
        ref = O.encode(p, pair, img, cfg)
        same = E.encode(p, pair, img, cfg, ())
        r16 = E.encode(p, pair, img, cfg, E.ALL)
    for k in ("lang", "okey", "clean"):
        assert torch.equal(ref[k], same[k]), k
    drift = float((r16["lang"] - ref["lang"]).norm() / ref["lang"].norm())
    assert 1e-3 < drift < 2e-2, drift


def test_mx_fake_quant_matches_the_quantiser_restatement():
    """The emulation's MX-fp8 site (tests/bf16_emulation.mx_fake_quant) = dequant(ref_quant(x)) of
    tests/test_fp8_gpu.py, the restatement the HIP quantiser is bit-exact against (zero blocks,
    saturating blocks and 10^-6..10^4 magnitudes included)."""
    import bf16_emulation as E
    from test_fp8_gpu import dequant, ref_quant
    g = torch.Generator().manual_seed(5)
    x = torch.randn(37, 256, generator=g)
    x = x * torch.pow(10.0, torch.randint(-6, 5, (37, 8, 1), generator=g).float()).repeat_interleave(32, -1).view(37, 256)
    x[0, :32] = 0
    x = x.bfloat16().float()
    assert torch.equal(E.mx_fake_quant(x), dequant(*ref_quant(x)))
