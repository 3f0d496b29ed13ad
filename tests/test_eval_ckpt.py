"""CPU tests of SURVEY §8f row 4: ordering metrics / cal_result against values the reference
computed (tests/golden/eval_metrics.json, make_golden_eval.py), checkpoint save/load with the
reference's key remaps, the reference-interop record (ckpt_interop.json), optimizer/scheduler
resume state, and the berson_evaluate loop with a stand-in decoder."""
import argparse
import json
import os

import numpy as np
import pytest
import torch

from golden_util import GOLDEN, load_fixture
from multimodal_sequencing_amd import checkpoint as C
from multimodal_sequencing_amd import metrics as M
from multimodal_sequencing_amd import model_zoo
from multimodal_sequencing_amd.berson import BertForOrdering, BersonConfig
from multimodal_sequencing_amd.evaluate import berson_evaluate, cal_result
from multimodal_sequencing_amd.lxrt import LXRTModel
from multimodal_sequencing_amd.trainer import FusedAdamW

with open(os.path.join(GOLDEN, "eval_metrics.json")) as _f:
    EM = json.load(_f)
ARGS = argparse.Namespace(**EM["args"])


def _check(got, want, what):
    if isinstance(want, str):  # the reference raised
        assert isinstance(got, Exception) and want == "error:" + type(got).__name__, (what, got)
    else:
        assert not isinstance(got, Exception), (what, got)
        assert got == pytest.approx(want, abs=1e-12), what


def _run(metric, preds, labels):
    try:
        return M.compute_metrics(ARGS, metric, preds, labels)
    except Exception as e:
        return e


@pytest.mark.parametrize("i", range(len(EM["single"])))
def test_metrics_single_reference(i):
    row = EM["single"][i]
    for m, want in row["values"].items():
        _check(_run(m, [list(row["pred"])], [list(row["label"])]), want, (i, m))


def test_metrics_multi_reference_and_batch():
    for row in EM["multi"]:
        for m, want in row["values"].items():
            _check(_run(m, [list(row["pred"])], [[list(r) for r in row["refs"]]]), want, m)
    perms = EM["single"][:60]
    for m, want in EM["batch"].items():
        _check(_run(m, [r["pred"] for r in perms], [r["label"] for r in perms]), want, m)
    with pytest.raises(NotImplementedError):
        M.compute_metrics(argparse.Namespace(multiref_metrics="mean"), "tau", [[0, 1]],
                          [[[0, 1], [1, 0]]])


def test_metric_helpers_known_answers():
    # trainers/metrics.py:299-317 worked examples
    assert M.lcs([1, 2, 3, 4], [4, 1, 2, 3]) == 3
    assert M.min_swaps([3, 2, 4, 1], [3, 4, 2, 1]) == 1
    assert M.lcs_substr([3, 2, 0, 1, 4], [2, 0, 1, 4, 3]) == 4


@pytest.mark.parametrize("k", range(len(EM["cal_result"])))
def test_cal_result_matches_reference(k, tmp_path):
    c = EM["cal_result"][k]
    best = []
    f = open(tmp_path / "o.txt", "w")
    accs, pmr, taus = cal_result(c["truth"], c["pred"], best, f, args=ARGS)
    assert f.closed
    assert float(accs) == pytest.approx(c["accs"], abs=1e-12)
    assert float(pmr) == pytest.approx(c["pmr"], abs=1e-12)
    assert float(taus) == pytest.approx(c["taus"], abs=1e-12)
    assert best[0] == pytest.approx(c["flat_acc"], abs=1e-12)


def test_cal_result_one_sentence_story_raises_like_reference(tmp_path):
    with pytest.raises(ZeroDivisionError):
        cal_result([[0, 1], [0]], [[1, 0], [0]], [], open(tmp_path / "o.txt", "w"), args=ARGS)


# ------------------------------------------------------------------------------------------------
def _tiny():
    meta, _, params = load_fixture("tiny")
    m = model_zoo.build_from_golden(meta["config"], device="cpu")
    m.load_state_dict(params)
    return meta, m, params


def test_interop_record_from_reference_runs():
    with open(os.path.join(GOLDEN, "ckpt_interop.json")) as f:
        rec = json.load(f)
    for k in ("ref_save_to_product_load", "product_save_to_ref_load"):
        assert rec[k]["max_abs_diff"] == 0.0 and not rec[k]["missing"] and not rec[k]["unexpected"]
        assert C.WEIGHTS_NAME in rec[k]["files"] and C.CONFIG_NAME in rec[k]["files"]
    assert rec["product_lxrt_save_to_ref_load"]["max_abs_diff"] == 0.0
    r = rec["roberta_gamma_beta_both_loaders"]
    assert r["ref_max_abs_diff"] == 0.0 and r["product_max_abs_diff"] == 0.0
    assert r["renamed_keys"] and not r["product_missing"]


def test_save_load_round_trip(tmp_path):
    meta, m, params = _tiny()
    m.config = BersonConfig(hidden_size=m.hidden_size, finetuning_task="sind")
    m.save_pretrained(str(tmp_path))
    assert sorted(os.listdir(tmp_path)) == [C.CONFIG_NAME, C.WEIGHTS_NAME]
    sd = C.load_weights_file(str(tmp_path / C.WEIGHTS_NAME))
    assert set(sd) == set(params)
    # standalone storages, tied params not duplicated needlessly
    assert all(v.device.type == "cpu" for v in sd.values())
    fresh = model_zoo.build_from_golden(meta["config"], device="cpu")
    fresh.bert.store.init_weights(seed=123)
    loaded = BertForOrdering.from_pretrained(
        str(tmp_path), inner_model=fresh.bert, tokenizer=None, load_inner_model=True,
        args=fresh.args, device="cpu")  # config from config.json
    assert loaded.config.finetuning_task == "sind" and loaded.config.hidden_size == m.hidden_size
    assert not loaded.training
    for k, v in loaded.state_dict().items():
        assert torch.equal(v, params[k]), k
    assert loaded.bert.store.shadow_stale  # the post-hook marks the compute shadows stale
    # config kwargs override existing attributes only (configuration_utils.py:147-156)
    cfg, unused = BersonConfig.from_pretrained(str(tmp_path), return_unused_kwargs=True,
                                               num_labels=1, finetuning_task="x", foo=3)
    assert cfg.finetuning_task == "x" and unused == {"foo": 3}


def test_base_model_prefix_rules(tmp_path):
    meta, m, params = _tiny()
    # a base-model state dict (no 'bert' keys) loads into model.bert (modeling_utils.py:399-400)
    inner = {k[5:]: v for k, v in params.items() if k.startswith("bert.")}
    fresh = model_zoo.build_from_golden(meta["config"], device="cpu")
    os.makedirs(tmp_path / "c")
    BersonConfig(hidden_size=m.hidden_size).save_pretrained(str(tmp_path / "c"))
    got, info = BertForOrdering.from_pretrained(
        str(tmp_path / "c"), state_dict=inner, inner_model=fresh.bert, tokenizer=None,
        load_inner_model=True, args=fresh.args, device="cpu", output_loading_info=True)
    assert not info["missing_keys"] and not info["unexpected_keys"]
    for k, v in got.bert.state_dict().items():
        assert torch.equal(v, inner[k]), k
    # shape mismatches raise (error_msgs), unknown keys are reported, not fatal
    bad = dict(params)
    bad["classifier.weight"] = torch.zeros(3, 3)
    with pytest.raises(RuntimeError, match="size mismatch"):
        BertForOrdering.from_pretrained(str(tmp_path / "c"), state_dict=bad,
                                        inner_model=fresh.bert, args=fresh.args, device="cpu")
    extra = dict(params)
    extra["bert.encoder.layer.9.output.dense.weight"] = torch.zeros(2)
    del extra["classifier.bias"]
    _, info = BertForOrdering.from_pretrained(
        str(tmp_path / "c"), state_dict=extra, inner_model=fresh.bert, args=fresh.args,
        device="cpu", output_loading_info=True)
    assert info["unexpected_keys"] == ["bert.encoder.layer.9.output.dense.weight"]
    assert info["missing_keys"] == ["classifier.bias"]


def test_lxrt_roberta_prefix_and_gamma_beta(tmp_path):
    meta, m, params = _tiny()
    m.bert.save_pretrained(str(tmp_path))
    inner = {k[5:]: v for k, v in params.items() if k.startswith("bert.")}
    rob = {}
    for k, v in inner.items():
        k2 = "roberta." + k
        if k2.endswith("LayerNorm.weight"):
            k2 = k2[:-6] + "gamma"
        rob[k2] = v
    kw = dict(device="cpu", vision=m.bert.vision, max_story_length=meta["config"]["N"])
    got = LXRTModel.from_pretrained(str(tmp_path), state_dict=dict(rob), **kw)
    assert not got.loading_info["missing_keys"]
    for k, v in got.state_dict().items():
        assert torch.equal(v, inner[k]), k
    # 'bert.' prefix, and the whole thing from the saved directory
    got2 = LXRTModel.from_pretrained(str(tmp_path), **kw)
    for k, v in got2.state_dict().items():
        assert torch.equal(v, inner[k]), k
    assert got2.config.hidden_size == m.bert.config.hidden_size


def test_pretraining_roberta_lm_head_remap():
    from multimodal_sequencing_amd.pretraining import build_config2
    tiny_vis = dict(width=128, layers=1, patch=8, res=32, embed=96)
    joint = dict(vocab_size=300, hidden_size=128, num_hidden_layers=1, num_attention_heads=2,
                 intermediate_size=512, max_position_embeddings=64)
    m = build_config2(device="cpu", dtype=torch.float32, vision=tiny_vis, joint=joint)
    ref = {k: torch.randn(v.shape) for k, v in m.state_dict().items()}
    ref["cls.predictions.decoder.weight"] = ref["bert.embeddings.word_embeddings.weight"]
    rob = {}
    for k, v in ref.items():
        if k.startswith("bert."):
            rob["roberta." + k[5:]] = v
        elif k == "cls.predictions.bias":
            rob["lm_head.bias"] = v
        elif k.startswith("cls.predictions.transform.dense"):
            rob[k.replace("cls.predictions.transform.dense", "lm_head.dense")] = v
        elif k.startswith("cls.predictions.transform.LayerNorm"):
            rob[k.replace("cls.predictions.transform.LayerNorm", "lm_head.layer_norm")] = v
        elif k == "cls.predictions.decoder.weight":
            rob["lm_head.decoder.weight"] = v
        else:
            rob[k] = v
    sd = C.roberta_to_bert_keys(dict(rob), set(m.state_dict()))
    assert set(sd) == set(ref)
    C.load_into(m, sd)
    for k, v in m.state_dict().items():
        assert torch.equal(v, ref[k]), k
    with pytest.raises(KeyError):
        C.roberta_to_bert_keys({"roberta.nope.weight": torch.zeros(1)}, set(m.state_dict()))


def test_clip_visual_weights_loader():
    meta, m, params = _tiny()
    fresh = model_zoo.build_from_golden(meta["config"], device="cpu")
    vis = {"module." + k[5:]: v for k, v in params.items() if "visual" in k}
    vis["module.classifier.weight"] = torch.zeros(1)  # no 'visual': ignored
    C.load_clip_visual_weights(fresh.bert, vis)
    for k, v in fresh.bert.state_dict().items():
        if "visual" in k:
            assert torch.equal(v, params["bert." + k]), k


def test_optimizer_scheduler_resume(tmp_path):
    meta, m, params = _tiny()
    opt = FusedAdamW(m.stores(), lr=5e-5, weight_decay=0.01, warmup=10, total_steps=100)
    g = torch.Generator().manual_seed(0)
    for a, b in zip(opt.m, opt.v):
        a.copy_(torch.randn(a.shape, generator=g))
        b.copy_(torch.rand(b.shape, generator=g))
    opt.step_count = 7
    sd = opt.state_dict(m)
    groups = sd["param_groups"]
    assert len(groups) == 2 and groups[0]["weight_decay"] == 0.01 and groups[1]["weight_decay"] == 0
    assert all(any(nd in n for nd in ("bias", "LayerNorm.weight")) for n in groups[1]["param_names"])
    assert not any(any(nd in n for nd in ("bias", "LayerNorm.weight"))
                   for n in groups[0]["param_names"])
    n_params = len(list(m.parameters()))
    assert len(sd["state"]) == n_params
    st0 = sd["state"][0]
    assert st0["step"] == 7 and st0["exp_avg"].shape == m.get_parameter(
        groups[0]["param_names"][0]).shape
    opt.save(m, str(tmp_path))
    opt2 = FusedAdamW(m.stores(), lr=5e-5, weight_decay=0.01, warmup=10, total_steps=100)
    assert opt2.load(m, str(tmp_path))
    assert opt2.step_count == 7 and opt2.current_lr() == opt.current_lr()
    _same_moments(m, opt, opt2)
    # LambdaLR layout of scheduler.pt
    sch = C.load_weights_file(str(tmp_path / C.SCHEDULER_NAME))
    assert sch["last_epoch"] == 7 and sch["_step_count"] == 8
    # positional (reference-written, no names) state
    for gr in sd["param_groups"]:
        del gr["param_names"]
    opt3 = FusedAdamW(m.stores(), lr=5e-5)
    opt3.load_state_dict(m, sd)
    _same_moments(m, opt, opt3)


@pytest.mark.parametrize("name", ["tiny", "tiny_textonly", "rn50_eval"])
def test_parameter_order_is_the_references(name):
    """named_parameters() runs in the reference's module order (modeling_bert.py:860-866 sets
    `self.bert` before the head; AttentionPool2d creates k_proj before q_proj, clip/model.py:
    60-64). The fixture's `shapes` were written from the reference's state_dict() in order."""
    meta, _, _ = load_fixture(name)
    m = model_zoo.build_from_golden(meta["config"], device="cpu")
    ours = [n for n, _ in m.named_parameters()]
    ref = [k for k in meta["shapes"] if k in set(ours)]
    assert len(ref) == len(ours) and ref == ours


def test_positional_optimizer_state_from_reference_order():
    """A reference-written optimizer.pt carries no names: train.py:172-183 builds the decay and
    no-decay groups from model.named_parameters() in the REFERENCE's order, and AdamW numbers
    the parameters 0.. across the groups. Each moment here encodes its parameter's identity, so
    a wrong positional match shows up as a wrong value (or a numel mismatch)."""
    meta, m, params = _tiny()
    ref_names = list(meta["shapes"])
    no_decay = ("bias", "LayerNorm.weight")
    groups = [[n for n in ref_names if not any(nd in n for nd in no_decay)],
              [n for n in ref_names if any(nd in n for nd in no_decay)]]
    state, pg, idx = {}, [], 0
    for gi, names in enumerate(groups):
        ids = []
        for n in names:
            shape = tuple(meta["shapes"][n])
            state[idx] = {"step": 3, "exp_avg": torch.full(shape, float(idx)),
                          "exp_avg_sq": torch.full(shape, float(idx) + 0.5)}
            ids.append(idx)
            idx += 1
        pg.append({"lr": 1e-5, "betas": (0.9, 0.999), "eps": 1e-8,
                   "weight_decay": 0.01 if gi == 0 else 0.0, "correct_bias": True, "params": ids})
    opt = FusedAdamW(m.stores(), lr=1e-5)
    opt.load_state_dict(m, {"state": state, "param_groups": pg})
    assert opt.step_count == 3
    pos = {n: i for i, n in enumerate(groups[0] + groups[1])}
    for i, s in enumerate(m.stores()):
        for sname, p in s.params.items():
            full = next(n for n, q in m.named_parameters() if q is p)
            o, k = s.offsets[sname], p.numel()
            assert torch.all(opt.m[i][o:o + k] == pos[full]), full
            assert torch.all(opt.v[i][o:o + k] == pos[full] + 0.5), full


def _same_moments(m, a, b):
    """every parameter's span round-trips (alignment padding is not state)"""
    for i, s in enumerate(m.stores()):
        for name, p in s.params.items():
            o, n = s.offsets[name], p.numel()
            assert torch.equal(a.m[i][o:o + n], b.m[i][o:o + n]), name
            assert torch.equal(a.v[i][o:o + n], b.v[i][o:o + n]), name


def test_berson_evaluate_loop(tmp_path):
    """eval.py:39-187 end to end with a stand-in decoder (the device beam search runs in the
    -m gpu parity tests): files, one-sentence shortcut, multi-reference gold, results."""
    stories = [([1, 0, 2], [1, 0, 2]), ([0, 1, 2, 3], [3, 2, 1, 0]), ([2, 1, 0], [0, 1, 2])]
    preds = {0: [1, 0, 2], 1: [3, 2, 0, 1], 2: [0, 1, 2]}

    class DS(torch.utils.data.Dataset):
        def __len__(self):
            return len(stories)

        def __getitem__(self, i):
            gold = torch.tensor(stories[i][1])
            return (torch.full((8,), i), torch.ones(8), torch.zeros(8), gold, f"url{i}###x")

    calls = []

    def decoder(args, model, tok, inputs):
        i = int(inputs["input_ids"][0, 0])
        calls.append(i)
        return preds[i]

    class Dummy:
        def eval(self):
            return self

    args = argparse.Namespace(task_names=["sind"], output_dir=str(tmp_path), local_rank=-1,
                              per_gpu_eval_batch_size=1, n_gpu=1, max_eval_steps=0,
                              multimodal=False, eval_save_all_results=True,
                              max_story_length=5, multiref_metrics="max")
    res = berson_evaluate(args, Dummy(), lambda *a, **k: DS(), None, pointer_network=decoder)
    truth = [s[1] for s in stories]
    pr = [preds[i] for i in range(3)]
    want = cal_result(truth, pr, [], None, args)
    assert res["acc_dev"] == pytest.approx(want[0]) and res["pmr_dev"] == pytest.approx(want[1])
    assert res["taus_dev"] == pytest.approx(want[2])
    lines = open(tmp_path / "output_order.txt").read().splitlines()
    assert lines[1] == "3 2 0 1|||3 2 1 0"
    assert calls == [0, 1, 2]
    csv_rows = open(tmp_path / "all_predictions.csv").read().splitlines()
    assert csv_rows[0] == "url,pm,em,lcs_substr,lcs,ms,wms,dist,tau" and csv_rows[1].startswith("url0,")
    assert "acc_dev" in open(tmp_path / "eval_results_split_test.txt").read()
