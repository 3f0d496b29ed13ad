"""Generate golden fixtures by running the REFERENCE implementation in this container.

Test infrastructure only. This script is run by hand in the development container, where the
read-only reference tree is mounted at /root/reference. It never runs on the GPU box; the
fixtures it writes (small .npz + .json files in this directory) are what travel.

What it does (SURVEY.md Appendix A harness, re-created here as in-process module stubs only):
  * stubs `boto3`/`botocore`/`ftfy` (imported by the reference's vendored HF utilities, unused
    on the hot path) and aliases `transformers.modeling_roberta`;
  * replaces `visual_transformers.initialize_clip` (which downloads OpenAI weights by URL) with
    a direct `clip/model.py::CLIP(..., img_only=True)` construction (random init);
  * shims the two reference bugs on the ViT path: the `img_len` kwarg passed at
    `lxrt/modeling.py:882` and `VISUAL_CONFIG.visual_feat_dim` = proj width;
  * casts uint8 masks to bool in `Tensor.masked_fill_` (torch-1.8 byte masks, beam search only).
None of these alter hot-path arithmetic.

Weights are NOT stored: every parameter is set from `counter_init.counter_state_dict` (a pure
function of key and index) before the reference runs, and the tests rebuild the same values.
Each fixture holds: inputs (input_ids, labels, images), the reference loss and total grad norm,
gradients (`g::`, all of them for `tiny`, a representative subset otherwise), selected
intermediates (`i::`), the prepared pair tensors (`pair::`), and the beam-search ordering for
each story (`order`).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
import argparse
import importlib.machinery
import json
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _install_shims():
    import transformers.models.roberta.modeling_roberta as _rm  # before stubbing boto3

    def _mod(name, **attrs):
        m = types.ModuleType(name)
        m.__spec__ = importlib.machinery.ModuleSpec(name, None)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    class ClientError(Exception):
        pass

    _mod("boto3", resource=None, client=None)
    _mod("botocore")
    _mod("botocore.config", Config=object)
    _mod("botocore.exceptions", ClientError=ClientError)
    _mod("ftfy", fix_text=lambda s: s)
    sys.modules["transformers.modeling_roberta"] = _rm
    for p in [f"{REF}/models/CLIP/clip", f"{REF}/models/CLIP/src", REF]:
        sys.path.insert(0, p)
    _mf = torch.Tensor.masked_fill_
    torch.Tensor.masked_fill_ = lambda s, m, v: _mf(s, m.bool() if m.dtype == torch.uint8 else m, v)


def build_reference(cfg):
    import model as clipm  # models/CLIP/clip/model.py
    import models.CLIP.src.lxrt.visual_transformers as vt
    import models.CLIP.src.lxrt.modeling as lx
    from models.berson import BertForOrdering, BertConfig as BersonConfig

    V = cfg["vit"]

    def _init_clip(VC, num_patches=240, img_len=None, img_only=False):
        return clipm.CLIP(V["embed"], V["res"], V["layers"], V["width"], V["patch"], 77, 49408,
                          512, 8, 12, img_len=img_len, img_only=True)

    vt.initialize_clip = _init_clip
    _f = clipm.VisualTransformer.forward
    if not getattr(clipm.VisualTransformer, "_golden_shim", False):
        def _vf(self, x, skip_last_layer=False, img_len=None, **kw):
            assert img_len in (None, self.img_len)
            return _f(self, x, skip_last_layer=skip_last_layer, **kw)
        clipm.VisualTransformer.forward = _vf
        clipm.VisualTransformer._golden_shim = True
    lx.VISUAL_CONFIG.visual_feat_dim = V["embed"]

    J = cfg["joint"]
    bcfg = lx.BertConfig(J["vocab"], hidden_size=J["hidden"], num_hidden_layers=J["layers"],
                         num_attention_heads=J["heads"], intermediate_size=J["inter"],
                         max_position_embeddings=J["max_pos"], type_vocab_size=1)
    inner = lx.LXRTModel(bcfg, multimodal_text_part=cfg["text_only"], multimodal_img_part=False,
                         cls_id=0, sep_id=2, max_story_length=cfg["N"], hl_include_objectives=None,
                         mlm_ignore_index=-100, clip_model_name="ViT-B/16", num_labels=None)
    H = cfg["head"]
    args = argparse.Namespace(
        ff_size=H["ff"], heads=H["heads"], para_dropout=0.1, inter_layers=H["layers"],
        beam_size=16, pairwise_loss_lam=0.6, multimodal_loss=False,
        additional_wrapper_level_objectives=None, multimodal=True,
        use_multimodal_model=False, multimodal_model_type="clip", device=torch.device("cpu"),
        per_seq_max_length=cfg["per_seq"], max_story_length=cfg["N"], multimodal_img_part=False)
    bc = BersonConfig(vocab_size_or_config_json_file=J["vocab"], hidden_size=J["hidden"],
                      num_hidden_layers=1, num_attention_heads=J["heads"],
                      intermediate_size=J["inter"])
    bc.num_labels = 1
    bc.wrapper_model_with_heatmap = False
    bc.hierarchical_version = "v0"
    bc.hl_include_objectives = None
    bc.multimodal_loss = False
    bc.v_feature_size = 1024
    tok = types.SimpleNamespace(cls_token="<s>", sep_token="</s>", pad_token="<pad>",
                                convert_tokens_to_ids=lambda t: {"<s>": 0, "<pad>": 1, "</s>": 2}[t])
    m = BertForOrdering(config=bc, args=args, inner_model=None, tokenizer=tok)
    m.bert = inner
    m.tokenizer = tok
    return m, args, tok


def make_inputs(cfg, seed):
    """Synthetic story batch: each step = <s>(0) + k ids ~ U[3, vocab) + </s>(2)."""
    g = np.random.RandomState(seed)
    B, N, L = cfg["B"], cfg["N"], cfg["N"] * cfg["per_seq"]
    ids = np.ones((B, L), dtype=np.int64)  # pad id 1 (RoBERTa)
    for b in range(B):
        pos = 0
        for s in range(N):
            if cfg["ragged"]:
                k = int(g.randint(1, cfg["per_seq"] - 1))
            else:
                k = cfg["per_seq"] - 2
            step = [0] + list(g.randint(3, cfg["joint"]["vocab"], size=k)) + [2]
            ids[b, pos:pos + len(step)] = step
            pos += len(step)
    labels = np.stack([np.argsort(g.permutation(N)) for _ in range(B)]).astype(np.int64)
    R = cfg["vit"]["res"]
    images = g.standard_normal((B, N, 3, R, R)).astype(np.float32)
    return ids, labels, images


def run_one(name, cfg, seed):
    torch.manual_seed(seed)
    m, args, tok = build_reference(cfg)
    sys.path.insert(0, OUT)
    from counter_init import counter_state_dict
    sd = m.state_dict()
    cw = counter_state_dict({k: tuple(v.shape) for k, v in sd.items()})
    m.load_state_dict({k: torch.from_numpy(v) for k, v in cw.items()})
    m.eval()  # dropout off: the reference loss is bit-stable in eval mode
    ids, labels, images = make_inputs(cfg, seed + 1)
    inputs = {"input_ids": torch.from_numpy(ids), "attention_mask": torch.from_numpy((ids != 1).astype(np.int64)),
              "labels": torch.from_numpy(labels), "token_type_ids": None}
    # the dataset delivers f64 images; in text-only mode (--multimodal_text_part) they are ignored
    inputs["images"] = torch.from_numpy(images).double()

    inter = {}

    def hook(key):
        def _h(mod, inp, out):
            inter[key] = out
        return _h

    hooks = [m.bert.embeddings.register_forward_hook(hook("embeddings")),
             m.key_linear.register_forward_hook(hook("original_key")),
             m.encoder.register_forward_hook(hook("para_matrix")),
             m.two_level_encoder.register_forward_hook(hook("two_level")),
             m.bert.register_forward_hook(hook("bert"))]
    if not cfg["text_only"]:
        hooks.append(m.bert.encoder.visual_model.visual.register_forward_hook(hook("vit")))
        hooks.append(m.bert.encoder.visn_fc.register_forward_hook(hook("visn_fc")))

    from models.berson.process_inputs_for_berson import prepare_berson_inputs
    pair = prepare_berson_inputs(dict(inputs), tok, args=args)

    loss = m(dict(inputs))[0]
    loss.backward()
    for h in hooks:
        h.remove()

    out = {"input_ids": ids, "labels": labels, "loss": np.array(loss.item(), dtype=np.float64),
           "images": images}
    full = cfg.get("intermediates", False)
    keep = ("bert.encoder.layer.0.", "bert.encoder.visual_model.visual.transformer.resblocks.0.",
            "bert.embeddings.", "two_level_encoder.", "pw_k", "decoder.", "encoder.transformer_inter.1.")
    gsq = 0.0
    for k, p in m.named_parameters():
        if p.grad is not None:
            gsq += float((p.grad.double() ** 2).sum())
            if full or k.startswith(keep):
                out["g::" + k] = p.grad.detach().float().numpy()
    out["grad_norm"] = np.array(gsq ** 0.5, dtype=np.float64)
    for k in ["input_ids", "attention_mask", "token_type_ids", "pairs_list", "passage_length",
              "pairs_num", "sep_positions", "ground_truth", "mask_cls", "pairwise_labels"]:
        out["pair::" + k] = pair[k].numpy()
    if full:
        out["i::embeddings"] = inter["embeddings"].detach().numpy()
    (lang, visn), _pooled = inter["bert"]
    out["i::lang_feats"] = lang.detach().numpy()
    if visn is not None and full:
        out["i::vit"] = inter["vit"].detach().numpy()
        out["i::visn_fc"] = inter["visn_fc"].detach().numpy()
    fs, cls_mat, cls_score, cls_score_mat, _h1, _h2 = inter["two_level"]
    out["i::final_seq"] = fs.detach().numpy()
    out["i::cls_score"] = cls_score.detach().numpy()
    out["i::para_matrix"] = inter["para_matrix"].detach().numpy()
    out["i::original_key"] = inter["original_key"].detach().numpy()

    # Beam-search ordering per story (B = 1 each, as berson_evaluate does: eval.py:85,111)
    from models.berson.modeling_bert import berson_pointer_network
    orders = []
    with torch.no_grad():
        for b in range(cfg["B"]):
            one = {k: (v[b:b + 1] if torch.is_tensor(v) else v) for k, v in inputs.items()}
            orders.append(berson_pointer_network(args, m, tok, one))
    out["order"] = np.array(orders, dtype=np.int64)

    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)
    with open(os.path.join(OUT, f"{name}.json"), "w") as f:
        json.dump({"config": cfg, "seed": seed, "loss": float(loss.item()),
                   "shapes": {k: list(v.shape) for k, v in m.state_dict().items()},
                   "order": out["order"].tolist(),
                   "generator": "tests/golden/make_golden.py (reference run in-process, eval mode)"},
                  f, indent=1)
    print(name, "loss", loss.item(), "order", out["order"].tolist(), "params",
          sum(v.numel() for v in m.state_dict().values()), "grad_norm", float(out["grad_norm"]))


BASE = {
    "B": 2, "N": 5, "per_seq": 8, "ragged": False, "text_only": False,
    "vit": {"embed": 96, "res": 32, "layers": 2, "width": 128, "patch": 8},
    "joint": {"vocab": 300, "hidden": 128, "layers": 2, "heads": 2, "inter": 512, "max_pos": 514},
    "head": {"ff": 256, "heads": 8, "layers": 2},
}


def main():
    _install_shims()
    torch.set_num_threads(8)
    cfgs = {
        "tiny": dict(BASE, intermediates=True),
        "tiny_ragged": dict(BASE, ragged=True, B=3),
        "tiny_textonly": dict(BASE, text_only=True),
        "tiny_n4": dict(BASE, N=4, per_seq=10),
    }
    for i, (name, cfg) in enumerate(cfgs.items()):
        run_one(name, cfg, seed=100 + i)


if __name__ == "__main__":
    main()
