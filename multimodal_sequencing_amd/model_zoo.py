"""Assembly of the clip + berson path (trainers/train.py:1854-1880, 2005-2037) for the BASELINE
configs, with the reference's hard-coded BERSON hyper-parameters (train.py:2012-2017)."""
import argparse

import torch

from .berson import BersonConfig, BertForOrdering
from .lxrt import CLIP_VISION, LXRTConfig, LXRTModel

# name -> (joint BERT dims, vision dims or None, story length N, per-step tokens)
PRESETS = {
    # config 3/4: ViT-B/16 + RoBERTa-base shape joint encoder, N=5, 60 tok/step (seq 120+393=513)
    "config3": dict(joint=dict(vocab_size=50265, hidden_size=768, num_hidden_layers=12,
                               num_attention_heads=12, intermediate_size=3072,
                               max_position_embeddings=514),
                    vision="ViT-B/16", N=5, per_seq=60, ff=3072),
    # config 1: text-only LXRT (--multimodal_text_part), RoBERTa-base shape
    "config1": dict(joint=dict(vocab_size=50265, hidden_size=768, num_hidden_layers=12,
                               num_attention_heads=12, intermediate_size=3072,
                               max_position_embeddings=514),
                    vision=None, N=5, per_seq=60, ff=3072),
    # the reference's default backbone (train.py:1011-1019 --clip_model_name RN50, param.py:
    # 246-247) with the config-3 joint encoder: N=5, 60 tok/step (seq 120 + 99 = 219)
    "config3_rn50": dict(joint=dict(vocab_size=50265, hidden_size=768, num_hidden_layers=12,
                                    num_attention_heads=12, intermediate_size=3072,
                                    max_position_embeddings=514),
                         vision="RN50", N=5, per_seq=60, ff=3072),
    # config 5: ViT-L/14 + RoBERTa-large shape, N=9, 128 tok/step (seq 256+513=769)
    "config5": dict(joint=dict(vocab_size=50265, hidden_size=1024, num_hidden_layers=24,
                               num_attention_heads=16, intermediate_size=4096,
                               max_position_embeddings=514),
                    vision="ViT-L/14", N=9, per_seq=128, ff=3072),
}


def berson_args(N, per_seq, ff=3072, heads=8, inter_layers=2, beam=16, lam=0.6, text_only=False):
    return argparse.Namespace(ff_size=ff, heads=heads, para_dropout=0.1, inter_layers=inter_layers,
                              beam_size=beam, pairwise_loss_lam=lam, multimodal_loss=False,
                              multimodal=True, multimodal_text_part=text_only,
                              multimodal_model_type="clip", per_seq_max_length=per_seq,
                              max_story_length=N, multimodal_img_part=False)


def build(joint, vision, N, per_seq, ff=3072, heads=8, inter_layers=2, text_only=False,
          device="cuda", dtype=torch.bfloat16, seed=0):
    """Returns BertForOrdering with .bert = LXRTModel (train.py:2024-2028)."""
    cfg = LXRTConfig(**joint)
    vis = None
    if not text_only:
        vis = dict(vision) if isinstance(vision, dict) else dict(CLIP_VISION[vision])
    inner = LXRTModel(cfg, multimodal_text_part=text_only, cls_id=0, sep_id=2, max_story_length=N,
                      device=device, compute_dtype=dtype, vision=vis, seed=seed,
                      clip_model_name=vision if isinstance(vision, str) else
                      ("RN50" if vis and vis.get("type") == "rn50" else "ViT-B/16"))
    args = berson_args(N, per_seq, ff=ff, heads=heads, inter_layers=inter_layers,
                       text_only=text_only)
    model = BertForOrdering(BersonConfig(hidden_size=cfg.hidden_size), args, device=device,
                            seed=seed + 1)
    model.bert = inner
    return model


def build_preset(name, device="cuda", dtype=torch.bfloat16, seed=0):
    p = PRESETS[name]
    return build(p["joint"], p["vision"], p["N"], p["per_seq"], ff=p["ff"],
                 text_only=p["vision"] is None, device=device, dtype=dtype, seed=seed)


def build_from_golden(cfg, device="cuda", dtype=torch.float32):
    """Model matching a tests/golden fixture config (make_golden.py BASE)."""
    J = cfg["joint"]
    V = cfg["vit"]
    joint = dict(vocab_size=J["vocab"], hidden_size=J["hidden"], num_hidden_layers=J["layers"],
                 num_attention_heads=J["heads"], intermediate_size=J["inter"],
                 max_position_embeddings=J["max_pos"])
    if V.get("type") == "rn50":
        vision = dict(V, layers=tuple(V["layers"]))
    else:
        vision = dict(width=V["width"], layers=V["layers"], patch=V["patch"], res=V["res"],
                      embed=V["embed"])
    H = cfg["head"]
    return build(joint, vision, cfg["N"], cfg["per_seq"], ff=H["ff"], heads=H["heads"],
                 inter_layers=H["layers"], text_only=cfg["text_only"], device=device, dtype=dtype)
