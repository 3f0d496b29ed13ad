"""LXRTModel in VisualBERT style with a CLIP ViT visual backbone — the inner encoder of the path.

Mirrors the reference's drop-in surface:
  * models/CLIP/src/lxrt/modeling.py  LXRTModel (:1456-1598), LXRTEncoder (:737-1122),
    BertEmbeddings (:342-370), BertLayer (:496-507), VisualFeatEncoder (:569-602), BertPooler
  * models/CLIP/clip/model.py         VisualTransformer (:242-305) with img_len = 2 (BERSON input)
  * same constructor kwargs, same forward signature and return structure
    `((lang_feats, visn_feats), pooled)`, same state-dict key names.

Compute runs through the mmseq HIP kernels (kernels.py); there is no CPU path. Parameters live in
one flat ParamStore (params.py); the module tree only carries named views of it.
"""
import math
from types import SimpleNamespace

import torch
from torch import nn

from . import kernels as K
from .checkpoint import JsonConfigMixin, lxrt_from_pretrained, save_pretrained
from .params import (ParamStore, Spec, attach_buffers, attach_tree, linear_specs, ln_specs,
                     normal, ones, zeros)

VIT = "encoder.visual_model.visual."

# CLIP vision configs (clip/clip.py:18-23 + the two ViT sizes the BASELINE configs name)
CLIP_VISION = {
    "ViT-B/32": dict(width=768, layers=12, patch=32, res=224, embed=512),
    "ViT-B/16": dict(width=768, layers=12, patch=16, res=224, embed=512),
    "ViT-L/14": dict(width=1024, layers=24, patch=14, res=224, embed=768),
    # ModifiedResNet (clip.py model table: layers (3, 4, 6, 3), width 64, output 1024); the
    # LXRT visual feature is 2048 wide (param.py:62-64: attnpool output duplicated, :99-101)
    "RN50": dict(type="rn50", layers=(3, 4, 6, 3), width=64, res=224, embed=1024, feat=2048),
}


class LXRTConfig(JsonConfigMixin, SimpleNamespace):
    """Subset of lxrt BertConfig (:147-336) that the path reads."""

    def __init__(self, vocab_size=50265, hidden_size=768, num_hidden_layers=12,
                 num_attention_heads=12, intermediate_size=3072, max_position_embeddings=514,
                 type_vocab_size=1, hidden_act="gelu", initializer_range=0.02,
                 hidden_dropout_prob=0.1, attention_probs_dropout_prob=0.1, **kw):
        super().__init__(vocab_size=vocab_size, hidden_size=hidden_size,
                         num_hidden_layers=num_hidden_layers,
                         num_attention_heads=num_attention_heads,
                         intermediate_size=intermediate_size,
                         max_position_embeddings=max_position_embeddings,
                         type_vocab_size=type_vocab_size, hidden_act=hidden_act,
                         initializer_range=initializer_range,
                         hidden_dropout_prob=hidden_dropout_prob,
                         attention_probs_dropout_prob=attention_probs_dropout_prob, **kw)


def _lxrt_specs(cfg, vision, text_part, max_story_length, pos_num=25, img_part=False):
    H, I = cfg.hidden_size, cfg.intermediate_size
    std = cfg.initializer_range
    sp = [Spec("embeddings.word_embeddings.weight", (cfg.vocab_size, H), normal(std)),
          Spec("embeddings.position_embeddings.weight", (cfg.max_position_embeddings, H),
               normal(std)),
          Spec("embeddings.token_type_embeddings.weight", (cfg.type_vocab_size, H),
               normal(std))]
    sp += ln_specs("embeddings.LayerNorm", H)
    rn = vision is not None and vision.get("type") == "rn50"
    if not text_part:
        E = vision.get("feat", vision["embed"])
        sp += linear_specs("encoder.visn_fc.visn_fc", E, H, std=std)
        sp += ln_specs("encoder.visn_fc.visn_layer_norm", H)
        sp += linear_specs("encoder.visn_fc.box_fc", 4, H, std=std, transpose=False)
        sp += ln_specs("encoder.visn_fc.box_layer_norm", H)
    # the image-only model (multimodal_img_part) builds no BertLayer stack (lxrt:797-798)
    for i in range(0 if img_part else cfg.num_hidden_layers):
        b = f"encoder.layer.{i}."
        a = b + "attention.self."
        sp += [Spec(a + "query.weight", (H, H), normal(std), transpose=True, pack=f"qkvw{i}"),
               Spec(a + "key.weight", (H, H), normal(std), transpose=True, pack=f"qkvw{i}"),
               Spec(a + "value.weight", (H, H), normal(std), transpose=True, pack=f"qkvw{i}"),
               Spec(a + "query.bias", (H,), zeros, pack=f"qkvb{i}"),
               Spec(a + "key.bias", (H,), zeros, pack=f"qkvb{i}"),
               Spec(a + "value.bias", (H,), zeros, pack=f"qkvb{i}")]
        sp += linear_specs(b + "attention.output.dense", H, H, std=std)
        sp += ln_specs(b + "attention.output.LayerNorm", H)
        sp += linear_specs(b + "intermediate.dense", H, I, std=std)
        sp += linear_specs(b + "output.dense", I, H, std=std)
        sp += ln_specs(b + "output.LayerNorm", H)
    if not text_part and rn:
        from .resnet import rn50_specs
        sp += rn50_specs(VIT, vision["layers"], vision["width"], vision["embed"], vision["res"])
        sp += [Spec("encoder.visual_pos.x_position_embedding.weight", (pos_num, E), normal(std)),
               Spec("encoder.visual_pos.y_position_embedding.weight", (pos_num, E), normal(std)),
               Spec("encoder.visual_token_type.token_type_embedding.weight",
                    (5, E), normal(std))]
    if not text_part and not rn:
        W, L, p, R, E = (vision[k] for k in ("width", "layers", "patch", "res", "embed"))
        scale = W ** -0.5
        g = R // p
        sp += [Spec(VIT + "class_embedding", (W,), normal(scale)),
               Spec(VIT + "positional_embedding", (g * g + 1, W), normal(scale)),
               Spec(VIT + "proj", (W, E), normal(scale), transpose=True),
               Spec(VIT + "conv1.weight", (W, 3, p, p), normal(std))]
        sp += ln_specs(VIT + "ln_pre", W)
        for i in range(L):
            b = f"{VIT}transformer.resblocks.{i}."
            sp += [Spec(b + "attn.in_proj_weight", (3 * W, W), normal(std), transpose=True),
                   Spec(b + "attn.in_proj_bias", (3 * W,), zeros)]
            sp += linear_specs(b + "attn.out_proj", W, W, std=std)
            sp += ln_specs(b + "ln_1", W)
            sp += linear_specs(b + "mlp.c_fc", W, 4 * W, std=std)
            sp += linear_specs(b + "mlp.c_proj", 4 * W, W, std=std)
            sp += ln_specs(b + "ln_2", W)
        sp += ln_specs(VIT + "ln_post", W)
        # RN50-only modules, constructed by the reference regardless (VISUAL_CONFIG flags,
        # lxrt:819-822); unused on the ViT path but part of the state dict
        sp += [Spec("encoder.visual_pos.x_position_embedding.weight", (pos_num, E), normal(std)),
               Spec("encoder.visual_pos.y_position_embedding.weight", (pos_num, E), normal(std)),
               Spec("encoder.visual_token_type.token_type_embedding.weight",
                    (5, E), normal(std))]  # hard-coded max_story_length = 5 (lxrt:666-667)
    sp += linear_specs("pooler.dense", H, H, std=std)
    return sp


def _mark_stale(module, incompatible_keys):
    """load_state_dict post-hook: the parameters are views of the master buffer, so a load
    rewrites master weights behind the compute-dtype / transposed shadows."""
    for s in module.stores() if hasattr(module, "stores") else [module.store]:
        s.shadow_stale = True


class LXRTModel(nn.Module):
    """VisualBERT-style LXRT encoder over cat(text tokens, CLIP-ViT patch tokens)."""

    from_pretrained = classmethod(lxrt_from_pretrained)  # lxrt:1258-1433 (checkpoint.py)
    save_pretrained = save_pretrained  # lxrt:1435-1453

    def __init__(self, config, multimodal_text_part=False, multimodal_img_part=False, cls_id=0,
                 sep_id=2, max_story_length=5, hl_include_objectives=None, mlm_ignore_index=-100,
                 clip_model_name="ViT-B/16", num_labels=None, device="cuda",
                 compute_dtype=torch.bfloat16, vision=None, **kw):
        super().__init__()
        if multimodal_img_part and multimodal_text_part:
            raise ValueError("multimodal_img_part and multimodal_text_part are exclusive")
        if num_labels is not None:
            raise NotImplementedError("topological-sort head is out of scope (SURVEY §2 row 3)")
        self.config = config
        self.text_part = multimodal_text_part
        self.img_part = multimodal_img_part
        self.cls_id, self.sep_id = cls_id, sep_id
        self.clip_model_name = clip_model_name
        self.vision = dict(vision or CLIP_VISION[clip_model_name])
        self.img_len = 2  # VISUAL_CONFIG.max_subsample_image_length for BERSON input (lxrt:770)
        specs = _lxrt_specs(config, self.vision, multimodal_text_part, max_story_length,
                            img_part=multimodal_img_part)
        self.store = ParamStore(specs, device, compute_dtype)
        self.store.init_weights(seed=kw.get("seed", 0))
        from .resnet import rn50_attach_order
        attach_tree(self, self.store.params, order=rn50_attach_order)
        self._anchor = torch.zeros((), device=device, requires_grad=True)
        self.rn50 = None
        if not multimodal_text_part and self.vision.get("type") == "rn50":
            if multimodal_img_part:
                raise NotImplementedError("image-only pretraining runs the ViT backbones")
            from .resnet import RN50Backbone, rn50_buffer_names
            bufs = {}
            for name, c in rn50_buffer_names(VIT, self.vision["layers"],
                                             self.vision["width"]).items():
                t = (torch.zeros(c, device=device), torch.ones(c, device=device),
                     torch.zeros((), dtype=torch.long, device=device))
                attach_buffers(self, {name + ".running_mean": t[0], name + ".running_var": t[1],
                                      name + ".num_batches_tracked": t[2]})
                bufs[name] = t
            self.rn50 = RN50Backbone(self.store, bufs, VIT, "encoder.", self.vision["layers"],
                                     self.vision["width"])
        self._build_refs()
        self.register_load_state_dict_post_hook(_mark_stale)
        self.dropout_seed = kw.get("seed", 0)  # fold the rank in for data parallel (trainer.py)
        self._n_fwd = 0

    def new_dropouts(self):
        """Fresh dropout descriptors for one forward pass (eval mode: all disabled)."""
        self._n_fwd += 1
        seed = (self.dropout_seed * 0x9E3779B97F4A7C15 + self._n_fwd) & ((1 << 64) - 1)
        return K.Dropouts(seed, self.training)

    # -- parameter groups per layer ---------------------------------------------------------
    def _build_refs(self):
        st = self.store
        self.layer_refs = []
        for i in range(0 if self.img_part else self.config.num_hidden_layers):
            b = f"encoder.layer.{i}."
            a = b + "attention.self."
            self.layer_refs.append(K.LayerRefs(
                st, qkv_w=[a + "query.weight", a + "key.weight", a + "value.weight"],
                qkv_b=[a + "query.bias", a + "key.bias", a + "value.bias"],
                o_w=b + "attention.output.dense.weight", o_b=b + "attention.output.dense.bias",
                ln1_w=b + "attention.output.LayerNorm.weight",
                ln1_b=b + "attention.output.LayerNorm.bias",
                i_w=b + "intermediate.dense.weight", i_b=b + "intermediate.dense.bias",
                out_w=b + "output.dense.weight", out_b=b + "output.dense.bias",
                ln2_w=b + "output.LayerNorm.weight", ln2_b=b + "output.LayerNorm.bias"))
        e = "embeddings."
        v = "encoder.visn_fc."
        self.input_refs = K.LayerRefs(
            st, word=e + "word_embeddings.weight", pos=e + "position_embeddings.weight",
            type=e + "token_type_embeddings.weight", eln_w=e + "LayerNorm.weight",
            eln_b=e + "LayerNorm.bias", v_w=v + "visn_fc.weight", v_b=v + "visn_fc.bias",
            vln_w=v + "visn_layer_norm.weight", vln_b=v + "visn_layer_norm.bias")
        if not self.text_part and self.rn50 is None:
            # the projection lies between the positional embedding and conv1 in the buffer, so the
            # stem's grad span includes it (VitProjFn's backward runs before the stem's)
            self.stem_refs = K.LayerRefs(st, conv_w=VIT + "conv1.weight", cls=VIT + "class_embedding",
                                         pos=VIT + "positional_embedding", ln_w=VIT + "ln_pre.weight",
                                         ln_b=VIT + "ln_pre.bias", proj_in_span=VIT + "proj")
            self.proj_refs = K.LayerRefs(st, proj=VIT + "proj")
            self.block_refs = []
            for i in range(self.vision["layers"]):
                b = f"{VIT}transformer.resblocks.{i}."
                self.block_refs.append(K.LayerRefs(
                    st, in_w=b + "attn.in_proj_weight", in_b=b + "attn.in_proj_bias",
                    out_w=b + "attn.out_proj.weight", out_b=b + "attn.out_proj.bias",
                    ln1_w=b + "ln_1.weight", ln1_b=b + "ln_1.bias", fc_w=b + "mlp.c_fc.weight",
                    fc_b=b + "mlp.c_fc.bias", proj_w=b + "mlp.c_proj.weight",
                    proj_b=b + "mlp.c_proj.bias", ln2_w=b + "ln_2.weight", ln2_b=b + "ln_2.bias"))

    def grad_units(self):
        """Contiguous grad-buffer spans completed by one layer-level backward each (for the
        overlapped data-parallel all-reduce, trainer.GradAllReduce). The ViT projection sits
        inside the stem's span in the buffer, so it is reported with the stem."""
        units = [L.span for L in self.layer_refs] + [self.input_refs.span]
        if not self.text_part and self.rn50 is None:
            units += [L.span for L in self.block_refs]
            units.append(self.stem_refs.span)
        return [u for u in units if u is not None]

    @property
    def compute_dtype(self):
        return self.store.compute_dtype

    def set_compute_dtype(self, dtype):
        self.store.set_compute_dtype(dtype)

    # -- forward ----------------------------------------------------------------------------
    def visual_forward(self, images, pairs_list):  # CLIP ViT has no dropout (clip/model.py)
        """CLIP ViT over the paired images of every ordered pair (img_len = 2):
        images [B][N][3][R][R] f32 (device), pairs_list [B][npair][2] -> [P*Tv][E]."""
        if self.rn50 is not None:  # RN50: unique images through the backbone, pairs pooled
            return self.rn50.forward(images, pairs_list, self._anchor, self.training,
                                     self.store.compute_dtype)
        st = self.store
        V = self.vision
        W, patch = V["width"], V["patch"]
        heads = W // 64
        B, npair = pairs_list.shape[:2]
        P = B * npair
        g = images.shape[-1] // patch
        Tv = 1 + 2 * g * g
        cd = st.compute_dtype
        h = K.VitStemFn.apply(images, pairs_list, self._anchor, self.stem_refs, patch, 1e-5, cd)
        save = torch.is_grad_enabled()
        for L in self.block_refs:
            h = K.VitBlockFn.apply(h, self._anchor, L, P, Tv, heads, 1e-5, save)
        return K.VitProjFn.apply(h, self._anchor, self.proj_refs), Tv

    def encode_joint(self, input_ids, attention_mask, token_type_ids=None, images=None,
                     pairs_list=None, drops=None, text_rows=False):
        """Run embeddings (+ ViT + visn_fc) and the joint BERT stack.
        Returns the joint activation [P][T][H] (compute dtype) and Lt. text_rows=True (the caller
        keeps only lang_feats, as BertForOrdering.encode, modeling_bert.py:1289-1290): the last
        layer may run on the text rows only (BertLayerFn Tq, where rows_ok), and the activation
        returned is then [P][Lt][H] — identical rows, the same dropout masks."""
        st = self.store
        D = drops or self.new_dropouts()
        ph = self.config.hidden_dropout_prob
        pa = self.config.attention_probs_dropout_prob
        if st.shadow_stale:
            st.refresh_shadows()
        P, Lt = input_ids.shape
        if token_type_ids is None:
            token_type_ids = torch.zeros_like(input_ids)
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        vout, Tv = None, 0
        if not self.text_part and images is not None:
            vout, Tv = self.visual_forward(images, pairs_list)
        T = Lt + Tv
        x, key_bias = K.JointInputFn.apply(vout, input_ids.contiguous(), token_type_ids.contiguous(),
                                           attention_mask, self._anchor, self.input_refs, P, Lt,
                                           Tv, 1e-12, st.compute_dtype,
                                           (D.site(ph, "emb"), D.site(ph, "visn_fc")))
        heads = self.config.num_attention_heads
        save = torch.is_grad_enabled()
        nl = len(self.layer_refs)
        Tq = Lt if text_rows and Tv > 0 and K.BertLayerFn.rows_ok(x) else None
        for i, L in enumerate(self.layer_refs):
            x = K.BertLayerFn.apply(x, key_bias, self._anchor, L, P, T, heads, 1e-12,
                                    (D.site(pa, "att", i), D.site(ph, "att_out", i),
                                     D.site(ph, "out", i)), save, Tq if i == nl - 1 else None)
        return x.view(P, Tq if Tq and nl else T, -1), Lt

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, visual_feats=None,
                visual_attention_mask=None, pretraining_objective=None, labels=None,
                pairs_list=None):
        """LXRTModel.forward (:1513-1598). `visual_feats` is either the reference's
        [2P][3][R][R] pair-image tensor, or (images [B][N][3][R][R], pairs_list) via the
        `pairs_list` kwarg so the pair gather happens on device."""
        if visual_feats is not None and pairs_list is None:
            # reference layout: consecutive image pairs -> treat as B = P stories of 2 images
            R = visual_feats.shape[-1]
            imgs = visual_feats.reshape(-1, 2, 3, R, R).float().contiguous()
            pl = torch.tensor([[[0, 1]]], device=imgs.device).expand(imgs.shape[0], 1, 2).contiguous()
            visual_feats, pairs_list = imgs, pl
        joint, Lt = self.encode_joint(input_ids, attention_mask, token_type_ids, visual_feats,
                                      pairs_list)
        lang = joint[:, :Lt]
        visn = joint[:, Lt:] if joint.shape[1] > Lt else None
        # BertPooler (:1125-1137, tanh commented out in the reference): dense(lang[:, 0]) (:1584)
        pooled = K.LinearFn.apply(lang[:, 0], self._anchor, self.store, "pooler.dense.weight",
                                  "pooler.dense.bias", 0)
        return (lang, visn), pooled
