"""Image-only MRM pretraining (BASELINE config 2): LXRTPretraining with multimodal_img_part and
the patch_based_mrm_classification objective.

Drop-in for models/CLIP/src/lxrt/modeling.py LXRTPretraining (:1601-1734 construction,
:1734-2484 forward) on the path trainers/run_pretraining.py runs for
scripts/wikihow_image_only_pretrain.sh: same constructor kwargs, `model(batch)` ->
(total_loss, losses [1, n], answer_score), same state-dict names (the LM decoder is tied to the
word embeddings as in the reference).

Per story:
  * 2 of the N images are sub-sampled (:1979-1985) and encoded as ONE CLIP-ViT sequence of
    1 + 2 g^2 tokens (img_len = 2, the pos-embed quirk) — on device, by index, no copies;
  * 5 patch features per image are zeroed and their visn_fc features kept as targets
    (:948-1009); visn_fc on the masked sequence; pooler = dense(token 0), no tanh (:1125-1137);
  * BertPreTrainingHeads over every visual token (:1217-1227, :2247): the LM head to the vocab is
    one bf16 MFMA GEMM against the word table (computed as the reference does, not in the loss);
    the answer head on the pooled output (:2249-2250);
  * MRM classification (:2309-2351): each masked output is paired with every shuffled target,
    scored by a BertLMPredictionHead of width 2H with a 1-row decoder, cross-entropy against the
    inverse permutation, summed over stories, x 0.2.

The reference draws every random choice from np.random at run time; here they are explicit
(`draws`: sub_idx [B, 2], mask_idx [B, 10], shuffle [B, 10]) or drawn from `self.rng` in the
reference's order and distributions (SURVEY §8c determinism).

Gradient structure (exact, also true of the reference): the masked positions' ViT features are
zeroed BEFORE visn_fc and only those positions (and the detached targets) enter the loss, so the
loss's gradient with respect to the ViT is identically zero (the reference's autograd still runs
the ViT backward on zeros; the fixture's ViT gradients are all 0). The ViT output therefore enters
visn_fc detached, and the ViT parameters receive their exact (zero) gradient without the pass.
"""
import copy
from types import SimpleNamespace

import numpy as np
import torch
from torch import nn

from . import _native as N
from . import kernels as K
from .checkpoint import lxrt_from_pretrained, save_pretrained
from .lxrt import LXRTConfig, LXRTModel, _mark_stale
from .params import ParamStore, Spec, attach_tree, linear_specs, ln_specs, normal, zeros

OBJ_ID_NUM = 1600  # param.py:68 (VISUAL_CONFIG.obj_id_num, BertVisualObjHead 'obj' decoder)


def _pretrain_head_specs(H, vocab, std=0.02, num_answers=2):
    p = "cls.predictions."
    sp = [Spec(p + "bias", (vocab,), zeros)]
    sp += linear_specs(p + "transform.dense", H, H, std=std) + ln_specs(p + "transform.LayerNorm", H)
    sp += linear_specs("cls.seq_relationship", H, 2, std=std)
    o = "obj_predict_head."
    sp += linear_specs(o + "transform.dense", H, H, std=std) + ln_specs(o + "transform.LayerNorm", H)
    sp += linear_specs(o + "decoder_dict.obj", H, OBJ_ID_NUM, std=std, transpose=False)
    a = "answer_head.logit_fc."
    sp += linear_specs(a + "0", H, 2 * H, std=std) + ln_specs(a + "2", 2 * H)
    sp += linear_specs(a + "3", 2 * H, num_answers, std=std)
    m = "patch_based_mrm_classification_head."
    sp += [Spec(m + "bias", (1,), zeros)]
    sp += linear_specs(m + "transform.dense", 2 * H, 2 * H, std=std)
    sp += ln_specs(m + "transform.LayerNorm", 2 * H)
    sp += [Spec(m + "decoder.weight", (1, 2 * H), normal(std), transpose=True)]
    return sp


class LXRTPretraining(nn.Module):
    MASK_NUM = 5  # pb_mrm_cls_mask_num (:1694)
    MRM_SCALE = 0.2  # :2347
    from_pretrained = classmethod(lxrt_from_pretrained)  # roberta/lm_head remaps (checkpoint.py)
    save_pretrained = save_pretrained

    def __init__(self, config, task_mask_lm=True, task_matched=True, task_obj_predict=True,
                 visual_losses="", task_qa=True, num_answers=2, device="cuda",
                 compute_dtype=torch.bfloat16, seed=0, vision=None, **kwargs):
        super().__init__()
        if not kwargs.get("multimodal_img_part", False):
            raise NotImplementedError(
                "only the image-only MRM pretraining path (config 2) is on the hot path")
        objectives = list(kwargs.get("multimodal_pretrain_objectives") or [])
        if objectives != ["patch_based_mrm_classification"]:
            raise NotImplementedError(
                f"pretraining objectives {objectives}: only patch_based_mrm_classification "
                "(scripts/wikihow_image_only_pretrain.sh) is built")
        self.config = config
        self.multimodal_img_part = True
        self.multimodal_pretrain_objectives = objectives
        self.cls_id, self.sep_id = kwargs.get("cls_id", 0), kwargs.get("sep_id", 2)
        self.pad_id = kwargs.get("pad_id", 1)
        self.task_qa = task_qa
        inner_kw = {k: v for k, v in kwargs.items()
                    if k in ("cls_id", "sep_id", "max_story_length", "clip_model_name")}
        self.bert = LXRTModel(config, multimodal_img_part=True, device=device,
                              compute_dtype=compute_dtype, vision=vision, seed=seed, **inner_kw)
        H = config.hidden_size
        self.store = ParamStore(_pretrain_head_specs(H, config.vocab_size,
                                                     config.initializer_range, num_answers),
                                device, compute_dtype)
        self.store.init_weights(seed=seed + 7)
        # the reference builds the MRM head before BertPreTrainingHeads (lxrt/modeling.py:1713,
        # 1724-1728): registration order = named_parameters() order
        mrm = "patch_based_mrm_classification_head."
        attach_tree(self, self.store.params, order=lambda names: (
            [n for n in names if n.startswith(mrm)] + [n for n in names if not n.startswith(mrm)]))
        # tied LM decoder (:1164-1167): the word table registered under both names
        attach_tree(self, {"cls.predictions.decoder.weight":
                           self.bert.store.params["embeddings.word_embeddings.weight"]})
        self._anchor = torch.zeros((), device=device, requires_grad=True)
        self.register_load_state_dict_post_hook(_mark_stale)
        self.rng = np.random.RandomState(seed)
        self.device_ = torch.device(device)
        self.last_prediction_scores = None
        self.last_seq_relationship = None

    def stores(self):
        return [self.bert.store, self.store]

    def zero_grad(self, set_to_none=False):
        for s in self.stores():
            s.zero_grad()

    def ddp_units(self):
        """(units, begin_stores) for trainer.GradAllReduce: the heads and visn_fc finish together;
        no per-layer units (the ViT gradient is exactly zero, see the module docstring)."""
        return {}, []

    # ------------------------------------------------------------------------------------
    def draw(self, B, N, Tv):
        """The reference's np.random draws (:1981, :983-987, :2322-2323) for a batch of B
        stories of N images with Tv visual tokens (1 + 2 g^2)."""
        per = Tv // 2  # visn_per_seq_len (:955)
        sub_idx, mask_idx, shuffle = [], [], []
        for _ in range(B):
            sub_idx.append(sorted(self.rng.choice(N, 2, replace=False)))
        for _ in range(B):
            m = []
            for start in range(1, Tv, per):
                m += sorted(self.rng.choice(list(range(start, start + per)), self.MASK_NUM,
                                            replace=False))
            mask_idx.append(m)
        for _ in range(B):
            idx = np.arange(self.MASK_NUM * 2)
            self.rng.shuffle(idx)
            shuffle.append(idx)
        return {"sub_idx": np.asarray(sub_idx, np.int64), "mask_idx": np.asarray(mask_idx, np.int64),
                "shuffle": np.asarray(shuffle, np.int64)}

    def _lin(self, x, store, name, act=0, bias=True):
        return K.LinearFn.apply(x, self._anchor, store, name + ".weight",
                                name + ".bias" if bias else None, act)

    def _ln(self, x, store, name, eps=1e-12):
        return K.LayerNormFn.apply(x, self._anchor, store, name, eps)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, masked_lm_labels=None,
                visual_feats=None, pos=None, obj_labels=None, matched_label=None, ans=None,
                draws=None):
        """:1734-2484 for the image-only MRM objective. `input_ids` may be the batch dict
        (input_ids, attention_mask, images [B, N, 3, R, R]); `draws` the explicit random
        choices (else drawn from self.rng)."""
        if isinstance(input_ids, dict):
            batch = input_ids
            visual_feats = batch.get("images")
            draws = batch.get("draws", draws)
        images = visual_feats.to(self.device_, torch.float32).contiguous()
        B, Nimg = images.shape[:2]
        inner = self.bert
        st_in, st = inner.store, self.store
        for s in self.stores():
            if s.shadow_stale:
                s.refresh_shadows()
        V = inner.vision
        g = images.shape[-1] // V["patch"]
        Tv = 1 + 2 * g * g
        if draws is None:
            draws = self.draw(B, Nimg, Tv)
        dev = self.device_
        sub_idx = torch.as_tensor(np.asarray(draws["sub_idx"]), dtype=torch.int64)
        mask_idx = torch.as_tensor(np.asarray(draws["mask_idx"]), dtype=torch.int64)
        shuffle = np.asarray(draws["shuffle"], dtype=np.int64)
        nm = mask_idx.shape[1]
        sub_idx = sub_idx.to(dev).view(B, 1, 2).contiguous()
        mask_idx = mask_idx.to(dev)
        D = inner.new_dropouts()
        ph = self.config.hidden_dropout_prob
        # CLIP ViT over the two sub-sampled images of each story (img_len = 2)
        with torch.no_grad():  # only vout.detach() is used: the blocks skip their saves
            vout, Tv = inner.visual_forward(images, sub_idx)  # [B * Tv, E]
        E = vout.shape[-1]
        # MRM masking (:948-1009): targets = visn_fc(features at the masked patches), the
        # sequence fed on has them zeroed; the ViT's gradient is exactly zero (docstring)
        vseq = vout.detach().view(B, Tv, E)
        bidx = torch.arange(B, device=dev)[:, None]
        gt = vseq[bidx, mask_idx]  # [B, nm, E]
        keep = torch.ones(B, Tv, 1, device=dev, dtype=vseq.dtype)
        keep[bidx, mask_idx] = 0
        vmasked = vseq * keep
        vf = "encoder.visn_fc."
        visn = K.dropout(self._ln(self._lin(vmasked, st_in, vf + "visn_fc"), st_in,
                                  vf + "visn_layer_norm"), D.site(ph, "pt_visn_fc"))
        targets = K.dropout(self._ln(self._lin(gt.contiguous(), st_in, vf + "visn_fc"), st_in,
                                     vf + "visn_layer_norm"), D.site(ph, "pt_visn_fc_gt"))
        H = visn.shape[-1]
        # pooler (:1575-1578 with img_part): dense(token 0), no tanh
        pooled = self._lin(visn[:, 0].contiguous(), st_in, "pooler.dense")
        # BertPreTrainingHeads (:2247): LM head over every visual token + seq_relationship
        self.last_prediction_scores = self._lm_head(visn.reshape(B * Tv, H)).view(B, Tv, -1)
        self.last_seq_relationship = self._lin(pooled, st, "cls.seq_relationship")
        # answer head (:2249-2250): Linear(H, 2H) + GeLU + LN + Linear(2H, 2)
        a = "answer_head.logit_fc."
        answer = self._lin(self._ln(self._lin(pooled, st, a + "0", act=K.GELU), st, a + "2"),
                           st, a + "3")
        # MRM classification (:2309-2351)
        masked = visn[bidx, mask_idx]  # [B, nm, H], positions ascending = target order
        shuf = torch.as_tensor(shuffle, device=dev)
        tshuf = targets[bidx, shuf]  # mask_patch_gt[i][indices]
        qa = torch.cat([masked[:, :, None, :].expand(B, nm, nm, H),
                        tshuf[:, None, :, :].expand(B, nm, nm, H)], -1)  # [B, j, k, 2H]
        m = "patch_based_mrm_classification_head."
        hdn = self._ln(self._lin(qa.contiguous(), st, m + "transform.dense", act=K.GELU), st,
                       m + "transform.LayerNorm")
        scores = K.LinearFn.apply(hdn, self._anchor, st, m + "decoder.weight", m + "bias", 0)
        scores = scores.view(B, nm, nm).float()
        labels = torch.as_tensor(np.argsort(shuffle, axis=1), device=dev)  # indices_argsort
        logp = torch.log_softmax(scores, -1)
        ce = -logp.gather(-1, labels[:, :, None]).squeeze(-1).mean(-1)  # CrossEntropyLoss per story
        mrm = ce.sum() * self.MRM_SCALE
        losses = mrm.detach().view(1, 1)
        return mrm, losses, answer.detach()

    def _lm_head(self, x):
        """BertLMPredictionHead (:1157-1173): transform (dense + erf-GELU + LN 1e-12) and the tied
        decoder + bias as one MFMA GEMM into a row-padded buffer (ld = vocab rounded up to 64)."""
        st, st_in = self.store, self.bert.store
        p = "cls.predictions."
        h = self._ln(self._lin(x, st, p + "transform.dense", act=K.GELU), st, p + "transform.LayerNorm")
        Wd = st_in.w("embeddings.word_embeddings.weight")  # [V, H] compute dtype (tied)
        V = Wd.shape[0]
        ldc = (V + 63) // 64 * 64
        out = torch.empty(h.shape[0], ldc, device=h.device, dtype=h.dtype)
        with torch.no_grad():  # not in the loss (masked_lm_labels is None for img_part)
            N.gemm(h.detach(), Wd, out, h.shape[0], V, h.shape[-1], ldc=ldc,
                   bias=st.f32(p + "bias"))
        return out[:, :V]


def build_config2(device="cuda", dtype=torch.bfloat16, seed=0, vision="ViT-B/16", joint=None):
    """Config 2 (scripts/wikihow_image_only_pretrain.sh): bert-base-uncased sizes (vocab 30522,
    type vocab 2, 512 positions) around a CLIP ViT-B/16, N = 5 images per story."""
    from .lxrt import CLIP_VISION
    j = dict(vocab_size=30522, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
             intermediate_size=3072, max_position_embeddings=512, type_vocab_size=2)
    j.update(joint or {})
    vis = dict(vision) if isinstance(vision, dict) else dict(CLIP_VISION[vision])
    return LXRTPretraining(LXRTConfig(**j), visual_losses="obj", multimodal_text_part=False,
                           multimodal_img_part=True, cls_id=0, sep_id=2, pad_id=1,
                           max_story_length=5, mlm_ignore_index=-1,
                           multimodal_pretrain_objectives=["patch_based_mrm_classification"],
                           clip_model_name="ViT-B/16", pretraining=True, device=device,
                           compute_dtype=dtype, seed=seed, vision=vis)
