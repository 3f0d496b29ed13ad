"""BERSON ordering head: BertForOrdering, HierarchicalAttention, TransformerInterEncoder, the
pointer-network decoder, losses, and beam-search ordering.

Drop-in for models/berson/modeling_bert.py (BertForOrdering :825-1402, HierarchicalAttention
:666-817, beam_search_pointer :1411-1552, berson_pointer_network :1405-1408) and
models/berson/{encoder,neural,generator}.py: same constructor / forward contract
(`model(inputs) -> (loss,)`), same state-dict names.

What changes is HOW: no per-pair Python loops and no device->host syncs inside the forward —
the span pooling, pointer scoring and small attention run as HIP kernels, the pair<->sentence
scatters use static index maps for the fixed story length N, and the pointer decoder's mask
bookkeeping is vectorised over time steps. The head is tiny (< 0.1 % of FLOPs) and runs in fp32.
"""
import math
from types import SimpleNamespace

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from . import kernels as K
from .checkpoint import JsonConfigMixin, berson_from_pretrained, save_pretrained
from .params import ParamStore, Spec, attach_tree, linear_specs, ln_specs, normal, uniform, zeros
from .process_inputs import pairs_generator, prepare_berson_inputs


class BersonConfig(JsonConfigMixin, SimpleNamespace):
    """models/berson/configuration_bert.py:77-113 (the fields the head reads) plus the
    PretrainedConfig attributes (configuration_utils.py:46-58) that from_pretrained kwargs may
    override (train.py:2010-2011 passes num_labels and finetuning_task)."""

    def __init__(self, hidden_size=768, num_labels=1, initializer_range=0.02,
                 hidden_dropout_prob=0.1, **kw):
        for k, v in (("finetuning_task", None), ("output_attentions", False),
                     ("output_hidden_states", False), ("torchscript", False),
                     ("use_bfloat16", False), ("pruned_heads", {})):
            kw.setdefault(k, v)
        super().__init__(hidden_size=hidden_size, num_labels=num_labels,
                         initializer_range=initializer_range,
                         hidden_dropout_prob=hidden_dropout_prob, **kw)


def _head_specs(H, args, num_labels, std):
    ff, L = args.ff_size, args.inter_layers
    sp = linear_specs("classifier", H, num_labels, std=std)
    for i in range(L):
        b = f"encoder.transformer_inter.{i}."
        for n in ("linear_keys", "linear_values", "linear_query", "final_linear"):
            sp += linear_specs(b + "self_attn." + n, H, H, std=std)
        sp += linear_specs(b + "feed_forward.w_1", H, ff, std=std)
        sp += linear_specs(b + "feed_forward.w_2", ff, H, std=std)
        sp += ln_specs(b + "feed_forward.layer_norm", H)
        sp += ln_specs(b + "layer_norm", H)
    sp += ln_specs("encoder.layer_norm", H)
    sp += linear_specs("key_linear", 2 * H, H, std=std)
    sp += linear_specs("query_linear", H, H, std=std)
    sp += linear_specs("tanh_linear", H, 1, std=std)
    b = 1.0 / math.sqrt(H)  # nn.LSTM default init (re-initialised normal by _init_weights? no:
    # BertPreTrainedModel._init_weights touches Linear/Embedding/LayerNorm only)
    sp += [Spec("decoder.weight_ih_l0", (4 * H, H), uniform(b), transpose=True),
           Spec("decoder.weight_hh_l0", (4 * H, H), uniform(b), transpose=True),
           Spec("decoder.bias_ih_l0", (4 * H,), uniform(b)),
           Spec("decoder.bias_hh_l0", (4 * H,), uniform(b))]
    t = "two_level_encoder."
    sp += [Spec(t + "linear_in_2.weight", (1, H), normal(std), transpose=True)]
    sp += linear_specs(t + "sentence_tran", H, H, std=std)
    sp += linear_specs(t + "sentence_tran_2", H, 1, std=std)
    for n in ("pairwise_relationship", "h1_relationship", "h2_relationship"):
        sp += linear_specs(t + n, H, 2, std=std)
    sp += [Spec("pw_k.weight", (H, 4 * (H + 2)), normal(std), transpose=True)]
    return sp


class BertForOrdering(nn.Module):
    base_model_prefix = "bert"  # modeling_bert.py:462
    from_pretrained = classmethod(berson_from_pretrained)  # modeling_utils.py:208-428
    save_pretrained = save_pretrained  # modeling_utils.py:190-204

    def __init__(self, config, args, inner_model=None, tokenizer=None, load_inner_model=False,
                 device="cuda", seed=1, **kw):
        super().__init__()
        self.config = config
        self.args = args
        self.tokenizer = tokenizer
        H = config.hidden_size
        self.hidden_size = H
        self.pairwise_loss_lam = getattr(args, "pairwise_loss_lam", 0.6)
        self.n_steps = args.max_story_length
        self.store = ParamStore(_head_specs(H, args, getattr(config, "num_labels", 1),
                                            getattr(config, "initializer_range", 0.02)),
                                device, torch.float32)
        self.store.init_weights(seed=seed)
        # the inner model's slot comes first, as in the reference (`self.bert` is set before the
        # head at modeling_bert.py:860-866): named_parameters() order is what a reference-written
        # optimizer.pt indexes by position (trainer.FusedAdamW.load_state_dict)
        self.add_module("bert", inner_model)
        attach_tree(self, self.store.params)
        self._anchor = torch.zeros((), device=device, requires_grad=True)
        self.device_ = torch.device(device)
        self._maps = {}
        self.hidden_dropout_prob = getattr(config, "hidden_dropout_prob", 0.1)  # :677
        self.para_dropout = getattr(args, "para_dropout", 0.1)  # train.py:2014, :881
        self._drops = K.EVAL
        from .lxrt import _mark_stale
        self.register_load_state_dict_post_hook(_mark_stale)

    # ------------------------------------------------------------------------------------
    def ddp_units(self):
        """(units, begin_stores) for trainer.GradAllReduce: the inner model's per-layer spans;
        the head store completes as a whole before the inner model's backward begins."""
        units = {}
        if self.bert is not None:
            units[id(self.bert.store)] = self.bert.grad_units()
        return units, [self.store]

    def stores(self):
        return [self.bert.store, self.store] if self.bert is not None else [self.store]

    def zero_grad(self, set_to_none=False):  # keep the flat-buffer grad views alive
        for s in self.stores():
            s.zero_grad()

    def equip(self, critic):  # modeling_bert.py:916 (NLLLoss(reduction='none') is built in)
        self.critic = critic

    def _static_maps(self, N):
        """Index maps for the fixed story length (replace the host loops at :766-792)."""
        if N not in self._maps:
            pairs, npair = pairs_generator(N)
            E = 2 * (N - 1)
            slot = [[] for _ in range(N)]
            for j, (a, c) in enumerate(pairs):
                slot[a].append(2 * j)
                slot[c].append(2 * j + 1)
            dev = self.device_
            self._maps[N] = dict(
                slot=torch.tensor(slot, device=dev).view(N * E),  # into mix.view(B, 2*npair, H)
                pair_flat=torch.tensor([a * N + c for a, c in pairs], device=dev),
                E=E, npair=npair)
        return self._maps[N]

    def _lin(self, x, name, act=0, bias=True):
        return K.LinearFn.apply(x, self._anchor, self.store, name + ".weight",
                                name + ".bias" if bias else None, act)

    def _ln(self, x, name, eps):
        return K.LayerNormFn.apply(x, self._anchor, self.store, name, eps)

    # ------------------------------------------------------------------------------------
    def forward(self, inputs):
        """BertForOrdering.forward (:937-941): inputs = {input_ids [B][L], labels [B][N],
        images [B][N][3][R][R] (optional), ...} -> (loss,)."""
        berson = prepare_berson_inputs(inputs["input_ids"], inputs["labels"], self.n_steps,
                                       device=self.device_)
        images = inputs.get("images")
        if images is not None:
            images = images.to(self.device_, torch.float32, non_blocking=True).contiguous()
        berson["images"] = images
        return self._forward(**berson)

    def encode(self, input_ids, attention_mask=None, token_type_ids=None, pairs_list=None,
               passage_length=None, pairs_num=None, sep_positions=None, ground_truth=None,
               mask_cls=None, pairwise_labels=None, cuda=None, head_mask=None, images=None):
        """:1239-1366 — returns the same 10-tuple as the reference."""
        B, npair, Lt = input_ids.shape
        N = mask_cls.shape[1]
        H = self.hidden_size
        P = B * npair
        mp = self._static_maps(N)
        if self.store.shadow_stale:  # transposed fp32 weight shadows for the head's dgrad GEMMs
            self.store.refresh_shadows()
        D = self.bert.new_dropouts()
        D.training = D.training and self.training
        self._drops = D
        ph = self.hidden_dropout_prob
        joint, Lt = self.bert.encode_joint(input_ids.reshape(P, Lt),
                                           attention_mask.reshape(P, Lt),
                                           token_type_ids.reshape(P, Lt),
                                           images if not self.bert.text_part else None,
                                           pairs_list, drops=D, text_rows=True)
        top = joint[:, :Lt].float()  # lang_feats (:1289), fp32 for the head
        cls_pooled = top[:, 0]  # :1290
        # ---- HierarchicalAttention (:686-817) -------------------------------------------
        t = "two_level_encoder."
        if joint.dtype == torch.bfloat16:  # the head's one large GEMM on the bf16 MFMA kernels
            st = K.LinearLowpFn.apply(joint[:, :Lt], self._anchor, self.store,
                                      t + "sentence_tran.weight", t + "sentence_tran.bias", K.TANH)
        else:
            st = self._lin(top, t + "sentence_tran", act=K.TANH)
        score = self._lin(st, t + "sentence_tran_2")
        mix = K.SpanPoolFn.apply(top, score.view(P, Lt), sep_positions.reshape(P, 2).contiguous(),
                                 D.site(ph, "span"))  # :735
        sample = mix.view(B, 2 * npair, H)[:, mp["slot"]].view(B, N, mp["E"], H)
        q2 = K.LinearFn.apply(sample, self._anchor, self.store, t + "linear_in_2.weight", None, 0)
        wts = torch.softmax(q2.view(B, N, mp["E"]), -1)
        final = (wts.unsqueeze(-1) * sample).sum(2)  # [B, N, H]
        cls_score = self._lin(cls_pooled, t + "pairwise_relationship")  # [P, 2]
        cls_mat = torch.zeros(B, N * N, H, device=top.device)
        cls_mat = cls_mat.index_copy(1, mp["pair_flat"], cls_pooled.view(B, npair, H))
        cs_mat = torch.zeros(B, N * N, 2, device=top.device)
        cs_mat = cs_mat.index_copy(1, mp["pair_flat"], cls_score.view(B, npair, 2))
        cls_mat = cls_mat.view(B, N, N, H)
        cs_mat = cs_mat.view(B, N, N, 2)
        # h1/h2_relationship outputs are computed but never used downstream (:751-757, :1016):
        # they do not affect loss or gradients, so they are not evaluated here.
        # ---- encode tail (:1338-1357) -------------------------------------------------------
        mcf = mask_cls.float()
        clean = final * mcf[:, :, None]
        para = self._inter_encoder(clean, mcf) * mcf[:, :, None]
        plen = passage_length.float()
        para_vec = para.sum(1) / (plen + 1e-20)[:, None]
        hcn = (para_vec.unsqueeze(0), torch.zeros_like(para_vec).unsqueeze(0))
        okey = self._lin(torch.cat([clean, para], -1), "key_linear")
        return (clean, para, hcn, okey, cls_pooled, cls_mat, cls_score, cs_mat, cs_mat, cs_mat)

    def _inter_encoder(self, top_vecs, mask):
        """TransformerInterEncoder (encoder.py:46-61) + TransformerEncoderLayer (:20-30)."""
        x = top_vecs * mask[:, :, None]
        key_bias = ((1.0 - mask) * -10000.0).contiguous()  # neural.py:210-213 with mask = 1 - m
        heads = self.args.heads
        D = self._drops
        pd = self.para_dropout
        for i in range(self.args.inter_layers):
            b = f"encoder.transformer_inter.{i}."
            h = self._ln(x, b + "layer_norm", 1e-6) if i != 0 else x
            q = self._lin(h, b + "self_attn.linear_query")
            k = self._lin(h, b + "self_attn.linear_keys")
            v = self._lin(h, b + "self_attn.linear_values")
            ctx = K.SmallAttnFn.apply(q, k, v, key_bias, heads, D.site(pd, "inter_att", i))
            # encoder.py:28 and neural.py:31-33
            out = K.dropout(self._lin(ctx, b + "self_attn.final_linear"),
                            D.site(pd, "inter_ctx", i)) + x
            inter = K.dropout(self._lin(self._ln(out, b + "feed_forward.layer_norm", 1e-6),
                                        b + "feed_forward.w_1", act=K.GELU_TANH),
                              D.site(pd, "inter_ff1", i))
            f = K.dropout(self._lin(inter, b + "feed_forward.w_2"), D.site(pd, "inter_ff2", i))
            x = f + out
        return self._ln(x, "encoder.layer_norm", 1e-6)

    def _lstm_gx(self, x):
        """x W_ih^T + b_ih for every decoder input at once (one GEMM, not one per step)."""
        return K.LinearFn.apply(x, self._anchor, self.store, "decoder.weight_ih_l0",
                                "decoder.bias_ih_l0", 0)

    def _lstm_step(self, gx, h, c):
        """nn.LSTM single step (gate order i, f, g, o) from precomputed input gates: the h GEMM
        and one fused cell kernel (sigmoid/tanh gates, c', h')."""
        gh = K.LinearFn.apply(h, self._anchor, self.store, "decoder.weight_hh_l0",
                              "decoder.bias_hh_l0", 0)
        return K.LstmCellFn.apply(gx, gh, c)

    def _forward(self, input_ids, attention_mask=None, token_type_ids=None, pairs_list=None,
                 passage_length=None, pairs_num=None, sep_positions=None, ground_truth=None,
                 mask_cls=None, pairwise_labels=None, cuda=None, head_mask=None, images=None):
        """:943-1237 — pointer decoder + pointer NLL + 0.6 * pairwise NLL."""
        (doc, _para, hcn, okey, _cls, cls_mat, cls_score, cs_mat, _h1, _h2) = self.encode(
            input_ids, attention_mask, token_type_ids, pairs_list, passage_length, pairs_num,
            sep_positions, ground_truth, mask_cls, pairwise_labels, cuda, head_mask, images)
        target = ground_truth
        tgt_len = passage_length
        B, N = target.shape
        H = self.hidden_size
        dev = doc.device
        ar = torch.arange(N, device=dev)
        valid = ar[None] < tgt_len[:, None]  # [B, N]
        # pointed_before[b][t][j] = j in target[b, :t]  (cumulative masks of :1027-1050)
        onehot = F.one_hot(target, N).to(torch.int64)  # [B, N(t), N(j)]
        pointed = (onehot.cumsum(1) - onehot).clamp_(max=1)  # exclusive prefix
        base = (1 - torch.eye(N, dtype=torch.int64, device=dev))[None] * valid[:, :, None] * \
            valid[:, None, :]
        alive = 1 - pointed  # rows/cols of already-pointed sentences are zeroed (:1036-1037)
        rela_mask = base[:, None] * alive[:, :, :, None] * alive[:, :, None, :]  # [B,t,i,j]
        rela = torch.cat([cls_mat, torch.softmax(cs_mat, -1)], -1)  # rela_encode (:919-925)
        hist = rela  # history_encode with cls_score_matrix_nn for both (:1016)
        live = rela[:, None] * rela_mask[..., None].to(rela.dtype)  # [B, t, i, j, H+2]
        forw = live.mean(3)  # rela_vec.mean(2) per t (:1061)
        back = live.mean(2)  # rela_vec.mean(1) per t (:1062)
        bidx = torch.arange(B, device=dev)[:, None]
        prev1 = torch.cat([target.new_zeros(B, 1), target[:, :-1]], 1)
        prev2 = torch.cat([target.new_zeros(B, 2), target[:, :-2]], 1)[:, :N]
        l1 = hist[bidx, prev1]  # [B, t, j, H+2] row target[t-1] (:1043, :1053)
        l2 = hist[bidx, prev2]
        l1 = l1 * (ar >= 1).to(l1.dtype)[None, :, None, None]
        l2 = l2 * (ar >= 2).to(l2.dtype)[None, :, None, None]
        pw_info = torch.cat([l1, l2, forw, back], -1)  # [B, t, j, 4(H+2)]
        pw_keys = K.LinearFn.apply(pw_info, self._anchor, self.store, "pw_k.weight", None, 0)
        dec_in = torch.cat([doc.new_zeros(B, 1, H), doc[bidx, target[:, :-1]]], 1)  # :998-1002
        h, c = hcn[0][0], hcn[1][0]
        gx = self._lstm_gx(dec_in)  # [B, N, 4H]
        outs = []
        for t in range(N):
            h, c = self._lstm_step(gx[:, t], h, c)
            outs.append(h)
        query = self._lin(torch.stack(outs, 1), "query_linear")
        nll, _logp = K.PointerFn.apply(query, pw_keys, okey, self._anchor, self.store,
                                       "tanh_linear.weight", "tanh_linear.bias",
                                       pointed.to(torch.uint8).contiguous(), tgt_len.contiguous(),
                                       target.contiguous())
        l_ptr = (nll.sum(-1) / (tgt_len.float() + 1e-20 - 1)).sum() / B  # :1140-1142
        npair = pairwise_labels.shape[1]
        lc = torch.log_softmax(cls_score, -1)
        pnll = -lc.gather(-1, pairwise_labels.reshape(-1, 1)).view(B, npair)
        pmask = (torch.arange(npair, device=dev)[None] < pairs_num[:, None]).float()
        l_pair = ((pnll * pmask).sum(-1) / (pairs_num.float() + 1e-20)).sum() / B  # :1145-1172
        self.last_loss_terms = (l_ptr.detach(), l_pair.detach())  # (pointer, pairwise) losses
        return (l_ptr + l_pair * self.pairwise_loss_lam,)

    # ------------------------------------------------------------------------------------
    @torch.no_grad()
    def step(self, prev_y, prev_h, prev_c, original_keys, pointed, rela, rela_mask, hist, l1_idx,
             l2_idx):
        """BertForOrdering.step (:1368-1402) for a beam of candidates."""
        h, c = self._lstm_step(self._lstm_gx(prev_y), prev_h, prev_c)
        q = self._lin(h, "query_linear")[:, None]  # [beam, 1, H]
        nb, T = pointed.shape
        zeros = rela.new_zeros(nb, T, rela.shape[-1])
        left1 = hist[torch.arange(nb), l1_idx] if l1_idx is not None else zeros
        left2 = hist[torch.arange(nb), l2_idx] if l2_idx is not None else zeros
        rela = rela * rela_mask[..., None].to(rela.dtype)
        pw = torch.cat([left1, left2, rela.mean(2), rela.mean(1)], -1)
        keys = K.LinearFn.apply(pw, self._anchor, self.store, "pw_k.weight", None, 0)
        e = torch.tanh(q + keys + original_keys)
        e = K.LinearFn.apply(e, self._anchor, self.store, "tanh_linear.weight",
                             "tanh_linear.bias", 0).squeeze(-1)
        e = e.masked_fill(pointed.bool(), -1e9)
        return h, c, torch.log_softmax(e, -1), rela


@torch.no_grad()
def beam_search_pointer(args, model, input_ids, attention_mask=None, token_type_ids=None,
                        pairs_list=None, passage_length=None, pairs_num=None, sep_positions=None,
                        ground_truth=None, mask_cls=None, pairwise_labels=None, cuda=None,
                        head_mask=None, images=None):
    """:1411-1552 + generator.py Beam (B = 1). Ties in the k-smallest selection break toward the
    lowest flat index (deterministic); returns the ordering as a list of ints."""
    (sent, _p, dec_init, okeys, _cls, cls_mat, _cs, cs_mat, _h1, _h2) = model.encode(
        input_ids, attention_mask, token_type_ids, pairs_list, passage_length, pairs_num,
        sep_positions, ground_truth, mask_cls, pairwise_labels, cuda, head_mask, images)
    T = int(mask_cls.shape[1])
    doc = sent[0]
    H = doc.shape[-1]
    dev = doc.device
    rela = torch.cat([cls_mat, torch.softmax(cs_mat, -1)], -1)
    hist = rela.clone()
    W = getattr(args, "beam_size", 16)
    cands, scores, hyps = [[]], [0.0], []
    valid = W
    h, c = dec_init[0][0], dec_init[1][0]
    rela_mask = (1 - torch.eye(T, dtype=torch.int64, device=dev))[None]
    pointed = torch.zeros(1, T, dtype=torch.int64, device=dev)
    x = torch.zeros(1, H, device=dev)
    for t in range(T - 1):
        nb = len(cands)
        l1_idx = l2_idx = None
        if t > 0:
            index = torch.tensor([cd[-1] for cd in cands], device=dev)
            x = doc[index]
            ar = torch.arange(nb, device=dev)
            pointed = pointed.clone()
            pointed[ar, index] = 1
            rela_mask = rela_mask.clone()
            rela_mask[ar, :, index] = 0
            rela_mask[ar, index] = 0
            l1_idx = index
            if t > 1:
                l2_idx = torch.tensor([cd[-2] for cd in cands], device=dev)
        h, c, logp, rela = model.step(x, h, c, okeys, pointed, rela, rela_mask, hist, l1_idx, l2_idx)
        score = (-logp + torch.tensor(scores, device=dev)[:, None]).float().cpu()
        flat = score.reshape(-1).numpy()
        k = min(valid, flat.size)
        order = np.lexsort((np.arange(flat.size), flat))[:k]
        new_c, new_s, remain = [], [], []
        for ix in order:
            bi, ti = int(ix) // T, int(ix) % T
            cand = cands[bi] + [ti]
            if len(cand) == T - 1:
                hyps.append((cand, float(flat[ix])))
            else:
                remain.append(bi)
                new_c.append(cand)
                new_s.append(float(flat[ix]))
        valid -= k - len(remain)
        if valid == 0:
            break
        ri = torch.tensor(remain, dtype=torch.long, device=dev)
        h, c = h[ri], c[ri]
        pointed, rela_mask, rela, hist = pointed[ri], rela_mask[ri], rela[ri], hist[ri]
        cands, scores = new_c, new_s
    best = sorted(hyps, key=lambda z: z[1])[0][0]
    return best + sorted(set(range(T)) - set(best))[:1]


def berson_pointer_network(args, model, tokenizer, inputs):
    """:1405-1408 — ordering indices for one story."""
    berson = prepare_berson_inputs(inputs["input_ids"], inputs["labels"], model.n_steps,
                                   device=model.device_)
    images = inputs.get("images")
    if images is not None:
        images = images.to(model.device_, torch.float32).contiguous()
    berson["images"] = images
    return beam_search_pointer(args, model, **berson)
