"""CPU fp32 restatement of the reference hot path — TEST INFRASTRUCTURE ONLY.

This module is the parity oracle (and the `cpu_baseline` leg of bench.py). It is never imported
by the product package `multimodal_sequencing_amd`; only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s cpu_baseline may use it, and only as the checker / baseline.

It restates, as plain functional PyTorch on CPU in fp32, the reference's multimodal
sequence-ordering path, written from the reference semantics and
citing the reference file:line each function follows. Parity is PINNED: `tests/test_oracle.py`
checks it against golden fixtures produced by running the reference itself in the development
container (`tests/golden/make_golden.py`): losses, gradients, intermediates and beam orders.

Parameters are passed as a flat dict keyed by the reference state-dict names.
"""
import itertools
import math

import numpy as np
import torch
import torch.nn.functional as F

CLS_ID, PAD_ID, SEP_ID = 0, 1, 2  # RoBERTa ids (SURVEY §8c "Unavailable offline")


# ----------------------------------------------------------------------------------------------
# a1: pair expansion — models/berson/process_inputs_for_berson.py:13-368
# ----------------------------------------------------------------------------------------------
def pairs_generator(n):
    """process_inputs_for_berson.py:246-261: combinations(i<j) then the reversed pairs."""
    one = [[a, b] for a, b in itertools.combinations(range(n), 2)]
    return one + [[b, a] for a, b in one]


def prepare_berson_inputs(input_ids, labels, n_steps, cls_id=CLS_ID, sep_id=SEP_ID, pad_id=PAD_ID,
                          img_part=False):
    """Restates prepare_berson_inputs (:13-79), parse_input_ids (:100-110),
    prepare_single_instance (:113-243) and preprocess_batch (:264-368) on numpy ints."""
    input_ids = np.asarray(input_ids)
    labels = np.asarray(labels)
    B = input_ids.shape[0]
    pairs = pairs_generator(n_steps)
    per_story = []
    for b in range(B):
        row = input_ids[b]
        starts = np.nonzero(row == cls_id)[0]
        ends = np.nonzero(row == sep_id)[0]
        assert len(starts) == len(ends) == n_steps
        sents = [row[s:e + 1] for s, e in zip(starts, ends)]
        gt = list(labels[b])
        ids_l, tt_l, sep_l, pl_l = [], [], [], []
        for a, c in pairs:
            fa, fc = gt.index(a), gt.index(c)
            pl_l.append(1 if fa < fc else 0)
            s1, s2 = sents[a], sents[c]
            ids_l.append(np.concatenate([s1, s2]))
            # cls_id == 0 (RoBERTa): all token types 0 (:205-208)
            tt_l.append(np.zeros(len(s1) + len(s2), np.int64) if cls_id == 0 else
                        np.concatenate([np.zeros(len(s1), np.int64), np.ones(len(s2), np.int64)]))
            sep_l.append([0, 1] if img_part else [len(s1) - 1, len(s1) + len(s2) - 1])
        per_story.append((ids_l, tt_l, sep_l, pl_l, gt))
    maxlen = max(len(x) for st in per_story for x in st[0])
    npair = len(pairs)
    out = {k: [] for k in ["input_ids", "attention_mask", "token_type_ids", "sep_positions",
                           "pairwise_labels", "ground_truth"]}
    for ids_l, tt_l, sep_l, pl_l, gt in per_story:
        out["input_ids"].append([list(x) + [pad_id] * (maxlen - len(x)) for x in ids_l])
        # quirk (Appendix C.7): the pair mask is padded with pad_id (=1), so pads are attended
        out["attention_mask"].append([[1] * len(x) + [pad_id] * (maxlen - len(x)) for x in ids_l])
        out["token_type_ids"].append([list(x) + [0] * (maxlen - len(x)) for x in tt_l])
        out["sep_positions"].append(sep_l)
        out["pairwise_labels"].append(pl_l)
        out["ground_truth"].append(gt)
    res = {k: np.asarray(v, dtype=np.int64) for k, v in out.items()}
    res["pairs_list"] = np.tile(np.asarray(pairs, np.int64)[None], (B, 1, 1))
    res["passage_length"] = np.full((B,), n_steps, np.int64)
    res["pairs_num"] = np.full((B,), npair, np.int64)
    res["mask_cls"] = np.ones((B, n_steps), np.int64)
    return res


def gather_pair_images(images, pairs_list):
    """process_images (:82-97): [B,N,3,R,R] -> [B*P, 2, 3, R, R] in pair order."""
    B = images.shape[0]
    idx = torch.as_tensor(pairs_list)
    out = images[torch.arange(B)[:, None, None], idx]  # [B, P, 2, 3, R, R]
    return out.reshape(-1, *out.shape[2:])


# ----------------------------------------------------------------------------------------------
# shared primitives
# ----------------------------------------------------------------------------------------------
def linear(x, p, name, bias=True):
    y = x @ p[name + ".weight"].t()
    if bias and (name + ".bias") in p:
        y = y + p[name + ".bias"]
    return y


def layer_norm(x, p, name, eps):
    return F.layer_norm(x, (x.shape[-1],), p[name + ".weight"], p[name + ".bias"], eps)


def gelu_erf(x):  # lxrt/modeling.py:116-122
    return x * 0.5 * (1.0 + torch.erf(x / math.sqrt(2.0)))


def gelu_tanh(x):  # berson/neural.py:7-8
    return 0.5 * x * (1 + torch.tanh(math.sqrt(2 / math.pi) * (x + 0.044715 * torch.pow(x, 3))))


def quick_gelu(x):  # clip/model.py:199-201
    return x * torch.sigmoid(1.702 * x)


def mha(q, k, v, heads, key_bias=None):
    """softmax(q k^T / sqrt(d) + key_bias) v over [B, T, heads*d]; key_bias [B, Tk] additive."""
    B, Tq, D = q.shape
    Tk = k.shape[1]
    d = D // heads
    qh = q.view(B, Tq, heads, d).transpose(1, 2)
    kh = k.view(B, Tk, heads, d).transpose(1, 2)
    vh = v.view(B, Tk, heads, d).transpose(1, 2)
    s = qh @ kh.transpose(-1, -2) / math.sqrt(d)
    if key_bias is not None:
        s = s + key_bias[:, None, None, :]
    a = torch.softmax(s, -1)
    return (a @ vh).transpose(1, 2).reshape(B, Tq, D)


# ----------------------------------------------------------------------------------------------
# a4: CLIP VisualTransformer — models/CLIP/clip/model.py:242-305 (+204-239, 190-201)
# ----------------------------------------------------------------------------------------------
VIT = "bert.encoder.visual_model.visual."


def vit_forward(p, images, img_len=2, heads=None):
    """images [P*img_len, 3, R, R] -> [P, 1 + img_len*g*g, E] (no ln_post: lxrt:783, model.py:301-304)."""
    w = p[VIT + "conv1.weight"]  # [W, 3, ps, ps]
    W, _, ps, _ = w.shape
    heads = heads or W // 64
    x = F.conv2d(images, w, stride=ps)  # :263
    npatch = x.shape[2] * x.shape[3]
    x = x.reshape(x.shape[0], W, -1).permute(0, 2, 1)  # [*, g*g, W]
    Pn = x.shape[0] // img_len
    x = x.reshape(Pn, -1, W)  # img0 patches then img1 patches (:267-268)
    cls = p[VIT + "class_embedding"] + torch.zeros(Pn, 1, W)
    x = torch.cat([cls, x], 1)
    pos = p[VIT + "positional_embedding"]
    if img_len > 1:  # quirk (App. C.1): img1 reuses rows [0..npatch-1] (:271-275)
        pos = torch.cat([pos] + [pos[:npatch]] * (img_len - 1), 0)
    x = x + pos
    x = layer_norm(x, p, VIT + "ln_pre", 1e-5)
    nl = len({k.split(".")[6] for k in p if k.startswith(VIT + "transformer.resblocks.")})
    for i in range(nl):
        b = f"{VIT}transformer.resblocks.{i}."
        h = layer_norm(x, p, b + "ln_1", 1e-5)
        qkv = h @ p[b + "attn.in_proj_weight"].t() + p[b + "attn.in_proj_bias"]
        q, k, v = qkv.split(W, -1)
        a = mha(q, k, v, heads)
        x = x + linear(a, p, b + "attn.out_proj")
        h = layer_norm(x, p, b + "ln_2", 1e-5)
        x = x + linear(quick_gelu(linear(h, p, b + "mlp.c_fc")), p, b + "mlp.c_proj")
    return x @ p[VIT + "proj"]


# ----------------------------------------------------------------------------------------------
# a3, a5-a8: LXRTModel / LXRTEncoder (VisualBERT style) — models/CLIP/src/lxrt/modeling.py
# ----------------------------------------------------------------------------------------------
def bert_embeddings(p, ids, tt):
    """BertEmbeddings.forward (:356-370): positions 0..L-1, LN eps 1e-12 (App. C.6)."""
    L = ids.shape[1]
    pos = torch.arange(L)[None].expand_as(ids)
    # padding_idx=0 on all three tables (:347-349): row 0 never receives a gradient
    e = (F.embedding(ids, p["bert.embeddings.word_embeddings.weight"], padding_idx=0)
         + F.embedding(pos, p["bert.embeddings.position_embeddings.weight"], padding_idx=0)
         + F.embedding(tt, p["bert.embeddings.token_type_embeddings.weight"], padding_idx=0))
    return layer_norm(e, p, "bert.embeddings.LayerNorm", 1e-12)


def bert_layer(p, i, x, key_bias, heads):
    """BertLayer (:496-507) = BertSelfattLayer (:454-464) + BertIntermediate + BertOutput."""
    b = f"bert.encoder.layer.{i}."
    q = linear(x, p, b + "attention.self.query")
    k = linear(x, p, b + "attention.self.key")
    v = linear(x, p, b + "attention.self.value")
    a = mha(q, k, v, heads, key_bias)  # BertAttention.forward (:398-425)
    h = layer_norm(linear(a, p, b + "attention.output.dense") + x, p,
                   b + "attention.output.LayerNorm", 1e-12)  # BertAttOutput (:435-439)
    f = gelu_erf(linear(h, p, b + "intermediate.dense"))  # :470-479
    return layer_norm(linear(f, p, b + "output.dense") + h, p, b + "output.LayerNorm", 1e-12)


def lxrt_forward(p, ids, mask, tt, images=None, heads=12, img_len=2, vit_heads=None):
    """LXRTModel.forward (:1513-1598) -> (lang_feats [P,Lt,H], visn_feats or None)."""
    ext = (1.0 - mask.float()) * -10000.0  # :1537-1545
    lang = bert_embeddings(p, ids, tt)
    nl = len({k.split(".")[3] for k in p if k.startswith("bert.encoder.layer.")})
    if images is not None:
        vis = vit_forward(p, images, img_len, vit_heads)  # lxrt:881-882
        vis = layer_norm(linear(vis, p, "bert.encoder.visn_fc.visn_fc"), p,
                         "bert.encoder.visn_fc.visn_layer_norm", 1e-12)  # :597-602
        joint = torch.cat([lang, vis], 1)  # :1093
        key_bias = torch.cat([ext, torch.zeros(vis.shape[0], vis.shape[1])], 1)  # :1071-1094
    else:
        joint, key_bias = lang, ext
    for i in range(nl):
        joint = bert_layer(p, i, joint, key_bias, heads)
    Lt = ids.shape[1]
    return joint[:, :Lt], (joint[:, Lt:] if images is not None else None)


# ----------------------------------------------------------------------------------------------
# a9: HierarchicalAttention — models/berson/modeling_bert.py:666-817
# ----------------------------------------------------------------------------------------------
def hierarchical_attention(p, top_vec, cls_pooled, pairs_list, sep_positions, n_steps):
    P, Lt, H = top_vec.shape
    B = pairs_list.shape[0]
    npair = pairs_list.shape[1]
    pre = "two_level_encoder."
    score = linear(torch.tanh(linear(top_vec, p, pre + "sentence_tran")), p,
                   pre + "sentence_tran_2").squeeze(-1)  # :697-701
    sep = torch.as_tensor(sep_positions).reshape(P, 2)
    pos = torch.arange(Lt)[None]
    m0 = ((pos >= 1) & (pos <= sep[:, :1])).float()  # :711
    m1 = ((pos > sep[:, :1]) & (pos <= sep[:, 1:])).float()  # :712
    sel = torch.stack([m0, m1], 1)  # [P, 2, Lt]
    scores = sel * score[:, None, :] + (1.0 - sel) * -10000.0  # :722-731
    probs = torch.softmax(scores, -1)
    mix = (probs @ top_vec).reshape(B, npair, 2, H)  # :738-741

    cls_score = linear(cls_pooled, p, pre + "pairwise_relationship")  # :745
    cls_b = cls_pooled.reshape(B, npair, H)
    cs_b = cls_score.reshape(B, npair, 2)
    N = n_steps
    final = torch.zeros(B, N, H)
    cls_mat = torch.zeros(B, N, N, H)
    cs_mat = torch.zeros(B, N, N, 2)
    pl = np.asarray(pairs_list)
    for b in range(B):  # :766-815
        slots = [[] for _ in range(N)]
        for j in range(npair):
            a, c = int(pl[b, j, 0]), int(pl[b, j, 1])
            slots[a].append(mix[b, j, 0])
            slots[c].append(mix[b, j, 1])
            cls_mat[b, a, c] = cls_b[b, j]
            cs_mat[b, a, c] = cs_b[b, j]
        sample = torch.stack([torch.stack(s) for s in slots])  # [N, edge, H]
        q2 = (sample @ p[pre + "linear_in_2.weight"].t()).squeeze(-1)  # [N, edge]
        w = torch.softmax(q2, -1)
        final[b] = (w[:, None, :] @ sample).squeeze(1)
    return final, cls_mat, cls_score, cs_mat


# ----------------------------------------------------------------------------------------------
# a10: TransformerInterEncoder — models/berson/encoder.py:9-61, neural.py:11-235
# ----------------------------------------------------------------------------------------------
def inter_encoder(p, x, mask, heads):
    mask = mask.float()
    x = x * mask[:, :, None]  # encoder.py:53
    key_bias = (1.0 - mask) * -10000.0  # neural.py:210-213 with mask = 1 - mask_cls
    nl = len({k.split(".")[2] for k in p if k.startswith("encoder.transformer_inter.")})
    for i in range(nl):
        b = f"encoder.transformer_inter.{i}."
        h = layer_norm(x, p, b + "layer_norm", 1e-6) if i != 0 else x  # encoder.py:21-24
        q = linear(h, p, b + "self_attn.linear_query")
        k = linear(h, p, b + "self_attn.linear_keys")
        v = linear(h, p, b + "self_attn.linear_values")
        ctx = mha(q, k, v, heads, key_bias)
        out = linear(ctx, p, b + "self_attn.final_linear") + x  # encoder.py:28-29
        f = linear(gelu_tanh(linear(layer_norm(out, p, b + "feed_forward.layer_norm", 1e-6), p,
                                    b + "feed_forward.w_1")), p, b + "feed_forward.w_2")
        x = f + out  # neural.py:30-33
    return layer_norm(x, p, "encoder.layer_norm", 1e-6)  # encoder.py:58


# ----------------------------------------------------------------------------------------------
# a11-a12: encode tail + pointer decoder + losses — modeling_bert.py:1338-1357, 943-1174
# ----------------------------------------------------------------------------------------------
def lstm_cell(p, x, h, c):
    g = (x @ p["decoder.weight_ih_l0"].t() + p["decoder.bias_ih_l0"]
         + h @ p["decoder.weight_hh_l0"].t() + p["decoder.bias_hh_l0"])
    i, f, gg, o = g.chunk(4, -1)
    c2 = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
    h2 = torch.sigmoid(o) * torch.tanh(c2)
    return h2, c2


def encode(p, pair, images, cfg):
    """BertForOrdering.encode (:1239-1366) with the clip inner model."""
    B, npair, Lt = pair["input_ids"].shape
    P = B * npair
    ids = torch.as_tensor(pair["input_ids"]).reshape(P, Lt)
    msk = torch.as_tensor(pair["attention_mask"]).reshape(P, Lt)
    tt = torch.as_tensor(pair["token_type_ids"]).reshape(P, Lt)
    img = None
    if images is not None and not cfg.get("text_only", False):
        img = gather_pair_images(images, pair["pairs_list"]).reshape(-1, *images.shape[2:])
    lang, _vis = lxrt_forward(p, ids, msk, tt, img, cfg["heads"], 2, cfg.get("vit_heads"))
    cls_pooled = lang[:, 0]  # :1290 (no pooler on the clip path)
    N = pair["mask_cls"].shape[1]
    final, cls_mat, cls_score, cs_mat = hierarchical_attention(
        p, lang, cls_pooled, pair["pairs_list"], pair["sep_positions"], N)
    mask_cls = torch.as_tensor(pair["mask_cls"])
    clean = final * mask_cls[:, :, None].float()  # :1338
    para = inter_encoder(p, clean, mask_cls, cfg["inter_heads"]) * mask_cls[:, :, None]  # :1343-1346
    plen = torch.as_tensor(pair["passage_length"]).float()
    para_vec = para.sum(1) / (plen + 1e-20)[:, None]  # :1348-1350
    okey = linear(torch.cat([clean, para], -1), p, "key_linear")  # :1356-1357
    return dict(clean=clean, para=para, hcn=(para_vec, torch.zeros_like(para_vec)), okey=okey,
                cls_mat=cls_mat, cls_score=cls_score, cs_mat=cs_mat, lang=lang)


def pointer_forward(p, enc, pair, lam=0.6):
    """_forward (:943-1174): pointer decoder + losses; returns (loss, logp [B,N,N])."""
    target = torch.as_tensor(pair["ground_truth"])
    tgt_len = torch.as_tensor(pair["passage_length"])
    B, N = target.shape
    doc = enc["clean"]
    ar = torch.arange(B)
    valid = torch.arange(N)[None] < tgt_len[:, None]  # pointed_mask_by_target / target_mask
    rela_mask = (1 - torch.eye(N, dtype=torch.long))[None].repeat(B, 1, 1)
    rela_mask = rela_mask * valid[:, :, None] * valid[:, None, :]  # :989-994
    dec_in = torch.cat([torch.zeros(B, 1, doc.shape[2]), doc[ar[:, None], target[:, :-1]]], 1)
    rela = torch.cat([enc["cls_mat"], torch.softmax(enc["cs_mat"], -1)], -1)  # rela_encode :919
    hist = rela.clone()  # history_encode with cls_score_matrix_nn for both (:1016)
    h, c = enc["hcn"]
    pointed = [torch.zeros(B, N, dtype=torch.long)]
    keys, outs = [], []
    rela_live = rela
    for t in range(N):
        l1 = torch.zeros(B, N, 1)
        l2 = torch.zeros(B, N, 1)
        if t > 0:
            tar = target[:, t - 1]
            rela_mask = rela_mask.clone()
            rela_mask[ar, tar] = 0
            rela_mask[ar, :, tar] = 0
            l1[ar, tar] = 1
            if t > 1:
                l2[ar, target[:, t - 2]] = 1
            pm = pointed[-1].clone()
            pm[ar, tar] = 1
            pointed.append(pm)
        cur1 = (hist * l1[:, :, None, :]).sum(1)  # :1053
        cur2 = (hist * l2[:, :, None, :]).sum(1)  # :1055
        rela_live = rela_live * (rela_mask[..., None] != 0)  # cumulative in-place mask (:1059)
        forw = rela_live.mean(2)
        back = rela_live.mean(1)
        keys.append(linear(torch.cat([cur1, cur2, forw, back], -1), p, "pw_k", bias=False))
        h, c = lstm_cell(p, dec_in[:, t], h, c)
        outs.append(h)
    query = linear(torch.stack(outs, 1), p, "query_linear")[:, :, None]  # :1083
    e = torch.tanh(query + torch.stack(keys, 1) + enc["okey"][:, None])  # :1098
    e = linear(e, p, "tanh_linear").squeeze(-1)
    pm = torch.stack(pointed, 1)
    e = e.masked_fill(pm == 1, -1e9).masked_fill(~valid[:, None, :], -1e9)  # :1112-1113
    logp = torch.log_softmax(e, -1)
    nll = -logp.gather(-1, target[:, :, None]).squeeze(-1) * valid.float()
    l_ptr = (nll.sum(-1) / (tgt_len.float() + 1e-20 - 1)).sum() / B  # :1140-1142
    pl = torch.as_tensor(pair["pairwise_labels"]).reshape(-1)
    lc = torch.log_softmax(enc["cls_score"], -1)
    pnll = -lc.gather(-1, pl[:, None]).squeeze(-1)
    npair = pair["pairwise_labels"].shape[1]
    pmask = (torch.arange(npair)[None] < torch.as_tensor(pair["pairs_num"])[:, None]).float()
    pnll = (pnll.reshape(B, npair) * pmask).sum(-1) / (torch.as_tensor(pair["pairs_num"]).float() + 1e-20)
    l_pair = pnll.sum() / B  # :1145-1172
    return l_ptr + l_pair * lam, logp


def forward_loss(p, input_ids, labels, images, cfg):
    """BertForOrdering.forward (:937-941) -> scalar fp32 loss (train.py:312,334)."""
    pair = prepare_berson_inputs(input_ids, labels, cfg["N"])
    enc = encode(p, pair, images, cfg)
    loss, _ = pointer_forward(p, enc, pair)
    return loss, pair, enc


# ----------------------------------------------------------------------------------------------
# a14: beam-search ordering — modeling_bert.py:1368-1552, generator.py:8-38
# ----------------------------------------------------------------------------------------------
def beam_order(p, enc, beam_size=16):
    """beam_search_pointer for one story (B = 1): returns the ordering as a list of ints."""
    doc = enc["clean"][0]
    T, H = doc.shape
    okeys = enc["okey"]  # [1, T, H]
    rela = torch.cat([enc["cls_mat"], torch.softmax(enc["cs_mat"], -1)], -1)
    hist = rela.clone()
    h, c = enc["hcn"]
    eye0 = (1 - torch.eye(T, dtype=torch.long))[None]
    cands, scores = [[]], [0.0]
    hyps = []
    valid = beam_size
    rela_mask = eye0.clone()
    pointed = torch.zeros(1, T, dtype=torch.long)
    x = torch.zeros(1, H)
    for t in range(T - 1):
        nb = len(cands)
        l1 = torch.zeros(rela_mask.shape[0], T)
        l2 = torch.zeros(rela_mask.shape[0], T)
        if t > 0:
            index = torch.tensor([cd[-1] for cd in cands])
            x = doc[index]
            ar = torch.arange(nb)
            pointed = pointed.clone()
            pointed[ar, index] = 1
            rela_mask = rela_mask.clone()
            rela_mask[ar, :, index] = 0
            rela_mask[ar, index] = 0
            l1[ar, index] = 1
            if t > 1:
                l2[ar, torch.tensor([cd[-2] for cd in cands])] = 1
        h, c = lstm_cell(p, x, h, c)  # step (:1375)
        q = linear(h, p, "query_linear")[:, None]
        left1 = (hist * l1[:, :, None, None]).sum(1)
        left2 = (hist * l2[:, :, None, None]).sum(1)
        rela = rela * (rela_mask[..., None] != 0)
        keys = linear(torch.cat([left1, left2, rela.mean(2), rela.mean(1)], -1), p, "pw_k", bias=False)
        e = linear(torch.tanh(q + keys + okeys), p, "tanh_linear").squeeze(-1)
        e = e.masked_fill(pointed == 1, -1e9)
        logp = torch.log_softmax(e, -1)
        # Beam.step (generator.py:15-38): k smallest of (-logp + prev score)
        score = -logp + torch.tensor(scores)[:, None]
        k = min(valid, score.numel())
        flat = score.reshape(-1)
        order = np.lexsort((np.arange(flat.numel()), flat.numpy()))[:k]  # ties -> lowest index
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
        ri = torch.tensor(remain, dtype=torch.long)
        h, c = h[ri], c[ri]
        pointed, rela_mask, rela, hist = pointed[ri], rela_mask[ri], rela[ri], hist[ri]
        cands, scores = new_c, new_s
    best = sorted(hyps, key=lambda z: z[1])[0][0]
    best = best + sorted(set(range(T)) - set(best))[:1]  # :1549-1550
    return best
