"""Where does the bf16 error of the decisive config-3 margin come from? (VERDICT r3, next-round
item 1.) Measurement only, GPU.

Same counter weights (decisive_config3 scaling) in an fp32 model (the parity mode, which matches
the reference to 1e-4) and a bf16 model (the benchmarked mode). Per story of the fixture:

  * accumulated drift: relative L2 of every ViT block / joint BertLayer output, bf16 vs fp32;
  * local drift: the same layer run in bf16 on the fp32 model's input to that layer (rounded to
    bf16), against the fp32 layer output — the error each layer adds by itself;
  * head intermediates (lang_feats, clean/para/original keys) bf16 vs fp32;
  * the margin (second-best minus best order NLL) error against the fp32 margin for variants
      A  bf16 model as benchmarked,
      B  bf16 model with the head's sentence_tran GEMM in fp32,
      C  fp32 model with only its encoder output (lang_feats) rounded to bf16,
      D  fp32 model with the last joint layer's output rounded to bf16 and the rest fp32 (= C),
    so that "bf16 compute through 24 layers" and "bf16 storage of the head's input" separate.

usage: python tools/drift_probe.py [stories]  -> one JSON line per story + a summary line
"""
import itertools
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
from counter_init import counter_state_dict  # noqa: E402
from make_golden_real import CONFIG3, real_inputs, scale_decisive  # noqa: E402
from multimodal_sequencing_amd import kernels as K  # noqa: E402
from multimodal_sequencing_amd import model_zoo  # noqa: E402

NAME = "decisive_config3"
REC = {"on": False, "out": [], "inp": [], "replay": None}


def _wrap(cls):
    orig = cls.apply

    def apply(x, *a):
        if REC["replay"] is not None:  # local drift: this layer on the fp32 model's input
            x = REC["replay"].pop(0).to(x.dtype).view_as(x)
        y = orig(x, *a)
        if REC["on"]:
            REC["inp"].append(x.detach().float().clone())
            REC["out"].append(y.detach().float().clone())
        return y
    cls.apply = apply
    return orig


def model(dtype):
    cfg = dict(CONFIG3, B=4)
    m = model_zoo.build_from_golden(cfg, device="cuda", dtype=dtype)
    sd = scale_decisive(counter_state_dict({k: tuple(v.shape) for k, v in m.state_dict().items()}),
                        NAME)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m.eval()
    return m, cfg


def nll(m, inp, order):
    with torch.no_grad():
        m({**inp, "labels": torch.tensor([list(order)])})
    return float(m.last_loss_terms[0]) * (len(order) - 1)


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


def encode_rec(m, inp):
    from multimodal_sequencing_amd.process_inputs import prepare_berson_inputs
    bi = prepare_berson_inputs(inp["input_ids"], inp["labels"], m.n_steps, device="cuda")
    REC.update(on=True, out=[], inp=[])
    with torch.no_grad():
        enc = m.encode(**bi, images=inp["images"])
    REC["on"] = False
    return [x for x in REC["out"]], [x for x in REC["inp"]], enc


def main():
    stories = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    orig_vit = _wrap(K.VitBlockFn)
    orig_bert = _wrap(K.BertLayerFn)
    del orig_vit, orig_bert
    m32, cfg = model(torch.float32)
    m16, _ = model(torch.bfloat16)
    ids, labels, images = real_inputs(310, cfg)
    perms = list(itertools.permutations(range(cfg["N"])))
    nv = cfg["vit"]["layers"]
    summary = []
    for b in range(min(stories, ids.shape[0])):
        inp = {"input_ids": torch.from_numpy(ids[b:b + 1]), "labels": torch.from_numpy(labels[b:b + 1]),
               "images": torch.from_numpy(images[b:b + 1]).cuda()}
        # layer drift
        out32, in32, e32 = encode_rec(m32, inp)
        out16, _, e16 = encode_rec(m16, inp)
        acc = [rel(a, c) for a, c in zip(out16, out32)]
        REC["replay"] = [x.clone() for x in in32]
        loc16, _, _ = encode_rec(m16, inp)
        REC["replay"] = None
        loc = [rel(a, c) for a, c in zip(loc16, out32)]
        heads = {n: rel(e16[i].float(), e32[i].float()) for i, n in ((0, "clean"), (1, "para"), (3, "okey"))}
        # margins
        v32 = np.array([nll(m32, inp, p) for p in perms])
        o = np.argsort(v32)
        best, second = perms[o[0]], perms[o[1]]
        margin = float(v32[o[1]] - v32[o[0]])

        def gap(mm):
            return nll(mm, inp, second) - nll(mm, inp, best)
        errA = abs(gap(m16) - margin)
        lowp = K.LinearLowpFn.apply
        K.LinearLowpFn.apply = lambda x, a, s, w, bb, act: K.LinearFn.apply(x.float(), a, s, w, bb, act)
        errB = abs(gap(m16) - margin)
        K.LinearLowpFn.apply = lowp
        ej = m32.bert.encode_joint

        def rounded(*a, **k):
            j, lt = ej(*a, **k)
            return j.to(torch.bfloat16).float(), lt
        m32.bert.encode_joint = rounded
        errC = abs(gap(m32) - margin)
        m32.bert.encode_joint = ej
        row = {"story": b, "margin": round(margin, 4), "err_bf16": round(errA, 4),
               "err_bf16_head_f32": round(errB, 4), "err_f32_lang_rounded": round(errC, 4),
               "vit_acc": [round(x, 5) for x in acc[:nv]], "joint_acc": [round(x, 5) for x in acc[nv:]],
               "vit_local": [round(x, 5) for x in loc[:nv]], "joint_local": [round(x, 5) for x in loc[nv:]],
               "head": {k: round(v, 5) for k, v in heads.items()}}
        print(json.dumps(row), flush=True)
        summary.append(row)
    print(json.dumps({"summary": {k: [r[k] for r in summary] for k in
                                  ("margin", "err_bf16", "err_bf16_head_f32", "err_f32_lang_rounded")}}))


if __name__ == "__main__":
    main()
