"""Which bf16 rounding sites make the decisive config-3 margins move? (measurement, GPU; test
infrastructure: uses the oracle through tests/bf16_emulation.py.)

For each story of the decisive_config3 fixture: the fp32 oracle's margin (second-best minus best
order NLL; the reference's own values are in the fixture), then, per rounding-site variant of
the emulated encoder and for the product's bf16 model, the relative L2 drift of lang_feats
against fp32 and the error of the margin.

usage: python tests/bf16_placement_probe.py [stories] [bf16w]   (one JSON line per story)
  bf16w: every weight rounded to a bf16-representable value first (then the fp32 oracle IS the
         reference on those weights, and bf16 weight operands are exact)
"""
import itertools
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE, os.path.join(HERE, "golden")]
import bf16_emulation as E  # noqa: E402
from counter_init import counter_state_dict  # noqa: E402
from make_golden_real import CONFIG3, real_inputs, scale_decisive  # noqa: E402
from oracle import berson_oracle as O  # noqa: E402

VARIANTS = {"all": E.ALL, "stream_f32": E.ALL - {"stream"}, "prob_f32": E.ALL - {"prob"},
            "output_f32": E.ALL - {"output"}, "stream_only": {"stream"}, "operand_only": {"operand"},
            "weight_only": {"weight"}, "weight_f32": E.ALL - {"weight"}}


def main():
    from multimodal_sequencing_amd import model_zoo
    from multimodal_sequencing_amd.process_inputs import prepare_berson_inputs
    stories = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    cfg = dict(CONFIG3, B=4)
    ocfg = {"N": 5, "heads": 12, "inter_heads": 8, "text_only": False, "vit_heads": 12}
    m16 = model_zoo.build_from_golden(cfg, device="cuda", dtype=torch.bfloat16)
    sd = scale_decisive(counter_state_dict({k: tuple(v.shape) for k, v in m16.state_dict().items()}),
                        "decisive_config3")
    if "bf16w" in sys.argv[2:]:
        sd = {k: (torch.from_numpy(v).to(torch.bfloat16).float().numpy() if v.dtype == np.float32 else v)
              for k, v in sd.items()}
    m16.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m16.eval()
    p = {k: torch.from_numpy(v).cuda() for k, v in sd.items()}
    ids, labels, images = real_inputs(310, cfg)
    perms = list(itertools.permutations(range(5)))

    def rel(a, b):
        return float((a.double() - b.double()).norm() / b.double().norm())

    with torch.no_grad(), torch.device("cuda"):
        for b in range(min(stories, ids.shape[0])):
            img = torch.from_numpy(images[b:b + 1]).cuda()
            pair = O.prepare_berson_inputs(ids[b:b + 1], labels[b:b + 1], 5)
            enc32 = E.encode(p, pair, img, ocfg, ())
            v32 = np.array([E.order_nll(p, enc32, ids[b:b + 1], o, 5) for o in perms])
            srt = np.argsort(v32)
            best, second = perms[srt[0]], perms[srt[1]]
            margin = float(v32[srt[1]] - v32[srt[0]])
            row = {"story": b, "margin": round(margin, 4)}
            for name, sites in VARIANTS.items():
                enc = E.encode(p, pair, img, ocfg, sites)
                gap = (E.order_nll(p, enc, ids[b:b + 1], second, 5)
                       - E.order_nll(p, enc, ids[b:b + 1], best, 5))
                row[name] = {"lang_drift": round(rel(enc["lang"], enc32["lang"]), 5),
                             "okey_drift": round(rel(enc["okey"], enc32["okey"]), 5),
                             "margin_err": round(abs(gap - margin), 4)}
            # the product's bf16 model (HIP kernels) on the same story
            inp = {"input_ids": torch.from_numpy(ids[b:b + 1]), "labels": torch.from_numpy(labels[b:b + 1]),
                   "images": img}
            bi = prepare_berson_inputs(inp["input_ids"], inp["labels"], 5, device="cuda")
            Lt = bi["input_ids"].shape[2]
            joint, _ = m16.bert.encode_joint(bi["input_ids"].view(20, Lt), bi["attention_mask"].view(20, Lt),
                                             bi["token_type_ids"].view(20, Lt), img, bi["pairs_list"])

            def nll(o):
                m16({**inp, "labels": torch.tensor([list(o)])})
                return float(m16.last_loss_terms[0]) * 4
            row["product_bf16"] = {"lang_drift": round(rel(joint[:, :Lt].float(), enc32["lang"]), 5),
                                   "margin_err": round(abs(nll(second) - nll(best) - margin), 4)}
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
