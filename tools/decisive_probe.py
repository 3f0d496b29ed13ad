"""Pick the decisive-ordering fixture's weight scaling (tests/golden/make_golden_real.py
DECISIVE_SCALE): for candidate scalings of the pointer head, the fp32 model's NLL of every order
(margin = second best - best) and the bf16 model's error on that margin. Measurement only."""
import itertools
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
from counter_init import counter_state_dict  # noqa: E402
from make_golden_real import CONFIG3, DECISIVE_TINY, real_inputs  # noqa: E402
from multimodal_sequencing_amd import model_zoo  # noqa: E402

CANDIDATES = {
    "tl50_q50_kl50_pw50": {"tanh_linear.weight": 50, "query_linear.weight": 50, "key_linear.weight": 50,
                           "pw_k.weight": 50},
    "tl100_q50_kl50": {"tanh_linear.weight": 100, "query_linear.weight": 50, "key_linear.weight": 50},
    "tl50_q100_kl100": {"tanh_linear.weight": 50, "query_linear.weight": 100, "key_linear.weight": 100},
    "tl50_pw50_kl50": {"tanh_linear.weight": 50, "pw_k.weight": 50, "key_linear.weight": 50},
    "tl50": {"tanh_linear.weight": 50},
    "tl200": {"tanh_linear.weight": 200},
    "tl50_q50": {"tanh_linear.weight": 50, "query_linear.weight": 50},
    "tl100_pw10": {"tanh_linear.weight": 100, "pw_k.weight": 10},
    "tl50_q50_kl50": {"tanh_linear.weight": 50, "query_linear.weight": 50, "key_linear.weight": 50},
    "tl20_q200": {"tanh_linear.weight": 20, "query_linear.weight": 200},
}


BF16W = os.environ.get("DECISIVE_BF16W") == "1"  # every weight rounded to bf16 (the _bf16w fixtures)
SEED = int(os.environ.get("DECISIVE_SEED", "310"))


def model(cfg, dtype, scale):
    m = model_zoo.build_from_golden(cfg, device="cuda", dtype=dtype)
    sd = counter_state_dict({k: tuple(v.shape) for k, v in m.state_dict().items()})
    for k, f in scale.items():
        sd[k] = sd[k] * f
    if BF16W:
        sd = {k: (torch.from_numpy(v).bfloat16().float().numpy() if v.dtype == np.float32 else v)
              for k, v in sd.items()}
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m.eval()
    return m


def nll(m, inp, order):
    with torch.no_grad():
        m({**inp, "labels": torch.tensor([list(order)])})
    return float(m.last_loss_terms[0]) * (len(order) - 1)


def main():
    # usage: decisive_probe.py [config3_stories [candidate ...]] (default: both fixtures, B as made)
    B3 = int(sys.argv[1]) if len(sys.argv) > 1 else CONFIG3["B"]
    names = sys.argv[2:] or list(CANDIDATES)
    runs = (("config3", dict(CONFIG3, B=B3), SEED),) if len(sys.argv) > 1 else \
        (("tiny", DECISIVE_TINY, 311), ("config3", CONFIG3, 310))
    for cname, cfg, seed in runs:
        ids, labels, images = real_inputs(seed, cfg)
        perms = list(itertools.permutations(range(cfg["N"])))
        for sname in names:
            scale = CANDIDATES[sname]
            m32, m16 = model(cfg, torch.float32, scale), model(cfg, torch.bfloat16, scale)
            rows = []
            for b in range(ids.shape[0]):
                inp = {"input_ids": torch.from_numpy(ids[b:b + 1]),
                       "labels": torch.from_numpy(labels[b:b + 1]),
                       "images": torch.from_numpy(images[b:b + 1]).cuda()}
                v = np.array([nll(m32, inp, p) for p in perms])
                o = np.argsort(v)
                gap32 = v[o[1]] - v[o[0]]
                gap16 = nll(m16, inp, perms[o[1]]) - nll(m16, inp, perms[o[0]])
                rows.append((round(float(gap32), 4), round(abs(gap16 - gap32), 4)))
            dec = sum(1 for g, e in rows if g > 5 * e)
            print(json.dumps({"cfg": cname, "scale": sname, "bf16w": BF16W, "decisive": dec,
                              "stories": len(rows), "margin_and_bf16_error": rows}), flush=True)
            del m32, m16


if __name__ == "__main__":
    main()
