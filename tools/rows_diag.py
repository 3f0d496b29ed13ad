"""Per-parameter gradient differences: full vs full (run-to-run) and full vs text-rows last layer."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
import torch
from counter_init import counter_state_dict
from golden_util import GOLDEN
from make_golden_real import real_inputs
from multimodal_sequencing_amd import model_zoo, kernels as K, _native as N

meta = json.load(open(os.path.join(GOLDEN, "real_config5_l2.json")))
m = model_zoo.build_from_golden(meta["config"], device="cuda", dtype=torch.bfloat16)
sd = counter_state_dict({k: tuple(v.shape) for k, v in m.state_dict().items()})
m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
ids, labels, images = real_inputs(meta["input_seed"], meta["config"])
inputs = {"input_ids": torch.from_numpy(ids), "labels": torch.from_numpy(labels),
          "images": torch.from_numpy(images).to("cuda")}
m.train()
m.bert.config.hidden_dropout_prob = 0.0
N.gemm_set_fast(4)


def run(on):
    K.ROWS["on"] = on
    m.zero_grad()
    m.bert._n_fwd = 0
    loss = m(inputs)[0]
    loss.backward()
    torch.cuda.synchronize()
    return float(loss), {k: p.grad.detach().double().clone() for k, p in m.named_parameters()}


(l0, g0), (l0b, g0b), (l1, g1) = run(False), run(False), run(True)
print("losses", l0, l0b, l1)
rows = []
for k in g0:
    n = float(g0[k].norm())
    if n == 0:
        continue
    rows.append((float((g0b[k] - g0[k]).norm()) / n, float((g1[k] - g0[k]).norm()) / n, k))
rows.sort(key=lambda r: -r[1])
for r in rows[:25]:
    print(f"{r[0]:.3e} {r[1]:.3e} {r[2]}")
print("run-to-run nonzero:", sum(1 for r in rows if r[0] > 0), "of", len(rows))
