"""__graft_entry__.smoke(): one tiny fwd+bwd of the flagship path on cuda:0, checked against the
CPU oracle (test infrastructure; the oracle is only the checker)."""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "golden"))


def run_smoke():
    from golden_util import load_fixture, oracle_cfg
    from oracle import berson_oracle as O
    from multimodal_sequencing_amd import model_zoo

    assert torch.cuda.is_available(), "smoke needs a GPU"
    meta, d, params = load_fixture("tiny")
    m = model_zoo.build_from_golden(meta["config"], device="cuda:0", dtype=torch.float32)
    m.load_state_dict(params)
    m.eval()  # eval-mode loss is what the oracle restates (dropout off)
    m.zero_grad()
    inputs = {"input_ids": torch.from_numpy(d["input_ids"]), "labels": torch.from_numpy(d["labels"]),
              "images": torch.from_numpy(d["images"]).cuda()}
    loss = m(inputs)[0]
    loss.backward()
    torch.cuda.synchronize()
    ref, _, _ = O.forward_loss(params, d["input_ids"], d["labels"], torch.from_numpy(d["images"]),
                               oracle_cfg(meta))
    err = abs(loss.item() - ref.item())
    gsq = float(sum((p.grad.double() ** 2).sum() for p in m.parameters()))
    print(f"smoke: hip loss {loss.item():.7f} oracle {ref.item():.7f} |diff| {err:.2e} "
          f"grad-norm {gsq ** 0.5:.6f}")
    assert err < 1e-4, err
    assert gsq > 0 and gsq == gsq
