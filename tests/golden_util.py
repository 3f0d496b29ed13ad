"""Shared helpers: load golden fixtures and rebuild their counter-based weights."""
import json
import os

import numpy as np
import torch

from counter_init import counter_state_dict

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = ["tiny", "tiny_ragged", "tiny_textonly", "tiny_n4"]


def load_fixture(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        meta = json.load(f)
    data = dict(np.load(os.path.join(GOLDEN, name + ".npz")))
    params = {k: torch.from_numpy(v) for k, v in
              counter_state_dict({k: tuple(s) for k, s in meta["shapes"].items()}).items()}
    return meta, data, params


def oracle_cfg(meta):
    c = meta["config"]
    return {"N": c["N"], "heads": c["joint"]["heads"], "inter_heads": c["head"]["heads"],
            "text_only": c["text_only"], "vit_heads": c["vit"]["width"] // 64}
