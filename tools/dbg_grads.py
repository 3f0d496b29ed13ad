import sys, torch, numpy as np
sys.path.insert(0, 'tests'); sys.path.insert(0, 'tests/golden'); sys.path.insert(0, '.')
from golden_util import load_fixture
from multimodal_sequencing_amd import model_zoo
meta, d, params = load_fixture('tiny')
m = model_zoo.build_from_golden(meta['config'], device='cuda', dtype=torch.float32)
m.load_state_dict(params); m.zero_grad()
inputs = {"input_ids": torch.from_numpy(d["input_ids"]), "labels": torch.from_numpy(d["labels"]), "images": torch.from_numpy(d["images"]).cuda()}
loss = m(inputs)[0]; loss.backward(); torch.cuda.synchronize()
print('loss', loss.item(), float(d['loss']))
for k, p in m.named_parameters():
    r = d.get('g::' + k)
    ours = p.grad.norm().item()
    ref = float(np.linalg.norm(r)) if r is not None else float('nan')
    flag = '' if (r is not None and abs(ours - ref) <= 1e-3 * max(ref, 1e-4)) else '  <<<'
    print(f'{k:80s} {ours:.6g} {ref:.6g}{flag}')
