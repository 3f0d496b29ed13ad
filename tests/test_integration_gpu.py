"""The reference-side binding documented in INTEGRATION.md ("Reference-side binding a maintainer
would add") stays callable: the code block is executed verbatim (only the library path
substituted) and compared with torch.nn.functional.layer_norm; on CPU its call is checked
against the declaration in include/mmseq.h (argument count)."""
import ast
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _snippet():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"```python\n(# models/_mmseq\.py.*?)```", text, re.S)
    assert m, "binding snippet not found in INTEGRATION.md"
    return m.group(1)


def _decl_nargs(name):
    hdr = open(os.path.join(ROOT, "include", "mmseq.h")).read()
    m = re.search(name + r"\((.*?)\);", hdr, re.S)
    return len([a for a in m.group(1).split(",") if a.strip()])


def test_snippet_call_matches_header():
    tree = ast.parse(_snippet())
    calls = [n for n in ast.walk(tree) if isinstance(n, ast.Call) and
             isinstance(n.func, ast.Attribute) and n.func.attr == "mmseq_layernorm_fwd"]
    assert len(calls) == 1
    assert len(calls[0].args) == _decl_nargs("mmseq_layernorm_fwd") == 15


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_snippet_runs_and_matches_layer_norm(dtype):
    from multimodal_sequencing_amd import _native
    ns = {}
    exec(_snippet().replace("/path/to/libmmseq.so", _native.LIB_PATH), ns)
    g = torch.Generator(device="cpu").manual_seed(3)
    R, C = 1000, 768
    x = (torch.randn(R, C, generator=g) * 2 + 0.5).to("cuda", dtype)
    w = torch.randn(C, generator=g).cuda()
    b = torch.randn(C, generator=g).cuda()
    y = ns["layer_norm"](x, w, b, 1e-12)
    torch.cuda.synchronize()
    ref = torch.nn.functional.layer_norm(x.float(), (C,), w, b, 1e-12)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)
