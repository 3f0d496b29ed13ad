"""Fused LSTM cell (mmseq_lstm_cell_fwd/bwd via kernels.LstmCellFn) against torch's nn.LSTM cell
equations in fp32 (plain PyTorch reference of the same op): outputs and all input gradients,
for a strided gate input (a step slice of the one x-GEMM over all decoder steps)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(gx, gh, c):
    i, f, g, o = (gx + gh).chunk(4, -1)
    c2 = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
    return torch.sigmoid(o) * torch.tanh(c2), c2


@pytest.mark.parametrize("B,H,use_dc", [(1, 768, True), (16, 768, True), (5, 1024, False),
                                        (3, 130, True)])
def test_lstm_cell_matches_torch(B, H, use_dc):
    from multimodal_sequencing_amd.kernels import LstmCellFn
    g = torch.Generator(device="cuda").manual_seed(B * H)
    gx_all = torch.randn(B, 3, 4 * H, device="cuda", generator=g) * 2
    gh = torch.randn(B, 4 * H, device="cuda", generator=g) * 2
    c = torch.randn(B, H, device="cuda", generator=g)
    leaves = [t.clone().requires_grad_(True) for t in (gx_all, gh, c)]
    refs = [t.clone().requires_grad_(True) for t in (gx_all, gh, c)]
    h1, c1 = LstmCellFn.apply(leaves[0][:, 1], leaves[1], leaves[2])
    h2, c2 = _ref(refs[0][:, 1], refs[1], refs[2])
    torch.testing.assert_close(h1, h2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(c1, c2, rtol=1e-5, atol=1e-6)
    dh = torch.randn(B, H, device="cuda", generator=g)
    dc = torch.randn(B, H, device="cuda", generator=g)
    l1 = (h1 * dh).sum() + ((c1 * dc).sum() if use_dc else 0)
    l2 = (h2 * dh).sum() + ((c2 * dc).sum() if use_dc else 0)
    l1.backward()
    l2.backward()
    for a, b in zip(leaves, refs):
        torch.testing.assert_close(a.grad, b.grad, rtol=1e-5, atol=1e-5)
    assert float(leaves[0].grad[:, 0].abs().max()) == 0.0  # untouched steps get no gradient
