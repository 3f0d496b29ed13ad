"""One shape of the MX-fp8 NT GEMM and of the bf16 NT GEMM, for PMC passes (tools/fp8_pmc.sh):
    python tools/fp8_one.py [N K [rows]]   (default: the config-5 FC2, 1024 x 4096)"""
import sys

import torch

sys.path.insert(0, ".")
from multimodal_sequencing_amd import _native as N  # noqa: E402

Nn = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
K = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
M = int(sys.argv[3]) if len(sys.argv) > 3 else 72 * 769
A = torch.randn(M, K, device="cuda").bfloat16()
W = (torch.randn(Nn, K, device="cuda") * 0.02).bfloat16()
C = torch.empty(M, Nn, device="cuda", dtype=torch.bfloat16)
qa, qw = N.quant_mxfp8(A), N.quant_mxfp8(W)
for _ in range(3):
    N.gemm_mxfp8(qa, qw, C)
    N.gemm(A, W, C, M, Nn, K)
torch.cuda.synchronize()
print("done", M, Nn, K)
