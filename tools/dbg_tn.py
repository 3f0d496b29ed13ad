"""Debug the 256x256 TN kernel: A = [K][M] one-hot rows so C = rows of B, print error pattern."""
import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_sequencing_amd import _native as N
M = Nn = 256; K = 128
A = torch.zeros(K, M); 
for k in range(K): A[k, k] = 1.0     # C[m][n] = B[m][n] for m < K
B = torch.arange(K * Nn, dtype=torch.float32).view(K, Nn) % 251
A = A.cuda().bfloat16(); B = B.cuda().bfloat16()
C = torch.zeros(M, Nn, device="cuda")
N.gemm_set_fast(1)
N.gemm(A, B, C, M, Nn, K, trans=1, accumulate=False)
torch.cuda.synchronize()
ref = A.float().t() @ B.float()
bad = (C - ref).abs() > 0.5
print("bad", bad.sum().item(), "of", bad.numel())
Cc = C.cpu(); Bc = B.float().cpu()
for m in [0, 1, 2, 3, 4, 5, 8, 15, 16, 17, 31, 32, 64, 127]:
    row = Cc[m, :16].tolist()
    # which B row / col does C[m][n] equal?
    src = []
    for n in range(16):
        hits = (Bc == Cc[m, n]).nonzero()
        src.append(tuple(hits[0].tolist()) if len(hits) else None)
    print(m, [int(x) for x in row[:8]], src[:6])
br = bad.any(1).nonzero().flatten().tolist(); bc = bad.any(0).nonzero().flatten().tolist()
print("bad rows", br[:10], "...", len(br)); print("bad cols", bc[:10], "...", len(bc))
m = br[0]; print("row", m, "got", Cc[m, bc[:8]].tolist(), "want", ref.cpu()[m, bc[:8]].tolist())
