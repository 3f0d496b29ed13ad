"""Probe which E8M0 scale the MX MFMA applies to each K position / row (mmseq_gemm_mxfp8):
A = B = identity pattern over K = 128 (row r has e4m3 1.0 at k = r), scales chosen per
(row, k-block) so that log2 of the diagonal output names the blocks / rows the hardware used."""
import math
import sys

import torch

sys.path.insert(0, ".")
from multimodal_sequencing_amd import _native as N  # noqa: E402


def packed_index(m, kb, KB):
    return ((m // 64) * KB + kb) * 64 + (m % 16) * 4 + (m % 64) // 16


def make(rows, K, scale_fn):
    q = torch.zeros(rows, K, dtype=torch.uint8)
    for r in range(rows):
        q[r, r % K] = 0x38  # e4m3 1.0
    KB = K // 32
    sc = torch.zeros(N.lib().mmseq_mxfp8_scale_bytes(rows, K), dtype=torch.uint8)
    for m in range(rows):
        for kb in range(KB):
            sc[packed_index(m, kb, KB)] = scale_fn(m, kb)
    return N.MXFP8(q.cuda(), sc.cuda(), rows, K)


def main():
    K, R = 128, 128
    for name, fa, fb in [("kblock", lambda m, kb: 127 + kb, lambda m, kb: 127 + 4 * kb),
                         ("row%16", lambda m, kb: 127 + (m % 16) // 4 + 4 * ((m % 64) // 16),
                          lambda m, kb: 127)]:
        a, b = make(R, K, fa), make(R, K, fb)
        C = torch.zeros(R, R, dtype=torch.bfloat16, device="cuda")
        N.gemm_mxfp8(a, b, C)
        d = C.float().diag().cpu()
        off = (C.float() - torch.diag(C.float().diag())).abs().max().item()
        print(name, "offdiag max", off)
        print(" ".join(f"{int(round(math.log2(v))) if v > 0 else 'x'}" for v in d.tolist()))


if __name__ == "__main__":
    main()
