"""Instruction mix per basic block of one kernel in a hipcc `-S` device assembly file.

usage: python tools/asm_mix.py FILE.s KERNEL_SUBSTRING [min_instructions]
  hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S attention.hip -o /tmp/attn.s

Counts per block: MFMA, transcendental VALU (v_exp/v_log/v_rcp/...), other VALU, LDS (ds_*),
vector memory (buffer_/global_), scalar, waitcnt/barrier, and the VALU issue estimate in cycles
from MI355X_MICROARCH.md's issue-cost row (transcendental 8, other VALU 4, MFMA holds 8 of 16/32).
Blocks that end in a branch back to an earlier label are marked LOOP.
"""
import re
import sys

TRANS = re.compile(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)_")


def kernel_lines(path, name):
    out, on = [], False
    for l in open(path):
        if not on and re.match(r"^\S*" + re.escape(name) + r"\S*:", l):
            on = True
            continue
        if on and l.startswith(".Lfunc_end"):
            break
        if on:
            out.append(l.rstrip("\n"))
    return out


def blocks(lines):
    cur, name = [], "entry"
    for l in lines:
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            yield name, cur
            cur, name = [], m.group(1)
            continue
        s = l.split(";")[0].strip()
        if s and not s.startswith("."):
            cur.append(s)
    yield name, cur


def mix(ins):
    c = dict(mfma=0, trans=0, valu=0, lds=0, vmem=0, salu=0, wait=0)
    for s in ins:
        op = s.split()[0]
        if "mfma" in op:
            c["mfma"] += 1
        elif TRANS.match(op):
            c["trans"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith(("buffer_", "global_", "flat_")):
            c["vmem"] += 1
        elif op.startswith(("s_waitcnt", "s_barrier")):
            c["wait"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
    c["valu_cyc"] = 8 * c["trans"] + 4 * c["valu"]
    return c


def main():
    path, name = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    lines = kernel_lines(path, name)
    seen = []
    for bname, ins in blocks(lines):
        seen.append(bname)
        if len(ins) < mn:
            continue
        loop = ""
        for s in ins[-2:]:
            m = re.match(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", s)
            if m and (m.group(1) or m.group(2)) in seen:
                loop = " LOOP->" + (m.group(1) or m.group(2))
        print(f"{bname:16s} n={len(ins):4d} {mix(ins)}{loop}")


if __name__ == "__main__":
    main()
