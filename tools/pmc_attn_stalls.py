"""Attention kernels' SQ stall and instruction-mix counters from two rocprofv3 --pmc passes over
tools/attn_bench.py (tools/gpu_run.sh steps pmc:a / pmc:b), averaged per (kernel, grid size):
fractions of wave cycles issuing / waiting on s_waitcnt / ready but not issued, VALU per MFMA and
MFMA busy.  usage: python tools/pmc_attn_stalls.py <pmc_a.csv> <pmc_b.csv> <out.json>"""
import collections
import csv
import json
import sys


def main():
    pa, pb, out = sys.argv[1:4]
    res = collections.defaultdict(dict)
    for path in (pa, pb):
        per = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(path)):
            n = r["Kernel_Name"]
            if "attn_" not in n:
                continue
            k = n[n.index("attn_"):n.index(">") + 1] + " grid=" + r["Grid_Size"]
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, c in per.items():
            res[k].update({n: sum(v) / len(v) for n, v in c.items()})
    for k, d in res.items():
        w = d.get("SQ_WAVE_CYCLES")
        if w:
            d["frac_active_any"] = d["SQ_ACTIVE_INST_ANY"] / w
            d["frac_wait_any"] = d["SQ_WAIT_ANY"] / w
            d["frac_wait_inst_any"] = d["SQ_WAIT_INST_ANY"] / w
        if d.get("SQ_INSTS_MFMA"):
            d["valu_per_mfma"] = d["SQ_INSTS_VALU"] / d["SQ_INSTS_MFMA"]
        if d.get("GRBM_GUI_ACTIVE"):
            d["mfma_busy"] = d["SQ_VALU_MFMA_BUSY_CYCLES"] / (d["GRBM_GUI_ACTIVE"] / 8 * 4 * 256)
    json.dump({"source": "rocprofv3 --pmc, passes a and b over tools/attn_bench.py 1 (P = 640, 12 "
                         "heads, T = 513 and 393, with and without dropout)", "kernels": res},
              open(out, "w"), indent=1)
    for k in sorted(res):
        d = res[k]
        print(f"{k:60s} active {d.get('frac_active_any', 0):.2f} wait {d.get('frac_wait_any', 0):.2f} "
              f"ready {d.get('frac_wait_inst_any', 0):.2f} mfma_busy {d.get('mfma_busy', 0):.3f}")


if __name__ == "__main__":
    main()
