"""Per attention kernel: SQ instruction mix and MFMA busy from one rocprofv3 --pmc pass
(SQ_INSTS_VALU, SQ_INSTS_MFMA, SQ_INSTS_SALU, SQ_INSTS_LDS, SQ_WAVES, SQ_BUSY_CYCLES,
SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE) over tools/attn_bench.py (P = 640, T = 513 and 393).

usage: python tools/pmc_attn_sq.py <counter_collection.csv> <out.json>
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 4 SIMDs x 256 CUs), as
tools/pmc_mfma.py; VALU per MFMA = SQ_INSTS_VALU / SQ_INSTS_MFMA (wave instructions)."""
import collections
import csv
import json
import sys


def main():
    path, out = sys.argv[1], sys.argv[2]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "attn_" not in name:
            continue
        key = name.split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")
        if "<" in name:
            key = name[name.index("attn_"):name.index(">") + 1]
        per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {"source": "rocprofv3 --pmc (one pass) over tools/attn_bench.py 1", "kernels": {}}
    for k, c in sorted(per.items()):
        avg = {n: sum(v) / len(v) for n, v in c.items()}
        d = {"dispatches": len(next(iter(c.values()))), **{n: avg[n] for n in sorted(avg)}}
        if avg.get("SQ_INSTS_MFMA"):
            d["valu_per_mfma"] = avg.get("SQ_INSTS_VALU", 0) / avg["SQ_INSTS_MFMA"]
            d["salu_per_mfma"] = avg.get("SQ_INSTS_SALU", 0) / avg["SQ_INSTS_MFMA"]
        if avg.get("GRBM_GUI_ACTIVE"):
            d["mfma_busy"] = avg.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (avg["GRBM_GUI_ACTIVE"] / 8 * 4 * 256)
        res["kernels"][k] = d
    json.dump(res, open(out, "w"), indent=1)
    for k, d in res["kernels"].items():
        print(f"{k:45s} n={d['dispatches']:3d} valu/mfma={d.get('valu_per_mfma', 0):6.2f} "
              f"mfma_busy={d.get('mfma_busy', 0):.3f}")


if __name__ == "__main__":
    main()
