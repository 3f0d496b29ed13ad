"""MFMA utilisation per kernel group from one rocprofv3 --pmc pass
(SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES) over a bench.py step.

Units per /opt/skills/guides/MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES counts MFMA cycles
summed over the chip (32 per v_mfma_f32_32x32x16_bf16, 16 per 16x16x32); GRBM_GUI_ACTIVE is summed
over the 8 XCDs, so a dispatch lasts GRBM_GUI_ACTIVE / 8 cycles; one MFMA pipe per SIMD, 4 SIMDs per
CU: utilisation = MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 * 4 * CUs).

usage: python tools/pmc_mfma.py <counter_collection.csv> <out.json> [cus]
"""
import collections
import csv
import json
import sys

GROUPS = {
    "gemm256_nt": "gemm256_nt_kernel",
    "gemm256_tn": "gemm256_tn_kernel",
    "attn_fwd": "attn_fwd_bf16_kernel",
    "attn_fwd32": "attn_fwd32_kernel",
    "attn_dq": "attn_dq_bf16_kernel",
    "attn_dkdv": "attn_dkdv_bf16_kernel",
}


def is_f8(name):
    """gemm256_nt_kernel<ACT, BWD, XIN, Q8, F8>: MX-fp8 instantiations are not the bf16 roofline kernel."""
    i = name.find("gemm256_nt_kernel<")
    if i < 0:
        return False
    args = name[i + len("gemm256_nt_kernel<"):].split(">")[0].split(",")
    return len(args) >= 5 and args[4].strip() == "true"


def main():
    cus = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    for r in csv.DictReader(open(sys.argv[1])):
        for g, key in GROUPS.items():
            if key in r["Kernel_Name"] and not (g == "gemm256_nt" and is_f8(r["Kernel_Name"])):
                per[g][r.get("Dispatch_Id") or r.get("Correlation_Id")][r["Counter_Name"]] = \
                    float(r["Counter_Value"])
    out = {"cus": cus, "source": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE "
                                 "SQ_BUSY_CYCLES, bench.py (default config-3 workload, training step only: "
                                 "--fwd-steps 0) --steps 1 --warmup 1 via tools/profile_round.sh",
           "definition": "MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 * 4 SIMD * CUs), per dispatch, averaged"}
    for g, disp in per.items():
        utils = []
        for d in disp.values():
            if "SQ_VALU_MFMA_BUSY_CYCLES" in d and d.get("GRBM_GUI_ACTIVE"):
                utils.append(d["SQ_VALU_MFMA_BUSY_CYCLES"] /
                             (d["GRBM_GUI_ACTIVE"] / 8.0 * 4 * cus))
        if utils:
            out[g] = {"dispatches": len(utils), "mfma_util_mean": sum(utils) / len(utils),
                      "mfma_util_min": min(utils), "mfma_util_max": max(utils)}
    json.dump(out, open(sys.argv[2], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
