"""Per-launch HBM traffic of kernel groups from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Corrections per /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section): both derived
counters are in KB; on gfx950 FETCH_SIZE reports exactly half of the bytes of wide (16 B/lane)
coalesced streaming reads (global_load and buffer_load ... lds alike), so it is doubled; WRITE_SIZE
is exact for 16 B/lane stores. Infinity-Cache hits are counted, so traffic is an upper bound on
true HBM bytes.

usage: python tools/pmc_traffic.py <fetch.csv> <write.csv> <out.json>
"""
import collections
import csv
import json
import sys

GROUPS = {
    "gemm256_nt": "gemm256_nt_kernel",   # the roofline kernel (fwd + dgrad NT GEMMs)
    "gemm256_tn": "gemm256_tn_kernel",
    "attn_fwd": "attn_fwd_bf16_kernel",
    "attn_dq": "attn_dq_bf16_kernel",
    "attn_dkdv": "attn_dkdv_bf16_kernel",
    "ln_fwd": "ln_fwd16_kernel",
    "ln_bwd": "ln_bwd16_kernel",
}


def is_f8(name):
    """gemm256_nt_kernel<ACT, BWD, XIN, Q8, F8>: the MX-fp8 operand instantiations (config 5) are
    not the bf16 roofline kernel."""
    i = name.find("gemm256_nt_kernel<")
    if i < 0:
        return False
    args = name[i + len("gemm256_nt_kernel<"):].split(">")[0].split(",")
    return len(args) >= 5 and args[4].strip() == "true"


def load(path, counter):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        for g, key in GROUPS.items():
            if key in r["Kernel_Name"] and not (g == "gemm256_nt" and is_f8(r["Kernel_Name"])):
                per[g].append(float(r["Counter_Value"]) * 1024.0)
    return per


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {"units": "bytes per launch", "fetch_correction": 2.0,
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), "
                     "bench.py (default config-3 workload, training step only: --fwd-steps 0) --steps 1 --warmup 0 "
                     "via tools/profile_round.sh"}
    for g in GROUPS:
        if not fetch.get(g) or not write.get(g):
            continue
        f = 2.0 * sum(fetch[g]) / len(fetch[g])
        w = sum(write[g]) / len(write[g])
        out[g] = {"launches": len(fetch[g]), "read_bytes": f, "write_bytes": w, "traffic_bytes": f + w}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
