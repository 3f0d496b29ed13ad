"""Per-kernel register report of one HIP source (hipcc -Rpass-analysis=kernel-resource-usage):
VGPRs, AGPRs, VGPR spills, scratch bytes and occupancy, optionally filtered by a name substring.
usage: python tools/reg_report.py multimodal_sequencing_amd/csrc/gemm256.hip [substring] [extra hipcc flags]"""
import re
import subprocess
import sys


def main():
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    extra = sys.argv[3:]
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fno-slp-vectorize",
           "--cuda-device-only", "-c", src, "-o", "/tmp/reg_report.o",
           "-Rpass-analysis=kernel-resource-usage"] + extra
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    cur = None
    rows = []
    for line in out.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    for r in rows:
        if filt in r["name"]:
            print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('AGPRs', '?'):>3} agpr  spill {r.get('VGPRs Spill', '?'):>3}"
                  f"  scratch {r.get('ScratchSize [bytes/lane]', '?'):>3}  occ {r.get('Occupancy [waves/SIMD]', '?')}"
                  f"  {r['name'][:110]}")


if __name__ == "__main__":
    main()
