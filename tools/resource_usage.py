"""Per-kernel register / scratch / occupancy table from the compiler's resource-usage remarks.

    python tools/resource_usage.py [--filter k_primary] [--source csrc/rt_kernels.hip] [--define X ...]

Runs `hipcc -Rpass-analysis=kernel-resource-usage` (the Makefile's `resource-usage` flags) on the
kernel source and prints one line per kernel: VGPRs, VGPR spill, scratch bytes/lane, waves/SIMD.
"""
import argparse
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "python-raytracer_amd" / "csrc"


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                         text=True).stdout.splitlines()
    return out if len(out) == len(names) else names


def usage(source, defines=()):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
           "-munsafe-fp-atomics", "--cuda-device-only", "-c", "-Rpass-analysis=kernel-resource-usage",
           "-o", "/dev/null", str(source)] + ["-D" + d for d in defines]
    err = subprocess.run(cmd, capture_output=True, text=True, cwd=str(CSRC)).stderr
    rows, cur = [], None
    for line in err.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z /\[\]]+?): (\S+) \[", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    names = demangle([r["name"] for r in rows])
    for r, n in zip(rows, names):
        r["pretty"] = n.replace("(anonymous namespace)::", "")
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--filter", default="k_primary|k_trace|k_frame")
    ap.add_argument("--source", default=str(CSRC / "rt_kernels.hip"))
    ap.add_argument("--define", action="append", default=[])
    a = ap.parse_args()
    rows = usage(a.source, a.define)
    pat = re.compile(a.filter)
    print("%-60s %6s %6s %8s %5s" % ("kernel", "VGPRs", "spill", "scratch", "occ"))
    for r in rows:
        if pat.search(r["pretty"]):
            print("%-60s %6s %6s %8s %5s" % (r["pretty"][:60], r.get("VGPRs"), r.get("VGPRs Spill"),
                                           r.get("ScratchSize [bytes/lane]"), r.get("Occupancy [waves/SIMD]")))
    return 0


if __name__ == "__main__":
    sys.exit(main())
