"""Summarise rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE, collected in separate runs of the
same bench command, see tools/gpu_session.sh pmc_fetch / pmc_write) into per-launch HBM traffic of
each kernel, with the gfx950 corrections of MI355X_MICROARCH.md § HBM:

  FETCH_SIZE counts TCC_EA0_RDREQ x 64 B, i.e. 1/2 of the bytes of wide coalesced reads -> x2;
  WRITE_SIZE is exact for streaming stores and float atomics.  Both are reported in KiB.

Our loads are 8 B per lane (SoA f64) rather than the calibrated 16 B, so the x2 is an upper
estimate for fetches; the raw counter values are kept next to the corrected bytes.

    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --out profiles/r01_traffic.json
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(dirpath, counter):
    files = glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--out", required=True)
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    fetch = load(a.fetch_dir, "FETCH_SIZE")
    write = load(a.write_dir, "WRITE_SIZE")
    out = {"label": a.label, "units": "bytes per launch (mean over launches)",
           "correction": "fetch_bytes = 2 x FETCH_SIZE KiB x 1024 (gfx950), write_bytes = WRITE_SIZE KiB x 1024",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fk = sum(f) / len(f) if f else None
        wk = sum(w) / len(w) if w else None
        rec = {"launches_fetch": len(f), "launches_write": len(w), "FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk}
        if fk is not None and wk is not None:
            rec["fetch_bytes"] = 2 * fk * 1024
            rec["write_bytes"] = wk * 1024
            rec["traffic_bytes"] = rec["fetch_bytes"] + rec["write_bytes"]
        out["kernels"][short(k)] = rec
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    for k, r in out["kernels"].items():
        print("%-40s %s" % (k, r.get("traffic_bytes")))


if __name__ == "__main__":
    main()
