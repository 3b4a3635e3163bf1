"""Summarise rocprofv3 PMC passes of one bench command into per-launch counter means per kernel, plus
the derived figures the bench roofline reads (profiles/rNN_counters_<config>.json).

Each pass is a separate `rocprofv3 --pmc <counters> --kernel-trace` run of the same command
(rocprofv3 does not split counters over passes; tools/gpu_session.sh pmc_* steps).  Derived, per
launch (MI355X_MICROARCH.md § HBM and § Execution model):

  traffic_bytes = 2 x FETCH_SIZE + WRITE_SIZE    (KiB x 1024; FETCH_SIZE counts half the bytes of
                                                  wide reads on gfx950)
  fp64_flop     = 64 x (ADD_F64 + MUL_F64 + TRANS_F64 + 2 x FMA_F64)
                  (wave-instruction counts x 64 lanes: an upper bound, lanes masked off by divergence
                  are counted)
  valu_issue_frac = SQ_ACTIVE_INST_VALU / (SQ_BUSY_CU_CYCLES or GRBM_GUI_ACTIVE x CUs x 4 SIMDs)
                  when the counters are present (how busy the VALU issue ports are)

    python tools/pmc_summary.py gpurun_out/pmc_a gpurun_out/pmc_b ... --out profiles/r02_counters_X.json
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

CUS = 256


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0]


def load(dirpath):
    """{kernel: {counter: [value per launch]}}"""
    per = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True):
        rows = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            rows[(r["Dispatch_Id"], r["Kernel_Name"])][r["Counter_Name"]] = float(r["Counter_Value"])
        for (_, k), cs in rows.items():
            for c, v in cs.items():
                per[short(k)][c].append(v)
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--out", required=True)
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    merged = defaultdict(dict)
    launches = defaultdict(dict)
    for d in a.dirs:
        for k, cs in load(d).items():
            for c, vals in cs.items():
                merged[k][c] = sum(vals) / len(vals)
                launches[k][c] = len(vals)
    out = {"label": a.label, "units": "per launch (mean over the launches of each pass)", "passes": a.dirs,
           "derived": {"traffic_bytes": "2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024",
                       "fp64_flop": "64 x (SQ_INSTS_VALU_ADD_F64 + MUL_F64 + TRANS_F64 + 2 x FMA_F64)",
                       "valu_issue_frac": "SQ_ACTIVE_INST_VALU / (GRBM_GUI_ACTIVE x %d CUs x 4 SIMDs)" % CUS},
           "kernels": {}}
    for k in sorted(merged):
        c = merged[k]
        rec = {"counters": c, "launches": launches[k]}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            rec["fetch_bytes"] = 2 * c["FETCH_SIZE"] * 1024
            rec["write_bytes"] = c["WRITE_SIZE"] * 1024
            rec["traffic_bytes"] = rec["fetch_bytes"] + rec["write_bytes"]
        f64 = [c.get("SQ_INSTS_VALU_%s_F64" % op) for op in ("ADD", "MUL", "TRANS", "FMA")]
        if all(v is not None for v in f64):
            rec["fp64_flop"] = 64 * (f64[0] + f64[1] + f64[2] + 2 * f64[3])
        if "SQ_ACTIVE_INST_VALU" in c and c.get("GRBM_GUI_ACTIVE"):
            rec["valu_issue_frac"] = c["SQ_ACTIVE_INST_VALU"] / (c["GRBM_GUI_ACTIVE"] * CUS * 4)
        out["kernels"][k] = rec
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    for k, r in out["kernels"].items():
        print("%-40s traffic %s fp64_flop %s valu %s" % (k, r.get("traffic_bytes"), r.get("fp64_flop"),
                                                         r.get("valu_issue_frac")))


if __name__ == "__main__":
    main()
