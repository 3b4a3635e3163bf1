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
  GRBM_GUI_ACTIVE is summed over the 8 XCDs: the dispatch's active cycles are GRBM_GUI_ACTIVE / 8.
  SQ_ACTIVE_INST_* and SQ_WAVE_CYCLES / SQ_WAIT_* count quad-cycles (x 4 = cycles).
  valu_issue_frac = (4 x f64 VALU instructions + 2 x other VALU instructions)
                    / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
                  issue cycles of the VALU instructions (wave64 on a SIMD: 2 cycles, f64 at half rate:
                  4) over the SIMD cycles of the dispatch -- the bench's formula (bench.py roofline)
  valu_active_frac = 4 x SQ_ACTIVE_INST_VALU / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
                  cycles waves spent issuing VALU (summed over waves) over the SIMD cycles
  wave_wait_frac  = SQ_WAIT_ANY / SQ_WAVE_CYCLES
  valu_lane_util  = SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU)
                  the active lanes of the VALU instructions (rocprofv3's VALUUtilization): the
                  fraction of the fp64_flop upper bound that lanes really executed

    python tools/pmc_summary.py gpurun_out/pmc_a gpurun_out/pmc_b ... --out profiles/r03_counters_X.json
    python tools/pmc_summary.py --recompute profiles/r02_counters_X.json ...   (derived fields again
                                                                                 from stored counters)
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

CUS = 256
SIMDS = 4 * CUS
XCDS = 8


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


DERIVED = {"traffic_bytes": "2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024",
           "fp64_flop": "64 x (SQ_INSTS_VALU_ADD_F64 + MUL_F64 + TRANS_F64 + 2 x FMA_F64)",
           "valu_issue_frac": "(4 x f64 VALU insts + 2 x other VALU insts) / (GRBM_GUI_ACTIVE / %d XCDs x %d SIMDs)"
                              % (XCDS, SIMDS),
           "valu_active_frac": "4 x SQ_ACTIVE_INST_VALU (quad-cycles) / (GRBM_GUI_ACTIVE / %d XCDs x %d SIMDs)"
                               % (XCDS, SIMDS),
           "wave_wait_frac": "SQ_WAIT_ANY / SQ_WAVE_CYCLES",
           "valu_lane_util": "SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU) (rocprofv3 VALUUtilization)"}


def derive(c):
    """Derived per-launch figures from the counter means `c`."""
    rec = {}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        rec["fetch_bytes"] = 2 * c["FETCH_SIZE"] * 1024
        rec["write_bytes"] = c["WRITE_SIZE"] * 1024
        rec["traffic_bytes"] = rec["fetch_bytes"] + rec["write_bytes"]
    f64 = [c.get("SQ_INSTS_VALU_%s_F64" % op) for op in ("ADD", "MUL", "TRANS", "FMA")]
    if all(v is not None for v in f64):
        rec["fp64_flop"] = 64 * (f64[0] + f64[1] + f64[2] + 2 * f64[3])
    cyc = c.get("GRBM_GUI_ACTIVE", 0) / XCDS * SIMDS
    if cyc and "SQ_INSTS_VALU" in c and all(v is not None for v in f64[:2]) and f64[3] is not None:
        n64 = f64[0] + f64[1] + f64[3]
        rec["valu_issue_frac"] = (4 * n64 + 2 * (c["SQ_INSTS_VALU"] - n64)) / cyc
    if cyc and "SQ_ACTIVE_INST_VALU" in c:
        rec["valu_active_frac"] = 4 * c["SQ_ACTIVE_INST_VALU"] / cyc
    if c.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in c:
        rec["wave_wait_frac"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
    if c.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in c:
        rec["valu_lane_util"] = c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"])
    return rec


def recompute(paths):
    for p in paths:
        out = json.load(open(p))
        out["derived"] = DERIVED
        for k, rec in out["kernels"].items():
            for key in ("valu_issue_frac", "valu_active_frac", "wave_wait_frac", "valu_lane_util"):
                rec.pop(key, None)
            rec.update(derive(rec["counters"]))
        with open(p, "w") as fh:
            json.dump(out, fh, indent=1)
        print(p, {k: (round(r.get("valu_issue_frac", -1), 4), round(r.get("valu_active_frac", -1), 4))
                  for k, r in out["kernels"].items() if "k_primary" in k or "k_frame" in k or "k_trace" in k})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="*")
    ap.add_argument("--out")
    ap.add_argument("--label", default="")
    ap.add_argument("--recompute", nargs="+", help="summary files whose derived fields are recomputed")
    a = ap.parse_args()
    if a.recompute:
        return recompute(a.recompute)
    merged = defaultdict(dict)
    launches = defaultdict(dict)
    for d in a.dirs:
        for k, cs in load(d).items():
            for c, vals in cs.items():
                merged[k][c] = sum(vals) / len(vals)
                launches[k][c] = len(vals)
    out = {"label": a.label, "units": "per launch (mean over the launches of each pass)", "passes": a.dirs,
           "derived": DERIVED, "kernels": {}}
    for k in sorted(merged):
        c = merged[k]
        rec = {"counters": c, "launches": launches[k]}
        rec.update(derive(c))
        out["kernels"][k] = rec
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    for k, r in out["kernels"].items():
        print("%-40s traffic %s fp64_flop %s valu %s" % (k, r.get("traffic_bytes"), r.get("fp64_flop"),
                                                         r.get("valu_issue_frac")))


if __name__ == "__main__":
    main()
