"""Busy fractions of a rocprofv3 kernel/memory-copy trace over the last N frames' window: the union of
kernel intervals, the union of copy intervals and their overlap (how well a pipelined frame hides its
copies and its jitter generation)."""
import csv
import glob
import sys


def intervals(d, kind):
    out = []
    pat = "/**/*kernel_trace.csv" if kind == "k" else "/**/*memory_copy_trace.csv"
    for f in glob.glob(d + pat, recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", r.get("Direction", ""))
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    return sorted(out)


def union(iv, lo, hi):
    tot, cur_s, cur_e = 0, None, None
    for s, e, _ in iv:
        s, e = max(s, lo), min(e, hi)
        if e <= s:
            continue
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


d = sys.argv[1]
k, m = intervals(d, "k"), intervals(d, "m")
mt = [x for x in k if "k_mt" in x[2]]
starts = [x[0] for x in k if "k_primary" in x[2] or "k_frame" in x[2]]
lo, hi = starts[-8], max(e for _, e, _ in k + m)  # the last frames
span = hi - lo
print("window %.1f us: kernels busy %.1f%%, copies busy %.1f%%, MT busy %.1f%%" % (
    span / 1e3, 100 * union(k, lo, hi) / span, 100 * union(m, lo, hi) / span, 100 * union(mt, lo, hi) / span))
tot = {}
for s, e, n in k:
    if s >= lo:
        key = n.replace("(anonymous namespace)::", "").split("(")[0][:34]
        tot[key] = tot.get(key, 0) + (e - s)
for key, v in sorted(tot.items(), key=lambda x: -x[1]):
    print("  %-36s %9.1f us (sum of durations)" % (key, v / 1e3))
