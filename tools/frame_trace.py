"""Per-frame kernel breakdown of a pipelined rocprofv3 kernel trace (bench.py run): for the last N
frames (delimited by the dominant trace kernel's launches), per-kernel calls / busy time per frame,
the GPU-busy union per frame, and one frame's launches with their queue, start, duration and grid.

    python tools/frame_trace.py gpurun_out/shardprof_8_r0 [frames]
"""
import csv
import glob
import sys
from collections import defaultdict


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def main():
    d = sys.argv[1]
    nf = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"], r["Grid_Size_X"])
          for r in rows]
    marks = [k[0] for k in ks if k[2].startswith("k_primary") or k[2].startswith("k_frame")]
    if len(marks) < nf + 2:
        nf = len(marks) - 2
    t0, t1 = marks[-nf - 1], marks[-1]
    win = [k for k in ks if t0 <= k[0] < t1]
    agg = defaultdict(lambda: [0, 0])
    for s, e, n, q, g in win:
        agg[n][0] += 1
        agg[n][1] += e - s
    # union of busy intervals
    iv = sorted((max(s, t0), min(e, t1)) for s, e, *_ in ks if e > t0 and s < t1)
    busy, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        busy += ce - cs
    per = (t1 - t0) / nf
    print("frames %d  ms/frame %.4f  GPU busy (any kernel) %.1f %%" % (nf, per / 1e6, 100.0 * busy / (t1 - t0)))
    for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print("  %-34s calls/frame %5.2f  us/frame %8.1f  us/call %8.1f" % (n[:34], c / nf, t / nf / 1e3, t / c / 1e3))
    a, b = marks[-3], marks[-2]
    print("one frame (offsets from its k_primary):")
    for s, e, n, q, g in ks:
        if a - 450000 <= s < b:
            print("  %9.1f %8.1f  q%-2s %-30s grid %s" % ((s - a) / 1e3, (e - s) / 1e3, q, n[:30], g))


if __name__ == "__main__":
    main()
