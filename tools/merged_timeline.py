"""Print the last launches and memory copies of a rocprofv3 --kernel-trace --memory-copy-trace run
in time order (start, end, duration, stream), to see how frames overlap."""
import csv
import glob
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
ev = []
for r in csv.DictReader(open(glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0])):
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:28]
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Stream_Id", "")))
for f in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"][12:], r.get("Stream_Id", "")))
ev.sort()
ev = ev[-n:]
t0 = ev[0][0]
for s, e, name, st in ev:
    print("%-30s st%-3s %9.1f -> %9.1f  (%7.1f)" % (name, st, (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3))
