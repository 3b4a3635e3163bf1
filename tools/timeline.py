"""Print the last frame's launches from a rocprofv3 kernel-trace CSV: start offset, duration, grid."""
import csv
import glob
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
f = glob.glob(path + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))[-n:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    print("%-40s start %8.1f us  dur %7.1f us  grid %s" % (name[:40], (s - t0) / 1e3, (e - s) / 1e3, r["Grid_Size_X"]))
