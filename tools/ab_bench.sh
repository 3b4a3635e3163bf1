#!/bin/bash
# Same-box A/B of library builds: bench.py with each library in turn, REPS rounds, one line each
# (frame ms pipelined, device-resident frame ms, k_primary/k_frame ms per launch).
# Usage: tools/ab_bench.sh "LIB_A LIB_B ..." [bench args...]   (REPS=2 by default)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
libs=$1; shift
for rep in $(seq 1 "${REPS:-2}"); do
  for v in $libs; do
    timeout -k 5 240 env SIGHTPY_HIP_LIB="$v" python3 bench.py --no-cpu-baseline "$@" > gpurun_out/ab_run.log 2>&1 || { tail -20 gpurun_out/ab_run.log; exit 1; }
    python3 - "$v" "$@" <<'EOF'
import json, sys
line = [x for x in open("gpurun_out/ab_run.log") if x.startswith("{")][-1]
d = json.loads(line)
print(sys.argv[1].split("/")[-1], " ".join(sys.argv[2:]), "frame_ms", d["ms_per_step"],
      "resident_ms", d.get("device_resident", {}).get("ms_per_step"),
      "kernel_ms", d.get("roofline", {}).get("kernel_ms"), "ranks", d.get("rank_frame_ms"), flush=True)
EOF
  done
done
