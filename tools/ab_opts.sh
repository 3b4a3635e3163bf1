#!/bin/bash
# Same-box A/B of library builds x option sets: bench.py once per (lib, options) per round, one line each
# (frame ms pipelined, device-resident ms, k_primary ms per launch, frame latency).
# Usage: tools/ab_opts.sh "LIB[:opt=v,opt=v] ..." [bench args...]   (REPS=2 by default)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
specs=$1; shift
for rep in $(seq 1 "${REPS:-2}"); do
  for sp in $specs; do
    lib=${sp%%:*}; opts=""
    [ "$sp" != "$lib" ] && for o in $(echo "${sp#*:}" | tr ',' ' '); do opts="$opts --option $o"; done
    timeout -k 5 240 env SIGHTPY_HIP_LIB="$lib" python3 bench.py --no-cpu-baseline $opts "$@" > gpurun_out/ab_run.log 2>&1 || { tail -20 gpurun_out/ab_run.log; exit 1; }
    python3 - "$sp" "$@" <<'PY'
import json, sys
line = [x for x in open("gpurun_out/ab_run.log") if x.startswith("{")][-1]
d = json.loads(line)
print(sys.argv[1].split("/")[-1], " ".join(sys.argv[2:]), "frame_ms", d["ms_per_step"],
      "resident_ms", d.get("device_resident", {}).get("ms_per_step"),
      "kernel_ms", d.get("roofline", {}).get("kernel_ms"), "latency_ms", d["config"].get("frame_latency_ms"),
      "host_rgb_ms", (d.get("host_rgb") or {}).get("ms_per_step"), "ranks", d.get("rank_frame_ms"), flush=True)
PY
  done
done
