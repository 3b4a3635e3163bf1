#!/bin/bash
# Build a variant of libsightpy_hip.so with extra defines into tools/_build/libsightpy_hip_<name>.so
# and print the resource usage of the k_primary kernels.  Usage: tools/build_variant.sh NAME [-DFOO ...]
set -eu
name=$1; shift
cd "$(dirname "$0")/../python-raytracer_amd/csrc"
mkdir -p ../../tools/_build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -munsafe-fp-atomics \
  -Wall -Wno-unused-function "$@" -Rpass-analysis=kernel-resource-usage \
  -o ../../tools/_build/libsightpy_hip_$name.so rt_kernels.hip -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib 2>&1 |
  python3 -c '
import re, sys
cur = None
for l in sys.stdin:
    m = re.search(r"Function Name: (\S+)", l)
    if m: cur = m.group(1); continue
    m = re.search(r"remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|SGPRs Spill|VGPRs Spill|Occupancy \[waves/SIMD\]): (\S+)", l)
    if m and cur and "k_primaryILj33E" in cur: print(cur[28:50], m.group(1), m.group(2))
    if "error" in l: print(l, end="")
'
