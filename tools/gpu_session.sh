#!/bin/bash
# Run a sequence of GPU steps on the gpurun box, each under its own time limit.
# Usage: tools/gpu_session.sh STEP... where STEP is one of: smoke tests bench prof pmc bench_all
# Stops at the first step that ends in a fault / abort / time limit (rc not in {0,1}).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
run() {
  local name=$1 limit=$2; shift 2
  echo "== $name: $*" >> gpurun_out/summary.txt
  local t0=$(date +%s)
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(( $(date +%s) - t0 ))s" | tee -a gpurun_out/summary.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  # a failed smoke test means the library is broken: run nothing else on the GPU
  if [ $rc -ne 0 ] && [ "$name" = smoke ]; then echo "stopping after failed smoke"; exit $rc; fi
}
for step in "$@"; do
  case $step in
    smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run tests 900 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -rf ;;
    bench) run bench 600 python3 bench.py ;;
    bench_nocpu) run bench_nocpu 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ;;
    shard8) for n in 2 4 8; do run "bench_shard$n" 300 python3 bench.py --no-cpu-baseline --shard-of $n; done ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ;;
    pmc_fetch) run pmc_fetch_${CONFIG:-example1_1080p_d5} 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_${CONFIG:-example1_1080p_d5} -o bench --output-format csv -- python3 bench.py --config ${CONFIG:-example1_1080p_d5} --steps 3 --warmup 1 --no-cpu-baseline ;;
    pmc_write) run pmc_write_${CONFIG:-example1_1080p_d5} 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_${CONFIG:-example1_1080p_d5} -o bench --output-format csv -- python3 bench.py --config ${CONFIG:-example1_1080p_d5} --steps 3 --warmup 1 --no-cpu-baseline ;;
    configs_long) run bench_example3_1080p_d8 600 python3 bench.py --config example3_1080p_d8 --steps 100 --warmup 20
                  run bench_example4_4k_d6 600 python3 bench.py --config example4_4k_d6 --steps 20 --warmup 5
                  run bench_cornell_800_s512 900 python3 bench.py --config cornell_800_s512 --steps 2 --warmup 1
                  run bench_mesh_1080p_d3 600 python3 bench.py --config mesh_1080p_d3 --steps 100 --warmup 20 ;;
    configs) for c in example3_1080p_d8 example4_4k_d6 cornell_800_s512; do run "bench_$c" 600 python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline; done ;;
    pmc_list) run pmc_list 120 rocprofv3 -L ;;
    pmc_sq) run pmc_sq1 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d gpurun_out/pmc_sq1 -o bench --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
            run pmc_sq2 600 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_sq2 -o bench --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    pmc4) C=${CONFIG:-example1_1080p_d5}; T=${PMC_TAG:-r03}
          for pass in "A:SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE" \
                      "B:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
                      "F:FETCH_SIZE" "W:WRITE_SIZE"; do
            k=${pass%%:*}; ctr=${pass#*:}
            run pmc${k}_$C 240 rocprofv3 --pmc $ctr --kernel-trace -d gpurun_out/pmc_${T}_${C}_$k -o bench --output-format csv -- python3 bench.py --config $C --steps ${PMC_STEPS:-3} --warmup 1 --no-cpu-baseline --no-secondary
          done ;;
    shardall) for C in ${SHARD_CONFIGS:-example1_1080p_d5 example4_4k_d6 cornell_800_s512}; do
                case $C in cornell*) st=2;; example4*) st=10;; *) st=100;; esac
                run "whole_$C" 300 python3 bench.py --config $C --no-cpu-baseline --no-secondary --steps $st --warmup $((st > 50 ? 300 : 2))
                for n in ${SHARD_NS:-2 4 8}; do
                  run "shard${n}_$C" 300 python3 bench.py --config $C --no-cpu-baseline --no-secondary --steps $st --warmup 2 --shard-of $n --shard-rank all ${SHARD_ARGS:-}
                done
              done ;;
    mttests) run mttests 600 python3 -u -m pytest tests/test_multirank.py tests/test_mt.py tests/test_gpu.py -x -v -m gpu -k "band or shard or mt or numpy_stream or async" --timeout 300 --timeout-method thread -rf ;;
    mctests) run mctests 600 python3 -u -m pytest tests/test_gpu_mc.py -x -v -m gpu --timeout 300 --timeout-method thread -rf ;;
    shardtests) run shardtests 600 python3 -u -m pytest tests/test_gpu_shards.py -x -v -s -m gpu --timeout 300 --timeout-method thread -rf ;;
    ab) run ab 900 bash tools/ab_bench.sh "tools/_build/libsightpy_hip_old.so python-raytracer_amd/sightpy/libsightpy_hip.so" --steps ${STEPS:-50} ${AB_ARGS:-} ;;
    shardsweep) for n in ${SHARD_NS:-8}; do for k in ${KMAXS:-2 4 8 17 32}; do run "sweep_${CONFIG:-example1_1080p_d5}_n${n}_k$k" 300 python3 bench.py --config ${CONFIG:-example1_1080p_d5} --no-cpu-baseline --no-secondary --steps ${STEPS:-100} --shard-of $n --shard-rank all --shard-bands $k; done; done
                run "sweep_${CONFIG:-example1_1080p_d5}_whole" 300 python3 bench.py --config ${CONFIG:-example1_1080p_d5} --no-cpu-baseline --no-secondary --steps ${STEPS:-100} ;;
    mt) run mt 300 python3 tools/mt_timing.py ;;
    api) run api 300 python3 tools/api_timing.py --repeats 5 --profile ;;
    api_prof) run api_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/api_prof -o api --output-format csv -- python3 tools/api_timing.py --repeats 5 ;;
    shardprof) run shardprof_${SHARD:-8}_r${SHARD_RANK:-0} 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/shardprof_${SHARD:-8}_r${SHARD_RANK:-0} -o s --output-format csv -- python3 bench.py --config ${CONFIG:-example1_1080p_d5} --steps 20 --warmup 2 --no-cpu-baseline --no-secondary --shard-of ${SHARD:-8} --shard-rank ${SHARD_RANK:-0} ;;
    profsync) run profsync 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profsync -o bench --output-format csv -- python3 bench.py --sync --no-cpu-baseline --no-secondary ;;
    profsync_lean) run profsync_lean 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profsync_lean -o bench --output-format csv -- python3 bench.py --sync --option sync_lean=1 --no-cpu-baseline --no-secondary --steps ${STEPS:-45} --warmup 5 ;;
    driver) run driver 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    rngdev) run bench_rngdev 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --rng device ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
