bash tools/gpu_session.sh smoke tests || exit 1
for cr in 0 200000 600000 1500000; do
  timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --option chain_rays=$cr > gpurun_out/chain_$cr.log 2>&1 || exit 1
  timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --option chain_rays=$cr --shard-of 8 > gpurun_out/chain8_$cr.log 2>&1 || exit 1
done
