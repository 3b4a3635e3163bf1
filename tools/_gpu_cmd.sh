timeout -k 10 300 python3 bench.py --config mesh_1080p_d3 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/mesh_bvh.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --config mesh_1080p_d3 --size 480x270 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/mesh_bvh_small.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --config mesh_1080p_d3 --size 480x270 --steps 1 --warmup 1 --no-cpu-baseline --option bvh=0 > gpurun_out/mesh_linear_small.log 2>&1 || exit 1
