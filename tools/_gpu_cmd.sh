for fk in 1 0; do
  for c in example1_1080p_d5 example3_1080p_d8 example4_4k_d6 cornell_800_s512; do
    SIGHTPY_FRAME_KERNEL=$fk timeout -k 10 300 python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_${c}_fk$fk.log 2>&1 || exit 1
  done
done
