bash tools/gpu_session.sh smoke tests || exit 1
CONFIG=example3_1080p_d8 bash tools/gpu_session.sh pmc_fetch pmc_write || exit 1
CONFIG=example4_4k_d6 bash tools/gpu_session.sh pmc_fetch pmc_write || exit 1
