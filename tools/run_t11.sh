#!/bin/bash
# step-clock breakdown of the trial kernels (ATZ_STEP_CLOCKS build) on C4, then small-shard queue A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t11
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'.'); from antiz_amd import datagen; datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=100000)" > gpurun_out/t11/gen.log 2>&1 || exit 1
ATZ_LIB=antiz_amd/_build/libatz_steps.so ATZ_TIMING=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > gpurun_out/t11/steps.json 2> gpurun_out/t11/steps.err || exit 2
AB_STREAMS=12500 bash tools/ab_env.sh ab8 2 "-" "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=8 ATZ_PIPES=6" || exit 3
