#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t14
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_full.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t14/test.log 2>&1 || exit 2
ATZ_LIB=antiz_amd/_build/libatz_steps.so ATZ_TIMING=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > gpurun_out/t14/steps.json 2> gpurun_out/t14/steps.err || exit 3
