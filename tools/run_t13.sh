#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t13
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_knobs.py tests/test_gpu_shard.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t13/knobs.log 2>&1 || exit 2
bash tools/gpu_measure.sh t13 file8 || exit 3
