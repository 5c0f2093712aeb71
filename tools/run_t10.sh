#!/bin/bash
# multi-wave cap for small rounds: knob test, then full C4 and 12 500-stream A/Bs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t10
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_knobs.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t10/knobs.log 2>&1 || exit 2
AB_STREAMS=12500 bash tools/ab_env.sh ab6 2 "-" "ATZ_MW_SMALL=4096" "ATZ_MW_SMALL=8192" "ATZ_MW_SMALL=8192 ATZ_MW_CAP=5" || exit 3
bash tools/ab_env.sh ab7 2 "-" "ATZ_MW_SMALL=4096" "ATZ_MW_SMALL=8192" || exit 4
