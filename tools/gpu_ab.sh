#!/bin/bash
# tests/test_gpu.py + knob test, then interleaved env A/B on the full C4 and on the 12 500-stream share.
# usage: tools/gpu_ab.sh <tag> <reps> "<env A>" "<env B>" ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; R=$2; shift 2
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_knobs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/test.log 2>&1 || exit 2
bash tools/ab_env.sh ${TAG}_f $R "$@" || exit 3
AB_STREAMS=12500 bash tools/ab_env.sh ${TAG}_s $R "$@" || exit 4
echo done
