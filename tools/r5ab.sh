#!/bin/bash
# Round-5 A/B call: the GPU parity tests (test_gpu.py + knobs), then interleaved env A/B on the full C4
# and on the 12 500-stream share with six pipes on eight hardware queues (one rank's share at N = 8).
# usage: tools/r5ab.sh <tag> <reps> "<env A>" "<env B>" ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; R=$2; shift 2
mkdir -p gpurun_out/$TAG
if [ -z "$NO_TEST" ]; then
timeout -k 10 900 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_knobs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/test.log 2>&1 || exit 2
fi
bash tools/ab_env.sh ${TAG}_f $R "$@" || exit 3
S6=()
for E in "$@"; do [ "$E" = "-" ] && E=""; S6+=("ATZ_PIPES=6 GPU_MAX_HW_QUEUES=8 $E"); done
AB_STREAMS=12500 bash tools/ab_env.sh ${TAG}_s $R "${S6[@]}" || exit 4
echo done
