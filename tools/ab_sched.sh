#!/bin/bash
# Scheduler A/B in one GPU call: parity (test_gpu.py, the knob test, the multi-rank tests), then the
# C4 bench line and the 12 500-stream share under the flow scheduler (default) and ATZ_SCHED=rounds,
# interleaved.  usage: tools/ab_sched.sh <tag> [notest]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-absched}; mkdir -p $O
if [ "$2" != notest ]; then
  timeout -k 10 900 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_knobs.py tests/test_gpu_shard.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/test.log 2>&1 || exit 2
fi
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'.'); from antiz_amd import datagen; datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=100000); datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=12500)" > $O/gen.log 2>&1 || exit 3
for i in 1 2; do
  for s in flow rounds; do
    ATZ_SCHED=$s timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-h2h --no-recon > $O/full_${s}_$i.json 2> $O/full_${s}_$i.err || exit 4
    ATZ_SCHED=$s timeout -k 10 300 python3 bench.py --streams 12500 --steps 3 --warmup 1 --no-cpu --no-h2h --no-recon > $O/small_${s}_$i.json 2> $O/small_${s}_$i.err || exit 5
    ATZ_SCHED=$s GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 bench.py --streams 12500 --steps 3 --warmup 1 --no-cpu --no-h2h --no-recon > $O/small8_${s}_$i.json 2> $O/small8_${s}_$i.err || exit 6
  done
done
echo done
