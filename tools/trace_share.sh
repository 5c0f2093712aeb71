#!/bin/bash
# Kernel timeline of one 12 500-stream share step (six pipes on eight hardware queues, the N = 8
# configuration) and of one full C4 step: rocprofv3 --kernel-trace, analysed by tools/trace_gaps.py.
# usage: tools/trace_share.sh <tag> [env settings for both runs]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-trace}; shift; mkdir -p $O
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'.'); from antiz_amd import datagen; datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=100000); datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=12500)" > $O/gen.log 2>&1 || exit 3
[ $# -gt 0 ] && export "$@"
ATZ_PIPES=6 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/s6 -o t --output-format csv -- python3 bench.py --streams 12500 --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/s6.json 2> $O/s6.err || exit 4
python3 tools/trace_gaps.py $O/s6 > $O/s6_gaps.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/full -o t --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/full.json 2> $O/full.err || exit 5
python3 tools/trace_gaps.py $O/full > $O/full_gaps.txt 2>&1 || true
rm -rf $O/s6 $O/full
echo done
