#!/bin/bash
# C5 parity test, ATZ_TIMING=2 timeline of one C4 step, and a C5 (--brute-window) bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-probe}; mkdir -p $O
timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0,'.')
from antiz_amd import datagen; print(datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=100000)); print(datagen.cached('c5','/tmp/atz_bench_cache',seed=5,n_streams=100000))" > $O/gen.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "c5 or bench_config" > $O/test.log 2>&1 || exit 2
ATZ_TIMING=2 timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --no-cpu --no-recon > $O/timing.json 2> $O/timing.err || exit 3
timeout -k 10 400 python3 bench.py --workload c5 --steps 3 --warmup 1 > $O/c5.json 2> $O/c5.err || exit 4
echo done
