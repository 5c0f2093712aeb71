#!/bin/bash
# Per-trial phase clocks (ATZ_STEP_CLOCKS build, tools/variant.sh clocks -DATZ_STEP_CLOCKS=1) on the
# 12 500-stream file and the full C4 file, with the ATZ_TIMING=2 round timeline and slowest trials.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${1:-clocks}; mkdir -p $O
ATZ_LIB=antiz_amd/_build/libatz_clocks.so ATZ_TIMING=2 timeout -k 10 200 python3 bench.py --streams 12500 --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/small.json 2> $O/small.err || exit 1
ATZ_LIB=antiz_amd/_build/libatz_clocks.so ATZ_TIMING=2 timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/full.json 2> $O/full.err || exit 2
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-recon --no-h2h > $O/bench.json 2> $O/bench.err || exit 3
echo done
