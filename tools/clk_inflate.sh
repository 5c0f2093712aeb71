#!/bin/bash
# Inflate diagnostics: the -m gpu inflate/scan tests, then one C4 precompress on the ATZ_INF_CLOCKS
# build (per-job clocks, blocks, header and copy cycles).  usage: tools/clk_inflate.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-clk}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread -k "inflate or scan or golden or consumption" > $O/test.log 2>&1 || exit 2
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'.'); from antiz_amd import datagen; datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=100000)" > $O/gen.log 2>&1 || exit 3
ATZ_LIB=antiz_amd/_build/libatz_clk.so ATZ_TIMING=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/clk.json 2> $O/clk.err || exit 4
ATZ_TIMING=1 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-recon --no-h2h > $O/bench.json 2> $O/bench.err || exit 5
echo done
