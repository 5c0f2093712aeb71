#!/bin/bash
# speculation target by share size: 100k / 50k / 25k / 12.5k streams at ATZ_TARGET 4096 / 8192 / 12288
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-target}; mkdir -p $O
timeout -k 10 400 python3 -c "import sys; sys.path.insert(0,'.'); from antiz_amd import datagen
for n in (100000, 50000, 25000, 12500): datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=n)" > $O/gen.log 2>&1 || exit 3
for n in 12500 25000 50000 100000; do
  for t in 4096 8192 12288; do
    ATZ_TARGET=$t timeout -k 10 300 python3 bench.py --streams $n --steps 2 --warmup 1 --no-cpu --no-recon --no-h2h > $O/n${n}_t$t.json 2> $O/n${n}_t$t.err || exit 4
  done
done
echo done
