#!/bin/bash
# Rank balance of the one-file split: 8 ranks on the one GPU (gloo), C4 and the
# C3-clustered file, the hint-based split (default) and round 3's fixed weights (ATZ_SPLIT_HINT=0).
# Each run prints bench.py's JSON line; its rank_balance holds per-rank trials / cycles / sweep time.
# usage: tools/balance.sh <tag> [world]
set -o pipefail
tag=${1:-bal}; W=${2:-8}
out=gpurun_out/$tag; mkdir -p $out
export ATZ_BENCH_BACKEND=gloo ATZ_BENCH_CACHE=/tmp/atz_bench_cache
# eight ranks share the one GPU's 288 GB here: the smaller round target keeps their round scratch within
# it (on a node each rank has a GPU of its own)
export ATZ_TARGET=${ATZ_TARGET:-4096}
port=29611
for wl in ${WLS:-c4 c4c3}; do
  for hint in ${HINTS:-1 0}; do
    port=$((port + 1))
    echo "== $wl hint=$hint $(date +%T)"
    ATZ_SPLIT_HINT=$hint timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus $W --steps 1 --warmup 1 --workload $wl \
      --no-cpu > $out/${wl}_h$hint.json 2> $out/${wl}_h$hint.log || { echo "FAILED rc=$?"; tail -20 $out/${wl}_h$hint.log; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('$out/${wl}_h$hint.json').read().strip().splitlines()[-1])
b=d['rank_balance']; print('$wl hint=$hint', d['value'], 'MB/s', d['ms_per_step'], 'ms; alg max/mean', b['alg_max_over_mean'], 'cyc max/mean', b['cyc_max_over_mean'], 'sweep_ms', b['sweep_ms'], 'streams', b['n_streams'], 'parity', d.get('atz_parity'))"
  done
done
