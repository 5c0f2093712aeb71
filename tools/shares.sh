#!/bin/bash
# One GPU, one file per share size: what one rank's share of the 1 GB file costs at N = 2, 4, 8
# (50 000 / 25 000 / 12 500 streams; the same generator, seed 4), default settings; then the 12 500-stream
# share once more with the round timeline (ATZ_TIMING=2).  usage: tools/shares.sh <tag>
set -o pipefail
O=gpurun_out/${1:-shares}; mkdir -p $O
for n in 50000 25000 12500; do
  timeout -k 10 300 python3 bench.py --streams $n --steps 3 --warmup 1 --no-cpu --no-recon --no-h2h > $O/s$n.json 2> $O/s$n.err || exit 1
  python3 -c "
import json; d=json.loads(open('$O/s$n.json').read().strip().splitlines()[-1]); x=d['detail']
print('$n', d['value'], 'MB/s', d['ms_per_step'], 'ms; scan', x['scan_ms'], 'sweep', x['sweep_ms'], 'k_trial', x['k_trial_ms'])"
done
ATZ_TIMING=2 timeout -k 10 300 python3 bench.py --streams 12500 --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/t12500.json 2> $O/t12500.err || exit 2
echo done
