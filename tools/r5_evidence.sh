#!/bin/bash
# Round-5 evidence calls (each under gpurun's 20-minute limit).  usage: tools/r5_evidence.sh <tag> <part>
#   a: the whole -m gpu suite, the driver's default bench line, one profiled step (kernel trace + stats)
#   b: SQ and FETCH_SIZE / WRITE_SIZE passes, the share lines (50 000 / 25 000 / 12 500 streams), the C5 line
#   c: the 3-context ceiling run, then the 8-rank one-file rehearsal on this GPU (c4 and c4c3)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r5e}; P=${2:-a}
O=gpurun_out/$T; mkdir -p $O
case $P in
  a) bash tools/measure.sh $T test bench prof || exit $? ;;
  b) bash tools/measure.sh $T sq pmc || exit $?
     bash tools/shares.sh ${T}_sh || exit 20
     timeout -k 10 400 python3 bench.py --workload c5 --steps 3 --warmup 1 --no-recon --no-h2h > $O/c5.json 2> $O/c5.err || exit 21 ;;
  c) for n in 12500 25000; do   # one rank's share at N = 8 / 4, as bench.py runs it there (8 hardware queues)
       GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 bench.py --streams $n --steps 3 --warmup 1 --no-cpu --no-recon --no-h2h > $O/q8_s$n.json 2> $O/q8_s$n.err || exit 29
     done
     bash tools/ceiling.sh ${T}_ceil || exit 30
     WLS="c4 c4c3" HINTS=1 bash tools/balance.sh ${T}_bal 8 || exit 31 ;;
esac
echo done
