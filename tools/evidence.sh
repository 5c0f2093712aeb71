#!/bin/bash
# Evidence calls for the round's profiles/ (each under gpurun's 20-minute limit).  usage: tools/evidence.sh <tag> <part>
#   a: the whole -m gpu suite, the driver's default bench line, one profiled step (kernel trace + stats)
#   b: SQ and FETCH_SIZE / WRITE_SIZE passes over one C4 step
#   c: the share lines (50 000 / 25 000 / 12 500 streams), the 12 500-stream share on six pipes and eight
#      queues as an N = 8 rank runs it (shard_sweep sizes its pipes by the rank's records; the one-GPU
#      path by the scan's candidate bound, hence ATZ_PIPES here), and the C2 / C3 / C5 bench lines
#   d: the 8-rank one-file rehearsal on this GPU (gloo; C4 and the C3-clustered file)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-ev}; P=${2:-a}
O=gpurun_out/$T; mkdir -p $O
case $P in
  a) bash tools/measure.sh $T test bench prof || exit $? ;;
  b) bash tools/measure.sh $T sq pmc || exit $? ;;
  c) bash tools/shares.sh ${T}_sh || exit 20
     for i in 1 2 3; do
       ATZ_PIPES=6 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 bench.py --streams 12500 --steps 3 --warmup 1 --no-cpu --no-recon --no-h2h > $O/q8p6_s12500_$i.json 2> $O/q8p6_s12500_$i.err || exit 21
     done
     for w in c2 c3 c5; do
       timeout -k 10 600 python3 bench.py --workload $w > $O/$w.json 2> $O/$w.err || exit 22
     done ;;
  d) WLS="c4 c4c3" HINTS=1 bash tools/balance.sh ${T}_bal 8 || exit 31 ;;
  e) for i in 1 2 3; do
       ATZ_PIPES=6 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 bench.py --streams 12500 --steps 3 --warmup 1 --no-cpu --no-recon --no-h2h > $O/q8p6_s12500_$i.json 2> $O/q8p6_s12500_$i.err || exit 21
     done ;;
esac
echo done
