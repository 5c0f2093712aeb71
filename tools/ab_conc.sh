#!/bin/bash
# Concurrency probes: two processes sharing the GPU, each precompressing its own C4 file (gloo, shards
# mode: the GPU's headroom beyond one file), the flow scheduler with 6 pipes on 8 hardware queues, and
# ATZ_TIMING=2 timelines of the 12 500-stream share under both schedulers.  usage: tools/ab_conc.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-abconc}; mkdir -p $O
timeout -k 10 400 python3 -c "import sys; sys.path.insert(0,'.'); from antiz_amd import datagen
for s in (4, 5): datagen.cached('c4','/tmp/atz_bench_cache',seed=s,n_streams=100000)
datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=12500)" > $O/gen.log 2>&1 || exit 3
for s in rounds flow; do
  ATZ_SCHED=$s ATZ_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --mode shards --steps 2 --warmup 1 --no-cpu --no-recon --no-h2h > $O/two_$s.json 2> $O/two_$s.err || exit 4
done
for s in rounds flow; do
  ATZ_SCHED=$s ATZ_PIPES=6 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-h2h --no-recon > $O/full6_$s.json 2> $O/full6_$s.err || exit 5
  ATZ_SCHED=$s ATZ_PIPES=6 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 bench.py --streams 12500 --steps 3 --warmup 1 --no-cpu --no-h2h --no-recon > $O/small6_$s.json 2> $O/small6_$s.err || exit 6
  ATZ_SCHED=$s ATZ_TIMING=2 timeout -k 10 300 python3 bench.py --streams 12500 --steps 1 --warmup 1 --no-cpu --no-h2h --no-recon > $O/smallt_$s.json 2> $O/smallt_$s.err || exit 7
done
echo done
