#!/bin/bash
# heap A/B + shard tests + an 8-rank one-file rehearsal on the box's one GPU (gloo), with rank_balance
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-heap6}; mkdir -p $O
bash tools/gpu_ab.sh $(basename $O) 2 - ATZ_LIB=antiz_amd/_build/libatz_heap0.so || exit 2
ATZ_LIB=antiz_amd/_build/libatz_clocks.so ATZ_TIMING=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/clk.json 2> $O/clk.err || exit 3
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_shard.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/shard.log 2>&1 || exit 4
ATZ_BENCH_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29508 bench.py --gpus 8 --steps 2 --warmup 1 --no-recon > $O/file8.json 2> $O/file8.err || exit 5
echo done
