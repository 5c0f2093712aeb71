set -o pipefail
O=gpurun_out/r5base; mkdir -p $O
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu --no-recon --no-h2h > $O/full.json 2> $O/full.err || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python3 bench.py --streams 12500 --steps 5 --warmup 1 --no-cpu --no-recon --no-h2h > $O/s12.json 2> $O/s12.err || exit 2
GPU_MAX_HW_QUEUES=8 ATZ_TIMING=2 timeout -k 10 300 python3 bench.py --streams 12500 --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/t12.json 2> $O/t12.err || exit 3
ATZ_TIMING=2 timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/tfull.json 2> $O/tfull.err || exit 4
echo done
