# round 6: bucket-sort change -- verify against the other bucket kernels, parity tests, then C4 / N = 8-share / one-pipe A/Bs against lib_prev2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r6p}
mkdir -p gpurun_out/$T
ATZ_BUCKETS_VERIFY=1 timeout -k 10 200 python3 bench.py --steps 1 --warmup 0 --no-cpu --no-recon --no-h2h > gpurun_out/$T/verify.json 2> gpurun_out/$T/verify.err || exit 3
timeout -k 10 900 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_grid.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/test.log 2>&1 || exit 2
AB_STREAMS=100000 bash tools/ab_env.sh ${T}_iso 2 "ATZ_PIPES=1" "ATZ_PIPES=1 ATZ_LIB=antiz_amd/_build/diag/lib_prev2.so" > gpurun_out/$T/ab_iso.txt 2>&1 || exit 4
bash tools/ab_env.sh ${T}_c4 3 "-" "ATZ_LIB=antiz_amd/_build/diag/lib_prev2.so" > gpurun_out/$T/ab_c4.txt 2>&1 || exit 5
AB_STREAMS=12500 bash tools/ab_env.sh ${T}_p6 3 "ATZ_PIPES=6 GPU_MAX_HW_QUEUES=8" "ATZ_PIPES=6 GPU_MAX_HW_QUEUES=8 ATZ_LIB=antiz_amd/_build/diag/lib_prev2.so" > gpurun_out/$T/ab_p6.txt 2>&1 || exit 6
echo done
