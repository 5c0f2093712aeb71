# round 6: fast-level parity, then C4 (with the round timeline's slowest trials) and N = 8-share A/Bs against lib_prev2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r6l}
mkdir -p gpurun_out/$T
timeout -k 10 900 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_grid.py -m gpu -x -v --timeout 300 --timeout-method thread -k "deflate or holes or long_streams or golden or c5 or bench_config or maxdist or grid" > gpurun_out/$T/test.log 2>&1 || exit 2
bash tools/ab_env.sh ${T}_c4 3 "-" "ATZ_LIB=antiz_amd/_build/diag/lib_prev2.so" > gpurun_out/$T/ab_c4.txt 2>&1 || exit 5
AB_STREAMS=12500 bash tools/ab_env.sh ${T}_p6 3 "ATZ_PIPES=6 GPU_MAX_HW_QUEUES=8" "ATZ_PIPES=6 GPU_MAX_HW_QUEUES=8 ATZ_LIB=antiz_amd/_build/diag/lib_prev2.so" > gpurun_out/$T/ab_p6.txt 2>&1 || exit 6
ATZ_TIMING=2 timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > gpurun_out/$T/timing.json 2> gpurun_out/$T/timing.err || exit 7
echo done
