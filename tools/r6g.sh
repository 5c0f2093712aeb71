# round 6: parity of the fast-level paths, then C4 and 12 500-stream-share A/Bs against the previous commit
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r6g}
mkdir -p gpurun_out/$T
timeout -k 10 900 python3 -u -m pytest tests/test_gpu.py tests/test_gpu_grid.py -m gpu -x -v --timeout 300 --timeout-method thread -k "deflate or holes or long_streams or golden or c5 or bench_config or maxdist or replay or grid or zt" > gpurun_out/$T/test.log 2>&1 || exit 2
bash tools/ab_env.sh ${T}_c4 3 "-" "ATZ_LIB=antiz_amd/_build/diag/lib_prev.so" > gpurun_out/$T/ab_c4.txt 2>&1 || exit 5
AB_STREAMS=12500 bash tools/ab_env.sh ${T}_s8 3 "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=8 ATZ_LIB=antiz_amd/_build/diag/lib_prev.so" > gpurun_out/$T/ab_s8.txt 2>&1 || exit 6
echo done
