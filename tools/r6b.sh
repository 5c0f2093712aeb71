cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6b
timeout -k 10 900 python3 -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "deflate or far_history or long_streams or c5 or bench_config or maxdist or holes or golden or replay" > gpurun_out/r6b/test.log 2>&1 || exit 2
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_full.py -m gpu -x -v --timeout 300 --timeout-method thread -k "c1 or c3" > gpurun_out/r6b/full.log 2>&1 || exit 3
AB_WORKLOAD=c3 bash tools/ab_env.sh r6b_c3 2 "-" "ATZ_MATCH_WIN=0" "ATZ_LIB=antiz_amd/_build/diag/lib_base.so" > gpurun_out/r6b/ab_c3.txt 2>&1 || exit 4
bash tools/ab_env.sh r6b_c4 3 "-" "ATZ_LIB=antiz_amd/_build/diag/lib_base.so" > gpurun_out/r6b/ab_c4.txt 2>&1 || exit 5
echo done
