# round 6: deflate/match parity, then C4 and C3 A/Bs against the previous commit's library (ATZ_LIB)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r6e}; shift
mkdir -p gpurun_out/$T
timeout -k 10 900 python3 -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "deflate or holes or long_streams or golden or c5 or bench_config or maxdist or replay or bucket" > gpurun_out/$T/test.log 2>&1 || exit 2
bash tools/ab_env.sh ${T}_c4 3 "-" "ATZ_LIB=antiz_amd/_build/diag/lib_prev.so" > gpurun_out/$T/ab_c4.txt 2>&1 || exit 5
AB_WORKLOAD=c3 bash tools/ab_env.sh ${T}_c3 2 "-" "ATZ_LIB=antiz_amd/_build/diag/lib_prev.so" > gpurun_out/$T/ab_c3.txt 2>&1 || exit 4
echo done
