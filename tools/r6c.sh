# round 6: parity (the whole -m gpu suite minus the full-size configs) and a C4 A/B against the round's base
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r6c}
mkdir -p gpurun_out/$T
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --deselect tests/test_gpu_full.py > gpurun_out/$T/test.log 2>&1 || exit 2
bash tools/ab_env.sh ${T}_c4 3 "-" "ATZ_LIB=antiz_amd/_build/diag/lib_base.so" > gpurun_out/$T/ab_c4.txt 2>&1 || exit 5
AB_WORKLOAD=c3 bash tools/ab_env.sh ${T}_c3 1 "-" > gpurun_out/$T/ab_c3.txt 2>&1 || exit 4
echo done
