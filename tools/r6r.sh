# k_bucket_depth: kernel time under rocprofv3 (one C4 step each build) and a C4 A/B against lib_prev3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r6r}
mkdir -p gpurun_out/$T
timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0,'.')
from antiz_amd import datagen
datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=100000)" || exit 1
B1="bench.py --steps 1 --warmup 0 --no-cpu --no-recon --no-h2h"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/pnew -o p --output-format csv -- python3 $B1 > gpurun_out/$T/pnew.json 2> gpurun_out/$T/pnew.err || exit 2
ATZ_LIB=antiz_amd/_build/diag/lib_prev3.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/pold -o p --output-format csv -- python3 $B1 > gpurun_out/$T/pold.json 2> gpurun_out/$T/pold.err || exit 3
bash tools/ab_env.sh ${T}_c4 3 "-" "ATZ_LIB=antiz_amd/_build/diag/lib_prev3.so" > gpurun_out/$T/ab_c4.txt 2>&1 || exit 5
echo done
