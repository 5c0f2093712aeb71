# allocation counters per sweep (ATZ_TIMING=1): the 12 500-stream share on six pipes, then C4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r6q}
mkdir -p gpurun_out/$T
timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0,'.')
from antiz_amd import datagen
datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=12500); datagen.cached('c4','/tmp/atz_bench_cache',seed=4,n_streams=100000)" || exit 1
ATZ_PIPES=6 GPU_MAX_HW_QUEUES=8 ATZ_TIMING=1 timeout -k 10 200 python3 bench.py --streams 12500 --steps 5 --warmup 1 --no-cpu --no-recon --no-h2h > gpurun_out/$T/share.json 2> gpurun_out/$T/share.err || exit 2
ATZ_TIMING=1 timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-recon --no-h2h > gpurun_out/$T/c4.json 2> gpurun_out/$T/c4.err || exit 3
echo done
