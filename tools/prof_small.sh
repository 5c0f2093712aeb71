#!/bin/bash
# rocprofv3 kernel trace of one 12 500-stream precompress (one rank's share of C4 at 8 GPUs)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-prof_small}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o p --output-format csv -- python3 bench.py --streams 12500 --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/prof.json 2> $O/prof.err || exit 4
echo done
