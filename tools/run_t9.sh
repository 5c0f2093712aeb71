#!/bin/bash
# round-3 session 3: the r3_v4 measurement (bench, kernel stats, PMC traffic, small-shard timeline),
# then small-shard (12 500 streams, one rank's share at 8 GPUs) pipe and multi-wave A/Bs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_measure.sh r3_v4 bench prof pmc small || exit 2
AB_STREAMS=12500 bash tools/ab_env.sh ab5 2 "-" "ATZ_PIPES=4" "ATZ_PIPES=6" "ATZ_MW=4" || exit 3
