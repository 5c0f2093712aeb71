#!/bin/bash
# queues x pipes on one rank's share of C4 at 8 / 4 / 2 GPUs (12 500 / 25 000 / 50 000 streams)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
AB_STREAMS=12500 bash tools/ab_env.sh ab9 1 "-" "GPU_MAX_HW_QUEUES=8 ATZ_PIPES=6" "GPU_MAX_HW_QUEUES=16 ATZ_PIPES=6" "GPU_MAX_HW_QUEUES=16 ATZ_PIPES=8" "GPU_MAX_HW_QUEUES=8 ATZ_PIPES=4" "GPU_MAX_HW_QUEUES=12 ATZ_PIPES=6" || exit 3
AB_STREAMS=25000 bash tools/ab_env.sh ab10 1 "-" "GPU_MAX_HW_QUEUES=8 ATZ_PIPES=6" "GPU_MAX_HW_QUEUES=16 ATZ_PIPES=8" || exit 4
AB_STREAMS=50000 bash tools/ab_env.sh ab11 1 "-" "GPU_MAX_HW_QUEUES=8 ATZ_PIPES=6" || exit 5
