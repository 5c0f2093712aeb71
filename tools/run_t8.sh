#!/bin/bash
# round-3 session 3: full GPU suite, then tail-table and small-shard A/Bs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t8
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t8/test.log 2>&1 || exit 2
bash tools/ab_env.sh ab3 2 "ATZ_FULL_SMALL=0" "ATZ_FULL_SMALL=2048" "ATZ_FULL_SMALL=8192" || exit 3
AB_STREAMS=12500 bash tools/ab_env.sh ab4 2 "ATZ_FULL_SMALL=0" "ATZ_FULL_SMALL=2048" "ATZ_TARGET=16384" "ATZ_TARGET=16384 ATZ_FULL_SMALL=8192" || exit 4
