#!/bin/bash
# the round-end checks the driver runs: the whole -m gpu suite, then smoke()
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final/test.log 2>&1 || exit 2
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit 3
echo done
