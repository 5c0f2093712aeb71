#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t16
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread -k "inflate or scan or golden or far or consumption or roundtrip" > gpurun_out/t16/test.log 2>&1 || exit 2
bash tools/ab.sh ab13 2 antiz_amd/_build/libatz_prev.so antiz_amd/_build/libatz_accel.so || exit 3
for f in gpurun_out/ab13/*.json; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);x=d['detail'];print('$f',d['value'],x['scan_ms'],x['k_inflate_ms'])"; done
