#!/bin/bash
# k_inflate register cap (waves per SIMD) A/B: the scan's k_inflate time on C4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab.sh ab12 2 antiz_amd/_build/libatz_accel.so antiz_amd/_build/libatz_w5.so antiz_amd/_build/libatz_w7.so antiz_amd/_build/libatz_w8.so || exit 2
for f in gpurun_out/ab12/*.json; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);x=d['detail'];print('$f',d['value'],x['scan_ms'],x['k_inflate_ms'])"; done
