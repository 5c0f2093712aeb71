#!/bin/bash
# Device assembly of k_inflate<4096> (for reading the decode loop's instruction mix on the CPU):
# tools/isa_inflate.sh [extra hipcc flags] -> /tmp/isa/inf.s
mkdir -p /tmp/isa
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -x hip --cuda-device-only -S "$@" antiz_amd/csrc/atz_accel.cpp -o /tmp/isa/atz.s 2>&1 | grep -A4 " error" && exit 1
K=_ZN3atz9k_inflateILj4096EEEvPKhPhPKNS_6InfJobEPNS_6InfResEjS3_Pym
a=$(grep -n "^$K:" /tmp/isa/atz.s | cut -d: -f1); b=$(grep -n "^.Lfunc_end" /tmp/isa/atz.s | awk -F: -v a=$a '$1>a{print $1; exit}')
sed -n "${a},${b}p" /tmp/isa/atz.s > /tmp/isa/inf.s
grep -E "\.(sgpr|vgpr)_(count|spill)|ScratchSize|Occupancy|NumVgprs|NumSgprs" /tmp/isa/atz.s | grep -A0 "" | sed -n "1,0p"
wc -l /tmp/isa/inf.s
