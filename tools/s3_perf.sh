#!/bin/bash
# Two-waves-per-SIMD kernel, performance iteration: quick bf16x3 parity tests + bench lines
# (s3_check.sh), then the per-phase stamps of libmarf_stamps.so.   bash tools/s3_perf.sh <tag>
set -o pipefail
TAG=${1:-s3p}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
bash tools/s3_check.sh $TAG || exit $?
MARF_STEP3=1 MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_stamps.so timeout -k 10 200 \
  python tools/step2_phases.py --kernel step3 > $OUT/phases.txt 2>&1 || { echo "phases failed"; tail -5 $OUT/phases.txt; exit 1; }
grep -v amdgpu.ids $OUT/phases.txt
