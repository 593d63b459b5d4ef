#!/bin/bash
# GPU iteration: parity tests, short bench, phase stamps.  bash tools/gpu_diag.sh <tag>
set -o pipefail
TAG=${1:-d}
bash tools/gpu_quick.sh $TAG || exit $?
MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_stamps.so timeout -k 10 300 python tools/phase_stamps.py > gpurun_out/stamps_$TAG.txt 2>&1
tail -17 gpurun_out/stamps_$TAG.txt
