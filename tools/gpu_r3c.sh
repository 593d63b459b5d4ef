#!/bin/bash
# ReLU-mask A/B (bit-identity + timing vs lib/libmarf_old.so), C5 tests and A/B, phase stamps.
set -o pipefail
T=${1:-r3c}
mkdir -p gpurun_out/$T
bash tools/ab_check.sh $T/ab || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread -k 'c5 or dist' > gpurun_out/$T/tests.log 2>&1
RC=$?; tail -3 gpurun_out/$T/tests.log
case $RC in 0|1) ;; *) exit $RC;; esac
bash tools/c5_ab.sh $T/c5 || exit $?
MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_stamps.so timeout -k 10 200 python tools/step2_phases.py > gpurun_out/$T/phases.txt 2>&1; cat gpurun_out/$T/phases.txt | grep -v warning
