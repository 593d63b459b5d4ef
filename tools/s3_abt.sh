#!/bin/bash
# bf16x3 parity tests against each library variant, then the timing A/B (s3_ab.sh).
#   bash tools/s3_abt.sh <tag> <variant.so> ...      (only variants whose results must be unchanged)
set -o pipefail
TAG=$1; shift
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
LIBD=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib
for v in "$@"; do
  [ "$v" = default ] && continue
  MARF_LIB=$LIBD/$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "bf16x3 and not 3000 and not train" > $OUT/tests_${v%.so}.log 2>&1
  rc=$?
  echo "tests $v: rc $rc: $(tail -1 $OUT/tests_${v%.so}.log)"
  case $rc in 0|1) ;; *) echo "pytest died ($rc): stopping"; exit $rc;; esac
done
bash tools/s3_ab.sh $TAG default "$@"
