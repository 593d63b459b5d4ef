# C5: the 4,096 forward biases in an LDS table (the bias loads no longer queue behind the saved-tile
# stores that now end each GEMM): C5 tests, same-box A/B
set -o pipefail
mkdir -p gpurun_out/r4y
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread \
   -k "c5" > gpurun_out/r4y/tests.log 2>&1
RC=$?; tail -2 gpurun_out/r4y/tests.log
case $RC in 0) ;; *) echo "pytest exit $RC: stopping"; exit $RC;; esac
AB_ARGS="--config c5 --precision bf16" bash tools/ab_r4.sh c5b2 "base=|libmarf_base.so" "bl=|" || exit 1
