# C5 tile kernel with its 4,096 biases in LDS (the 8-wave block's bias table): C5 tests, same-box A/B
set -o pipefail
mkdir -p gpurun_out/r4w
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread \
   -k "c5" > gpurun_out/r4w/tests.log 2>&1
RC=$?; tail -2 gpurun_out/r4w/tests.log
case $RC in 0) ;; *) echo "pytest exit $RC: stopping"; exit $RC;; esac
AB_ARGS="--config c5 --precision bf16" bash tools/ab_r4.sh c5bl "base=|libmarf_base.so" "new=|" || exit 1
AB_ARGS="--config c5 --precision bf16" bash tools/ab_r4.sh c5sa "base=|" "after=|libmarf_stafter.so" || exit 1
