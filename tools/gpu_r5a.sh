# tile kernel: the saved tile's stores at the top of the GEMM's last 4-k-step iteration (after its
# last real weight loads) instead of after the GEMM: C5 tests on the variant, same-box A/B at C5 and C3 bf16
set -o pipefail
mkdir -p gpurun_out/r5a
MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_late4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread \
   -k "c5 or bf16_step" > gpurun_out/r5a/tests.log 2>&1
RC=$?; tail -2 gpurun_out/r5a/tests.log
case $RC in 0) ;; *) echo "pytest exit $RC: stopping"; exit $RC;; esac
AB_ARGS="--config c5 --precision bf16" bash tools/ab_r4.sh late4 "base=|" "late4=|libmarf_late4.so" || exit 1
AB_ARGS="--precision bf16" bash tools/ab_r4.sh late4c3 "base=|" "late4=|libmarf_late4.so" || exit 1
