# layer 0 of the specialized k_step2 without gap hooks (the previous row tile's epilogue after its
# GEMM, freely scheduled): bitwise tests on the variant, same-box A/B
set -o pipefail
mkdir -p gpurun_out/r5f
MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_l0free.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread \
   -k "bitwise or c3_two_patch" > gpurun_out/r5f/tests.log 2>&1
RC=$?; tail -1 gpurun_out/r5f/tests.log
case $RC in 0) ;; *) echo "pytest exit $RC: stopping"; exit $RC;; esac
bash tools/ab_r4.sh l0free "base=|" "l0free=|libmarf_l0free.so" || exit 1
