# ring slots as wrapping counters in k_step2 (no modulo per stage)
set -o pipefail
mkdir -p gpurun_out/r5g
MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_wrap.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread \
   -k "bitwise or c3_two_patch" > gpurun_out/r5g/tests.log 2>&1
RC=$?; tail -1 gpurun_out/r5g/tests.log
case $RC in 0) ;; *) echo "pytest exit $RC: stopping"; exit $RC;; esac
bash tools/ab_r4.sh wrap "base=|" "wrap=|libmarf_wrap.so" || exit 1
