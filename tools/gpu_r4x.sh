# tile kernel: saved-tile stores after the GEMM (default for the 8-wave C5 block); C5 + plain-bf16
# tests, the C5 line, and the same placement for the 4-wave blocks (plain bf16 at C3) as an A/B
set -o pipefail
mkdir -p gpurun_out/r4x
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread \
   -k "c5 or bf16 or fp16" > gpurun_out/r4x/tests.log 2>&1
RC=$?; tail -2 gpurun_out/r4x/tests.log
case $RC in 0) ;; *) echo "pytest exit $RC: stopping"; exit $RC;; esac
AB_ARGS="--precision bf16" bash tools/ab_r4.sh tile4 "base=|" "after4=|libmarf_after4.so" || exit 1
AB_ARGS="--config c5 --precision bf16" bash tools/ab_r4.sh c5new "new=|" || exit 1
