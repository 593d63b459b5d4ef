set -o pipefail
mkdir -p gpurun_out
bash tools/ab_r4.sh a "s2=MARF_STEP3=0|" "s3=MARF_STEP3=1|" "s3prio=MARF_STEP3=1|libmarf_prio.so" || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist.py -q -rf -p no:cacheprovider --timeout 600 --timeout-method thread -s > gpurun_out/t_r4d_dist.log 2>&1
RC=$?
grep -E "C4|passed|failed|Error|error" gpurun_out/t_r4d_dist.log | tail -30
exit $RC
