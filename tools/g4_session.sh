set -o pipefail
O=gpurun_out/g4
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_fp16x2.py tests/test_gpu_parity.py -k "fp16x2 or wide_skip" -v --timeout 150 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1; rc=$?
echo "pytest rc $rc"; grep -E "passed|failed" $O/t.log | tail -3
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u tools/seed_sweep.py --seeds 3 --precisions fp16x2 --perturb 0 --out $O/seed3_fp16x2.json > $O/seed3_fp16x2.log 2>&1 || exit 5
tail -2 $O/seed3_fp16x2.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "test_c1_3000" -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t3000.log 2>&1; rc=$?
echo "3000 rc $rc"; grep -E "final PSNR|passed|failed" $O/t3000.log | tail -6
[ $rc -le 1 ] || exit $rc
bash tools/pmc_traffic.sh g4/pmc_c3h c3 fp16x2 || exit 6
bash tools/pmc_traffic.sh g4/pmc_c3x c3 bf16x3 || exit 7
grep -A30 "k_step2" $O/pmc_c3h/pmc.csv | head -3 ; python - <<'PY'
import csv
for t in ("pmc_c3h", "pmc_c3x"):
    for r in csv.DictReader(open(f"gpurun_out/g4/{t}/pmc.csv")):
        if r["kernel"].startswith("k_step2") or r["kernel"].startswith("k_wgrad_dma_layers"):
            print(t, r["kernel"], {k: r[k] for k in ("mfma_busy", "valu_per_mfma", "SQ_INSTS_VMEM_RD", "hbm_read_bytes", "hbm_write_bytes", "pmc_avg_ns") if k in r})
PY
