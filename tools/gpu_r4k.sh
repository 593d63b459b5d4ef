# the rest of the emulated-recipe draws (r4j ran out of time with three sweeps side by side)
set -o pipefail
mkdir -p gpurun_out/r4k
LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_diagrt.so
MARF_LIB=$LIB MARF_DIAG_PREC=2221,2221,2221,2221,2222 timeout -k 10 400 python -u tools/seed_sweep.py --seeds 3 --precisions fp32 \
  --perturb $(seq 52 64) --out gpurun_out/r4k/rs_x3_b.json > gpurun_out/r4k/rs_x3_b.log 2>&1 || { echo "x3 failed"; tail -3 gpurun_out/r4k/rs_x3_b.log; exit 1; }
tail -1 gpurun_out/r4k/rs_x3_b.log
MARF_LIB=$LIB MARF_DIAG_PREC=4433 timeout -k 10 400 python -u tools/seed_sweep.py --seeds 3 --precisions fp32 \
  --perturb $(seq 53 64) --out gpurun_out/r4k/rs_f16s_b.json > gpurun_out/r4k/rs_f16s_b.log 2>&1 || { echo "f16s failed"; tail -3 gpurun_out/r4k/rs_f16s_b.log; exit 1; }
tail -1 gpurun_out/r4k/rs_f16s_b.log
