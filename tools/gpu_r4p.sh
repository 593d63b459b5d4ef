# layer-0 forward breakdown of k_step2 (MARF_STAMPS_L0 build: per-stage / per-row-tile slots count layer 0 only)
set -o pipefail
mkdir -p gpurun_out/r4p
MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_stampsl0.so timeout -k 10 300 python tools/step2_phases.py --kernel step2 > gpurun_out/r4p/phases_step2_l0.txt 2>&1 || { echo "phases failed"; tail -5 gpurun_out/r4p/phases_step2_l0.txt; exit 1; }
cat gpurun_out/r4p/phases_step2_l0.txt
