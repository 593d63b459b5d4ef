# phase stamps of both split step kernels at C3 (layer-0 forward stamped on its own in k_step2)
set -o pipefail
mkdir -p gpurun_out/r4n
for k in step2 step3; do
  MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_stamps.so timeout -k 10 300 python tools/step2_phases.py --kernel $k > gpurun_out/r4n/phases_$k.txt 2>&1 || { echo "phases $k failed"; tail -5 gpurun_out/r4n/phases_$k.txt; exit 1; }
done
cat gpurun_out/r4n/phases_step2.txt
