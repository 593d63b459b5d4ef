set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-stamps d_nodma d_nostore d_nobar d_bare}; do
  echo "== $v" >> gpurun_out/diag.log
  timeout -k 10 120 env MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_$v.so python tools/step2_phases.py --precision bf16x3 >> gpurun_out/diag.log 2>&1 || { echo "fail $v"; exit 1; }
done
