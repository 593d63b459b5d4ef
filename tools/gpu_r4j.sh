# emulated-recipe basin sweeps on the one-ulp init draws 25-64 (the draws of profiles/r3k_basin), three
# recipes side by side (three processes on the GPU): the bf16x3 emulation, the fp16 split-weight
# recipe (verdict r3 item 5) and fp32 with bf16-rounded saved tensors (the weight gradients' operands)
set -o pipefail
mkdir -p gpurun_out/r4j
LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_diagrt.so
pids=""
for spec in "x3=2221,2221,2221,2221,2222" "f16s=4433" "save1=00001,0000"; do
  name=${spec%%=*}; code=${spec#*=}
  MARF_LIB=$LIB MARF_DIAG_PREC=$code timeout -k 10 1000 python -u tools/seed_sweep.py --seeds 3 --precisions fp32 \
    --perturb $(seq 25 64) --out gpurun_out/r4j/rs_$name.json > gpurun_out/r4j/rs_$name.log 2>&1 &
  pids="$pids $!"
done
rc=0
for p in $pids; do wait $p || rc=$?; done
for n in x3 f16s save1; do echo "$n: $(tail -1 gpurun_out/r4j/rs_$n.log)"; done
exit $rc
