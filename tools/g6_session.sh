set -o pipefail
O=gpurun_out/g6
mkdir -p $O
LIBD=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib
# emulated candidate recipes: E3 = every operand fp16 (weights hi + lo, activations, dz; the saved
# tensors fp16), E2 = the fp16x2 forward with the hidden dgrad's dz split (dz_1 bf16)
timeout -k 10 1130 python -u tools/basin_table.py --draws 0,25-84 --workers 6 --chunk 5 --deadline 840 --hard-deadline 1080 \
  --out $O/basin "e3=fp32:MARF_LIB=$LIBD/libmarf_rtg.so,MARF_DIAG_PREC=4433,4433,4433,4433,4434" \
  "e2=fp32:MARF_LIB=$LIBD/libmarf_rtg.so,MARF_DIAG_PREC=42311,4232,4232,4232,4232" > $O/basin.log 2>&1; rc=$?
tail -4 $O/basin.log; exit $rc
