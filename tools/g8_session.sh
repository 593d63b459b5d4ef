set -o pipefail
O=gpurun_out/g8
mkdir -p $O
LIBD=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib
for P in fp16x2 bf16x3; do
  MARF_LIB=$LIBD/libmarf_stamps.so timeout -k 10 200 python -u tools/step2_phases.py --precision $P > $O/phases_$P.log 2>&1 || { tail -5 $O/phases_$P.log; exit 1; }
  echo "== $P"; cat $O/phases_$P.log | grep -v Warning | tail -20
done
