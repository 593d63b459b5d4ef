#!/bin/bash
# 3000-step seed sweeps of the C1 run for several library variants (numerics experiments).
#   bash tools/numerics_sweep.sh "<seeds>" <variant>:<precision> ...
# variant "default" = lib/libmarf.so, otherwise lib/libmarf_<variant>.so (build_lib.py --variant).
SEEDS=$1; shift
mkdir -p gpurun_out
for vp in "$@"; do
  v=${vp%%:*}; p=${vp##*:}
  if [ "$v" = default ]; then lib=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf.so
  else lib=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_$v.so; fi
  MARF_LIB=$lib timeout -k 10 900 python -u tools/seed_sweep.py --seeds $SEEDS --precisions $p --perturb ${PERTURB:-0} \
    --out gpurun_out/ns_${v}_$p.json > gpurun_out/ns_${v}_$p.log 2>&1
  rc=$?
  tail -3 gpurun_out/ns_${v}_$p.log
  case $rc in 0) ;; *) echo "variant $v failed ($rc): stopping"; exit $rc;; esac
done
