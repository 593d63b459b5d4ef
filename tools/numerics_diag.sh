#!/bin/bash
# fp32 3000-step C1 runs with one class of values rounded to a lower precision (diagnostic builds
# lib/libmarf_diag_<V>.so = build_lib.py --stamps with MARF_LIB_NAME / MARF_EXTRA_FLAGS=-DMARF_DIAG_<V>):
# which rounding costs PSNR?    bash tools/numerics_diag.sh V1 V2 ...
for v in "$@"; do
  echo "== $v"
  MARF_LIB=$PWD/masking-bundle-adjusting-neural-radiance-fields_amd/lib/libmarf_diag_$v.so timeout -k 10 300 \
    python -u -m pytest tests/test_gpu_parity.py -q -s -k "3000 and fp32 and not tail" -p no:cacheprovider > gpurun_out/nd_$v.log 2>&1
  grep -E "final PSNR|every" gpurun_out/nd_$v.log
done
exit 0
