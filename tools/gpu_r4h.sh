# hidden-layer weight-gradient stage shape A/B; plain-bf16 step kernels at C3 (pixel-per-wave vs tile)
set -o pipefail
bash tools/ab_r4.sh wh "base=|" "sph64=|libmarf_sph64.so" "nbufh5=|libmarf_nbufh5.so" || exit 1
AB_ARGS="--precision bf16" bash tools/ab_r4.sh pb "tile=|" "step2=MARF_STEP2=1|" || exit 1
AB_ARGS="--precision bf16 --config c5" bash tools/ab_r4.sh c5 "tile=|" || exit 1
