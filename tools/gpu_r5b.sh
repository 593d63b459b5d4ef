# upper bound of the weight gradients' bias sums: a timing-only build without them (wrong db)
set -o pipefail
MARF_AB_TIMING_ONLY=1 bash tools/ab_r4.sh nobias "base=|" "nobias=|libmarf_nobias.so" || exit 1
