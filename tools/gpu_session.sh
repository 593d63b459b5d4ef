#!/bin/bash
# One GPU session, steps chosen on the command line (replaces the per-round gpu_r*.sh one-offs):
#   bash tools/gpu_session.sh <tag> <step> [<step> ...]
# steps:
#   tests[=<pytest -k expr>]  the GPU suite (or a -k selection) -> <tag>/gpu_tests.log
#   smoke                     __graft_entry__.smoke()
#   bench                     the default bench line (C3 headline, CPU baseline) -> <tag>/bench.json
#   prof                      rocprofv3 --kernel-trace --stats of a short C3 bench -> <tag>/prof/
#   bits                      tools/make_step2_bits.py -> <tag>/step2_bits.json
#   ab=<v1,v2,...>[@prec]     C3 bench of lib/libmarf_<v>.so variants ("default" = lib/libmarf.so),
#                             alternating twice, in recipe prec (default bf16x3; timing-only variants
#                             ab_*: MARF_AB_TIMING_ONLY=1)
#   envab=VAR:v1,v2[:c1,c3]   C1 / C3 benches with VAR=v1, v2, ... alternating twice (library A/B switches)
#   cfg                       secondary bench lines (tools/bench_configs.sh)
#   pmc=<config>/<precision>  FETCH_SIZE / WRITE_SIZE / matrix-core passes (tools/pmc_traffic.sh)
#   basin=<draws>:<n>=<recipe>;...  seed-3 C1 basin rates over one-ulp init draws (tools/basin_table.py)
#   phases                    step-kernel phase stamps, bf16x3 and fp16x2 (lib/libmarf_stamps.so)
#   c1graph                   C1 eager vs captured iteration, bf16x3 and fp16x2, alternating twice
#   rbits=<v1,v2>[@prec]      a recipe's step bit images per library (tools/recipe_bits.py), compared
# Every GPU step has its own time limit; the session stops at the first failure, abort or timeout.
set -o pipefail
TAG=$1; shift
OUT=$PWD/gpurun_out/$TAG
ROOT=$PWD
LIBD=$ROOT/masking-bundle-adjusting-neural-radiance-fields_amd/lib
mkdir -p $OUT
line() {  # summary of a bench json
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels", {})
r = d.get("roofline") or {}
print("%-22s %.4g px/s  %.3f ms/step  %s %.3f ms  frac %s  kernels/step %.3f ms" % (
    sys.argv[2], d["value"], d["ms_per_step"], r.get("kernel"), r.get("avg_launch_ms", 0), r.get("frac"),
    d.get("kernel_ms_per_step", 0)) + "  " + " ".join("%s=%.3f" % (n, v["avg_ms"] * v["launches_per_step"]) for n, v in
                                                      sorted(k.items(), key=lambda kv: -kv[1]["avg_ms"] * kv[1]["launches_per_step"])[:6]))
PY
}
for step in "$@"; do
  case $step in
    tests|tests=*)
      K=${step#tests}; K=${K#=}
      if [ -n "$K" ]; then SEL=(-k "$K"); else SEL=(); fi
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread "${SEL[@]}" > $OUT/gpu_tests.log 2>&1
      RC=$?; tail -3 $OUT/gpu_tests.log
      [ $RC = 0 ] || { echo "pytest exit $RC: stopping"; exit $RC; } ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
      tail -1 $OUT/smoke.log ;;
    bench)
      timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
      line $OUT/bench.json bench ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
         python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-render --no-alt-recipe > $OUT/prof.log 2>&1) || { echo "rocprof failed"; tail -5 $OUT/prof.log; exit 1; }
      find $OUT/prof -name "*kernel_stats*" | head -3 ;;
    bits)
      timeout -k 10 300 python tools/make_step2_bits.py $OUT/step2_bits.json > $OUT/bits.log 2>&1 || { echo "bits failed"; tail -5 $OUT/bits.log; exit 1; }
      tail -2 $OUT/bits.log ;;
    ab=*)
      # ab=<v1,v2,...>[@<precision>]  (e.g. ab=default,prev@fp16x2: lib/libmarf_prev.so against the default)
      SPEC=${step#ab=}; PR=bf16x3
      if [[ $SPEC == *@* ]]; then PR=${SPEC#*@}; SPEC=${SPEC%@*}; fi
      IFS=, read -ra VS <<< "$SPEC"
      for rep in 1 2; do
        for v in "${VS[@]}"; do
          if [ "$v" = default ]; then L=""; TO=""; else L=$LIBD/libmarf_$v.so; TO=$([[ $v == ab_* ]] && echo 1); fi
          MARF_LIB=$L MARF_AB_TIMING_ONLY=$TO timeout -k 10 200 python bench.py --precision $PR --steps 10 --warmup 2 --no-cpu-baseline --no-render --no-alt-recipe \
            > $OUT/ab_${v}_${PR}_$rep.json 2> $OUT/ab_$v.err || { echo "ab $v failed"; tail -5 $OUT/ab_$v.err; exit 1; }
          line $OUT/ab_${v}_${PR}_$rep.json "$v $PR"
        done
      done ;;
    envab=*)
      # envab=VAR:v1,v2[:c1,c3]  C1 / C3 benches of the product library with VAR=v1, VAR=v2, ...
      # alternating twice (A/B switches of the library read per launch)
      SPEC=${step#envab=}; VAR=${SPEC%%:*}; REST=${SPEC#*:}; VALS=${REST%%:*}; CFGS=c1,c3
      [ "$REST" != "$VALS" ] && CFGS=${REST#*:}
      IFS=, read -ra VS <<< "$VALS"; IFS=, read -ra CS <<< "$CFGS"
      for rep in 1 2; do
        for v in "${VS[@]}"; do
          for c in "${CS[@]}"; do
            if [ $c = c1 ]; then A=(--config c1 --precision bf16x3 --steps 30 --warmup 3); else A=(--config $c --steps 10 --warmup 2); fi
            env $VAR=$v timeout -k 10 200 python bench.py "${A[@]}" --no-cpu-baseline --no-render --no-alt-recipe \
              > $OUT/envab_${c}_$v.json 2> $OUT/envab_${c}_$v.err || { echo "envab $c $v failed"; tail -5 $OUT/envab_${c}_$v.err; exit 1; }
            line $OUT/envab_${c}_$v.json "$c $VAR=$v"
          done
        done
      done ;;
    cfg)
      bash tools/bench_configs.sh $TAG/cfg || exit 1 ;;
    pmc=*)
      C=${step#pmc=}
      bash tools/pmc_traffic.sh $TAG/pmc_${C%/*}_${C#*/} ${C%/*} ${C#*/} || exit 1 ;;
    basin=*)
      # basin=<draws>:<name>=<recipe>[;<name>=<recipe>...]  the seed-3 C1 3000-step run over one-ulp
      # init draws per recipe (tools/basin_table.py; a recipe = precision[:VAR=value,...]) ->
      # <tag>/basin/table.json.  The committed basin table (profiles/basin_table.json) is the
      # merge of these runs: e.g. basin=25-144:fp32=fp32;bf16x3=bf16x3;fp16x2=fp16x2
      SPEC=${step#basin=}; DRAWS=${SPEC%%:*}; IFS=';' read -ra RS <<< "${SPEC#*:}"
      timeout -k 10 ${BASIN_TIMEOUT:-1100} python -u tools/basin_table.py --draws $DRAWS --workers ${BASIN_WORKERS:-4} \
        --chunk ${BASIN_CHUNK:-5} --deadline ${BASIN_DEADLINE:-800} --hard-deadline ${BASIN_HARD:-1000} --out $OUT/basin "${RS[@]}" > $OUT/basin.log 2>&1
      RC=$?; tail -6 $OUT/basin.log
      [ $RC = 0 ] || { echo "basin exit $RC: stopping"; exit $RC; } ;;
    phases)
      # in-kernel phase stamps of the step kernel per recipe (lib/libmarf_stamps.so: build_lib.py --stamps)
      for P in bf16x3 fp16x2; do
        MARF_LIB=$LIBD/libmarf_stamps.so timeout -k 10 200 python -u tools/step2_phases.py --precision $P > $OUT/phases_$P.log 2>&1 \
          || { echo "phases $P failed"; tail -5 $OUT/phases_$P.log; exit 1; }
        grep "tile loop total" $OUT/phases_$P.log
      done ;;
    c1graph)
      # C1 per recipe, eager against the captured iteration (--graph), alternating twice
      for rep in 1 2; do
        for A in "bf16x3" "bf16x3 --graph" "fp16x2" "fp16x2 --graph"; do
          read -ra AA <<< "$A"
          N=c1_${AA[0]}${AA[1]:+_graph}_$rep
          timeout -k 10 200 python bench.py --config c1 --precision ${AA[0]} ${AA[1]} --steps 50 --warmup 5 --no-cpu-baseline --no-render --no-alt-recipe \
            > $OUT/$N.json 2> $OUT/$N.err || { echo "c1 $A failed"; tail -5 $OUT/$N.err; exit 1; }
          line $OUT/$N.json "$N"
        done
      done ;;
    rbits=*)
      # rbits=<v1,v2,...>[@precision]: bit images of a recipe's step per library (tools/recipe_bits.py),
      # compared: identical = the change is bit-neutral for that recipe
      SPEC=${step#rbits=}; PR=fp16x2
      if [[ $SPEC == *@* ]]; then PR=${SPEC#*@}; SPEC=${SPEC%@*}; fi
      IFS=, read -ra VS <<< "$SPEC"
      for v in "${VS[@]}"; do
        if [ "$v" = default ]; then L=""; else L=$LIBD/libmarf_$v.so; fi
        MARF_LIB=$L timeout -k 10 300 python tools/recipe_bits.py --precision $PR $OUT/rbits_${v}_$PR.json > $OUT/rbits_$v.log 2>&1 \
          || { echo "rbits $v failed"; tail -5 $OUT/rbits_$v.log; exit 1; }
      done
      python - $OUT/rbits_*_$PR.json <<'PY'
import json, sys
r = [json.load(open(f)) for f in sys.argv[1:]]
for c in r[0]["cases"]:
    same = all(x["cases"][c]["bits"] == r[0]["cases"][c]["bits"] for x in r)
    print(f"{c:10s} {r[0]['cases'][c]['kernel']:10s} {'identical' if same else 'DIFFER'}")
PY
      ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
