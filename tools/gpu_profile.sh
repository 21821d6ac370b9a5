#!/bin/bash
# rocprofv3 evidence for bench configs at HEAD: a kernel-trace --stats summary of each config's
# bench run, and the FETCH_SIZE / WRITE_SIZE PMC passes (separate runs, MI355X_MICROARCH.md
# "rocprofv3 PMC slots") summarised per kernel by profiles/summarize_pmc.py.
#   tools/gpu_profile.sh <tag> [config ...]        (outputs under gpurun_out/<tag>/)
#   PROF_TESTS=1 also runs the -m gpu suite first; PROF_PMC=0 skips the PMC passes;
#   PROF_EXTRA_PASSES="TCC_HIT_sum+TCC_MISS_sum" adds PMC passes (L2 hit rate per kernel).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-prof}
shift || true
CONFIGS=${*:-c2 c3 c4 c5}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R"
export TMPDIR=/tmp
if [ "${PROF_TESTS:-0}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  echo "tests: $(tail -1 "$OUT/gpu_tests.log")"
fi
for c in $CONFIGS; do
  steps=3; [ "$c" = "c4" ] && steps=2; [ "$c" = "c2" ] && steps=10
  timeout -k 10 400 python bench.py --config "$c" --steps $steps --warmup 1 --no-cpu-baseline \
    > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err"
  echo "bench $c: $(python -c "import json,sys; d=json.load(open('$OUT/bench_$c.json')); print(d['value'], d['roofline']['frac'])")"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$c" -o prof -- \
    python3 "$R/bench.py" --config "$c" --steps $steps --warmup 1 --no-cpu-baseline \
    > "$OUT/bench_${c}_under_rocprof.json" 2> "$OUT/prof_$c.err"
  cp "$(find "$OUT/prof_$c" -name '*kernel_stats.csv' | head -1)" "$OUT/${c}_kernel_stats.csv"
  echo "rocprof $c ok"
  if [ "${PROF_PMC:-1}" = "1" ]; then
    # PROF_EXTRA_PASSES: more passes, counters of one pass joined by '+' (e.g. TCC_HIT_sum+TCC_MISS_sum)
    for pass in FETCH_SIZE WRITE_SIZE ${PROF_EXTRA_PASSES:-}; do
      timeout -k 10 -s KILL 400 rocprofv3 --pmc ${pass//+/ } --output-format csv -d "$OUT/pmc_$c/pass_$pass" -o pmc -- \
        python3 "$R/bench.py" --config "$c" --steps 1 --warmup 0 --no-cpu-baseline \
        > "$OUT/pmc_${c}_$pass.json" 2> "$OUT/pmc_${c}_$pass.err"
    done
    python3 profiles/summarize_pmc.py "$OUT/pmc_$c" "$OUT/pmc_$c.json" > "$OUT/pmc_$c.txt"
    echo "pmc $c ok"
  fi
done
