#!/bin/bash
# rocprofv3 evidence for the demo geometries of tools/bench_modes.py (engine only): the bench line,
# a kernel-trace --stats summary of the same command and FETCH_SIZE / WRITE_SIZE PMC passes.
#   tools/gpu_profile_modes.sh <tag> [geometry ...]        (outputs under gpurun_out/<tag>/)
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-prof}
shift || true
GEOMS=${*:-tbl}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R"
export TMPDIR=/tmp
for g in $GEOMS; do
  timeout -k 10 300 python tools/bench_modes.py "$g" > "$OUT/modes_$g.jsonl" 2> "$OUT/modes_$g.err"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$g" -o prof -- \
    python3 "$R/tools/bench_modes.py" "$g" > "$OUT/modes_${g}_under_rocprof.jsonl" 2> "$OUT/prof_$g.err"
  cp "$(find "$OUT/prof_$g" -name '*kernel_stats.csv' | head -1)" "$OUT/${g}_kernel_stats.csv"
  echo "rocprof $g ok"
  for pass in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 -s KILL 300 rocprofv3 --pmc $pass --output-format csv -d "$OUT/pmc_$g/pass_$pass" -o pmc -- \
      python3 "$R/tools/bench_modes.py" "$g" --reps 1 > "$OUT/pmc_${g}_$pass.jsonl" 2> "$OUT/pmc_${g}_$pass.err"
  done
  python3 profiles/summarize_pmc.py "$OUT/pmc_$g" "$OUT/pmc_$g.json" > "$OUT/pmc_$g.txt"
  echo "pmc $g ok"
done
