#!/bin/bash
# Round-4 L2-residency evidence: the hand-off microbenchmark timed and under PMC, then
# the stripe passes' L2 hit rate at c3 / c5 and the c4 refresh (tools/gpu_profile.sh).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT="$R/gpurun_out/${1:-r04l}"
mkdir -p "$OUT"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 tools/l2_handoff > "$OUT/l2_handoff.jsonl"
echo "handoff timed ok"
for pass in FETCH_SIZE WRITE_SIZE+TCC_HIT_sum+TCC_MISS_sum; do
  timeout -k 10 -s KILL 300 rocprofv3 --pmc ${pass//+/ } --output-format csv -d "$OUT/pmc_handoff/pass_$pass" -o pmc -- \
    "$R/tools/l2_handoff" --once > "$OUT/l2_handoff_once_$pass.jsonl" 2> "$OUT/l2_handoff_pmc_$pass.err"
done
echo "handoff pmc ok"
PROF_EXTRA_PASSES="TCC_HIT_sum+TCC_MISS_sum" tools/gpu_profile.sh "${1:-r04l}" c3 c5 c4
