#!/bin/bash
# One GPU-box measurement round: parity tests, bench (with CPU baseline), rocprofv3 kernel trace
# summary and PMC passes.  Every GPU step has its own time limit; the first failure ends the run.
#   tools/gpu_round.sh <tag>        (outputs under gpurun_out/<tag>/)
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-round}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "tests ok"
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench ok"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o prof -- \
  python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_under_rocprof.json" 2> "$OUT/prof.err"
echo "rocprof ok"
bash "$R/profiles/collect_pmc.sh" "$OUT/pmc" > "$OUT/pmc.log" 2>&1
python3 "$R/profiles/summarize_pmc.py" "$OUT/pmc" "$OUT/pmc_c2.json" > "$OUT/pmc_summary.txt"
echo "pmc ok"
