#!/bin/bash
# End-of-round GPU pass: parity suite, smoke(), every bench config (c2 with the CPU baseline),
# a rocprofv3 kernel-trace summary of the c2 bench and PMC passes of the stripe engine.
#   tools/gpu_round_final.sh <tag>        (outputs under gpurun_out/<tag>/)
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-final}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "tests ok: $(tail -1 "$OUT/gpu_tests.log")"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
echo "bench c2 ok"
for c in c5 c3 c2-strong; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err"
  echo "bench $c ok"
done
timeout -k 10 400 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
echo "bench c4 ok"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o prof -- \
  python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_under_rocprof.json" 2> "$OUT/prof.err"
echo "rocprof ok"
for c in c5 c3; do
  bash profiles/collect_pmc.sh "$OUT/pmc_$c" --config $c --patterns 4096 > "$OUT/pmc_$c.log" 2>&1
  python3 profiles/summarize_pmc.py "$OUT/pmc_$c" "$OUT/pmc_$c.json" > "$OUT/pmc_$c.txt"
  echo "$c pmc ok"
done
