#!/bin/bash
# N = 256 general-engine check: the parity test of the fused stage chains, the GPU suite, the
# demo geometries (tools/bench_modes.py) and the c3 bench (stripe engine, shares k_probe_spectrum).
#   tools/gpu_check_g256.sh <tag>          (outputs under gpurun_out/<tag>/)
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT="$R/gpurun_out/${1:-g256}"
mkdir -p "$OUT"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k n256 --timeout 240 --timeout-method thread > "$OUT/parity_n256.log" 2>&1
echo "n256 parity: $(tail -1 "$OUT/parity_n256.log")"
timeout -k 10 300 python -u tools/bench_modes.py pso tbl --patterns 2048 --reps 2 > "$OUT/modes.jsonl" 2> "$OUT/modes.err"
cat "$OUT/modes.jsonl"
timeout -k 10 800 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "tests: $(tail -1 "$OUT/gpu_tests.log")"
timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
python -c "import json; d=json.load(open('$OUT/bench_c3.json')); print('c3', d['value'], d['roofline']['frac'])"
