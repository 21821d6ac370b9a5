#!/bin/bash
# r06: the whole GPU suite at HEAD, smoke, the default c2 bench line and the reference-cadence line
# (with their CPU baselines).
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O="$R/gpurun_out/r06/${1:-h}"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread > "$O/gpu_tests.log" 2>&1 &&
echo "suite: $(tail -1 "$O/gpu_tests.log")" &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 &&
tail -1 "$O/smoke.log" &&
timeout -k 10 300 python bench.py > "$O/bench_c2.json" 2> "$O/bench_c2.err" &&
echo "c2: $(cut -c1-400 "$O/bench_c2.json")" &&
timeout -k 10 300 python bench.py --cadence reference --steps 3 --warmup 1 > "$O/bench_refcad.json" 2> "$O/bench_refcad.err" &&
echo "refcad: $(cut -c1-300 "$O/bench_refcad.json")"
