#!/bin/bash
# r06 re-entry: targeted split/stepgraph/model tests, the whole GPU suite, smoke and the c2 bench at HEAD.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O="$R/gpurun_out/r06/${1:-d}"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_stepgraph.py tests/test_gpu_model.py -x -v --timeout 180 --timeout-method thread > "$O/targeted.log" 2>&1 &&
echo "targeted: $(tail -1 "$O/targeted.log")" &&
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread > "$O/gpu_tests.log" 2>&1 &&
echo "suite: $(tail -1 "$O/gpu_tests.log")" &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 &&
tail -1 "$O/smoke.log" &&
timeout -k 10 200 python bench.py --no-cpu-baseline > "$O/bench_c2.json" 2> "$O/bench_c2.err" &&
echo "c2: $(cut -c1-300 "$O/bench_c2.json")"
