#!/bin/bash
# r06: k_small_prep object rows: every row of a small object, column chunks loaded together — the graph /
# fused-step / small-call tests (bitwise), the c2 default-cadence line three times, a kernel trace.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O="$R/gpurun_out/r06/${1:-u}"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stepgraph.py tests/test_gpu_configs.py -x -v --timeout 180 --timeout-method thread > "$O/tests.log" 2>&1 &&
echo "tests: $(tail -1 "$O/tests.log")" &&
for rep in 1 2 3; do
  for t in "--tune prep_all_rows=0" ""; do
    timeout -k 10 200 python tools/bench_recon.py --ga 1 $t >> "$O/c2.jsonl" 2>> "$O/err.txt" || exit 1
  done
done &&
timeout -k 10 300 python tools/bench_recon.py --ga 1 --pmodes 6 --slices 6 --scan 128 >> "$O/tbl.jsonl" 2>> "$O/err.txt" &&
python -c "
import json
for f in ('c2', 'tbl'):
    for l in open('$O/' + f + '.jsonl'):
        d = json.loads(l); print(f, d['tune'], d['ms_per_optimizer_step'], d['patterns_per_s'])
" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python tools/bench_recon.py --ga 1 > "$O/kt.txt" 2>&1 &&
python tools/trace_gaps.py "$O/kt/kt_kernel_trace.csv" --last 3000 > "$O/gaps.txt" &&
head -6 "$O/gaps.txt"
