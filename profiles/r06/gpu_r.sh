#!/bin/bash
# r06: k_gather_adam's probe-row / rest blocks dispatched first (tuning gadam_lead) — the bitwise
# fused-step tests, then c2 / tBL default-cadence lines alternating gadam_lead 0 / default, and a
# kernel trace of the c2 line.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O="$R/gpurun_out/r06/${1:-r}"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stepgraph.py -x -v --timeout 180 --timeout-method thread -k "fused" > "$O/tests.log" 2>&1 &&
echo "tests: $(tail -1 "$O/tests.log")" &&
for rep in 1 2 3; do
  for t in "--tune gadam_lead=0" ""; do
    timeout -k 10 200 python tools/bench_recon.py --ga 1 $t >> "$O/ab_c2.jsonl" 2>> "$O/ab_err.txt" || exit 1
  done
done &&
for t in "--tune gadam_lead=0" ""; do
  timeout -k 10 300 python tools/bench_recon.py --ga 1 --pmodes 6 --slices 6 --scan 128 $t >> "$O/ab_tbl.jsonl" 2>> "$O/ab_err.txt" || exit 1
done &&
python -c "
import json
for f in ('ab_c2', 'ab_tbl'):
    for l in open('$O/' + f + '.jsonl'):
        d = json.loads(l); print(f, d['tune'], d['ms_per_optimizer_step'], d['patterns_per_s'])
" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python tools/bench_recon.py --ga 1 > "$O/kt.txt" 2>&1 &&
python tools/trace_gaps.py "$O/kt/kt_kernel_trace.csv" --last 3000 > "$O/gaps.txt" &&
head -8 "$O/gaps.txt"
