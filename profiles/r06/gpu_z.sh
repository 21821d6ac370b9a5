#!/bin/bash
# r06: the mixed-state fused gather held to 128 VGPRs (tuning rows_hu 3, k_gather_adam_m4: four
# workgroups a CU) — the bitwise fused-step tests, then the tBL default-cadence line alternating
# rows_hu 3 / default, and a kernel trace of the m4 form.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O="$R/gpurun_out/r06/${1:-z}"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stepgraph.py -x -v --timeout 180 --timeout-method thread -k "fused" > "$O/tests.log" 2>&1 &&
echo "tests: $(tail -1 "$O/tests.log")" &&
for rep in 1 2 3; do
  for t in "--tune rows_hu=3" ""; do
    timeout -k 10 300 python tools/bench_recon.py --ga 1 --pmodes 6 --slices 6 --scan 128 $t >> "$O/ab_tbl.jsonl" 2>> "$O/ab_err.txt" || exit 1
  done
done &&
python -c "
import json
for l in open('$O/ab_tbl.jsonl'):
    d = json.loads(l); print('tbl', d['tune'], d['ms_per_optimizer_step'], d['patterns_per_s'])
" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python tools/bench_recon.py --ga 1 --pmodes 6 --slices 6 --scan 128 --tune rows_hu=3 > "$O/kt.txt" 2>&1 &&
python tools/trace_gaps.py "$O/kt/kt_kernel_trace.csv" --last 3000 > "$O/gaps.txt" &&
head -9 "$O/gaps.txt"
