#!/bin/bash
# r06: the one-plane row form of k_gather_adam held to 96 VGPRs (tuning gather_rows 3, k_gather_adam_r5, 20 B of spill:
# one-plane row tiles; unfused k_obj_gather_rows) — the bitwise fused-step tests, then the c2
# default-cadence line alternating gather_rows 3 / default (2), and a kernel trace of the r5 form.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O="$R/gpurun_out/r06/${1:-y}"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stepgraph.py -x -v --timeout 180 --timeout-method thread -k "fused" > "$O/tests.log" 2>&1 &&
echo "tests: $(tail -1 "$O/tests.log")" &&
for rep in 1 2 3; do
  for t in "--tune gather_rows=3" ""; do
    timeout -k 10 200 python tools/bench_recon.py --ga 1 $t >> "$O/ab_c2.jsonl" 2>> "$O/ab_err.txt" || exit 1
  done
done &&
python -c "
import json
for l in open('$O/ab_c2.jsonl'):
    d = json.loads(l); print('c2', d['tune'], d['ms_per_optimizer_step'], d['patterns_per_s'])
" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- python tools/bench_recon.py --ga 1 --tune gather_rows=3 > "$O/kt.txt" 2>&1 &&
python tools/trace_gaps.py "$O/kt/kt_kernel_trace.csv" --last 3000 > "$O/gaps.txt" &&
head -6 "$O/gaps.txt"
