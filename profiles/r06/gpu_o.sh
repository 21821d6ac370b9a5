#!/bin/bash
# r06: k_fused3 with ψ⁰ held in registers for small calls (tuning psi_hold 1) — the bitwise test,
# then the c2 default-cadence line alternating the variants, three rounds, and a kernel trace of each.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O="$R/gpurun_out/r06/${1:-o}"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 180 --timeout-method thread -k "psi_hold or small_call" > "$O/tests.log" 2>&1 &&
echo "tests: $(tail -1 "$O/tests.log")" &&
for rep in 1 2 3; do
  for t in "" "--tune psi_hold=1"; do
    timeout -k 10 200 python tools/bench_recon.py --ga 1 $t >> "$O/ab_c2.jsonl" 2>> "$O/ab_err.txt" || exit 1
  done
done &&
python -c "
import json
for l in open('$O/ab_c2.jsonl'):
    d = json.loads(l); print('c2', d['tune'], d['ms_per_optimizer_step'], d['patterns_per_s'])
" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_hold" -o kt --output-format csv -- python tools/bench_recon.py --ga 1 --tune psi_hold=1 > "$O/kt_hold.txt" 2>&1 &&
python tools/trace_gaps.py "$O/kt_hold/kt_kernel_trace.csv" --last 3000 > "$O/gaps_hold.txt" &&
head -8 "$O/gaps_hold.txt"
