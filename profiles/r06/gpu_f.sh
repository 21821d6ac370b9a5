#!/bin/bash
# r06: k_finalize folded into the small calls' tail (tail_fin) and the small calls' probe spectrum
# in k_small_prep (small_spec) — the new tests, then A/B lines at the default cadence (c2, tBL),
# then the c2 / tBL timelines.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O="$R/gpurun_out/r06/${1:-f}"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stepgraph.py tests/test_gpu_configs.py -x -v --timeout 180 --timeout-method thread -k "stepgraph or small_call or gather_rows or fused" > "$O/targeted.log" 2>&1 &&
echo "targeted: $(tail -1 "$O/targeted.log")" &&
for t in "" "--tune tail_fin=0" "--tune small_spec=0" "--tune tail_fin=0 --tune small_spec=0 --tune fuse_adam=0"; do
  timeout -k 10 200 python tools/bench_recon.py --ga 1 $t >> "$O/ab_c2.jsonl" 2>> "$O/ab_err.txt" || exit 1
  timeout -k 10 200 python tools/bench_recon.py --scan 128 --pmodes 6 --slices 6 --ga 1 $t >> "$O/ab_tbl.jsonl" 2>> "$O/ab_err.txt" || exit 1
done &&
python -c "
import json
for f in ('ab_c2', 'ab_tbl'):
    for l in open('$O/' + f + '.jsonl'):
        d = json.loads(l); print(f, d['tune'], d['ms_per_optimizer_step'], d['patterns_per_s'])
" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_c2" -o kt --output-format csv -- python tools/bench_recon.py --ga 1 > "$O/kt_c2.txt" 2>&1 &&
python tools/trace_gaps.py "$O/kt_c2/kt_kernel_trace.csv" --last 3000 > "$O/gaps_c2.txt" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_tbl" -o kt --output-format csv -- python tools/bench_recon.py --scan 128 --pmodes 6 --slices 6 --ga 1 > "$O/kt_tbl.txt" 2>&1 &&
python tools/trace_gaps.py "$O/kt_tbl/kt_kernel_trace.csv" --last 3000 > "$O/gaps_tbl.txt" &&
head -12 "$O/gaps_c2.txt" && head -14 "$O/gaps_tbl.txt"
