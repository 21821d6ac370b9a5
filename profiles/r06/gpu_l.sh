#!/bin/bash
# r06: the fused mixed-state step with two hits in flight a wave (tuning rows_hu 2) — the step-graph
# tests, then tBL (and c2) lines alternating the variants, three rounds.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O="$R/gpurun_out/r06/${1:-l}"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stepgraph.py -x -v --timeout 180 --timeout-method thread > "$O/stepgraph.log" 2>&1 &&
echo "stepgraph: $(tail -1 "$O/stepgraph.log")" &&
for rep in 1 2 3; do
  for t in "" "--tune rows_hu=2"; do
    timeout -k 10 200 python tools/bench_recon.py --scan 128 --pmodes 6 --slices 6 --ga 1 $t >> "$O/ab_tbl.jsonl" 2>> "$O/ab_err.txt" || exit 1
  done
done &&
python -c "
import json
for l in open('$O/ab_tbl.jsonl'):
    d = json.loads(l); print('tbl', d['tune'], d['ms_per_optimizer_step'], d['patterns_per_s'])
"
timeout -k 10 300 python bench.py --cadence reference --steps 2 --warmup 1 --no-cpu-baseline --always-reduce > "$O/refcad_ar.json" 2> "$O/refcad_ar.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_ar" -o kt --output-format csv -- python bench.py --cadence reference --steps 2 --warmup 1 --no-cpu-baseline --always-reduce > "$O/kt_ar.txt" 2>&1 &&
python tools/trace_gaps.py "$O/kt_ar/kt_kernel_trace.csv" --last 3000 > "$O/gaps_ar.txt" &&
echo "always-reduce: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['value'], d['ms_per_optimizer_step'])" "$O/refcad_ar.json")" &&
head -20 "$O/gaps_ar.txt"
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 180 --timeout-method thread -k "slot or rccl" > "$O/split.log" 2>&1 &&
echo "split: $(tail -1 "$O/split.log")"
