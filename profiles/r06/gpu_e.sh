#!/bin/bash
# r06: fused optimizer step (PTYX_PREP_FUSED_ADAM, ABI 209) — the step-graph tests first, then the
# reference-cadence lines and the c2 / tBL default-cadence timelines (rocprofv3 kernel trace ->
# tools/trace_gaps.py).
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O="$R/gpurun_out/r06/${1:-e}"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stepgraph.py -x -v --timeout 180 --timeout-method thread > "$O/stepgraph.log" 2>&1 &&
echo "stepgraph: $(tail -1 "$O/stepgraph.log")" &&
for v in "" "--always-reduce"; do
  tag=$(echo "x$v" | tr -d ' -')
  timeout -k 10 300 python bench.py --cadence reference --steps 3 --warmup 1 --no-cpu-baseline $v > "$O/refcad_$tag.json" 2> "$O/refcad_$tag.err" || exit 1
  echo "refcad $v: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['value'], d['ms_per_optimizer_step'])" "$O/refcad_$tag.json")"
done &&
timeout -k 10 300 python tools/bench_recon.py --ga 1 > "$O/recon_c2.jsonl" 2> "$O/err_c2.txt" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_c2" -o kt --output-format csv -- python tools/bench_recon.py --ga 1 > "$O/kt_c2.txt" 2>&1 &&
python tools/trace_gaps.py "$O/kt_c2/kt_kernel_trace.csv" --last 3000 > "$O/gaps_c2.txt" &&
timeout -k 10 300 python tools/bench_recon.py --scan 128 --pmodes 6 --slices 6 --ga 1 > "$O/recon_tbl.jsonl" 2> "$O/err_tbl.txt" &&
echo "c2: $(head -1 "$O/gaps_c2.txt")  $(tail -1 "$O/recon_c2.jsonl" | cut -c1-250)" &&
echo "tbl: $(tail -1 "$O/recon_tbl.jsonl" | cut -c1-250)"
