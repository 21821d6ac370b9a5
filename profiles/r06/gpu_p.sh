#!/bin/bash
# r06: consecutive same-shape optimizer steps replayed as one multi-step graph (StepGraphs.CHUNK) —
# the graph tests (bitwise vs eager / one-step graphs) and the split-path tests, then the c2 and tBL
# default-cadence lines alternating CHUNK 1 / 16, and a kernel trace of the c2 chunked line.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O="$R/gpurun_out/r06/${1:-p}"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_stepgraph.py tests/test_gpu_split.py -x -v --timeout 180 --timeout-method thread > "$O/tests.log" 2>&1 &&
echo "tests: $(tail -1 "$O/tests.log")" &&
for rep in 1 2 3; do
  for c in 1 16; do
    timeout -k 10 200 python tools/bench_recon.py --ga 1 --chunk $c >> "$O/ab_c2.jsonl" 2>> "$O/ab_err.txt" || exit 1
  done
done &&
for c in 1 16; do
  timeout -k 10 300 python tools/bench_recon.py --ga 1 --pmodes 6 --slices 6 --scan 128 --chunk $c >> "$O/ab_tbl.jsonl" 2>> "$O/ab_err.txt" || exit 1
done &&
python -c "
import json
for f in ('ab_c2', 'ab_tbl'):
    for l in open('$O/' + f + '.jsonl'):
        d = json.loads(l); print(f, d['chunk'], d['replays'], d['ms_per_optimizer_step'], d['patterns_per_s'])
" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_chunk" -o kt --output-format csv -- python tools/bench_recon.py --ga 1 > "$O/kt_chunk.txt" 2>&1 &&
python tools/trace_gaps.py "$O/kt_chunk/kt_kernel_trace.csv" --last 3000 > "$O/gaps_chunk.txt" &&
head -8 "$O/gaps_chunk.txt"
