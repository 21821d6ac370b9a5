#!/bin/bash
# r06: rocprofv3 kernel stats of the final HEAD's two bench lines (c2 default cadence, reference
# cadence) — the per-kernel durations behind profiles/r06/head8's JSON lines.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O="$R/gpurun_out/r06/${1:-final_prof}"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/c2" -o kt --output-format csv -- python bench.py --no-cpu-baseline --steps 5 > "$O/c2.json" 2> "$O/c2.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/refcad" -o kt --output-format csv -- python bench.py --cadence reference --no-cpu-baseline --steps 2 --warmup 1 > "$O/refcad.json" 2> "$O/refcad.err" &&
python tools/trace_gaps.py "$O/refcad/kt_kernel_trace.csv" --last 3000 > "$O/gaps_refcad.txt" &&
head -6 "$O/c2/kt_kernel_stats.csv" && head -6 "$O/gaps_refcad.txt"
