#!/bin/bash
# r06: the split-chain microbenchmark (tools/split_chain_bench.hip) — µs a call with HIP events,
# then the same under rocprofv3 kernel trace for per-kernel durations.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O="$R/gpurun_out/r06/${1:-q}"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 120 tools/split_chain_bench > "$O/split.jsonl" 2> "$O/split_err.txt" &&
cat "$O/split.jsonl" &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt --output-format csv -- tools/split_chain_bench > "$O/kt.txt" 2>&1 &&
cat "$O/kt/kt_kernel_stats.csv"
