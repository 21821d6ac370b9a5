#!/bin/bash
# Round 5: the tBL demo's default cadence (scan 128, 6 probe modes, 6 slices, ga = 1) timed by
# bench_recon and traced with rocprofv3 --kernel-trace (timeline summary by tools/trace_gaps.py).
#   bash tools/gpu_r05_e.sh <subdir> [extra bench_recon args ...]
set -o pipefail
O=gpurun_out/r05/${1:-e}
shift
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_recon.py --scan 128 --pmodes 6 --slices 6 --ga 1 "$@" > $O/recon_tbl.jsonl 2> $O/err.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python tools/bench_recon.py --scan 128 --pmodes 6 --slices 6 --ga 1 "$@" > $O/kt.txt 2>&1 &&
python tools/trace_gaps.py $O/kt/kt_kernel_trace.csv --last 3000 > $O/gaps_tbl.txt
