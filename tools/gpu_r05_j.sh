#!/bin/bash
# Round 5: c2 at the reference's default cadence (256² scan, ga = 1): bench_recon + kernel trace.
set -o pipefail
O=gpurun_out/r05/${1:-j}
shift
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_recon.py --scan 256 --ga 1 "$@" > $O/recon_c2.jsonl 2> $O/err.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python tools/bench_recon.py --scan 256 --ga 1 "$@" > $O/kt.txt 2>&1 &&
python tools/trace_gaps.py $O/kt/kt_kernel_trace.csv --last 3000 > $O/gaps_c2.txt
