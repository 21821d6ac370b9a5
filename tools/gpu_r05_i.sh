#!/bin/bash
# Round 5: kernel trace of loss_simlar beside the engine call (128² scan, 2 object modes, ga 16).
set -o pipefail
O=gpurun_out/r05/${1:-i}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python tools/bench_recon.py --scan 128 --omodes 2 --ga 16 --simlar call > $O/kt.txt 2>&1 &&
python tools/trace_gaps.py $O/kt/kt_kernel_trace.csv --last 3000 > $O/gaps.txt
