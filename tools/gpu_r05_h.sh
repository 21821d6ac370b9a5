#!/bin/bash
# Round 5: loss_simlar beside the engine call vs per mini-batch (A/B), 128² scan, 2 object modes.
set -o pipefail
O=gpurun_out/r05/${1:-h}
mkdir -p $O
for m in off call batch; do
  timeout -k 10 300 python tools/bench_recon.py --scan 128 --omodes 2 --ga 1 16 --simlar $m >> $O/simlar.jsonl 2>> $O/err.txt || exit 1
done
