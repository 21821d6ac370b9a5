#!/bin/bash
# Round-4 A/B on one MI355X: gather split (tBL-shaped calls), c2 gather after the split rework,
# recon_step at the reference's default cadence with RCCL collectives captured in the step graphs.
#   tools/gpu_r04_ab.sh <tag>   → gpurun_out/<tag>/
set -o pipefail
T=gpurun_out/${1:-r04ab}
mkdir -p "$T"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_stepgraph.py \
  -q --timeout 200 --timeout-method thread > "$T/tests.txt" 2>&1 || exit 1
for s in -1 1 2 4 8; do
  timeout -k 10 200 python tools/bench_modes.py tbl tbl_p1 tbl_z1 --tune gather_split=$s >> "$T/modes_split.jsonl" 2>> "$T/err.txt" || exit 1
done
timeout -k 10 200 python bench.py --steps 10 --warmup 3 > "$T/bench_c2.json" 2>> "$T/err.txt" || exit 1
timeout -k 10 300 python tools/bench_recon.py --ga 1 --graphs auto > "$T/recon.jsonl" 2>> "$T/err.txt" || exit 1
for m in split whole; do
  for g in on off; do
    timeout -k 10 300 python tools/bench_recon.py --ga 1 --graphs $g --rccl $m >> "$T/recon.jsonl" 2>> "$T/err.txt" || exit 1
  done
done
