#!/bin/bash
# Round 5: gather_rows A/B on the big-call gathers (c2, c4) + the variant's parity test.
set -o pipefail
O=gpurun_out/r05/${1:-k}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_optim.py tests/test_gpu_stepgraph.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 &&
for t in -1 1; do
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --tune gather_rows=$t >> $O/bench_c2.jsonl 2>> $O/err.txt || exit 1
done &&
for t in -1 1; do
  timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --tune gather_rows=$t >> $O/bench_c4.jsonl 2>> $O/err.txt || exit 1
done
