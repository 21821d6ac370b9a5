#!/bin/bash
# Full GPU parity suite, then c4 / c2 bench lines (tools/gpu_tests_c4.sh <tag>)
set -euo pipefail
tag=$1
O=gpurun_out/$tag
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash tools/ab_bench.sh $O c4:c4:-: c2:c2:-:
