#!/bin/bash
# Whole GPU test suite, then an A/B of bench variants (specs as tools/ab_bench.sh).
set -euo pipefail
tag=$1; shift
O=gpurun_out/$tag
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
bash tools/ab_bench.sh $O "$@"
