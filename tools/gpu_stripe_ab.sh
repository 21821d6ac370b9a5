#!/bin/bash
# Stripe-engine parity subset + c5 / c3 bench lines (tools/gpu_stripe_ab.sh <tag> [ab specs...])
set -euo pipefail
tag=$1; shift
O=gpurun_out/$tag
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -v --timeout 120 \
  --timeout-method thread -m gpu -k "c3 or c5 or stripe or n256 or rank_local" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
bash tools/ab_bench.sh $O "$@"
