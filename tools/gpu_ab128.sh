#!/bin/bash
# N = 128 register-engine parity subset, then an A/B of bench variants.
set -euo pipefail
tag=$1; shift
O=gpurun_out/$tag
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py -x -v \
  --timeout 300 --timeout-method thread -m gpu -k "register or multislice or c2_ or bench_config or c1_shape or resume" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
bash tools/ab_bench.sh $O "$@"
