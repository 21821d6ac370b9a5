#!/bin/bash
# k_fused3 hold-variant parity subset (N = 128 register engine) + A/B benches.
set -euo pipefail
tag=$1; shift
O=gpurun_out/$tag
mkdir -p $O
PTYX_LIB=$PWD/ptyrad_amd/lib/var/libptyx_f3hold.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread -m gpu \
  -k "bench_config or register_engine_ragged or register_engine_is or band_of_tall or c2_full or c2_geometry" \
  > $O/tests_hold.log 2>&1 || { tail -30 $O/tests_hold.log; exit 1; }
tail -3 $O/tests_hold.log
bash tools/ab_bench.sh $O "$@"
