#!/bin/bash
set -euo pipefail
tag=$1; shift
O=gpurun_out/$tag
mkdir -p $O
for v in f3ph f3phnp; do
  PTYX_LIB=$PWD/ptyrad_amd/lib/var/libptyx_$v.so timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline \
    > $O/$v.out 2> $O/$v.err
  grep F3PHASES $O/$v.out | head -4
done
bash tools/ab_bench.sh $O "$@"
