#!/bin/bash
set -euo pipefail
mkdir -p gpurun_out/r02y
for c in c2 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02y/$c.json 2> gpurun_out/r02y/$c.err
  python -c "import json; d=json.load(open('gpurun_out/r02y/$c.json')); print('$c', d['value'], d['ms_per_step'], d['per_rank_ms'])"
done
