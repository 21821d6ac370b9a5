#!/bin/bash
# A/B several libptyx variants on the bench workload in one GPU session:
#   tools/ab_bench.sh <outdir> "<label>:<lib path>:<env assignments>" ...
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$1; shift
mkdir -p "$OUT"
for spec in "$@"; do
  IFS=: read -r label lib envs <<< "$spec"
  env $envs PTYX_LIB="$R/$lib" timeout -k 10 300 python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline \
     > "$OUT/$label.json" 2> "$OUT/$label.err" || { echo "variant $label failed rc=$?"; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/$label.json')); print('$label', d['value'], d['kernels_ms_per_step'])"
done
