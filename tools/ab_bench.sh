#!/bin/bash
# A/B several libptyx variants / env settings on bench.py workloads in one GPU session:
#   tools/ab_bench.sh <outdir> "<label>:<config>:<lib path or ->:<env assignments>" ...
# (lib "-" = the in-tree default library; envs space-separated, e.g. "PTYX_S3_HOLD=2 PTYX_S_PSI0=0")
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$1; shift
mkdir -p "$OUT"
for spec in "$@"; do
  IFS=: read -r label cfg lib envs <<< "$spec"
  libenv=""
  [ "$lib" != "-" ] && libenv="PTYX_LIB=$R/$lib"
  steps=5; warm=2
  case "$cfg" in c3|c5) steps=3; warm=1;; c4) steps=1; warm=1;; esac
  env $envs $libenv timeout -k 10 300 python "$R/bench.py" --config "$cfg" --steps $steps --warmup $warm --no-cpu-baseline \
     > "$OUT/$label.json" 2> "$OUT/$label.err" || { echo "variant $label failed rc=$?"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$label.json')); print('$label', d['value'], d['kernels_ms_per_step'])"
done
