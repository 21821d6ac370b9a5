#!/bin/bash
# A/B of the stripe engine's call size (c3 / c5): patterns per engine call set through the
# PTYX_STRIPE_MB capacity (per pattern: (P + P·O [+ P ψ⁰ park]) · 512 KiB of intermediates), with
# the probe-gradient epilogue deferred to the step's last call (PTYX_PREP_DEFER_PROBE) or not
# (--tune s_defer_groups=0).  Small calls keep the live intermediates in the 256 MiB Infinity Cache.
#   tools/gpu_stripe_chunks.sh <tag> <config> <MB list> [extra bench args]
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1; CFG=$2; LIST=$3; shift 3
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R"
for mb in $LIST; do
  PTYX_STRIPE_MB=$mb timeout -k 10 300 python bench.py --config "$CFG" --steps 3 --warmup 1 --no-cpu-baseline "$@" \
    > "$OUT/${CFG}_mb$mb.json" 2> "$OUT/${CFG}_mb$mb.err"
  python -c "import json; d=json.load(open('$OUT/${CFG}_mb$mb.json')); print('$CFG', 'MB', $mb, d['value'], d['roofline']['frac'], d['kernels_ms_per_step'])"
done
