#!/bin/bash
# PMC counter passes (one counter group per rocprofv3 run; FETCH_SIZE and WRITE_SIZE in separate
# passes, MI355X_MICROARCH.md "rocprofv3 PMC slots").  Run on the GPU box:
#   bash profiles/collect_pmc.sh <outdir> [extra bench args, e.g. --config c5]
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-$R/gpurun_out/pmc}
shift || true
mkdir -p "$OUT"
OUT=$(cd "$OUT" && pwd)
export TMPDIR=/tmp
SCRIPT=bench.py
EXTRA="--no-cpu-baseline"
cd /tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
for pass in "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES" \
            "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" \
            "TCC_HIT_sum TCC_MISS_sum" \
            "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d "$OUT/pass$i" -o pmc -- \
    python3 "$R/$SCRIPT" --steps 1 --warmup 1 $EXTRA "$@" > "$OUT/pass$i.json" 2> "$OUT/pass$i.err"
done
echo "pmc passes done: $i"
