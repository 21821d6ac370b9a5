#!/bin/bash
# List the PMC counters of this box, then one pass of VALU-utilisation counters on the c2 bench.
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:-cnt}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*VALU[A-Z_0-9]*\|SQ_[A-Z_0-9]*CYCLES[A-Z_0-9]*\|SQ_INSTS_[A-Z_0-9]*\|SQ_WAIT[A-Z_0-9]*\|SQ_IFETCH[A-Z_0-9]*" $O/counters_list.txt | sort -u > $O/sq_counters.txt || true
cat $O/sq_counters.txt | tr '\n' ' '
echo
for pass in "$@"; do :; done
