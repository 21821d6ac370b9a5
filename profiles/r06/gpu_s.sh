#!/bin/bash
# r06: ψ⁰ held in registers on LARGE calls (tuning psi_hold 2: one k_fused3 workgroup a CU, several
# patterns each) vs the parking kernel at two a CU — parity test, then the c2 bench line alternating
# the two, and the rocprofv3 kernel stats of each.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O="$R/gpurun_out/r06/${1:-s}"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 180 --timeout-method thread -k "psi_hold" > "$O/tests.log" 2>&1 &&
echo "tests: $(tail -1 "$O/tests.log")" &&
for rep in 1 2; do
  for t in "" "--tune psi_hold=2"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline $t >> "$O/ab_c2.jsonl" 2>> "$O/ab_err.txt" || exit 1
  done
done &&
python -c "
import json
for l in open('$O/ab_c2.jsonl'):
    d = json.loads(l); print('c2', d.get('tune'), d['value'], d['ms_per_step'], d['roofline']['frac'])
" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_hold" -o kt --output-format csv -- python bench.py --no-cpu-baseline --steps 5 --tune psi_hold=2 > "$O/kt_hold.txt" 2>&1 &&
head -4 "$O/kt_hold/kt_kernel_stats.csv"
