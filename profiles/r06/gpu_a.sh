#!/bin/bash
# r06 first pass: GPU suite at HEAD, smoke, c2 bench, reference cadence, the launcher's refusal
# of --gpus 2 on a one-GPU lease.
set -euo pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
OUT="$R/gpurun_out/r06/a"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "tests ok: $(tail -1 "$OUT/gpu_tests.log")"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
echo "bench c2 ok"
timeout -k 10 300 python bench.py --cadence reference --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_refcad.json" 2> "$OUT/bench_refcad.err"
echo "bench refcad ok"
rc=0
timeout -k 10 120 python bench.py --gpus 2 --steps 1 > "$OUT/bench_gpus2.json" 2> "$OUT/bench_gpus2.err" || rc=$?
echo "bench --gpus 2 on one GPU: exit $rc, stdout bytes $(wc -c < "$OUT/bench_gpus2.json")"
