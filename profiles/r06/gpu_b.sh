#!/bin/bash
# r06: slot exchange (ABI 208) — new split tests first, then the whole GPU suite, then the
# reference-cadence bench with no collective / forced collectives (slots, flat) / 8-rank accounting.
set -euo pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
OUT="$R/gpurun_out/r06/b"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 120 --timeout-method thread -k "slot or gloo or rccl" > "$OUT/split_tests.log" 2>&1
echo "split tests: $(tail -1 "$OUT/split_tests.log")"
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
echo "tests ok: $(tail -1 "$OUT/gpu_tests.log")"
for v in "" "--always-reduce" "--always-reduce --flat-exchange" "--always-reduce --geom-world 8" "--always-reduce --flat-exchange --geom-world 8"; do
  tag=$(echo "x$v" | tr -d ' -')
  timeout -k 10 300 python bench.py --cadence reference --steps 3 --warmup 1 --no-cpu-baseline $v > "$OUT/refcad_$tag.json" 2> "$OUT/refcad_$tag.err"
  echo "refcad $v: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(d['value'], d['ms_per_optimizer_step'], d['exchange'])" "$OUT/refcad_$tag.json")"
done
