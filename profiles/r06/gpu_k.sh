#!/bin/bash
# r06 at HEAD: the whole GPU suite, smoke, then every bench line WITH its CPU baseline (c2 default,
# the reference cadence, c3 / c4 / c5).
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O="$R/gpurun_out/r06/${1:-k}"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread > "$O/gpu_tests.log" 2>&1 &&
echo "suite: $(tail -1 "$O/gpu_tests.log")" &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 &&
tail -1 "$O/smoke.log" &&
timeout -k 10 300 python bench.py > "$O/bench_c2.json" 2> "$O/bench_c2.err" &&
timeout -k 10 300 python bench.py --cadence reference --steps 3 --warmup 1 > "$O/bench_refcad.json" 2> "$O/bench_refcad.err" &&
timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 > "$O/bench_c3.json" 2> "$O/bench_c3.err" &&
timeout -k 10 300 python bench.py --config c4 --steps 2 --warmup 1 > "$O/bench_c4.json" 2> "$O/bench_c4.err" &&
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 > "$O/bench_c5.json" 2> "$O/bench_c5.err" &&
python - "$O" <<'PY'
import json, sys
for c in ("c2", "refcad", "c3", "c4", "c5"):
    d = json.loads(open(f"{sys.argv[1]}/bench_{c}.json").read().splitlines()[-1])
    cb = d.get("cpu_baseline") or {}
    print(c, d["value"], d.get("ms_per_optimizer_step"), (d.get("roofline") or {}).get("frac"), cb.get("value"), cb.get("shape"))
PY
