#!/bin/bash
# Round 5: tBL default-cadence trace, the whole GPU suite, the reference-cadence bench with its
# Adam-inclusive CPU baseline, the default bench and smoke.
set -o pipefail
O=gpurun_out/r05/${1:-g}
mkdir -p $O
bash tools/gpu_r05_e.sh ${1:-g}/trace &&
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests_gpu.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --cadence reference --steps 5 --warmup 2 > $O/bench_refcad.json 2> $O/bench_refcad.err &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
