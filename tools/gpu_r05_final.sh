#!/bin/bash
# Round 5, end of round: the whole GPU suite, smoke, the default bench line (with its CPU
# baseline) and a rocprofv3 kernel-trace summary of it, the reference-cadence lines (one rank,
# and with every RCCL collective forced), c4 / c3 / c5 lines, the tBL default-cadence timeline.
#   bash tools/gpu_r05_final.sh <subdir>      (outputs under gpurun_out/r05/<subdir>/)
set -o pipefail
O=gpurun_out/r05/${1:-final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_gpu.txt 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
timeout -k 10 400 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/prof.err &&
timeout -k 10 400 python -u bench.py --cadence reference --steps 5 --warmup 2 > $O/bench_refcad.json 2> $O/bench_refcad.err &&
timeout -k 10 300 python -u bench.py --cadence reference --always-reduce --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_refcad_rccl.json 2> $O/bench_refcad_rccl.err &&
bash tools/gpu_r05_e.sh ${1:-final}/tbl &&
timeout -k 10 400 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err &&
timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err &&
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err
