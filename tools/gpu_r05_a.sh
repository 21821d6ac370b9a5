#!/bin/bash
# Round 5 GPU pass: the whole GPU suite (ingest pad/resample parity, the RCCL-captured step path
# with the per-iteration agreement check, ...), the reference-cadence bench at world size 1
# (collectives forced), the default bench and smoke.
set -o pipefail
O=gpurun_out/r05/${1:-a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests_gpu.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --cadence reference --always-reduce --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_refcad_rccl.json 2> $O/bench_refcad_rccl.err &&
timeout -k 10 300 python -u bench.py --cadence reference --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_refcad.json 2> $O/bench_refcad.err &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_c2.json 2> $O/bench_c2.err &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
