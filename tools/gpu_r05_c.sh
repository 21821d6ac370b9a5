#!/bin/bash
# Round 5: which general-engine sizes fail (no -x), and the 512-thread FFT microbenchmark
# (compiled here on the box: build/ does not travel).
set -o pipefail
O=gpurun_out/r05/${1:-c}
mkdir -p $O build
hipcc --offload-arch=gfx950 -O3 -std=c++17 -I ptyrad_amd/csrc -I tools tools/regfft512bench.hip -o build/regfft512bench > $O/bench_build.txt 2>&1 &&
timeout -k 10 120 ./build/regfft512bench 50 > $O/regfft512bench.jsonl 2>&1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread -k "smooth or golden or maximum_modes or unsupported" > $O/tests_parity.txt 2>&1
exit 0
