#!/bin/bash
# r06: bench lines + rocprofv3 kernel stats + FETCH/WRITE (and L2 hit) PMC passes for c3 / c5 at
# HEAD (the stripe engine's traffic re-taken), then c2 / c4.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
cd "$R"
PROF_EXTRA_PASSES="TCC_HIT_sum+TCC_MISS_sum" timeout -k 10 1000 bash tools/gpu_profile.sh r06/${1:-prof} ${2:-c3 c5}
