// Device-only compile unit for the k_fused3 engine (fast register/spill iteration):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -I include -I ptyrad_amd/csrc \
//         tools/f3_isa.hip --cuda-device-only -c -o /tmp/f3.o -Rpass-analysis=kernel-resource-usage
#include "ptyx_fused3.hpp"
template __global__ void ptyx::f3::k_fused3<true, true, 0>(ptyx::f3::F3Args);
