// Float scatter-add throughput on gfx950 by atomic scope / form (design input for the object
// gradient accumulation).  Each workgroup (256 threads) adds 128x128 patches (one pattern's
// gradient footprint) at pseudo-random offsets of a 1033x1033 f32 plane pair (8.5 MB total).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/atomicbench.hip -o build/atomicbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int NX = 1033, NP = 128;

template <int MODE>
__global__ __launch_bounds__(256) void scatter(float* buf, int patches_per_wg, unsigned seed) {
  unsigned s = seed ^ (blockIdx.x * 2654435761u);
  for (int p = 0; p < patches_per_wg; ++p) {
    s = s * 1664525u + 1013904223u;
    const int cy = (s >> 8) % (NX - NP), cx = (s >> 20) % (NX - NP);
    for (int e = threadIdx.x; e < NP * NP; e += 256) {
      const int y = e / NP, x = e % NP;
      float* q = buf + (size_t)(cy + y) * NX + cx + x;
      const float v = 1e-3f * (float)(e & 7);
      if constexpr (MODE == 0) atomicAdd(q, v);                                           // agent (default)
      if constexpr (MODE == 1) __hip_atomic_fetch_add(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if constexpr (MODE == 2) *q += v;                                                    // racy plain RMW (reference)
      if constexpr (MODE == 3) __hip_atomic_fetch_add(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
  }
}

int main(int argc, char** argv) {
  const int ppw = argc > 1 ? std::atoi(argv[1]) : 64;
  int cu = 0;
  (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
  const int grid = cu * 4;
  float* buf;
  if (hipMalloc(&buf, sizeof(float) * NX * NX * 2) != hipSuccess) return 1;
  (void)hipMemset(buf, 0, sizeof(float) * NX * NX * 2);
  const char* names[] = {"atomicAdd(agent)", "fetch_add(workgroup)", "plain RMW (racy)", "fetch_add(wavefront)"};
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int mode = 0; mode < 4; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipEventRecord(a);
      switch (mode) {
        case 0: hipLaunchKernelGGL(scatter<0>, dim3(grid), dim3(256), 0, 0, buf, ppw, 7u); break;
        case 1: hipLaunchKernelGGL(scatter<1>, dim3(grid), dim3(256), 0, 0, buf, ppw, 7u); break;
        case 2: hipLaunchKernelGGL(scatter<2>, dim3(grid), dim3(256), 0, 0, buf, ppw, 7u); break;
        case 3: hipLaunchKernelGGL(scatter<3>, dim3(grid), dim3(256), 0, 0, buf, ppw, 7u); break;
      }
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, b);
      const double bytes = (double)grid * ppw * NP * NP * 4;
      if (rep) std::printf("{\"mode\": \"%s\", \"ms\": %.3f, \"added_TBps\": %.3f, \"us_per_patch_per_CU\": %.2f}\n",
                           names[mode], ms, bytes / ms / 1e9, ms * 1e3 * cu / ((double)grid * ppw));
    }
  }
  return 0;
}
