// Float scatter-add throughput on gfx950 by atomic scope / form / active CUs (design input for
// the object-gradient accumulation).  Each workgroup (256 threads) adds 128x128 patches (one
// pattern's gradient footprint) at pseudo-random offsets of a 1033x1033 plane.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/atomicbench.hip -o build/atomicbench
//   ./build/atomicbench [patches per WG] [WGs per CU | -n for n WGs in total]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int NX = 1033, NP = 128;

template <int MODE, typename T>
__global__ __launch_bounds__(256) void scatter(T* buf, int patches_per_wg, unsigned seed) {
  unsigned s = seed ^ (blockIdx.x * 2654435761u);
  for (int p = 0; p < patches_per_wg; ++p) {
    s = s * 1664525u + 1013904223u;
    const int cy = (s >> 8) % (NX - NP), cx = (s >> 20) % (NX - NP);
    for (int e = threadIdx.x; e < NP * NP; e += 256) {
      const int y = e / NP, x = e % NP;
      T* q = buf + (size_t)(cy + y) * NX + cx + x;
      const float v = 1e-3f * (float)(e & 7);
      if constexpr (MODE == 0) atomicAdd(q, (T)v);                                        // agent (default)
      if constexpr (MODE == 1) __hip_atomic_fetch_add(q, (T)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if constexpr (MODE == 2) *q += (T)v;                                                // racy plain RMW
      if constexpr (MODE == 3) *q = (T)v;                                                 // plain store
      if constexpr (MODE == 4) __builtin_nontemporal_store((T)v, q);                      // nt store
    }
  }
}

struct Row {
  const char* name;
  int bytes;
};

template <int MODE, typename T>
static void run(const char* name, void* buf, int grid, int ppw, int cu) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float ms = 0;
  for (int rep = 0; rep < 2; ++rep) {
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((scatter<MODE, T>), dim3(grid), dim3(256), 0, 0, (T*)buf, ppw, 7u);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
  }
  const double patches = (double)grid * ppw, bytes = patches * NP * NP * sizeof(T);
  const int cus = grid < cu ? grid : cu;
  std::printf("{\"mode\": \"%s\", \"grid\": %d, \"ms\": %.3f, \"TBps\": %.3f, \"us_per_patch_per_active_CU\": %.2f}\n",
              name, grid, ms, bytes / ms / 1e9, ms * 1e3 * cus / patches);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
}

int main(int argc, char** argv) {
  const int ppw = argc > 1 ? std::atoi(argv[1]) : 32;
  int cu = 0;
  (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
  void* buf;
  if (hipMalloc(&buf, sizeof(double) * NX * NX) != hipSuccess) return 1;
  (void)hipMemset(buf, 0, sizeof(double) * NX * NX);
  const int grids[] = {32, 64, 128, cu, cu * 4};
  for (int grid : grids) {
    run<0, float>("f32 atomicAdd(agent)", buf, grid, ppw, cu);
    run<1, float>("f32 fetch_add(workgroup)", buf, grid, ppw, cu);
    run<0, double>("f64 atomicAdd", buf, grid, ppw, cu);
    run<2, float>("f32 plain RMW (racy)", buf, grid, ppw, cu);
    run<3, float>("f32 plain store", buf, grid, ppw, cu);
    run<4, float>("f32 nt store", buf, grid, ppw, cu);
  }
  return 0;
}
