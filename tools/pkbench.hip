// Issue-rate microbenchmark: scalar vs packed f32 VALU on gfx950, 1 or 2 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/pkbench.hip -o build/pkbench && ./build/pkbench
// Each lane runs 8 independent accumulator chains; the loop body is 8 instructions of one kind
// (inline asm, so the compiler cannot fuse or pack them).  Reports shader cycles (s_memtime)
// per wave-instruction for every mode, measured in wave 0 of workgroup 0.
#include <hip/hip_runtime.h>

#include <cstdio>

template <int MODE, int NCH>
__global__ __launch_bounds__(256) void k_issue(float* out, int iters, unsigned long long* cyc) {
  float a[2 * NCH + 4];
#pragma unroll
  for (int i = 0; i < 2 * NCH + 4; ++i) a[i] = threadIdx.x * 1e-3f + i;
  const float b0 = 1.0000001f, b1 = 0.9999999f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if constexpr (MODE == 0) {
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[2 * c]) : "v"(b0), "v"(b1));
      } else if constexpr (MODE == 1) {
        asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(*(double*)&a[2 * c]) : "v"(*(const double*)&a[2 * NCH + 2]), "v"(*(const double*)&a[2 * NCH]));
      } else if constexpr (MODE == 2) {
        asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(*(double*)&a[2 * c]) : "v"(*(const double*)&a[2 * NCH + 2]));
      } else if constexpr (MODE == 3) {
        asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(*(double*)&a[2 * c]) : "v"(*(const double*)&a[2 * NCH + 2]));
      } else if constexpr (MODE == 4) {
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[2 * c]) : "v"(b0));
      } else if constexpr (MODE == 5) {
        asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[2 * c]) : "v"(b0));
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
#pragma unroll
  for (int i = 0; i < 2 * NCH + 4; ++i) s += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) *cyc = t1 - t0;
}

template <int MODE, int NCH = 8>
void run(const char* name, int wg_per_cu, float* out, unsigned long long* dcyc) {
  const int iters = 20000, grid = 256 * wg_per_cu;
  auto kern = k_issue<MODE, NCH>;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, out, 100, dcyc);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, out, iters, dcyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long cyc = 0;
  hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
  const double ninst = (double)NCH * iters;
  printf("%-14s chains %2d waves/SIMD %d: %.2f memtime-cyc/inst/wave, %.3f ms, %.1f Ginst/s chip (wave-instr)\n", name, NCH,
         wg_per_cu, cyc / ninst, ms, ninst * grid * 4 / (ms * 1e-3) / 1e9);
}

int main() {
  float* out;
  unsigned long long* dcyc;
  hipMalloc(&out, 256 * 8 * 256 * sizeof(float));
  hipMalloc(&dcyc, 8);
  for (int w = 1; w <= 2; ++w) {
    run<0>("v_fma_f32", w, out, dcyc);
    run<4>("v_add_f32", w, out, dcyc);
    run<5>("v_mul_f32", w, out, dcyc);
    run<1>("v_pk_fma_f32", w, out, dcyc);
    run<2>("v_pk_add_f32", w, out, dcyc);
    run<3>("v_pk_mul_f32", w, out, dcyc);
    run<0, 24>("v_fma_f32", w, out, dcyc);
    run<4, 24>("v_add_f32", w, out, dcyc);
    run<1, 24>("v_pk_fma_f32", w, out, dcyc);
    run<2, 24>("v_pk_add_f32", w, out, dcyc);
  }
  return 0;
}
