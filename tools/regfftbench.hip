// Check + microbenchmark of the register-resident 128x128 FFT (ptyrad_amd/csrc/ptyx_regfft.hpp).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I ptyrad_amd/csrc tools/regfftbench.hip -o build/regfftbench
//   ./build/regfftbench [iters]
// k_check: one forward transform (R layout in, K layout out) + the inverse back, compared with a
// double-precision separable DFT on the host.  k_loop: `iters` inverse+forward pairs per
// workgroup with no global traffic inside the loop, 2 workgroups per CU; reports the time per
// "pattern" of 4 transforms (the fused forward/adjoint chain's FFT count at P = O = Nz = 1).
#include <hip/hip_runtime.h>

#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ptyx_regfft.hpp"

using namespace ptyx::rf;

__global__ __launch_bounds__(256, 2) void k_check(const float2* in, float2* out_fwd, float2* out_rt) {
  __shared__ float2 buf[kLdsElems];
  const int tid = threadIdx.x;
  const Coord c = coord(tid);
  const LaneCtx lc = lane_ctx(c.lane);
  const size_t base = (size_t)blockIdx.x * 16384;
  float2 v[64];
#pragma unroll
  for (int j = 0; j < 64; ++j) v[j] = in[base + (j + 64 * c.l0) * 128 + c.fixed];
  fft_fwd(v, buf, lc, c.wsign);
#pragma unroll
  for (int k = 0; k < 64; ++k) out_fwd[base + c.fixed * 128 + k + 64 * c.l0] = v[k];
  fft_inv(v, buf, lc, c.wsign);
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    const float s = 1.0f / 16384.0f;
    out_rt[base + (j + 64 * c.l0) * 128 + c.fixed] = make_float2(v[j].x * s, v[j].y * s);
  }
}

__global__ __launch_bounds__(256, 2) void k_loop(const float2* in, float2* out, int iters) {
  __shared__ float2 buf[kLdsElems];
  const int tid = threadIdx.x;
  const Coord c = coord(tid);
  const LaneCtx lc = lane_ctx(c.lane);
  const size_t base = (size_t)blockIdx.x * 16384;
  float2 v[64];
#pragma unroll
  for (int j = 0; j < 64; ++j) v[j] = in[base + j * 256 + tid];
  const float s = 1.0f / 128.0f;
  for (int it = 0; it < iters; ++it) {
    fft_inv(v, buf, lc, c.wsign);
#pragma unroll
    for (int j = 0; j < 64; ++j) v[j] = make_float2(v[j].x * s, v[j].y * s);
    fft_fwd(v, buf, lc, c.wsign);
#pragma unroll
    for (int j = 0; j < 64; ++j) v[j] = make_float2(v[j].x * s, v[j].y * s);
  }
#pragma unroll
  for (int j = 0; j < 64; ++j) out[base + j * 256 + tid] = v[j];
}

#define CHECK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                           \
    }                                                                                     \
  } while (0)

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 64;
  int cu = 0;
  CHECK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
  int occ = 0;
  CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_loop, 256, 0));
  const int wpc = argc > 2 ? std::atoi(argv[2]) : 2;   // workgroups per CU (1: one wave per SIMD)
  const int grid = cu * wpc;
  constexpr int N = 128;
  std::vector<float2> h((size_t)grid * N * N);
  for (size_t i = 0; i < h.size(); ++i)
    h[i] = make_float2((float)std::sin(0.37 * i), (float)std::cos(0.11 * i + 0.001 * (i % 977)));
  float2 *din, *dout, *drt;
  CHECK(hipMalloc(&din, h.size() * sizeof(float2)));
  CHECK(hipMalloc(&dout, h.size() * sizeof(float2)));
  CHECK(hipMalloc(&drt, h.size() * sizeof(float2)));
  CHECK(hipMemcpy(din, h.data(), h.size() * sizeof(float2), hipMemcpyHostToDevice));

  // ---- correctness (workgroup 0 and 1)
  hipLaunchKernelGGL(k_check, dim3(2), dim3(256), 0, 0, din, dout, drt);
  CHECK(hipDeviceSynchronize());
  std::vector<float2> o(2 * N * N), rt(2 * N * N);
  CHECK(hipMemcpy(o.data(), dout, o.size() * sizeof(float2), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(rt.data(), drt, rt.size() * sizeof(float2), hipMemcpyDeviceToHost));
  using C = std::complex<double>;
  double worst = 0, worst_rt = 0;
  for (int w = 0; w < 2; ++w) {
    std::vector<C> a(N * N), b(N * N);
    for (int i = 0; i < N * N; ++i) a[i] = C(h[w * N * N + i].x, h[w * N * N + i].y);
    for (int y = 0; y < N; ++y)
      for (int k = 0; k < N; ++k) {
        C acc = 0;
        for (int x = 0; x < N; ++x) acc += a[y * N + x] * std::polar(1.0, -2 * M_PI * (double)x * k / N);
        b[y * N + k] = acc;
      }
    double err = 0, ref = 0, e2 = 0, r2 = 0;
    for (int k = 0; k < N; ++k)
      for (int x = 0; x < N; ++x) {
        C acc = 0;
        for (int y = 0; y < N; ++y) acc += b[y * N + x] * std::polar(1.0, -2 * M_PI * (double)y * k / N);
        const C got(o[w * N * N + k * N + x].x, o[w * N * N + k * N + x].y);
        err += std::norm(got - acc);
        ref += std::norm(acc);
      }
    for (int i = 0; i < N * N; ++i) {
      const C got(rt[w * N * N + i].x, rt[w * N * N + i].y);
      e2 += std::norm(got - a[i]);
      r2 += std::norm(a[i]);
    }
    worst = std::max(worst, std::sqrt(err / ref));
    worst_rt = std::max(worst_rt, std::sqrt(e2 / r2));
  }

  // ---- throughput
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_loop, dim3(grid), dim3(256), 0, 0, din, dout, 4);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_loop, dim3(grid), dim3(256), 0, 0, din, dout, iters);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double ffts = 2.0 * iters * grid;
  const double pat_per_s = ffts / 4.0 / (ms * 1e-3);
  std::printf("{\"occupancy_wg_per_cu\": %d, \"grid\": %d, \"iters\": %d, \"ms\": %.3f, \"us_per_fft_per_wg\": %.3f, "
              "\"chip_ffts_per_s\": %.4g, \"nominal_tflops\": %.2f, \"patterns_per_s_at_4fft\": %.4g, "
              "\"c2_step_ms_fft_only\": %.3f, \"fwd_rel_err_vs_fp64\": %.3g, \"roundtrip_rel_err\": %.3g}\n",
              occ, grid, iters, ms, ms * 1e3 / (2.0 * iters), ffts / (ms * 1e-3),
              ffts / (ms * 1e-3) * 5.0 * N * N * std::log2((double)N * N) / 1e12, pat_per_s, 65536.0 / pat_per_s * 1e3,
              worst, worst_rt);
  return (worst < 1e-5 && worst_rt < 1e-5) ? 0 : 2;
}
