// Check + microbenchmark of the 512-thread register-resident 128×128 FFT (tools/ptyx_regfft512.hpp)
// against the 256-thread one the engines use (ptyrad_amd/csrc/ptyx_regfft.hpp).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I ptyrad_amd/csrc -I tools tools/regfft512bench.hip \
//         -o build/regfft512bench
//   ./build/regfft512bench [iters]
// k_check2: forward (R layout in, K layout out) + inverse back, vs a double-precision DFT on the
// host.  k_loop2 / k_loop: `iters` inverse + forward pairs per workgroup, no global traffic inside
// the loop; HOLD keeps 128 more floats a thread live across the loop (the ψ⁰ and probe-gradient
// state a one-pass engine would hold on chip instead of parking it in HBM).  Reported: ns per
// pattern of 4 transforms (the fused chain's FFT count at P = O = Nz = 1) at full occupancy
// (throughput) and for 192 patterns on 256 CUs (latency: the tBL demo's default-cadence step).
#include <hip/hip_runtime.h>

#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ptyx_regfft.hpp"
#include "ptyx_regfft512.hpp"

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e = (x);                                                                 \
    if (e != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)

using namespace ptyx;

__global__ __launch_bounds__(512, 1) void k_check2(const float2* in, float2* out_fwd, float2* out_rt) {
  __shared__ float2 buf[rf2::kLdsElems];
  const rf2::Coord c = rf2::coord(threadIdx.x);
  const size_t base = (size_t)blockIdx.x * 16384;
  float2 v[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) v[j] = in[base + (j + 32 * c.l0 + 64 * c.l1) * 128 + c.fixed];
  rf2::fft_fwd(v, buf, c);
#pragma unroll
  for (int k = 0; k < 32; ++k) out_fwd[base + c.fixed * 128 + 4 * k + 2 * c.l0 + c.l1] = v[k];
  rf2::fft_inv(v, buf, c);
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const float s = 1.0f / 16384.0f;
    out_rt[base + (j + 32 * c.l0 + 64 * c.l1) * 128 + c.fixed] = make_float2(v[j].x * s, v[j].y * s);
  }
}

template <bool HOLD>
__global__ __launch_bounds__(512, 1) void k_loop2(const float2* in, float2* out, int iters) {
  __shared__ float2 buf[rf2::kLdsElems];
  const rf2::Coord c = rf2::coord(threadIdx.x);
  const size_t base = (size_t)blockIdx.x * 16384;
  float2 v[32];
  float2 h[64];
#pragma unroll
  for (int j = 0; j < 32; ++j) v[j] = in[base + j * 512 + threadIdx.x];
#pragma unroll
  for (int j = 0; j < 64; ++j) h[j] = make_float2(0.f, 0.f);
  const float s = 1.0f / 128.0f;
  for (int it = 0; it < iters; ++it) {
    rf2::fft_inv(v, buf, c);
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = make_float2(v[j].x * s, v[j].y * s);
    if constexpr (HOLD) {
#pragma unroll
      for (int j = 0; j < 32; ++j) h[j] = make_float2(h[j].x + v[j].x, h[j].y - v[j].y);
    }
    rf2::fft_fwd(v, buf, c);
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = make_float2(v[j].x * s, v[j].y * s);
    if constexpr (HOLD) {
#pragma unroll
      for (int j = 0; j < 32; ++j) h[32 + j] = make_float2(h[32 + j].x + v[j].y, h[32 + j].y + v[j].x);
    }
  }
#pragma unroll
  for (int j = 0; j < 32; ++j) out[base + j * 512 + threadIdx.x] = v[j];
  if constexpr (HOLD) {
    float2 a = make_float2(0.f, 0.f);
#pragma unroll
    for (int j = 0; j < 64; ++j) a = make_float2(a.x + h[j].x, a.y + h[j].y);
    if (a.x == 12345.f) out[base] = a;
  }
}

__global__ __launch_bounds__(256, 2) void k_loop(const float2* in, float2* out, int iters) {
  __shared__ float2 buf[rf::kLdsElems];
  const int tid = threadIdx.x;
  const rf::Coord c = rf::coord(tid);
  const rf::LaneCtx lc = rf::lane_ctx(c.lane);
  const size_t base = (size_t)blockIdx.x * 16384;
  float2 v[64];
#pragma unroll
  for (int j = 0; j < 64; ++j) v[j] = in[base + j * 256 + tid];
  const float s = 1.0f / 128.0f;
  for (int it = 0; it < iters; ++it) {
    rf::fft_inv(v, buf, lc, c.wsign);
#pragma unroll
    for (int j = 0; j < 64; ++j) v[j] = make_float2(v[j].x * s, v[j].y * s);
    rf::fft_fwd(v, buf, lc, c.wsign);
#pragma unroll
    for (int j = 0; j < 64; ++j) v[j] = make_float2(v[j].x * s, v[j].y * s);
  }
#pragma unroll
  for (int j = 0; j < 64; ++j) out[base + j * 256 + tid] = v[j];
}

static void dft2(const std::vector<std::complex<double>>& a, std::vector<std::complex<double>>& o, int sgn) {
  const int N = 128;
  std::vector<std::complex<double>> t(N * N);
  for (int y = 0; y < N; ++y)
    for (int k = 0; k < N; ++k) {
      std::complex<double> s = 0;
      for (int x = 0; x < N; ++x) s += a[y * N + x] * std::polar(1.0, sgn * 2 * M_PI * x * k / N);
      t[y * N + k] = s;
    }
  for (int k = 0; k < N; ++k)
    for (int ky = 0; ky < N; ++ky) {
      std::complex<double> s = 0;
      for (int y = 0; y < N; ++y) s += t[y * N + k] * std::polar(1.0, sgn * 2 * M_PI * y * ky / N);
      o[ky * N + k] = s;
    }
}

template <class F>
static float time_ms(F&& launch, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 50;
  const int NP = 4096;                       // patterns of the throughput runs
  const size_t n = (size_t)NP * 16384;
  std::vector<float2> h(n);
  srand(1);
  for (size_t i = 0; i < n; ++i) h[i] = make_float2(rand() / (float)RAND_MAX - 0.5f, rand() / (float)RAND_MAX - 0.5f);
  float2 *d_in, *d_a, *d_b;
  CK(hipMalloc(&d_in, n * sizeof(float2)));
  CK(hipMalloc(&d_a, n * sizeof(float2)));
  CK(hipMalloc(&d_b, n * sizeof(float2)));
  CK(hipMemcpy(d_in, h.data(), n * sizeof(float2), hipMemcpyHostToDevice));

  // ---- check: two patterns vs the double-precision DFT
  hipLaunchKernelGGL(k_check2, dim3(2), dim3(512), 0, 0, d_in, d_a, d_b);
  CK(hipDeviceSynchronize());
  std::vector<float2> fw(2 * 16384), rt(2 * 16384);
  CK(hipMemcpy(fw.data(), d_a, fw.size() * sizeof(float2), hipMemcpyDeviceToHost));
  CK(hipMemcpy(rt.data(), d_b, rt.size() * sizeof(float2), hipMemcpyDeviceToHost));
  double emax = 0, rmax = 0, nrm = 0;
  for (int p = 0; p < 2; ++p) {
    std::vector<std::complex<double>> a(16384), o(16384);
    for (int i = 0; i < 16384; ++i) a[i] = {h[p * 16384 + i].x, h[p * 16384 + i].y};
    dft2(a, o, -1);
    for (int i = 0; i < 16384; ++i) {
      const std::complex<double> g(fw[p * 16384 + i].x, fw[p * 16384 + i].y);
      emax = std::max(emax, std::abs(g - o[i]));
      nrm = std::max(nrm, std::abs(o[i]));
      const std::complex<double> r(rt[p * 16384 + i].x, rt[p * 16384 + i].y);
      rmax = std::max(rmax, std::abs(r - a[i]));
    }
  }
  std::printf("{\"check\": {\"fwd_max_err_rel\": %.3e, \"roundtrip_max_err\": %.3e}}\n", emax / nrm, rmax);

  // ---- throughput: NP patterns, every CU full
  const float t256 = time_ms([&] { hipLaunchKernelGGL(k_loop, dim3(NP), dim3(256), 0, 0, d_in, d_a, iters); }, 3);
  const float t512 = time_ms([&] { hipLaunchKernelGGL(k_loop2<false>, dim3(NP), dim3(512), 0, 0, d_in, d_b, iters); }, 3);
  const float t512h = time_ms([&] { hipLaunchKernelGGL(k_loop2<true>, dim3(NP), dim3(512), 0, 0, d_in, d_b, iters); }, 3);
  // ---- latency: 192 patterns (one per CU at most)
  const int NL = 192;
  const float l256 = time_ms([&] { hipLaunchKernelGGL(k_loop, dim3(NL), dim3(256), 0, 0, d_in, d_a, iters); }, 3);
  const float l512 = time_ms([&] { hipLaunchKernelGGL(k_loop2<false>, dim3(NL), dim3(512), 0, 0, d_in, d_b, iters); }, 3);
  const float l512h = time_ms([&] { hipLaunchKernelGGL(k_loop2<true>, dim3(NL), dim3(512), 0, 0, d_in, d_b, iters); }, 3);
  auto per = [&](float ms, int np) { return 1e6 * ms / ((double)np * iters / 2.0); };   // ns per 4 transforms
  std::printf("{\"iters\": %d, \"throughput_ns_per_pattern_4fft\": {\"rf256_2wg\": %.1f, \"rf512\": %.1f, "
              "\"rf512_hold128\": %.1f}, \"latency_us_per_4fft_192_patterns\": {\"rf256\": %.2f, \"rf512\": %.2f, "
              "\"rf512_hold128\": %.2f}}\n",
              iters, per(t256, NP), per(t512, NP), per(t512h, NP), 1e3 * l256 / (iters / 2.0),
              1e3 * l512 / (iters / 2.0), 1e3 * l512h / (iters / 2.0));
  CK(hipFree(d_in));
  CK(hipFree(d_a));
  CK(hipFree(d_b));
  return 0;
}
