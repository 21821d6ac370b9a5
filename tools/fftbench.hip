// Microbenchmark + check of the workgroup-resident 2-D FFTs (ptyx_fft.hpp) on gfx950.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I ptyrad_amd/csrc tools/fftbench.hip -o build/fftbench
//   ./build/fftbench [iters]
// V0 = Stockham 4-pass fft2d (8 workgroup barriers), V1 = wave-owned fft2d_w (2 barriers).
// Each workgroup keeps one N x N complex array in LDS and runs `iters` forward+inverse pairs
// (no global traffic in the loop), one workgroup per CU.  A single forward transform of each
// variant is checked against a double-precision separable DFT on the host.
#include <hip/hip_runtime.h>

#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ptyx_fft.hpp"

using namespace ptyx;

template <int N, int V>
struct Impl;
template <int N>
struct Impl<N, 0> {
  static constexpr int NT = N == 128 ? 1024 : (N == 64 ? 512 : 256);
  using Arr = LdsArray<N>;
  template <int DIR, class Post>
  __device__ static void fft(const Arr& a, const float2* tw, Post&& post) {
    fft2d<N, NT, DIR, true>(a, tw, [](int, int, float2 v) { return v; }, post);
  }
};
template <int N>
struct Impl<N, 1> {
  static constexpr int NT = WGeom<N>::NT;
  using Arr = LdsArrayW<N>;
  template <int DIR, class Post>
  __device__ static void fft(const Arr& a, const float2* tw, Post&& post) {
    fft2d_w<N, DIR, true>(a, tw, [](int, int, float2 v) { return v; }, post);
  }
};

// V2 / V3: the V0 Stockham transform with 1/2 and 1/4 of the threads (more registers per thread)
template <int N>
struct Impl<N, 2> {
  static constexpr int NT = Impl<N, 0>::NT / 2;
  using Arr = LdsArray<N>;
  template <int DIR, class Post>
  __device__ static void fft(const Arr& a, const float2* tw, Post&& post) {
    fft2d<N, NT, DIR, true>(a, tw, [](int, int, float2 v) { return v; }, post);
  }
};
template <int N>
struct Impl<N, 3> {
  static constexpr int NT = Impl<N, 0>::NT / 4;
  using Arr = LdsArray<N>;
  template <int DIR, class Post>
  __device__ static void fft(const Arr& a, const float2* tw, Post&& post) {
    fft2d<N, NT, DIR, true>(a, tw, [](int, int, float2 v) { return v; }, post);
  }
};

template <int N, int V>
__global__ __launch_bounds__((Impl<N, V>::NT)) void fft_loop(const float2* in, float2* out, const float2* twg,
                                                            int iters, int forward_only) {
  using I = Impl<N, V>;
  constexpr int NT = I::NT;
  __shared__ float2 s_tw[N];
  __shared__ float2 s_buf[I::Arr::kElems];
  for (int i = threadIdx.x; i < N; i += NT) s_tw[i] = twg[i];
  const typename I::Arr arr{s_buf};
  const float2* src = in + (size_t)blockIdx.x * N * N;
  for (int e = threadIdx.x; e < N * N; e += NT) arr.st(e / N, e % N, src[e]);
  __syncthreads();
  const float s = 1.0f / (N * N);
  if (forward_only) {
    I::template fft<-1>(arr, s_tw, [](int, int, float2&) { return true; });
  } else {
    for (int it = 0; it < iters; ++it) {
      I::template fft<-1>(arr, s_tw, [](int, int, float2&) { return true; });
      I::template fft<+1>(arr, s_tw, [&](int, int, float2& v) {
        v = cscale(v, s);
        return true;
      });
    }
  }
  float2* dst = out + (size_t)blockIdx.x * N * N;
  for (int e = threadIdx.x; e < N * N; e += NT) dst[e] = arr.ld(e / N, e % N);
}

#define CHECK(x)                                                                            \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);   \
      return 1;                                                                             \
    }                                                                                       \
  } while (0)

template <int N, int V>
int run(int iters, int grid, const std::vector<float2>& h, float2* din, float2* dout, float2* dtw) {
  using I = Impl<N, V>;
  // correctness: one forward FFT of array 0 vs host double DFT
  hipLaunchKernelGGL((fft_loop<N, V>), dim3(1), dim3(I::NT), 0, 0, din, dout, dtw, 0, 1);
  CHECK(hipDeviceSynchronize());
  std::vector<float2> o((size_t)N * N);
  CHECK(hipMemcpy(o.data(), dout, o.size() * sizeof(float2), hipMemcpyDeviceToHost));
  using C = std::complex<double>;
  std::vector<C> a((size_t)N * N), b((size_t)N * N);
  for (int i = 0; i < N * N; ++i) a[i] = C(h[i].x, h[i].y);
  for (int y = 0; y < N; ++y)
    for (int k = 0; k < N; ++k) {
      C acc = 0;
      for (int x = 0; x < N; ++x) acc += a[y * N + x] * std::polar(1.0, -2 * M_PI * (double)x * k / N);
      b[y * N + k] = acc;
    }
  double err = 0, ref = 0;
  for (int k = 0; k < N; ++k)
    for (int x = 0; x < N; ++x) {
      C acc = 0;
      for (int y = 0; y < N; ++y) acc += b[y * N + x] * std::polar(1.0, -2 * M_PI * (double)y * k / N);
      const C got(o[k * N + x].x, o[k * N + x].y);
      err += std::norm(got - acc);
      ref += std::norm(acc);
    }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((fft_loop<N, V>), dim3(grid), dim3(I::NT), 0, 0, din, dout, dtw, 2, 0);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL((fft_loop<N, V>), dim3(grid), dim3(I::NT), 0, 0, din, dout, dtw, iters, 0);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double ns = ms * 1e6 / (2.0 * iters);
  std::printf("{\"variant\": %d, \"N\": %d, \"NT\": %d, \"iters\": %d, \"grid\": %d, \"ns_per_fft_per_wg\": %.1f, "
              "\"chip_ffts_per_s\": %.4g, \"nominal_tflops\": %.2f, \"fwd_rel_err_vs_fp64\": %.3g}\n",
              V, N, I::NT, iters, grid, ns, grid * 1e9 / ns,
              grid * 1e9 / ns * 5.0 * N * N * std::log2((double)N * N) / 1e12, std::sqrt(err / ref));
  return 0;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 50;
  int cu = 0;
  CHECK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
  int rc = 0;
  auto go = [&](auto nn, int wgs_per_cu) {
    constexpr int N = decltype(nn)::value;
    const int grid = cu * wgs_per_cu;
    std::vector<float2> h((size_t)grid * N * N), tw(N);
    for (size_t i = 0; i < h.size(); ++i) h[i] = make_float2(std::sin(0.37 * i), std::cos(0.11 * i + 0.001 * (i % 977)));
    for (int m = 0; m < N; ++m) tw[m] = make_float2((float)std::cos(-2 * M_PI * m / N), (float)std::sin(-2 * M_PI * m / N));
    float2 *din, *dout, *dtw;
    if (hipMalloc(&din, h.size() * sizeof(float2)) || hipMalloc(&dout, h.size() * sizeof(float2)) ||
        hipMalloc(&dtw, N * sizeof(float2)))
      return 1;
    (void)hipMemcpy(din, h.data(), h.size() * sizeof(float2), hipMemcpyHostToDevice);
    (void)hipMemcpy(dtw, tw.data(), N * sizeof(float2), hipMemcpyHostToDevice);
    rc |= run<N, 0>(iters, grid, h, din, dout, dtw);
    rc |= run<N, 1>(iters, grid, h, din, dout, dtw);
    rc |= run<N, 2>(iters, grid, h, din, dout, dtw);
    rc |= run<N, 3>(iters, grid, h, din, dout, dtw);
    (void)hipFree(din);
    (void)hipFree(dout);
    (void)hipFree(dtw);
    return rc;
  };
  go(std::integral_constant<int, 128>{}, 1);
  go(std::integral_constant<int, 64>{}, 4);
  go(std::integral_constant<int, 32>{}, 8);
  return rc;
}
