// Microbenchmark of the workgroup-resident 2-D FFT (ptyx_fft.hpp) on gfx950.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I ptyrad_amd/csrc tools/fftbench.hip -o build/fftbench
//   ./build/fftbench [iters]
// Each workgroup keeps one 128x128 complex array in LDS and runs `iters` forward+inverse FFT
// pairs on it (no global traffic inside the loop), one workgroup per CU.  Reports ns per FFT
// per CU and the implied chip-wide FFT rate, plus a round-trip error check.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ptyx_fft.hpp"

using namespace ptyx;

template <int N, int NT>
__global__ __launch_bounds__(NT) void fft_loop(const float2* in, float2* out, const float2* twg, int iters) {
  __shared__ float2 s_tw[N];
  __shared__ float2 s_buf[LdsArray<N>::kElems];
  for (int i = threadIdx.x; i < N; i += NT) s_tw[i] = twg[i];
  const LdsArray<N> arr{s_buf};
  const float2* src = in + (size_t)blockIdx.x * N * N;
  for (int e = threadIdx.x; e < N * N; e += NT) arr.st(e / N, e % N, src[e]);
  __syncthreads();
  const float s = 1.0f / (N * N);
  for (int it = 0; it < iters; ++it) {
    fft2d<N, NT, -1, true>(arr, s_tw, [](int, int, float2 v) { return v; }, [](int, int, float2&) { return true; });
    fft2d<N, NT, +1, true>(arr, s_tw, [](int, int, float2 v) { return v; }, [&](int, int, float2& v) {
      v = cscale(v, s);
      return true;
    });
  }
  float2* dst = out + (size_t)blockIdx.x * N * N;
  for (int e = threadIdx.x; e < N * N; e += NT) dst[e] = arr.ld(e / N, e % N);
}

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                               \
    }                                                                         \
  } while (0)

int main(int argc, char** argv) {
  constexpr int N = 128, NT = 1024;
  const int iters = argc > 1 ? std::atoi(argv[1]) : 50;
  int cu = 0;
  CHECK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = cu;
  std::vector<float2> h((size_t)grid * N * N), tw(N);
  for (size_t i = 0; i < h.size(); ++i) h[i] = make_float2(std::sin(0.37 * i), std::cos(0.11 * i));
  for (int m = 0; m < N; ++m) tw[m] = make_float2((float)std::cos(-2 * M_PI * m / N), (float)std::sin(-2 * M_PI * m / N));
  float2 *din, *dout, *dtw;
  CHECK(hipMalloc(&din, h.size() * sizeof(float2)));
  CHECK(hipMalloc(&dout, h.size() * sizeof(float2)));
  CHECK(hipMalloc(&dtw, N * sizeof(float2)));
  CHECK(hipMemcpy(din, h.data(), h.size() * sizeof(float2), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dtw, tw.data(), N * sizeof(float2), hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL((fft_loop<N, NT>), dim3(grid), dim3(NT), 0, 0, din, dout, dtw, 2);   // warm-up
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL((fft_loop<N, NT>), dim3(grid), dim3(NT), 0, 0, din, dout, dtw, iters);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  std::vector<float2> o(h.size());
  CHECK(hipMemcpy(o.data(), dout, o.size() * sizeof(float2), hipMemcpyDeviceToHost));
  double err = 0, ref = 0;
  for (size_t i = 0; i < o.size(); ++i) {
    err += std::pow(o[i].x - h[i].x, 2) + std::pow(o[i].y - h[i].y, 2);
    ref += std::pow(h[i].x, 2) + std::pow(h[i].y, 2);
  }
  const double nfft = 2.0 * iters;
  const double ns_per_fft_cu = ms * 1e6 / nfft;
  std::printf("{\"N\": %d, \"iters\": %d, \"grid\": %d, \"ms\": %.3f, \"ns_per_fft_per_cu\": %.1f, "
              "\"chip_ffts_per_s\": %.4g, \"nominal_tflops\": %.2f, \"roundtrip_rel_err\": %.3g}\n",
              N, iters, grid, ms, ns_per_fft_cu, grid * 1e9 / ns_per_fft_cu,
              grid * 1e9 / ns_per_fft_cu * 5.0 * N * N * std::log2((double)N * N) / 1e12, std::sqrt(err / ref));
  return 0;
}
