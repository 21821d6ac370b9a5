// split_chain_bench.hip — how fast can ONE small call's transform chain go if each pattern's chain
// is spread over W workgroups instead of one?
//
// A default-cadence step (c2, grad_accumulation 1) runs k_fused3 on 32 patterns: 32 workgroups on
// 32 of 256 CUs, each a serial chain of four 128² transforms with point-wise work between them
// (ψ⁰ = F⁻¹(F(P)W); ψ⁰·O → F; g_Ψ → F⁻¹; ×conj(O) → F).  This program times that chain shape alone:
//   reg      — the production register engine's transform (ptyx_regfft.hpp), one workgroup a pattern;
//   lds W=1  — the LDS line-pass transform (ptyx_fft.hpp line_pass), one workgroup a pattern;
//   lds W=2/4/8 — the same line passes with each pattern's lines dealt to W workgroups (128/W rows
//              or columns each, all W on one XCD), one global exchange + a per-pattern arrival
//              counter per transform (consecutive transforms alternate the pass order, so a chain
//              of four needs four exchanges, not eight).  Two exchange forms: "agent" (the memory
//              model's agent-scope release / acquire: an L2 write-back per wave) and "xcd" (stores
//              acknowledged, then the readers' L1 invalidated: enough when one L2 holds the pattern);
//              A third, "xcd_flags", keeps the arrival counter in that L2 as well (workgroup-scope
//              atomics and polls) and invalidates only L1 on the acquire side;
//   meet_only   — the four exchanges alone, nothing transformed (their sync cost).
// Every variant multiplies by a point-wise factor between transforms (the object / loss stand-ins,
// read from global memory like the real ones).  The split variants are bitwise the W = 1 result
// (the same line passes in the same order), which checks the exchange.  Output: one JSON line per
// variant (µs a launch, HIP events over 200 launches).  Build: tools/build_split_chain.sh.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../ptyrad_amd/csrc/ptyx_fft.hpp"
#include "../ptyrad_amd/csrc/ptyx_regfft.hpp"

using namespace ptyx;
constexpr int N = 128, N2 = N * N, kPat = 32, kLaunches = 200, kWarm = 20;

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

// the W workgroups of a pattern meet here: every wave's stores made visible at agent scope, one
// arrival each, a bounded wait (an exit every wave reaches: after 2^20 polls it counts an error
// and goes on), then acquire
__device__ __forceinline__ void pattern_barrier(int* c, int target, int* err) {
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(c, 1);
    int it = 0;
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (++it > (1 << 20)) {
        atomicAdd(err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  __threadfence();
}

// XCD-local form (all W workgroups of a pattern on one XCD, which shares one L2): no L2 write-back
// on the release side — each wave waits for its stores to be acknowledged (L1 writes through to
// L2), and the acquire invalidates the readers' L1.  Valid only under that placement; the bitwise
// check against W = 1 is what tells.
__device__ __forceinline__ void pattern_barrier_xcd(int* c, int target, int* err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(c, 1);
    int it = 0;
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (++it > (1 << 20)) {
        atomicAdd(err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// XCD-local with one flag a workgroup instead of a shared counter (no serialised atomics): each
// workgroup stores its epoch to its own flag (agent-scope relaxed store after its data stores are
// acknowledged), threads 0 … W−1 each poll one flag, then the readers' L1 is invalidated.
// (A first form kept the counter in L2 with workgroup-scope atomics and polls: the polls hit the
// poller's own L1 and never saw the other arrivals — barrier time-outs — and is gone.)
__device__ __forceinline__ void pattern_barrier_flags(int* flags, int W, int target, int* err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int sub = (int)(blockIdx.x >> 3) % W;
  if (threadIdx.x == 0) __hip_atomic_store(flags + sub, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((int)threadIdx.x < W) {
    int it = 0;
    while (__hip_atomic_load(flags + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (++it > (1 << 20)) {
        atomicAdd(err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// c: the pattern's counter (modes 0, 1) or its 8 flags (mode 2); target: arrivals (modes 0, 1) or
// the exchange's epoch (mode 2)
template <int MODE, int W>
__device__ __forceinline__ void meet(int* c, int target, int* err) {
  if constexpr (MODE == 0) pattern_barrier(c, target, err);
  else if constexpr (MODE == 1) pattern_barrier_xcd(c, target, err);
  else pattern_barrier_flags(c, W, target / W, err);
}

// the four exchanges alone (the sync cost of a split chain, nothing transformed)
template <int W, int MODE>
__global__ __launch_bounds__(256) void k_meet_only(int* cnt, int base, int* err) {
  const int b = blockIdx.x, xcd = b & 7, r = b >> 3;
  const int pat = (r / W) * 8 + xcd;
  for (int k = 0; k < 4; ++k) meet<MODE, W>(cnt + (MODE == 2 ? 8 : 1) * pat, base + (k + 1) * W, err);
}

template <int W, int MODE = 0>
__global__ __launch_bounds__(256) void k_lds_chain(float2* f, const float2* M, const float2* twg, int* cnt, int base,
                                                   int* err) {
  constexpr int L = N / W;
  using LT = LineTile<N, L>;
  using P1 = Plan1D<N>;
  __shared__ float2 s_tw[N];
  __shared__ float2 T[LT::kElems];
  // blocks of one pattern on one XCD (dispatch deals blocks round-robin over the 8 XCDs)
  const int b = blockIdx.x, xcd = b & 7, r = b >> 3;
  const int pat = (r / W) * 8 + xcd, sub = r % W;
  float2* F = f + (size_t)pat * N2;
  const int l0 = sub * L;
  for (int i = threadIdx.x; i < N; i += 256) s_tw[i] = twg[i];
  auto load_rows = [&] {
    for (int e = threadIdx.x; e < L * N; e += 256) T[LT::off(e / N, e % N)] = F[(size_t)(l0 + e / N) * N + e % N];
    __syncthreads();
  };
  auto store_rows = [&] {
    for (int e = threadIdx.x; e < L * N; e += 256) F[(size_t)(l0 + e / N) * N + e % N] = T[LT::off(e / N, e % N)];
  };
  auto load_cols = [&] {
    for (int e = threadIdx.x; e < L * N; e += 256) {
      const int y = e / L, c = e % L;
      T[LT::off(c, y)] = F[(size_t)y * N + l0 + c];
    }
    __syncthreads();
  };
  auto store_cols = [&] {
    for (int e = threadIdx.x; e < L * N; e += 256) {
      const int y = e / L, c = e % L;
      F[(size_t)y * N + l0 + c] = T[LT::off(c, y)];
    }
  };
  auto mul_rows = [&](const float2* m) {
    for (int e = threadIdx.x; e < L * N; e += 256) {
      float2& t = T[LT::off(e / N, e % N)];
      t = cmul(t, m[(size_t)(l0 + e / N) * N + e % N]);
    }
    __syncthreads();
  };
  auto mul_cols = [&](const float2* m) {
    for (int e = threadIdx.x; e < L * N; e += 256) {
      const int y = e / L, c = e % L;
      float2& t = T[LT::off(c, y)];
      t = cmul(t, m[(size_t)y * N + l0 + c]);
    }
    __syncthreads();
  };
  auto xchg = [&](int k) {
    if constexpr (W == 1) __syncthreads();
    else meet<MODE, W>(cnt + (MODE == 2 ? 8 : 1) * pat, base + (k + 1) * W, err);
  };
  // F1 = F⁻¹ (rows, then columns) · M0 · F2 = F (columns, then rows) · M1 · F3 = F⁻¹ (rows, columns)
  // · M2 · F4 = F (columns, rows) · M3
  load_rows();
  line_pass<N, 256, P1::R1, 1, +1, L>(T, s_tw, L);
  line_pass<N, 256, P1::R2, P1::R1, +1, L>(T, s_tw, L);
  store_rows();
  xchg(0);
  load_cols();
  line_pass<N, 256, P1::R1, 1, +1, L>(T, s_tw, L);
  line_pass<N, 256, P1::R2, P1::R1, +1, L>(T, s_tw, L);
  mul_cols(M);
  line_pass<N, 256, P1::R1, 1, -1, L>(T, s_tw, L);
  line_pass<N, 256, P1::R2, P1::R1, -1, L>(T, s_tw, L);
  store_cols();
  xchg(1);
  load_rows();
  line_pass<N, 256, P1::R1, 1, -1, L>(T, s_tw, L);
  line_pass<N, 256, P1::R2, P1::R1, -1, L>(T, s_tw, L);
  mul_rows(M + N2);
  line_pass<N, 256, P1::R1, 1, +1, L>(T, s_tw, L);
  line_pass<N, 256, P1::R2, P1::R1, +1, L>(T, s_tw, L);
  store_rows();
  xchg(2);
  load_cols();
  line_pass<N, 256, P1::R1, 1, +1, L>(T, s_tw, L);
  line_pass<N, 256, P1::R2, P1::R1, +1, L>(T, s_tw, L);
  mul_cols(M + 2 * N2);
  line_pass<N, 256, P1::R1, 1, -1, L>(T, s_tw, L);
  line_pass<N, 256, P1::R2, P1::R1, -1, L>(T, s_tw, L);
  store_cols();
  xchg(3);
  load_rows();
  line_pass<N, 256, P1::R1, 1, -1, L>(T, s_tw, L);
  line_pass<N, 256, P1::R2, P1::R1, -1, L>(T, s_tw, L);
  mul_rows(M + 3 * N2);
  store_rows();
}

// the production register transform, one workgroup a pattern (k_fused3's chain without its DMA
// rings, loss, slots and slabs)
__global__ __launch_bounds__(256, 1) void k_reg_chain(float2* f, const float2* M) {
  using namespace rf;
  __shared__ float2 buf[kLdsElems];
  const Coord cd = coord(threadIdx.x);
  const LaneCtx lc = lane_ctx(cd.lane);
  float2 v[64];
  float2* F = f + (size_t)blockIdx.x * N2;
  const int fx = cd.fixed, l0 = cd.l0, t = threadIdx.x;
  // K-layout operands packed as the engine's F(P) (element k of thread t at 256 k + t: coalesced),
  // R-layout ones row-major (two 256-B row segments a wave and register)
#pragma unroll
  for (int k = 0; k < 64; ++k) v[k] = F[(size_t)k * 256 + t];                // K layout
  fft_inv(v, buf, lc, cd.wsign);                                              // → R layout
#pragma unroll
  for (int j = 0; j < 64; ++j) v[j] = cmul(v[j], M[(size_t)(j + 64 * l0) * N + fx]);
  fft_fwd(v, buf, lc, cd.wsign);
#pragma unroll
  for (int k = 0; k < 64; ++k) v[k] = cmul(v[k], M[N2 + (size_t)k * 256 + t]);
  fft_inv(v, buf, lc, cd.wsign);
#pragma unroll
  for (int j = 0; j < 64; ++j) v[j] = cmul(v[j], M[2 * N2 + (size_t)(j + 64 * l0) * N + fx]);
  fft_fwd(v, buf, lc, cd.wsign);
#pragma unroll
  for (int k = 0; k < 64; ++k) F[(size_t)k * 256 + t] = cmul(v[k], M[3 * N2 + (size_t)k * 256 + t]);
}

struct Bufs {
  float2 *f, *M, *twg;
  int *cnt, *err;
};

template <class Launch>
static double time_us(Launch&& launch) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < kWarm; ++i) launch(i);
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < kLaunches; ++i) launch(kWarm + i);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 1e3 * ms / kLaunches;
}

template <int W, int MODE>
static void run_lds(Bufs& d, const std::vector<float2>& f0, std::vector<float2>& ref, bool& ok) {
  const size_t fb = f0.size() * sizeof(float2);
  // one launch from f0 for the bitwise check, then the timing (the field keeps transforming)
  CK(hipMemcpy(d.f, f0.data(), fb, hipMemcpyHostToDevice));
  CK(hipMemset(d.cnt, 0, 8 * kPat * sizeof(int)));
  CK(hipMemset(d.err, 0, sizeof(int)));
  int launches = 0;
  auto launch = [&](int) {
    hipLaunchKernelGGL((k_lds_chain<W, MODE>), dim3(kPat * W), dim3(256), 0, 0, d.f, d.M, d.twg, d.cnt,
                       launches * 4 * W, d.err);
    ++launches;
  };
  launch(0);
  CK(hipDeviceSynchronize());
  std::vector<float2> out(f0.size());
  CK(hipMemcpy(out.data(), d.f, fb, hipMemcpyDeviceToHost));
  bool same = true;
  if (W == 1) ref = out;
  else same = std::memcmp(out.data(), ref.data(), fb) == 0;
  const double us = time_us(launch);
  int err = 0;
  CK(hipMemcpy(&err, d.err, sizeof(int), hipMemcpyDeviceToHost));
  ok = ok && same && err == 0;
  std::printf("{\"variant\": \"lds\", \"W\": %d, \"exchange\": \"%s\", \"workgroups\": %d, \"us_per_call\": %.2f, "
              "\"bitwise_w1\": %s, \"barrier_timeouts\": %d}\n",
              W, W == 1 ? "none" : MODE == 0 ? "agent" : MODE == 1 ? "xcd" : "xcd_flags", kPat * W, us, same ? "true" : "false", err);
  if (W > 1) {   // the exchanges alone
    CK(hipMemset(d.cnt, 0, 8 * kPat * sizeof(int)));
    int nl = 0;
    const double um = time_us([&](int) {
      hipLaunchKernelGGL((k_meet_only<W, MODE>), dim3(kPat * W), dim3(256), 0, 0, d.cnt, nl * 4 * W, d.err);
      ++nl;
    });
    CK(hipMemcpy(&err, d.err, sizeof(int), hipMemcpyDeviceToHost));
    ok = ok && err == 0;
    std::printf("{\"variant\": \"meet_only\", \"W\": %d, \"exchange\": \"%s\", \"us_per_call\": %.2f, "
                "\"barrier_timeouts\": %d}\n", W, MODE == 0 ? "agent" : MODE == 1 ? "xcd" : "xcd_flags", um, err);
  }
}

int main() {
  Bufs d;
  const size_t n = (size_t)kPat * N2;
  std::vector<float2> f0(n), M(4 * N2), tw(N);
  unsigned s = 12345u;
  auto rnd = [&] {
    s = s * 1664525u + 1013904223u;
    return (float)((s >> 8) & 0xffff) / 65536.0f - 0.5f;
  };
  for (auto& x : f0) x = make_float2(rnd(), rnd());
  for (auto& x : M) {   // unit-modulus factors (the chain stays bounded over 220 launches)
    const double ph = 6.283185307179586 * rnd();
    x = make_float2((float)std::cos(ph), (float)std::sin(ph));
  }
  for (int i = 0; i < N; ++i)
    tw[i] = make_float2((float)std::cos(-6.283185307179586 * i / N), (float)std::sin(-6.283185307179586 * i / N));
  CK(hipMalloc(&d.f, n * sizeof(float2)));
  CK(hipMalloc(&d.M, M.size() * sizeof(float2)));
  CK(hipMalloc(&d.twg, N * sizeof(float2)));
  CK(hipMalloc(&d.cnt, 8 * kPat * sizeof(int)));
  CK(hipMalloc(&d.err, sizeof(int)));
  CK(hipMemcpy(d.M, M.data(), M.size() * sizeof(float2), hipMemcpyHostToDevice));
  CK(hipMemcpy(d.twg, tw.data(), N * sizeof(float2), hipMemcpyHostToDevice));
  // (the chain normalises nothing: after a few timed launches the fields are inf / nan, which
  // costs the same arithmetic; the bitwise check uses the first launch from f0)
  CK(hipMemcpy(d.f, f0.data(), n * sizeof(float2), hipMemcpyHostToDevice));
  const double us_reg = time_us([&](int) { hipLaunchKernelGGL(k_reg_chain, dim3(kPat), dim3(256), 0, 0, d.f, d.M); });
  std::printf("{\"variant\": \"reg\", \"W\": 1, \"workgroups\": %d, \"us_per_call\": %.2f}\n", kPat, us_reg);
  std::vector<float2> ref;
  bool ok = true;
  run_lds<1, 0>(d, f0, ref, ok);
  run_lds<2, 0>(d, f0, ref, ok);
  run_lds<4, 0>(d, f0, ref, ok);
  run_lds<8, 0>(d, f0, ref, ok);
  run_lds<2, 1>(d, f0, ref, ok);
  run_lds<4, 1>(d, f0, ref, ok);
  run_lds<8, 1>(d, f0, ref, ok);
  run_lds<2, 2>(d, f0, ref, ok);
  run_lds<4, 2>(d, f0, ref, ok);
  run_lds<8, 2>(d, f0, ref, ok);
  CK(hipFree(d.f));
  CK(hipFree(d.M));
  CK(hipFree(d.twg));
  CK(hipFree(d.cnt));
  CK(hipFree(d.err));
  return ok ? 0 : 2;
}
