// ptyx_common.hpp — constants, kernel argument block and small device helpers shared by every
// ptyx kernel (ptyx_kernels.hip and the per-engine headers it includes).
#pragma once
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include "ptyx.h"
#include "ptyx_fft.hpp"

namespace ptyx {

constexpr int kMaxModesO = 32;                // object modes (loss_sparse sums / coefficients per mode)
constexpr int kSumBase = 4;                    // [S_single, ΣM^q1, S_poissn, ΣM^q2] then O sparse sums
constexpr int kNSum = kSumBase + kMaxModesO;
constexpr int kNCoef = 2 + kMaxModesO;         // [c_single, c_poissn, c_sparse[o]...]
constexpr int kNBatchSum = 5 + kMaxModesO;     // per mini-batch: [count, S1, ΣM^q1, S2, ΣM^q2, sparse[o]...]
static_assert(kNBatchSum == PTYX_BATCH_SUMS, "include/ptyx.h PTYX_BATCH_SUMS");
constexpr float kDpEps = 1e-10f;               // forward.py:20 eps

// Launch geometry of the general engine's workgroup-resident FFT kernels.
//  N ≤ 128: the N×N wave in LDS (in place, ≤ 136 KiB), NT = 8·N threads (≤ 1024).
//  N > 128: the per-workgroup global scratch pair (two line-block round trips a 2-D FFT), 1024
//  threads.  512 threads whenever a radix above 16 holds up to 49 points a thread (125, 162, 200,
//  216, 243, 250 and most N > 256: one wave a SIMD, up to 512 registers); N = 256 has its own
//  two-stage path with two 512-thread workgroups a CU (LDS ≈ 78 KiB each).
// kWaves: minimum waves per SIMD the kernels are compiled for (≤ 512 / kWaves VGPRs): enough for
// every workgroup LDS and threads allow on a CU to be resident at once (capped at 8 = 64 VGPRs).
// Measured (profiles/r04/occ/): N 135-240 +12-21 %, 45 / 60 / 75 / 81 / 90 +11-32 %, no size
// slower by more than 1.5 %; the floor of waves / 4 instead of rounding a workgroup's waves up per
// SIMD made N 80 16 % slower (two workgroups still did not fit, so the cap only added spills).
template <int N>
struct Geo {
  static constexpr bool kLds = N <= 128;
  static constexpr int NT = N == 256 ? kG256Threads
                          : Plan1D<N>::R1 > 16 ? 512
                          : kLds ? ((8 * N + 63) / 64 * 64 > 1024 ? 1024 : (8 * N + 63) / 64 * 64)
                          : 1024;
  // workgroups a CU holds by LDS and threads (as GenLaunch::blocks_per_cu)
  static constexpr int kLdsBytes = (int)sizeof(float2) * (5 * N + kFieldLds<N, kLds>) + 256;
  static constexpr int kResident = (160 * 1024 / kLdsBytes) < (2048 / NT) ? (160 * 1024 / kLdsBytes) : (2048 / NT);
  static constexpr int kWavesRes = kResident * ((NT + 255) / 256);   // a workgroup's waves round up per SIMD
  static constexpr int kWaves = N == 256 ? 4 : Plan1D<N>::R1 > 16 ? 1 : kWavesRes > 8 ? 8 : kWavesRes;
};

struct KArgs {
  int P, O, Nz, Ny, Nx, n_scans;
  int shift, meas_f16;
  const float* obja;
  const float* objp;
  const float2* probe;
  const float2* Fp;
  const float* shifts;
  const int* crop;
  const float2* H;
  const float* occu;
  const void* meas;
  const int* idx;
  int n_idx;
  const int* boff;
  int n_batches;
  int single_on, pois_on, sparse_on, sparse_n;
  float q1, q2, eps2;
  const float* coef;
  float* psums;
  float* Ibuf;
  float* dp_out;
  const float* dLdI_ext;
  float ext_scale;
  float* d_obja;
  float* d_objp;
  float* d_shifts;
  int need_probe;
  float2* slab;
  float2* scratch;
  long long scratch_stride;
  const float2* twg;
  float w1, w2, ws, grad_scale;
  // rank-local measurement block: row of meas holding scan position s (NULL: row s)
  const int* mrow;
  int mrows;        // rows of meas (the bound meas_rows entries are checked and clamped against)
  int* err;         // the plan's input-error flags (check_pattern), host-mapped
  // propagator gradient (PTYX_PROP_GRAD): per-workgroup dL/dH slabs; F(ψⁿ⊙Oⁿ) parked after gacc
  float2* hslab;
  // per-position tilts: ramps exp(i dz k tan(θ/1e3)) along y and x, and their gradient
  const float* ptilt;
  const float* kvec;
  float dz;
  float* d_tilts;
  float* d_dz;      // ramp part of dL/d(dz) with per-position tilts
  // far-field cache (general engine, P·O > 1): k_forward leaves every mode's F(ψ_out) and ψ⁰ of
  // every probe mode (Nz = 1) or every slice's ψⁿ (Nz > 1) per pattern, so k_adjoint skips the
  // recomputed forward
  float2* ffc;
  long long ffc_per;   // float2 per pattern: (P·O + P)·N² (Nz = 1) or P·O·(1 + Nz)·N²
  // probe-mode split (small calls, P > 1): msplit = P makes every (pattern, probe mode) its own
  // job in k_forward / k_adjoint; k_forward then leaves Σ_o occ|Ψ_{p,o}|² per mode in Imodes
  // ((pattern·P + p)·N² floats) and k_forward_modesum forms I, dp and the loss sums
  int msplit = 1;
  float* Imodes = nullptr;
  // compact probe slabs (split calls without propagator slabs): k_adjoint runs on a grid that is
  // a multiple of P, so workgroup w only ever sees probe mode w % P and owns one slab plane
  // (zeroed and reduced alone: k_slab_reduce over grid / P "virtual workgroups")
  int cslab = 0;
  // N = 128 register engines: k_probe_spectrum also leaves F(P) in their packed K layout (the
  // layout k_pack128<true> makes), so a step launches no separate pack kernel
  float2* fpk = nullptr;
  // N = 256 fused chains (g256_fstage): F(P_p) and H transposed, written by k_probe_spectrum,
  // so the stages that run on the transposed array read them along its rows
  float2* FpT = nullptr;   // (P, N, N): FpT[p][x][y] = F(P_p)[y][x]   (shifted probes)
  float2* HT = nullptr;    // (N, N):    HT[x][y] = H[y][x]             (Nz > 1)
};
// calls of at most this many patterns split their probe modes over workgroups (general engine)
constexpr int kModeSplitCap = 128;

// ---------------------------------------------------------------- small helpers
// threadIdx.x behind an empty asm: per-pattern address arithmetic stays inside the pattern
// loop instead of being hoisted (and spilled) by loop-invariant code motion.
__device__ __forceinline__ int opaque_tid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

// x^q for x >= 0 (DP intensities): exact forms for the schema values 0.5 / 1, otherwise
// exp2(q·log2 x) on the v_exp_f32 / v_log_f32 units (no libm slow path in the fused epilogues).
__device__ __forceinline__ float powq(float x, float q) {
  if (q == 0.5f) return sqrtf(x);
  if (q == 1.0f) return x;
  if (!(x > 0.f)) return q > 0.f ? 0.f : __builtin_inff();
  return __builtin_amdgcn_exp2f(q * __builtin_amdgcn_logf(x));
}

__device__ __forceinline__ float fast_ln(float x) { return __builtin_amdgcn_logf(x) * 0.69314718055994531f; }

// sin/cos of an object phase: reduce to revolutions in [-1/2, 1/2], then v_sin_f32 / v_cos_f32
// (which take revolutions).  Absolute error ≈ |φ|·6e-8 + 1 ulp, far inside the parity budget.
__device__ __forceinline__ void phase_sincos(float ph, float* sn, float* cs) {
  float r = ph * 0.15915494309189535f;
  r = r - rintf(r);
  *sn = __builtin_amdgcn_sinf(r);
  *cs = __builtin_amdgcn_cosf(r);
}

__device__ __forceinline__ float meas_at(const KArgs& a, int s, int e, int N2) {
  const size_t off = (size_t)s * N2 + e;
  if (a.meas_f16) return __half2float(reinterpret_cast<const __half*>(a.meas)[off]);
  return reinterpret_cast<const float*>(a.meas)[off];
}

__device__ __forceinline__ size_t obj_off(const KArgs& a, int o, int n, int yy, int xx) {
  return ((size_t)(o * a.Nz + n) * a.Ny + yy) * a.Nx + xx;
}

// wave64 + workgroup sum of NV floats, fixed order (deterministic); result valid in thread 0.
template <int NT, int NV>
__device__ __forceinline__ void block_sum(float (&v)[NV], float* red) {
#pragma unroll
  for (int i = 0; i < NV; ++i) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v[i] += __shfl_xor(v[i], m, 64);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) red[wv * NV + i] = v[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      float t = 0.f;
      for (int w = 0; w < NT / 64; ++w) t += red[w * NV + i];
      v[i] = t;
    }
  }
  __syncthreads();
}

// Input validation (include/ptyx.h preconditions).  The engines' table kernels check every
// pattern of a call: a scan index outside [0, n_scans), a window crop_pos + N outside the object
// or a measurement row outside the block sets its flag in the plan's error words (host-mapped
// memory, plain vector stores of 1, no atomics) and the kernels go on with the value clamped, so
// nothing is read out of bounds; the next call on the plan (or ptyx_plan_check) reports
// PTYX_EINVAL.  No host synchronisation on the hot path.
enum { kErrIdx = 0, kErrWindow = 1, kErrRow = 2, kErrWords = 4 };
__device__ __forceinline__ void check_pattern(int* err, int s_raw, int n_scans, const int* crop, int Ny, int Nx, int N,
                                              const int* mrow, int mrows) {
  if (!err) return;
  if (s_raw < 0 || s_raw >= n_scans) err[kErrIdx] = 1;
  const int s = min(max(s_raw, 0), n_scans - 1);
  const int cy = crop[2 * s], cx = crop[2 * s + 1];
  if (cy < 0 || cx < 0 || cy > Ny - N || cx > Nx - N) err[kErrWindow] = 1;
  if (mrow) {
    const int m = mrow[s];
    if (m < 0 || m >= mrows) err[kErrRow] = 1;
  }
}
// measurement row of scan position s, clamped into the block
__device__ __forceinline__ int meas_row(const int* mrow, int mrows, int s) {
  return mrow ? min(max(mrow[s], 0), mrows - 1) : s;
}

struct PatternGeom {
  int s, m, cy, cx;   // scan index, its measurement row, clamped window origin
  float sy, sx;
};

__device__ __forceinline__ PatternGeom pattern_geom(const KArgs& a, int pat, int N) {
  PatternGeom g;
  const int s_raw = a.idx[pat];
  if (threadIdx.x == 0) check_pattern(a.err, s_raw, a.n_scans, a.crop, a.Ny, a.Nx, N, a.mrow, a.mrows);
  const int s = min(max(s_raw, 0), a.n_scans - 1);   // (invalid inputs: flagged above, clamped here)
  g.s = s;
  g.m = meas_row(a.mrow, a.mrows, s);
  g.cy = min(max(a.crop[2 * s], 0), a.Ny - N);
  g.cx = min(max(a.crop[2 * s + 1], 0), a.Nx - N);
  g.sy = a.shifts[2 * s];
  g.sx = a.shifts[2 * s + 1];
  return g;
}

// W_b ramps along y and x: exp(-2πi s g[k]), g[k] = ((k + N/2) mod N)/N  (image_proc.py:531,
// models.py:179 grid arange(N)/N after ifftshift).
template <int N, int NT>
__device__ __forceinline__ void build_ramps(const PatternGeom& g, float2* wy, float2* wx) {
  for (int k = opaque_tid(); k < 2 * N; k += NT) {
    const int kk = k % N;
    const float gr = (float)((kk + N / 2) % N) / (float)N;
    const float s = k < N ? g.sy : g.sx;
    float sn, cs;
    sincospif(-2.0f * s * gr, &sn, &cs);
    (k < N ? wy : wx)[kk] = make_float2(cs, sn);
  }
  __syncthreads();
}

template <int N>
__device__ __forceinline__ float shift_g(int k) {
  return (float)((k + N / 2) % N) / (float)N;
}

template <int N, bool LDS>
struct ArrayFor;
template <int N>
struct ArrayFor<N, true> {
  using type = LdsArray<N>;
};
template <int N>
struct ArrayFor<N, false> {
  using type = GlobalPair<N>;
};

// Scratch layout per workgroup (float2 units): [fft a, fft b (N=256 only)] [psi: Nz·N²] [gacc: N²]
template <int N>
__device__ __forceinline__ float2* scratch_psi(const KArgs& a) {
  return a.scratch + (long long)blockIdx.x * a.scratch_stride + (Geo<N>::kLds ? 0 : 2 * N * N);
}

}  // namespace ptyx
