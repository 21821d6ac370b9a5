// ptyx_fmm.hpp — the mixed-state register engine: N = 128, P probe modes (P > 1), one object
// mode, Nz ≥ 1 slices, on the register-resident FFT of ptyx_regfft.hpp.  The geometry of the
// reference's own demo (tBL_WSe2: 6 probe modes × 6 slices, demo/params/tBL_WSe2_reconstruct.yml
// :23-27).  Included by ptyx_kernels.hip after ptyx_fused3.hpp.
//
// k_fused3ms carries one pattern's whole forward → loss → adjoint in one workgroup's registers.
// With P modes the loss needs I = Σ_p occ|Ψ_p|² before any mode's adjoint can start, and a second
// 128-VGPR field per mode does not fit, so the chain is cut at the far field into three launches,
// each a JOB per (pattern, probe mode) — P times the workgroups of a pattern-per-workgroup design,
// which is what keeps the reference's default cadence (one 32-pattern mini-batch a step) busy:
//
//   k_fmm_fwd   job (b, p): ψ⁰ = F⁻¹(F(P_p)·W_b)/N²; for n: park ψⁿ (slot plane (b, n, p)), ×O_n,
//               ×H between slices (forward.py:50-63, image_proc.py:531-532); far field
//               v = F(ψ_out) stored K-packed (Ψ = v/N, forward.py:79)
//   k_fmm_loss  pattern b, in kLossParts parts of its K points: I = Σ_p occ|v_p|²/N² + 1e-10,
//               dp_out, the loss partial sums and u = ∂ℓ/∂I per unit mini-batch coefficient, one
//               plane per data term (K-packed; losses.py:36-75)
//   k_finalize  c_m per mini-batch
//   k_fmm_adj   job (b, p): g = F⁻¹(v_p·2 occ (c1 u1 + c2 u2)/N)/N (the coefficients applied here:
//               this kernel runs after k_finalize, so both data terms fit one field); for
//               n = Nz−1 … 0: slot (b, n, p) = g·conj(ψⁿ) (k_obj_gather sums the P planes), g ←
//               g·conj(O_n), ×conj(H) between slices; then g → probe-gradient spectrum
//               (per-workgroup segment of one mode) and the position sums, as k_fused3ms
//
// 4·Nz FFTs per job, 4·Nz·P per pattern, no recomputed forward.  Slots and far fields live in the
// plan's far-field cache: per pattern P·(Nz + 1) planes of N² float2, slot plane (b, n, p) at
// (b·pstride + n·P + p)·N², far field of mode p at (b·pstride + Nz·P + p)·N².  Jobs are numbered
// mode-major (job = p·n_idx + b) and workgroup w takes the contiguous range
// [w·J/G, (w+1)·J/G): consecutive jobs share F(P_p) and the object band, and a workgroup's jobs
// fall in at most a few probe modes (segment id p + w: unique, since every segment boundary
// advances p or w).
#pragma once
#include "ptyx_fused3.hpp"

namespace ptyx {
namespace f3 {

struct FmArgs {
  F3Args f;             // fpk: P planes (K-packed F(P_p), or the probes R-packed without shifts)
  int P;
  long long pstride;    // float2 planes per pattern in f.slots: P·(Nz + 1)
  float* ubuf;          // (patterns, N²) f32 K-packed: ∂ℓ_single/∂I (or ∂ℓ_poissn/∂I) per unit coefficient
  float* ubuf2;         // both data terms: ∂ℓ_poissn/∂I per unit coefficient (else unused)
  float q1, q2;         // dp_pow of loss_single / loss_poissn (f.eps2: the poissn eps)
  const float* coef;    // k_finalize's per-mini-batch coefficients
  int ci;               // one data term: its coefficient index (0 single, 1 poissn)
  float* lparts;        // (patterns, kLossParts, 4) loss partial sums of k_fmm_loss
};

__device__ __forceinline__ float ld1(Rsrc r, int voff, int off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff + off, 0, 0));
}
__device__ __forceinline__ void st1(float v, Rsrc r, int voff, int off) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, voff + off, 0, 0);
}
struct Ch4u {
  float2 x[4];
  float u[4];
};

__device__ __forceinline__ size_t fmm_slot(const FmArgs& m, int pat, int n, int p) {
  return ((size_t)pat * m.pstride + (size_t)n * m.P + p) * kN2;
}
__device__ __forceinline__ size_t fmm_far(const FmArgs& m, int pat, int p) {
  return ((size_t)pat * m.pstride + (size_t)m.f.Nz * m.P + p) * kN2;
}

// ------------------------------------------------------------------ forward: job → far field
// HOLDH (calls of at most one workgroup per CU, e.g. the reference's default cadence): the
// K-packed H/N² is loaded into registers once per workgroup (64 more float2 a thread: one
// workgroup a CU, so the unified register file holds them) instead of streaming 128 KiB from L2
// in every propagation.
template <bool SHIFT, bool HOLDH>
__global__ __launch_bounds__(256, HOLDH ? 1 : 2) void k_fmm_fwd(FmArgs m) {
  using namespace rf;
  const F3Args& a = m.f;
  __shared__ float2 buf[kLdsElems];
  const Coord cd = coord(threadIdx.x);
  const LaneCtx lc = lane_ctx(cd.lane);
  constexpr float inv_n2 = 1.0f / kN2;
  const int w = blockIdx.x, G = gridDim.x;
  const int nj = a.n_idx * m.P;
  const int j0 = (int)((long long)w * nj / G), j1 = (int)((long long)(w + 1) * nj / G);
  if (j0 >= j1) return;
  const int Nx = a.Nx, Nz = a.Nz;
  const size_t plane = (size_t)a.Ny * a.Nx;
  const Rsrc r_hpk = rsrc(a.hpk, kN2 * 8);
  const float gy = (float)((cd.fixed + 64) & 127) * (1.0f / kN);
  constexpr bool kRing = SHIFT;
  const int lds0 = (int)(size_t)(__attribute__((address_space(3))) float2*)buf;
  float2 v[64];

  float2 hreg[HOLDH ? 64 : 1];
  if constexpr (HOLDH) {
    if (Nz > 1) {
      const int vpk = 8 * threadIdx.x;
#pragma unroll
      for (int k = 0; k < 64; ++k) hreg[k] = ld2(r_hpk, vpk, 2048 * k);
    }
  }
  auto prop_k = [&] {   // v ← v ⊙ H/N² (K layout)
    if constexpr (HOLDH) {
#pragma unroll
      for (int k = 0; k < 64; ++k) {
        v[k] = pcm(v[k], hreg[k]);
        pin(v[k]);
      }
      return;
    }
    const int vpk = rf::opaque(8 * rf::opaque(threadIdx.x));
    pipeline<16>(
        [&](auto C) {
          Ch4x2 t;
#pragma unroll
          for (int r = 0; r < 4; ++r) t.x[r] = ld2(r_hpk, vpk, 2048 * (4 * C + r));
          return t;
        },
        [&](auto C, const Ch4x2& t) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int k = 4 * C + r;
            v[k] = pcm(v[k], t.x[r]);
            pin(v[k]);
          }
        });
  };

  for (int job = j0; job < j1; ++job) {
    const int p = __builtin_amdgcn_readfirstlane(job / a.n_idx);
    const int pat = job - p * a.n_idx;
    const int tid = rf::opaque(threadIdx.x);
    const PatInfo pi = pat_info<SHIFT>(a, pat);
    // v = F(P_p)·W_b (K layout), or the probe (R layout) without shifts
    {
      const Rsrc r_fpk = rsrc(a.fpk + (size_t)p * kN2, kN2 * 8);
      const int vpk = 8 * tid;
      Ramp rp;
      rp.init(pi.sy, pi.sx, gy, tid & 1);
      pipeline<16>(
          [&](auto C) {
            Ch4x2 t;
#pragma unroll
            for (int r = 0; r < 4; ++r) t.x[r] = ld2(r_fpk, vpk, 2048 * (4 * C + r));
            return t;
          },
          [&](auto C, const Ch4x2& t) {
            const float2 A = rp.a(C);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[4 * C + r] = SHIFT ? pcm(t.x[r], pcm(A, rp.B[r])) : t.x[r];
              pin(v[4 * C + r]);
            }
          });
    }
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int m0w = lds0 + (wv << 14);
    const float2* ringw = buf + (wv << 11);
    const int os = __builtin_amdgcn_readfirstlane(8 * Nx);
    const unsigned obytes = (unsigned)(((kN - 1) * Nx + kN) * 8);
    auto s_obj = [&](int n) { return srd(a.oc + n * plane + (size_t)pi.cy * Nx + pi.cx, obytes); };
    auto issue1 = [&](auto Q, const v4u& so, int voff) {
      constexpr int q = decltype(Q)::value;
      dma_m<2 * q>(so, voff, m0w + (q % 16) * 1024, os);
    };
    auto pre1 = [&](int n) {
      if constexpr (kRing) {
        const v4u so = s_obj(n);
        const int vo = dma_off_obj(rf::opaque(tid) & 63, wv, os);
        rf::sfor<0, 16>([&](auto Q) { issue1(Q, so, vo); });
      }
    };
    if constexpr (SHIFT) {
      fft_inv(v, buf, lc, cd.wsign, [&] { pre1(0); });
#pragma unroll
      for (int j = 0; j < 64; ++j) v[j] = pscale(v[j], inv_n2);
    }
    // ------------------------------------------------ slices: park ψⁿ, ×O_n, propagate
    for (int n = 0; n < Nz; ++n) {
      const Rsrc r_slot = rsrc(a.slots + fmm_slot(m, pat, n, p), kN2 * 8);
      if constexpr (kRing) {
        const v4u so = s_obj(n);
        const int lam = rf::opaque(tid) & 63;
        const int vo = dma_off_obj(lam, wv, os);
        const int vpark = park_off(lam, wv);
        const int io = obj_img(lam);
        rf::sfor<0, 32>([&](auto Q) {
          constexpr int q = decltype(Q)::value;
          vm_wait<ring_wait_count(q, 1, 0, 16)>();
          const float2* sl = ringw + (q % 16) * 128;
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) {
            const int j = 2 * q + rb;
            const float2 O = sl[rb * 64 + io];
            st2_stream(v[j], r_slot, vpark, 2048 * j);   // ψⁿ park (ring layout: read back by k_fmm_adj)
            v[j] = pcm(v[j], O);
            pin(v[j]);
          }
          if constexpr (q + 16 < 32) issue1(std::integral_constant<int, q + 16>{}, so, vo);
          __builtin_amdgcn_sched_barrier(0);
        });
        __syncthreads();   // every wave is done with its ring before the next exchange
      } else {
        const Rsrc r_obj = rsrc(a.oc + n * plane + (size_t)pi.cy * Nx + pi.cx, obytes);
        const int tq = rf::opaque(threadIdx.x);
        const int vslot = 8 * ((tq & 1) * kN + fixed_of(tq)), vobj = 8 * (64 * (tq & 1) * Nx + fixed_of(tq));
        const int ostr = rf::opaque(8 * Nx);
        pipeline<8>(
            [&](auto C) {
              Ch8 t;
#pragma unroll
              for (int r = 0; r < 8; ++r) t.x[r] = ld2(r_obj, vobj, ostr * (8 * C + r));
              return t;
            },
            [&](auto C, const Ch8& t) {
#pragma unroll
              for (int r = 0; r < 8; ++r) {
                const int j = 8 * C + r;
                st2(v[j], r_slot, vslot, 2048 * j);
                v[j] = pcm(v[j], t.x[r]);
                pin(v[j]);
              }
            });
      }
      if (n + 1 < Nz) {
        fft_fwd(v, buf, lc, cd.wsign);
        prop_k();
        fft_inv(v, buf, lc, cd.wsign, [&] { pre1(n + 1); });
      }
    }
    // ------------------------------------------------ far field v = F(ψ_out), K-packed
    fft_fwd(v, buf, lc, cd.wsign);
    {
      const Rsrc r_far = rsrc(a.slots + fmm_far(m, pat, p), kN2 * 8);
      const int vpk = rf::opaque(8 * tid);
#pragma unroll
      for (int k = 0; k < 64; ++k) {
        st2_stream(v[k], r_far, vpk, 2048 * k);
        if ((k & 7) == 7) __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
}

// ------------------------------------------------------------------ loss: pattern part → u, sums
// kLossParts workgroups per pattern, part s owning the K-packed registers k ∈ [s·KP, (s+1)·KP) of
// every thread (KP = 64 / kLossParts): the P far fields are read in mode order and their
// intensities summed, the DP values of those points are read directly (row (ky + 64) mod 128,
// columns 4⌊k/4⌋ + 64(1 − l0) …: the fftshifted image), and the part's loss partial sums go to
// lparts[pattern][part] (k_finalize adds the parts in order, fp64).  At the reference's default
// cadence a call is one 32-pattern mini-batch: one workgroup per pattern would leave 224 CUs idle
// behind a serial 6 × 128 KiB read; the same split at every call size keeps each pattern's sums
// independent of how the call is cut.
// TERMS: 1 loss_single, 2 loss_poissn, 3 both (QM: loss_single's dp_pow form; loss_poissn
// always takes the general form)
constexpr int kLossParts = 8;
template <int QM, int TERMS>
__global__ __launch_bounds__(256) void k_fmm_loss(FmArgs m) {
  constexpr int KP = 64 / kLossParts;
  const F3Args& a = m.f;
  __shared__ float s_red[4 * 4];
  const int pat = blockIdx.x / kLossParts, part = blockIdx.x % kLossParts;
  const PatInfo pi = pat_info<false>(a, pat);
  const int tid = rf::opaque(threadIdx.x);
  const int fx = fixed_of(tid), l0 = tid & 1;
  constexpr float inv_n2 = 1.0f / kN2;
  const int k0 = part * KP;
  // this part's DP values: KP / 4 float4 of row r, columns 4 kq + 64 b
  const int r = (fx + 64) & 127;   // fftshifted DP row of ky
  const int b = 1 - l0;            // fftshifted column half of kx = k + 64 l0
  const float4* dp4 = reinterpret_cast<const float4*>(a.meas + (size_t)pi.mi * kN2 + r * kN + 64 * b) + k0 / 4;
  float4 M4[KP / 4];
#pragma unroll
  for (int q = 0; q < KP / 4; ++q) M4[q] = dp4[q];
  const float occ_n2 = a.occp[0] * inv_n2;
  float acc[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) acc[k] = 0.f;
  const int vpk = 8 * tid;
  for (int p = 0; p < m.P; ++p) {
    const Rsrc r_far = rsrc(a.slots + fmm_far(m, pat, p), kN2 * 8);
    float2 t[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) t[k] = ld2(r_far, vpk, 2048 * (k0 + k));
#pragma unroll
    for (int k = 0; k < KP; ++k) acc[k] = fmaf(occ_n2, cabs2(t[k]), acc[k]);
  }
  float S1 = 0.f, Ms1 = 0.f, S2 = 0.f, Ms2 = 0.f;
  {
    const Rsrc r_dp = rsrc(a.dp_out ? a.dp_out + (size_t)pat * kN2 : a.psums, a.dp_out ? kN2 * 4 : 0);
    const int vdp = 4 * (r * kN + 64 * b + k0);
    const Rsrc r_u = rsrc(m.ubuf + (size_t)pat * kN2, kN2 * 4);
    const Rsrc r_u2 = rsrc(TERMS == 3 ? m.ubuf2 + (size_t)pat * kN2 : m.ubuf, TERMS == 3 ? kN2 * 4 : 0);
    const int vu = 4 * tid;
#pragma unroll
    for (int q = 0; q < KP / 4; ++q) {
      const float Mv[4] = {M4[q].x, M4[q].y, M4[q].z, M4[q].w};
      float Iv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int kk = 4 * q + e, k = k0 + kk;
        Iv[e] = acc[kk] + kDpEps;
        if constexpr (TERMS & 1) st1(loss_point<QM, true>(Iv[e], Mv[e], m.q1, a.eps2, S1, Ms1), r_u, vu, 1024 * k);
        if constexpr (TERMS == 2) st1(loss_point<2, false>(Iv[e], Mv[e], m.q2, a.eps2, S2, Ms2), r_u, vu, 1024 * k);
        if constexpr (TERMS == 3) st1(loss_point<2, false>(Iv[e], Mv[e], m.q2, a.eps2, S2, Ms2), r_u2, vu, 1024 * k);
      }
      const __attribute__((ext_vector_type(4))) float i4 = {Iv[0], Iv[1], Iv[2], Iv[3]};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, i4),
                                             r_dp, vdp + 16 * q, 0, 0);
    }
  }
  float v4[4] = {S1, Ms1, S2, Ms2};
  block_sum4<4>(v4, s_red);
  if (threadIdx.x == 0) {
    float* lp = m.lparts + ((size_t)pat * kLossParts + part) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) lp[i] = v4[i];
  }
}

// ------------------------------------------------------------------ adjoint: job → slots, slab
// BOTH: loss_single and loss_poissn; the data coefficients c_m (k_finalize, which runs before this
// kernel) are applied to g_Ψ itself, so the slots, the probe spectrum and the position sums all
// carry them (k_obj_gather then takes data coefficient 1: FinArgs ci = 2)
template <bool SHIFT, bool BOTH, bool HOLDH>
__global__ __launch_bounds__(256, HOLDH ? 1 : 2) void k_fmm_adj(FmArgs m) {
  using namespace rf;
  const F3Args& a = m.f;
  __shared__ float2 buf[kLdsElems];
  __shared__ float s_red[4 * 2];
  const Coord cd = coord(threadIdx.x);
  const LaneCtx lc = lane_ctx(cd.lane);
  constexpr float inv_n = 1.0f / kN;
  const int w = blockIdx.x, G = gridDim.x;
  const int nj = a.n_idx * m.P;
  const int j0 = (int)((long long)w * nj / G), j1 = (int)((long long)(w + 1) * nj / G);
  if (j0 >= j1) return;
  const float occ2_n = 2.0f * a.occp[0] * inv_n;
  const bool tail = a.tail != 0;
  const int Nx = a.Nx, Nz = a.Nz;
  const size_t plane = (size_t)a.Ny * a.Nx;
  const Rsrc r_hpk = rsrc(a.hpk, kN2 * 8);
  const float gy = (float)((cd.fixed + 64) & 127) * inv_n;
  constexpr bool kRing = SHIFT;
  const int lds0 = (int)(size_t)(__attribute__((address_space(3))) float2*)buf;
  float2 v[64];

  float2 hreg[HOLDH ? 64 : 1];
  if constexpr (HOLDH) {
    if (Nz > 1) {
      const int vpk = 8 * threadIdx.x;
#pragma unroll
      for (int k = 0; k < 64; ++k) hreg[k] = ld2(r_hpk, vpk, 2048 * k);
    }
  }
  auto prop_kc = [&] {   // v ← v ⊙ conj(H)/N² (K layout)
    if constexpr (HOLDH) {
#pragma unroll
      for (int k = 0; k < 64; ++k) {
        v[k] = pcmc(v[k], hreg[k]);
        pin(v[k]);
      }
      return;
    }
    const int vpk = rf::opaque(8 * rf::opaque(threadIdx.x));
    pipeline<16>(
        [&](auto C) {
          Ch4x2 t;
#pragma unroll
          for (int r = 0; r < 4; ++r) t.x[r] = ld2(r_hpk, vpk, 2048 * (4 * C + r));
          return t;
        },
        [&](auto C, const Ch4x2& t) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int k = 4 * C + r;
            v[k] = pcmc(v[k], t.x[r]);
            pin(v[k]);
          }
        });
  };

  int p_prev = -1;
  for (int job = j0; job < j1; ++job) {
    const int p = __builtin_amdgcn_readfirstlane(job / a.n_idx);
    const int pat = job - p * a.n_idx;
    const int tid = rf::opaque(threadIdx.x);
    const PatInfo pi = pat_info<SHIFT>(a, pat);
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int m0w = lds0 + (wv << 14);
    const float2* ringw = buf + (wv << 11);
    const int os = __builtin_amdgcn_readfirstlane(8 * Nx);
    const unsigned obytes = (unsigned)(((kN - 1) * Nx + kN) * 8);
    auto s_obj = [&](int n) { return srd(a.oc + n * plane + (size_t)pi.cy * Nx + pi.cx, obytes); };
    auto s_park = [&](int n) { return srd(a.slots + fmm_slot(m, pat, n, p), kN2 * 8); };
    auto issue3 = [&](auto Q, const v4u& sp, const v4u& so, int vpo, int voo) {
      constexpr int q = decltype(Q)::value;
      dma_c<4096 * q>(sp, vpo, m0w + (q % 8) * 2048);
      dma_m<2 * q>(so, voo, m0w + (q % 8) * 2048 + 1024, os);
    };
    auto pre3 = [&](int n) {
      if constexpr (kRing) {
        const v4u sp = s_park(n), so = s_obj(n);
        const int lam = rf::opaque(tid) & 63;
        const int vpo = dma_off_park(lam, wv), voo = dma_off_obj(lam, wv, os);
        rf::sfor<0, 8>([&](auto Q) { issue3(Q, sp, so, vpo, voo); });
      }
    };
    // g_Ψ·N = v_p·(2 occ ∂ℓ/∂I/N), ∂ℓ/∂I = c1·u1 (+ c2·u2): the mini-batch's coefficients applied here
    {
      const float* cf = m.coef + (size_t)pi.m * kNCoef;
      const float c1 = occ2_n * (BOTH ? cf[0] : cf[m.ci]);
      const float c2 = BOTH ? occ2_n * cf[1] : 0.f;
      const Rsrc r_far = rsrc(a.slots + fmm_far(m, pat, p), kN2 * 8);
      const Rsrc r_u = rsrc(m.ubuf + (size_t)pat * kN2, kN2 * 4);
      const Rsrc r_u2 = rsrc(BOTH ? m.ubuf2 + (size_t)pat * kN2 : m.ubuf, BOTH ? kN2 * 4 : 0);
      const int vpk = 8 * tid, vu = 4 * tid;
      pipeline<16>(
          [&](auto C) {
            Ch4u t;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              t.x[r] = ld2(r_far, vpk, 2048 * (4 * C + r));
              t.u[r] = ld1(r_u, vu, 1024 * (4 * C + r));
              if constexpr (BOTH) t.u[r] = fmaf(c2, ld1(r_u2, vu, 1024 * (4 * C + r)), c1 * t.u[r]);
            }
            return t;
          },
          [&](auto C, const Ch4u& t) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[4 * C + r] = pscale(t.x[r], BOTH ? t.u[r] : c1 * t.u[r]);
              pin(v[4 * C + r]);
            }
          });
    }
    fft_inv(v, buf, lc, cd.wsign, [&] { pre3(Nz - 1); });
    // ------------------------------------------------ slices backwards
    for (int n = Nz - 1; n >= 0; --n) {
      const Rsrc r_slot = rsrc(a.slots + fmm_slot(m, pat, n, p), kN2 * 8);
      const float sc = n == Nz - 1 ? inv_n : 1.0f;   // far-field ortho scale once; propagation scaled in K
      if constexpr (kRing) {
        const v4u sp = s_park(n), so = s_obj(n);
        const int lam = rf::opaque(tid) & 63;
        const int vpo = dma_off_park(lam, wv), voo = dma_off_obj(lam, wv, os);
        const int io = obj_img(lam);
        const int vslot = 8 * ((rf::opaque(tid) & 1) * kN + fixed_of(rf::opaque(tid)));
        rf::sfor<0, 32>([&](auto Q) {
          constexpr int q = decltype(Q)::value;
          vm_wait<ring_wait_count(q, 2, 0, 8)>();
          const float2* sl = ringw + (q % 8) * 256;
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) {
            const int j = 2 * q + rb;
            const float2 ps = sl[rb * 64 + lam];
            const float2 O = sl[128 + rb * 64 + io];
            const float2 gv = pscale(v[j], sc);
            st2_stream(pcmc(gv, ps), r_slot, vslot, 2048 * j);   // slice n, mode p: g·conj(ψⁿ)
            v[j] = pcmc(gv, O);                                  // g·conj(O_n)
            pin(v[j]);
          }
          if constexpr (q + 8 < 32) issue3(std::integral_constant<int, q + 8>{}, sp, so, vpo, voo);
          __builtin_amdgcn_sched_barrier(0);
        });
        __syncthreads();   // every wave is done with its ring before the next exchange
      } else {
        const Rsrc r_obj = rsrc(a.oc + n * plane + (size_t)pi.cy * Nx + pi.cx, obytes);
        const int tq = rf::opaque(threadIdx.x);
        const int vslot = 8 * ((tq & 1) * kN + fixed_of(tq)), vobj = 8 * (64 * (tq & 1) * Nx + fixed_of(tq));
        const int ostr = rf::opaque(8 * Nx);
        pipeline<16>(
            [&](auto C) {
              Ch4x2 t;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int j = 4 * C + r;
                t.x[r] = ld2(r_slot, vslot, 2048 * j);
                t.y[r] = ld2(r_obj, vobj, ostr * j);
              }
              return t;
            },
            [&](auto C, const Ch4x2& t) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int j = 4 * C + r;
                const float2 gv = pscale(v[j], sc);
                st2_stream(pcmc(gv, t.x[r]), r_slot, vslot, 2048 * j);
                v[j] = pcmc(gv, t.y[r]);
                pin(v[j]);
              }
            });
      }
      if (n > 0) {
        fft_fwd(v, buf, lc, cd.wsign);
        prop_kc();
        fft_inv(v, buf, lc, cd.wsign, [&] { pre3(n - 1); });
      }
    }
    // ------------------------------------------------ probe / position gradient of mode p (× c_m)
    const bool first = job == j0 || p != p_prev;
    p_prev = p;
    if (!tail) continue;
    const int seg = p + w;
    float2* segs = a.segslab + (size_t)seg * kN2;
    const Rsrc r_slab_ld = rsrc(segs, first ? 0u : (unsigned)(kN2 * 8));
    const Rsrc r_slab_st = rsrc(segs, kN2 * 8);
    if (first && threadIdx.x == 0) a.segbid[seg] = p;
    const Rsrc r_fpk = rsrc(a.fpk + (size_t)p * kN2, kN2 * 8);
    if constexpr (SHIFT) {
      fft_fwd(v, buf, lc, cd.wsign);   // G = F(h), K layout
      const int vpk = rf::opaque(8 * tid);
      const int l0b = rf::opaque(tid) & 1;
      Ramp rc;
      rc.init(pi.sy, pi.sx, gy, l0b);
      float sim = 0.f, kim = 0.f;
      pipeline<16>(
          [&](auto C) {
            Ch4x2 t;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int k = 4 * C + r;
              t.x[r] = ld2(r_fpk, vpk, 2048 * k);
              t.y[r] = ld2(r_slab_ld, vpk, 2048 * k);
            }
            return t;
          },
          [&](auto C, const Ch4x2& t) {
            const float2 A = rc.a(C);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int k = 4 * C + r;
              const float2 W = pcm(A, rc.B[r]);
              const float2 FW = pcm(t.x[r], W);
              const float im = fmaf(FW.y, v[k].x, -FW.x * v[k].y);   // Im(F(P) W conj(G))
              sim += im;
              kim = fmaf((float)k, im, kim);
              st2(padd2(t.y[r], pcmc(v[k], W)), r_slab_st, vpk, 2048 * k);   // + conj(W) G
            }
          });
      float ds[2] = {gy * sim, fmaf(kim, inv_n, 0.5f * (float)(1 - l0b) * sim)};
      block_sum4<2>(ds, s_red);
      if (threadIdx.x == 0) {
        a.dsu[2 * job] = ds[0];
        a.dsu[2 * job + 1] = ds[1];
      }
    } else {
      const int vpk = rf::opaque(8 * tid);
      pipeline<16>(
          [&](auto C) {
            Ch4x2 t;
#pragma unroll
            for (int r = 0; r < 4; ++r) t.y[r] = ld2(r_slab_ld, vpk, 2048 * (4 * C + r));
            return t;
          },
          [&](auto C, const Ch4x2& t) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int j = 4 * C + r;
              st2(cadd(t.y[r], v[j]), r_slab_st, vpk, 2048 * j);   // + h (R layout)
            }
          });
    }
  }
}

// Per-mode probe-gradient spectra: block (x, y, p) sums the segments y, y + SPL, … whose mode is p
// (already scaled by c_m in k_fmm_adj) into part[p][y]; k_segslab_final (grid.y = p) adds the
// SPL partials in order and unpacks.  Fixed order: deterministic.
__global__ void k_segslab_reduce_modes(const float2* segslab, const int* segbid, int nseg, float2* part) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y, p = blockIdx.z;
  float2 acc = make_float2(0.f, 0.f);
  for (int g = y; g < nseg; g += kSegSplit) {
    if (segbid[g] != p) continue;
    acc = cadd(acc, segslab[(size_t)g * kN2 + e]);
  }
  part[((size_t)p * kSegSplit + y) * kN2 + e] = acc;
}

// d_shifts[s] += 2π/N² · Σ_p dsu[job (p, j)]  (c_m applied by k_fmm_adj; modes in order)
__global__ void k_shift_apply_modes(const int* idx, int n, int n_scans, int P, const float* dsu, float* d_shifts) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int s = min(max(idx[j], 0), n_scans - 1);
  float dy = 0.f, dx = 0.f;
  for (int p = 0; p < P; ++p) {
    dy += dsu[2 * ((size_t)p * n + j)];
    dx += dsu[2 * ((size_t)p * n + j) + 1];
  }
  constexpr float k = 6.283185307179586f / kN2;
  atomicAdd(d_shifts + 2 * s, dy * k);
  atomicAdd(d_shifts + 2 * s + 1, dx * k);
}

// Small calls: k_segslab_reduce_modes + k_segslab_final (every mode: blockIdx.y = p) and
// k_shift_apply_modes in ONE launch, the segment sums in exactly their order (bit-identical).
constexpr int kTailSegCap = 2048;   // segments (P + workgroups of k_fmm_adj) the LDS table holds
template <bool KL>
__global__ __launch_bounds__(256) void k_small_tail_modes(const float2* segslab, const int* segbid, int nseg,
                                                          float2* out, const int* idx, int n, int n_scans, int P,
                                                          const float* dsu, float* d_shifts,
                                                          const float2* twg = nullptr, float2* cols_out = nullptr) {
  constexpr int kSlabBlocks = kN2 / 256;
  if (blockIdx.x >= kSlabBlocks) {
    const int j = (blockIdx.x - kSlabBlocks) * 256 + threadIdx.x;
    if (blockIdx.y != 0 || !d_shifts || j >= n) return;
    const int s = min(max(idx[j], 0), n_scans - 1);
    float dy = 0.f, dx = 0.f;
    for (int p = 0; p < P; ++p) {
      dy += dsu[2 * ((size_t)p * n + j)];
      dx += dsu[2 * ((size_t)p * n + j) + 1];
    }
    constexpr float k = 6.283185307179586f / kN2;
    atomicAdd(d_shifts + 2 * s, dy * k);
    atomicAdd(d_shifts + 2 * s + 1, dx * k);
    return;
  }
  if (!out) return;
  // which segments are mode p's, as one bit each (ballots into LDS; read back into scalar
  // registers, so the per-segment test is a scalar branch); the kSegSplit partial chains are
  // independent, so each round issues the loads of all of them before adding: a missing segment
  // adds +0, which leaves a partial (never −0: it starts at +0) unchanged — the same sums, in the
  // same order, as k_segslab_reduce_modes + k_segslab_final
  static_assert(kSegSplit == 32, "one 32-bit mask word a round");
  __shared__ unsigned long long s_mask[kTailSegCap / 64];
  const int p = blockIdx.y;
  for (int g0 = 0; g0 < nseg; g0 += 256) {
    const int g = g0 + (int)threadIdx.x;
    const unsigned long long mk = __ballot(g < nseg && segbid[g] == p);
    if ((threadIdx.x & 63) == 0) s_mask[g0 / 64 + (threadIdx.x >> 6)] = mk;
  }
  __syncthreads();
  const int e = blockIdx.x * 256 + threadIdx.x;
  float2 part[kSegSplit];
#pragma unroll
  for (int y = 0; y < kSegSplit; ++y) part[y] = make_float2(0.f, 0.f);
  for (int g0 = 0; g0 < nseg; g0 += kSegSplit) {
    const unsigned mw = __builtin_amdgcn_readfirstlane((unsigned)(s_mask[g0 / 64] >> (g0 & 32)));
    if (!mw) continue;
    float2 t[kSegSplit];
#pragma unroll
    for (int y = 0; y < kSegSplit; ++y) {
      t[y] = make_float2(0.f, 0.f);
      if (mw & (1u << y)) t[y] = segslab[(size_t)(g0 + y) * kN2 + e];
    }
#pragma unroll
    for (int y = 0; y < kSegSplit; ++y) part[y] = cadd(part[y], t[y]);
  }
  float2 acc = make_float2(0.f, 0.f);
#pragma unroll
  for (int y = 0; y < kSegSplit; ++y) acc = cadd(acc, part[y]);
  if (KL && cols_out) {   // (block-uniform) the column pass of the probe gradient's inverse FFT
    tail_cols_ifft(acc, blockIdx.x, twg, cols_out + (size_t)p * kN2);
    return;
  }
  out[(size_t)p * kN2 + packed_rc<KL>(e & 255, e >> 8)] = acc;
}

}  // namespace f3
}  // namespace ptyx
