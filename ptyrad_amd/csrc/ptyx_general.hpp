// ptyx_general.hpp — the general engine's kernels (any P, O ≤ 32, Nz; every 2·3·5-smooth N in
// [32, 256]; f32 or f16 DPs).  One workgroup owns one pattern at a time and keeps the N×N wave in
// LDS (N ≤ 128) or in a per-workgroup global scratch pair (N > 128); the grid is persistent and
// walks the patterns with a grid stride.
//   k_probe_spectrum  F(P_p) once per call                       (image_proc.py:532, fft2(img))
//   k_forward         per pattern: shifted probe, object multiply, multislice, far field,
//                     Σ occ|Ψ|² + 1e-10, per-pattern loss partial sums      (models.py:422-436,
//                     forward.py:20-80, losses.py:45-46,70-71,101)
//   k_adjoint         per pattern: recompute forward (or read the far-field cache), dL/dI, back
//                     through the FFTs, object gradient scatter-add (fp32 atomics), probe-gradient
//                     partial (per-workgroup slab in k space), position gradient
//   k_probe_finalize  F^-1 of the k-space probe gradient → d_probe  (+=)
// plus k_forward1 / k_adjoint1 (ptyx_single.hpp, P = O = Nz = 1 on an LDS array).
//
// The kernels are instantiated per N in the ptyx_gen.hip translation units (GenLaunch below,
// one object per size group, compiled in parallel); ptyx_kernels.hip reaches them through the
// GenOps table of ptyx_genops.hpp and never instantiates them itself.
#pragma once
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include "ptyx.h"
#include "ptyx_common.hpp"
#include "ptyx_fft.hpp"
#include "ptyx_genops.hpp"

namespace ptyx {

// =====================================================================================
// Forward chain for one (pattern, p, o): leaves ψ_out = ψ^{Nz-1} ⊙ O_{Nz-1} in the array.
// STORE_PSI: store every ψ^n (n = 0..Nz-1, the wave ENTERING slice n) to psi[n·N²].
// SPARSE: accumulate Σ|φ|^n of every object pixel touched (once per pattern: caller gates).
// xs (optional): store Xⁿ = F(ψⁿ ⊙ Oⁿ), n = 0..Nz-2, for the propagator gradient.
template <int N, int NT, bool STORE_PSI, class Arr>
__device__ __forceinline__ void forward_chain(const KArgs& a, const Arr& arr, const float2* tw,
                                              const float2* wy, const float2* wx,
                                              const PatternGeom& g, int p, int o, float2* psi,
                                              bool sparse, float& sp_acc, float2* xs = nullptr,
                                              const float2* ty = nullptr, const float2* tx = nullptr,
                                              float2* psi0 = nullptr, bool reuse0 = false) {
  constexpr int N2 = N * N;
  constexpr float inv_n2 = 1.0f / (float)N2;
  auto mul_obj = [&](int n, int y, int x, float2 w) -> float2 {
    const size_t off = obj_off(a, o, n, g.cy + y, g.cx + x);
    const float A = a.obja[off], ph = a.objp[off];
    float sn, cs;
    phase_sincos(ph, &sn, &cs);
    if (sparse) {
      const float ap = fabsf(ph);
      sp_acc += a.sparse_n == 1 ? ap : powq(ap, (float)a.sparse_n);
    }
    return cmul(w, make_float2(A * cs, A * sn));
  };
  const float2* Fp = a.Fp + (size_t)p * N2;
  const float2* P0 = a.probe + (size_t)p * N2;
  // ψ^0: shifted probe F^-1(F(P) ⊙ W_b)   (image_proc.py:532) or the broadcast probe
  // psi0 (multi-object-mode calls): ψ⁰ of probe mode p depends on p only, so the o = 0 pass parks
  // it there and the o > 0 passes reload it instead of repeating the inverse FFT
  if (a.shift && reuse0) {
    for (int e = opaque_tid(); e < N2; e += NT) {
      const int y = e / N, x = e % N;
      const float2 w = psi0[e];
      if (STORE_PSI && psi != psi0) psi[e] = w;
      arr.st(y, x, mul_obj(0, y, x, w));
    }
    __syncthreads();
  } else if (a.shift) {
    fft2d<N, NT, +1, false>(
        arr, tw,
        [&](int y, int x, float2) { return cmul(cmul(Fp[y * N + x], wy[y]), wx[x]); },
        [&](int y, int x, float2& v) {
          const float2 w = cscale(v, inv_n2);
          if (STORE_PSI) psi[y * N + x] = w;
          if (psi0 && !(STORE_PSI && psi == psi0)) psi0[y * N + x] = w;
          v = mul_obj(0, y, x, w);
          return true;
        });
  } else {
    // broadcast probe: ψ⁰ = P_p, parked too when psi0 is the far-field cache's ψ⁰ slot (k_adjoint
    // reads it from there)
    for (int e = opaque_tid(); e < N2; e += NT) {
      const int y = e / N, x = e % N;
      const float2 w = P0[e];
      if (STORE_PSI) psi[e] = w;
      if (psi0 && !(STORE_PSI && psi == psi0)) psi0[e] = w;
      arr.st(y, x, mul_obj(0, y, x, w));
    }
    __syncthreads();
  }
  // multislice: ψ^{n} = F^-1(H ⊙ F(ψ^{n-1} ⊙ O_{n-1}))   (forward.py:60-63)
  for (int n = 1; n < a.Nz; ++n) {
    fft2d<N, NT, -1, true>(
        arr, tw, [&](int, int, float2 v) { return v; },
        [&](int y, int x, float2& v) {
          if (STORE_PSI && xs) xs[(size_t)(n - 1) * N2 + y * N + x] = v;
          v = cmul(v, a.H[y * N + x]);
          if (ty) v = cmul(v, cmul(ty[y], tx[x]));
          return true;
        });
    fft2d<N, NT, +1, true>(
        arr, tw, [&](int, int, float2 v) { return v; },
        [&](int y, int x, float2& v) {
          const float2 w = cscale(v, inv_n2);
          if (STORE_PSI) psi[(size_t)n * N2 + y * N + x] = w;
          v = mul_obj(n, y, x, w);
          return true;
        });
  }
}

// N = 256: forward_chain and the far-field FFT in 2·Nz + 1 stages instead of 4·Nz (shifted
// probes).  Every inverse FFT runs columns first, so each point-wise step sits between the two
// row DFTs of one g256_fstage: ×Oⁿ (and the ψⁿ stores) on natural rows, ×H on transposed rows
// (HT, read along them).  ff(y, x, v) is the far field's store hook (natural coordinates, like
// fft2d's post); returns the buffer of the scratch pair the far field went to (when ff stores).
template <bool STORE_PSI, class FF>
__device__ __forceinline__ float2* forward_far_g256(const KArgs& a, const GlobalPair<256>& arr, const float2* tw,
                                                    const float2* wy, const float2* wx, const PatternGeom& g, int p,
                                                    int o, float2* psi, bool sparse, float& sp_acc, const float2* ty,
                                                    const float2* tx, float2* psi0, bool reuse0, FF& ff) {
  constexpr int N = 256;
  constexpr int N2 = N * N;
  constexpr float inv_n2 = 1.0f / (float)N2;
  auto mul_obj = [&](int n, int y, int x, float2 w) -> float2 {
    const size_t off = obj_off(a, o, n, g.cy + y, g.cx + x);
    const float A = a.obja[off], ph = a.objp[off];
    float sn, cs;
    phase_sincos(ph, &sn, &cs);
    if (sparse) {
      const float ap = fabsf(ph);
      sp_acc += a.sparse_n == 1 ? ap : powq(ap, (float)a.sparse_n);
    }
    return cmul(w, make_float2(A * cs, A * sn));
  };
  float2* A = arr.a;
  float2* B = arr.b;
  float2* L = arr.lds;
  auto id_pre = [](int, int, float2 v) { return v; };
  auto store_all = [](int, int, float2&) { return true; };
  NoMid none;
  // first axis of F(ψ⁰ ⊙ O₀) → A (transposed)
  if (a.shift && reuse0) {   // ψ⁰ of p parked by the o = 0 pass
    auto pre = [&](int y, int x, float2 w) {
      if (STORE_PSI && psi != psi0) psi[y * N + x] = w;
      return mul_obj(0, y, x, w);
    };
    g256_fstage<-1, 0, false, true, true, true, false>(psi0, A, L, tw, pre, none, store_all);
  } else if (a.shift) {      // ψ⁰ = F⁻¹(F(P) ⊙ W_b): columns (transposed rows of F(P)ᵀ), then rows
    const float2* FpT = a.FpT + (size_t)p * N2;
    auto pre = [&](int y, int x, float2) { return cmul(cmul(FpT[x * N + y], wy[y]), wx[x]); };
    g256_fstage<+1, 0, true, true, false, true, false>(nullptr, B, L, tw, pre, none, store_all);
    auto mid = [&](int y, int x, float2& v) {
      const float2 w = cscale(v, inv_n2);
      if (STORE_PSI) psi[y * N + x] = w;
      if (psi0 && !(STORE_PSI && psi == psi0)) psi0[y * N + x] = w;
      v = mul_obj(0, y, x, w);
    };
    g256_fstage<+1, -1, false, false, false, true, false>(B, A, L, tw, id_pre, mid, store_all);
  } else {                   // broadcast probe
    const float2* P0 = a.probe + (size_t)p * N2;
    auto pre = [&](int y, int x, float2) {
      const float2 w = P0[y * N + x];
      if (STORE_PSI) psi[y * N + x] = w;
      if (psi0 && !(STORE_PSI && psi == psi0)) psi0[y * N + x] = w;
      return mul_obj(0, y, x, w);
    };
    g256_fstage<-1, 0, false, true, false, true, false>(nullptr, A, L, tw, pre, none, store_all);
  }
  // ψⁿ = F⁻¹(H ⊙ F(ψⁿ⁻¹ ⊙ Oⁿ⁻¹))   (forward.py:60-63)
  for (int n = 1; n < a.Nz; ++n) {
    auto mh = [&](int y, int x, float2& v) {
      v = cmul(v, a.HT[x * N + y]);
      if (ty) v = cmul(v, cmul(ty[y], tx[x]));
    };
    g256_fstage<-1, +1, true, false, false, true, false>(A, B, L, tw, id_pre, mh, store_all);
    auto mo = [&](int y, int x, float2& v) {
      const float2 w = cscale(v, inv_n2);
      if (STORE_PSI) psi[(size_t)n * N2 + y * N + x] = w;
      v = mul_obj(n, y, x, w);
    };
    g256_fstage<+1, -1, false, false, false, true, false>(B, A, L, tw, id_pre, mo, store_all);
  }
  // second axis of the far-field FFT, stored through ff
  g256_fstage<-1, 0, true, false, false, true, true>(A, B, L, tw, id_pre, none, ff);
  return B;
}

// per-position tilt ramps of pattern s: ty[y] = exp(i dz Ky[y] tan(θy/1e3)), tx likewise
// (the separable factor of exp(i dz (Ky tan θy + Kx tan θx)), models.py:330-356)
template <int N, int NT>
__device__ __forceinline__ void build_tilt_ramps(const KArgs& a, int s, float2* ty, float2* tx) {
  const float tty = tanf(a.ptilt[2 * s] / 1e3f), ttx = tanf(a.ptilt[2 * s + 1] / 1e3f);
  for (int k = opaque_tid(); k < 2 * N; k += NT) {
    const int kk = k % N;
    float sn, cs;
    sincosf(a.dz * a.kvec[kk] * (k < N ? tty : ttx), &sn, &cs);
    (k < N ? ty : tx)[kk] = make_float2(cs, sn);
  }
  __syncthreads();
}

// =====================================================================================
// k_probe_spectrum: Fp[p] = F(P_p)
template <int N>
__global__ __launch_bounds__(Geo<N>::NT, Geo<N>::kWaves) void k_probe_spectrum(KArgs a, float2* Fp_out) {
  constexpr int NT = Geo<N>::NT;
  constexpr bool LDS = Geo<N>::kLds;
  __shared__ float2 s_tw[N];
  __shared__ float2 s_buf[kFieldLds<N, LDS>];
  const int p = blockIdx.x;
  if constexpr (N == 256) {
    if (p == a.P) {   // the extra workgroup of a Nz > 1 call: HT = Hᵀ for the fused chains
      for (int e = threadIdx.x; e < N * N; e += NT) a.HT[(e % N) * N + e / N] = a.H[e];
      return;
    }
    if (!a.shift) return;
  }
  for (int i = threadIdx.x; i < N; i += NT) s_tw[i] = a.twg[i];
  __syncthreads();
  typename ArrayFor<N, LDS>::type arr;
  if constexpr (LDS) arr.p = s_buf;
  else {
    arr.a = a.scratch + (long long)blockIdx.x * a.scratch_stride;
    arr.b = arr.a + N * N;
    arr.lds = s_buf;
  }
  const float2* P0 = a.probe + (size_t)p * N * N;
  float2* out = Fp_out + (size_t)p * N * N;
  fft2d<N, NT, -1, false>(
      arr, s_tw, [&](int y, int x, float2) { return P0[y * N + x]; },
      [&](int y, int x, float2& v) {
        out[y * N + x] = v;
        if constexpr (N == 256) {
          if (a.FpT) a.FpT[(size_t)p * N * N + x * N + y] = v;
        }
        if constexpr (N == 128) {   // inverse of f3::packed_rc<true>: row y = fixed_of(t), column x = i + 64·(t & 1)
          if (a.fpk) a.fpk[(size_t)p * N * N + (x & 63) * 256 + ((x >> 6) | ((y & 31) << 1) | ((y >> 5) << 6))] = v;
        }
        return false;
      });
}

// =====================================================================================
// k_forward: I = Σ_{p,o} occ_o |S F_o ψ_out|² + eps per pattern; dp_out; loss partial sums.
// SINGLE: P·O == 1, the loss sums are taken straight from the far-field pass.
template <int N, bool SINGLE>
__global__ __launch_bounds__(Geo<N>::NT, Geo<N>::kWaves) void k_forward(KArgs a) {
  constexpr int NT = Geo<N>::NT;
  constexpr bool LDS = Geo<N>::kLds;
  constexpr int N2 = N * N;
  constexpr float inv_n = 1.0f / (float)N;
  __shared__ float2 s_tw[N], s_wy[N], s_wx[N], s_ty[N], s_tx[N];
  __shared__ float s_red[(NT / 64) * 4];
  __shared__ float2 s_buf[kFieldLds<N, LDS>];
  for (int i = threadIdx.x; i < N; i += NT) s_tw[i] = a.twg[i];
  typename ArrayFor<N, LDS>::type arr;
  if constexpr (LDS) arr.p = s_buf;
  else {
    arr.a = a.scratch + (long long)blockIdx.x * a.scratch_stride;
    arr.b = arr.a + N2;
    arr.lds = s_buf;
  }
  __syncthreads();
  const bool want_sums = a.psums != nullptr;
  const int PS = SINGLE ? 1 : a.msplit;   // jobs per pattern (probe-mode split)

  for (int job = blockIdx.x; job < a.n_idx * PS; job += gridDim.x) {
    const int pat = job / PS;
    const int pbeg = PS > 1 ? job % PS : 0, pend = PS > 1 ? pbeg + 1 : a.P;
    const PatternGeom g = pattern_geom(a, pat, N);
    if (a.shift) build_ramps<N, NT>(g, s_wy, s_wx);
    const bool tilt = a.ptilt != nullptr && a.Nz > 1;
    if (tilt) build_tilt_ramps<N, NT>(a, g.s, s_ty, s_tx);
    float sums[4] = {0.f, 0.f, 0.f, 0.f};
    auto add_sums = [&](float I, float M) {
      if (a.single_on) {
        const float Iq = powq(I, a.q1), Mq = powq(M, a.q1), d = Iq - Mq;
        sums[0] = fmaf(d, d, sums[0]);
        sums[1] += Mq;
      }
      if (a.pois_on) {
        const float Iq = powq(I, a.q2), Mq = powq(M, a.q2);
        sums[2] += Mq * fast_ln(Iq + a.eps2) - Iq;
        sums[3] += Mq;
      }
    };
    // split: this job's mode intensity Σ_o occ|Ψ_{p,o}|² in its own plane (k_forward_modesum adds)
    float* Ip = SINGLE ? nullptr : (PS > 1 ? a.Imodes + ((size_t)pat * PS + pbeg) * N2 : a.Ibuf + (size_t)pat * N2);
    float2* psi0 = scratch_psi<N>(a);   // this workgroup's ψ⁰ park (multi-object-mode calls)
    float2* cache = a.ffc ? a.ffc + (size_t)pat * a.ffc_per : nullptr;
    for (int p = pbeg; p < pend; ++p) {
      for (int o = 0; o < a.O; ++o) {
        const bool sparse = want_sums && a.sparse_on && p == 0;
        float sp = 0.f;
        float2* ffp = cache ? cache + (size_t)(p * a.O + o) * N2 : nullptr;
        const float occ = a.occu[o];
        const bool first = (p == pbeg && o == 0);
        // far field  Ψ = fftshift(F_o ψ_out)   (forward.py:79)
        auto ff = [&](int y, int x, float2& v) {
          if (ffp) ffp[y * N + x] = v;
          const float2 Psi = cscale(v, inv_n);
          const int e = ((y + N / 2) % N) * N + (x + N / 2) % N;
          const float c = occ * cabs2(Psi);
          if constexpr (SINGLE) {
            const float I = c + kDpEps;
            if (a.dp_out) a.dp_out[(size_t)pat * N2 + e] = I;
            if (want_sums) add_sums(I, meas_at(a, g.m, e, N2));
          } else {
            Ip[e] = first ? c : Ip[e] + c;
          }
          return false;
        };
        // the cache keeps every slice's ψⁿ of (p, o) for k_adjoint (Nz > 1), else ψ⁰ of p
        float2* psis = (cache && a.Nz > 1) ? cache + (size_t)(a.P * a.O + (p * a.O + o) * a.Nz) * N2 : nullptr;
        float2* park0 = psis ? (a.O > 1 ? psi0 : nullptr)
                             : cache ? cache + (size_t)(a.P * a.O + p) * N2 : (a.O > 1 ? psi0 : nullptr);
        const float2* ty = tilt ? s_ty : nullptr;
        const float2* tx = tilt ? s_tx : nullptr;
        if constexpr (N == 256) {
          if (psis) forward_far_g256<true>(a, arr, s_tw, s_wy, s_wx, g, p, o, psis, sparse, sp, ty, tx, park0, o > 0, ff);
          else forward_far_g256<false>(a, arr, s_tw, s_wy, s_wx, g, p, o, nullptr, sparse, sp, ty, tx, park0, o > 0, ff);
        } else {
          if (psis) forward_chain<N, NT, true>(a, arr, s_tw, s_wy, s_wx, g, p, o, psis, sparse, sp, nullptr, ty, tx, park0, o > 0);
          else forward_chain<N, NT, false>(a, arr, s_tw, s_wy, s_wx, g, p, o, nullptr, sparse, sp, nullptr, ty, tx, park0, o > 0);
          fft2d<N, NT, -1, true>(arr, s_tw, [&](int, int, float2 v) { return v; }, ff);
        }
        if (sparse) {
          float v1[1] = {sp};
          block_sum<NT, 1>(v1, s_red);
          if (threadIdx.x == 0) a.psums[(size_t)pat * kNSum + kSumBase + o] = v1[0];
        }
      }
    }
    if (PS > 1) {   // the mode planes are summed by k_forward_modesum
      __syncthreads();
      continue;
    }
    if constexpr (!SINGLE) {
      // epilogue: + eps, dp_out, loss sums (Ip was written by this workgroup; barrier above)
      for (int e = opaque_tid(); e < N2; e += NT) {
        const float I = Ip[e] + kDpEps;
        Ip[e] = I;
        if (a.dp_out) a.dp_out[(size_t)pat * N2 + e] = I;
        if (want_sums) add_sums(I, meas_at(a, g.m, e, N2));
      }
    }
    if (want_sums) {
      block_sum<NT, 4>(sums, s_red);
      if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a.psums[(size_t)pat * kNSum + i] = sums[i];
      }
    }
    __syncthreads();
  }
}

// Probe-mode split: I = Σ_p (mode planes, fixed order) + eps per pattern → Ibuf (k_adjoint reads
// it), dp_out and the loss partial sums — k_forward's epilogue, once all of a pattern's modes are in.
template <int N>
__global__ __launch_bounds__(Geo<N>::NT) void k_forward_modesum(KArgs a) {
  constexpr int NT = Geo<N>::NT;
  constexpr int N2 = N * N;
  __shared__ float s_red[(NT / 64) * 4];
  const int pat = blockIdx.x;
  const PatternGeom g = pattern_geom(a, pat, N);
  const bool want_sums = a.psums != nullptr;
  float sums[4] = {0.f, 0.f, 0.f, 0.f};
  // float4 units, up to four a thread in flight with every mode plane's loads issued together
  // (one workgroup a pattern: a split call is small, so latency, not bandwidth, bounds this)
  constexpr int N4 = N2 / 4;
  constexpr int U = (N4 + NT - 1) / NT;
  constexpr int UB = U < 4 ? U : 4;
  const float4* __restrict__ Im = reinterpret_cast<const float4*>(a.Imodes + (size_t)pat * a.msplit * N2);
  float4* __restrict__ Ip = reinterpret_cast<float4*>(a.Ibuf + (size_t)pat * N2);
  float* const dps = a.dp_out ? a.dp_out + (size_t)pat * N2 : nullptr;   // caller's array: maybe not 16-B aligned
  const bool dp4 = (reinterpret_cast<uintptr_t>(dps) & 15) == 0;
  const int tid = opaque_tid();
  auto add_sums = [&](float I1, int e) {
    const float M = meas_at(a, g.m, e, N2);
    if (a.single_on) {
      const float Iq = powq(I1, a.q1), Mq = powq(M, a.q1), d = Iq - Mq;
      sums[0] = fmaf(d, d, sums[0]);
      sums[1] += Mq;
    }
    if (a.pois_on) {
      const float Iq = powq(I1, a.q2), Mq = powq(M, a.q2);
      sums[2] += Mq * fast_ln(Iq + a.eps2) - Iq;
      sums[3] += Mq;
    }
  };
  if constexpr ((N2 & 3) != 0) {   // odd N: scalar units
    const float* Is = a.Imodes + (size_t)pat * a.msplit * N2;
    for (int e = tid; e < N2; e += NT) {
      float I = Is[e];
      for (int p = 1; p < a.msplit; ++p) I += Is[(size_t)p * N2 + e];
      I += kDpEps;
      a.Ibuf[(size_t)pat * N2 + e] = I;
      if (dps) dps[e] = I;
      if (want_sums) add_sums(I, e);
    }
  } else
  for (int b0 = 0; b0 < U; b0 += UB) {
    float4 I[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int e4 = tid + (b0 + u) * NT;
      I[u] = e4 < N4 ? Im[e4] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int p = 1; p < a.msplit; ++p) {
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int e4 = tid + (b0 + u) * NT;
        if (e4 < N4) {
          const float4 t = Im[(size_t)p * N4 + e4];
          I[u].x += t.x; I[u].y += t.y; I[u].z += t.z; I[u].w += t.w;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int e4 = tid + (b0 + u) * NT;
      if (e4 >= N4) continue;
      float4 v = I[u];
      v.x += kDpEps; v.y += kDpEps; v.z += kDpEps; v.w += kDpEps;
      Ip[e4] = v;
      if (dps) {
        if (dp4) {
          reinterpret_cast<float4*>(dps)[e4] = v;
        } else {
          dps[4 * e4] = v.x; dps[4 * e4 + 1] = v.y; dps[4 * e4 + 2] = v.z; dps[4 * e4 + 3] = v.w;
        }
      }
      if (want_sums) {
        const float Iv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) add_sums(Iv[c], 4 * e4 + c);
      }
    }
  }
  if (want_sums) {
    block_sum<NT, 4>(sums, s_red);
    if (threadIdx.x == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) a.psums[(size_t)pat * kNSum + i] = sums[i];
    }
  }
}

// =====================================================================================
// k_adjoint: gradients.  EXT: dL/dI supplied by the caller (ptyx_adjoint_dldi).
template <int N, bool SINGLE, bool EXT>
__global__ __launch_bounds__(Geo<N>::NT, Geo<N>::kWaves) void k_adjoint(KArgs a) {
  constexpr int NT = Geo<N>::NT;
  constexpr bool LDS = Geo<N>::kLds;
  constexpr int N2 = N * N;
  constexpr float inv_n = 1.0f / (float)N;
  constexpr float inv_n2 = 1.0f / (float)N2;
  __shared__ float2 s_tw[N], s_wy[N], s_wx[N], s_ty[N], s_tx[N];
  __shared__ float s_red[(NT / 64) * 2];
  __shared__ float2 s_buf[kFieldLds<N, LDS>];
  for (int i = threadIdx.x; i < N; i += NT) s_tw[i] = a.twg[i];
  typename ArrayFor<N, LDS>::type arr;
  if constexpr (LDS) arr.p = s_buf;
  else {
    arr.a = a.scratch + (long long)blockIdx.x * a.scratch_stride;
    arr.b = arr.a + N2;
    arr.lds = s_buf;
  }
  float2* psi = scratch_psi<N>(a);
  const float2* psi_rd = psi;   // ψⁿ the slice adjoints read: scratch, or the far-field cache's ψ⁰
  float2* gacc = psi + (size_t)a.Nz * N2;
  // compact slabs: workgroup w runs probe mode w % P only; its plane sits at mode w % P of the
  // slab of "virtual workgroup" w / P (the layout k_slab_reduce sums)
  const int cs = a.cslab ? (int)(blockIdx.x % a.P) : -1;
  float2* slab = a.slab + (size_t)(a.cslab ? blockIdx.x / a.P : blockIdx.x) * a.P * N2;
  // propagator gradient: dL/dH += Σ_{p,o,n<Nz-1} conj(Xⁿ) ⊙ F(g^{n+1}) / N²  (ψ^{n+1} = F⁻¹(H Xⁿ))
  float2* xs = (a.hslab || a.d_tilts || a.d_dz) ? gacc + N2 : nullptr;
  float2* hsl = a.hslab ? a.hslab + (size_t)blockIdx.x * N2 : nullptr;
  if (a.need_probe) {
    float2* z = cs >= 0 ? slab + (size_t)cs * N2 : slab;
    const int nz = cs >= 0 ? N2 : a.P * N2;
    for (int e = threadIdx.x; e < nz; e += NT) z[e] = make_float2(0.f, 0.f);
  }
  if (hsl)
    for (int e = threadIdx.x; e < N2; e += NT) hsl[e] = make_float2(0.f, 0.f);
  __syncthreads();

  const int PS = (SINGLE || EXT) ? 1 : a.msplit;   // jobs per pattern (probe-mode split)
  for (int job = blockIdx.x; job < a.n_idx * PS; job += gridDim.x) {
    const int pat = job / PS;
    const int pbeg = PS > 1 ? job % PS : 0, pend = PS > 1 ? pbeg + 1 : a.P;
    const PatternGeom g = pattern_geom(a, pat, N);
    float c1 = 0.f, c2 = 0.f;
    int m = 0;
    if constexpr (!EXT) {
      int lo = 0, hi = a.n_batches;  // batch containing pat: boff[m] <= pat < boff[m+1]
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (a.boff[mid] <= pat) lo = mid;
        else hi = mid;
      }
      m = lo;
      c1 = a.coef[(size_t)m * kNCoef + 0];
      c2 = a.coef[(size_t)m * kNCoef + 1];
    }
    if (a.shift) build_ramps<N, NT>(g, s_wy, s_wx);
    const bool tilt = a.ptilt != nullptr && a.Nz > 1;
    if (tilt) build_tilt_ramps<N, NT>(a, g.s, s_ty, s_tx);
    float ds[2] = {0.f, 0.f};
    float dt[2] = {0.f, 0.f};   // Σ_k Ky (resp. Kx) · Re(i conj(g_Hb) H_b)
    const float* Ip = (SINGLE || EXT) ? nullptr : a.Ibuf + (size_t)pat * N2;

    for (int p = pbeg; p < pend; ++p) {
      for (int o = 0; o < a.O; ++o) {
        const float occ = a.occu[o];
        const float csp = (!EXT && a.sparse_on && p == 0) ? a.coef[(size_t)m * kNCoef + 2 + o] : 0.f;
        float dummy = 0.f;
        // far field → g_Ψ = 2 occ Ψ ∂L/∂I  (left in natural FFT order)
        auto ff_post = [&](int y, int x, float2& v) {
              const float2 Psi = cscale(v, inv_n);
              const int e = ((y + N / 2) % N) * N + (x + N / 2) % N;
              float dLdI;
              if constexpr (EXT) {
                dLdI = a.ext_scale * a.dLdI_ext[(size_t)pat * N2 + e];
              } else {
                const float I = SINGLE ? fmaf(occ, cabs2(Psi), kDpEps) : Ip[e];
                const float M = meas_at(a, g.m, e, N2);
                const float rI = 1.0f / I;
                dLdI = 0.f;
                if (a.single_on) {
                  const float Iq = powq(I, a.q1), Mq = powq(M, a.q1);
                  dLdI = c1 * (Iq - Mq) * a.q1 * Iq * rI;
                }
                if (a.pois_on) {
                  const float Iq = powq(I, a.q2), Mq = powq(M, a.q2);
                  dLdI += c2 * (Mq / (Iq + a.eps2) - 1.0f) * a.q2 * Iq * rI;
                }
              }
              v = cscale(Psi, 2.0f * occ * dLdI);
              return true;
            };
        // adjoint of slice n: g_O += conj(ψ^n) g → dA, dφ; g ← g ⊙ conj(O_n)
        auto slice_adj = [&](int n, int y, int x, float2 gv) -> float2 {
          const size_t off = obj_off(a, o, n, g.cy + y, g.cx + x);
          const float A = a.obja[off], ph = a.objp[off];
          float sn, cs;
          phase_sincos(ph, &sn, &cs);
          const float2 Ov = make_float2(A * cs, A * sn);
          const float2 gO = cmulc(gv, psi_rd[(size_t)n * N2 + y * N + x]);
          if (a.d_obja) atomicAdd(a.d_obja + off, fmaf(gO.x, cs, gO.y * sn));   // Re(g_O e^{-iφ})
          if (a.d_objp) {
            float dph = fmaf(gO.y, Ov.x, -gO.x * Ov.y);                          // Im(conj(O) g_O)
            if (csp != 0.f) {
              const float sg = ph > 0.f ? 1.f : (ph < 0.f ? -1.f : 0.f);
              dph += a.sparse_n == 1 ? csp * sg : csp * powq(fabsf(ph), (float)(a.sparse_n - 1)) * sg;
            }
            atomicAdd(a.d_objp + off, dph);
          }
          return cmulc(gv, Ov);
        };
        auto acc_probe = [&](int y, int x, float2 gv) {
          const int e = y * N + x;
          gacc[e] = (o == 0) ? gv : cadd(gacc[e], gv);
        };
        const float2* cache = (!EXT && a.ffc) ? a.ffc + (size_t)pat * a.ffc_per : nullptr;
        // k_forward left F(ψ_out) of this (p, o) and ψ⁰ of p (Nz = 1) or every slice's ψⁿ of (p, o)
        // (Nz > 1) in the cache: no recomputed forward
        const float2* psi_c = cache ? cache + (size_t)(a.P * a.O + (a.Nz > 1 ? (p * a.O + o) * a.Nz : p)) * N2 : nullptr;
        if constexpr (N == 256) {
          if (!xs) {   // fused stages (forward_far_g256): 2·Nz + 1 round trips per mode (2 at Nz = 1) instead of 4·Nz - 1
            const int Nz = a.Nz;
            float2* A = arr.a;
            float2* B = arr.b;
            auto id_pre = [](int, int, float2 v) { return v; };
            auto store_all = [](int, int, float2&) { return true; };
            NoMid none;
            // g_Ψ: the cached far field (ff_post applied on the way in) or the recomputed one
            const float2* src0;
            if (cache) {
              psi_rd = psi_c;
              src0 = cache + (size_t)(p * a.O + o) * N2;
            } else {
              psi_rd = psi;
              src0 = forward_far_g256<true>(a, arr, s_tw, s_wy, s_wx, g, p, o, psi, false, dummy,
                                            tilt ? s_ty : nullptr, tilt ? s_tx : nullptr, psi, o > 0, ff_post);
            }
            auto pre = [&](int y, int x, float2 v) {
              if (cache) ff_post(y, x, v);
              return v;
            };
            if (Nz == 1) {   // F_o⁻¹ rows, then columns with the slice adjoint in the store hook
              g256_fstage<+1, 0, false, true, true, true, false>(src0, A, arr.lds, s_tw, pre, none, store_all);
              auto post0 = [&](int y, int x, float2& v) {
                acc_probe(y, x, slice_adj(0, y, x, cscale(v, inv_n)));
                return false;
              };
              g256_fstage<+1, 0, true, false, false, true, true>(A, B, arr.lds, s_tw, id_pre, none, post0);
              continue;
            }
            // Nz > 1: transpose g_Ψ into A, so the slice adjoints land on natural rows below
            g256_fstage<0, 0, false, true, true, true, false>(src0, A, arr.lds, s_tw, pre, none, store_all);
            // F_o⁻¹ columns first; each slice adjoint sits between its inverse rows and the next
            // forward rows, each conj(H) between forward columns and inverse columns
            g256_fstage<+1, 0, true, false, false, true, false>(A, B, arr.lds, s_tw, id_pre, none, store_all);
            for (int n = Nz - 1; n >= 1; --n) {
              const float sc = n == Nz - 1 ? inv_n : inv_n2;
              auto ma = [&](int y, int x, float2& v) { v = slice_adj(n, y, x, cscale(v, sc)); };
              g256_fstage<+1, -1, false, false, false, true, false>(B, A, arr.lds, s_tw, id_pre, ma, store_all);
              auto mh = [&](int y, int x, float2& v) {
                float2 Hb = a.HT[x * N + y];
                if (tilt) Hb = cmul(Hb, cmul(s_ty[y], s_tx[x]));
                v = cmulc(v, Hb);
              };
              g256_fstage<-1, +1, true, false, false, true, false>(A, B, arr.lds, s_tw, id_pre, mh, store_all);
            }
            auto m0 = [&](int y, int x, float2& v) { acc_probe(y, x, slice_adj(0, y, x, cscale(v, inv_n2))); };
            g256_fstage<+1, 0, false, false, false, false, false>(B, nullptr, arr.lds, s_tw, id_pre, m0, store_all);
            continue;
          }
        }
        if (cache) {
          psi_rd = psi_c;
          const float2* ffp = cache + (size_t)(p * a.O + o) * N2;
          for (int e = opaque_tid(); e < N2; e += NT) {
            const int y = e / N, x = e % N;
            float2 v = ffp[e];
            ff_post(y, x, v);
            arr.st(y, x, v);
          }
          __syncthreads();
        } else {
          psi_rd = psi;
          forward_chain<N, NT, true>(a, arr, s_tw, s_wy, s_wx, g, p, o, psi, false, dummy, xs,
                                     tilt ? s_ty : nullptr, tilt ? s_tx : nullptr, psi, o > 0);
          fft2d<N, NT, -1, true>(arr, s_tw, [&](int, int, float2 v) { return v; }, ff_post);
        }
        const int Nz = a.Nz;
        // F_o^-1 (ortho adjoint of F_o, fftshift undone by the index map above)
        fft2d<N, NT, +1, true>(
            arr, s_tw, [&](int, int, float2 v) { return v; },
            [&](int y, int x, float2& v) {
              const float2 gv = slice_adj(Nz - 1, y, x, cscale(v, inv_n));
              if (Nz == 1) {
                acc_probe(y, x, gv);
                return false;
              }
              v = gv;
              return true;
            });
        for (int n = Nz - 2; n >= 0; --n) {  // adjoint of F^-1 H F is F^-1 conj(H) F
          fft2d<N, NT, -1, true>(
              arr, s_tw, [&](int, int, float2 v) { return v; },
              [&](int y, int x, float2& v) {
                const int e = y * N + x;
                float2 Hb = a.H[e];
                if (tilt) {
                  const float2 r = cmul(s_ty[y], s_tx[x]);
                  Hb = cmul(Hb, r);
                  if (xs) {
                    const float2 q = cscale(cmulc(v, xs[(size_t)n * N2 + e]), inv_n2);   // g_{H_b}
                    if (hsl) hsl[e] = cadd(hsl[e], cmulc(q, r));                        // conj(r) g_{H_b}
                    if (a.d_tilts || a.d_dz) {
                      const float w = -cmulc(Hb, q).y;   // Re(i conj(q) H_b) = -Im(H_b conj(q))
                      dt[0] = fmaf(a.kvec[y], w, dt[0]);
                      dt[1] = fmaf(a.kvec[x], w, dt[1]);
                    }
                  }
                } else if (hsl) {
                  hsl[e] = cadd(hsl[e], cscale(cmulc(v, xs[(size_t)n * N2 + e]), inv_n2));
                }
                v = cmulc(v, Hb);
                return true;
              });
          fft2d<N, NT, +1, true>(
              arr, s_tw, [&](int, int, float2 v) { return v; },
              [&](int y, int x, float2& v) {
                const float2 gv = slice_adj(n, y, x, cscale(v, inv_n2));
                if (n == 0) {
                  acc_probe(y, x, gv);
                  return false;
                }
                v = gv;
                return true;
              });
        }
      }
      // probe mode p: g_{P_b} = Σ_o g (in gacc)
      if (a.shift) {
        if (a.need_probe || a.d_shifts) {
          const float2* Fp = a.Fp + (size_t)p * N2;
          float2* sl = slab + (size_t)p * N2;
          fft2d<N, NT, -1, false>(
              arr, s_tw, [&](int y, int x, float2) { return gacc[y * N + x]; },
              [&](int y, int x, float2& G) {
                const int e = y * N + x;
                const float2 W = cmul(s_wy[y], s_wx[x]);
                const float2 FW = cmul(Fp[e], W);
                const float im = cmulc(FW, G).y;  // Im(conj(G) F(P) W)
                ds[0] = fmaf(6.283185307179586f * shift_g<N>(y), im, ds[0]);
                ds[1] = fmaf(6.283185307179586f * shift_g<N>(x), im, ds[1]);
                if (a.need_probe) sl[e] = cadd(sl[e], cmulc(G, W));  // Σ_b conj(W_b) F(g_Pb)
                return false;
              });
        }
      } else if (a.need_probe) {
        float2* sl = slab + (size_t)p * N2;
        for (int e = opaque_tid(); e < N2; e += NT) sl[e] = cadd(sl[e], gacc[e]);
        __syncthreads();
      }
    }
    if (a.shift && a.d_shifts) {
      block_sum<NT, 2>(ds, s_red);
      if (threadIdx.x == 0) {
        atomicAdd(a.d_shifts + 2 * g.s, ds[0] * inv_n2);
        atomicAdd(a.d_shifts + 2 * g.s + 1, ds[1] * inv_n2);
      }
    }
    if (tilt && (a.d_tilts || a.d_dz)) {
      __syncthreads();
      block_sum<NT, 2>(dt, s_red);
      if (threadIdx.x == 0) {   // ∂/∂θ (mrad) of tan(θ/1e3) = sec²(θ/1e3)/1e3
        const float ay = a.ptilt[2 * g.s] / 1e3f, ax = a.ptilt[2 * g.s + 1] / 1e3f;
        const float cy = cosf(ay), cx = cosf(ax);
        if (a.d_tilts) {
          atomicAdd(a.d_tilts + 2 * g.s, dt[0] * a.dz / (cy * cy) / 1e3f);
          atomicAdd(a.d_tilts + 2 * g.s + 1, dt[1] * a.dz / (cx * cx) / 1e3f);
        }
        if (a.d_dz) atomicAdd(a.d_dz, fmaf(dt[0], tanf(ay), dt[1] * tanf(ax)));   // ∂/∂dz of the ramps
      }
    }
    __syncthreads();
  }
}

// d_probe[p] += F^-1(G_p) (shift) or G_p (no shift)
template <int N>
__global__ __launch_bounds__(Geo<N>::NT, Geo<N>::kWaves) void k_probe_finalize(KArgs a, const float2* G, float2* d_probe) {
  constexpr int NT = Geo<N>::NT;
  constexpr bool LDS = Geo<N>::kLds;
  constexpr int N2 = N * N;
  constexpr float inv_n2 = 1.0f / (float)N2;
  __shared__ float2 s_tw[N];
  __shared__ float2 s_buf[kFieldLds<N, LDS>];
  for (int i = threadIdx.x; i < N; i += NT) s_tw[i] = a.twg[i];
  __syncthreads();
  const int p = blockIdx.x;
  const float2* Gp = G + (size_t)p * N2;
  float2* dp = d_probe + (size_t)p * N2;
  if (!a.shift) {
    for (int e = opaque_tid(); e < N2; e += NT) dp[e] = cadd(dp[e], Gp[e]);
    return;
  }
  typename ArrayFor<N, LDS>::type arr;
  if constexpr (LDS) arr.p = s_buf;
  else {
    arr.a = a.scratch + (long long)blockIdx.x * a.scratch_stride;
    arr.b = arr.a + N2;
    arr.lds = s_buf;
  }
  fft2d<N, NT, +1, false>(
      arr, s_tw, [&](int y, int x, float2) { return Gp[y * N + x]; },
      [&](int y, int x, float2& v) {
        const int e = y * N + x;
        dp[e] = cadd(dp[e], cscale(v, inv_n2));
        return false;
      });
}

// ------------------------------------------------------------ multi-workgroup probe transforms
// The per-call probe spectrum F(P_p) and the probe-gradient inverse F⁻¹(G_p) as two launches of
// N/kSpecLines workgroups per mode (rows, then columns, kSpecLines lines each through LDS) instead
// of one workgroup per mode: a lone N² transform on one CU is latency-bound, and at the reference's
// default cadence (one 32-pattern call per optimizer step) both sit on every step's critical path.
constexpr int kSpecLines = 8;
constexpr int kSpecThreads = 256;

// rows of src (plane p at src + p·N²) → tmp, DIR transform, natural order
template <int N, int DIR>
__global__ __launch_bounds__(kSpecThreads) void k_lines_rows(const float2* src, float2* tmp, const float2* twg) {
  using LT = LineTile<N, kSpecLines>;
  using P1 = Plan1D<N>;
  __shared__ float2 s_tw[N];
  __shared__ float2 T[LT::kElems];
  const int l0 = blockIdx.x * kSpecLines, p = blockIdx.y;
  const float2* s = src + (size_t)p * N * N;
  float2* d = tmp + (size_t)p * N * N;
  for (int i = threadIdx.x; i < N; i += kSpecThreads) s_tw[i] = twg[i];
  const int nl = min(kSpecLines, N - l0);
  for (int e = threadIdx.x; e < nl * N; e += kSpecThreads) T[LT::off(e / N, e % N)] = s[(size_t)(l0 + e / N) * N + e % N];
  __syncthreads();
  line_pass<N, kSpecThreads, P1::R1, 1, DIR, kSpecLines>(T, s_tw, nl);
  line_pass<N, kSpecThreads, P1::R2, P1::R1, DIR, kSpecLines>(T, s_tw, nl);
  for (int e = threadIdx.x; e < nl * N; e += kSpecThreads) d[(size_t)(l0 + e / N) * N + e % N] = T[LT::off(e / N, e % N)];
}

// columns of tmp, DIR transform; KIND 0: the probe spectrum — Fp natural, plus the K-packed copy
// of the register engines at N = 128 (k_probe_spectrum's fpk layout); KIND 1: d_probe += v / N²
template <int N, int DIR, int KIND>
__global__ __launch_bounds__(kSpecThreads) void k_lines_cols(const float2* tmp, float2* out, float2* fpk,
                                                             const float2* twg) {
  using LT = LineTile<N, kSpecLines>;
  using P1 = Plan1D<N>;
  __shared__ float2 s_tw[N];
  __shared__ float2 T[LT::kElems];
  const int c0 = blockIdx.x * kSpecLines, p = blockIdx.y;
  const float2* s = tmp + (size_t)p * N * N;
  for (int i = threadIdx.x; i < N; i += kSpecThreads) s_tw[i] = twg[i];
  const int nc = min(kSpecLines, N - c0);
  for (int e = threadIdx.x; e < nc * N; e += kSpecThreads) {
    const int y = e / nc, c = e % nc;
    T[LT::off(c, y)] = s[(size_t)y * N + c0 + c];
  }
  __syncthreads();
  line_pass<N, kSpecThreads, P1::R1, 1, DIR, kSpecLines>(T, s_tw, nc);
  line_pass<N, kSpecThreads, P1::R2, P1::R1, DIR, kSpecLines>(T, s_tw, nc);
  constexpr float inv_n2 = 1.0f / (float)(N * N);
  for (int e = threadIdx.x; e < nc * N; e += kSpecThreads) {
    const int y = e / nc, c = e % nc, x = c0 + c;
    const float2 v = T[LT::off(c, y)];
    if constexpr (KIND == 0) {
      out[(size_t)p * N * N + y * N + x] = v;
      if constexpr (N == 128) {
        if (fpk) fpk[(size_t)p * N * N + (x & 63) * 256 + ((x >> 6) | ((y & 31) << 1) | ((y >> 5) << 6))] = v;
      }
    } else {
      float2* dp = out + (size_t)p * N * N + y * N + x;
      *dp = cadd(*dp, cscale(v, inv_n2));
    }
  }
}

#include "ptyx_single.hpp"

// ------------------------------------------------------------------- per-N launchers
template <int N>
struct GenLaunch {
  static constexpr int NT = Geo<N>::NT;
  static void spectrum(const KArgs& a, int nblk, float2* Fp, hipStream_t st) {
    hipLaunchKernelGGL(k_probe_spectrum<N>, dim3(nblk), dim3(NT), 0, st, a, Fp);
  }
  // one_mode: P·O = 1;  single: P·O·Nz = 1 (the LDS register-prefetch kernels)
  static void forward(const KArgs& a, int grid, bool one_mode, bool single, hipStream_t st) {
    if constexpr (Geo<N>::kLds) {
      if (single) {
        const bool sums = a.psums != nullptr;
        if (a.shift && sums) hipLaunchKernelGGL((k_forward1<N, true, true>), dim3(grid), dim3(NT), 0, st, a);
        else if (a.shift) hipLaunchKernelGGL((k_forward1<N, true, false>), dim3(grid), dim3(NT), 0, st, a);
        else if (sums) hipLaunchKernelGGL((k_forward1<N, false, true>), dim3(grid), dim3(NT), 0, st, a);
        else hipLaunchKernelGGL((k_forward1<N, false, false>), dim3(grid), dim3(NT), 0, st, a);
        return;
      }
    }
    if (one_mode) hipLaunchKernelGGL((k_forward<N, true>), dim3(grid), dim3(NT), 0, st, a);
    else hipLaunchKernelGGL((k_forward<N, false>), dim3(grid), dim3(NT), 0, st, a);
  }
  static void modesum(const KArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(k_forward_modesum<N>, dim3(a.n_idx), dim3(NT), 0, st, a);
  }
  static void adjoint(const KArgs& a, int grid, bool one_mode, bool single, bool ext, hipStream_t st) {
    if constexpr (Geo<N>::kLds) {
      if (single) {
        const dim3 gr(grid), bl(NT);
        if (a.shift && ext) hipLaunchKernelGGL((k_adjoint1<N, true, true>), gr, bl, 0, st, a);
        else if (a.shift) hipLaunchKernelGGL((k_adjoint1<N, true, false>), gr, bl, 0, st, a);
        else if (ext) hipLaunchKernelGGL((k_adjoint1<N, false, true>), gr, bl, 0, st, a);
        else hipLaunchKernelGGL((k_adjoint1<N, false, false>), gr, bl, 0, st, a);
        return;
      }
    }
    if (ext) hipLaunchKernelGGL((k_adjoint<N, false, true>), dim3(grid), dim3(NT), 0, st, a);
    else if (one_mode) hipLaunchKernelGGL((k_adjoint<N, true, false>), dim3(grid), dim3(NT), 0, st, a);
    else hipLaunchKernelGGL((k_adjoint<N, false, false>), dim3(grid), dim3(NT), 0, st, a);
  }
  static void probe_finalize(const KArgs& a, int nblk, const float2* G, float2* d_probe, hipStream_t st) {
    hipLaunchKernelGGL(k_probe_finalize<N>, dim3(nblk), dim3(NT), 0, st, a, G, d_probe);
  }
  // the two-launch forms (k_lines_rows / k_lines_cols), tmp: P·N² float2 of scratch
  static void spectrum_lines(const float2* probe, int P, float2* Fp, float2* fpk, float2* tmp, const float2* twg,
                             hipStream_t st) {
    const dim3 gr((N + kSpecLines - 1) / kSpecLines, P), bl(kSpecThreads);
    hipLaunchKernelGGL((k_lines_rows<N, -1>), gr, bl, 0, st, probe, tmp, twg);
    hipLaunchKernelGGL((k_lines_cols<N, -1, 0>), gr, bl, 0, st, tmp, Fp, fpk, twg);
  }
  static void spectrum_cols(const float2* tmp, int P, float2* Fp, float2* fpk, const float2* twg, hipStream_t st) {
    const dim3 gr((N + kSpecLines - 1) / kSpecLines, P), bl(kSpecThreads);
    hipLaunchKernelGGL((k_lines_cols<N, -1, 0>), gr, bl, 0, st, tmp, Fp, fpk, twg);
  }
  static void probe_finalize_lines(const float2* G, int P, float2* d_probe, float2* tmp, const float2* twg,
                                   hipStream_t st) {
    const dim3 gr((N + kSpecLines - 1) / kSpecLines, P), bl(kSpecThreads);
    hipLaunchKernelGGL((k_lines_rows<N, +1>), gr, bl, 0, st, G, tmp, twg);
    hipLaunchKernelGGL((k_lines_cols<N, +1, 1>), gr, bl, 0, st, tmp, d_probe, nullptr, twg);
  }
  // LDS-limited residency (160 KiB per CU, 2048 threads) of the workgroup-resident FFT kernels
  static constexpr int blocks_per_cu() { return Geo<N>::kResident; }
  static const GenOps* ops() {
    static const GenOps o{N, NT, Geo<N>::kLds, blocks_per_cu(), &spectrum, &forward, &modesum, &adjoint, &probe_finalize,
                          &spectrum_lines, &probe_finalize_lines, &spectrum_cols};
    return &o;
  }
};

}  // namespace ptyx
