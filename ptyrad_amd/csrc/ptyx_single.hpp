// ptyx_single.hpp — fast path for P = O = Nz = 1 on an LDS array (N ≤ 128): the bench
// configuration (c2).  Included by ptyx_kernels.hip inside namespace ptyx.
//
// Every global value a fused hook needs (probe spectrum, object amplitude/phase, DP, probe
// slab) is prefetched into registers one FFT ahead, in exactly the point order the hook visits
// (PassMap), so its latency hides under the LDS passes.  The shifted probe ψ⁰ stays in
// registers between its two uses (same last-pass point order), and g ⊙ conj(O) goes straight
// into LDS for the probe-gradient FFT.  No per-workgroup global scratch.
//
// All prefetches are unconditional and every switch that decides whether a register array is
// written is a template parameter: a conditionally written array is loop-carried by the
// compiler and stays live (and spilled) across the whole persistent pattern loop.

template <int N, int NT>
__device__ __forceinline__ void prefetch_object(const KArgs& a, const PatternGeom& g, int tid,
                                                float (&oa)[PassMap<N, NT>::kLastSlots],
                                                float (&op)[PassMap<N, NT>::kLastSlots]) {
  using PM = PassMap<N, NT>;
#pragma unroll
  for (int s = 0; s < PM::kLastSlots; ++s) {
    int y, x;
    PM::last(tid, s, y, x);
    const size_t off = obj_off(a, 0, 0, g.cy + y, g.cx + x);
    oa[s] = a.obja[off];
    op[s] = a.objp[off];
  }
}

__device__ __forceinline__ float load_meas_nt(const KArgs& a, int s, int e, int N2) {
  const size_t off = (size_t)s * N2 + e;
  if (a.meas_f16) {
    const unsigned short h =
        __builtin_nontemporal_load(reinterpret_cast<const unsigned short*>(a.meas) + off);
    return __half2float(__ushort_as_half(h));
  } else {
    return __builtin_nontemporal_load(reinterpret_cast<const float*>(a.meas) + off);
  }
}

template <int N>
__device__ __forceinline__ int fftshift_index(int y, int x) {
  return ((y + N / 2) % N) * N + (x + N / 2) % N;
}

// ψ⁰ ⊙ O into the LDS array (ψ⁰ = F^-1(F(P) ⊙ W_b) or the probe), with hooks for ψ⁰.
template <int N, int NT, bool SHIFT, class OnPsi>
__device__ __forceinline__ void exit_wave(const KArgs& a, const LdsArray<N>& arr, const float2* tw,
                                          const float2* wy, const float2* wx, int tid,
                                          const float2 (&fp)[PassMap<N, NT>::kFirstSlots],
                                          const float (&oa)[PassMap<N, NT>::kLastSlots],
                                          const float (&op)[PassMap<N, NT>::kLastSlots], OnPsi&& on_psi) {
  using PM = PassMap<N, NT>;
  constexpr float inv_n2 = 1.0f / (float)(N * N);
  auto times_obj = [&](float2 w, int s) -> float2 {
    float sn, cs;
    phase_sincos(op[s], &sn, &cs);
    return cmul(w, make_float2(oa[s] * cs, oa[s] * sn));
  };
  if constexpr (SHIFT) {
    fft2d<N, NT, +1, false>(
        arr, tw, [&](int y, int x, float2, int s) { return cmul(cmul(fp[s], wy[y]), wx[x]); },
        [&](int, int, float2& v, int s) {
          const float2 w = cscale(v, inv_n2);
          on_psi(w, s);
          v = times_obj(w, s);
          return true;
        });
  } else {
#pragma unroll
    for (int s = 0; s < PM::kLastSlots; ++s) {
      int y, x;
      PM::last(tid, s, y, x);
      const float2 w = a.probe[y * N + x];
      on_psi(w, s);
      if (PM::last_active(tid, s)) arr.st(y, x, times_obj(w, s));
    }
    __syncthreads();
  }
}

template <int N, int NT, bool SHIFT>
__device__ __forceinline__ void prefetch_spectrum(const KArgs& a, int tid,
                                                  float2 (&fp)[PassMap<N, NT>::kFirstSlots]) {
  using PM = PassMap<N, NT>;
  if constexpr (SHIFT) {
#pragma unroll
    for (int s = 0; s < PM::kFirstSlots; ++s) {
      int y, x;
      PM::first(tid, s, y, x);
      fp[s] = a.Fp[y * N + x];
    }
  }
}

// Forward + per-pattern loss partial sums (SUMS) and/or dp_out.
template <int N, bool SHIFT, bool SUMS>
__global__ __launch_bounds__(Geo<N>::NT, Geo<N>::kWaves) void k_forward1(KArgs a) {
  constexpr int NT = Geo<N>::NT;
  constexpr int N2 = N * N;
  using PM = PassMap<N, NT>;
  constexpr int SF = PM::kFirstSlots, SL = PM::kLastSlots;
  constexpr float inv_n = 1.0f / (float)N;
  __shared__ float2 s_tw[N], s_wy[N], s_wx[N];
  __shared__ float s_red[(NT / 64) * 5];
  __shared__ float2 s_buf[LdsArray<N>::kElems];
  for (int i = threadIdx.x; i < N; i += NT) s_tw[i] = a.twg[i];
  const LdsArray<N> arr{s_buf};
  __syncthreads();
  const float occ = a.occu[0];

  for (int pat = blockIdx.x; pat < a.n_idx; pat += gridDim.x) {
    const PatternGeom g = pattern_geom(a, pat, N);
    const int tid = opaque_tid();
    float2 fp[SF];
    float oa[SL], op[SL];
    prefetch_spectrum<N, NT, SHIFT>(a, tid, fp);
    prefetch_object<N, NT>(a, g, tid, oa, op);
    if constexpr (SHIFT) build_ramps<N, NT>(g, s_wy, s_wx);
    float sp = 0.f;
    if constexpr (SUMS) {
      if (a.sparse_on) {
#pragma unroll
        for (int s = 0; s < SL; ++s) {
          const float ap = PM::last_active(tid, s) ? fabsf(op[s]) : 0.f;
          sp += a.sparse_n == 1 ? ap : powq(ap, (float)a.sparse_n);
        }
      }
    }
    exit_wave<N, NT, SHIFT>(a, arr, s_tw, s_wy, s_wx, tid, fp, oa, op, [](float2, int) {});
    float mv[SL];
    if constexpr (SUMS) {
#pragma unroll
      for (int s = 0; s < SL; ++s) {
        int y, x;
        PM::last(tid, s, y, x);
        mv[s] = load_meas_nt(a, g.m, fftshift_index<N>(y, x), N2);
      }
    }
    float sums[4] = {0.f, 0.f, 0.f, 0.f};
    fft2d<N, NT, -1, true>(
        arr, s_tw, [&](int, int, float2 v, int) { return v; },
        [&](int y, int x, float2& v, int s) {
          const float I = fmaf(occ, cabs2(cscale(v, inv_n)), kDpEps);
          if (a.dp_out) a.dp_out[(size_t)pat * N2 + fftshift_index<N>(y, x)] = I;
          if constexpr (SUMS) {
            const float M = mv[s];
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
          }
          return false;
        });
    if constexpr (SUMS) {
      float v5[5] = {sums[0], sums[1], sums[2], sums[3], sp};
      block_sum<NT, 5>(v5, s_red);
      if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a.psums[(size_t)pat * kNSum + i] = v5[i];
        a.psums[(size_t)pat * kNSum + kSumBase] = v5[4];
      }
    }
  }
}

// Adjoint (EXT: dL/dI from the caller).
template <int N, bool SHIFT, bool EXT>
__global__ __launch_bounds__(Geo<N>::NT, Geo<N>::kWaves) void k_adjoint1(KArgs a) {
  constexpr int NT = Geo<N>::NT;
  constexpr int N2 = N * N;
  using PM = PassMap<N, NT>;
  constexpr int SF = PM::kFirstSlots, SL = PM::kLastSlots;
  constexpr float inv_n = 1.0f / (float)N, inv_n2 = 1.0f / (float)N2;
  __shared__ float2 s_tw[N], s_wy[N], s_wx[N];
  __shared__ float s_red[(NT / 64) * 2];
  __shared__ float2 s_buf[LdsArray<N>::kElems];
  for (int i = threadIdx.x; i < N; i += NT) s_tw[i] = a.twg[i];
  const LdsArray<N> arr{s_buf};
  float2* slab = a.slab + (size_t)blockIdx.x * N2;
  if (a.need_probe)
    for (int e = opaque_tid(); e < N2; e += NT) slab[e] = make_float2(0.f, 0.f);
  __syncthreads();
  const float occ = a.occu[0];

  for (int pat = blockIdx.x; pat < a.n_idx; pat += gridDim.x) {
    const PatternGeom g = pattern_geom(a, pat, N);
    float c1 = 0.f, c2 = 0.f, csp = 0.f;
    if constexpr (!EXT) {
      int lo = 0, hi = a.n_batches;
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (a.boff[mid] <= pat) lo = mid;
        else hi = mid;
      }
      c1 = a.coef[(size_t)lo * kNCoef + 0];
      c2 = a.coef[(size_t)lo * kNCoef + 1];
      csp = a.sparse_on ? a.coef[(size_t)lo * kNCoef + 2] : 0.f;
    }
    const int tid = opaque_tid();
    float2 fp[SF];
    float oa[SL], op[SL];
    prefetch_spectrum<N, NT, SHIFT>(a, tid, fp);
    prefetch_object<N, NT>(a, g, tid, oa, op);
    if constexpr (SHIFT) build_ramps<N, NT>(g, s_wy, s_wx);
    float2 pb[SL];   // ψ⁰, kept in registers until the object-gradient pass
    exit_wave<N, NT, SHIFT>(a, arr, s_tw, s_wy, s_wx, tid, fp, oa, op,
                            [&](float2 w, int s) { pb[s] = w; });
    // DPs (or the external dL/dI) for the far-field points
    float mv[SL];
#pragma unroll
    for (int s = 0; s < SL; ++s) {
      int y, x;
      PM::last(tid, s, y, x);
      const int e = fftshift_index<N>(y, x);
      if constexpr (EXT) mv[s] = __builtin_nontemporal_load(a.dLdI_ext + (size_t)pat * N2 + e);
      else mv[s] = load_meas_nt(a, g.m, e, N2);
    }
    // far field → g_Ψ = 2 occ Ψ ∂L/∂I
    fft2d<N, NT, -1, true>(
        arr, s_tw, [&](int, int, float2 v, int) { return v; },
        [&](int, int, float2& v, int s) {
          const float2 Psi = cscale(v, inv_n);
          float dLdI;
          if constexpr (EXT) {
            dLdI = a.ext_scale * mv[s];
          } else {
            const float I = fmaf(occ, cabs2(Psi), kDpEps), M = mv[s], rI = 1.0f / I;
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
        });
    // back to real space; object gradient (scatter-add); g ⊙ conj(O) into LDS
    fft2d<N, NT, +1, true>(
        arr, s_tw, [&](int, int, float2 v, int) { return v; },
        [&](int y, int x, float2& v, int s) {
          const float2 gv = cscale(v, inv_n);
          const size_t off = obj_off(a, 0, 0, g.cy + y, g.cx + x);
          const float A = a.obja[off], ph = a.objp[off];
          float sn, cs;
          phase_sincos(ph, &sn, &cs);
          const float2 gO = cmulc(gv, pb[s]);                                   // conj(ψ⁰) g
          if (a.d_obja) atomicAdd(a.d_obja + off, fmaf(gO.x, cs, gO.y * sn));   // Re(g_O e^{-iφ})
          if (a.d_objp) {
            float dph = A * fmaf(gO.y, cs, -gO.x * sn);                          // Im(conj(O) g_O)
            if constexpr (!EXT) {
              if (csp != 0.f) {
                const float sg = ph > 0.f ? 1.f : (ph < 0.f ? -1.f : 0.f);
                dph += a.sparse_n == 1 ? csp * sg : csp * powq(fabsf(ph), (float)(a.sparse_n - 1)) * sg;
              }
            }
            atomicAdd(a.d_objp + off, dph);
          }
          v = cmulc(gv, make_float2(A * cs, A * sn));
          return true;
        });
    if constexpr (SHIFT) {
      if (a.need_probe || a.d_shifts) {
#pragma unroll
        for (int s = 0; s < SL; ++s) {
          int y, x;
          PM::last(tid, s, y, x);
        }
        float ds[2] = {0.f, 0.f};
        fft2d<N, NT, -1, true>(
            arr, s_tw, [&](int, int, float2 v, int) { return v; },
            [&](int y, int x, float2& G, int s) {
              const float2 W = cmul(s_wy[y], s_wx[x]);
              const float2 fpk = a.Fp[y * N + x];
              const float im = cmulc(cmul(fpk, W), G).y;                         // Im(conj(G) F(P) W)
              ds[0] = fmaf(6.283185307179586f * shift_g<N>(y), im, ds[0]);
              ds[1] = fmaf(6.283185307179586f * shift_g<N>(x), im, ds[1]);
              const float2 old = slab[y * N + x];
              if (a.need_probe) slab[y * N + x] = cadd(old, cmulc(G, W));          // Σ_b conj(W_b) F(g_Pb)
              return false;
            });
        if (a.d_shifts) {
          block_sum<NT, 2>(ds, s_red);
          if (threadIdx.x == 0) {
            atomicAdd(a.d_shifts + 2 * g.s, ds[0] * inv_n2);
            atomicAdd(a.d_shifts + 2 * g.s + 1, ds[1] * inv_n2);
          }
        }
      }
    } else {
      if (a.need_probe) {
#pragma unroll
        for (int s = 0; s < SL; ++s) {
          int y, x;
          PM::last(tid, s, y, x);
          if (PM::last_active(tid, s)) slab[y * N + x] = cadd(slab[y * N + x], arr.ld(y, x));
        }
        __syncthreads();
      }
    }
  }
}
