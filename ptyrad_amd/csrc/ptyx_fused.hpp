// ptyx_fused.hpp — one-pass forward/loss/adjoint for P = O = Nz = 1, N ≤ 128 (the bench
// configuration, c2), and the object-gradient gather that completes it.  Included by
// ptyx_kernels.hip inside namespace ptyx.
//
// Why this shape (measurements in DESIGN.md §4):
//  * fp32 scatter-add atomics execute at the memory side at ≈1.0 TB/s for the whole chip
//    (tools/atomicbench.hip), i.e. ≥ 8.4 ms per c2 step for 128 KiB of object gradient per
//    pattern, and every later load of the issuing wave queues behind them (vmcnt is in-order).
//    Instead each pattern PLAIN-STORES its unit-coefficient object-gradient wave
//    g_O = conj(ψ⁰)·g to a per-pattern scratch slot, and k_obj_gather reduces the slots per
//    object tile in pattern order: no atomics, bitwise-deterministic object gradients.
//  * Everything downstream of ∂L/∂I is linear in the mini-batch coefficient c_m
//    (c_single or c_poissn, losses.py:45-47 / 70-72), so the far-field epilogue writes
//    g_Ψ / c_m straight into LDS (no separate g_Ψ pass) and the object part of the adjoint
//    runs before the batch is complete.  Only the probe slab and the position gradient need
//    c_m: the batch wait sits just before that last FFT, ≈ one inverse FFT after this
//    pattern's own arrival, so it rarely blocks.
//  * Patterns are dealt round-robin (pattern j → workgroup j mod G).  With all G workgroups
//    co-resident (the launcher sizes G from the occupancy API) and G ≥ the largest
//    mini-batch, the lowest incomplete mini-batch always completes: its patterns' owners only
//    wait on earlier mini-batches.  Spins are bounded; a timeout raises sync[1].
//  * 512 threads per workgroup at N = 128 (256 VGPRs per lane): every global operand of every
//    FFT epilogue is prefetched into registers one FFT ahead, without spills.

// FFT flavour (PTYX_F2_WAVE_FFT): 1 = wave-owned fft2d_w (two workgroup barriers per 2-D FFT,
// so waves drift and one wave's memory latency overlaps another's butterflies), 0 = Stockham
// fft2d (eight barriers).
#ifndef PTYX_F2_WAVE_FFT
#define PTYX_F2_WAVE_FFT 0
#endif

template <int N, bool WAVE>
struct FftKit;
template <int N>
struct FftKit<N, false> {
  static constexpr int NT = N == 128 ? 1024 : (N == 64 ? 256 : 128);
  using PM = PassMap<N, NT>;
  using Arr = LdsArray<N>;
  template <int DIR, bool PRELOAD, class Pre, class Post>
  __device__ __forceinline__ static void fft(const Arr& arr, const float2* tw, Pre&& pre, Post&& post) {
    fft2d<N, NT, DIR, PRELOAD>(arr, tw, pre, post);
  }
};
template <int N>
struct FftKit<N, true> {
  static constexpr int NT = WGeom<N>::NT;
  using PM = PassMapW<N>;
  using Arr = LdsArrayW<N>;
  template <int DIR, bool PRELOAD, class Pre, class Post>
  __device__ __forceinline__ static void fft(const Arr& arr, const float2* tw, Pre&& pre, Post&& post) {
    fft2d_w<N, DIR, PRELOAD>(arr, tw, pre, post);
  }
};
template <int N>
using FusedKit = FftKit<N, PTYX_F2_WAVE_FFT != 0>;

// pattern → (mini-batch id, clamped window origin) for the call's index list
__global__ void k_pattern_table(const int* idx, int n, const int* boff, int n_batches, const int* crop,
                                int n_scans, int Ny, int Nx, int N, int* bid, int2* geo) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  int lo = 0, hi = n_batches;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (boff[mid] <= j) lo = mid;
    else hi = mid;
  }
  bid[j] = lo;
  const int s = min(max(idx[j], 0), n_scans - 1);
  geo[j] = make_int2(min(max(crop[2 * s], 0), Ny - N), min(max(crop[2 * s + 1], 0), Nx - N));
}

template <int N, bool SHIFT>
__global__ __launch_bounds__(FusedKit<N>::NT) void k_fused2(KArgs a) {
  using Kit = FusedKit<N>;
  using PM = typename Kit::PM;
  constexpr int NT = Kit::NT;
  constexpr int N2 = N * N;
  constexpr int SF = PM::kFirstSlots, SL = PM::kLastSlots;
  constexpr float inv_n = 1.0f / (float)N, inv_n2 = 1.0f / (float)N2;
  __shared__ float2 s_tw[N], s_wy[N], s_wx[N];
  __shared__ float s_red[(NT / 64) * 5];
  __shared__ float s_c;
  __shared__ float2 s_buf[Kit::Arr::kElems];
  for (int i = threadIdx.x; i < N; i += NT) s_tw[i] = a.twg[i];
  const typename Kit::Arr arr{s_buf};
  const bool tail = a.need_probe || a.d_shifts;   // probe slab / position gradient wanted
  float2* slab = a.slab + (size_t)blockIdx.x * N2;
  if (a.need_probe)
    for (int e = opaque_tid(); e < N2; e += NT) slab[e] = make_float2(0.f, 0.f);
  unsigned* err = a.sync + 1;
  unsigned* arrive = a.sync + 2;
  const float occ = a.occu[0];
  const bool single = a.single_on != 0;           // exactly one data term on (launcher checks)
  const float q = single ? a.q1 : a.q2;
  __syncthreads();
#if PTYX_EXP_PHASE_TIMES
  unsigned long long ph_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long ph_prev = wall_clock64();
  int ph_n = 0;
#endif

  for (int pat = blockIdx.x; pat < a.n_idx; pat += gridDim.x) {
#if PTYX_EXP_PHASE_TIMES
    ++ph_n;
#endif
    const int m = a.bid[pat];
    const PatternGeom g = pattern_geom(a, pat, N);
    const int tid = opaque_tid();
    // ---- exit wave ψ⁰ ⊙ O from the prefetched probe spectrum and object window
    float2 fp[SF];
    float oa[SL], op[SL];
#pragma unroll
    for (int s = 0; s < SF; ++s) {
      int y, x;
      PM::first(tid, s, y, x);
      fp[s] = SHIFT ? a.Fp[y * N + x] : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int s = 0; s < SL; ++s) {
      int y, x;
      PM::last(tid, s, y, x);
      const size_t off = obj_off(a, 0, 0, g.cy + y, g.cx + x);
      oa[s] = a.obja[off];
      op[s] = a.objp[off];
    }
    if constexpr (SHIFT) build_ramps<N, NT>(g, s_wy, s_wx);
    float sp = 0.f;
    if (a.sparse_on) {
#pragma unroll
      for (int s = 0; s < SL; ++s) {
        const float ap = PM::last_active(tid, s) ? fabsf(op[s]) : 0.f;
        sp += a.sparse_n == 1 ? ap : powq(ap, (float)a.sparse_n);
      }
    }
    PTYX_PHASE(0);
    float2 pb[SL];   // ψ⁰ at the last-pass points, until the object-gradient epilogue
    {
      auto times_obj = [&](float2 w, int s) -> float2 {
        float sn, cs;
        phase_sincos(op[s], &sn, &cs);
        return cmul(w, make_float2(oa[s] * cs, oa[s] * sn));
      };
      if constexpr (SHIFT) {
        Kit::template fft<+1, false>(
            arr, s_tw, [&](int y, int x, float2, int s) { return cmul(cmul(fp[s], s_wy[y]), s_wx[x]); },
            [&](int, int, float2& v, int s) {
              const float2 w = cscale(v, inv_n2);
              pb[s] = w;
              v = times_obj(w, s);
              return true;
            });
      } else {
#pragma unroll
        for (int s = 0; s < SL; ++s) {
          int y, x;
          PM::last(tid, s, y, x);
          const float2 w = a.probe[y * N + x];
          pb[s] = w;
          const float2 wo = times_obj(w, s);
          if (PM::last_active(tid, s)) arr.st(y, x, wo);
        }
        __syncthreads();
      }
    }
    PTYX_PHASE(1);
    float mv[SL];
#pragma unroll
    for (int s = 0; s < SL; ++s) {
      int y, x;
      PM::last(tid, s, y, x);
      mv[s] = load_meas_nt(a, g.s, fftshift_index<N>(y, x), N2);
    }
    // ---- far field: loss partial sums and g_Ψ / c_m into LDS in one epilogue
    float sums[2] = {0.f, 0.f};
    Kit::template fft<-1, true>(
        arr, s_tw, [&](int, int, float2 v, int) { return v; },
        [&](int y, int x, float2& v, int s) {
          const float2 Psi = cscale(v, inv_n);
          const float I = fmaf(occ, cabs2(Psi), kDpEps), rI = 1.0f / I;
          if (a.dp_out) a.dp_out[(size_t)pat * N2 + fftshift_index<N>(y, x)] = I;
          const float Iq = powq(I, q), Mq = powq(mv[s], q);
          float u;
          if (single) {                        // ∂/∂I of Σ(I^q - M^q)², per unit c_single
            const float d = Iq - Mq;
            sums[0] = fmaf(d, d, sums[0]);
            sums[1] += Mq;
            u = d * q * Iq * rI;
          } else {                             // ∂/∂I of Σ(M^q ln(I^q+ε) - I^q), per unit c_poissn
            sums[0] += Mq * fast_ln(Iq + a.eps2) - Iq;
            sums[1] += Mq;
            u = (Mq / (Iq + a.eps2) - 1.0f) * q * Iq * rI;
          }
          v = cscale(Psi, 2.0f * occ * u);
          return true;
        });
    PTYX_PHASE(2);
    {
      float v5[3] = {sums[0], sums[1], sp};
      block_sum<NT, 3>(v5, s_red);
      if (threadIdx.x == 0) {
        // write-through (sc1) stores of the partial sums, drained, then the arrival
        float* ps = a.psums + (size_t)pat * kNSum;
        const int base = single ? 0 : 2;
        __hip_atomic_store(ps + base, v5[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ps + base + 1, v5[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ps + (2 - base), 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ps + (3 - base), 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ps + kSumBase, v5[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(arrive + m, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    PTYX_PHASE(3);
    // ---- back to real space: g_O / c_m = conj(ψ⁰) g → this pattern's scratch slot;
    //      g ⊙ conj(O) → LDS for the probe / position gradient
    {
      float2* slot = a.ogscr + (size_t)pat * N2;
      Kit::template fft<+1, true>(
          arr, s_tw, [&](int, int, float2 v, int) { return v; },
          [&](int y, int x, float2& v, int s) {
            const float2 gv = cscale(v, inv_n);
            if (PM::last_active(tid, s)) slot[y * N + x] = cmulc(gv, pb[s]);
            const size_t off = obj_off(a, 0, 0, g.cy + y, g.cx + x);
            const float A = a.obja[off], ph = a.objp[off];
            float sn, cs;
            phase_sincos(ph, &sn, &cs);
            v = cmulc(gv, make_float2(A * cs, A * sn));
            return true;
          });
    }
    PTYX_PHASE(4);
    if (tail) {
      if (threadIdx.x < 64) {
        // wait for the mini-batch, then c_m from its partial sums: one pattern per lane
        // (write-through loads), added on lane 0 in k_finalize's order and arithmetic
        const int lane = threadIdx.x;
        const int b0 = a.boff[m], b1 = a.boff[m + 1];
        if (lane == 0) {
          const unsigned want = (unsigned)(b1 - b0);
          unsigned spins = 0;
          while (!a.debug_nowait &&
                 __hip_atomic_load(arrive + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > kMaxSpins) {
              atomicOr(err, 1u);
              break;
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
        const int base = single ? 0 : 2;
        double S = 0, M = 0;
        for (int t0 = b0; t0 < b1; t0 += 64) {
          float vs = 0.f, vm = 0.f;
          if (t0 + lane < b1) {
            const float* pq = a.psums + (size_t)(t0 + lane) * kNSum + base;
            vs = __hip_atomic_load(pq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            vm = __hip_atomic_load(pq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          const int cnt = min(64, b1 - t0);
          for (int i = 0; i < cnt; ++i) {
            S += (double)__shfl(vs, i, 64);
            M += (double)__shfl(vm, i, 64);
          }
        }
        if (lane == 0) {
          const double K = (double)(b1 - b0) * N2;
          float c = 0.f;
          if (single) {
            const double mu = M / K, rmse = sqrt(S / K);
            c = rmse > 0 ? (float)(a.w1 / (mu * K * rmse) * a.grad_scale) : 0.f;
          } else {
            c = (float)(-a.w2 / ((M / K) * K) * a.grad_scale);
          }
          s_c = c;
        }
      }
      __syncthreads();
      PTYX_PHASE(5);
      const float c = s_c;
      if constexpr (SHIFT) {
        float ds[2] = {0.f, 0.f};
        Kit::template fft<-1, true>(
            arr, s_tw, [&](int, int, float2 v, int) { return v; },
            [&](int y, int x, float2& G, int s) {
              const float2 W = cmul(s_wy[y], s_wx[x]);
              const float im = cmulc(cmul(a.Fp[y * N + x], W), G).y;   // Im(conj(G) F(P) W)
              ds[0] = fmaf(shift_g<N>(y), im, ds[0]);
              ds[1] = fmaf(shift_g<N>(x), im, ds[1]);
              if (a.need_probe && PM::last_active(tid, s))              // Σ_b c_b conj(W_b) F(g_Pb)
                slab[y * N + x] = cadd(slab[y * N + x], cscale(cmulc(G, W), c));
              return false;
            });
        if (a.d_shifts) {
          block_sum<NT, 2>(ds, s_red);
          if (threadIdx.x == 0) {
            const float k = 6.283185307179586f * c * inv_n2;
            atomicAdd(a.d_shifts + 2 * g.s, ds[0] * k);
            atomicAdd(a.d_shifts + 2 * g.s + 1, ds[1] * k);
          }
        }
      } else {
        if (a.need_probe) {
#pragma unroll
          for (int s = 0; s < SL; ++s) {
            int y, x;
            PM::last(tid, s, y, x);
            if (PM::last_active(tid, s)) slab[y * N + x] = cadd(slab[y * N + x], cscale(arr.ld(y, x), c));
          }
        }
      }
    }
    __syncthreads();   // LDS array and ramps are reused by the next pattern
    PTYX_PHASE(6);
  }
#if PTYX_EXP_PHASE_TIMES
  if (threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == 128))
    printf("PHASES2 wg %d n %d us: pre %.1f ifft1 %.1f fft2 %.1f publish %.1f ifft3 %.1f wait %.1f fft4 %.1f\n",
           (int)blockIdx.x, ph_n, ph_acc[0] * 0.01, ph_acc[1] * 0.01, ph_acc[2] * 0.01, ph_acc[3] * 0.01,
           ph_acc[4] * 0.01, ph_acc[5] * 0.01, ph_acc[6] * 0.01);
#endif
}

// =====================================================================================
// Object gradient from the per-pattern g_O slots (pattern order, fixed reduction order):
//   S(r) = Σ_j c_{m(j)} g_O,j(r - r_j),   C(r) = Σ_j cs_{m(j)} [r inside window j]
//   d_obja(r) += Re(S e^{-iφ}),   d_objp(r) += A Im(S e^{-iφ}) + C sgn(φ)|φ|^(n-1)
// (the per-pattern adjoint of O = A e^{iφ} and of the sparse term, summed).
// One 64 x 16 object tile per workgroup; wave w scans the pattern list in 64-pattern chunks
// w, w+4, ... (coalesced window origins, ballot of the overlapping ones) and accumulates the
// whole tile; the four wave partials are added in wave order.
struct GatherArgs {
  const float2* ogscr;
  const int2* geo;
  const float2* pcoef;   // per pattern: (c_data, c_sparse) of its mini-batch
  int n;
  int Ny, Nx, tiles_x;
  int sparse_n;
  const float* obja;
  const float* objp;
  float* d_obja;
  float* d_objp;
  int nz = 1, z = 0;     // slots hold nz planes per pattern; this launch gathers plane z
  const int* bbox = nullptr;   // {min cy, max cy, min cx, max cx} of the call's windows: other tiles exit
};
#ifndef PTYX_GTY
#define PTYX_GTY 16
#endif
#ifndef PTYX_GWAVES
#define PTYX_GWAVES 16
#endif
constexpr int kGTX = 64, kGTY = PTYX_GTY, kGWaves = PTYX_GWAVES;

// ROWPERM: slots written by k_fused3 (N = 128), row y stored at row 2(y & 63) + (y >> 6).
template <int N, bool ROWPERM = false>
__global__ __launch_bounds__(64 * kGWaves) void k_obj_gather(GatherArgs ga) {
  constexpr int N2 = N * N;
  __shared__ float2 s_acc[kGTY * kGTX];
  __shared__ float s_cnt[kGTY * kGTX];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ty = (blockIdx.x / ga.tiles_x) * kGTY, tx = (blockIdx.x % ga.tiles_x) * kGTX;
  if (ga.bbox && (ty + kGTY <= ga.bbox[0] || ty >= ga.bbox[1] + N || tx + kGTX <= ga.bbox[2] || tx >= ga.bbox[3] + N))
    return;   // no window of this call touches the tile: its gradient contribution is zero
  const int x = tx + lane;
  float2 acc[kGTY];
  float cnt[kGTY];
#pragma unroll
  for (int r = 0; r < kGTY; ++r) {
    acc[r] = make_float2(0.f, 0.f);
    cnt[r] = 0.f;
  }
  for (int base = wave * 64; base < ga.n; base += 64 * kGWaves) {
    const int j = base + lane;
    int2 o = make_int2(-(1 << 29), -(1 << 29));
    float2 cj = make_float2(0.f, 0.f);
    if (j < ga.n) {
      o = ga.geo[j];
      cj = ga.pcoef[j];
    }
    const bool hit = o.x > ty - N && o.x < ty + kGTY && o.y > tx - N && o.y < tx + kGTX;
    unsigned long long mask = __ballot(hit);
    while (mask) {
      const int b = __builtin_ctzll(mask);
      mask &= mask - 1;
      const int cy = __shfl(o.x, b, 64), cx = __shfl(o.y, b, 64);
      const float c = __shfl(cj.x, b, 64), cs = __shfl(cj.y, b, 64);
      const float2* src = ga.ogscr + ((size_t)(base + b) * ga.nz + ga.z) * N2;
      const int col = x - cx;
      const bool colok = col >= 0 && col < N;
      float2 v[kGTY];
#pragma unroll
      for (int r = 0; r < kGTY; ++r) {
        const int row = ty + r - cy;
        const int srow = ROWPERM ? 2 * (row & (N / 2 - 1)) + (row >> 6) : row;
        v[r] = (colok && row >= 0 && row < N) ? src[srow * N + col] : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int r = 0; r < kGTY; ++r) {
        const int row = ty + r - cy;
        acc[r].x = fmaf(c, v[r].x, acc[r].x);
        acc[r].y = fmaf(c, v[r].y, acc[r].y);
        if (colok && row >= 0 && row < N) cnt[r] += cs;
      }
    }
  }
  // wave partials in fixed order
  for (int w = 0; w < kGWaves; ++w) {
    if (wave == w) {
#pragma unroll
      for (int r = 0; r < kGTY; ++r) {
        const int e = r * kGTX + lane;
        if (w == 0) {
          s_acc[e] = acc[r];
          s_cnt[e] = cnt[r];
        } else {
          s_acc[e] = cadd(s_acc[e], acc[r]);
          s_cnt[e] += cnt[r];
        }
      }
    }
    __syncthreads();
  }
  for (int e = threadIdx.x; e < kGTY * kGTX; e += 64 * kGWaves) {
    const int y = ty + e / kGTX, xx = tx + e % kGTX;
    if (y >= ga.Ny || xx >= ga.Nx) continue;
    const size_t off = (size_t)y * ga.Nx + xx;
    const float2 S = s_acc[e];
    const float A = ga.obja[off], ph = ga.objp[off];
    float sn, cs;
    phase_sincos(ph, &sn, &cs);
    if (ga.d_obja) ga.d_obja[off] += fmaf(S.x, cs, S.y * sn);
    if (ga.d_objp) {
      float dph = A * fmaf(S.y, cs, -S.x * sn);
      const float C = s_cnt[e];
      if (C != 0.f) {
        const float sg = ph > 0.f ? 1.f : (ph < 0.f ? -1.f : 0.f);
        dph += ga.sparse_n == 1 ? C * sg : C * powq(fabsf(ph), (float)(ga.sparse_n - 1)) * sg;
      }
      ga.d_objp[off] += dph;
    }
  }
}
