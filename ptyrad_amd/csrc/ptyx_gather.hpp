// ptyx_gather.hpp — deterministic object-gradient gather for the register engines
// (k_fused3 / k_fused3ms, ptyx_fused3.hpp).  Included by ptyx_kernels.hip inside namespace ptyx.
//
// fp32 scatter-add atomics execute at the memory side at ≈1.3 TB/s for the whole chip
// (MI355X_MICROARCH.md, global float atomics), i.e. ≥ 6.6 ms per c2 step for 128 KiB of object
// gradient per pattern.  Instead each pattern PLAIN-STORES its unit-coefficient object-gradient
// wave g_O = conj(ψ⁰)·g to a per-pattern slot, and k_obj_gather reduces the slots per object
// tile in pattern order: no atomics, bitwise-deterministic object gradients.

// =====================================================================================
// Object gradient from the per-pattern g_O slots (pattern order, fixed reduction order):
//   S(r) = Σ_j c_{m(j)} g_O,j(r - r_j),   C(r) = Σ_j cs_{m(j)} [r inside window j]
//   d_obja(r) += Re(S e^{-iφ}),   d_objp(r) += A Im(S e^{-iφ}) + C sgn(φ)|φ|^(n-1)
// (the per-pattern adjoint of O = A e^{iφ} and of the sparse term, summed).
// One 64 x 16 object tile per workgroup; its waves take the candidate patterns in 64-pattern
// chunks w, w + kGWaves, ... (ballot of the ones whose window overlaps the tile) and accumulate
// the whole tile; the wave partials are added in wave order.
//
// Candidates: the patterns of a call are binned by the tile that holds their window origin
// (k_bin_*: counting sort, each bin then sorted by pattern index, so the order is deterministic);
// a 128-pixel window reaches at most 9 tile rows and 3 tile columns, so a tile scans the 27 bins
// up-left of it instead of every pattern of the call (c4: 8,192 patterns per call over 13,340
// tiles, ≈ 17 of them per tile).
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
  int nz = 1, z = 0;     // slots hold nz planes per pattern; this launch gathers plane z, or, with
  int zgrid = 0;         // zgrid, plane blockIdx.y (obja / objp / d_* then point at plane 0)
  int np = 1;            // MP: plane z of pattern j is the sum of np (≤ kGatherMaxNp) consecutive slot planes
  long long pstride = 0; // slot planes per pattern (0: nz·np); plane (j, z, p) at j·pstride + z·np + p
  // candidate split (gridDim.z = S > 1, small objects whose tiles do not fill the GPU): split s
  // takes every S-th candidate and leaves its tile sums in part / pcnt; k_obj_gather_fin adds the
  // S partials in order and applies the epilogue
  float2* part = nullptr;
  float* pcnt = nullptr;
  const int* bbox = nullptr;   // {min cy, max cy, min cx, max cx} of the call's windows: other tiles exit
  const int* boff = nullptr;   // bin offsets (tiles + 1) into blist, or NULL: scan every pattern
  const int* blist = nullptr;  // pattern indices by bin, ascending within a bin
  // slots in rank blocks (the slot exchange's all-gathered buffer): pattern j's slot at block
  // j / blk, row j % blk, blocks bstride float2 apart (blk 0: plain pattern rows)
  int blk = 0;
  long long bstride = 0;
  // PTYX_PREP_GRAD_STORE: d_obja / d_objp are OVERWRITTEN with this call's gradient (tiles no
  // window touches get zeros), so the caller need not zero them and no old value is read
  int store = 0;
};
// float2 offset of pattern j's slot plane zp (non-MP layouts)
__device__ __forceinline__ size_t slot_plane(const GatherArgs& ga, int j, int zp, int N2) {
  if (ga.blk > 0) return (size_t)(j / ga.blk) * ga.bstride + ((size_t)(j % ga.blk) * ga.nz + zp) * N2;
  return ((size_t)j * ga.nz + zp) * N2;
}
// 64 × 16 object tiles, 16 waves per tile (measured: 128-wide tiles and 2 patterns per round
// were slower)
constexpr int kGTX = 64, kGTY = 16, kGWaves = 16;
constexpr int kGatherMaxNp = 8;          // probe-mode planes summed per slot (MP)
constexpr int kGatherPartCap = 4096;     // tile partials of a split gather (× 64·16 × 12 B = 48 MiB)

// d_obja / d_objp of one object pixel from its gathered S = Σ c g_O and sparse count C
__device__ __forceinline__ void gather_apply(const GatherArgs& ga, size_t off, float2 S, float C) {
  const float A = ga.obja[off], ph = ga.objp[off];
  float sn, cs;
  phase_sincos(ph, &sn, &cs);
  if (ga.d_obja) {
    const float da = fmaf(S.x, cs, S.y * sn);
    ga.d_obja[off] = (ga.store ? 0.f : ga.d_obja[off]) + da;   // (0 + x: bitwise the accumulate into zeros)
  }
  if (ga.d_objp) {
    float dph = A * fmaf(S.y, cs, -S.x * sn);
    if (C != 0.f) {
      const float sg = ph > 0.f ? 1.f : (ph < 0.f ? -1.f : 0.f);
      dph += ga.sparse_n == 1 ? C * sg : C * powq(fabsf(ph), (float)(ga.sparse_n - 1)) * sg;
    }
    ga.d_objp[off] = (ga.store ? 0.f : ga.d_objp[off]) + dph;
  }
}
// A tile no window of the call reaches: its contribution is zero (store mode writes the zeros).
template <int N>
__device__ __forceinline__ bool gather_tile_skip(const GatherArgs& ga, int ty, int tx) {
  const bool skip = ga.bbox && (ty + kGTY <= ga.bbox[0] || ty >= ga.bbox[1] + N || tx + kGTX <= ga.bbox[2] ||
                                tx >= ga.bbox[3] + N);
  if (skip && ga.store) {
    const size_t zoff = ga.zgrid ? (size_t)blockIdx.y * ga.Ny * ga.Nx : 0;
    for (int e = threadIdx.x; e < kGTY * kGTX; e += blockDim.x) {
      const int y = ty + e / kGTX, x = tx + e % kGTX;
      if (y >= ga.Ny || x >= ga.Nx) continue;
      const size_t off = zoff + (size_t)y * ga.Nx + x;
      if (ga.d_obja) ga.d_obja[off] = 0.f;
      if (ga.d_objp) ga.d_objp[off] = 0.f;
    }
  }
  return skip;
}

// ROWPERM: slots written by k_fused3 (N = 128), row y stored at row 2(y & 63) + (y >> 6).
// bins of a tile's candidates: home tiles (ty − kBinRows + 1 … ty) × (tx − kBinCols + 1 … tx)
template <int N>
struct BinReach {
  static constexpr int rows = (N + kGTY - 1) / kGTY + 1, cols = (N + kGTX - 1) / kGTX + 1, n = rows * cols;
};

// A tile's sums S (s_acc) and sparse counts C (s_cnt) over its candidates, in fixed order (the
// workgroup's GW waves; LDS results valid after the final barrier).  Tile (tyi, txi), slot plane zp;
// split s of S.
template <int N, bool ROWPERM, int GW, bool MP, bool SPLIT>
__device__ __forceinline__ void gather_tile_sums(const GatherArgs& ga, int tyi, int txi, int zp, float2* s_acc,
                                                 float* s_cnt) {
  constexpr int N2 = N * N;
  constexpr int NB = BinReach<N>::n;
  __shared__ int s_b0[NB], s_pre[NB + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ty = tyi * kGTY, tx = txi * kGTX;
  const int S = SPLIT ? (int)gridDim.z : 1, s = SPLIT ? (int)blockIdx.z : 0;
  int total = ga.n;
  if (ga.boff) {
    if (threadIdx.x < NB) {
      const int by = tyi - (BinReach<N>::rows - 1) + (int)threadIdx.x / BinReach<N>::cols;
      const int bx = txi - (BinReach<N>::cols - 1) + (int)threadIdx.x % BinReach<N>::cols;
      int b0 = 0, len = 0;
      if (by >= 0 && bx >= 0) {
        const int b = by * ga.tiles_x + bx;
        b0 = ga.boff[b];
        len = ga.boff[b + 1] - b0;
      }
      s_b0[threadIdx.x] = b0;
      s_pre[threadIdx.x + 1] = len;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      s_pre[0] = 0;
      for (int k = 0; k < NB; ++k) s_pre[k + 1] += s_pre[k];
    }
    __syncthreads();
    total = s_pre[NB];
  }
  const int x = tx + lane;
  float2 acc[kGTY];
  float cnt[kGTY];
#pragma unroll
  for (int r = 0; r < kGTY; ++r) {
    acc[r] = make_float2(0.f, 0.f);
    cnt[r] = 0.f;
  }
  // scan: candidate i = s + S·(w + GW·(lane + 64·k)) of the bins' list (or of the call's patterns,
  // small calls): a tile's candidates spread over all its waves and splits
  const int first = s + S * wave;
  for (int base = first; base < total; base += 64 * GW * S) {
    const int i = base + S * GW * lane;
    int j = i;
    int2 o = make_int2(-(1 << 29), -(1 << 29));
    float2 cj = make_float2(0.f, 0.f);
    if (i < total) {
      if (ga.boff) {
        int k = 0;
        while (k + 1 < NB && s_pre[k + 1] <= i) ++k;
        j = ga.blist[s_b0[k] + (i - s_pre[k])];
      }
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
      const int jb = __shfl(j, b, 64);
      const float2* src = MP ? ga.ogscr + ((size_t)jb * ga.pstride + (size_t)zp * ga.np) * N2
                             : ga.ogscr + slot_plane(ga, jb, zp, N2);
      const int col = x - cx;
      const bool colok = col >= 0 && col < N;
      float2 v[kGTY];
#pragma unroll
      for (int r = 0; r < kGTY; ++r) {
        const int row = ty + r - cy;
        const int srow = ROWPERM ? 2 * (row & (N / 2 - 1)) + (row >> 6) : row;
        if (colok && row >= 0 && row < N) {
          if constexpr (MP) {   // the probe modes' planes of this slice: loads issued together, summed in mode order
            float2 t[kGatherMaxNp];
#pragma unroll
            for (int pp = 0; pp < kGatherMaxNp; ++pp)
              t[pp] = pp < ga.np ? src[(size_t)pp * N2 + srow * N + col] : make_float2(0.f, 0.f);
            v[r] = t[0];
#pragma unroll
            for (int pp = 1; pp < kGatherMaxNp; ++pp) v[r] = cadd(v[r], t[pp]);
          } else {
            v[r] = src[srow * N + col];
          }
        } else {
          v[r] = make_float2(0.f, 0.f);
        }
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
  for (int w = 0; w < GW; ++w) {
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
}

// GW: waves per tile (kGWaves for dense calls; 4 when a tile has only a few candidates, so that
// the per-tile fixed cost, the wave-partial reduction, stays small)
template <int N, bool ROWPERM = false, int GW = kGWaves, bool MP = false, bool SPLIT = false>
__global__ __launch_bounds__(64 * GW) void k_obj_gather(GatherArgs ga) {
  __shared__ float2 s_acc[kGTY * kGTX];
  __shared__ float s_cnt[kGTY * kGTX];
  const int tyi = blockIdx.x / ga.tiles_x, txi = blockIdx.x % ga.tiles_x;
  const int zp = ga.zgrid ? (int)blockIdx.y : ga.z;                        // slot plane
  const size_t zoff = ga.zgrid ? (size_t)blockIdx.y * ga.Ny * ga.Nx : 0;   // object plane
  const int ty = tyi * kGTY, tx = txi * kGTX;
  if (gather_tile_skip<N>(ga, ty, tx)) return;   // no window of this call touches the tile: its contribution is zero
  gather_tile_sums<N, ROWPERM, GW, MP, SPLIT>(ga, tyi, txi, zp, s_acc, s_cnt);
  const int S = SPLIT ? (int)gridDim.z : 1, s = SPLIT ? (int)blockIdx.z : 0;
  if constexpr (SPLIT) {   // this split's tile sums; k_obj_gather_fin adds the splits in order
    const size_t pb = (((size_t)blockIdx.y * gridDim.x + blockIdx.x) * S + s) * (kGTY * kGTX);
    for (int e = threadIdx.x; e < kGTY * kGTX; e += 64 * GW) {
      ga.part[pb + e] = s_acc[e];
      ga.pcnt[pb + e] = s_cnt[e];
    }
    return;
  }
  for (int e = threadIdx.x; e < kGTY * kGTX; e += 64 * GW) {
    const int y = ty + e / kGTX, xx = tx + e % kGTX;
    if (y >= ga.Ny || xx >= ga.Nx) continue;
    gather_apply(ga, zoff + (size_t)y * ga.Nx + xx, s_acc[e], s_cnt[e]);
  }
}

// Row-split variant (small calls of the mixed-state engine): the workgroup first lists the hits
// of a chunk of 64·GW candidates in candidate order (ballot + prefix, LDS), then EVERY wave takes
// all of them for its own kGTY / GW rows, HU hits' loads in flight at once.  k_obj_gather gives a
// wave whole hits, 16 rows × np planes each, and at np = 6 the compiler issues them row by row (16
// round trips a hit); here a hit costs one.  Each wave owns its rows to the end, so there is no
// wave-partial reduction either.  Hits are summed in candidate order (deterministic) with a
// compensated (Kahan) accumulators, for the g_O sum and the loss_sparse count alike: one
// sequential fp32 sum over every hit of a pixel (≈ 2,000 at the c2 coverage) drifts by ≈ 5e-6 of
// the gradient's norm between call splits (a full-c2 split-invariance failure
// of dφ — the count adds ≈ 2,000 near-equal c_sparse terms, whose rounding is systematic, not
// random; a missing or doubled hit would move the norm by ≈ 6e-5); compensated, both stay at fp32
// rounding.
// The row-split gather's sums of one tile: wave w's rows ty + w·RW … (acc, cnt: running sums after
// the Kahan-compensated accumulation over every hit, candidate order).  Tile (tyi, txi), slot plane zp.
// HUX > 0: that many hits in flight per wave instead of what 32 registers' worth of loads allow.
template <int N, bool ROWPERM, int GW, bool MP, int HUX = 0>
__device__ __forceinline__ void gather_rows_sums(const GatherArgs& ga, int tyi, int txi, int zp,
                                                 float2 (&acc)[kGTY / GW], float (&cnt)[kGTY / GW]) {
  constexpr int N2 = N * N;
  constexpr int NB = BinReach<N>::n;
  constexpr int RW = kGTY / GW;                          // rows per wave
  constexpr int NPL = MP ? kGatherMaxNp : 1;             // planes per row and hit (≤; np at run time)
  constexpr int HU = HUX > 0 ? HUX : (32 / (RW * NPL) > 0 ? 32 / (RW * NPL) : 1);   // hits in flight per wave
  __shared__ int4 s_hit[64 * GW];     // (cy, cx, j, c) of the chunk's hits, candidate order
  __shared__ float s_hcs[64 * GW];
  __shared__ int s_wcnt[GW];
  __shared__ int s_b0[NB], s_pre[NB + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ty = tyi * kGTY, tx = txi * kGTX;
  int total = ga.n;
  if (ga.boff) {
    if (threadIdx.x < NB) {
      const int by = tyi - (BinReach<N>::rows - 1) + (int)threadIdx.x / BinReach<N>::cols;
      const int bx = txi - (BinReach<N>::cols - 1) + (int)threadIdx.x % BinReach<N>::cols;
      int b0 = 0, len = 0;
      if (by >= 0 && bx >= 0) {
        const int b = by * ga.tiles_x + bx;
        b0 = ga.boff[b];
        len = ga.boff[b + 1] - b0;
      }
      s_b0[threadIdx.x] = b0;
      s_pre[threadIdx.x + 1] = len;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      s_pre[0] = 0;
      for (int k = 0; k < NB; ++k) s_pre[k + 1] += s_pre[k];
    }
    __syncthreads();
    total = s_pre[NB];
  }
  const int x = tx + lane;
  const int r0 = ty + wave * RW;   // this wave's first object row
  float2 cmp[RW];   // the running sums' Kahan compensations
  float ccmp[RW];
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    acc[r] = make_float2(0.f, 0.f);
    cmp[r] = make_float2(0.f, 0.f);
    cnt[r] = 0.f;
    ccmp[r] = 0.f;
  }
  const int np = MP ? ga.np : 1;
  for (int base = 0; base < total; base += 64 * GW) {
    const int i = base + (int)threadIdx.x;
    int j = i;
    int2 o = make_int2(-(1 << 29), -(1 << 29));
    float2 cj = make_float2(0.f, 0.f);
    if (i < total) {
      if (ga.boff) {
        int k = 0;
        while (k + 1 < NB && s_pre[k + 1] <= i) ++k;
        j = ga.blist[s_b0[k] + (i - s_pre[k])];
      }
      o = ga.geo[j];
      cj = ga.pcoef[j];
    }
    const bool hit = o.x > ty - N && o.x < ty + kGTY && o.y > tx - N && o.y < tx + kGTX;
    const unsigned long long mk = __ballot(hit);
    if (lane == 0) s_wcnt[wave] = __popcll(mk);
    __syncthreads();
    int off = 0, nh = 0;
#pragma unroll
    for (int w = 0; w < GW; ++w) {
      const int c = s_wcnt[w];
      off += w < wave ? c : 0;
      nh += c;
    }
    if (hit) {
      const int at = off + __popcll(mk & ((1ull << lane) - 1ull));
      s_hit[at] = make_int4(o.x, o.y, j, __float_as_int(cj.x));
      s_hcs[at] = cj.y;
    }
    __syncthreads();
    for (int h0 = 0; h0 < nh; h0 += HU) {
      float2 t[HU][RW][NPL];
#pragma unroll
      for (int hu = 0; hu < HU; ++hu) {
        const int h = h0 + hu;
        const int4 H = s_hit[h < nh ? h : 0];
        const int col = x - H.y;
        const bool colok = h < nh && col >= 0 && col < N;
        const float2* src = MP ? ga.ogscr + ((size_t)H.z * ga.pstride + (size_t)zp * ga.np) * N2
                               : ga.ogscr + slot_plane(ga, H.z, zp, N2);
#pragma unroll
        for (int r = 0; r < RW; ++r) {
          const int row = r0 + r - H.x;
          const int srow = ROWPERM ? 2 * (row & (N / 2 - 1)) + (row >> 6) : row;
          const bool ok = colok && row >= 0 && row < N;
#pragma unroll
          for (int pp = 0; pp < NPL; ++pp)
            t[hu][r][pp] = ok && pp < np ? src[(size_t)pp * N2 + srow * N + col] : make_float2(0.f, 0.f);
        }
      }
#pragma unroll
      for (int hu = 0; hu < HU; ++hu) {
        const int h = h0 + hu;
        if (h >= nh) break;
        const int4 H = s_hit[h];
        const float c = __int_as_float(H.w), cs = s_hcs[h];
        const int col = x - H.y;
        const bool colok = col >= 0 && col < N;
#pragma unroll
        for (int r = 0; r < RW; ++r) {
          float2 v = t[hu][r][0];
#pragma unroll
          for (int pp = 1; pp < NPL; ++pp) v = cadd(v, t[hu][r][pp]);
          const float yx = fmaf(c, v.x, -cmp[r].x), yy = fmaf(c, v.y, -cmp[r].y);
          const float sx = acc[r].x + yx, sy = acc[r].y + yy;
          cmp[r].x = (sx - acc[r].x) - yx;
          cmp[r].y = (sy - acc[r].y) - yy;
          acc[r] = make_float2(sx, sy);
          const int row = r0 + r - H.x;
          if (colok && row >= 0 && row < N) {   // (≈ 2,000 near-equal c_sparse terms: compensated too)
            const float yc = cs - ccmp[r];
            const float sc = cnt[r] + yc;
            ccmp[r] = (sc - cnt[r]) - yc;
            cnt[r] = sc;
          }
        }
      }
    }
    __syncthreads();   // the next chunk rewrites the hit list
  }
}

template <int N, bool ROWPERM, int GW, bool MP>
__global__ __launch_bounds__(64 * GW) void k_obj_gather_rows(GatherArgs ga) {
  constexpr int RW = kGTY / GW;                          // rows per wave
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tyi = blockIdx.x / ga.tiles_x, txi = blockIdx.x % ga.tiles_x;
  const int zp = ga.zgrid ? (int)blockIdx.y : ga.z;
  const size_t zoff = ga.zgrid ? (size_t)blockIdx.y * ga.Ny * ga.Nx : 0;
  const int ty = tyi * kGTY, tx = txi * kGTX;
  if (gather_tile_skip<N>(ga, ty, tx)) return;
  const int x = tx + lane;
  const int r0 = ty + wave * RW;   // this wave's first object row
  // the epilogue's operands of this wave's pixels (A, φ and the gradients it adds to), loaded
  // now: they do not depend on the hits, and only this workgroup touches these pixels
  float pa[RW], pp[RW], pga[RW], pgp[RW];
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    pa[r] = pp[r] = pga[r] = pgp[r] = 0.f;
    if (r0 + r < ga.Ny && x < ga.Nx) {
      const size_t off = zoff + (size_t)(r0 + r) * ga.Nx + x;
      pa[r] = ga.obja[off];
      pp[r] = ga.objp[off];
      if (ga.d_obja && !ga.store) pga[r] = ga.d_obja[off];
      if (ga.d_objp && !ga.store) pgp[r] = ga.d_objp[off];
    }
  }
  float2 acc[RW];
  float cnt[RW];
  gather_rows_sums<N, ROWPERM, GW, MP>(ga, tyi, txi, zp, acc, cnt);
#pragma unroll
  for (int r = 0; r < RW; ++r) {   // gather_apply on the prefetched operands
    const int y = r0 + r;
    if (y >= ga.Ny || x >= ga.Nx) continue;
    const size_t off = zoff + (size_t)y * ga.Nx + x;
    float sn, cs;
    phase_sincos(pp[r], &sn, &cs);
    if (ga.d_obja) ga.d_obja[off] = pga[r] + fmaf(acc[r].x, cs, acc[r].y * sn);
    if (ga.d_objp) {
      float dph = pa[r] * fmaf(acc[r].y, cs, -acc[r].x * sn);
      if (cnt[r] != 0.f) {
        const float ph = pp[r];
        const float sg = ph > 0.f ? 1.f : (ph < 0.f ? -1.f : 0.f);
        dph += ga.sparse_n == 1 ? cnt[r] * sg : cnt[r] * powq(fabsf(ph), (float)(ga.sparse_n - 1)) * sg;
      }
      ga.d_objp[off] = pgp[r] + dph;
    }
  }
}

// Split gather epilogue: tile (blockIdx.x, blockIdx.y) sums its S partials in split order.
template <int N>
__global__ __launch_bounds__(256) void k_obj_gather_fin(GatherArgs ga, int S) {
  const int tyi = blockIdx.x / ga.tiles_x, txi = blockIdx.x % ga.tiles_x;
  const int ty = tyi * kGTY, tx = txi * kGTX;
  if (gather_tile_skip<N>(ga, ty, tx)) return;
  const size_t zoff = ga.zgrid ? (size_t)blockIdx.y * ga.Ny * ga.Nx : 0;
  const size_t pb = ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * S * (kGTY * kGTX);
  for (int e = threadIdx.x; e < kGTY * kGTX; e += blockDim.x) {
    const int y = ty + e / kGTX, xx = tx + e % kGTX;
    if (y >= ga.Ny || xx >= ga.Nx) continue;
    float2 acc = ga.part[pb + e];
    float c = ga.pcnt[pb + e];
    for (int s = 1; s < S; ++s) {
      acc = cadd(acc, ga.part[pb + (size_t)s * (kGTY * kGTX) + e]);
      c += ga.pcnt[pb + (size_t)s * (kGTY * kGTX) + e];
    }
    gather_apply(ga, zoff + (size_t)y * ga.Nx + xx, acc, c);
  }
}

// ----------------------------------------------------------------------------- pattern bins
// Counting sort of a call's patterns by the tile holding their window origin, then each bin
// sorted by pattern index (deterministic candidate order for k_obj_gather).
__global__ void k_bin_count(const int2* geo, int n, int tiles_x, int* cnt, int* key) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int2 o = geo[j];
  const int b = (o.x / kGTY) * tiles_x + o.y / kGTX;
  key[j] = b;
  atomicAdd(cnt + b, 1);
}

// exclusive scan of cnt[0 .. nb) into off[0 .. nb] (and the fill cursors cur = off), one block
__global__ __launch_bounds__(1024) void k_bin_scan(const int* cnt, int nb, int* off, int* cur) {
  __shared__ int s[1024];
  const int t = threadIdx.x, per = (nb + 1023) / 1024;
  const int b0 = min(nb, t * per), b1 = min(nb, b0 + per);
  int sum = 0;
  for (int b = b0; b < b1; ++b) sum += cnt[b];
  s[t] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {   // Hillis-Steele inclusive scan of the chunk sums
    const int v = t >= d ? s[t - d] : 0;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
  int run = s[t] - sum;
  for (int b = b0; b < b1; ++b) {
    off[b] = run;
    cur[b] = run;
    run += cnt[b];
  }
  if (t == 1023) off[nb] = s[1023];
}

__global__ void k_bin_fill(const int* key, int n, int* cur, int* list) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  list[atomicAdd(cur + key[j], 1)] = j;
}

// one workgroup per bin: rank sort of its (distinct) pattern indices through LDS
constexpr int kBinSortCap = 2048;
__global__ __launch_bounds__(256) void k_bin_sort(const int* off, int* list) {
  __shared__ int s[kBinSortCap];
  const int b0 = off[blockIdx.x], len = off[blockIdx.x + 1] - b0;
  if (len < 2) return;
  if (len > kBinSortCap) {   // (a denser scan than any BASELINE config: one thread, in place)
    if (threadIdx.x == 0)
      for (int i = 1; i < len; ++i) {
        const int v = list[b0 + i];
        int k = i - 1;
        while (k >= 0 && list[b0 + k] > v) {
          list[b0 + k + 1] = list[b0 + k];
          --k;
        }
        list[b0 + k + 1] = v;
      }
    return;
  }
  for (int i = threadIdx.x; i < len; i += blockDim.x) s[i] = list[b0 + i];
  __syncthreads();
  for (int i = threadIdx.x; i < len; i += blockDim.x) {
    const int v = s[i];
    int r = 0;
    for (int k = 0; k < len; ++k) r += s[k] < v;
    list[b0 + r] = v;
  }
}
