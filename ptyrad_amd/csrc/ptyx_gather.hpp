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
