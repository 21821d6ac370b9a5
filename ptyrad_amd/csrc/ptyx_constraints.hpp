// ptyx_constraints.hpp — PtyRAD's iteration-wise constraints on the device.
// Included by ptyx_kernels.hip; the C ABI is ptyx_obj_rblur / ptyx_obj_constrain /
// ptyx_probe_fix_int / ptyx_probe_ortho (include/ptyx.h).
//
// Object constraints are HBM-bound streams over (O, Nz, Ny, Nx) f32, so they are fused:
//   k_rblur       obj_rblur   (constraints.py:83-98, torchvision gaussian_blur): separable 2-D
//                 Gaussian, reflect padding, one LDS tile (TY + 2h) × (TX + 2h) per workgroup;
//                 each voxel read once from HBM and written once (out of place).
//   k_obj_column  obj_zblur (:100-114, gaussian_blur_1d: conv1d 'same', replicate padding) +
//                 complex_ratio (:147-163, :333-358) + mirrored_amp (:165-179) + obja_thresh
//                 (:181-190) + objp_postiv (:192-208) in ONE pass: one thread per (o, y, x)
//                 column walks z with a register window of 2h + 1 slices, so the z-blur needs no
//                 second read and works in place; lanes run along x, so every z-slice access of
//                 a wave is one contiguous 256-B segment.
//   k_obj_reduce / k_reduce_final   the global scalars some options need (complex_ratio's Cbar,
//                 objp_postiv 'subtract_min''s minimum): fp64 per-block partials summed in a
//                 fixed order (deterministic), kept on the device — no host round trip.
// Probe constraints (P ≤ 64 modes of N × N):
//   fix_probe_int (:70-81): k_sumsq partials → k_fix_int_final (scale) → k_cscale.
//   ortho_pmode (:34-41, orthogonalize_modes_vec :255-291): k_gram (A = M M^H, one block column
//   per mode pair, fp64) → k_ortho_eig (one wave: fixed-order partial sums, cyclic complex
//   Jacobi in fp64 — the rotation by lane 0, its row / column updates one lane per k — LAPACK
//   geev eigenvector normalisation — unit norm, largest component real positive — and the
//   descending-eigenvalue order that sort_by_mode_int produces) → k_ortho_apply (ortho = V^H M
//   per pixel, in place; P a template parameter up to 16, then padded to 32 / 64).
#pragma once
#include <hip/hip_runtime.h>

namespace ptyx {
namespace cons {

constexpr int kMaxHalf = 7;        // kernel_size ≤ 15
constexpr int kMaxTaps = 2 * kMaxHalf + 1;
constexpr int kMaxModes = 64;        // ortho_pmode probe modes (static LDS of k_ortho_eig: 2·64²·16 B)
constexpr int kRedBlocks = 512;    // fixed reduction grid (deterministic partials)

struct Taps {
  float w[kMaxTaps];
  int half;
};

// ------------------------------------------------------------------ obj_rblur
constexpr int kTX = 64;   // columns of a blur tile
__device__ __forceinline__ int reflect_idx(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * (n - 1) - i : i;
}
// grid (ceil(Nx/kTX), ceil(Ny/kBTY), planes); block 256.  H = kernel_size / 2 at compile time
// (unrolled taps, constant tile geometry); the taps in the same order as before (j = 0 … 2H).
constexpr int kBTY = 32;   // rows of a blur tile (halo overhead (32 + 2H) / 32)
template <int H>
__global__ __launch_bounds__(256) void k_rblur(const float* __restrict__ in, float* __restrict__ out, int Ny, int Nx,
                                               Taps t) {
  constexpr int rows = kBTY + 2 * H, cols = kTX + 2 * H;
  __shared__ float s_in[rows][cols + 1];
  __shared__ float s_mid[rows][kTX + 1];
  const size_t plane = (size_t)blockIdx.z * Ny * Nx;
  const int x0 = blockIdx.x * kTX, y0 = blockIdx.y * kBTY;
  for (int e = threadIdx.x; e < rows * cols; e += blockDim.x) {
    const int r = e / cols, c = e - r * cols;
    const int gy = reflect_idx(min(y0 + r - H, Ny - 1 + H), Ny);
    const int gx = reflect_idx(min(x0 + c - H, Nx - 1 + H), Nx);
    s_in[r][c] = in[plane + (size_t)gy * Nx + gx];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < rows * kTX; e += blockDim.x) {
    const int r = e / kTX, c = e - r * kTX;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j <= 2 * H; ++j) acc = fmaf(t.w[j], s_in[r][c + j], acc);
    s_mid[r][c] = acc;
  }
  __syncthreads();
  const int c = threadIdx.x & (kTX - 1);
  for (int r = threadIdx.x >> 6; r < kBTY; r += blockDim.x >> 6) {
    const int gy = y0 + r, gx = x0 + c;
    if (gy >= Ny || gx >= Nx) continue;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i <= 2 * H; ++i) acc = fmaf(t.w[i], s_mid[r + i][c], acc);
    out[plane + (size_t)gy * Nx + gx] = acc;
  }
}

// ------------------------------------------------------------------ optional forward stages
// (detector_blur_std models.py:379-380, obj_preblur_std :275-284)
//
// k_rblur_adj   exact transpose of k_rblur (reflect-padded separable Gaussian): the backward of
//               gaussian_blur.  Output pixel u collects the input pixels s whose padded
//               neighbourhood reads u at tap t: s = u - t + h (interior), s = -u - t + h (top /
//               left reflection, u > 0) and s = 2(n-1) - u - t + h (bottom / right, u < n-1).
//               Gather form, fixed order (deterministic, no atomics), LDS-tiled and separable.
// k_patch_gather   (O,Nz,Ny,Nx) plane → (O,Nz,B,N,N) patch stack at crop_pos[idx[b]]
//               (get_obj_ROI, models.py:251-265); lanes along x, one 256-B row segment per wave.
// k_patch_scatter  the transpose: gobj[crop + (y, x)] += gpatch, f32 atomics (overlapping
//               patches; summation order is arrival order).
// grid (ceil(Nx/kTX), ceil(Ny/kBTY), planes); block 256.  The transpose of k_rblur's (horizontal,
// then vertical) pass is the vertical transpose, then the horizontal one, tiled like k_rblur.  A
// 1-D transpose is the transposed convolution onto the reflect-padded line, folded back: output
// u takes the padded sample u + H (Σ_t w_t g[u + H − t], branch-free: the LDS tile is zero
// outside the plane) plus, within H of an edge, the padded sample its reflection came from (top
// u ∈ [1, H]: H − u; bottom u ∈ [n−1−H, n−2]: 2(n−1) − u + H).  Every source lies within H of the
// tile, so the (kBTY + 2H) × (kTX + 2H) input tile is read once, each output written once.
template <int H>
__device__ __forceinline__ float blur_adj_line(const float* col, int stride, int r, int u, int n, int base,
                                               const Taps& t) {
  // col[k·stride] = g[base + k] (0 outside [0, n)); r = u − base − H
  float acc = 0.f;
#pragma unroll
  for (int j = 0; j <= 2 * H; ++j) acc = fmaf(t.w[j], col[(r + 2 * H - j) * stride], acc);
  if (H > 0 && u >= 1 && u <= H) {   // the top reflection of u: padded H − u → g[H − u − j]
#pragma unroll
    for (int j = 0; j <= 2 * H; ++j) {
      const int sidx = H - u - j;
      if (sidx >= 0) acc = fmaf(t.w[j], col[(sidx - base) * stride], acc);
    }
  }
  if (H > 0 && u >= n - 1 - H && u <= n - 2) {   // the bottom reflection: padded 2(n−1) − u + H
#pragma unroll
    for (int j = 0; j <= 2 * H; ++j) {
      const int sidx = 2 * (n - 1) - u + H - j;
      if (sidx < n) acc = fmaf(t.w[j], col[(sidx - base) * stride], acc);
    }
  }
  return acc;
}
template <int H>
__global__ __launch_bounds__(256) void k_rblur_adj(const float* __restrict__ g, float* __restrict__ out, int Ny,
                                                   int Nx, Taps t) {
  constexpr int rows = kBTY + 2 * H, cols = kTX + 2 * H;
  __shared__ float s_g[rows][cols + 1];
  __shared__ float s_mid[kBTY][cols + 1];
  const size_t plane = (size_t)blockIdx.z * Ny * Nx;
  const int x0 = blockIdx.x * kTX, y0 = blockIdx.y * kBTY;
  for (int e = threadIdx.x; e < rows * cols; e += blockDim.x) {
    const int r = e / cols, c = e - r * cols;
    const int gy = y0 + r - H, gx = x0 + c - H;
    s_g[r][c] = gy >= 0 && gy < Ny && gx >= 0 && gx < Nx ? g[plane + (size_t)gy * Nx + gx] : 0.f;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < kBTY * cols; e += blockDim.x) {   // vertical transpose, rows u of the tile
    const int r = e / cols, c = e - r * cols;
    const int u = y0 + r;
    s_mid[r][c] = u < Ny ? blur_adj_line<H>(&s_g[0][c], cols + 1, r, u, Ny, y0 - H, t) : 0.f;
  }
  __syncthreads();
  const int c = threadIdx.x & (kTX - 1);
  const int v = x0 + c;
  for (int r = threadIdx.x >> 6; r < kBTY; r += blockDim.x >> 6) {   // horizontal transpose
    const int u = y0 + r;
    if (u >= Ny || v >= Nx) continue;
    out[plane + (size_t)u * Nx + v] = blur_adj_line<H>(&s_mid[r][0], 1, c, v, Nx, x0 - H, t);
  }
}

// ------------------------------------------------------------------ loss_simlar
// k_simlar_std: one workgroup per plane q: per pixel the unbiased std over the O modes of
// occ_o·x[o,q,pix] (mean, then the squared deviations — torch.std), summed per thread, then the
// waves in order.  k_simlar_std_grad: its backward per pixel.  OT > 0: O known at compile time
// and 4 pixels a float4 (n_pix % 4 == 0), two of them in flight per thread and mode; OT = 0 any
// O ≤ kSimlarMaxO, one pixel at a time.
constexpr int kSimlarMaxO = 32;
template <int OT>
__device__ __forceinline__ float simlar_px(const float (&w)[OT > 0 ? OT : kSimlarMaxO], int O, float& m) {
  constexpr int OM = OT > 0 ? OT : kSimlarMaxO;
  float mm = 0.f;
#pragma unroll
  for (int o = 0; o < OM; ++o)
    if (o < O) mm += w[o];
  mm *= 1.0f / (float)O;
  float v = 0.f;
#pragma unroll
  for (int o = 0; o < OM; ++o)
    if (o < O) v = fmaf(w[o] - mm, w[o] - mm, v);
  m = mm;
  return sqrtf(v * (1.0f / (float)(O - 1)));
}
template <int OT>
__global__ __launch_bounds__(256) void k_simlar_std(const float* __restrict__ x, int Odyn, long long n_planes,
                                                    int n_pix, const float* __restrict__ occ, float* __restrict__ sums) {
  constexpr int OM = OT > 0 ? OT : kSimlarMaxO;
  const int O = OT > 0 ? OT : Odyn;
  __shared__ float s_w[4];
  const long long q = blockIdx.x;
  const size_t ostr = (size_t)n_planes * n_pix;
  const float* xq = x + (size_t)q * n_pix;
  float oc[OM];
#pragma unroll
  for (int o = 0; o < OM; ++o) oc[o] = o < O ? occ[o] : 0.f;
  float acc = 0.f;
  if constexpr (OT > 0) {
    const int n4 = n_pix >> 2;
    for (int e0 = threadIdx.x; e0 < n4; e0 += 512) {
      float4 t[2][OT];
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int o = 0; o < OT; ++o)
          t[k][o] = e0 + 256 * k < n4 ? reinterpret_cast<const float4*>(xq + o * ostr)[e0 + 256 * k]
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if (e0 + 256 * k >= n4) break;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float w[OM];
#pragma unroll
          for (int o = 0; o < OT; ++o) w[o] = oc[o] * (&t[k][o].x)[c];
          float m;
          acc += simlar_px<OT>(w, O, m);
        }
      }
    }
  } else {
    for (int e = threadIdx.x; e < n_pix; e += 256) {
      float w[OM];
#pragma unroll
      for (int o = 0; o < OM; ++o) w[o] = o < O ? oc[o] * xq[o * ostr + e] : 0.f;
      float m;
      acc += simlar_px<OT>(w, O, m);
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) sums[q] = (s_w[0] + s_w[1]) + (s_w[2] + s_w[3]);
}
// grid: ceil(n_planes·n_pix / (256·PXT)) with PXT = 4 (OT > 0) or 1; thread → PXT pixels
template <int OT>
__global__ __launch_bounds__(256) void k_simlar_std_grad(const float* __restrict__ x, int Odyn, long long n_planes,
                                                         int n_pix, const float* __restrict__ occ,
                                                         const float* __restrict__ gsum, float* __restrict__ gx) {
  constexpr int OM = OT > 0 ? OT : kSimlarMaxO;
  constexpr int PXT = OT > 0 ? 4 : 1;
  const int O = OT > 0 ? OT : Odyn;
  const long long total = n_planes * n_pix;
  const long long i0 = ((long long)blockIdx.x * 256 + threadIdx.x) * PXT;
  if (i0 >= total) return;
  const long long q = i0 / n_pix;   // (n_pix % PXT == 0: a thread's pixels share the plane)
  const size_t ostr = (size_t)total;
  float oc[OM];
#pragma unroll
  for (int o = 0; o < OM; ++o) oc[o] = o < O ? occ[o] : 0.f;
  const float gq = gsum[q];
  float xv[OM][PXT];
#pragma unroll
  for (int o = 0; o < OM; ++o) {
    if (o >= O) break;
    if constexpr (PXT == 4) {
      const float4 t = *reinterpret_cast<const float4*>(x + o * ostr + i0);
      xv[o][0] = t.x; xv[o][1] = t.y; xv[o][2] = t.z; xv[o][3] = t.w;
    } else {
      xv[o][0] = x[o * ostr + i0];
    }
  }
  float gv[OM][PXT];
#pragma unroll
  for (int c = 0; c < PXT; ++c) {
    float w[OM];
#pragma unroll
    for (int o = 0; o < OM; ++o) w[o] = o < O ? oc[o] * xv[o][c] : 0.f;
    float m;
    const float sd = simlar_px<OT>(w, O, m);
    const float cc = gq / (sd * (float)(O - 1));
#pragma unroll
    for (int o = 0; o < OM; ++o) gv[o][c] = cc * oc[o] * (w[o] - m);
  }
#pragma unroll
  for (int o = 0; o < OM; ++o) {
    if (o >= O) break;
    if constexpr (PXT == 4) *reinterpret_cast<float4*>(gx + o * ostr + i0) = make_float4(gv[o][0], gv[o][1], gv[o][2], gv[o][3]);
    else gx[o * ostr + i0] = gv[o][0];
  }
}

// grid (ceil(N*N/256), B, O*Nz); block 256.  Out-of-object windows read / write nothing.
__global__ __launch_bounds__(256) void k_patch_gather(const float* __restrict__ obj, int Ny, int Nx,
                                                      const int* __restrict__ crop_pos, const int* __restrict__ idx,
                                                      int B, int N, float* __restrict__ out) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= N * N) return;
  const int b = blockIdx.y, oz = blockIdx.z;
  const int y = e / N, x = e - y * N;
  const int s = idx[b];
  const int cy = crop_pos[2 * s], cx = crop_pos[2 * s + 1];
  float val = 0.f;
  if (cy >= 0 && cx >= 0 && cy + N <= Ny && cx + N <= Nx)
    val = obj[(size_t)oz * Ny * Nx + (size_t)(cy + y) * Nx + (cx + x)];
  out[((size_t)oz * B + b) * N * N + e] = val;
}

__global__ __launch_bounds__(256) void k_patch_scatter(const float* __restrict__ gpatch, int Ny, int Nx,
                                                       const int* __restrict__ crop_pos, const int* __restrict__ idx,
                                                       int B, int N, float* __restrict__ gobj) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= N * N) return;
  const int b = blockIdx.y, oz = blockIdx.z;
  const int y = e / N, x = e - y * N;
  const int s = idx[b];
  const int cy = crop_pos[2 * s], cx = crop_pos[2 * s + 1];
  if (cy < 0 || cx < 0 || cy + N > Ny || cx + N > Nx) return;
  unsafeAtomicAdd(gobj + (size_t)oz * Ny * Nx + (size_t)(cy + y) * Nx + (cx + x),
                  gpatch[((size_t)oz * B + b) * N * N + e]);
}

// ------------------------------------------------------------------ object column pass
struct ObjCfg {
  int O, Nz, Ny, Nx;
  int zb_a, zb_p;            // obj_zblur on amplitude / phase
  Taps zt;
  int cr_a, cr_p;            // complex_ratio writes amplitude / phase
  float alpha1, alpha2;
  int mir;
  float mir_relax, mir_scale, mir_power;
  int thr;
  float thr_relax, thr_lo, thr_hi;
  int pos, pos_submin;
  float pos_relax;
  const double* stats;       // [Σ|ln a|, Σ|p|, Cbar, min p'] (device), when cr / submin are on
};

__device__ __forceinline__ float powf_pos(float x, float e) {
  // x ≥ 0; torch.pow(x, e) for float e (x = 0 → 0 for e > 0, 1 for e = 0)
  if (e == 4.0f) { const float x2 = x * x; return x2 * x2; }
  if (e == 2.0f) return x * x;
  if (e == 1.0f) return x;
  if (x == 0.f) return e == 0.f ? 1.f : 0.f;
  return exp2f(e * log2f(x));
}

// complex_ratio (both outputs from the pre-constraint a, p), then mirrored_amp, obja_thresh,
// objp_postiv, in the order of CombinedConstraint.forward (constraints.py:227-246)
__device__ __forceinline__ void pointwise(const ObjCfg& c, float cbar, float pmin, float& a, float& p) {
  if (c.cr_a | c.cr_p) {
    const float la = logf(a);
    const float an = expf((1.f - c.alpha1) * la - c.alpha1 * cbar * p);
    const float pn = (1.f - c.alpha2) * p - c.alpha2 / (cbar + 1e-8f) * la;
    if (c.cr_a) a = an;
    if (c.cr_p) p = pn;
  }
  if (c.mir) a = c.mir_relax * a + (1.f - c.mir_relax) * (1.f - c.mir_scale * powf_pos(fmaxf(p, 0.f), c.mir_power));
  if (c.thr) a = c.thr_relax * a + (1.f - c.thr_relax) * fminf(fmaxf(a, c.thr_lo), c.thr_hi);
  if (c.pos) p = c.pos_relax * p + (1.f - c.pos_relax) * (c.pos_submin ? p - pmin : fmaxf(p, 0.f));
}

// One thread per (o, y, x); register window over z.  In place: slice z is written after every
// read that needs its original value (the window holds z − h .. z + h; the only later read of
// an already-written slice would be the clamped index Nz − 1, which is written last).
template <int H>
__global__ __launch_bounds__(256) void k_obj_column(float* __restrict__ A, float* __restrict__ Pp, ObjCfg c, int pointwise_on) {
  const long long col = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long plane = (long long)c.Ny * c.Nx;
  if (col >= (long long)c.O * plane) return;
  const long long o = col / plane, yx = col - o * plane;
  float* a = A + o * c.Nz * plane + yx;
  float* p = Pp + o * c.Nz * plane + yx;
  const float cbar = (c.cr_a | c.cr_p) ? (float)c.stats[2] : 0.f;
  const float pmin = c.pos_submin ? (float)c.stats[3] : 0.f;
  const int nz = c.Nz;
  float wa[2 * H + 1], wp[2 * H + 1];
#pragma unroll
  for (int j = 0; j <= 2 * H; ++j) {
    const int z = min(max(j - H, 0), nz - 1);
    wa[j] = a[z * plane];
    wp[j] = p[z * plane];
  }
  for (int z = 0; z < nz; ++z) {
    float va = wa[H], vp = wp[H];
    if (H > 0) {
      if (c.zb_a) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j <= 2 * H; ++j) s = fmaf(c.zt.w[j], wa[j], s);
        va = s;
      }
      if (c.zb_p) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j <= 2 * H; ++j) s = fmaf(c.zt.w[j], wp[j], s);
        vp = s;
      }
    }
    // advance the window before slice z is overwritten
    const int zn = min(z + 1 + H, nz - 1);
    const float na = a[zn * plane], np_ = p[zn * plane];
#pragma unroll
    for (int j = 0; j < 2 * H; ++j) {
      wa[j] = wa[j + 1];
      wp[j] = wp[j + 1];
    }
    wa[2 * H] = na;
    wp[2 * H] = np_;
    if (pointwise_on) pointwise(c, cbar, pmin, va, vp);
    a[z * plane] = va;
    p[z * plane] = vp;
  }
}

// Block partials (fp64) for the global scalars:
//   MODE 0: Σ|ln a|, Σ|p|                 (complex_ratio Cbar, constraints.py:344)
//   MODE 1: min over p after complex_ratio (objp_postiv 'subtract_min', constraints.py:200)
template <int MODE>
__global__ __launch_bounds__(256) void k_obj_reduce(const float* __restrict__ A, const float* __restrict__ Pp, long long n,
                                                    ObjCfg c, double* part) {
  __shared__ double s0[256], s1[256];
  double v0 = MODE == 0 ? 0.0 : __builtin_huge_val(), v1 = 0.0;
  const float cbar = MODE == 1 && (c.cr_p) ? (float)c.stats[2] : 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float a = A[i], p = Pp[i];
    if (MODE == 0) {
      v0 += fabs((double)logf(a));
      v1 += fabs((double)p);
    } else {
      float pv = p;
      if (c.cr_p) pv = (1.f - c.alpha2) * p - c.alpha2 / (cbar + 1e-8f) * logf(a);
      v0 = fmin(v0, (double)pv);
    }
  }
  s0[threadIdx.x] = v0;
  s1[threadIdx.x] = v1;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      s0[threadIdx.x] = MODE == 0 ? s0[threadIdx.x] + s0[threadIdx.x + s] : fmin(s0[threadIdx.x], s0[threadIdx.x + s]);
      s1[threadIdx.x] += s1[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s0[0];
    part[2 * blockIdx.x + 1] = s1[0];
  }
}
// one block: fixed-order sum of the partials → stats
template <int MODE>
__global__ void k_reduce_final(const double* part, int nblk, double* stats) {
  if (threadIdx.x != 0) return;
  if (MODE == 0) {
    double s0 = 0, s1 = 0;
    for (int b = 0; b < nblk; ++b) {
      s0 += part[2 * b];
      s1 += part[2 * b + 1];
    }
    stats[0] = s0;
    stats[1] = s1;
    // Cbar in f32 arithmetic as the reference (sums are f32 tensors there)
    stats[2] = (double)((float)s0 / ((float)s1 + 1e-8f));
  } else {
    double m = __builtin_huge_val();
    for (int b = 0; b < nblk; ++b) m = fmin(m, part[2 * b]);
    stats[3] = m;
  }
}

// ------------------------------------------------------------------ probe: fix_probe_int
__global__ __launch_bounds__(256) void k_sumsq(const float2* __restrict__ x, long long n, double* part) {
  __shared__ double s[256];
  double v = 0;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float2 u = x[i];
    v += (double)u.x * u.x + (double)u.y * u.y;
  }
  s[threadIdx.x] = v;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) s[threadIdx.x] += s[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = s[0];
}
// scale = sqrt(target) / sqrt(Σ|P|²)   (constraints.py:76-79)
__global__ void k_fix_int_final(const double* part, int nblk, const float* target, double* stats) {
  if (threadIdx.x != 0) return;
  double s = 0;
  for (int b = 0; b < nblk; ++b) s += part[b];
  stats[4] = s;
  stats[5] = sqrt((double)target[0]) / sqrt(s);
}
__global__ __launch_bounds__(256) void k_cscale(float2* x, long long n, const double* stats) {
  const float k = (float)stats[5];
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float2 u = x[i];
    x[i] = make_float2(u.x * k, u.y * k);
  }
}

// ------------------------------------------------------------------ probe: ortho_pmode
struct Cd {
  double x, y;
};
__device__ __forceinline__ Cd cd_mul(Cd a, Cd b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
__device__ __forceinline__ Cd cd_conj(Cd a) { return {a.x, -a.y}; }
__device__ __forceinline__ Cd cd_add(Cd a, Cd b) { return {a.x + b.x, a.y + b.y}; }

// grid (nchunk, npairs): pair (i ≤ j) → partial Σ_n M_i[n] conj(M_j[n]) over chunk, fp64
__global__ __launch_bounds__(256) void k_gram(const float2* __restrict__ M, int P, long long n2, int nchunk, double* part) {
  __shared__ double sx[256], sy[256];
  int pr = blockIdx.y, i = 0;
  while (pr >= P - i) {
    pr -= P - i;
    ++i;
  }
  const int j = i + pr;
  const float2* mi = M + (size_t)i * n2;
  const float2* mj = M + (size_t)j * n2;
  const long long per = (n2 + nchunk - 1) / nchunk;
  const long long b = blockIdx.x * per, e = min(n2, b + per);
  double ax = 0, ay = 0;
  for (long long k = b + threadIdx.x; k < e; k += blockDim.x) {
    const float2 u = mi[k], v = mj[k];
    ax += (double)u.x * v.x + (double)u.y * v.y;     // u conj(v)
    ay += (double)u.y * v.x - (double)u.x * v.y;
  }
  sx[threadIdx.x] = ax;
  sy[threadIdx.x] = ay;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      sx[threadIdx.x] += sx[threadIdx.x + s];
      sy[threadIdx.x] += sy[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * ((size_t)blockIdx.y * nchunk + blockIdx.x)] = sx[0];
    part[2 * ((size_t)blockIdx.y * nchunk + blockIdx.x) + 1] = sy[0];
  }
}

// one wave: Gram matrix from the partials (fixed order), Hermitian eigendecomposition by cyclic
// complex Jacobi (fp64), geev normalisation, descending order; writes U (P × P, f32 complex,
// U[p][q] = conj(V[q][perm[p]]) so that ortho_p = Σ_q U[p][q] M_q).  Lane 0 computes each
// rotation and the convergence sum in the sequential order; the rotation's updates of row /
// column element k run on lane k (the same arithmetic per element as a sequential loop).
struct Rot {
  Cd upp, upq, uqp, uqq;
  int skip;
};
__global__ __launch_bounds__(64) void k_ortho_eig(const double* part, int P, int nchunk, float2* U, double* evals) {
  __shared__ Cd A[kMaxModes][kMaxModes];
  __shared__ Cd V[kMaxModes][kMaxModes];
  __shared__ Rot rot;
  __shared__ int done;
  const int npair = P * (P + 1) / 2;
  for (int pr = threadIdx.x; pr < npair; pr += blockDim.x) {
    int r = pr, i = 0;
    while (r >= P - i) {
      r -= P - i;
      ++i;
    }
    const int j = i + r;
    double sx = 0, sy = 0;
    for (int c = 0; c < nchunk; ++c) {
      sx += part[2 * ((size_t)pr * nchunk + c)];
      sy += part[2 * ((size_t)pr * nchunk + c) + 1];
    }
    A[i][j] = {sx, sy};
    A[j][i] = {sx, -sy};
  }
  __syncthreads();
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    A[i][i].y = 0;
    for (int j = 0; j < P; ++j) V[i][j] = {i == j ? 1.0 : 0.0, 0.0};
  }
  __syncthreads();
  double scale = 0;
  for (int i = 0; i < P; ++i) scale += A[i][i].x;
  for (int sweep = 0; sweep < 40; ++sweep) {
    if (threadIdx.x == 0) {
      double off = 0;
      for (int i = 0; i < P; ++i)
        for (int j = i + 1; j < P; ++j) off += A[i][j].x * A[i][j].x + A[i][j].y * A[i][j].y;
      done = off <= 1e-30 * scale * scale;
    }
    __syncthreads();
    if (done) break;
    for (int p = 0; p < P; ++p)
      for (int q = p + 1; q < P; ++q) {
        if (threadIdx.x == 0) {
          const double g = sqrt(A[p][q].x * A[p][q].x + A[p][q].y * A[p][q].y);
          rot.skip = g <= 1e-300;
          if (!rot.skip) {
            const Cd e = {A[p][q].x / g, A[p][q].y / g};            // phase of A_pq
            const double tau = (A[q][q].x - A[p][p].x) / (2 * g);
            const double t = (tau >= 0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1 + tau * tau));
            const double cs = 1 / sqrt(1 + t * t), sn = t * cs;
            // U = diag(1, conj(e)) · [[c, s], [-s, c]] on (p, q)
            rot.upp = {cs, 0};
            rot.upq = {sn, 0};
            rot.uqp = cd_mul({-sn, 0}, cd_conj(e));
            rot.uqq = cd_mul({cs, 0}, cd_conj(e));
          }
        }
        __syncthreads();
        if (rot.skip) {
          __syncthreads();
          continue;
        }
        const Cd upp = rot.upp, upq = rot.upq, uqp = rot.uqp, uqq = rot.uqq;
        for (int k = threadIdx.x; k < P; k += blockDim.x) {   // A ← A U, V ← V U (columns p, q)
          const Cd akp = A[k][p], akq = A[k][q];
          A[k][p] = cd_add(cd_mul(akp, upp), cd_mul(akq, uqp));
          A[k][q] = cd_add(cd_mul(akp, upq), cd_mul(akq, uqq));
          const Cd vkp = V[k][p], vkq = V[k][q];
          V[k][p] = cd_add(cd_mul(vkp, upp), cd_mul(vkq, uqp));
          V[k][q] = cd_add(cd_mul(vkp, upq), cd_mul(vkq, uqq));
        }
        __syncthreads();
        for (int k = threadIdx.x; k < P; k += blockDim.x) {   // A ← U^H A (rows p, q)
          const Cd apk = A[p][k], aqk = A[q][k];
          A[p][k] = cd_add(cd_mul(cd_conj(upp), apk), cd_mul(cd_conj(uqp), aqk));
          A[q][k] = cd_add(cd_mul(cd_conj(upq), apk), cd_mul(cd_conj(uqq), aqk));
        }
        __syncthreads();
        if (threadIdx.x == 0) {
          A[p][q] = {0, 0};
          A[q][p] = {0, 0};
          A[p][p].y = 0;
          A[q][q].y = 0;
        }
        __syncthreads();
      }
  }
  if (threadIdx.x != 0) return;
// geev normalisation: unit norm, largest-modulus component (first on ties) real positive
  for (int j = 0; j < P; ++j) {
    double nrm = 0;
    for (int k = 0; k < P; ++k) nrm += V[k][j].x * V[k][j].x + V[k][j].y * V[k][j].y;
    nrm = sqrt(nrm);
    int km = 0;
    double best = -1;
    for (int k = 0; k < P; ++k) {
      V[k][j] = {V[k][j].x / nrm, V[k][j].y / nrm};
      const double m2 = V[k][j].x * V[k][j].x + V[k][j].y * V[k][j].y;
      if (m2 > best) {
        best = m2;
        km = k;
      }
    }
    const double am = sqrt(best);
    const Cd ph = {V[km][j].x / am, -V[km][j].y / am};
    for (int k = 0; k < P; ++k) V[k][j] = cd_mul(V[k][j], ph);
    V[km][j].y = 0;
  }
  // descending eigenvalue order (stable)
  int perm[kMaxModes];
  for (int i = 0; i < P; ++i) perm[i] = i;
  for (int i = 1; i < P; ++i) {
    const int pi = perm[i];
    int k = i - 1;
    while (k >= 0 && A[perm[k]][perm[k]].x < A[pi][pi].x) {
      perm[k + 1] = perm[k];
      --k;
    }
    perm[k + 1] = pi;
  }
  for (int p = 0; p < P; ++p) {
    evals[p] = A[perm[p]][perm[p]].x;
    for (int q = 0; q < P; ++q) {
      const Cd v = V[q][perm[p]];
      U[p * P + q] = make_float2((float)v.x, (float)-v.y);
    }
  }
}

// ortho_p[n] = Σ_q U[p][q] M_q[n], one pixel per thread, in place.  PM (a compile-time constant
// so the modes of a pixel stay in registers) = P up to 16, then 32 or 64 with the modes past P
// masked (P runtime): the same fma chain for every P.
template <int PM>
__global__ __launch_bounds__(PM > 32 ? 128 : 256) void k_ortho_apply(float2* M, long long n2, const float2* U, int P) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n2) return;
  float2 m[PM];
#pragma unroll
  for (int q = 0; q < PM; ++q) m[q] = q < P ? M[(size_t)q * n2 + k] : make_float2(0.f, 0.f);
#pragma unroll
  for (int p = 0; p < PM; ++p) {
    if (p >= P) break;
    float ax = 0.f, ay = 0.f;
#pragma unroll
    for (int q = 0; q < PM; ++q) {
      if (q >= P) break;
      const float2 u = U[p * P + q];
      ax = fmaf(u.x, m[q].x, fmaf(-u.y, m[q].y, ax));
      ay = fmaf(u.x, m[q].y, fmaf(u.y, m[q].x, ay));
    }
    M[(size_t)p * n2 + k] = make_float2(ax, ay);
  }
}

}  // namespace cons
}  // namespace ptyx
