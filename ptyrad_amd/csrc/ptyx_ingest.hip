// ptyx_ingest.hip — measurement ingest straight into HBM, a translation
// unit of libptyx.so.  Replaces load_raw (src/ptyrad/load.py:19-49) and
// Initializer._process_meas (src/ptyrad/initialization.py:709-752: flipT, crop,
// remove_neg_values, normalization, final clip) for EMPAD-style raw stacks.
//
//  ptyx_raw_read     host streaming reader: large sequential pread()s of [frames + gaps] into two
//                    pinned buffers, each chunk handed to the DMA engine as ONE strided 2-D copy
//                    (source pitch = frame + gap, so the gaps are dropped by the copy engine,
//                    never touched by a kernel) while the next chunk is read.
//  ptyx_meas_stats   per output pixel, fp64 sums over frames of the transformed (flipT + crop)
//                    values, raw and with the negative-value rule applied, plus the minimum:
//                    everything _meas_remove_neg_values / _meas_normalization need, accumulated
//                    (+=) so a stack can be streamed in chunks, and summable across ranks
//                    (min with MIN, the rest with SUM) before ptyx_meas_finish.
//  ptyx_meas_finish  decides (on the device) whether the negative-value rule applies and the
//                    normalisation constant, then writes the processed stack (f32, or f16 for
//                    the fp16-storage configs) in one pass.
// Sums run in a fixed order (frame groups g = f mod G, then g = 0..G-1): bitwise reproducible.
#include <fcntl.h>
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cerrno>
#include <cstring>
#include <string>

#include "ptyx.h"
#include "ptyx_abi.hpp"

using namespace ptyx;

namespace {
constexpr int kGroups = 64;   // frame groups of the stats pass (partials per pixel)

struct Geom {
  int H, W, Ho, Wo, ky0, kx0, fu, fl, tr;
};
// output pixel (oy, ox) → source offset in the (H, W) frame: T = transpose(fliplr(flipud(S)))
__device__ __forceinline__ int src_of(const Geom& g, int oy, int ox) {
  const int a = g.ky0 + oy, b = g.kx0 + ox;
  int y = g.tr ? b : a, x = g.tr ? a : b;
  if (g.fu) y = g.H - 1 - y;
  if (g.fl) x = g.W - 1 - x;
  return y * g.W + x;
}

struct NegRule {
  int mode, force;   // 0 clip_neg, 1 subtract_min, 2 clip_value, 3 subtract_value
  float value;
};
// value after the rule and the clip that follows it (initialization.py:863-888)
__device__ __forceinline__ float neg_apply(float x, const NegRule& r, float mn) {
  switch (r.mode) {
    case 1: x = x - mn; break;
    case 2: x = x < r.value ? 0.f : x; break;
    case 3: x = x - r.value; break;
    default: break;
  }
  return fmaxf(x, 0.f);
}

// grid (ceil(P / 256), kGroups); part layout [g][0..P) raw, [g][P..2P) applied (rule with the
// min unknown: subtract_min is derived from the raw sum at the end), [g][2P + block] min
__global__ __launch_bounds__(256) void k_meas_stats(const float* __restrict__ raw, long long n, Geom g, NegRule r,
                                                    double* __restrict__ part) {
  __shared__ float s_min[256];
  const int P = g.Ho * g.Wo;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int grp = blockIdx.y;
  double sr = 0, sa = 0;
  float mn = __builtin_huge_valf();
  if (p < P) {
    const int src = src_of(g, p / g.Wo, p % g.Wo);
    const long long fs = (long long)g.H * g.W;
    for (long long f = grp; f < n; f += kGroups) {
      const float x = raw[f * fs + src];
      sr += x;
      sa += r.mode == 1 ? 0.0 : (double)neg_apply(x, r, 0.f);
      mn = fminf(mn, x);
    }
    double* pg = part + (size_t)grp * (2 * P + gridDim.x);
    pg[p] += sr;
    pg[P + p] += sa;
  }
  s_min[threadIdx.x] = mn;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) s_min[threadIdx.x] = fminf(s_min[threadIdx.x], s_min[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double* pm = part + (size_t)grp * (2 * P + gridDim.x) + 2 * P + blockIdx.x;
    *pm = fmin(*pm, (double)s_min[0]);
  }
}
__global__ void k_part_init(double* part, int P, int nblk) {
  const long long per = 2LL * P + nblk;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < per * kGroups;
       i += (long long)gridDim.x * blockDim.x)
    part[i] = (i % per) >= 2 * P ? __builtin_huge_val() : 0.0;
}
// stats = [min, n, S_raw[P], S_app[P]]; += the group partials in fixed order
__global__ __launch_bounds__(256) void k_meas_stats_final(const double* __restrict__ part, int P, int nblk, long long n,
                                                          double* __restrict__ stats) {
  const long long per = 2LL * P + nblk;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < P; p += gridDim.x * blockDim.x) {
    double sr = 0, sa = 0;
    for (int grp = 0; grp < kGroups; ++grp) {
      sr += part[grp * per + p];
      sa += part[grp * per + P + p];
    }
    stats[2 + p] += sr;
    stats[2 + P + p] += sa;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    double m = stats[0];
    for (int grp = 0; grp < kGroups; ++grp)
      for (int b = 0; b < nblk; ++b) m = fmin(m, part[grp * per + 2 * P + b]);
    stats[0] = m;
    stats[1] += (double)n;
  }
}

// [applied flag, normalisation constant] from the (rank-reduced) stats; one workgroup
__global__ __launch_bounds__(256) void k_meas_const(const double* __restrict__ stats, int P, NegRule r, int norm_mode,
                                                    float norm_value, float* __restrict__ out) {
  __shared__ double s_v[256];
  const double mn = stats[0], n = stats[1];
  const bool applied = mn < 0.0 || r.force;
  double acc = norm_mode == 0 ? -__builtin_huge_val() : 0.0;
  for (int p = threadIdx.x; p < P; p += blockDim.x) {
    double s = stats[2 + p];
    if (applied) s = r.mode == 1 ? s - n * mn : stats[2 + P + p];
    const double avg = s / n;
    acc = norm_mode == 0 ? fmax(acc, avg) : acc + avg;
  }
  s_v[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = s_v[0];
    for (int i = 1; i < (int)blockDim.x; ++i) a = norm_mode == 0 ? fmax(a, s_v[i]) : a + s_v[i];
    double c = a;
    if (norm_mode == 1) c = a / P;
    if (norm_mode == 3) c = norm_value;
    out[0] = applied ? 1.f : 0.f;
    out[1] = (float)c;
    out[2] = (float)mn;
  }
}

template <bool F16>
__global__ __launch_bounds__(256) void k_meas_finish(const float* __restrict__ raw, long long n, Geom g, NegRule r,
                                                     const float* __restrict__ cst, void* __restrict__ dst) {
  const int P = g.Ho * g.Wo;
  const long long total = n * P;
  const bool applied = cst[0] != 0.f;
  const float c = cst[1], mn = cst[2];
  const long long fs = (long long)g.H * g.W;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long f = i / P;
    const int p = (int)(i - f * P);
    float x = raw[f * fs + src_of(g, p / g.Wo, p % g.Wo)];
    if (applied) x = neg_apply(x, r, mn);
    x = fmaxf(x / c, 0.f);
    if constexpr (F16) reinterpret_cast<__half*>(dst)[i] = __float2half(x);
    else reinterpret_cast<float*>(dst)[i] = x;
  }
}

int make_geom(const ptyx_meas_proc* pp, int H, int W, Geom& g, NegRule& r) {
  if (!pp) return abi::fail(PTYX_EINVAL, "meas: proc is null");
  if (H <= 0 || W <= 0) return abi::fail(PTYX_EINVAL, "meas: bad frame shape");
  g.H = H;
  g.W = W;
  g.fu = pp->flipud != 0;
  g.fl = pp->fliplr != 0;
  g.tr = pp->transpose != 0;
  const int Ht = g.tr ? W : H, Wt = g.tr ? H : W;
  const int ky0 = pp->crop_ky0 < 0 ? 0 : pp->crop_ky0, ky1 = pp->crop_ky1 < 0 ? Ht : pp->crop_ky1;
  const int kx0 = pp->crop_kx0 < 0 ? 0 : pp->crop_kx0, kx1 = pp->crop_kx1 < 0 ? Wt : pp->crop_kx1;
  if (ky0 >= ky1 || kx0 >= kx1 || ky1 > Ht || kx1 > Wt) return abi::fail(PTYX_EINVAL, "meas: crop out of range");
  g.ky0 = ky0;
  g.kx0 = kx0;
  g.Ho = ky1 - ky0;
  g.Wo = kx1 - kx0;
  if (pp->neg_mode < 0 || pp->neg_mode > 3) return abi::fail(PTYX_EINVAL, "meas: neg_mode must be 0..3");
  if (pp->norm_mode < 0 || pp->norm_mode > 3) return abi::fail(PTYX_EINVAL, "meas: norm_mode must be 0..3");
  r.mode = pp->neg_mode;
  r.force = pp->neg_force;
  r.value = pp->neg_value;
  return PTYX_OK;
}
}  // namespace

extern "C" size_t ptyx_meas_stats_len(int32_t Ho, int32_t Wo) { return 2 + 2 * (size_t)Ho * Wo; }
extern "C" size_t ptyx_meas_ws_bytes(int32_t Ho, int32_t Wo) {
  const size_t P = (size_t)Ho * Wo, nblk = (P + 255) / 256;
  return (kGroups * (2 * P + nblk) + 4) * sizeof(double);
}

extern "C" int ptyx_meas_stats(void* stream, const float* raw, int64_t n, int32_t H, int32_t W,
                               const ptyx_meas_proc* p, double* stats, void* ws) {
  abi::clear_error();
  Geom g;
  NegRule r;
  int rc = make_geom(p, H, W, g, r);
  if (rc) return rc;
  if (n < 0) return abi::fail(PTYX_EINVAL, "meas_stats: n < 0");
  if (!stats || !ws || (n > 0 && !raw)) return abi::fail(PTYX_EINVAL, "meas_stats: null pointer");
  if (n == 0) return PTYX_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int P = g.Ho * g.Wo, nblk = (P + 255) / 256;
  double* part = reinterpret_cast<double*>(ws);
  hipLaunchKernelGGL(k_part_init, dim3(256), dim3(256), 0, st, part, P, nblk);
  hipLaunchKernelGGL(k_meas_stats, dim3(nblk, kGroups), dim3(256), 0, st, raw, (long long)n, g, r, part);
  hipLaunchKernelGGL(k_meas_stats_final, dim3(nblk), dim3(256), 0, st, part, P, nblk, (long long)n, stats);
  return abi::launch_status("meas_stats launch");
}

extern "C" int ptyx_meas_finish(void* stream, const float* raw, int64_t n, int32_t H, int32_t W,
                                const ptyx_meas_proc* p, const double* stats, void* ws, void* dst, int32_t dst_f16) {
  abi::clear_error();
  Geom g;
  NegRule r;
  int rc = make_geom(p, H, W, g, r);
  if (rc) return rc;
  if (n < 0) return abi::fail(PTYX_EINVAL, "meas_finish: n < 0");
  if (!stats || !ws || (n > 0 && (!raw || !dst))) return abi::fail(PTYX_EINVAL, "meas_finish: null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int P = g.Ho * g.Wo;
  float* cst = reinterpret_cast<float*>(ws);
  hipLaunchKernelGGL(k_meas_const, dim3(1), dim3(256), 0, st, stats, P, r, p->norm_mode, p->norm_value, cst);
  if (n > 0) {
    const long long total = n * (long long)P;
    const unsigned grid = (unsigned)std::min<long long>((total + 255) / 256, 65536);
    if (dst_f16) hipLaunchKernelGGL(k_meas_finish<true>, dim3(grid), dim3(256), 0, st, raw, (long long)n, g, r, cst, dst);
    else hipLaunchKernelGGL(k_meas_finish<false>, dim3(grid), dim3(256), 0, st, raw, (long long)n, g, r, cst, dst);
  }
  return abi::launch_status("meas_finish launch");
}

// ---------------------------------------------------------------------------------------------
// meas_pad / meas_resample (initialization.py:956-1102).  The mean pattern comes from the stats
// (the same per-pixel sums the normalisation used, so a sharded ingest fits the global mean);
// the 2-parameter background fit runs on the host (ptyrad_amd/ingest.py); the background and the
// fused paste + bilinear zoom run here.
namespace {
__global__ __launch_bounds__(256) void k_meas_mean(const double* __restrict__ stats, int P, NegRule r,
                                                   const float* __restrict__ cst, double* __restrict__ mean) {
  const double mn = stats[0], n = stats[1];
  const bool applied = cst[0] != 0.f;
  const double c = (double)cst[1];
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < P; p += gridDim.x * blockDim.x) {
    double s = stats[2 + p];
    if (applied) s = r.mode == 1 ? s - n * mn : stats[2 + P + p];
    mean[p] = s / n / c;
  }
}

// The reference's own f32 mean pattern (numpy's meas.mean(0) on a float32 stack: frame by frame
// in f32, then / n in f32 — a sequential sum, bit for bit): one thread per output pixel, frames in
// order, of the value after the negative-value rule (normalized = 0), or of that value divided by
// the normalisation constant as ptyx_meas_finish stores it (normalized = 1).  Not decomposable
// over ranks or chunks (the f64 stats are); the single-rank ingest uses it so that the
// normalisation constant and meas_pad's background fit see exactly the reference's values.
__global__ __launch_bounds__(256) void k_meas_mean_seq(const float* __restrict__ raw, long long n, Geom g, NegRule r,
                                                       const float* __restrict__ cst, int normalized,
                                                       float* __restrict__ mean) {
  const int P = g.Ho * g.Wo;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const bool applied = cst[0] != 0.f;
  const float c = cst[1], mn = cst[2];
  const long long fs = (long long)g.H * g.W;
  const float* src = raw + src_of(g, p / g.Wo, p % g.Wo);
  float acc = 0.f;
  long long f = 0;
  for (; f + 8 <= n; f += 8) {
    float x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = src[(f + i) * fs];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float v = applied ? neg_apply(x[i], r, mn) : x[i];
      if (normalized) v = fmaxf(v / c, 0.f);
      acc = __fadd_rn(acc, v);
    }
  }
  for (; f < n; ++f) {
    float v = applied ? neg_apply(src[f * fs], r, mn) : src[f * fs];
    if (normalized) v = fmaxf(v / c, 0.f);
    acc = __fadd_rn(acc, v);
  }
  mean[p] = acc / (float)n;
}

struct PadGeom {
  int Hm, Wm, Hp, Wp, h1, w1, type;
  double a, b, value;
};

// numpy.linspace(end, edge, w, endpoint=False)[k] = k·((edge - end)/w) + end, cast to f32
__device__ __forceinline__ float ramp_at(float edge, double end, int w, int k) {
  return (float)((double)k * (((double)edge - end) / (double)w) + end);
}
__device__ __forceinline__ float amp_of(const double* __restrict__ mean, const PadGeom& g, int y, int x) {
  return sqrtf((float)mean[(size_t)y * g.Wm + x]);
}
// numpy.pad(linear_ramp) pads axis 0 over the frame's columns first, then axis 1 over all rows
__device__ float ramp_col(const double* __restrict__ mean, const PadGeom& g, int i, int jj) {
  const int ii = i - g.h1;
  if (ii < 0) return ramp_at(amp_of(mean, g, 0, jj), g.value, g.h1, i);
  if (ii >= g.Hm) {
    const int w = g.Hp - g.h1 - g.Hm;
    return ramp_at(amp_of(mean, g, g.Hm - 1, jj), g.value, w, w - 1 - (ii - g.Hm));
  }
  return amp_of(mean, g, ii, jj);
}

__global__ __launch_bounds__(256) void k_pad_background(const double* __restrict__ mean, PadGeom g,
                                                        double* __restrict__ bg) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= g.Hp * g.Wp) return;
  const int y = e / g.Wp, x = e - y * g.Wp;
  const int yy = y - g.h1, xx = x - g.w1;
  if (yy >= 0 && yy < g.Hm && xx >= 0 && xx < g.Wm) {
    bg[e] = 0.0;
    return;
  }
  double v;
  if (g.type <= 2) {
    float amp;
    if (g.type == 0) {
      amp = (float)g.value;
    } else if (g.type == 1) {
      amp = amp_of(mean, g, min(max(yy, 0), g.Hm - 1), min(max(xx, 0), g.Wm - 1));
    } else if (xx < 0) {
      amp = ramp_at(ramp_col(mean, g, y, 0), g.value, g.w1, x);
    } else if (xx >= g.Wm) {
      const int w = g.Wp - g.w1 - g.Wm;
      amp = ramp_at(ramp_col(mean, g, y, g.Wm - 1), g.value, w, w - 1 - (xx - g.Wm));
    } else {
      amp = ramp_col(mean, g, y, xx);
    }
    v = (double)(amp * amp);   // np.square of the f32 amplitude
  } else {
    const double dy = (double)y - (double)(g.Hm / 2 + g.h1), dx = (double)x - (double)(g.Wm / 2 + g.w1);
    const double r = sqrt(dy * dy + dx * dx) + 1e-10;
    const double amp = g.type == 3 ? g.a * exp(-g.b * r) : g.a * pow(r, -g.b);
    v = amp * amp;
  }
  bg[e] = v;
}

struct ZoomGeom {
  int Hm, Wm, Hp, Wp, h1, w1, Ho, Wo, src_f16, dst_f16, zoom;
  double ry, rx;   // (Hp-1)/(Ho-1), (Wp-1)/(Wo-1); 1 when the output axis has one pixel
};

__device__ __forceinline__ double canvas_at(const void* __restrict__ src, size_t base, const double* __restrict__ bg,
                                            const ZoomGeom& g, int r, int c) {
  const int rr = r - g.h1, cc = c - g.w1;
  if (rr >= 0 && rr < g.Hm && cc >= 0 && cc < g.Wm) {
    const size_t off = base + (size_t)rr * g.Wm + cc;
    return g.src_f16 ? (double)__half2float(reinterpret_cast<const __half*>(src)[off])
                     : (double)reinterpret_cast<const float*>(src)[off];
  }
  return bg ? bg[(size_t)r * g.Wp + c] : 0.0;
}

// order-1 spline weights at coordinate c on an axis of n points: (i0, i1, t); false when c lies
// past the last pixel — scipy's mode 'constant' then returns cval = 0 for the whole output pixel,
// even when only the rounding of o·(n-1)/(no-1) put it there (32 px zoomed by 0.5: 31.000000000000004)
__device__ __forceinline__ bool zoom_src(int o, double ratio, int n, int& i0, int& i1, double& t) {
  const double c = (double)o * ratio;
  i0 = min((int)floor(c), n - 1);
  t = c - (double)i0;
  if (t < 0.0) t = 0.0;
  i1 = i0 + 1 < n ? i0 + 1 : i0;
  return c <= (double)(n - 1);
}

__global__ __launch_bounds__(256) void k_pad_resample(const void* __restrict__ src, long long n,
                                                      const double* __restrict__ bg, ZoomGeom g,
                                                      void* __restrict__ dst) {
  const long long per = (long long)g.Ho * g.Wo, total = n * per;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long f = i / per;
    const int e = (int)(i - f * per);
    const int y = e / g.Wo, x = e - y * g.Wo;
    const size_t base = (size_t)f * g.Hm * g.Wm;
    double v;
    if (!g.zoom) {
      v = canvas_at(src, base, bg, g, y, x);
    } else {
      int y0, y1, x0, x1;
      double ty, tx;
      const bool iny = zoom_src(y, g.ry, g.Hp, y0, y1, ty);
      const bool inx = zoom_src(x, g.rx, g.Wp, x0, x1, tx);
      const double wy = 1.0 - ty, wx = 1.0 - tx;
      v = canvas_at(src, base, bg, g, y0, x0) * wy * wx;
      v += canvas_at(src, base, bg, g, y0, x1) * wy * tx;
      v += canvas_at(src, base, bg, g, y1, x0) * ty * wx;
      v += canvas_at(src, base, bg, g, y1, x1) * ty * tx;
      if (!(iny && inx)) v = 0.0;
    }
    if (g.dst_f16) reinterpret_cast<__half*>(dst)[i] = __float2half((float)v);
    else reinterpret_cast<float*>(dst)[i] = (float)v;
  }
}
}  // namespace

extern "C" int ptyx_meas_mean(void* stream, int32_t H, int32_t W, const ptyx_meas_proc* p, const double* stats,
                              void* ws, double* mean) {
  abi::clear_error();
  Geom g;
  NegRule r;
  int rc = make_geom(p, H, W, g, r);
  if (rc) return rc;
  if (!stats || !ws || !mean) return abi::fail(PTYX_EINVAL, "meas_mean: null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int P = g.Ho * g.Wo;
  float* cst = reinterpret_cast<float*>(ws);
  hipLaunchKernelGGL(k_meas_const, dim3(1), dim3(256), 0, st, stats, P, r, p->norm_mode, p->norm_value, cst);
  hipLaunchKernelGGL(k_meas_mean, dim3((P + 255) / 256), dim3(256), 0, st, stats, P, r, cst, mean);
  return abi::launch_status("meas_mean launch");
}

extern "C" int ptyx_meas_mean_seq(void* stream, const float* raw, int64_t n, int32_t H, int32_t W,
                                  const ptyx_meas_proc* p, const double* stats, void* ws, int32_t normalized,
                                  float* mean) {
  abi::clear_error();
  Geom g;
  NegRule r;
  int rc = make_geom(p, H, W, g, r);
  if (rc) return rc;
  if (n <= 0) return abi::fail(PTYX_EINVAL, "meas_mean_seq: n must be > 0");
  if (!raw || !stats || !ws || !mean) return abi::fail(PTYX_EINVAL, "meas_mean_seq: null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int P = g.Ho * g.Wo;
  float* cst = reinterpret_cast<float*>(ws);
  hipLaunchKernelGGL(k_meas_const, dim3(1), dim3(256), 0, st, stats, P, r, p->norm_mode, p->norm_value, cst);
  hipLaunchKernelGGL(k_meas_mean_seq, dim3((P + 255) / 256), dim3(256), 0, st, raw, (long long)n, g, r, cst,
                     normalized ? 1 : 0, mean);
  return abi::launch_status("meas_mean_seq launch");
}

extern "C" int ptyx_meas_pad_background(void* stream, const double* mean, int32_t Hm, int32_t Wm, int32_t pad_type,
                                        double a, double b, double value, int32_t Hp, int32_t Wp, int32_t h1,
                                        int32_t w1, double* bg) {
  abi::clear_error();
  if (Hm <= 0 || Wm <= 0 || Hp <= 0 || Wp <= 0) return abi::fail(PTYX_EINVAL, "meas_pad_background: bad shape");
  if (pad_type < 0 || pad_type > 4) return abi::fail(PTYX_EINVAL, "meas_pad_background: pad_type must be 0..4");
  if (h1 < 0 || w1 < 0 || h1 + Hm > Hp || w1 + Wm > Wp)
    return abi::fail(PTYX_EINVAL, "meas_pad_background: the frame does not fit the canvas");
  if (!bg || (pad_type >= 1 && pad_type <= 2 && !mean)) return abi::fail(PTYX_EINVAL, "meas_pad_background: null pointer");
  PadGeom g{Hm, Wm, Hp, Wp, h1, w1, pad_type, a, b, value};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_pad_background, dim3((Hp * Wp + 255) / 256), dim3(256), 0, st, mean, g, bg);
  return abi::launch_status("meas_pad_background launch");
}

extern "C" int ptyx_meas_pad_resample(void* stream, const void* src, int32_t src_f16, int64_t n, int32_t Hm,
                                      int32_t Wm, const double* bg, int32_t Hp, int32_t Wp, int32_t h1, int32_t w1,
                                      int32_t Ho, int32_t Wo, void* dst, int32_t dst_f16) {
  abi::clear_error();
  if (Hm <= 0 || Wm <= 0 || Ho <= 0 || Wo <= 0 || n < 0) return abi::fail(PTYX_EINVAL, "meas_pad_resample: bad shape");
  if (!bg && (Hp != Hm || Wp != Wm || h1 != 0 || w1 != 0))
    return abi::fail(PTYX_EINVAL, "meas_pad_resample: without a background Hp, Wp must equal Hm, Wm and h1 = w1 = 0");
  if (h1 < 0 || w1 < 0 || h1 + Hm > Hp || w1 + Wm > Wp)
    return abi::fail(PTYX_EINVAL, "meas_pad_resample: the frame does not fit the canvas");
  if (n == 0) return PTYX_OK;
  if (!src || !dst) return abi::fail(PTYX_EINVAL, "meas_pad_resample: null pointer");
  const bool zoom = Ho != Hp || Wo != Wp;
  ZoomGeom g{Hm, Wm, Hp, Wp, h1, w1, Ho, Wo, src_f16 ? 1 : 0, dst_f16 ? 1 : 0, zoom ? 1 : 0,
             Ho > 1 ? (double)(Hp - 1) / (double)(Ho - 1) : 1.0, Wo > 1 ? (double)(Wp - 1) / (double)(Wo - 1) : 1.0};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const long long total = n * (long long)Ho * Wo;
  const unsigned grid = (unsigned)std::min<long long>((total + 255) / 256, 65536);
  hipLaunchKernelGGL(k_pad_resample, dim3(grid), dim3(256), 0, st, src, (long long)n, bg, g, dst);
  return abi::launch_status("meas_pad_resample launch");
}

extern "C" int ptyx_raw_read(void* stream, const char* path, int64_t offset, int32_t H, int32_t W, int32_t gap,
                             int64_t file_frames, int64_t first, int64_t count, float* dst) {
  abi::clear_error();
  if (!path || H <= 0 || W <= 0 || gap < 0 || offset < 0 || file_frames < 0)
    return abi::fail(PTYX_EINVAL, "raw_read: bad arguments");
  if (first < 0 || count < 0 || first + count > file_frames) return abi::fail(PTYX_EINVAL, "raw_read: frame range");
  if (count > 0 && !dst) return abi::fail(PTYX_EINVAL, "raw_read: dst is null");
  const size_t frame = (size_t)H * W * 4, stride = frame + (size_t)gap;
  struct stat sb;
  if (stat(path, &sb) != 0) return abi::fail(PTYX_EINVAL, std::string("raw_read: cannot stat ") + path);
  const long long expected = offset + file_frames * (long long)stride;   // load.py:27-31
  if ((long long)sb.st_size != expected)
    return abi::fail(PTYX_EINVAL, "raw_read: file size " + std::to_string((long long)sb.st_size) + " != offset + N*(H*W*4 + gap) = " +
                                      std::to_string(expected));
  if (count == 0) return PTYX_OK;
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return abi::fail(PTYX_EINVAL, std::string("raw_read: open failed: ") + std::strerror(errno));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const size_t chunk_frames = std::max<size_t>(1, (64u << 20) / stride);
  void* buf[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  int rc = PTYX_OK;
  for (int i = 0; i < 2 && rc == PTYX_OK; ++i) {
    if (hipHostMalloc(&buf[i], chunk_frames * stride, hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess)
      rc = abi::fail(PTYX_ENOMEM, "raw_read: pinned buffer allocation failed");
  }
  bool pending[2] = {false, false};
  for (long long f = 0, k = 0; rc == PTYX_OK && f < count; f += (long long)chunk_frames, ++k) {
    const int b = (int)(k & 1);
    if (pending[b] && hipEventSynchronize(ev[b]) != hipSuccess) {
      rc = abi::fail(PTYX_EHIP, "raw_read: event sync failed");
      break;
    }
    const size_t nf = (size_t)std::min<long long>((long long)chunk_frames, count - f);
    // the last frame's trailing gap is not needed
    const size_t bytes = nf * stride - (size_t)gap;
    size_t got = 0;
    const off_t base = (off_t)(offset + (first + f) * (long long)stride);
    while (got < bytes) {
      const ssize_t r = pread(fd, (char*)buf[b] + got, bytes - got, base + (off_t)got);
      if (r <= 0) {
        rc = abi::fail(PTYX_EINVAL, std::string("raw_read: short read: ") + (r < 0 ? std::strerror(errno) : "EOF"));
        break;
      }
      got += (size_t)r;
    }
    if (rc) break;
    if (hipMemcpy2DAsync(dst + (size_t)f * H * W, frame, buf[b], stride, frame, nf, hipMemcpyHostToDevice, st) !=
            hipSuccess ||
        hipEventRecord(ev[b], st) != hipSuccess) {
      rc = abi::fail(PTYX_EHIP, "raw_read: strided DMA failed");
      break;
    }
    pending[b] = true;
  }
  for (int i = 0; i < 2; ++i) {
    if (pending[i]) (void)hipEventSynchronize(ev[i]);
    if (ev[i]) (void)hipEventDestroy(ev[i]);
    if (buf[i]) (void)hipHostFree(buf[i]);
  }
  close(fd);
  return rc;
}

// ---------------------------------------------------------------------------------------------
// ptyx_meas_gather — PtychoAD.get_measurements(indices) with the on-the-fly options
// (src/ptyrad/models.py:384-412): each selected frame is pasted into the padding canvas
// (canvas[h1:h1+Hm, w1:w1+Wm] = meas[idx[b]]), then bilinearly resampled as
// torch.nn.functional.interpolate(scale_factor, mode='bilinear', align_corners=False) does
// (source index s·(i+0.5)-0.5 clamped at 0, s = 1/scale_factor rounded to f32) and divided by
// scale_y·scale_x.  One thread per output pixel; the canvas composite is never materialised.
namespace {
struct OtfGeom {
  int Hm, Wm, Hp, Wp, h1, w1, Ho, Wo;
  float inv_sy, inv_sx, norm;
  int resample, f16;
};

__device__ __forceinline__ float otf_canvas(const void* __restrict__ meas, size_t base,
                                            const float* __restrict__ canvas, const OtfGeom& g, int r, int c) {
  const int rr = r - g.h1, cc = c - g.w1;
  if (rr >= 0 && rr < g.Hm && cc >= 0 && cc < g.Wm) {
    const size_t off = base + (size_t)rr * g.Wm + cc;
    return g.f16 ? __half2float(reinterpret_cast<const __half*>(meas)[off]) : reinterpret_cast<const float*>(meas)[off];
  }
  return canvas ? canvas[(size_t)r * g.Wp + c] : 0.f;
}

// aten area_pixel_compute_source_index (align_corners=False, linear) + guard_index_and_lambda
__device__ __forceinline__ void otf_src(int i, float inv_s, int in, int& i0, int& i1, float& l1) {
  float real = __fsub_rn(__fmul_rn(inv_s, __fadd_rn((float)i, 0.5f)), 0.5f);
  if (real < 0.f) real = 0.f;
  i0 = min((int)floorf(real), in - 1);
  l1 = fminf(fmaxf(real - (float)i0, 0.f), 1.f);
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
}

__global__ __launch_bounds__(256) void k_meas_gather(const void* __restrict__ meas, const int* __restrict__ idx,
                                                     const float* __restrict__ canvas, OtfGeom g,
                                                     float* __restrict__ out) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= g.Ho * g.Wo) return;
  const int b = blockIdx.y;
  const int y = e / g.Wo, x = e - y * g.Wo;
  const size_t base = (size_t)idx[b] * g.Hm * g.Wm;
  float v;
  if (!g.resample) {
    v = otf_canvas(meas, base, canvas, g, y, x);
  } else {
    int y0, y1, x0, x1;
    float ly, lx;
    otf_src(y, g.inv_sy, g.Hp, y0, y1, ly);
    otf_src(x, g.inv_sx, g.Wp, x0, x1, lx);
    const float a00 = otf_canvas(meas, base, canvas, g, y0, x0), a01 = otf_canvas(meas, base, canvas, g, y0, x1);
    const float a10 = otf_canvas(meas, base, canvas, g, y1, x0), a11 = otf_canvas(meas, base, canvas, g, y1, x1);
    v = (1.f - ly) * ((1.f - lx) * a00 + lx * a01) + ly * ((1.f - lx) * a10 + lx * a11);
    v = v / g.norm;
  }
  out[(size_t)b * g.Ho * g.Wo + e] = v;
}
}  // namespace

extern "C" int ptyx_meas_gather(void* stream, const void* meas, int32_t meas_f16, int32_t Hm, int32_t Wm,
                                const int32_t* idx, int32_t n_idx, const float* canvas, int32_t Hp, int32_t Wp,
                                int32_t h1, int32_t w1, double scale_y, double scale_x, int32_t Ho, int32_t Wo,
                                float* out) {
  abi::clear_error();
  if (Hm <= 0 || Wm <= 0 || n_idx < 0 || Ho <= 0 || Wo <= 0) return abi::fail(PTYX_EINVAL, "meas_gather: bad shape");
  if (!canvas && (Hp != Hm || Wp != Wm || h1 != 0 || w1 != 0))
    return abi::fail(PTYX_EINVAL, "meas_gather: without a canvas Hp, Wp must equal Hm, Wm and h1 = w1 = 0");
  if (h1 < 0 || w1 < 0 || h1 + Hm > Hp || w1 + Wm > Wp)
    return abi::fail(PTYX_EINVAL, "meas_gather: the frame does not fit the padding canvas");
  if (!(scale_y > 0.0) || !(scale_x > 0.0)) return abi::fail(PTYX_EINVAL, "meas_gather: scale factors must be > 0");
  const bool resample = scale_y != 1.0 || scale_x != 1.0;
  if (Ho != (resample ? (int32_t)std::floor(Hp * scale_y) : Hp) ||
      Wo != (resample ? (int32_t)std::floor(Wp * scale_x) : Wp))
    return abi::fail(PTYX_EINVAL, "meas_gather: output size must be floor(padded size * scale_factor)");
  if (n_idx > 65535) return abi::fail(PTYX_EUNSUPPORTED, "meas_gather: at most 65535 frames per call");
  if (n_idx == 0) return PTYX_OK;
  if (!meas || !idx || !out) return abi::fail(PTYX_EINVAL, "meas_gather: null pointer");
  OtfGeom g{Hm, Wm, Hp, Wp, h1, w1, Ho, Wo, (float)(1.0 / scale_y), (float)(1.0 / scale_x),
            (float)(scale_y * scale_x), resample ? 1 : 0, meas_f16 ? 1 : 0};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_meas_gather, dim3((Ho * Wo + 255) / 256, n_idx), dim3(256), 0, st, meas, idx, canvas, g, out);
  return abi::launch_status("k_meas_gather launch");
}
