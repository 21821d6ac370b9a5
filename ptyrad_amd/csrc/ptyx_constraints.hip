// ptyx_constraints.hip — C ABI of the on-device constraints (include/ptyx.h), a translation unit
// of libptyx.so of its own (kernels in ptyx_constraints.hpp).
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>

#include "ptyx.h"
#include "ptyx_abi.hpp"
#include "ptyx_constraints.hpp"

using namespace ptyx;

namespace {
using cons::kMaxHalf;
using cons::kMaxModes;
using cons::kRedBlocks;
constexpr int kGramChunks = 64;
// workspace layout (doubles): stats[8] | partials[2·kRedBlocks] | gram[2·pairs·chunks] | evals[kMaxModes]
// | U (kMaxModes² float2)
constexpr size_t kWsStats = 0, kWsPart = 8, kWsGram = kWsPart + 2 * kRedBlocks,
                 kWsEvals = kWsGram + 2 * (kMaxModes * (kMaxModes + 1) / 2) * kGramChunks, kWsU = kWsEvals + kMaxModes;
constexpr size_t kWsBytes = kWsU * sizeof(double) + kMaxModes * kMaxModes * sizeof(float2);

// scipy.signal.windows.gaussian(k, std) / sum, f64 then f32 (utils/image_proc.py:435-449)
cons::Taps scipy_taps(int ks, double std) {
  cons::Taps t{};
  t.half = ks / 2;
  double w[cons::kMaxTaps], sum = 0;
  for (int i = 0; i < ks; ++i) {
    const double n = i - (ks - 1) / 2.0;
    w[i] = std::exp(-0.5 * (n / std) * (n / std));
    sum += w[i];
  }
  for (int i = 0; i < ks; ++i) t.w[i] = (float)(w[i] / sum);
  return t;
}
// torchvision _get_gaussian_kernel1d: f32 linspace, exp, normalise in f32
cons::Taps torchvision_taps(int ks, float sigma) {
  cons::Taps t{};
  t.half = ks / 2;
  const float half = (ks - 1) * 0.5f;
  float sum = 0.f;
  for (int i = 0; i < ks; ++i) {
    const float x = ks > 1 ? -half + i * ((2 * half) / (float)(ks - 1)) : 0.f;
    t.w[i] = std::exp(-0.5f * (x / sigma) * (x / sigma));
    sum += t.w[i];
  }
  for (int i = 0; i < ks; ++i) t.w[i] /= sum;
  return t;
}

// the separable blur (or its transpose) with H = kernel_size / 2 at compile time
template <bool ADJ, int H>
void launch_blur(hipStream_t st, const float* in, float* out, int n_planes, int Ny, int Nx, const cons::Taps& t) {
  const dim3 gr((Nx + cons::kTX - 1) / cons::kTX, (Ny + cons::kBTY - 1) / cons::kBTY, n_planes);
  if constexpr (ADJ) hipLaunchKernelGGL(cons::k_rblur_adj<H>, gr, dim3(256), 0, st, in, out, Ny, Nx, t);
  else hipLaunchKernelGGL(cons::k_rblur<H>, gr, dim3(256), 0, st, in, out, Ny, Nx, t);
}
template <bool ADJ>
void launch_blur_h(int h, hipStream_t st, const float* in, float* out, int n_planes, int Ny, int Nx,
                   const cons::Taps& t) {
  switch (h) {
    case 0: launch_blur<ADJ, 0>(st, in, out, n_planes, Ny, Nx, t); break;
    case 1: launch_blur<ADJ, 1>(st, in, out, n_planes, Ny, Nx, t); break;
    case 2: launch_blur<ADJ, 2>(st, in, out, n_planes, Ny, Nx, t); break;
    case 3: launch_blur<ADJ, 3>(st, in, out, n_planes, Ny, Nx, t); break;
    case 4: launch_blur<ADJ, 4>(st, in, out, n_planes, Ny, Nx, t); break;
    case 5: launch_blur<ADJ, 5>(st, in, out, n_planes, Ny, Nx, t); break;
    case 6: launch_blur<ADJ, 6>(st, in, out, n_planes, Ny, Nx, t); break;
    default: launch_blur<ADJ, 7>(st, in, out, n_planes, Ny, Nx, t); break;
  }
}

template <int H>
void launch_column(hipStream_t st, float* a, float* p, const cons::ObjCfg& c, int pointwise_on) {
  const long long cols = (long long)c.O * c.Ny * c.Nx;
  hipLaunchKernelGGL(cons::k_obj_column<H>, dim3((unsigned)((cols + 255) / 256)), dim3(256), 0, st, a, p, c,
                     pointwise_on);
}
void launch_column_h(int h, hipStream_t st, float* a, float* p, const cons::ObjCfg& c, int pw) {
  switch (h) {
    case 0: launch_column<0>(st, a, p, c, pw); break;
    case 1: launch_column<1>(st, a, p, c, pw); break;
    case 2: launch_column<2>(st, a, p, c, pw); break;
    case 3: launch_column<3>(st, a, p, c, pw); break;
    case 4: launch_column<4>(st, a, p, c, pw); break;
    case 5: launch_column<5>(st, a, p, c, pw); break;
    case 6: launch_column<6>(st, a, p, c, pw); break;
    default: launch_column<7>(st, a, p, c, pw); break;
  }
}
template <int PM>
void launch_ortho_apply(hipStream_t st, float2* M, long long n2, const float2* U, int P) {
  constexpr int B = PM > 32 ? 128 : 256;
  hipLaunchKernelGGL(cons::k_ortho_apply<PM>, dim3((unsigned)((n2 + B - 1) / B)), dim3(B), 0, st, M, n2, U, P);
}
}  // namespace

extern "C" size_t ptyx_constraints_ws_bytes(void) { return kWsBytes; }
extern "C" size_t ptyx_constraints_evals_offset(void) { return kWsEvals * sizeof(double); }

extern "C" int ptyx_obj_rblur(void* stream, const float* in, float* out, int32_t n_planes, int32_t Ny, int32_t Nx,
                              int32_t kernel_size, float sigma) {
  abi::clear_error();
  if (n_planes < 0 || Ny <= 0 || Nx <= 0) return abi::fail(PTYX_EINVAL, "obj_rblur: bad shape");
  if (kernel_size < 1 || kernel_size % 2 == 0 || kernel_size / 2 > kMaxHalf)
    return abi::fail(PTYX_EUNSUPPORTED, "obj_rblur: kernel_size must be odd and <= 15");
  if (!(sigma > 0.f)) return abi::fail(PTYX_EINVAL, "obj_rblur: sigma must be > 0");
  if (kernel_size / 2 >= Ny || kernel_size / 2 >= Nx)
    return abi::fail(PTYX_EINVAL, "obj_rblur: reflect padding needs kernel_size/2 < Ny, Nx");
  if (n_planes == 0) return PTYX_OK;
  if (!in || !out || in == out) return abi::fail(PTYX_EINVAL, "obj_rblur: in / out null or aliased");
  const cons::Taps t = torchvision_taps(kernel_size, sigma);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  launch_blur_h<false>(t.half, st, in, out, n_planes, Ny, Nx, t);
  return abi::launch_status("k_rblur launch");
}

extern "C" int ptyx_blur_adjoint(void* stream, const float* in, float* out, int32_t n_planes, int32_t Ny,
                                 int32_t Nx, int32_t kernel_size, float sigma) {
  abi::clear_error();
  if (n_planes < 0 || Ny <= 0 || Nx <= 0) return abi::fail(PTYX_EINVAL, "blur_adjoint: bad shape");
  if (kernel_size < 1 || kernel_size % 2 == 0 || kernel_size / 2 > kMaxHalf)
    return abi::fail(PTYX_EUNSUPPORTED, "blur_adjoint: kernel_size must be odd and <= 15");
  if (!(sigma > 0.f)) return abi::fail(PTYX_EINVAL, "blur_adjoint: sigma must be > 0");
  if (kernel_size / 2 >= Ny || kernel_size / 2 >= Nx)
    return abi::fail(PTYX_EINVAL, "blur_adjoint: reflect padding needs kernel_size/2 < Ny, Nx");
  if (n_planes == 0) return PTYX_OK;
  if (!in || !out || in == out) return abi::fail(PTYX_EINVAL, "blur_adjoint: in / out null or aliased");
  if (n_planes > 65535) return abi::fail(PTYX_EUNSUPPORTED, "blur_adjoint: at most 65535 planes per call");
  const cons::Taps t = torchvision_taps(kernel_size, sigma);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  launch_blur_h<true>(t.half, st, in, out, n_planes, Ny, Nx, t);
  return abi::launch_status("k_rblur_adj launch");
}

extern "C" int ptyx_simlar_std(void* stream, const float* x, int32_t O, int64_t n_planes, int32_t n_pix,
                               const float* occ, float* sums) {
  abi::clear_error();
  if (O < 1 || n_planes < 0 || n_pix < 0) return abi::fail(PTYX_EINVAL, "simlar_std: bad shape");
  if (O > cons::kSimlarMaxO) return abi::fail(PTYX_EUNSUPPORTED, "simlar_std: at most 32 object modes");
  if (n_planes > 2147483647LL) return abi::fail(PTYX_EUNSUPPORTED, "simlar_std: at most 2^31 - 1 planes");
  if (n_planes == 0) return PTYX_OK;
  if (!x || !occ || !sums) return abi::fail(PTYX_EINVAL, "simlar_std: null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 gr((unsigned)n_planes), bl(256);
  const bool v4 = n_pix % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  if (v4 && O == 2) hipLaunchKernelGGL(cons::k_simlar_std<2>, gr, bl, 0, st, x, O, (long long)n_planes, n_pix, occ, sums);
  else if (v4 && O == 3) hipLaunchKernelGGL(cons::k_simlar_std<3>, gr, bl, 0, st, x, O, (long long)n_planes, n_pix, occ, sums);
  else if (v4 && O == 4) hipLaunchKernelGGL(cons::k_simlar_std<4>, gr, bl, 0, st, x, O, (long long)n_planes, n_pix, occ, sums);
  else hipLaunchKernelGGL(cons::k_simlar_std<0>, gr, bl, 0, st, x, O, (long long)n_planes, n_pix, occ, sums);
  return abi::launch_status("k_simlar_std launch");
}

extern "C" int ptyx_simlar_std_grad(void* stream, const float* x, int32_t O, int64_t n_planes, int32_t n_pix,
                                    const float* occ, const float* gsum, float* gx) {
  abi::clear_error();
  if (O < 1 || n_planes < 0 || n_pix < 0) return abi::fail(PTYX_EINVAL, "simlar_std_grad: bad shape");
  if (O > cons::kSimlarMaxO) return abi::fail(PTYX_EUNSUPPORTED, "simlar_std_grad: at most 32 object modes");
  const long long total = (long long)n_planes * n_pix;
  if (total == 0) return PTYX_OK;
  if (!x || !occ || !gsum || !gx || x == gx) return abi::fail(PTYX_EINVAL, "simlar_std_grad: null or aliased pointer");
  const bool v4 = n_pix % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(gx) & 15) == 0 &&
                  O >= 2 && O <= 4;
  const long long blocks = (total / (v4 ? 4 : 1) + 255) / 256;
  if (blocks > 2147483647LL) return abi::fail(PTYX_EUNSUPPORTED, "simlar_std_grad: too many elements");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 gr((unsigned)blocks), bl(256);
  const long long np = n_planes;
  if (v4 && O == 2) hipLaunchKernelGGL(cons::k_simlar_std_grad<2>, gr, bl, 0, st, x, O, np, n_pix, occ, gsum, gx);
  else if (v4 && O == 3) hipLaunchKernelGGL(cons::k_simlar_std_grad<3>, gr, bl, 0, st, x, O, np, n_pix, occ, gsum, gx);
  else if (v4 && O == 4) hipLaunchKernelGGL(cons::k_simlar_std_grad<4>, gr, bl, 0, st, x, O, np, n_pix, occ, gsum, gx);
  else hipLaunchKernelGGL(cons::k_simlar_std_grad<0>, gr, bl, 0, st, x, O, np, n_pix, occ, gsum, gx);
  return abi::launch_status("k_simlar_std_grad launch");
}

namespace {
int patch_args(const char* what, int32_t O, int32_t Nz, int32_t Ny, int32_t Nx, const int32_t* crop_pos,
               const int32_t* idx, int32_t n_idx, int32_t N, const void* a, const void* b) {
  if (O <= 0 || Nz <= 0 || Ny <= 0 || Nx <= 0 || N <= 0 || n_idx < 0)
    return abi::fail(PTYX_EINVAL, std::string(what) + ": bad shape");
  if (N > Ny || N > Nx) return abi::fail(PTYX_EINVAL, std::string(what) + ": patch larger than the object");
  if (n_idx > 65535 || (long long)O * Nz > 65535)
    return abi::fail(PTYX_EUNSUPPORTED, std::string(what) + ": at most 65535 patches and O*Nz planes per call");
  if (n_idx && (!crop_pos || !idx || !a || !b)) return abi::fail(PTYX_EINVAL, std::string(what) + ": null pointer");
  return PTYX_OK;
}
}  // namespace

extern "C" int ptyx_patch_gather(void* stream, const float* obj, int32_t O, int32_t Nz, int32_t Ny, int32_t Nx,
                                 const int32_t* crop_pos, const int32_t* idx, int32_t n_idx, int32_t N,
                                 float* patches) {
  abi::clear_error();
  if (int rc = patch_args("patch_gather", O, Nz, Ny, Nx, crop_pos, idx, n_idx, N, obj, patches)) return rc;
  if (n_idx == 0) return PTYX_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(cons::k_patch_gather, dim3((N * N + 255) / 256, n_idx, O * Nz), dim3(256), 0, st, obj, Ny, Nx,
                     crop_pos, idx, n_idx, N, patches);
  return abi::launch_status("k_patch_gather launch");
}

extern "C" int ptyx_patch_scatter_add(void* stream, const float* gpatches, int32_t O, int32_t Nz, int32_t Ny,
                                      int32_t Nx, const int32_t* crop_pos, const int32_t* idx, int32_t n_idx,
                                      int32_t N, float* gobj) {
  abi::clear_error();
  if (int rc = patch_args("patch_scatter_add", O, Nz, Ny, Nx, crop_pos, idx, n_idx, N, gpatches, gobj)) return rc;
  if (n_idx == 0) return PTYX_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(cons::k_patch_scatter, dim3((N * N + 255) / 256, n_idx, O * Nz), dim3(256), 0, st, gpatches,
                     Ny, Nx, crop_pos, idx, n_idx, N, gobj);
  return abi::launch_status("k_patch_scatter launch");
}

extern "C" int ptyx_obj_constrain(void* stream, float* obja, float* objp, int32_t O, int32_t Nz, int32_t Ny,
                                  int32_t Nx, const ptyx_obj_constraints* cc, void* ws) {
  abi::clear_error();
  if (!cc) return abi::fail(PTYX_EINVAL, "obj_constrain: config is null");
  if (O <= 0 || Nz <= 0 || Ny <= 0 || Nx <= 0) return abi::fail(PTYX_EINVAL, "obj_constrain: bad shape");
  if (!obja || !objp) return abi::fail(PTYX_EINVAL, "obj_constrain: obja / objp null");
  const bool zb = (cc->zblur_a || cc->zblur_p) && cc->zblur_std != 0.f;
  if (zb && (cc->zblur_ks < 1 || cc->zblur_ks % 2 == 0 || cc->zblur_ks / 2 > kMaxHalf))
    return abi::fail(PTYX_EUNSUPPORTED, "obj_zblur: kernel_size must be odd and <= 15");
  const bool cr = cc->cr_a || cc->cr_p, submin = cc->pos_on && cc->pos_subtract_min;
  if ((cr || submin) && !ws) return abi::fail(PTYX_EINVAL, "obj_constrain: workspace needed for complex_ratio / subtract_min");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  double* wsd = reinterpret_cast<double*>(ws);
  cons::ObjCfg c{};
  c.O = O;
  c.Nz = Nz;
  c.Ny = Ny;
  c.Nx = Nx;
  c.zb_a = zb && cc->zblur_a;
  c.zb_p = zb && cc->zblur_p;
  if (zb) c.zt = scipy_taps(cc->zblur_ks, cc->zblur_std);
  c.cr_a = cc->cr_a;
  c.cr_p = cc->cr_p;
  c.alpha1 = cc->cr_alpha1;
  c.alpha2 = cc->cr_alpha2;
  c.mir = cc->mir_on;
  c.mir_relax = cc->mir_relax;
  c.mir_scale = cc->mir_scale;
  c.mir_power = cc->mir_power;
  c.thr = cc->thr_on;
  c.thr_relax = cc->thr_relax;
  c.thr_lo = cc->thr_lo;
  c.thr_hi = cc->thr_hi;
  c.pos = cc->pos_on;
  c.pos_submin = submin;
  c.pos_relax = cc->pos_relax;
  c.stats = wsd ? wsd + kWsStats : nullptr;
  const int h = zb ? cc->zblur_ks / 2 : 0;
  const bool pw = cr || c.mir || c.thr || c.pos;
  if (!cr && !submin) {              // the default chain: ONE pass over the object
    if (zb || pw) launch_column_h(h, st, obja, objp, c, pw ? 1 : 0);
    return abi::launch_status("k_obj_column launch");
  }
  // options needing global scalars: z-blur pass, reductions, then the point-wise pass
  if (zb) {
    cons::ObjCfg z = c;
    launch_column_h(h, st, obja, objp, z, 0);
  }
  const long long n = (long long)O * Nz * Ny * Nx;
  if (cr) {
    hipLaunchKernelGGL(cons::k_obj_reduce<0>, dim3(kRedBlocks), dim3(256), 0, st, obja, objp, n, c, wsd + kWsPart);
    hipLaunchKernelGGL(cons::k_reduce_final<0>, dim3(1), dim3(64), 0, st, wsd + kWsPart, kRedBlocks, wsd + kWsStats);
  }
  if (submin) {
    hipLaunchKernelGGL(cons::k_obj_reduce<1>, dim3(kRedBlocks), dim3(256), 0, st, obja, objp, n, c, wsd + kWsPart);
    hipLaunchKernelGGL(cons::k_reduce_final<1>, dim3(1), dim3(64), 0, st, wsd + kWsPart, kRedBlocks, wsd + kWsStats);
  }
  cons::ObjCfg q = c;
  q.zb_a = q.zb_p = 0;
  launch_column_h(0, st, obja, objp, q, 1);
  return abi::launch_status("obj_constrain launch");
}

extern "C" int ptyx_probe_fix_int(void* stream, float* probe, int32_t P, int32_t N, const float* probe_int_sum,
                                  void* ws) {
  abi::clear_error();
  if (P <= 0 || N <= 0) return abi::fail(PTYX_EINVAL, "fix_probe_int: bad shape");
  if (!probe || !probe_int_sum || !ws) return abi::fail(PTYX_EINVAL, "fix_probe_int: null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  double* wsd = reinterpret_cast<double*>(ws);
  const long long n = (long long)P * N * N;
  float2* x = reinterpret_cast<float2*>(probe);
  hipLaunchKernelGGL(cons::k_sumsq, dim3(kRedBlocks), dim3(256), 0, st, x, n, wsd + kWsPart);
  hipLaunchKernelGGL(cons::k_fix_int_final, dim3(1), dim3(64), 0, st, wsd + kWsPart, kRedBlocks, probe_int_sum,
                     wsd + kWsStats);
  hipLaunchKernelGGL(cons::k_cscale, dim3(256), dim3(256), 0, st, x, n, wsd + kWsStats);
  return abi::launch_status("fix_probe_int launch");
}

extern "C" int ptyx_probe_ortho(void* stream, float* probe, int32_t P, int32_t N, void* ws) {
  abi::clear_error();
  if (P <= 0 || N <= 0) return abi::fail(PTYX_EINVAL, "ortho_pmode: bad shape");
  if (P > kMaxModes) return abi::fail(PTYX_EUNSUPPORTED, "ortho_pmode: at most 64 probe modes");
  if (!probe || !ws) return abi::fail(PTYX_EINVAL, "ortho_pmode: null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  double* wsd = reinterpret_cast<double*>(ws);
  float2* M = reinterpret_cast<float2*>(probe);
  const long long n2 = (long long)N * N;
  const int npair = P * (P + 1) / 2;
  float2* U = reinterpret_cast<float2*>(wsd + kWsU);
  hipLaunchKernelGGL(cons::k_gram, dim3(kGramChunks, npair), dim3(256), 0, st, M, P, n2, kGramChunks, wsd + kWsGram);
  hipLaunchKernelGGL(cons::k_ortho_eig, dim3(1), dim3(64), 0, st, wsd + kWsGram, P, kGramChunks, U, wsd + kWsEvals);
  switch (P) {
    case 1: launch_ortho_apply<1>(st, M, n2, U, P); break;
    case 2: launch_ortho_apply<2>(st, M, n2, U, P); break;
    case 3: launch_ortho_apply<3>(st, M, n2, U, P); break;
    case 4: launch_ortho_apply<4>(st, M, n2, U, P); break;
    case 5: launch_ortho_apply<5>(st, M, n2, U, P); break;
    case 6: launch_ortho_apply<6>(st, M, n2, U, P); break;
    case 7: launch_ortho_apply<7>(st, M, n2, U, P); break;
    case 8: launch_ortho_apply<8>(st, M, n2, U, P); break;
    case 9: launch_ortho_apply<9>(st, M, n2, U, P); break;
    case 10: launch_ortho_apply<10>(st, M, n2, U, P); break;
    case 11: launch_ortho_apply<11>(st, M, n2, U, P); break;
    case 12: launch_ortho_apply<12>(st, M, n2, U, P); break;
    case 13: launch_ortho_apply<13>(st, M, n2, U, P); break;
    case 14: launch_ortho_apply<14>(st, M, n2, U, P); break;
    case 15: launch_ortho_apply<15>(st, M, n2, U, P); break;
    case 16: launch_ortho_apply<16>(st, M, n2, U, P); break;
    default:
      if (P <= 32) launch_ortho_apply<32>(st, M, n2, U, P);
      else launch_ortho_apply<64>(st, M, n2, U, P);
      break;
  }
  return abi::launch_status("ortho_pmode launch");
}

// ---------------------------------------------------------------------------------------------
// loss_pacbed (src/ptyrad/losses.py:77-89) per mini-batch m of B_m patterns:
//   Ī = mean_b I_b,  M̄ = mean_b M_b (per pixel),  d = Ī^q − M̄^q,
//   L_m = w · sqrt(Σ_k d_k² / N²) / mean_{b,k} M^q,
//   dL_m/dI_{b,k} = w / (mu · N² · rmse · B_m) · d_k · q · Ī_k^(q−1).
// k_pac_pixel: one thread per (pixel, batch): fp64 sums over the batch's patterns in order;
// k_pac_batch: one workgroup per batch, fixed-order fp64 reduction → L_m and its coefficient;
// k_pac_dldi: dLdI = grad_scale · coef_m · e_k.  Deterministic; ws = n_batches·(N²·(8+8+4)+16) B.
namespace {
__device__ __forceinline__ double pac_pow(double x, float q) {
  if (q == 1.0f) return x;
  if (q == 0.5f) return sqrt(x);
  return x > 0.0 ? pow(x, (double)q) : 0.0;
}

__global__ __launch_bounds__(256) void k_pac_pixel(const float* __restrict__ dp, const void* __restrict__ meas,
                                                   int meas_f16, const int* __restrict__ idx,
                                                   const int* __restrict__ boff, int n2, float q, double* d2,
                                                   double* mq, float* e) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= n2) return;
  const int m = blockIdx.y;
  const int b0 = boff[m], b1 = boff[m + 1];
  double sI = 0.0, sM = 0.0, sMq = 0.0;
  for (int b = b0; b < b1; ++b) {
    const size_t moff = (size_t)idx[b] * n2 + k;
    const double M = meas_f16 ? (double)__half2float(reinterpret_cast<const __half*>(meas)[moff])
                              : (double)reinterpret_cast<const float*>(meas)[moff];
    sI += (double)dp[(size_t)b * n2 + k];
    sM += M;
    sMq += pac_pow(M, q);
  }
  const double inv = b1 > b0 ? 1.0 / (double)(b1 - b0) : 0.0;
  const double Ib = sI * inv, Mb = sM * inv;
  const double d = pac_pow(Ib, q) - pac_pow(Mb, q);
  const size_t o = (size_t)m * n2 + k;
  d2[o] = d * d;
  mq[o] = sMq;
  e[o] = (float)(d * (double)q * (Ib > 0.0 ? pac_pow(Ib, q) / Ib : 0.0));
}

__global__ __launch_bounds__(256) void k_pac_batch(const double* __restrict__ d2, const double* __restrict__ mq,
                                                   const int* __restrict__ boff, int n2, float w, double* coef,
                                                   float* loss_terms) {
  __shared__ double s0[256], s1[256];
  const int m = blockIdx.x;
  double a = 0.0, c = 0.0;
  for (int k = threadIdx.x; k < n2; k += 256) {
    a += d2[(size_t)m * n2 + k];
    c += mq[(size_t)m * n2 + k];
  }
  s0[threadIdx.x] = a;
  s1[threadIdx.x] = c;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (threadIdx.x < h) {
      s0[threadIdx.x] += s0[threadIdx.x + h];
      s1[threadIdx.x] += s1[threadIdx.x + h];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const int B = boff[m + 1] - boff[m];
    const double rmse = sqrt(s0[0] / (double)n2);
    const double mu = B > 0 ? s1[0] / ((double)B * n2) : 0.0;
    loss_terms[(size_t)m * 5 + 2] = mu > 0.0 ? (float)(w * rmse / mu) : 0.f;
    coef[m] = (rmse > 0.0 && mu > 0.0 && B > 0) ? w / (mu * (double)n2 * rmse * (double)B) : 0.0;
  }
}

__global__ __launch_bounds__(256) void k_pac_dldi(const float* __restrict__ e, const double* __restrict__ coef,
                                                  const int* __restrict__ boff, int n_batches, int n2, float scale,
                                                  float* __restrict__ dLdI) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= n2) return;
  const int n_idx = boff[n_batches];
  for (int b = blockIdx.y; b < n_idx; b += gridDim.y) {
    int lo = 0, hi = n_batches;   // batch containing b: boff[lo] <= b < boff[lo+1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (boff[mid] <= b) lo = mid;
      else hi = mid;
    }
    dLdI[(size_t)b * n2 + k] = (float)((double)scale * coef[lo] * (double)e[(size_t)lo * n2 + k]);
  }
}
}  // namespace

extern "C" size_t ptyx_pacbed_ws_bytes(int32_t N, int32_t n_batches) {
  const size_t n2 = (size_t)N * N;
  return (size_t)n_batches * (n2 * (8 + 8 + 4) + 8) + 64;
}

extern "C" int ptyx_loss_pacbed(void* stream, const float* dp, const void* meas, int32_t meas_f16, const int32_t* idx,
                                const int32_t* batch_offsets, int32_t n_batches, int32_t n_idx, int32_t N,
                                float weight, float dp_pow, float grad_scale, float* loss_terms, float* dLdI,
                                void* ws) {
  abi::clear_error();
  if (N <= 0 || n_batches < 0 || n_idx < 0) return abi::fail(PTYX_EINVAL, "loss_pacbed: bad shape");
  if (n_batches > 65535) return abi::fail(PTYX_EUNSUPPORTED, "loss_pacbed: at most 65535 batches per call");
  if (n_batches == 0) return PTYX_OK;
  if (!dp || !meas || !idx || !batch_offsets || !loss_terms || !ws)
    return abi::fail(PTYX_EINVAL, "loss_pacbed: null pointer");
  const int n2 = N * N;
  double* d2 = reinterpret_cast<double*>(ws);
  double* mq = d2 + (size_t)n_batches * n2;
  double* coef = mq + (size_t)n_batches * n2;
  float* e = reinterpret_cast<float*>(coef + n_batches);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_pac_pixel, dim3((n2 + 255) / 256, n_batches), dim3(256), 0, st, dp, meas, meas_f16, idx,
                     batch_offsets, n2, dp_pow, d2, mq, e);
  hipLaunchKernelGGL(k_pac_batch, dim3(n_batches), dim3(256), 0, st, d2, mq, batch_offsets, n2, weight, coef,
                     loss_terms);
  if (dLdI && n_idx > 0)
    hipLaunchKernelGGL(k_pac_dldi, dim3((n2 + 255) / 256, std::min(n_idx, 65535)), dim3(256), 0, st, e, coef,
                       batch_offsets, n_batches, n2, grad_scale, dLdI);
  return abi::launch_status("loss_pacbed launch");
}
