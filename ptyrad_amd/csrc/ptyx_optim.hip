// ptyx_optim.hip — the Adam / AdamW update of every trainable tensor in ONE grid-filling launch.
//
// recon_step (src/ptyrad/reconstruction.py:658-781) calls optimizer.step() once per optimizer
// step; at the reference's default grad_accumulation = 1 that is once per 32-pattern
// mini-batch.  torch's fused Adam launches one multi_tensor_apply kernel per parameter group with
// one workgroup per 65,536-element chunk: 17 workgroups for a 1033² object, so on 256 CUs each
// group's update is latency-bound (≈ 130 µs per object tensor at the c2 geometry, 64 % of a
// graph-replayed step; tools/trace_gaps.py).  Here one launch covers all groups, grid-stride over
// the concatenated elements with enough workgroups to fill the chip, so the update streams at the
// HBM rate (28 B per element: p, g, m, v in; p, m, v out).
//
// Arithmetic: torch.optim.Adam's single-tensor formula (torch/optim/adam.py, the path PtyRAD's
// CPU runs take), fp32 element math in the same operation order with no FMA contraction, the
// bias corrections in fp64 from the device step count (already incremented by the caller):
//   g += wd·p (Adam) | p *= 1 − lr·wd (AdamW);   m = lerp(m, g, 1 − β1);   v = v·β2 + (1 − β2)·g·g
//   p += (−lr / (1 − β1^t))·m / (√v / √(1 − β2^t) + ε)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

#include "ptyx.h"
#include "ptyx_abi.hpp"

namespace ptyx {
namespace opt {

constexpr int kMaxT = 16;   // tensors per launch (more are split over launches)

constexpr int kU = 4;                  // units per thread of a chunk
constexpr int kThreads = 256;
constexpr int64_t kChunk = (int64_t)kU * kThreads;   // units per workgroup chunk

struct AdamArgs {
  float* p[kMaxT];
  const float* g[kMaxT];
  float* m[kMaxT];
  float* v[kMaxT];
  const float* step[kMaxT];
  double lr[kMaxT];
  // prefix sums of the tensors' unit ranges (4 elements a unit if vec, else 1), each range padded
  // to whole chunks, so a chunk belongs to ONE tensor: the tensor index is uniform per workgroup
  // and the per-tensor pointers and flags are scalar loads
  int64_t off[kMaxT + 1];
  int64_t units[kMaxT];
  int vec[kMaxT];           // p, g, m, v 16-B aligned and numel % 4 == 0: float4 units
  int nt;
  float beta1, beta2, eps, wd;
  double beta1d, beta2d;
  int adamw, maximize;
  // optional graph-step bookkeeping in workgroup 0 (ptyx_adam_step_store): the step's loss terms
  // into the iteration's table, then the device step counter advanced
  const float* sterms;
  const int64_t* srstart;
  int64_t* scnt;
  float* sterms_all;
  int snb;
};

// β^t for the integer step count t by square-and-multiply in fp64 (a few fp64 ulps from pow(),
// far below the fp32 rounding of the factors it feeds; pow() for a non-integer t)
__device__ __forceinline__ double pow_step(double b, double t) {
  if (!(t >= 0.0 && t < 9007199254740992.0 && t == floor(t))) return pow(b, t);
  unsigned long long n = (unsigned long long)t;
  double r = 1.0, x = b;
  while (n) {
    if (n & 1) r *= x;
    x *= x;
    n >>= 1;
  }
  return r;
}

__global__ __launch_bounds__(kThreads) void k_adam(AdamArgs a) {
  // the tensors' step scalars, once per workgroup (lane t of wave 0 for tensor t)
  __shared__ float s_nstep[kMaxT], s_bc2s[kMaxT];
  if (threadIdx.x < (unsigned)a.nt) {
    const int t = threadIdx.x;
    const double step = (double)*a.step[t];
    const double bc1 = 1.0 - pow_step(a.beta1d, step), bc2 = 1.0 - pow_step(a.beta2d, step);
    s_nstep[t] = (float)(-(a.lr[t] / bc1));
    s_bc2s[t] = (float)sqrt(bc2);
  }
  __syncthreads();
  if (a.scnt && blockIdx.x == 0) {   // as k_step_store: every thread reads *scnt before it advances
    const int64_t c = *a.scnt;
    const int64_t r0 = a.srstart[c];
    for (int i = threadIdx.x; i < a.snb * 5; i += blockDim.x) a.sterms_all[r0 * 5 + i] = a.sterms[i];
    __syncthreads();
    if (threadIdx.x == 0) *a.scnt = c + 1;
  }
  const int64_t total = a.off[a.nt];
  const float w1 = (float)(1.0 - a.beta1d), c2 = (float)(1.0 - a.beta2d);
  // a workgroup takes chunks of 4·256 consecutive units of one tensor, a thread four of them 256
  // apart (coalesced; 16-B units where the tensor allows); chunks grid-stride
  int t = 0;
  for (int64_t c0 = (int64_t)blockIdx.x * kChunk; c0 < total; c0 += (int64_t)gridDim.x * kChunk) {
    while (c0 >= a.off[t + 1]) ++t;   // chunk starts only grow
    t = __builtin_amdgcn_readfirstlane(t);
    const int64_t j0 = c0 - a.off[t], nu = a.units[t];
    const bool vec = a.vec[t] != 0;
    float* __restrict__ P = a.p[t];
    const float* __restrict__ G = a.g[t];
    float* __restrict__ M = a.m[t];
    float* __restrict__ V = a.v[t];
    const float nstep = s_nstep[t], bc2s = s_bc2s[t];
    const float decay = (float)(1.0 - a.lr[t] * (double)a.wd);
    float4 g[kU], p[kU], m[kU], v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t j = j0 + u * kThreads + threadIdx.x;
      if (j < nu) {
        if (vec) {
          g[u] = reinterpret_cast<const float4*>(G)[j];
          p[u] = reinterpret_cast<const float4*>(P)[j];
          m[u] = reinterpret_cast<const float4*>(M)[j];
          v[u] = reinterpret_cast<const float4*>(V)[j];
        } else {
          g[u].x = G[j];
          p[u].x = P[j];
          m[u].x = M[j];
          v[u].x = V[j];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t j = j0 + u * kThreads + threadIdx.x;
      if (j >= nu) continue;
      float* gp = &g[u].x;
      float* pp = &p[u].x;
      float* mp = &m[u].x;
      float* vp = &v[u].x;
      const int ne = vec ? 4 : 1;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (e >= ne) break;
        float gu = gp[e], pu = pp[e], mu = mp[e], vu = vp[e];
        if (a.maximize) gu = -gu;
        if (a.wd != 0.f) {
          if (a.adamw) pu = __fmul_rn(pu, decay);
          else gu = __fadd_rn(gu, __fmul_rn(pu, a.wd));
        }
        mu = __fadd_rn(mu, __fmul_rn(w1, __fsub_rn(gu, mu)));                        // lerp, weight < 0.5
        vu = __fadd_rn(__fmul_rn(vu, a.beta2), __fmul_rn(__fmul_rn(c2, gu), gu));     // mul_(β2).addcmul_
        const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(vu), bc2s), a.eps);
        pu = __fadd_rn(pu, __fdiv_rn(__fmul_rn(nstep, mu), denom));                  // addcdiv_
        pp[e] = pu;
        mp[e] = mu;
        vp[e] = vu;
      }
      if (vec) {
        reinterpret_cast<float4*>(P)[j] = p[u];
        reinterpret_cast<float4*>(M)[j] = m[u];
        reinterpret_cast<float4*>(V)[j] = v[u];
      } else {
        P[j] = p[u].x;
        M[j] = m[u].x;
        V[j] = v[u].x;
      }
    }
  }
}

}  // namespace opt
}  // namespace ptyx

using ptyx::abi::fail;
using ptyx::abi::launch_status;
namespace opt = ptyx::opt;

namespace {
struct StepStore {
  const float* terms;
  int32_t nb;
  const int64_t* rstart;
  int64_t* cnt;
  float* terms_all;
};

int adam_step(void* stream, int32_t n, float* const* params, const float* const* grads, float* const* exp_avgs,
              float* const* exp_avg_sqs, const float* const* steps, const int64_t* numels, const double* lrs,
              double beta1, double beta2, double eps, double weight_decay, int32_t flags, const StepStore* ss) {
  if (n < 0 || (n && (!params || !grads || !exp_avgs || !exp_avg_sqs || !steps || !numels || !lrs)))
    return fail(PTYX_EINVAL, "ptyx_adam_step: null array or negative count");
  // Each tensor is one or two ranges: its first 4·⌊numel/4⌋ elements in float4 units when p, g,
  // m, v are 16-B aligned, the (≤ 3) others as scalar units — a 591² × 6 object plane is not a
  // multiple of 4 and would otherwise run at 4-byte accesses.  Ranges are grouped kMaxT a launch.
  struct Range {
    float* p;
    const float* g;
    float* m;
    float* v;
    const float* step;
    double lr;
    int64_t numel;
    int vec;
  };
  std::vector<Range> rs;
  rs.reserve(2 * (size_t)n);
  const auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  for (int i = 0; i < n; ++i) {
    if (numels[i] < 0 || (numels[i] && (!params[i] || !grads[i] || !exp_avgs[i] || !exp_avg_sqs[i] || !steps[i])))
      return fail(PTYX_EINVAL, "ptyx_adam_step: null tensor pointer or negative size");
    if (!numels[i]) continue;
    const bool aligned = al16(params[i]) && al16(grads[i]) && al16(exp_avgs[i]) && al16(exp_avg_sqs[i]);
    const int64_t body = aligned ? numels[i] / 4 * 4 : 0;
    if (body) rs.push_back({params[i], grads[i], exp_avgs[i], exp_avg_sqs[i], steps[i], lrs[i], body, 1});
    if (numels[i] > body)
      rs.push_back({params[i] + body, grads[i] + body, exp_avgs[i] + body, exp_avg_sqs[i] + body, steps[i], lrs[i],
                    numels[i] - body, 0});
  }
  for (size_t i0 = 0; i0 < rs.size(); i0 += opt::kMaxT) {
    opt::AdamArgs a{};
    a.nt = (int)std::min<size_t>(opt::kMaxT, rs.size() - i0);
    a.off[0] = 0;
    for (int k = 0; k < a.nt; ++k) {
      const Range& r = rs[i0 + k];
      a.p[k] = r.p;
      a.g[k] = r.g;
      a.m[k] = r.m;
      a.v[k] = r.v;
      a.step[k] = r.step;
      a.lr[k] = r.lr;
      a.vec[k] = r.vec;
      a.units[k] = r.vec ? r.numel / 4 : r.numel;
      a.off[k + 1] = a.off[k] + (a.units[k] + opt::kChunk - 1) / opt::kChunk * opt::kChunk;
    }
    for (int k = a.nt; k < opt::kMaxT; ++k) a.off[k + 1] = a.off[a.nt];
    a.beta1 = (float)beta1;
    a.beta2 = (float)beta2;
    a.beta1d = beta1;
    a.beta2d = beta2;
    a.eps = (float)eps;
    a.wd = (float)weight_decay;
    a.adamw = flags & 1;
    a.maximize = (flags >> 1) & 1;
    const int64_t total = a.off[a.nt];
    if (!total) continue;
    if (ss) {   // the bookkeeping rides in the first launch
      a.sterms = ss->terms;
      a.snb = ss->nb;
      a.srstart = ss->rstart;
      a.scnt = ss->cnt;
      a.sterms_all = ss->terms_all;
      ss = nullptr;
    }
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(4096, total / opt::kChunk));
    hipLaunchKernelGGL(opt::k_adam, dim3(blocks), dim3(opt::kThreads), 0, (hipStream_t)stream, a);
    if (int rc = launch_status("k_adam launch")) return rc;
  }
  if (ss) {   // nothing to update: the bookkeeping alone (one workgroup, no tensors)
    opt::AdamArgs a{};
    a.sterms = ss->terms;
    a.snb = ss->nb;
    a.srstart = ss->rstart;
    a.scnt = ss->cnt;
    a.sterms_all = ss->terms_all;
    hipLaunchKernelGGL(opt::k_adam, dim3(1), dim3(opt::kThreads), 0, (hipStream_t)stream, a);
    if (int rc = launch_status("k_adam launch")) return rc;
  }
  return PTYX_OK;
}
}  // namespace

extern "C" int ptyx_adam_step(void* stream, int32_t n, float* const* params, const float* const* grads,
                              float* const* exp_avgs, float* const* exp_avg_sqs, const float* const* steps,
                              const int64_t* numels, const double* lrs, double beta1, double beta2, double eps,
                              double weight_decay, int32_t flags) {
  ptyx::abi::clear_error();
  return adam_step(stream, n, params, grads, exp_avgs, exp_avg_sqs, steps, numels, lrs, beta1, beta2, eps,
                   weight_decay, flags, nullptr);
}

extern "C" int ptyx_adam_step_store(void* stream, int32_t n, float* const* params, const float* const* grads,
                                    float* const* exp_avgs, float* const* exp_avg_sqs, const float* const* steps,
                                    const int64_t* numels, const double* lrs, double beta1, double beta2, double eps,
                                    double weight_decay, int32_t flags, const float* terms, int32_t nb,
                                    const int64_t* rstart, int64_t* cnt, float* terms_all) {
  ptyx::abi::clear_error();
  if (!terms || !rstart || !cnt || !terms_all || nb < 0)
    return fail(PTYX_EINVAL, "ptyx_adam_step_store: null pointer or negative size");
  const StepStore ss{terms, nb, rstart, cnt, terms_all};
  return adam_step(stream, n, params, grads, exp_avgs, exp_avg_sqs, steps, numels, lrs, beta1, beta2, eps,
                   weight_decay, flags, &ss);
}
