// ptyx_adam.hpp — the Adam / AdamW element update shared by ptyx_adam_step's k_adam
// (ptyx_optim.hip) and the optimizer step fused into a call's epilogue (PTYX_PREP_FUSED_ADAM,
// k_gather_adam in ptyx_kernels.hip), so the two paths are the same arithmetic bit for bit.
//
// torch.optim.Adam's single-tensor formula (torch/optim/adam.py, the path PtyRAD's CPU runs take),
// fp32 element math in the same operation order with no FMA contraction, the bias corrections in
// fp64 from the device step count (already incremented by the caller):
//   g += wd·p (Adam) | p *= 1 − lr·wd (AdamW);   m = lerp(m, g, 1 − β1);   v = v·β2 + (1 − β2)·g·g
//   p += (−lr / (1 − β1^t))·m / (√v / √(1 − β2^t) + ε)
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <vector>

namespace ptyx {
namespace opt {

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

// Per-launch constants (uniform over the tensors of one Adam batch).
struct AdamHyper {
  float beta1, beta2, eps, wd;
  double beta1d, beta2d;
  int adamw, maximize;
};

// flags: 1 = decoupled weight decay (AdamW), 2 = maximize (ptyx_adam_step)
inline AdamHyper hyper(double beta1, double beta2, double eps, double weight_decay, int flags) {
  AdamHyper h;
  h.beta1 = (float)beta1;
  h.beta2 = (float)beta2;
  h.beta1d = beta1;
  h.beta2d = beta2;
  h.eps = (float)eps;
  h.wd = (float)weight_decay;
  h.adamw = flags & 1;
  h.maximize = (flags >> 1) & 1;
  return h;
}

// Per-tensor step scalars: −lr / (1 − β1^t) and √(1 − β2^t), from the device step count.
__device__ __forceinline__ void adam_step_scalars(const AdamHyper& h, double lr, float step, float* nstep,
                                                  float* bc2s) {
  const double s = (double)step;
  const double bc1 = 1.0 - pow_step(h.beta1d, s), bc2 = 1.0 - pow_step(h.beta2d, s);
  *nstep = (float)(-(lr / bc1));
  *bc2s = (float)sqrt(bc2);
}

// One element: p, m, v updated in place from the gradient g.  decay = 1 − lr·wd (AdamW).
__device__ __forceinline__ void adam_elem(const AdamHyper& h, float nstep, float bc2s, float decay, float g,
                                          float& p, float& m, float& v) {
  const float w1 = (float)(1.0 - h.beta1d), c2 = (float)(1.0 - h.beta2d);
  float gu = g, pu = p, mu = m, vu = v;
  if (h.maximize) gu = -gu;
  if (h.wd != 0.f) {
    if (h.adamw) pu = __fmul_rn(pu, decay);
    else gu = __fadd_rn(gu, __fmul_rn(pu, h.wd));
  }
  mu = __fadd_rn(mu, __fmul_rn(w1, __fsub_rn(gu, mu)));                        // lerp, weight < 0.5
  vu = __fadd_rn(__fmul_rn(vu, h.beta2), __fmul_rn(__fmul_rn(c2, gu), gu));     // mul_(β2).addcmul_
  const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(vu), bc2s), h.eps);
  pu = __fadd_rn(pu, __fdiv_rn(__fmul_rn(nstep, mu), denom));                  // addcdiv_
  p = pu;
  m = mu;
  v = vu;
}

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
  AdamHyper h;
  // optional graph-step bookkeeping in workgroup 0 (ptyx_adam_step_store): the step's loss terms
  // into the iteration's table, then the device step counter advanced
  const float* sterms;
  const int64_t* srstart;
  int64_t* scnt;
  float* sterms_all;
  int snb;
};

// The chunk loop of k_adam: workgroup blk of nblk takes chunks of kU·256 consecutive units of one
// tensor, a thread kU of them 256 apart (coalesced; 16-B units where the tensor allows); chunks
// grid-stride.  s_nstep / s_bc2s: the tensors' step scalars (adam_step_scalars).
__device__ __forceinline__ void adam_chunks(const AdamArgs& a, const float* s_nstep, const float* s_bc2s, int64_t blk,
                                            int64_t nblk) {
  const int64_t total = a.off[a.nt];
  int t = 0;
  for (int64_t c0 = (int64_t)blk * kChunk; c0 < total; c0 += (int64_t)nblk * kChunk) {
    while (c0 >= a.off[t + 1]) ++t;   // chunk starts only grow
    t = __builtin_amdgcn_readfirstlane(t);
    const int64_t j0 = c0 - a.off[t], nu = a.units[t];
    const bool vec = a.vec[t] != 0;
    float* __restrict__ P = a.p[t];
    const float* __restrict__ G = a.g[t];
    float* __restrict__ M = a.m[t];
    float* __restrict__ V = a.v[t];
    const float nstep = s_nstep[t], bc2s = s_bc2s[t];
    const float decay = (float)(1.0 - a.lr[t] * (double)a.h.wd);
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
        adam_elem(a.h, nstep, bc2s, decay, gp[e], pp[e], mp[e], vp[e]);
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

// ---------------------------------------------------------------- host side
// One tensor of an Adam batch (device pointers; step: the device f32 step count).
struct AdamTensor {
  float* p;
  const float* g;
  float* m;
  float* v;
  const float* step;
  double lr;
  int64_t numel;
};
// The graph step's bookkeeping riding in an Adam launch's workgroup 0 (ptyx_adam_step_store).
struct StepStore {
  const float* terms;
  int32_t nb;
  const int64_t* rstart;
  int64_t* cnt;
  float* terms_all;
};

// Each tensor is one or two ranges: its first 4·⌊numel/4⌋ elements in float4 units when p, g,
// m, v are 16-B aligned, the (≤ 3) others as scalar units — a 591² × 6 object plane is not a
// multiple of 4 and would otherwise run at 4-byte accesses.  Ranges are grouped kMaxT a launch;
// launches with no elements are dropped.
inline std::vector<AdamArgs> adam_pack(const std::vector<AdamTensor>& ts, const AdamHyper& h) {
  struct Range {
    AdamTensor t;
    int vec;
  };
  std::vector<Range> rs;
  rs.reserve(2 * ts.size());
  const auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  for (const AdamTensor& x : ts) {
    if (!x.numel) continue;
    const bool aligned = al16(x.p) && al16(x.g) && al16(x.m) && al16(x.v);
    const int64_t body = aligned ? x.numel / 4 * 4 : 0;
    if (body) rs.push_back({{x.p, x.g, x.m, x.v, x.step, x.lr, body}, 1});
    if (x.numel > body)
      rs.push_back({{x.p + body, x.g + body, x.m + body, x.v + body, x.step, x.lr, x.numel - body}, 0});
  }
  std::vector<AdamArgs> out;
  for (size_t i0 = 0; i0 < rs.size(); i0 += kMaxT) {
    AdamArgs a{};
    a.nt = (int)std::min<size_t>(kMaxT, rs.size() - i0);
    a.off[0] = 0;
    for (int k = 0; k < a.nt; ++k) {
      const Range& r = rs[i0 + k];
      a.p[k] = r.t.p;
      a.g[k] = r.t.g;
      a.m[k] = r.t.m;
      a.v[k] = r.t.v;
      a.step[k] = r.t.step;
      a.lr[k] = r.t.lr;
      a.vec[k] = r.vec;
      a.units[k] = r.vec ? r.t.numel / 4 : r.t.numel;
      a.off[k + 1] = a.off[k] + (a.units[k] + kChunk - 1) / kChunk * kChunk;
    }
    for (int k = a.nt; k < kMaxT; ++k) a.off[k + 1] = a.off[a.nt];
    a.h = h;
    if (a.off[a.nt]) out.push_back(a);
  }
  return out;
}
inline void adam_set_store(AdamArgs& a, const StepStore& ss) {
  a.sterms = ss.terms;
  a.snb = ss.nb;
  a.srstart = ss.rstart;
  a.scnt = ss.cnt;
  a.sterms_all = ss.terms_all;
}
// k_adam over ts (ptyx_optim.hip): the ptyx_adam_step[_store] launches
int adam_launch(hipStream_t st, const std::vector<AdamTensor>& ts, const AdamHyper& h, const StepStore* ss);

}  // namespace opt
}  // namespace ptyx
