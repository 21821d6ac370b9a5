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
// Arithmetic: ptyx_adam.hpp (shared with the optimizer step fused into an engine call's epilogue).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

#include "ptyx.h"
#include "ptyx_abi.hpp"
#include "ptyx_adam.hpp"

namespace ptyx {
namespace opt {

__global__ __launch_bounds__(kThreads) void k_adam(AdamArgs a) {
  // the tensors' step scalars, once per workgroup (lane t of wave 0 for tensor t)
  __shared__ float s_nstep[kMaxT], s_bc2s[kMaxT];
  if (threadIdx.x < (unsigned)a.nt) {
    const int t = threadIdx.x;
    adam_step_scalars(a.h, a.lr[t], *a.step[t], &s_nstep[t], &s_bc2s[t]);
  }
  __syncthreads();
  if (a.scnt && blockIdx.x == 0) {   // as k_step_store: every thread reads *scnt before it advances
    const int64_t c = *a.scnt;
    const int64_t r0 = a.srstart[c];
    for (int i = threadIdx.x; i < a.snb * 5; i += blockDim.x) a.sterms_all[r0 * 5 + i] = a.sterms[i];
    __syncthreads();
    if (threadIdx.x == 0) *a.scnt = c + 1;
  }
  adam_chunks(a, s_nstep, s_bc2s, blockIdx.x, gridDim.x);
}

}  // namespace opt
}  // namespace ptyx

using ptyx::abi::fail;
using ptyx::abi::launch_status;
namespace opt = ptyx::opt;

namespace {
int adam_step(void* stream, int32_t n, float* const* params, const float* const* grads, float* const* exp_avgs,
              float* const* exp_avg_sqs, const float* const* steps, const int64_t* numels, const double* lrs,
              double beta1, double beta2, double eps, double weight_decay, int32_t flags, const opt::StepStore* ss) {
  if (n < 0 || (n && (!params || !grads || !exp_avgs || !exp_avg_sqs || !steps || !numels || !lrs)))
    return fail(PTYX_EINVAL, "ptyx_adam_step: null array or negative count");
  std::vector<opt::AdamTensor> ts;
  ts.reserve((size_t)n);
  for (int i = 0; i < n; ++i) {
    if (numels[i] < 0 || (numels[i] && (!params[i] || !grads[i] || !exp_avgs[i] || !exp_avg_sqs[i] || !steps[i])))
      return fail(PTYX_EINVAL, "ptyx_adam_step: null tensor pointer or negative size");
    ts.push_back({params[i], grads[i], exp_avgs[i], exp_avg_sqs[i], steps[i], lrs[i], numels[i]});
  }
  return opt::adam_launch((hipStream_t)stream, ts, opt::hyper(beta1, beta2, eps, weight_decay, flags), ss);
}
}  // namespace

namespace ptyx {
namespace opt {
int adam_launch(hipStream_t st, const std::vector<AdamTensor>& ts, const AdamHyper& h, const StepStore* ss) {
  for (AdamArgs& a : adam_pack(ts, h)) {
    if (ss) {   // the bookkeeping rides in the first launch
      adam_set_store(a, *ss);
      ss = nullptr;
    }
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(4096, a.off[a.nt] / kChunk));
    hipLaunchKernelGGL(k_adam, dim3(blocks), dim3(kThreads), 0, st, a);
    if (int rc = launch_status("k_adam launch")) return rc;
  }
  if (ss) {   // nothing to update: the bookkeeping alone (one workgroup, no tensors)
    AdamArgs a{};
    adam_set_store(a, *ss);
    hipLaunchKernelGGL(k_adam, dim3(1), dim3(kThreads), 0, st, a);
    if (int rc = launch_status("k_adam launch")) return rc;
  }
  return PTYX_OK;
}
}  // namespace opt
}  // namespace ptyx

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
  const opt::StepStore ss{terms, nb, rstart, cnt, terms_all};
  return adam_step(stream, n, params, grads, exp_avgs, exp_avg_sqs, steps, numels, lrs, beta1, beta2, eps,
                   weight_decay, flags, &ss);
}
