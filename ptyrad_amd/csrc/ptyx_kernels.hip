// ptyx_kernels.hip — plans, engine selection and the C ABI of the PtyRAD forward/loss/adjoint
// hot path (gfx950), with the register / stripe engines' launch code.
//
// Per call (one group of mini-batches, include/ptyx.h), the general engine (ptyx_general.hpp,
// instantiated per N in the ptyx_gen.hip size groups and reached through GenOps):
//   k_probe_spectrum → k_forward → k_finalize (here: loss terms + adjoint coefficients,
//   losses.py:36-104) → k_adjoint → k_slab_reduce (here: fixed-order Σ over workgroup slabs)
//   → k_probe_finalize.
// The register engines (N = 128: ptyx_fused3.hpp, ptyx_fmm.hpp) and the stripe engine (N = 256:
// ptyx_stripe.hpp) replace k_forward / k_adjoint where their geometry applies (setup_call).
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <cstdlib>

#include "ptyx.h"
#include "ptyx_fft.hpp"
#include "ptyx_regfft.hpp"

#include "ptyx_common.hpp"
#include "ptyx_fused3.hpp"
#include "ptyx_fmm.hpp"
#include "ptyx_stripe.hpp"
#include "ptyx_abi.hpp"
#include "ptyx_adam.hpp"
#include "ptyx_genops.hpp"

namespace ptyx {

// the general engine's size registry (filled by the ptyx_gen.hip groups' static initialisers)
static std::vector<const GenOps*>& gen_registry() {
  static std::vector<const GenOps*> r;
  return r;
}
void gen_register(const GenOps* ops) { gen_registry().push_back(ops); }
const GenOps* gen_ops(int N) {
  for (const GenOps* o : gen_registry())
    if (o->N == N) return o;
  return nullptr;
}

// =====================================================================================
// k_finalize: one wave per mini-batch — loss terms and adjoint coefficients.
// bsums_out: write the mini-batch's additive sums (PTYX_BATCH_SUMS doubles: count, S_single,
// ΣM^q1, S_poissn, ΣM^q2, sparse sums per object mode) and stop (ptyx_forward_loss_grad_begin);
// bsums_in: take them from there instead of this call's patterns (ptyx_forward_loss_grad_end: the
// sums of a mini-batch whose patterns are split over ranks, all-reduced by the caller).
struct FinArgs {
  const int* boff;
  int n_batches, N, Nz, O;
  const float* psums;
  const float* occu;
  int single_on, pois_on, sparse_on, sparse_n;
  float w1, w2, ws, grad_scale;
  float* coef;
  float* loss_terms;
  float2* pcoef;   // optional, per pattern: (coef[ci], c_sparse) of its mini-batch (k_obj_gather)
  int ci;
  int pcoef_O = 1;             // object modes with a pcoef plane (plane o holds c_sparse of mode o)
  long long pcoef_stride = 0;  // patterns per plane
  double* bsums_out = nullptr;
  const double* bsums_in = nullptr;
  const float* lparts = nullptr;   // the data-term sums [0, kSumBase) as nparts partials per pattern
  int nparts = 0;                  // (k_fmm_loss, ≤ kFinMaxParts), added in part order
  const double* zsum = nullptr;    // object mode 0's sparse sum as zNz per-slice partials per pattern
  int zNz = 0;                     // (k_small_prep with use_zsum), added in slice order
};
constexpr int kFinMaxParts = 8;
static_assert(kSumBase == 4, "k_finalize reads the data-term sums as one float4");

// One wave per mini-batch: lane l sums patterns b0 + l, b0 + l + 64, … (fp64), then a fixed
// xor-tree over the lanes (deterministic, independent of how a call is split into pieces).  After
// the tree every lane holds the same sums, so every lane computes the (uniform) terms and
// coefficients; lane 0 stores them, every lane writes its share of the per-pattern coefficients.
// The object modes are a runtime loop with one accumulator at a time (no per-mode register arrays:
// indexed by the runtime O they went to scratch).
// finalize_batch: one wave, mini-batch m.  write: store the terms and coefficients (k_finalize);
// else only return the data-term coefficients (c_single, c_pois) in cdata — the small calls' tail
// launch recomputes them per workgroup instead of waiting for a k_finalize launch (one of its
// workgroups also writes, the same bits).
constexpr int kFinWaves = 2;   // mini-batches per 128-thread workgroup
__device__ __forceinline__ void finalize_batch(const FinArgs& f, int m, int lane, bool write, float* cdata) {
  const int b0 = f.boff[m], b1 = f.boff[m + 1];
  const double* bin = f.bsums_in ? f.bsums_in + (size_t)m * kNBatchSum : nullptr;
  // additive sum k of the mini-batch (k < kSumBase: the data terms, kSumBase + o: sparse mode o)
  auto wsum = [&](int k) -> double {
    if (bin) return bin[1 + k];
    double s = 0;
    if (f.zsum && k == kSumBase) {
      for (int t = b0 + lane; t < b1; t += 64)
        for (int z = 0; z < f.zNz; ++z) s += f.zsum[(size_t)t * f.zNz + z];
    } else {
      for (int t = b0 + lane; t < b1; t += 64) s += f.psums[(size_t)t * kNSum + k];
    }
#pragma unroll
    for (int x = 32; x >= 1; x >>= 1) s += __shfl_xor(s, x, 64);
    return s;
  };
  // the four data-term sums together (their loads in flight at once): from psums, or from the
  // per-pattern part partials (lparts, parts in order)
  double D[4] = {0, 0, 0, 0};
  if (bin) {
#pragma unroll
    for (int k = 0; k < 4; ++k) D[k] = bin[1 + k];
  } else {
    for (int t = b0 + lane; t < b1; t += 64) {
      if (f.lparts) {
        const float4* lp = reinterpret_cast<const float4*>(f.lparts) + (size_t)t * f.nparts;
        float4 q4[kFinMaxParts];
#pragma unroll
        for (int q = 0; q < kFinMaxParts; ++q)
          if (q < f.nparts) q4[q] = lp[q];
#pragma unroll
        for (int q = 0; q < kFinMaxParts; ++q)
          if (q < f.nparts) {
            D[0] += q4[q].x;
            D[1] += q4[q].y;
            D[2] += q4[q].z;
            D[3] += q4[q].w;
          }
      } else {
        const float4 v = *reinterpret_cast<const float4*>(f.psums + (size_t)t * kNSum);
        D[0] += v.x;
        D[1] += v.y;
        D[2] += v.z;
        D[3] += v.w;
      }
    }
#pragma unroll
    for (int x = 32; x >= 1; x >>= 1)
#pragma unroll
      for (int k = 0; k < 4; ++k) D[k] += __shfl_xor(D[k], x, 64);
  }
  const double B = bin ? bin[0] : (double)(b1 - b0);
  const double S1 = D[0], M1 = D[1], S2 = D[2], M2 = D[3];
  if (f.bsums_out) {
    double* bs = f.bsums_out + (size_t)m * kNBatchSum;
    if (lane == 0) {
      bs[0] = B; bs[1] = S1; bs[2] = M1; bs[3] = S2; bs[4] = M2;
    }
    for (int o = 0; o < kMaxModesO; ++o) {
      const double so = o < f.O ? wsum(kSumBase + o) : 0.0;
      if (lane == 0) bs[5 + o] = so;
    }
    return;
  }
  const double K = B * f.N * f.N;  // elements of the mini-batch DP stack
  float terms[5] = {0, 0, 0, 0, 0};
  float c_single = 0.f, c_pois = 0.f;
  if (f.single_on && B > 0) {  // w·sqrt(mean((I^q-M^q)^2)) / mean(M^q)   losses.py:45-47
    const double mu = M1 / K, rmse = sqrt(S1 / K);
    terms[0] = (float)(f.w1 * rmse / mu);
    c_single = rmse > 0 ? (float)(f.w1 / (mu * K * rmse) * f.grad_scale) : 0.f;
  }
  if (f.pois_on && B > 0) {  // -w·mean(M^q log(I^q+eps) - I^q) / mean(M^q)   losses.py:70-72
    const double mu = M2 / K;
    terms[1] = (float)(-f.w2 * (S2 / K) / mu);
    c_pois = (float)(-f.w2 / (mu * K) * f.grad_scale);
  }
  float* cfo = f.coef + (size_t)m * kNCoef;
  if (cdata) {
    cdata[0] = c_single;
    cdata[1] = c_pois;
  }
  if (!write) return;
  if (lane == 0) {
    cfo[0] = c_single;
    cfo[1] = c_pois;
  }
  const float c = f.ci == 0 ? c_single : f.ci == 1 ? c_pois : 1.f;   // (ci 2: already applied)
  const bool sparse = f.sparse_on && B > 0;
  const int nO = f.pcoef ? max(f.O, f.pcoef_O) : f.O;
  double t_sp = 0;
  for (int o = 0; o < nO; ++o) {   // w·Σ_o occ_o (mean |φ|^n)^(1/n)   losses.py:101
    float cs = 0.f;
    if (o < f.O && sparse) {
      const double cnt = B * f.Nz * f.N * f.N;
      const double mo = wsum(kSumBase + o) / cnt;
      const double inv = 1.0 / f.sparse_n;
      t_sp += f.occu[o] * pow(mo, inv);
      const double dm = (f.sparse_n == 1) ? 1.0 : (mo > 0 ? pow(mo, inv - 1.0) : 0.0);
      cs = (float)(f.ws * f.occu[o] * dm / cnt * f.grad_scale);
    }
    if (o < f.O && lane == 0) cfo[2 + o] = cs;
    if (f.pcoef && o < f.pcoef_O) {   // the mini-batch's coefficients, written for every pattern
      const float2 pc = make_float2(c, cs);
      for (int t = b0 + lane; t < b1; t += 64) f.pcoef[o * f.pcoef_stride + t] = pc;
    }
  }
  if (sparse) terms[3] = (float)(f.ws * t_sp);
  if (lane == 0 && f.loss_terms)
    for (int i = 0; i < 5; ++i) f.loss_terms[(size_t)m * 5 + i] = terms[i];
}
__global__ __launch_bounds__(64 * kFinWaves) void k_finalize(FinArgs f) {
  const int m = blockIdx.x * kFinWaves + (threadIdx.x >> 6);
  if (m >= f.n_batches) return;   // (wave-uniform)
  finalize_batch(f, m, threadIdx.x & 63, true, nullptr);
}

// Small calls of at most kTailFinBatches mini-batches: k_finalize folded into the probe / position
// tail launch (f3::small_tail_body).  Workgroup 0 is k_finalize (terms, coef, pcoef — the next
// launch's object gather reads pcoef); every other workgroup issues its first segment loads, then
// wave w computes mini-batch w's data-term coefficients (finalize_batch without the stores: the
// same fixed-order fp64 sums, so the same bits as workgroup 0's) while they are in flight.  One
// launch and its gap fewer per optimizer step at the default cadence; the same results.
constexpr int kTailFinBatches = 4;
template <bool KL>
__global__ __launch_bounds__(256) void k_small_tail_fin(FinArgs fa, const float2* segslab, const int* segbid, int nseg,
                                                        int ci, float2* out, const int* idx, int n, int n_scans,
                                                        const int* bid, const float* dsu, float* d_shifts,
                                                        const float2* twg, float2* cols_out) {
  __shared__ float s_c[kTailFinBatches][2];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (blockIdx.x == 0) {
    if (wave < fa.n_batches) finalize_batch(fa, wave, lane, true, nullptr);
    return;
  }
  f3::small_tail_body<KL>(
      (int)blockIdx.x - 1, segslab, segbid, nseg, [&](int m) { return ci >= 2 ? 1.f : s_c[m][ci]; },
      [&] {
        if (wave < fa.n_batches) finalize_batch(fa, wave, lane, false, s_c[wave]);
        __syncthreads();
      },
      out, idx, n, n_scans, bid, dsu, d_shifts, twg, cols_out);
}

#include "ptyx_gather.hpp"
#include "ptyx_stepfuse.hpp"

// d_H += Σ over workgroup propagator-gradient slabs, fixed order.
__global__ void k_hslab_reduce(const float2* hslab, int nwg, int n2, float2* d_H) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n2) return;
  float2 acc = make_float2(0.f, 0.f);
  for (int w = 0; w < nwg; ++w) acc = cadd(acc, hslab[(size_t)w * n2 + e]);
  d_H[e] = cadd(d_H[e], acc);
}

// Σ over workgroup slabs, fixed order.
__global__ void k_slab_reduce(const float2* slab, int nwg, long long per, float2* out) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= per) return;
  float2 acc = make_float2(0.f, 0.f);
  for (int w = 0; w < nwg; ++w) acc = cadd(acc, slab[(long long)w * per + e]);
  out[e] = acc;
}


}  // namespace ptyx

// =========================================================================================
// C ABI
// =========================================================================================
using namespace ptyx;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(PTYX_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

struct DeviceGuard {
  int prev = -1, want;
  explicit DeviceGuard(int d) : want(d) {
    (void)hipGetDevice(&prev);
    if (prev != want) (void)hipSetDevice(want);
  }
  ~DeviceGuard() {
    if (prev >= 0 && prev != want) (void)hipSetDevice(prev);
  }
};
// Engine-variant tuning (ptyx_set_tuning): -1 = the measured default.  Process-wide; the
// variants all compute the same results (tests/test_gpu_configs.py checks each against the oracle).
enum TuneKey { kTuneHold = 0, kTunePsi0, kTuneGather, kTuneDeferGroups, kTuneGatherSplit, kTuneGenWg, kTuneGatherRows,
               kTuneFmmHoldH, kTuneFuseAdam, kTuneTailFin, kTuneSmallSpec, kTuneSelFold, kTuneRowsHu, kTunePsiHold,
               kTuneGadamLead, kTuneCount };
const char* const kTuneNames[kTuneCount] = {"s3_hold", "s_psi0", "s_gather", "s_defer_groups", "gather_split",
                                            "gen_wg_per_cu", "gather_rows", "fmm_hold_h", "fuse_adam",
                                            "tail_fin", "small_spec", "sel_fold", "rows_hu", "psi_hold",
                                            "gadam_lead"};
const long long kTuneMax[kTuneCount] = {4, 1, 1, 4096, 16, 16, 3, 1, 1, 1, 1, 1, 2, 2, 1};
long long g_tuning[kTuneCount] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
}  // namespace

extern "C" int ptyx_set_tuning(const char* key, int64_t value) {
  g_err.clear();
  for (int k = 0; key && k < kTuneCount; ++k)
    if (std::strcmp(key, kTuneNames[k]) == 0) {
      if (value < -1 || value > kTuneMax[k]) return fail(PTYX_EINVAL, std::string("tuning value out of range: ") + key);
      g_tuning[k] = value;
      return PTYX_OK;
    }
  return fail(PTYX_EINVAL, std::string("unknown tuning key: ") + (key ? key : "(null)"));
}

extern "C" int64_t ptyx_get_tuning(const char* key) {
  for (int k = 0; key && k < kTuneCount; ++k)
    if (std::strcmp(key, kTuneNames[k]) == 0) return g_tuning[k];
  return -2;
}

struct ptyx_plan {
  ptyx_dims d;
  int device = 0;
  int n_cu = 0;
  const GenOps* gen = nullptr;   // the general engine's kernels for this N (ptyx_genops.hpp)
  int nwg = 0;  // persistent workgroups for k_forward / k_adjoint
  float2* twg = nullptr;
  float2* Fp = nullptr;
  float2* FpT = nullptr;      // N = 256: F(P) and H transposed for the fused chains (KArgs::FpT / HT)
  float2* HT = nullptr;
  float* psums = nullptr;
  float* coef = nullptr;
  float* Ibuf = nullptr;
  float* Ibuf2 = nullptr;     // mixed-state register engine with both data terms: ∂ℓ_poissn/∂I planes
  float* lparts = nullptr;    // mixed-state register engine: k_fmm_loss partial sums (patterns, parts, 4)
  double* zsum = nullptr;     // small multislice calls: loss_sparse window sums per (pattern, slice)
  bool zsum_call = false;     // the current call's k_small_prep wrote zsum (k_finalize reads it)
  float* Imodes = nullptr;    // probe-mode split: P mode-intensity planes per pattern (≤ kModeSplitCap)
  float2* slab = nullptr;
  float2* Gsum = nullptr;
  float2* hslab = nullptr;    // PTYX_PROP_GRAD: per-workgroup dL/dH slabs
  float2* ffc = nullptr;      // far-field cache (general engine: P·O > 1, N > 128 or Nz > 1)
  long long ffc_per = 0, ffc_cap = 0;
  float2* scratch = nullptr;
  // register engines (k_fused3 / k_fused3ms): per-pattern object-gradient slots
  long long og_cap = 0;       // patterns per call the slots can hold (0: path unavailable)
  float2* ogscr = nullptr;
  int* bid = nullptr;
  int2* geo = nullptr;
  float2* pcoef = nullptr;
  // k_fused3 (N = 128, single mode, f32 DPs): register-resident FFT, 2 workgroups per CU
  int nwg3 = 0;
  float2* fpk = nullptr;      // packed probe spectrum / probe
  float2* oc = nullptr;       // A e^{iφ}
  double* pref = nullptr;     // summed-area table of |φ|^n (loss_sparse), (Nz, Ny, Nx + 1)
  double* preftot = nullptr;  // its per-chunk column totals, (Nz, ⌈Ny / kPrefChunk⌉, Nx + 1)
  float2* segslab = nullptr;  // per-segment unit probe-gradient spectra, packed
  int* segbid = nullptr;      // batch of each segment id (-1 unused)
  // k_obj_gather candidate bins (tile of each pattern's window origin), per call
  int nbins = 0;
  int* bcnt = nullptr;        // (nbins) counts
  int* boff = nullptr;        // (nbins + 1) offsets
  int* bcur = nullptr;        // (nbins) fill cursors
  int* bkey = nullptr;        // (max_patterns) bin of each pattern
  int* blist = nullptr;       // (max_patterns) patterns by bin
  float2* gpart = nullptr;    // split gather: tile partials (kGatherPartCap × 64·16)
  float* gpcnt = nullptr;
  int gpart_cap = 0;          // partial tiles gpart / gpcnt hold
  float* dsu = nullptr;       // per-pattern unit position-gradient sums
  float2* segpart = nullptr;  // k_segslab_reduce partials (kSegSplit × N²)
  float2* hpk = nullptr;      // k_fused3ms: K-packed propagator / N²
  int* bbox = nullptr;        // k_fused3*: bounding box of a call's windows
  bool ms3 = false;           // k_fused3ms (multislice register engine) available
  bool fmm = false;           // k_fmm_* (mixed-state register engine, N = 128, P > 1, O = 1) available
  int* err_host = nullptr;    // input-error flags (kErrWords ints, host-mapped; the kernels write 1s)
  int* err_dev = nullptr;     // their device address
  // N = 256 stripe engine (ptyx_stripe.hpp): per-call intermediates for stripe_cap patterns
  long long stripe_cap = 0;
  int stripe_groups = 0;
  int stripe_defer_groups = 0;  // k_s5 groups of calls that defer the probe epilogue (fills the GPU once)
  bool slab_live = false;       // k_s5 partials of earlier calls of the step await their reduction
  int slab_live_groups = 0;
  const float* slab_live_probe = nullptr;
  float2* st14 = nullptr;
  float2* spsi0 = nullptr;
  float2* st23 = nullptr;
  float* spsum = nullptr;
  float* sdsp = nullptr;
  float2* ssxy = nullptr;     // (max_patterns) per-call (sy, sx)
  float2* sslab = nullptr;
  bool sgather = false;       // stripe object gradient: per-pattern slots + k_obj_gather (else f32 atomics)
  long long seg_cap = 0;      // segment ids the segslab holds
  long long scratch_stride = 0;
  size_t ws_bytes = 0;
  std::vector<void*> allocs;
  // What the last PTYX_PREP_FULL call left in Fp / fpk / hpk / oc / pref: a PTYX_PREP_REUSE call
  // that does not match it prepares in full (include/ptyx.h)
  struct PrepRecord {
    bool valid = false;
    int engine = -1;
    const void *obja = nullptr, *objp = nullptr, *probe = nullptr, *H = nullptr;
    int sparse_on = 0, sparse_n = 0;
  } prep;
  // ptyx_forward_loss_grad_begin → _end: the call in flight
  bool pend = false;
  ptyx_inputs pend_in{};
  ptyx_grads pend_gz{};
  ptyx_loss_cfg pend_cfg{};
  const int32_t* pend_idx = nullptr;
  const int32_t* pend_boff = nullptr;
  int32_t pend_nb = 0, pend_n = 0;
  float* pend_dp = nullptr;
  int pend_engine = -1;
  bool pend_defer_gather = false;   // PTYX_PREP_DEFER_GATHER on the call in flight
  bool pend_store = false;          // PTYX_PREP_GRAD_STORE served by its engine's gather
  // the last split call that deferred its object gather (ptyx_slots_export reads it): its slots,
  // pattern table and coefficients stay in the plan until the next compute call
  // ptyx_plan_slot_target: the next deferring call writes its slots straight into the caller's
  // block (no copy in ptyx_slots_export); consumed by that call
  float* slot_tgt = nullptr;
  int32_t slot_tgt_cap = 0;
  bool use_tgt = false;             // the call in flight writes its slots to slot_tgt
  float* slots_at = nullptr;        // where the last deferring call's slots are
  bool gather_deferred = false;     // set while that call's _end runs (run_fused3 skips the gather)
  bool grad_store = false;          // PTYX_PREP_GRAD_STORE on the call in flight
  bool slots_ready = false;
  int32_t slots_n = 0;
  const int32_t* slots_idx = nullptr;
  // ptyx_plan_set_select: the step selection the next PTYX_PREP_SELECT call takes (one-shot); sel_fold:
  // the call in flight does it inside k_small_prep (register_prep)
  bool sel_set = false;
  bool sel_fold = false;
  const int32_t* sel_all = nullptr;
  const int64_t* sel_start = nullptr;
  const int64_t* sel_cnt = nullptr;
  float* sel_grad = nullptr;
  int64_t sel_grad_n = 0;
  float* const* sel_steps = nullptr;
  int32_t sel_n_steps = 0;
  // ptyx_plan_set_adam: the optimizer step the next PTYX_PREP_FUSED_ADAM call takes (one-shot)
  bool fadam_set = false;
  bool fadam_on = false;            // the call in flight takes it
  bool fadam_done = false;          // its engine fused it into the epilogue (else a k_adam launch follows)
  std::vector<opt::AdamTensor> fadam_ts;
  opt::AdamHyper fadam_h{};
  bool fadam_store = false;
  opt::StepStore fadam_ss{};
  // ptyx_profile_begin/end: HIP events around every launch (kind, start, stop)
  bool prof = false;
  struct ProfRec {
    int kind;
    hipEvent_t a, b;
  };
  mutable std::vector<ProfRec> recs;
};

static int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, what);
  return PTYX_OK;
}

// Fill n 32-bit words with v on the stream: a kernel, not hipMemsetAsync — a memset captured into a
// hipGraph (graph-replayed optimizer steps) was measured to leave a buffer's unaligned 8-byte tail
// untouched on replay (the PTYX_PREP_GRAD_STORE clear of a 19,208-byte object plane,
// tools/diag_store.py), so every in-stream fill of the engine is this kernel.
__global__ void k_fill32(uint32_t* p, int64_t n, uint32_t v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}
static int fill32(void* p, int64_t n, uint32_t v, hipStream_t st) {
  if (n <= 0) return PTYX_OK;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(2048, (n + 255) / 256));
  hipLaunchKernelGGL(k_fill32, dim3(blocks), dim3(256), 0, st, reinterpret_cast<uint32_t*>(p), n, v);
  return launch_status("k_fill32 launch");
}

static int busy(const ptyx_plan* pl) {
  return pl->pend ? fail(PTYX_EINVAL, "a ptyx_forward_loss_grad_begin call is waiting for its _end on this plan") : 0;
}

enum KernelKind {
  kKSpectrum, kKForward, kKFinalize, kKAdjoint, kKSlabReduce, kKProbeFinalize, kKFused, kKTable, kKGather,
  kKObjPrep, kKPack, kKS1, kKS2, kKS3, kKS4, kKS5, kKFmmFwd, kKFmmLoss, kKFmmAdj, kKGatherAdam, kKCount
};
static const char* const kKernelNames[kKCount] = {"k_probe_spectrum", "k_forward",        "k_finalize",
                                                  "k_adjoint",        "k_slab_reduce",    "k_probe_finalize",
                                                  "k_fused",          "k_pattern_table",  "k_obj_gather",
                                                  "k_obj_prep",       "k_pack",           "k_s1",
                                                  "k_s2",             "k_s3",             "k_s4",
                                                  "k_s5",             "k_fmm_fwd",        "k_fmm_loss",
                                                  "k_fmm_adj",        "k_gather_adam"};

// Brackets one launch with HIP events on its stream while the plan is profiling.
struct ProfScope {
  const ptyx_plan* pl;
  int kind;
  hipStream_t st;
  hipEvent_t a = nullptr, b = nullptr;
  ProfScope(const ptyx_plan* p, int k, hipStream_t s) : pl(p), kind(k), st(s) {
    if (pl->prof && hipEventCreate(&a) == hipSuccess && hipEventCreate(&b) == hipSuccess)
      (void)hipEventRecord(a, st);
  }
  ~ProfScope() {
    if (pl->prof && a && b) {
      (void)hipEventRecord(b, st);
      pl->recs.push_back({kind, a, b});
    }
  }
};

template <class T>
static int dalloc(ptyx_plan* pl, T** p, size_t count) {
  *p = nullptr;
  if (count == 0) return PTYX_OK;
  void* q = nullptr;
  hipError_t e = hipMalloc(&q, count * sizeof(T));
  if (e != hipSuccess) return fail(PTYX_ENOMEM, std::string("hipMalloc failed: ") + hipGetErrorString(e));
  pl->allocs.push_back(q);
  pl->ws_bytes += count * sizeof(T);
  *p = static_cast<T*>(q);
  return PTYX_OK;
}

// k_obj_gather's pattern bins: one per object tile
static int alloc_bins(ptyx_plan* pl) {
  const ptyx_dims& d = pl->d;
  pl->nbins = ((d.Nx + kGTX - 1) / kGTX) * ((d.Ny + kGTY - 1) / kGTY);
  int rc;
  if ((rc = dalloc(pl, &pl->bcnt, (size_t)pl->nbins)) || (rc = dalloc(pl, &pl->boff, (size_t)pl->nbins + 1)) ||
      (rc = dalloc(pl, &pl->bcur, (size_t)pl->nbins)) || (rc = dalloc(pl, &pl->bkey, (size_t)d.max_patterns)) ||
      (rc = dalloc(pl, &pl->blist, (size_t)d.max_patterns)))
    return rc;
  // split-gather partials: the default rule (launch_gather) splits only below 1,024 tile planes and
  // then uses at most parts·min(8, ⌈2048/parts⌉) < 3,072 partial tiles; a plan whose single slice
  // already has 1,024 tiles never splits (no buffer) unless the gather_split tuning key was set
  // when it was created (then the whole kGatherPartCap)
  pl->gpart_cap = g_tuning[kTuneGatherSplit] >= 1 ? kGatherPartCap : pl->nbins >= 1024 ? 0 : 3072;
  if ((rc = dalloc(pl, &pl->gpart, (size_t)pl->gpart_cap * kGTY * kGTX)) ||
      (rc = dalloc(pl, &pl->gpcnt, (size_t)pl->gpart_cap * kGTY * kGTX)))
    return rc;
  return PTYX_OK;
}

// k_obj_gather over `tiles` × `nzg` tile planes.  A grid that cannot fill the GPU (a small object:
// the tBL demo's 370² has 144 tiles a slice) splits every tile's candidates over S workgroups whose
// partial sums k_obj_gather_fin adds in split order (deterministic for a given call shape).
// The small gathers' form: 0 = tiles (k_obj_gather; fused: gather_adam_tile), 1 = row-split
// (k_obj_gather_rows; fused: the row tiles), 2 = row-split with the fused single-plane launch held
// to 128 VGPRs (k_gather_adam_r4: four workgroups a CU; mixed-state calls: as 1), 3 = the same at
// 96 VGPRs (k_gather_adam_r5: five a CU, 20 B of spill; every tile of a c2 call in one round).
// Tuning gather_rows overrides for every unsplit gather; by default calls of at most kSmallCall
// patterns run row-split — single-state ones in form 3 (c2 at ga = 1: the fused launch 22.2 →
// 20.4 (form 2) → 19.0 µs, profiles/r06/rows_r4/, rows_r5/) — and larger ones in tiles.  One decision for the fused and the unfused
// launches, so both sum every pixel's hits in the same order (bitwise the same gradients).
static int gather_form(bool mp, long long n) {
  const long long tr = g_tuning[kTuneGatherRows];
  if (tr >= 0) return (int)tr;
  if (n > f3::kSmallCall) return 0;
  return mp ? 1 : 3;
}

template <int N, bool ROWPERM, bool MP>
static void launch_gather(const ptyx_plan* pl, GatherArgs g, int tiles, int nzg, bool sparse_tiles, hipStream_t st) {
  const int parts = tiles * nzg;
  int S = 1;
  // (not for small calls: a tile's few candidates are not worth the extra partial-sum launch)
  if (parts < 1024 && pl->gpart && g.n > f3::kSmallCall)
    S = std::max(1, std::min({8, (2048 + parts - 1) / parts, pl->gpart_cap / parts}));
  if (g_tuning[kTuneGatherSplit] >= 1 && pl->gpart)
    S = std::max(1, std::min<int>((int)g_tuning[kTuneGatherSplit], pl->gpart_cap / parts));
  g.part = pl->gpart;
  g.pcnt = pl->gpcnt;
  // rows over waves (k_obj_gather_rows): gather_form
  if (S == 1 && gather_form(MP, g.n) >= 1) {
    if (sparse_tiles) hipLaunchKernelGGL((k_obj_gather_rows<N, ROWPERM, 4, MP>), dim3(tiles, nzg), dim3(64 * 4), 0, st, g);
    else hipLaunchKernelGGL((k_obj_gather_rows<N, ROWPERM, kGWaves, MP>), dim3(tiles, nzg), dim3(64 * kGWaves), 0, st, g);
    return;
  }
  if (S == 1) {
    if (sparse_tiles) hipLaunchKernelGGL((k_obj_gather<N, ROWPERM, 4, MP>), dim3(tiles, nzg), dim3(64 * 4), 0, st, g);
    else hipLaunchKernelGGL((k_obj_gather<N, ROWPERM, kGWaves, MP>), dim3(tiles, nzg), dim3(64 * kGWaves), 0, st, g);
    return;
  }
  const dim3 gr(tiles, nzg, S);
  if (sparse_tiles) hipLaunchKernelGGL((k_obj_gather<N, ROWPERM, 4, MP, true>), gr, dim3(64 * 4), 0, st, g);
  else hipLaunchKernelGGL((k_obj_gather<N, ROWPERM, kGWaves, MP, true>), gr, dim3(64 * kGWaves), 0, st, g);
  hipLaunchKernelGGL(k_obj_gather_fin<N>, dim3(tiles, nzg), dim3(256), 0, st, g, S);
}

static void free_plan(ptyx_plan* pl) {
  if (pl->err_host) (void)hipHostFree(pl->err_host);
  for (void* q : pl->allocs) (void)hipFree(q);
  delete pl;
}

extern "C" int ptyx_version(void) { return PTYX_ABI_VERSION; }

extern "C" int ptyx_abi_struct_sizes(size_t* out, int32_t cap) {
  const size_t sz[7] = {sizeof(ptyx_dims),        sizeof(ptyx_inputs),          sizeof(ptyx_grads),
                        sizeof(ptyx_loss_cfg),    sizeof(ptyx_kernel_stat),     sizeof(ptyx_obj_constraints),
                        sizeof(ptyx_meas_proc)};
  for (int i = 0; out && i < cap && i < 7; ++i) out[i] = sz[i];
  return 7;
}

extern "C" const char* ptyx_last_error(void) { return g_err.c_str(); }

extern "C" size_t ptyx_plan_workspace_bytes(const ptyx_plan* plan) { return plan ? plan->ws_bytes : 0; }

extern "C" int64_t ptyx_plan_register_capacity(const ptyx_plan* plan) {
  if (plan && plan->nwg3 > 0) return (int64_t)plan->og_cap;
  if (plan && plan->stripe_cap > 0) return (int64_t)plan->stripe_cap;
  return (plan && plan->ffc_cap > 0) ? (int64_t)plan->ffc_cap : 0;   // far-field cache capacity
}

extern "C" int ptyx_plan_create(ptyx_plan** out, const ptyx_dims* dims, int device) {
  g_err.clear();
  if (!out || !dims) return fail(PTYX_EINVAL, "null argument");
  *out = nullptr;
  const ptyx_dims& d = *dims;
  if (d.abi_version != PTYX_ABI_VERSION)
    return fail(PTYX_EINVAL, "ptyx_dims.abi_version " + std::to_string(d.abi_version) + " != " +
                                 std::to_string(PTYX_ABI_VERSION) +
                                 ": the binding's structs follow another revision of include/ptyx.h");
  const GenOps* gen = gen_ops(d.N);
  if (!gen)
    return fail(PTYX_EUNSUPPORTED, "N = " + std::to_string(d.N) +
                                       ": N must be 2·3·5·7-smooth in [32, 512] (2^a 3^b 5^c 7^d: 32, 35, 36, 40, 42, 45, ..., 504, 512)");
  if (d.P < 1 || d.O < 1 || d.Nz < 1 || d.n_scans < 1 || d.max_patterns < 1)
    return fail(PTYX_EINVAL, "P, O, Nz, n_scans, max_patterns must be >= 1");
  if (d.O > kMaxModesO) return fail(PTYX_EUNSUPPORTED, "at most 32 object modes");
  if (d.Ny < d.N || d.Nx < d.N) return fail(PTYX_EINVAL, "object smaller than the probe window");
  DeviceGuard dg(device);
  int cu = 0;
  hipError_t e = hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, device);
  if (e != hipSuccess) return hip_fail(e, "hipDeviceGetAttribute");
  auto* pl = new ptyx_plan();
  pl->d = d;
  pl->device = device;
  pl->n_cu = cu;
  pl->gen = gen;
  const int wg_cu = g_tuning[kTuneGenWg] >= 1 ? (int)g_tuning[kTuneGenWg] : gen->blocks_per_cu;
  pl->nwg = std::max(d.P, std::min(d.max_patterns, cu * wg_cu));
  const size_t N2 = (size_t)d.N * d.N;
  const bool lds = gen->lds;
  const bool prop_grad = (d.flags & PTYX_PROP_GRAD) && d.Nz > 1;
  pl->scratch_stride = (long long)((lds ? 0 : 2 * N2) + (size_t)d.Nz * N2 + N2 +
                                   (prop_grad ? (size_t)(d.Nz - 1) * N2 : 0));
  int rc = PTYX_OK;
  const bool multi = (d.P * d.O) > 1;
  if ((rc = dalloc(pl, &pl->twg, d.N)) || (rc = dalloc(pl, &pl->Fp, d.P * N2)) ||
      (rc = dalloc(pl, &pl->psums, (size_t)d.max_patterns * kNSum)) ||
      (rc = dalloc(pl, &pl->coef, (size_t)d.max_patterns * kNCoef)) ||
      (rc = dalloc(pl, &pl->Ibuf, multi ? (size_t)d.max_patterns * N2 : 0)) ||
      (rc = dalloc(pl, &pl->Imodes, d.P > 1 ? (size_t)d.P * std::min(d.max_patterns, kModeSplitCap) * N2 : 0)) ||
      (rc = dalloc(pl, &pl->slab, (size_t)pl->nwg * d.P * N2)) ||
      (rc = dalloc(pl, &pl->Gsum, d.P * N2)) ||
      (rc = dalloc(pl, &pl->hslab, prop_grad ? (size_t)pl->nwg * N2 : 0)) ||
      (rc = dalloc(pl, &pl->scratch, (size_t)pl->nwg * pl->scratch_stride)) ||
      (rc = dalloc(pl, &pl->FpT, d.N == 256 && (d.flags & PTYX_SHIFT_PROBES) ? d.P * N2 : 0)) ||
      (rc = dalloc(pl, &pl->HT, d.N == 256 && d.Nz > 1 ? N2 : 0))) {
    free_plan(pl);
    return rc;
  }
  const bool stripe = d.N == 256 && d.Nz == 1 && d.O <= sp::kMaxO && (d.flags & PTYX_SHIFT_PROBES);
  if (stripe) {
    // per-call intermediates (T1/T4, ψ⁰: P fields; T2/T3: P·O fields per pattern; without the ψ⁰
    // park, k_s4 recomputes it) within PTYX_STRIPE_MB (default the smaller of 16 GiB
    // and a quarter of the free HBM); calls beyond the capacity are split by the host at
    // mini-batch boundaries
    size_t free_b = 0, total_b = 0;
    (void)hipMemGetInfo(&free_b, &total_b);
    long long mb = std::min<long long>(16384, (long long)(free_b / 4 / (1 << 20)));
    if (const char* e = std::getenv("PTYX_STRIPE_MB")) mb = std::atoll(e);
    // measured (profiles/r02/r02k_*): one object mode recomputes ψ⁰ in P4 (c5 221 k vs 205 k
    // patterns/s: the park's write in P2 costs more than the row IFFT); two object modes park it
    // (c3 66.0 k vs 59.9 k: P4 with the extra transform spills)
    const bool park = g_tuning[kTunePsi0] >= 0 ? g_tuning[kTunePsi0] != 0 : d.O > 1;
    const long long per = (long long)((park ? 2 : 1) * d.P + d.P * d.O) * (long long)N2 * (long long)sizeof(float2);
    const long long cap = std::min<long long>(d.max_patterns, (mb << 20) / per);
    if (cap >= 1) {
      const int groups = std::max(1, std::min<int>((int)cap, (2048 + 16 * d.P - 1) / (16 * d.P)));
      if ((rc = dalloc(pl, &pl->st14, (size_t)cap * d.P * N2)) ||
          (rc = dalloc(pl, &pl->spsi0, park ? (size_t)cap * d.P * N2 : 0)) ||
          (rc = dalloc(pl, &pl->st23, (size_t)cap * d.P * d.O * N2)) ||
          (rc = dalloc(pl, &pl->spsum, (size_t)cap * sp::kStripes * kNSum)) ||
          (rc = dalloc(pl, &pl->sdsp, (size_t)cap * sp::kStripes * d.P * 2)) ||
          (rc = dalloc(pl, &pl->ssxy, (size_t)d.max_patterns)) ||
          (rc = dalloc(pl, &pl->sslab, (size_t)groups * d.P * N2)) ||
          (rc = dalloc(pl, &pl->bid, (size_t)d.max_patterns)) || (rc = dalloc(pl, &pl->geo, (size_t)d.max_patterns)) ||
          (rc = dalloc(pl, &pl->oc, (size_t)d.O * d.Ny * d.Nx)) || (rc = dalloc(pl, &pl->bbox, 4))) {
        free_plan(pl);
        return rc;
      }
      pl->stripe_cap = cap;
      pl->stripe_groups = groups;
      pl->stripe_defer_groups = std::max(1, std::min(groups, 2 * cu / (sp::kStripes * d.P)));
      // object gradient of two object modes: k_s4 writes per-pattern slots (over the T3 fields it
      // has consumed) and k_obj_gather reduces them per tile (deterministic, no atomics).  One
      // object mode keeps k_s4's f32 atomics (profiles/r02/ab/r02y_*: the epilogue costs c3 20 ms
      // of 66 in k_s4 but c5 only 2.7 of 23, less than the slot stores plus the gather would).
      pl->sgather = g_tuning[kTuneGather] >= 0 ? g_tuning[kTuneGather] != 0 : d.O > 1;
      if (pl->sgather && ((rc = dalloc(pl, &pl->pcoef, (size_t)d.max_patterns * d.O)) || (rc = alloc_bins(pl)))) {
        free_plan(pl);
        return rc;
      }
    }
  }
  // (one probe and object mode: the global-scratch general engine (N > 128) and the multislice one
  // (Nz > 1) cache too, so k_adjoint reads the far field and the ψⁿ instead of recomputing the
  // forward; N = 128 single-mode calls run on the register engines)
  const bool ffc_single = d.P * d.O == 1 && d.N != 128 && (d.N > 128 || d.Nz > 1);
  if (d.P * d.O > 1 || ffc_single) {
    // far-field cache: per pattern of a call the P·O far fields plus ψ⁰ of every probe mode (Nz = 1)
    // or every slice's ψⁿ of every (p, o) (Nz > 1) — (P·O + P)·N² or P·O·(1 + Nz)·N² float2 —
    // within PTYX_FFC_MB (default the smaller of 64 GiB and a third of the free HBM); calls beyond
    // its capacity are split by the host.  A stripe plan keeps one for the calls the stripe engine
    // declines (both data terms on), sized to its call size within a sixth of the free HBM
    // (without it those calls recompute k_adjoint's forward).
    size_t free_b = 0, total_b = 0;
    (void)hipMemGetInfo(&free_b, &total_b);
    long long mb = std::min<long long>(stripe ? free_b / 6 / (1 << 20) : 65536, (long long)(free_b / 3 / (1 << 20)));
    if (const char* e = std::getenv("PTYX_FFC_MB")) mb = std::atoll(e);
    const long long per = (long long)(d.Nz > 1 ? d.P * d.O * (1 + d.Nz) : d.P * d.O + d.P) * (long long)N2;
    // (the mixed-state register engine, N = 128 with one object mode and f32 DPs, keeps its slots
    // here and works with any capacity)
    const bool fmm_geo = d.N == 128 && d.O == 1 && d.P <= kGatherMaxNp && !(d.flags & PTYX_MEAS_F16);
    const long long need = fmm_geo ? 1 : std::min<long long>(d.max_patterns, stripe ? pl->stripe_cap : pl->nwg);
    long long cap = std::min<long long>(d.max_patterns, (mb << 20) / (per * (long long)sizeof(float2)));
    if (stripe) cap = std::min(cap, need);
    if (need > 0 && cap >= need) {
      if ((rc = dalloc(pl, &pl->ffc, (size_t)cap * per))) {
        free_plan(pl);
        return rc;
      }
      pl->ffc_per = per;
      pl->ffc_cap = cap;
    }
  }
  if (d.N == 128 && d.P > 1 && d.P <= kGatherMaxNp && d.O == 1 && !(d.flags & PTYX_MEAS_F16) && pl->ffc) {
    // mixed-state register engine (ptyx_fmm.hpp): its slots (parked ψⁿ, then the object gradient)
    // and far fields are the far-field cache's planes, P·(Nz + 1) per pattern, so it needs no
    // per-pattern memory of its own and takes the same call sizes; jobs are (pattern, probe mode)
    int occ3 = 0, o2 = 0;
    bool ok = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ3, f3::k_fmm_fwd<true, false>, 256, 0) == hipSuccess && occ3 > 0;
    for (auto kf : {f3::k_fmm_fwd<false, false>, f3::k_fmm_adj<true, false, false>, f3::k_fmm_adj<false, false, false>,
                    f3::k_fmm_adj<true, true, false>, f3::k_fmm_adj<false, true, false>})
      if (ok && hipOccupancyMaxActiveBlocksPerMultiprocessor(&o2, kf, 256, 0) == hipSuccess) occ3 = std::min(occ3, o2);
    if (ok && occ3 > 0) {
      pl->nwg3 = (int)std::min<long long>((long long)cu * occ3, std::max<long long>(1, (long long)d.max_patterns * d.P));
      pl->seg_cap = d.P + pl->nwg3;   // segment ids p + w
      if ((rc = dalloc(pl, &pl->bid, (size_t)d.max_patterns)) || (rc = dalloc(pl, &pl->geo, (size_t)d.max_patterns)) ||
          (rc = dalloc(pl, &pl->pcoef, (size_t)d.max_patterns)) || (rc = dalloc(pl, &pl->fpk, (size_t)d.P * N2)) ||
          (rc = dalloc(pl, &pl->hpk, N2)) || (rc = dalloc(pl, &pl->bbox, 4)) ||
          (rc = dalloc(pl, &pl->oc, (size_t)d.Nz * d.Ny * d.Nx)) ||
          (rc = dalloc(pl, &pl->pref, (size_t)d.Nz * d.Ny * (d.Nx + 1))) ||
          (rc = dalloc(pl, &pl->preftot, (size_t)d.Nz * ((d.Ny + f3::kPrefChunk - 1) / f3::kPrefChunk) * (d.Nx + 1))) ||
          (rc = dalloc(pl, &pl->segslab, (size_t)pl->seg_cap * N2)) || (rc = dalloc(pl, &pl->segbid, (size_t)pl->seg_cap)) ||
          (rc = dalloc(pl, &pl->dsu, (size_t)d.max_patterns * d.P * 2)) ||
          (rc = dalloc(pl, &pl->segpart, (size_t)d.P * f3::kSegSplit * N2)) || (rc = alloc_bins(pl)) ||
          (rc = dalloc(pl, &pl->Ibuf2, (size_t)pl->ffc_cap * N2)) ||
          (rc = dalloc(pl, &pl->lparts, (size_t)d.max_patterns * f3::kLossParts * kSumBase))) {
        free_plan(pl);
        return rc;
      }
      pl->og_cap = pl->ffc_cap;
      pl->fmm = true;
    }
  }
  if (d.N == 128 && d.P * d.O * d.Nz == 1 && !(d.flags & PTYX_MEAS_F16)) {
    // single-slice register engine: one g_O slot per pattern of a call (N² float2), bounded by
    // PTYX_OBJ_SCRATCH_MB; larger calls are split by the host at mini-batch boundaries
    long long mb = 16384;
    if (const char* s = std::getenv("PTYX_OBJ_SCRATCH_MB")) mb = std::max(0LL, std::atoll(s));
    const long long cap = std::min<long long>(d.max_patterns, (mb << 20) / (long long)(sizeof(float2) * N2));
    int occ3 = 0;
    if (cap > 0 &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ3, f3::k_fused3<true, true, 0>, 256, 0) == hipSuccess &&
        occ3 > 0) {
      int o2 = 0;
      for (auto kf : {f3::k_fused3<true, true, 2>, f3::k_fused3<true, false, 2>, f3::k_fused3<false, true, 0>,
                      f3::k_fused3<false, true, 2>, f3::k_fused3<false, false, 2>})
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o2, kf, 256, 0) == hipSuccess) occ3 = std::min(occ3, o2);
      pl->nwg3 = std::min(cu * occ3, std::max(1, d.max_patterns));
      // segment ids = mini-batches + workgroups of a call; sized for a mean mini-batch of ≥ 8
      // patterns; calls with more segments take the two-pass engine
      constexpr long long div = 8;
      pl->seg_cap = pl->nwg3 + (cap + div - 1) / div;   // a call holds at most `cap` patterns
      if ((rc = dalloc(pl, &pl->ogscr, (size_t)cap * N2)) || (rc = dalloc(pl, &pl->bid, (size_t)d.max_patterns)) ||
          (rc = dalloc(pl, &pl->geo, (size_t)d.max_patterns)) || (rc = dalloc(pl, &pl->pcoef, (size_t)d.max_patterns)) ||
          (rc = dalloc(pl, &pl->fpk, N2)) || (rc = dalloc(pl, &pl->oc, (size_t)d.Ny * d.Nx)) ||
          (rc = dalloc(pl, &pl->bbox, 4)) ||
          (rc = dalloc(pl, &pl->pref, (size_t)d.Ny * (d.Nx + 1))) ||
          (rc = dalloc(pl, &pl->preftot, (size_t)((d.Ny + f3::kPrefChunk - 1) / f3::kPrefChunk) * (d.Nx + 1))) ||
          (rc = dalloc(pl, &pl->segslab, (size_t)pl->seg_cap * N2)) ||
          (rc = dalloc(pl, &pl->segbid, (size_t)pl->seg_cap)) ||
          (rc = dalloc(pl, &pl->dsu, (size_t)d.max_patterns * 2)) ||
          (rc = dalloc(pl, &pl->segpart, (size_t)f3::kSegSplit * N2)) || (rc = alloc_bins(pl))) {
        free_plan(pl);
        return rc;
      }
      pl->og_cap = cap;
    }
  }
  if (d.N == 128 && d.P * d.O == 1 && d.Nz > 1 && !(d.flags & PTYX_MEAS_F16)) {
    // multislice register engine: Nz slot planes per pattern (parked ψⁿ, then slice n's
    // object gradient), bounded by PTYX_OBJ_SCRATCH_MB (default the smaller of 64 GiB and a third
    // of the free HBM).  Every call's k_obj_gather reads and writes the object band its windows
    // reach, once per slice: fewer, larger calls cut that traffic (c4: 8,192 → 32,768 patterns
    // per call, 128 → 32 gathers of the 16 × 3679² object per step).
    size_t free_b = 0, total_b = 0;
    (void)hipMemGetInfo(&free_b, &total_b);
    long long mb = std::min<long long>(65536, (long long)(free_b / 3 / (1 << 20)));
    if (const char* s = std::getenv("PTYX_OBJ_SCRATCH_MB")) mb = std::max(0LL, std::atoll(s));
    const long long cap = std::min<long long>(d.max_patterns, (mb << 20) / (long long)(sizeof(float2) * N2 * d.Nz));
    int occ3 = 0;
    if (cap > 0 &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ3, f3::k_fused3ms<true, true, 0>, 256, 0) == hipSuccess &&
        occ3 > 0) {
      int o2 = 0;
      for (auto kf : {f3::k_fused3ms<true, true, 2>, f3::k_fused3ms<true, false, 2>, f3::k_fused3ms<false, true, 0>,
                      f3::k_fused3ms<false, true, 2>, f3::k_fused3ms<false, false, 2>})
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o2, kf, 256, 0) == hipSuccess) occ3 = std::min(occ3, o2);
      pl->nwg3 = std::min(cu * occ3, std::max(1, d.max_patterns));
      constexpr long long div = 8;
      pl->seg_cap = pl->nwg3 + (cap + div - 1) / div;   // a call holds at most `cap` patterns
      if ((rc = dalloc(pl, &pl->ogscr, (size_t)cap * d.Nz * N2)) || (rc = dalloc(pl, &pl->bid, (size_t)d.max_patterns)) ||
          (rc = dalloc(pl, &pl->geo, (size_t)d.max_patterns)) || (rc = dalloc(pl, &pl->pcoef, (size_t)d.max_patterns)) ||
          (rc = dalloc(pl, &pl->fpk, N2)) || (rc = dalloc(pl, &pl->hpk, N2)) || (rc = dalloc(pl, &pl->bbox, 4)) ||
          (rc = dalloc(pl, &pl->oc, (size_t)d.Nz * d.Ny * d.Nx)) ||
          (rc = dalloc(pl, &pl->pref, (size_t)d.Nz * d.Ny * (d.Nx + 1))) ||
          (rc = dalloc(pl, &pl->preftot,
                       (size_t)d.Nz * ((d.Ny + f3::kPrefChunk - 1) / f3::kPrefChunk) * (d.Nx + 1))) ||
          (rc = dalloc(pl, &pl->segslab, (size_t)pl->seg_cap * N2)) ||
          (rc = dalloc(pl, &pl->segbid, (size_t)pl->seg_cap)) ||
          (rc = dalloc(pl, &pl->dsu, (size_t)d.max_patterns * 2)) ||
          (rc = dalloc(pl, &pl->segpart, (size_t)f3::kSegSplit * N2)) || (rc = alloc_bins(pl))) {
        free_plan(pl);
        return rc;
      }
      pl->og_cap = cap;
      pl->ms3 = true;
    }
  }
  // the per-slice loss_sparse window sums of small multislice calls (k_small_prep, use_zsum)
  if (pl->bbox && d.Nz > 1 && (rc = dalloc(pl, &pl->zsum, (size_t)f3::kSmallCall * d.Nz))) {
    free_plan(pl);
    return rc;
  }
  // input-error flags in host-mapped memory: the kernels set them (plain stores) and the next call
  // reads them without synchronising the stream
  e = hipHostMalloc(reinterpret_cast<void**>(&pl->err_host), sizeof(int) * kErrWords, hipHostMallocMapped);
  if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void**>(&pl->err_dev), pl->err_host, 0);
  if (e != hipSuccess) {
    free_plan(pl);
    return hip_fail(e, "hipHostMalloc(error flags)");
  }
  for (int k = 0; k < kErrWords; ++k) pl->err_host[k] = 0;
  // fp64 twiddles rounded once to fp32: tw[m] = exp(-2πi m/N)
  std::vector<float2> tw(d.N);
  for (int m = 0; m < d.N; ++m) {
    const double ang = -2.0 * M_PI * (double)m / (double)d.N;
    tw[m] = make_float2((float)std::cos(ang), (float)std::sin(ang));
  }
  e = hipMemcpy(pl->twg, tw.data(), sizeof(float2) * d.N, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    free_plan(pl);
    return hip_fail(e, "hipMemcpy twiddles");
  }
  *out = pl;
  return PTYX_OK;
}

extern "C" int ptyx_plan_destroy(ptyx_plan* plan) {
  if (!plan) return PTYX_OK;
  DeviceGuard dg(plan->device);
  free_plan(plan);
  return PTYX_OK;
}

// The input errors an earlier call's kernels flagged (check_pattern), reported once and cleared.
// Reads host memory the device writes: no stream synchronisation (a call still running reports at
// a later call, or at ptyx_plan_check after the caller synchronised).
static int take_error(ptyx_plan* pl) {
  volatile int* e = pl->err_host;
  if (!e || !(e[kErrIdx] | e[kErrWindow] | e[kErrRow])) return PTYX_OK;
  std::string msg = "invalid inputs in an earlier call on this plan:";
  if (e[kErrIdx]) msg += " a scan index outside [0, n_scans);";
  if (e[kErrWindow]) msg += " a window crop_pos + N outside the (Ny, Nx) object;";
  if (e[kErrRow]) msg += " a meas_rows entry outside [0, meas_row_count);";
  msg += " the kernels clamped them, so that call's results are not valid";
  for (int k = 0; k < kErrWords; ++k) e[k] = 0;
  return fail(PTYX_EINVAL, msg);
}

extern "C" int ptyx_plan_check(ptyx_plan* plan) {
  g_err.clear();
  if (!plan) return fail(PTYX_EINVAL, "plan is null");
  return take_error(plan);
}

static int check_inputs(const ptyx_plan* pl, const ptyx_inputs* in, bool need_meas) {
  if (!in) return fail(PTYX_EINVAL, "inputs is null");
  if (in->meas_rows && in->meas_row_count < 1)
    return fail(PTYX_EINVAL, "meas_row_count must give the rows of meas when meas_rows is set");
  if (!in->obja || !in->objp || !in->probe || !in->shifts || !in->omode_occu || !in->crop_pos)
    return fail(PTYX_EINVAL, "a required input pointer is null");
  if (pl->d.Nz > 1 && !in->H) return fail(PTYX_EINVAL, "H is required for Nz > 1");
  if (need_meas && !in->meas) return fail(PTYX_EINVAL, "meas is null");
  if (in->obj_tilts && !in->kvec) return fail(PTYX_EINVAL, "per-position tilts need kvec");
  return PTYX_OK;
}

static KArgs make_args(const ptyx_plan* pl, const ptyx_inputs* in, const int32_t* idx, int n_idx) {
  KArgs a{};
  const ptyx_dims& d = pl->d;
  a.P = d.P; a.O = d.O; a.Nz = d.Nz; a.Ny = d.Ny; a.Nx = d.Nx; a.n_scans = d.n_scans;
  a.shift = (d.flags & PTYX_SHIFT_PROBES) ? 1 : 0;
  a.meas_f16 = (d.flags & PTYX_MEAS_F16) ? 1 : 0;
  a.obja = in->obja; a.objp = in->objp;
  a.probe = reinterpret_cast<const float2*>(in->probe);
  a.Fp = pl->Fp;
  a.shifts = in->shifts; a.crop = in->crop_pos;
  a.H = reinterpret_cast<const float2*>(in->H);
  a.occu = in->omode_occu; a.meas = in->meas;
  a.ptilt = in->obj_tilts; a.kvec = in->kvec; a.dz = in->dz;
  a.mrow = in->meas_rows;
  a.mrows = in->meas_rows ? in->meas_row_count : d.n_scans;
  a.err = pl->err_dev;
  a.idx = idx; a.n_idx = n_idx;
  a.Ibuf = pl->Ibuf;
  a.slab = pl->slab; a.scratch = pl->scratch; a.scratch_stride = pl->scratch_stride;
  a.twg = pl->twg;
  a.FpT = pl->FpT;
  a.HT = pl->HT;
  return a;
}

static void launch_spectrum(const ptyx_plan* pl, const KArgs& a, hipStream_t st) {
  ProfScope ps(pl, kKSpectrum, st);
  pl->gen->spectrum(a, pl->d.P + (a.HT ? 1 : 0), pl->Fp, st);
}
static void launch_forward(const ptyx_plan* pl, const KArgs& a, hipStream_t st) {
  ProfScope ps(pl, kKForward, st);
  const int grid = std::max(1, std::min(a.n_idx * a.msplit, pl->nwg));
  const ptyx_dims& d = pl->d;
  pl->gen->forward(a, grid, d.P * d.O == 1, d.P * d.O * d.Nz == 1, st);
}
static void launch_modesum(const ptyx_plan* pl, const KArgs& a, hipStream_t st) { pl->gen->modesum(a, st); }
// k_adjoint's grid: every workgroup zeroes its slab, so all of them run — except with compact
// slabs, where the grid is the split call's jobs (or the plan's workgroups) rounded down to a
// multiple of P and k_slab_reduce sums grid / P slabs
static int adjoint_grid(const ptyx_plan* pl, const KArgs& a) {
  if (!a.cslab) return pl->nwg;
  return std::max(a.P, std::min(pl->nwg, a.n_idx * a.P) / a.P * a.P);
}
static int adjoint_slabs(const ptyx_plan* pl, const KArgs& a) { return a.cslab ? adjoint_grid(pl, a) / a.P : pl->nwg; }

static void launch_adjoint(const ptyx_plan* pl, const KArgs& a, hipStream_t st, bool ext) {
  ProfScope ps(pl, kKAdjoint, st);
  const ptyx_dims& d = pl->d;
  pl->gen->adjoint(a, adjoint_grid(pl, a), d.P * d.O == 1, d.P * d.O * d.Nz == 1, ext, st);
}
// d_probe += F⁻¹(G) of the probe modes [0, np) from G (k_probe_finalize)
static void launch_probe_fin(const ptyx_plan* pl, const KArgs& a, hipStream_t st, float* d_probe, int np) {
  ProfScope ps(pl, kKProbeFinalize, st);
  pl->gen->probe_finalize(a, np, pl->Gsum, reinterpret_cast<float2*>(d_probe), st);
}
// The register engines' form: with shifted probes the inverse transform as two multi-workgroup
// launches (k_lines_rows / k_lines_cols; the general engine's slab as scratch, unused by them)
static void launch_probe_fin_reg(const ptyx_plan* pl, const KArgs& a, hipStream_t st, float* d_probe, int np) {
  if (!a.shift) {
    launch_probe_fin(pl, a, st, d_probe, np);
    return;
  }
  ProfScope ps(pl, kKProbeFinalize, st);
  pl->gen->probe_finalize_lines(pl->Gsum, np, reinterpret_cast<float2*>(d_probe), pl->slab, pl->twg, st);
}
static void launch_probe_finalize(const ptyx_plan* pl, const KArgs& a, hipStream_t st, float* d_probe,
                                  int n_slabs) {
  const long long per = (long long)pl->d.P * pl->d.N * pl->d.N;
  const int tb = 256;
  {
    ProfScope ps(pl, kKSlabReduce, st);
    hipLaunchKernelGGL(k_slab_reduce, dim3((unsigned)((per + tb - 1) / tb)), dim3(tb), 0, st, pl->slab, n_slabs,
                       per, pl->Gsum);
  }
  launch_probe_fin(pl, a, st, d_probe, pl->d.P);
}

// shared with the other translation units of libptyx.so (ptyx_abi.hpp)
namespace ptyx {
namespace abi {
void clear_error() { g_err.clear(); }
int fail(int code, const std::string& msg) { return ::fail(code, msg); }
int launch_status(const char* what) { return ::launch_status(what); }
}  // namespace abi
}  // namespace ptyx

// ---------------------------------------------------------------- k_fused3 path (N = 128)
// Launch sequence of one ptyx_forward_loss_grad call on the register-resident engine.
// ptyx_forward_loss_grad_begin / _end phases of one call (kPhaseAll: both, with the call's own sums)
enum CallPhase { kPhaseAll = 0, kPhaseBegin = 1, kPhaseEnd = 2 };
enum EngineKind { kEngTwoPass = 0, kEngFused3 = 1, kEngStripe = 2, kEngFmm = 3 };

// Preparation shared by the register engines (k_fused3 / k_fused3ms / k_fmm_*): F(P) packed for
// every probe mode (or the probes R-packed), H/N² packed, the call's bounding box, O = A e^{iφ}
// and the loss_sparse tables, the pattern table; the segment table (nseg ids) cleared.
static int register_prep(ptyx_plan* pl, const ptyx_inputs* in, const KArgs& a, const ptyx_loss_cfg* cfg,
                         hipStream_t st, int nseg) {
  constexpr int N = 128, N2 = N * N;
  const ptyx_dims& d = pl->d;
  const bool sparse = cfg->sparse_on != 0;
  const int Nz = d.Nz;
  const bool reuse = cfg->prep == PTYX_PREP_REUSE;   // object / probe / H prepared by the previous call
  pl->zsum_call = false;
  // small calls (one mini-batch per optimizer step): one-workgroup bbox that also clears the
  // segment table, and direct loss_sparse window sums instead of the summed-area table; the
  // probe spectrum's row pass and the H packing ride in the same launch (PrepExtra)
  const bool small = a.n_idx <= f3::kSmallCall && pl->bbox;
  const bool merged = small && cfg->prep == PTYX_PREP_CALL;
  if (reuse) {
  } else if (a.shift) {   // F(P_p), natural and K-packed: rows then columns, N/8 workgroups a mode each
    if (!merged) {
      ProfScope ps(pl, kKSpectrum, st);
      pl->gen->spectrum_lines(a.probe, d.P, pl->Fp, pl->fpk, pl->Gsum, pl->twg, st);
    }
  } else {
    ProfScope ps(pl, kKPack, st);
    hipLaunchKernelGGL(f3::k_pack128<false>, dim3(N2 / 256, d.P), dim3(256), 0, st,
                       reinterpret_cast<const float2*>(in->probe), pl->fpk);
  }
  if (Nz > 1 && !reuse && !merged) {
    ProfScope ps(pl, kKPack, st);
    hipLaunchKernelGGL(f3::k_pack128<true>, dim3(N2 / 256), dim3(256), 0, st, a.H, pl->hpk, 1.0f / N2);   // H/N²
  }
  const bool direct_sums = sparse && small && cfg->prep == PTYX_PREP_CALL;
  if (merged) {   // table, object rows, bbox (+ probe rows, H packing): one launch (k_small_prep)
    f3::PrepExtra ex;
    if (a.shift) {
      ex.probe = a.probe;
      ex.P = d.P;
      ex.tmp = pl->Gsum;
      ex.twg = pl->twg;
      if (g_tuning[kTuneSmallSpec] != 0) ex.fpk = pl->fpk;   // the whole spectrum in this launch
    }
    if (pl->sel_fold) {   // PTYX_PREP_SELECT: the step's indices, gradient zeroing and step counts here
      ex.sel_all = pl->sel_all;
      ex.sel_start = pl->sel_start;
      ex.sel_cnt = pl->sel_cnt;
      ex.sel_out = const_cast<int32_t*>(a.idx);
      ex.zero = pl->sel_grad;
      ex.zero_n = pl->sel_grad_n;
      ex.steps = pl->sel_steps;
      ex.n_steps = pl->sel_n_steps;
    }
    if (Nz > 1) {
      ex.H = a.H;
      ex.hpk = pl->hpk;
      ex.hscale = 1.0f / N2;
    }
    if (sparse && Nz > 1 && pl->zsum) {   // the window sums one (pattern, slice) a workgroup
      ex.zsum = pl->zsum;
      pl->zsum_call = true;
    }
    {
      ProfScope ps(pl, kKTable, st);
      const dim3 gr(ex.lead_blocks() + ex.sel_blocks() + f3::small_prep_blocks(a.n_idx, Nz, d.Ny, ex.zsum != nullptr) +
                    ex.row_blocks() + ex.h_blocks()),
          bl(256);
      const f3::TableCheck tc{a.err, a.mrow, a.mrows};
      if (sparse)
        hipLaunchKernelGGL(f3::k_small_prep<true>, gr, bl, 0, st, a.idx, a.n_idx, a.boff, a.n_batches, a.crop,
                           a.n_scans, d.Ny, d.Nx, pl->bid, pl->geo, a.obja, a.objp, cfg->sparse_n, pl->psums, Nz, tc,
                           pl->oc, pl->bbox, pl->segbid, nseg, ex);
      else
        hipLaunchKernelGGL(f3::k_small_prep<false>, gr, bl, 0, st, a.idx, a.n_idx, a.boff, a.n_batches, a.crop,
                           a.n_scans, d.Ny, d.Nx, pl->bid, pl->geo, a.obja, a.objp, cfg->sparse_n, pl->psums, Nz, tc,
                           pl->oc, pl->bbox, pl->segbid, nseg, ex);
    }
    if (a.shift && !ex.fpk) {   // the spectrum's column pass (Fp natural, fpk K-packed)
      ProfScope ps(pl, kKSpectrum, st);
      pl->gen->spectrum_cols(pl->Gsum, d.P, pl->Fp, pl->fpk, pl->twg, st);
    }
    return launch_status("register engine preparation (small call)");
  }
  if (small) {
    ProfScope ps(pl, kKTable, st);
    hipLaunchKernelGGL(f3::k_bbox_small, dim3(1), dim3(256), 0, st, a.idx, a.n_idx, a.crop, a.n_scans, d.Ny, d.Nx,
                       pl->bbox, 128, pl->segbid, nseg);
  } else if (pl->bbox) {   // rows / tiles outside the call's windows are skipped (a rank's shard of a
                           // multi-GPU scan touches only its band of the replicated object)
    ProfScope ps(pl, kKTable, st);
    hipLaunchKernelGGL(f3::k_bbox_init, dim3(1), dim3(64), 0, st, pl->bbox);
    hipLaunchKernelGGL(f3::k_bbox, dim3(std::max(1, std::min(f3::kBboxBlocks, (a.n_idx + 255) / 256))), dim3(256), 0, st, a.idx, a.n_idx, a.crop, a.n_scans,
                       d.Ny, d.Nx, pl->bbox);
  }
  if (!reuse) {
    ProfScope ps(pl, kKObjPrep, st);   // (Nz, Ny) rows: every slice's O and |φ|^n prefix sums
    hipLaunchKernelGGL(f3::k_obj_prep, dim3(d.Ny * Nz), dim3(256), 0, st, a.obja, a.objp, d.Ny * Nz, d.Nx, pl->oc,
                       sparse && !direct_sums ? pl->pref : nullptr, cfg->sparse_n,
                       cfg->prep == PTYX_PREP_FULL ? nullptr : pl->bbox, d.Ny, 128);
    if (sparse && !direct_sums) {   // row prefix sums → summed-area table (k_pattern_table3's window sums)
      const int* bb = cfg->prep == PTYX_PREP_FULL ? nullptr : pl->bbox;
      const dim3 gp((d.Nx + 1 + 255) / 256, (d.Ny + f3::kPrefChunk - 1) / f3::kPrefChunk, Nz);
      hipLaunchKernelGGL(f3::k_pref_cols1, gp, dim3(256), 0, st, pl->pref, pl->preftot, d.Ny, d.Nx, bb, 128);
      hipLaunchKernelGGL(f3::k_pref_cols2, gp, dim3(256), 0, st, pl->pref, pl->preftot, d.Ny, d.Nx, bb, 128);
    }
  }
  {
    // (the table's first row: the bbox of the call that prepared it, PTYX_PREP_CALL only)
    ProfScope ps(pl, kKTable, st);
    if (direct_sums)
      hipLaunchKernelGGL(f3::k_pattern_table_direct, dim3(a.n_idx), dim3(256), 0, st, a.idx, a.n_idx, a.boff,
                         a.n_batches, a.crop, a.n_scans, d.Ny, d.Nx, pl->bid, pl->geo, a.objp, cfg->sparse_n,
                         pl->psums, Nz, f3::TableCheck{a.err, a.mrow, a.mrows});
    else
      hipLaunchKernelGGL(f3::k_pattern_table3, dim3((a.n_idx + 3) / 4), dim3(256), 0, st, a.idx, a.n_idx, a.boff,
                         a.n_batches, a.crop, a.n_scans, d.Ny, d.Nx, pl->bid, pl->geo, sparse ? pl->pref : nullptr,
                         pl->psums, Nz, cfg->prep == PTYX_PREP_CALL ? pl->bbox : nullptr,
                         f3::TableCheck{a.err, a.mrow, a.mrows});
  }
  if (!small) {
    int rc0 = fill32(pl->segbid, nseg, 0xFFFFFFFFu, st);
    if (rc0) return rc0;
  }
  return launch_status("register engine preparation");
}

// The register engines' argument block.
static f3::F3Args register_args(const ptyx_plan* pl, const ptyx_inputs* in, const KArgs& a, const ptyx_loss_cfg* cfg,
                                const ptyx_grads& gz) {
  const ptyx_dims& d = pl->d;
  const bool single = cfg->single_on != 0;
  f3::F3Args f{};
  f.n_idx = a.n_idx; f.n_scans = a.n_scans; f.Ny = d.Ny; f.Nx = d.Nx;
  f.idx = a.idx; f.bid = pl->bid; f.geo = pl->geo; f.shifts = a.shifts;
  f.fpk = pl->fpk; f.oc = pl->oc; f.meas = reinterpret_cast<const float*>(a.meas); f.mrow = a.mrow; f.mrows = a.mrows;
  f.occp = in->omode_occu;
  f.q = single ? cfg->single_q : cfg->poissn_q;
  f.eps2 = cfg->poissn_eps;
  f.psums = pl->psums;
  f.slots = pl->use_tgt ? reinterpret_cast<float2*>(pl->slot_tgt) : pl->ogscr; f.segslab = pl->segslab; f.segbid = pl->segbid; f.dsu = pl->dsu;
  f.tail = (gz.d_probe != nullptr || (a.shift && gz.d_shifts != nullptr)) ? 1 : 0;
  f.dp_out = a.dp_out;
  f.Nz = d.Nz;
  f.hpk = pl->hpk;
  f.q2 = cfg->poissn_q;
  f.coef = pl->coef;
  return f;
}

// k_fused3 with both data terms: MODE 1 (forward + both terms' sums) before k_finalize, MODE 2
// (the full pass with the mini-batch coefficients) after it
static void launch_fused3_both(const ptyx_plan* pl, const f3::F3Args& f, bool shift, int mode, int G, hipStream_t st) {
  ProfScope ps(pl, kKFused, st);
  const dim3 gr(G), bl(256);
  const bool half = f.q == 0.5f;
  const bool ms = f.Nz > 1;   // k_fused3ms
#define PTYX_F3B(SH, QM, MD)                                                               \
  do {                                                                                     \
    if (ms) hipLaunchKernelGGL((f3::k_fused3ms<SH, true, QM, MD>), gr, bl, 0, st, f);     \
    else hipLaunchKernelGGL((f3::k_fused3<SH, true, QM, MD>), gr, bl, 0, st, f);          \
  } while (0)
  if (mode == 1) {
    if (shift) { if (half) PTYX_F3B(true, 0, 1); else PTYX_F3B(true, 2, 1); }
    else { if (half) PTYX_F3B(false, 0, 1); else PTYX_F3B(false, 2, 1); }
  } else {
    if (shift) { if (half) PTYX_F3B(true, 0, 2); else PTYX_F3B(true, 2, 2); }
    else { if (half) PTYX_F3B(false, 0, 2); else PTYX_F3B(false, 2, 2); }
  }
#undef PTYX_F3B
}

// k_fused3's workgroups for a call: nwg3 (two a CU) — or, with tuning psi_hold 2 (an A/B switch for
// large calls), one a CU so that every call runs the register-held ψ⁰ variant
static bool fused3_force_hold(const ptyx_plan* pl, const KArgs& a, const ptyx_loss_cfg* cfg) {
  return g_tuning[kTunePsiHold] == 2 && pl->d.Nz == 1 && a.shift && !(cfg->single_on && cfg->poissn_on);
}
static int fused3_groups(const ptyx_plan* pl, const KArgs& a, const ptyx_loss_cfg* cfg) {
  const int cap = fused3_force_hold(pl, a, cfg) ? std::min(pl->nwg3, pl->n_cu) : pl->nwg3;
  return std::max(1, std::min(cap, a.n_idx));
}

// Preparation, pattern table and the k_fused3 / k_fused3ms pass (everything before k_finalize).
static int fused3_pass(ptyx_plan* pl, const ptyx_inputs* in, const KArgs& a, const ptyx_loss_cfg* cfg,
                       const ptyx_grads& gz, hipStream_t st) {
  const int Nz = pl->d.Nz;                 // > 1: k_fused3ms (multislice)
  const int G = fused3_groups(pl, a, cfg);
  const int nseg = a.n_batches + G;
  int rc = register_prep(pl, in, a, cfg, st, nseg);
  if (rc) return rc;
  const bool single = cfg->single_on != 0;
  const f3::F3Args f = register_args(pl, in, a, cfg, gz);
  if (cfg->single_on && cfg->poissn_on) {
    launch_fused3_both(pl, f, a.shift, 1, G, st);
  } else if (Nz > 1) {
    ProfScope ps(pl, kKFused, st);
    const dim3 gr(G), bl(256);
    const bool half = single && f.q == 0.5f;
    if (a.shift) {
      if (half) hipLaunchKernelGGL((f3::k_fused3ms<true, true, 0>), gr, bl, 0, st, f);
      else if (single) hipLaunchKernelGGL((f3::k_fused3ms<true, true, 2>), gr, bl, 0, st, f);
      else hipLaunchKernelGGL((f3::k_fused3ms<true, false, 2>), gr, bl, 0, st, f);
    } else {
      if (half) hipLaunchKernelGGL((f3::k_fused3ms<false, true, 0>), gr, bl, 0, st, f);
      else if (single) hipLaunchKernelGGL((f3::k_fused3ms<false, true, 2>), gr, bl, 0, st, f);
      else hipLaunchKernelGGL((f3::k_fused3ms<false, false, 2>), gr, bl, 0, st, f);
    }
  } else {
    ProfScope ps(pl, kKFused, st);
    const dim3 gr(G), bl(256);
    const bool half = single && f.q == 0.5f;   // dp_pow 1/2 (the schema default): sqrt / rsqrt form
    // at most one workgroup a CU (the default cadence's small calls): ψ⁰ may stay in registers
    // (measured: c2 at ga = 1 0.1099 → 0.1080 ms a step, profiles/r06/psi_hold/; tuning psi_hold 0 parks)
    const bool hold = (G <= pl->n_cu && g_tuning[kTunePsiHold] != 0) || fused3_force_hold(pl, a, cfg);
    if (a.shift) {
      if (half && hold) hipLaunchKernelGGL((f3::k_fused3<true, true, 0, 0, true>), gr, bl, 0, st, f);
      else if (single && hold) hipLaunchKernelGGL((f3::k_fused3<true, true, 2, 0, true>), gr, bl, 0, st, f);
      else if (hold) hipLaunchKernelGGL((f3::k_fused3<true, false, 2, 0, true>), gr, bl, 0, st, f);
      else if (half) hipLaunchKernelGGL((f3::k_fused3<true, true, 0>), gr, bl, 0, st, f);
      else if (single) hipLaunchKernelGGL((f3::k_fused3<true, true, 2>), gr, bl, 0, st, f);
      else hipLaunchKernelGGL((f3::k_fused3<true, false, 2>), gr, bl, 0, st, f);
    } else {
      if (half) hipLaunchKernelGGL((f3::k_fused3<false, true, 0>), gr, bl, 0, st, f);
      else if (single) hipLaunchKernelGGL((f3::k_fused3<false, true, 2>), gr, bl, 0, st, f);
      else hipLaunchKernelGGL((f3::k_fused3<false, false, 2>), gr, bl, 0, st, f);
    }
  }
  return launch_status("k_fused3 launch");
}

// PTYX_PREP_FUSED_ADAM: k_gather_adam's arguments for a small single-slice k_fused3 call, or false
// (then the call runs its ordinary epilogue and the registered step is a k_adam launch after it).
// The Adam tensors that ARE obja / objp (parameter = the call's object, gradient = its d_obja /
// d_objp) take their step in the tile blocks, the probe's in the probe-row blocks; every other
// tensor must fit one k_adam launch and must not overlap what those blocks write.
// (probe_rows: the probe gradient's row pass is part of the launch; else it is final before it)
static bool fused_adam_setup(const ptyx_plan* pl, const float* obja, const float* objp, const float* probe,
                             const ptyx_grads& gz, bool probe_rows, const GatherArgs& g, int tiles, FusedAdamArgs* f) {
  constexpr int N = 128;
  const ptyx_dims& d = pl->d;
  if (d.O != 1) return false;
  const int64_t nobj = (int64_t)d.Nz * d.Ny * d.Nx, nprobe = 2LL * N * N * d.P;
  probe_rows = probe_rows && gz.d_probe;
  *f = FusedAdamArgs{};
  f->ga = g;
  f->h = pl->fadam_h;
  f->ptiles = tiles;       // (per object plane)
  f->tiles = tiles * d.Nz;
  std::vector<opt::AdamTensor> rest;
  struct Span {
    uintptr_t lo, hi;
  };
  std::vector<Span> owned;   // what the tile / probe blocks read or write
  const auto span = [](const void* p, int64_t n) {
    const uintptr_t lo = reinterpret_cast<uintptr_t>(p);
    return Span{lo, lo + (uintptr_t)(4 * n)};
  };
  owned.push_back(span(obja, nobj));
  owned.push_back(span(objp, nobj));
  if (gz.d_obja) owned.push_back(span(gz.d_obja, nobj));
  if (gz.d_objp) owned.push_back(span(gz.d_objp, nobj));
  if (probe_rows) owned.push_back(span(gz.d_probe, nprobe));
  for (const opt::AdamTensor& t : pl->fadam_ts) {
    if (!t.numel) continue;
    int plane = -1;
    if (t.numel == nobj && gz.d_obja && t.g == gz.d_obja && t.p == obja) plane = 0;
    else if (t.numel == nobj && gz.d_objp && t.g == gz.d_objp && t.p == objp) plane = 1;
    if (plane >= 0) {
      if (f->om[plane]) return false;   // (the same tensor twice)
      f->op[plane] = t.p; f->om[plane] = t.m; f->ov[plane] = t.v; f->ostep[plane] = t.step; f->olr[plane] = t.lr;
      owned.push_back(span(t.m, nobj));
      owned.push_back(span(t.v, nobj));
      continue;
    }
    if (probe_rows && t.numel == nprobe && t.g == gz.d_probe && t.p == probe) {
      if (f->pp) return false;
      f->pp = t.p; f->pm = t.m; f->pv = t.v; f->pstep = t.step; f->plr = t.lr;
      owned.push_back(span(t.p, nprobe));
      owned.push_back(span(t.m, nprobe));
      owned.push_back(span(t.v, nprobe));
      continue;
    }
    rest.push_back(t);
  }
  for (const opt::AdamTensor& t : rest)
    for (const void* q : {(const void*)t.p, (const void*)t.g, (const void*)t.m, (const void*)t.v}) {
      const Span r = span(q, t.numel);
      for (const Span& o : owned)
        if (r.lo < o.hi && o.lo < r.hi) return false;
    }
  const std::vector<opt::AdamArgs> packs = opt::adam_pack(rest, f->h);
  if (packs.size() > 1) return false;
  if (!packs.empty()) {
    f->rest = packs[0];
    f->rblocks = (int)std::max<int64_t>(1, std::min<int64_t>(4096, f->rest.off[f->rest.nt] / opt::kChunk));
  } else {
    f->rest.h = f->h;
  }
  if (pl->fadam_store) opt::adam_set_store(f->rest, pl->fadam_ss);
  f->lead = g_tuning[kTuneGadamLead] != 0 ? 1 : 0;
  if (probe_rows) {
    f->pblocks = N / f3::kPrLinesT * d.P;
    f->ptmp = pl->slab;
    f->d_probe = reinterpret_cast<float2*>(gz.d_probe);
    f->twg = pl->twg;
  }
  return true;
}

static int run_fused3(ptyx_plan* pl, const ptyx_inputs* in, const KArgs& a, const ptyx_loss_cfg* cfg,
                      const ptyx_grads& gz, hipStream_t st, float* loss_terms, int ph, double* bsums) {
  constexpr int N = 128, N2 = N * N;
  const ptyx_dims& d = pl->d;
  const bool sparse = cfg->sparse_on != 0;
  const int Nz = d.Nz;
  const bool single = cfg->single_on != 0;
  const bool both = single && cfg->poissn_on;               // k_fused3 / k_fused3ms MODE 1 / 2
  const int ci = both ? 2 : single ? 0 : 1;                // (2: the kernel applies the coefficients)
  const int G = fused3_groups(pl, a, cfg);
  const int nseg = a.n_batches + G;
  int rc = PTYX_OK;
  if (ph != kPhaseEnd && (rc = fused3_pass(pl, in, a, cfg, gz, st))) return rc;
  // small calls: every tile scans the call's few patterns directly (no binning launches)
  const bool bins = a.n_idx > f3::kSmallCall;
  // PTYX_PREP_DEFER_GATHER: the slots, pattern table and coefficients stay for ptyx_slots_export
  // and the caller's ptyx_obj_gather_slots over every rank's patterns (split mini-batches)
  const bool gather_here = (gz.d_obja || gz.d_objp) && !pl->gather_deferred;
  GatherArgs g{};
  int tiles = 0;
  bool sparse_tiles = false;
  if (gather_here) {
    g.ogscr = pl->ogscr; g.geo = pl->geo; g.pcoef = pl->pcoef; g.n = a.n_idx;
    g.boff = bins ? pl->boff : nullptr;
    g.blist = bins ? pl->blist : nullptr;
    g.Ny = d.Ny; g.Nx = d.Nx; g.tiles_x = (d.Nx + kGTX - 1) / kGTX; g.sparse_n = sparse ? cfg->sparse_n : 1;
    g.obja = a.obja; g.objp = a.objp; g.d_obja = gz.d_obja; g.d_objp = gz.d_objp;
    tiles = g.tiles_x * ((d.Ny + kGTY - 1) / kGTY);
    // fewer than 64 candidates per tile on average (c4's 8,192-pattern calls over 13,340 tiles:
    // ≈ 17): 4 waves a tile instead of kGWaves
    sparse_tiles = (long long)a.n_idx * BinReach<N>::n < 64LL * tiles;
    g.nz = Nz;
    g.bbox = pl->bbox;   // also for Nz = 1
    g.zgrid = 1;         // every slice plane in one launch (blockIdx.y = slice)
    g.store = pl->grad_store;
  }
  // PTYX_PREP_FUSED_ADAM on a small single-slice call: the gather, the probe rows and the optimizer
  // step in one launch after the probe / position sums (ptyx_stepfuse.hpp)
  float* d_shifts = a.shift ? gz.d_shifts : nullptr;
  FusedAdamArgs fz{};
  // (the gather's form and order as launch_gather would run it unfused)
  const int gform = gather_form(false, a.n_idx);
  const bool rows_fuse = gform >= 1;
  const bool fuse = ph == kPhaseAll && pl->fadam_on && gather_here && !bins && Nz == 1 && sparse_tiles &&
                    g_tuning[kTuneFuseAdam] != 0 &&
                    fused_adam_setup(pl, a.obja, a.objp, in->probe, gz, a.shift, g, tiles, &fz);
  // k_finalize folded into the small call's tail launch when nothing between them needs the
  // coefficients (one data term; the object gather, if any, after the tail: k_gather_adam)
  const bool tail_small = !bins && (gz.d_probe || d_shifts);
  const bool fold_fin = ph == kPhaseAll && !both && tail_small && a.n_batches <= kTailFinBatches &&
                        (fuse || !gather_here) && g_tuning[kTuneTailFin] != 0;
  FinArgs fa{};
  fa.boff = a.boff; fa.n_batches = a.n_batches; fa.N = N; fa.Nz = Nz; fa.O = 1;
  fa.psums = pl->psums; fa.occu = in->omode_occu;
  if (pl->zsum_call) {   // the sparse sums as per-slice partials (k_small_prep)
    fa.zsum = pl->zsum;
    fa.zNz = Nz;
  }
  fa.single_on = cfg->single_on; fa.pois_on = cfg->poissn_on; fa.sparse_on = cfg->sparse_on;
  fa.sparse_n = cfg->sparse_n; fa.w1 = cfg->single_w; fa.w2 = cfg->poissn_w; fa.ws = cfg->sparse_w;
  fa.grad_scale = cfg->grad_scale; fa.coef = pl->coef; fa.loss_terms = loss_terms;
  if (gz.d_obja || gz.d_objp) {
    fa.pcoef = pl->pcoef;
    fa.ci = ci;
  }
  fa.bsums_out = ph == kPhaseBegin ? bsums : nullptr;
  fa.bsums_in = ph == kPhaseEnd ? bsums : nullptr;
  if (!fold_fin) {
    ProfScope ps(pl, kKFinalize, st);
    hipLaunchKernelGGL(k_finalize, dim3((a.n_batches + kFinWaves - 1) / kFinWaves), dim3(64 * kFinWaves), 0, st, fa);
  }
  if ((rc = launch_status("k_finalize launch")) || ph == kPhaseBegin) return rc;
  if (both) {   // the adjoint pass, now that the coefficients are known (dp_out written by MODE 1)
    f3::F3Args f = register_args(pl, in, a, cfg, gz);
    f.dp_out = nullptr;
    launch_fused3_both(pl, f, a.shift, 2, G, st);
    if ((rc = launch_status("k_fused3 (both terms) launch"))) return rc;
  }
  if (gather_here && bins) {
    // candidate bins of the gather: the patterns by object tile of their window origin
    ProfScope ps(pl, kKTable, st);
    const int tiles_x = (d.Nx + kGTX - 1) / kGTX;
    if (int rc2 = fill32(pl->bcnt, pl->nbins, 0u, st)) return rc2;
    const dim3 gn((a.n_idx + 255) / 256);
    hipLaunchKernelGGL(k_bin_count, gn, dim3(256), 0, st, pl->geo, a.n_idx, tiles_x, pl->bcnt, pl->bkey);
    hipLaunchKernelGGL(k_bin_scan, dim3(1), dim3(1024), 0, st, pl->bcnt, pl->nbins, pl->boff, pl->bcur);
    hipLaunchKernelGGL(k_bin_fill, gn, dim3(256), 0, st, pl->bkey, a.n_idx, pl->bcur, pl->blist);
    hipLaunchKernelGGL(k_bin_sort, dim3(pl->nbins), dim3(256), 0, st, pl->boff, pl->blist);
  }
  if (gather_here && !fuse) {
    ProfScope ps(pl, kKGather, st);
    launch_gather<N, true, false>(pl, g, tiles, Nz, sparse_tiles, st);
  }
  if ((rc = launch_status("k_obj_gather launch"))) return rc;
  if (!bins && (gz.d_probe || d_shifts)) {   // small call: one launch for the probe / position sums
    {
      ProfScope ps(pl, kKSlabReduce, st);
      const dim3 gr(N2 / 256 + (d_shifts ? (a.n_idx + 255) / 256 : 0));
      const dim3 grf(gr.x + 1);   // (+ k_small_tail_fin's finalize workgroup)
      float2* out = gz.d_probe ? pl->Gsum : nullptr;
      if (fold_fin && a.shift)
        hipLaunchKernelGGL(k_small_tail_fin<true>, grf, dim3(256), 0, st, fa, pl->segslab, pl->segbid, nseg, ci, out,
                           a.idx, a.n_idx, a.n_scans, pl->bid, pl->dsu, d_shifts, pl->twg,
                           gz.d_probe ? pl->slab : nullptr);
      else if (fold_fin)
        hipLaunchKernelGGL(k_small_tail_fin<false>, grf, dim3(256), 0, st, fa, pl->segslab, pl->segbid, nseg, ci, out,
                           a.idx, a.n_idx, a.n_scans, pl->bid, pl->dsu, d_shifts, nullptr, nullptr);
      else if (a.shift)   // (with the probe gradient: its column IFFT in the same launch, into pl->slab)
        hipLaunchKernelGGL(f3::k_small_tail<true>, gr, dim3(256), 0, st, pl->segslab, pl->segbid, nseg, pl->coef, ci,
                           out, a.idx, a.n_idx, a.n_scans, pl->bid, pl->dsu, d_shifts, pl->twg,
                           gz.d_probe ? pl->slab : nullptr);
      else
        hipLaunchKernelGGL(f3::k_small_tail<false>, gr, dim3(256), 0, st, pl->segslab, pl->segbid, nseg, pl->coef, ci,
                           out, a.idx, a.n_idx, a.n_scans, pl->bid, pl->dsu, d_shifts, nullptr, nullptr);
    }
    if (gz.d_probe && a.shift) {
      if (!fuse) {
        ProfScope ps(pl, kKProbeFinalize, st);
        hipLaunchKernelGGL(f3::k_probe_rows_acc, dim3(N / f3::kPrLinesT, 1), dim3(256), 0, st, pl->slab,
                           reinterpret_cast<float2*>(gz.d_probe), pl->twg);
      }
    } else if (gz.d_probe) {
      launch_probe_fin_reg(pl, a, st, gz.d_probe, 1);
    }
    if ((rc = launch_status("probe finalize launch"))) return rc;
  }
  if (fuse) {
    ProfScope ps(pl, kKGatherAdam, st);
    const dim3 gr(fz.tiles + fz.pblocks + fz.rblocks);
    if (gform == 3) hipLaunchKernelGGL((k_gather_adam_r5<N>), gr, dim3(256), 0, st, fz);
    else if (gform == 2) hipLaunchKernelGGL((k_gather_adam_r4<N>), gr, dim3(256), 0, st, fz);
    else if (rows_fuse) hipLaunchKernelGGL((k_gather_adam<N, true, true, 1, false>), gr, dim3(256), 0, st, fz);
    else hipLaunchKernelGGL((k_gather_adam<N, true>), gr, dim3(256), 0, st, fz);
    pl->fadam_done = true;
    return launch_status("k_gather_adam launch");
  }
  if (!bins && (gz.d_probe || d_shifts)) return PTYX_OK;
  if (d_shifts) {
    ProfScope ps(pl, kKSlabReduce, st);
    hipLaunchKernelGGL(f3::k_shift_apply, dim3((a.n_idx + 255) / 256), dim3(256), 0, st, a.idx, a.n_idx, a.n_scans,
                       pl->bid, pl->coef, ci, pl->dsu, gz.d_shifts);
  }
  if (gz.d_probe) {
    {
      ProfScope ps(pl, kKSlabReduce, st);
      hipLaunchKernelGGL(f3::k_segslab_reduce, dim3(N2 / 256, f3::kSegSplit), dim3(256), 0, st, pl->segslab,
                         pl->segbid, nseg, pl->coef, ci, pl->segpart);
      if (a.shift)
        hipLaunchKernelGGL(f3::k_segslab_final<true>, dim3(N2 / 256), dim3(256), 0, st, pl->segpart, pl->Gsum);
      else
        hipLaunchKernelGGL(f3::k_segslab_final<false>, dim3(N2 / 256), dim3(256), 0, st, pl->segpart, pl->Gsum);
    }
    launch_probe_fin_reg(pl, a, st, gz.d_probe, 1);
  }
  if ((rc = launch_status("probe finalize launch"))) return rc;
  return PTYX_OK;
}

// ---------------------------------------------------------------- mixed-state register engine
// (N = 128, P > 1, O = 1; ptyx_fmm.hpp): k_fmm_fwd → k_fmm_loss → k_finalize → k_fmm_adj, then the
// object gather over the P mode planes of each slice and the per-mode probe / position reductions.
static int run_fmm(ptyx_plan* pl, const ptyx_inputs* in, const KArgs& a, const ptyx_loss_cfg* cfg,
                   const ptyx_grads& gz, hipStream_t st, float* loss_terms, int ph, double* bsums) {
  constexpr int N = 128, N2 = N * N;
  const ptyx_dims& d = pl->d;
  const int P = d.P, Nz = d.Nz;
  const bool single = cfg->single_on != 0;
  const int ci = single ? 0 : 1;
  const int nj = a.n_idx * P;
  const int G = std::max(1, std::min(pl->nwg3, nj));
  const int nseg = P + G;
  // at most one workgroup a CU (the default cadence's small calls): H/N² held in registers
  const bool holdh = Nz > 1 && G <= pl->n_cu && g_tuning[kTuneFmmHoldH] != 0;
  const bool both = cfg->single_on && cfg->poissn_on;
  f3::FmArgs m{};
  m.f = register_args(pl, in, a, cfg, gz);
  m.f.slots = pl->ffc;
  m.P = P;
  m.pstride = (long long)P * (Nz + 1);
  m.ubuf = pl->Ibuf;
  m.ubuf2 = both ? pl->Ibuf2 : nullptr;
  m.q1 = cfg->single_q;
  m.q2 = cfg->poissn_q;
  m.coef = pl->coef;
  m.ci = ci;
  m.lparts = pl->lparts;
  int rc = PTYX_OK;
  if (ph != kPhaseEnd) {
    if ((rc = register_prep(pl, in, a, cfg, st, nseg))) return rc;
    {
      ProfScope ps(pl, kKFmmFwd, st);
      if (a.shift && holdh) hipLaunchKernelGGL((f3::k_fmm_fwd<true, true>), dim3(G), dim3(256), 0, st, m);
      else if (a.shift) hipLaunchKernelGGL((f3::k_fmm_fwd<true, false>), dim3(G), dim3(256), 0, st, m);
      else if (holdh) hipLaunchKernelGGL((f3::k_fmm_fwd<false, true>), dim3(G), dim3(256), 0, st, m);
      else hipLaunchKernelGGL((f3::k_fmm_fwd<false, false>), dim3(G), dim3(256), 0, st, m);
    }
    {
      ProfScope ps(pl, kKFmmLoss, st);
      const dim3 gr(a.n_idx * f3::kLossParts), bl(256);
      const bool half = cfg->single_q == 0.5f;
      if (both && half) hipLaunchKernelGGL((f3::k_fmm_loss<0, 3>), gr, bl, 0, st, m);
      else if (both) hipLaunchKernelGGL((f3::k_fmm_loss<2, 3>), gr, bl, 0, st, m);
      else if (single && half) hipLaunchKernelGGL((f3::k_fmm_loss<0, 1>), gr, bl, 0, st, m);
      else if (single) hipLaunchKernelGGL((f3::k_fmm_loss<2, 1>), gr, bl, 0, st, m);
      else hipLaunchKernelGGL((f3::k_fmm_loss<2, 2>), gr, bl, 0, st, m);
    }
    if ((rc = launch_status("k_fmm forward launch"))) return rc;
  }
  FinArgs fa{};
  fa.boff = a.boff; fa.n_batches = a.n_batches; fa.N = N; fa.Nz = Nz; fa.O = 1;
  fa.psums = pl->psums; fa.occu = in->omode_occu;
  if (pl->zsum_call) {   // the sparse sums as per-slice partials (k_small_prep)
    fa.zsum = pl->zsum;
    fa.zNz = Nz;
  }
  fa.single_on = cfg->single_on; fa.pois_on = cfg->poissn_on; fa.sparse_on = cfg->sparse_on;
  fa.sparse_n = cfg->sparse_n; fa.w1 = cfg->single_w; fa.w2 = cfg->poissn_w; fa.ws = cfg->sparse_w;
  fa.grad_scale = cfg->grad_scale; fa.coef = pl->coef; fa.loss_terms = loss_terms;
  static_assert(f3::kLossParts <= kFinMaxParts, "k_finalize's part loop");
  fa.lparts = pl->lparts; fa.nparts = f3::kLossParts;
  if (gz.d_obja || gz.d_objp) {
    fa.pcoef = pl->pcoef;
    fa.ci = 2;   // the slots already carry the data coefficients (k_fmm_adj): the gather's is 1
  }
  fa.bsums_out = ph == kPhaseBegin ? bsums : nullptr;
  fa.bsums_in = ph == kPhaseEnd ? bsums : nullptr;
  {
    ProfScope ps(pl, kKFinalize, st);
    hipLaunchKernelGGL(k_finalize, dim3((a.n_batches + kFinWaves - 1) / kFinWaves), dim3(64 * kFinWaves), 0, st, fa);
  }
  if ((rc = launch_status("k_finalize launch")) || ph == kPhaseBegin) return rc;
  const bool any_grad = gz.d_obja || gz.d_objp || gz.d_probe || gz.d_shifts;
  if (!any_grad) return PTYX_OK;
  {
    ProfScope ps(pl, kKFmmAdj, st);
    if (holdh) {
      if (a.shift && both) hipLaunchKernelGGL((f3::k_fmm_adj<true, true, true>), dim3(G), dim3(256), 0, st, m);
      else if (a.shift) hipLaunchKernelGGL((f3::k_fmm_adj<true, false, true>), dim3(G), dim3(256), 0, st, m);
      else if (both) hipLaunchKernelGGL((f3::k_fmm_adj<false, true, true>), dim3(G), dim3(256), 0, st, m);
      else hipLaunchKernelGGL((f3::k_fmm_adj<false, false, true>), dim3(G), dim3(256), 0, st, m);
    } else {
      if (a.shift && both) hipLaunchKernelGGL((f3::k_fmm_adj<true, true, false>), dim3(G), dim3(256), 0, st, m);
      else if (a.shift) hipLaunchKernelGGL((f3::k_fmm_adj<true, false, false>), dim3(G), dim3(256), 0, st, m);
      else if (both) hipLaunchKernelGGL((f3::k_fmm_adj<false, true, false>), dim3(G), dim3(256), 0, st, m);
      else hipLaunchKernelGGL((f3::k_fmm_adj<false, false, false>), dim3(G), dim3(256), 0, st, m);
    }
  }
  if ((rc = launch_status("k_fmm_adj launch"))) return rc;
  const bool bins = a.n_idx > f3::kSmallCall;
  if ((gz.d_obja || gz.d_objp) && bins) {
    ProfScope ps(pl, kKTable, st);
    const int tiles_x = (d.Nx + kGTX - 1) / kGTX;
    if (int rc2 = fill32(pl->bcnt, pl->nbins, 0u, st)) return rc2;
    const dim3 gn((a.n_idx + 255) / 256);
    hipLaunchKernelGGL(k_bin_count, gn, dim3(256), 0, st, pl->geo, a.n_idx, tiles_x, pl->bcnt, pl->bkey);
    hipLaunchKernelGGL(k_bin_scan, dim3(1), dim3(1024), 0, st, pl->bcnt, pl->nbins, pl->boff, pl->bcur);
    hipLaunchKernelGGL(k_bin_fill, gn, dim3(256), 0, st, pl->bkey, a.n_idx, pl->bcur, pl->blist);
    hipLaunchKernelGGL(k_bin_sort, dim3(pl->nbins), dim3(256), 0, st, pl->boff, pl->blist);
  }
  const bool gather_here = gz.d_obja || gz.d_objp;
  GatherArgs g{};
  int tiles = 0;
  bool sparse_tiles = false;
  if (gather_here) {
    g.ogscr = pl->ffc; g.geo = pl->geo; g.pcoef = pl->pcoef; g.n = a.n_idx;
    g.boff = bins ? pl->boff : nullptr;
    g.blist = bins ? pl->blist : nullptr;
    g.Ny = d.Ny; g.Nx = d.Nx; g.tiles_x = (d.Nx + kGTX - 1) / kGTX; g.sparse_n = cfg->sparse_on ? cfg->sparse_n : 1;
    g.obja = a.obja; g.objp = a.objp; g.d_obja = gz.d_obja; g.d_objp = gz.d_objp;
    g.nz = Nz; g.np = P; g.pstride = m.pstride;
    g.bbox = pl->bbox;
    g.zgrid = 1;
    g.store = pl->grad_store;
    tiles = g.tiles_x * ((d.Ny + kGTY - 1) / kGTY);
    sparse_tiles = (long long)a.n_idx * BinReach<N>::n < 64LL * tiles;
  }
  float* d_shifts = a.shift ? gz.d_shifts : nullptr;
  const bool small_tail = !bins && nseg <= f3::kTailSegCap && (gz.d_probe || d_shifts);
  // PTYX_PREP_FUSED_ADAM on a small call whose gather is the default row-split one: the gather, the
  // probe rows and the optimizer step in one launch after the probe / position sums
  FusedAdamArgs fz{};
  const bool fuse = ph == kPhaseAll && pl->fadam_on && gather_here && !bins && sparse_tiles && P <= kGatherMaxNp &&
                    gather_form(true, g.n) >= 1 && g_tuning[kTuneGatherSplit] < 1 && g_tuning[kTuneFuseAdam] != 0 &&
                    (small_tail || !(gz.d_probe || d_shifts)) &&
                    fused_adam_setup(pl, a.obja, a.objp, in->probe, gz, a.shift, g, tiles, &fz);
  if (gather_here && !fuse) {
    ProfScope ps(pl, kKGather, st);
    launch_gather<N, true, true>(pl, g, tiles, Nz, sparse_tiles, st);
  }
  if ((rc = launch_status("k_obj_gather launch"))) return rc;
  // (tuning rows_hu 2: two hits' loads in flight a wave, at two workgroups a CU instead of three)
  const auto launch_fused = [&] {
    ProfScope ps(pl, kKGatherAdam, st);
    const dim3 gr(fz.tiles + fz.pblocks + fz.rblocks);
    if (g_tuning[kTuneRowsHu] == 2) hipLaunchKernelGGL((k_gather_adam<N, true, true, 2>), gr, dim3(256), 0, st, fz);
    else hipLaunchKernelGGL((k_gather_adam<N, true, true, 1>), gr, dim3(256), 0, st, fz);
    pl->fadam_done = true;
    return launch_status("k_gather_adam launch");
  };
  if (fuse && !small_tail) return launch_fused();
  if (small_tail) {   // small call: one launch for the probe / position sums
    {
      ProfScope ps(pl, kKSlabReduce, st);
      const dim3 gr(N2 / 256 + (d_shifts ? (a.n_idx + 255) / 256 : 0), P);
      float2* out = gz.d_probe ? pl->Gsum : nullptr;
      if (a.shift)   // (with the probe gradient: its column IFFT in the same launch, into pl->slab)
        hipLaunchKernelGGL(f3::k_small_tail_modes<true>, gr, dim3(256), 0, st, pl->segslab, pl->segbid, nseg, out,
                           a.idx, a.n_idx, a.n_scans, P, pl->dsu, d_shifts, pl->twg, gz.d_probe ? pl->slab : nullptr);
      else
        hipLaunchKernelGGL(f3::k_small_tail_modes<false>, gr, dim3(256), 0, st, pl->segslab, pl->segbid, nseg, out,
                           a.idx, a.n_idx, a.n_scans, P, pl->dsu, d_shifts, nullptr, nullptr);
    }
    if (gz.d_probe && a.shift) {
      if (!fuse) {
        ProfScope ps(pl, kKProbeFinalize, st);
        hipLaunchKernelGGL(f3::k_probe_rows_acc, dim3(N / f3::kPrLinesT, P), dim3(256), 0, st, pl->slab,
                           reinterpret_cast<float2*>(gz.d_probe), pl->twg);
      }
    } else if (gz.d_probe) {
      launch_probe_fin_reg(pl, a, st, gz.d_probe, P);
    }
    if ((rc = launch_status("k_fmm probe / position reduction launch"))) return rc;
    if (fuse) return launch_fused();
    return PTYX_OK;
  }
  if (d_shifts) {
    ProfScope ps(pl, kKSlabReduce, st);
    hipLaunchKernelGGL(f3::k_shift_apply_modes, dim3((a.n_idx + 255) / 256), dim3(256), 0, st, a.idx, a.n_idx,
                       a.n_scans, P, pl->dsu, gz.d_shifts);
  }
  if (gz.d_probe) {
    {
      ProfScope ps(pl, kKSlabReduce, st);
      hipLaunchKernelGGL(f3::k_segslab_reduce_modes, dim3(N2 / 256, f3::kSegSplit, P), dim3(256), 0, st, pl->segslab,
                         pl->segbid, nseg, pl->segpart);
      if (a.shift)
        hipLaunchKernelGGL(f3::k_segslab_final<true>, dim3(N2 / 256, P), dim3(256), 0, st, pl->segpart, pl->Gsum);
      else
        hipLaunchKernelGGL(f3::k_segslab_final<false>, dim3(N2 / 256, P), dim3(256), 0, st, pl->segpart, pl->Gsum);
    }
    launch_probe_fin_reg(pl, a, st, gz.d_probe, P);
  }
  return launch_status("k_fmm probe / position reduction launch");
}

// ---------------------------------------------------------------- stripe engine (N = 256)
// Launch sequence of one ptyx_forward_loss_grad call on the stripe engine (ptyx_stripe.hpp).
// The stripe engine's per-call argument block (shared by the passes before and after k_finalize).
static sp::SArgs stripe_args(const ptyx_plan* pl, const KArgs& a, const ptyx_loss_cfg* cfg, const ptyx_grads& gz,
                             int defer_groups) {
  using namespace sp;
  const ptyx_dims& d = pl->d;
  const int n = a.n_idx, P = d.P, O = d.O;
  const bool single = cfg->single_on != 0;
  SArgs s{};
  s.n = n; s.P = P; s.O = O; s.Ny = d.Ny; s.Nx = d.Nx; s.n_scans = d.n_scans; s.meas_f16 = a.meas_f16;
  s.idx = a.idx; s.bid = pl->bid; s.geo = pl->geo; s.shifts = a.shifts; s.sxy = pl->ssxy; s.mrow = a.mrow;
  s.mrows = a.mrows;
  s.Fp = pl->Fp; s.oc = pl->oc; s.obja = a.obja; s.objp = a.objp; s.meas = a.meas; s.occu = a.occu;
  s.q = single ? cfg->single_q : cfg->poissn_q;
  s.q2 = cfg->poissn_q;
  s.eps2 = cfg->poissn_eps;
  s.sparse_on = cfg->sparse_on; s.sparse_n = cfg->sparse_n;
  s.t14 = pl->st14; s.psi0 = pl->spsi0; s.t23 = pl->st23; s.psum_s = pl->spsum; s.dp_out = a.dp_out;
  s.coef = pl->coef; s.ci = (single && cfg->poissn_on) ? 2 : single ? 0 : 1;
  s.d_obja = gz.d_obja; s.d_objp = gz.d_objp;
  const bool sgather = pl->sgather && (gz.d_obja || gz.d_objp);
  s.oslot = sgather ? pl->st23 : nullptr;
  s.groups = std::max(1, std::min(pl->stripe_groups, n));
  if (pl->slab_live) {                 // an earlier piece of the step left its k_s5 partials
    s.groups = pl->slab_live_groups;
    s.slab_acc = 1;
  } else if (defer_groups > 0) {
    s.groups = defer_groups;
  }
  s.slabpart = pl->sslab; s.dsp = pl->sdsp;
  s.twg = pl->twg;
  return s;
}

// k_s3.  ph 0: one data term (unit-coefficient g_Ψ);  both terms: ph 1 the partial sums before
// k_finalize, ph 2 the coefficient-weighted g_Ψ after it.
static void launch_s3(const ptyx_plan* pl, const sp::SArgs& s, const ptyx_loss_cfg* cfg, int ph, hipStream_t st) {
  using namespace sp;
  ProfScope ps(pl, kKS3, st);
  const dim3 gr(s.n, kStripes), bl(256);
  const int P = s.P, O = s.O;
  const bool single = cfg->single_on != 0;
  const bool half = single && s.q == 0.5f;
  if (ph == 1) {
    if (half) hipLaunchKernelGGL((k_s3<true, 0, 0, 1>), gr, bl, 0, st, s);
    else hipLaunchKernelGGL((k_s3<true, 2, 0, 1>), gr, bl, 0, st, s);
    return;
  }
  // Ψ of the first min(P·O, hold) modes stays in registers between k_s3's two sweeps, the other
  // modes' column FFTs are redone.  Default (profiles/r02/ab/r02n_*): 2 of P·O ≤ 4 (c5: three
  // workgroups per CU beat the saved re-reads), 4 above (c3)
  const int hold_max = g_tuning[kTuneHold] >= 0 ? std::min<int>(4, (int)g_tuning[kTuneHold]) : (P * O <= 4 ? 2 : 4);
  const int H = std::min(P * O, hold_max);
#define PTYX_S3(SG, QM, PH)                                                                              \
  switch (H) {                                                                                         \
    case 1: hipLaunchKernelGGL((k_s3<SG, QM, 1, PH>), gr, bl, 0, st, s); break;                         \
    case 2: hipLaunchKernelGGL((k_s3<SG, QM, 2, PH>), gr, bl, 0, st, s); break;                         \
    case 3: hipLaunchKernelGGL((k_s3<SG, QM, 3, PH>), gr, bl, 0, st, s); break;                         \
    case 4: hipLaunchKernelGGL((k_s3<SG, QM, 4, PH>), gr, bl, 0, st, s); break;                         \
    default: hipLaunchKernelGGL((k_s3<SG, QM, 0, PH>), gr, bl, 0, st, s); break;                        \
  }
  if (ph == 2) {
    if (half) { PTYX_S3(true, 0, 2) }
    else { PTYX_S3(true, 2, 2) }
  } else if (half) { PTYX_S3(true, 0, 0) }
  else if (single) { PTYX_S3(true, 2, 0) }
  else { PTYX_S3(false, 2, 0) }
#undef PTYX_S3
}

// Stripe engine before k_finalize: preparation, pattern table, k_s1..k_s3, per-pattern sums.
static int stripe_pass(ptyx_plan* pl, const KArgs& a, const ptyx_loss_cfg* cfg, const sp::SArgs& s, hipStream_t st) {
  using namespace sp;
  const ptyx_dims& d = pl->d;
  const int n = a.n_idx, P = d.P, O = d.O;
  const bool single = cfg->single_on != 0;
  const bool reuse = cfg->prep == PTYX_PREP_REUSE;     // object / probe prepared by the previous call
  if (!reuse) {                                         // F(P_p), natural order (no transposed copy)
    KArgs b = a;
    b.FpT = nullptr;
    launch_spectrum(pl, b, st);
  }
  {
    ProfScope ps(pl, kKTable, st);
    hipLaunchKernelGGL(k_s_table, dim3((n + 255) / 256), dim3(256), 0, st, a.idx, n, a.boff, a.n_batches, a.crop,
                       a.n_scans, d.Ny, d.Nx, pl->bid, pl->geo, a.shifts, pl->ssxy, a.err, a.mrow, a.mrows);
    hipLaunchKernelGGL(f3::k_bbox_init, dim3(1), dim3(64), 0, st, pl->bbox);
    hipLaunchKernelGGL(f3::k_bbox, dim3(std::max(1, std::min(f3::kBboxBlocks, (n + 255) / 256))), dim3(256), 0, st, a.idx, n, a.crop, a.n_scans, d.Ny, d.Nx,
                       pl->bbox, kN);
  }
  if (!reuse) {
    ProfScope ps(pl, kKObjPrep, st);   // O = A e^{iφ} on the rows the call's windows touch (or all)
    hipLaunchKernelGGL(f3::k_obj_prep, dim3(d.O * d.Ny), dim3(256), 0, st, a.obja, a.objp, d.O * d.Ny, d.Nx, pl->oc,
                       nullptr, 1, cfg->prep == PTYX_PREP_FULL ? nullptr : pl->bbox, d.Ny, kN);
  }
  const dim3 bl(256);
  {
    ProfScope ps(pl, kKS1, st);
    hipLaunchKernelGGL(k_s1, dim3(n, kStripes, P), bl, 0, st, s);
  }
  {
    ProfScope ps(pl, kKS2, st);
    if (O == 1) hipLaunchKernelGGL(k_s2<1>, dim3(n, kStripes), bl, 0, st, s);
    else hipLaunchKernelGGL(k_s2<2>, dim3(n, kStripes), bl, 0, st, s);
  }
  launch_s3(pl, s, cfg, s.ci == 2 ? 1 : 0, st);
  int rc = launch_status("stripe forward launch");
  if (rc) return rc;
  {
    ProfScope ps(pl, kKTable, st);
    hipLaunchKernelGGL(k_s_psum, dim3((n * kNSum + 255) / 256), dim3(256), 0, st, pl->spsum, n, pl->psums);
  }
  return launch_status("k_s_psum launch");
}

static int run_stripe(ptyx_plan* pl, const ptyx_inputs* in, const KArgs& a, const ptyx_loss_cfg* cfg,
                      const ptyx_grads& gz, hipStream_t st, float* loss_terms, int ph, double* bsums, bool defer) {
  using namespace sp;
  const ptyx_dims& d = pl->d;
  const int n = a.n_idx, P = d.P, O = d.O;
  const bool tail = gz.d_probe != nullptr || gz.d_shifts != nullptr;
  const bool any_grad = gz.d_obja || gz.d_objp || tail;
  if (pl->slab_live && gz.d_probe != pl->slab_live_probe)
    return fail(PTYX_EINVAL, "a deferred probe gradient awaits a call with the same d_probe");
  // s_defer_groups tuning: 0 = never defer, > 0 = k_s5 groups of deferring calls
  const long long dg = g_tuning[kTuneDeferGroups];
  if (dg == 0 || !gz.d_probe) defer = false;
  const int defer_groups = !defer ? 0 : dg > 0 ? (int)std::min<long long>(dg, pl->stripe_groups) : pl->stripe_defer_groups;
  const sp::SArgs s = stripe_args(pl, a, cfg, gz, defer_groups);
  const bool sgather = s.oslot != nullptr;
  const dim3 bl(256);
  int rc = PTYX_OK;
  if (ph != kPhaseEnd && (rc = stripe_pass(pl, a, cfg, s, st))) return rc;
  FinArgs fa{};
  fa.boff = a.boff; fa.n_batches = a.n_batches; fa.N = kN; fa.Nz = 1; fa.O = O;
  fa.psums = pl->psums; fa.occu = in->omode_occu;
  fa.single_on = cfg->single_on; fa.pois_on = cfg->poissn_on; fa.sparse_on = cfg->sparse_on;
  fa.sparse_n = cfg->sparse_n; fa.w1 = cfg->single_w; fa.w2 = cfg->poissn_w; fa.ws = cfg->sparse_w;
  fa.grad_scale = cfg->grad_scale; fa.coef = pl->coef; fa.loss_terms = loss_terms;
  if (sgather) {
    fa.pcoef = pl->pcoef;
    fa.ci = s.ci;
    fa.pcoef_O = O;
    fa.pcoef_stride = n;
  }
  fa.bsums_out = ph == kPhaseBegin ? bsums : nullptr;
  fa.bsums_in = ph == kPhaseEnd ? bsums : nullptr;
  {
    ProfScope ps(pl, kKFinalize, st);
    hipLaunchKernelGGL(k_finalize, dim3((a.n_batches + kFinWaves - 1) / kFinWaves), dim3(64 * kFinWaves), 0, st, fa);
  }
  if ((rc = launch_status("k_finalize launch")) || ph == kPhaseBegin) return rc;
  if (!any_grad) return PTYX_OK;
  if (s.ci == 2) {   // both data terms: g_Ψ with the mini-batch coefficients, now known
    launch_s3(pl, s, cfg, 2, st);
    if ((rc = launch_status("k_s3 launch"))) return rc;
  }
  {
    ProfScope ps(pl, kKS4, st);
    SArgs s4 = s;
    s4.t4 = tail ? pl->st14 : nullptr;   // no probe / position gradient: skip the gP transform
    const bool park = s4.psi0 != nullptr;
    if (O == 1 && park) hipLaunchKernelGGL((k_s4<1, true>), dim3(n, kStripes), bl, 0, st, s4);
    else if (O == 1) hipLaunchKernelGGL((k_s4<1, false>), dim3(n, kStripes), bl, 0, st, s4);
    else if (park) hipLaunchKernelGGL((k_s4<2, true>), dim3(n, kStripes), bl, 0, st, s4);
    else hipLaunchKernelGGL((k_s4<2, false>), dim3(n, kStripes), bl, 0, st, s4);
  }
  if ((rc = launch_status("k_s4 launch"))) return rc;
  if (sgather) {
    // object gradient from the slots: candidate bins per call, then one k_obj_gather per mode
    const int tiles_x = (d.Nx + kGTX - 1) / kGTX;
    {
      ProfScope ps(pl, kKTable, st);
      if (int rc2 = fill32(pl->bcnt, pl->nbins, 0u, st)) return rc2;
      const dim3 gn((n + 255) / 256);
      hipLaunchKernelGGL(k_bin_count, gn, dim3(256), 0, st, pl->geo, n, tiles_x, pl->bcnt, pl->bkey);
      hipLaunchKernelGGL(k_bin_scan, dim3(1), dim3(1024), 0, st, pl->bcnt, pl->nbins, pl->boff, pl->bcur);
      hipLaunchKernelGGL(k_bin_fill, gn, dim3(256), 0, st, pl->bkey, n, pl->bcur, pl->blist);
      hipLaunchKernelGGL(k_bin_sort, dim3(pl->nbins), dim3(256), 0, st, pl->boff, pl->blist);
    }
    GatherArgs g{};
    g.ogscr = pl->st23; g.geo = pl->geo; g.n = n; g.boff = pl->boff; g.blist = pl->blist;
    g.Ny = d.Ny; g.Nx = d.Nx; g.tiles_x = tiles_x; g.sparse_n = cfg->sparse_on ? cfg->sparse_n : 1;
    g.nz = P * O;   // slot o = field o of the pattern's P·O T3 fields
    g.bbox = pl->bbox;
    const int tiles = tiles_x * ((d.Ny + kGTY - 1) / kGTY);
    const bool sparse_tiles = (long long)n * BinReach<kN>::n < 64LL * tiles;
    const size_t plane = (size_t)d.Ny * d.Nx;
    ProfScope ps(pl, kKGather, st);
    for (int o = 0; o < O; ++o) {
      g.z = o;
      g.pcoef = pl->pcoef + (size_t)o * n;
      g.obja = a.obja + o * plane;
      g.objp = a.objp + o * plane;
      g.d_obja = gz.d_obja ? gz.d_obja + o * plane : nullptr;
      g.d_objp = gz.d_objp ? gz.d_objp + o * plane : nullptr;
      launch_gather<kN, false, false>(pl, g, tiles, 1, sparse_tiles, st);
    }
    if ((rc = launch_status("stripe k_obj_gather launch"))) return rc;
  }
  if (!tail) return PTYX_OK;
  {
    ProfScope ps(pl, kKS5, st);
    hipLaunchKernelGGL(k_s5, dim3(kStripes, P, s.groups), bl, 0, st, s);
  }
  if ((rc = launch_status("k_s5 launch"))) return rc;
  if (gz.d_shifts) {
    ProfScope ps(pl, kKSlabReduce, st);
    hipLaunchKernelGGL(k_s_shift, dim3((n + 255) / 256), dim3(256), 0, st, pl->sdsp, n, kStripes * P, a.idx,
                       a.n_scans, gz.d_shifts);
  }
  if (gz.d_probe && defer) {   // the reduction and the inverse FFT wait for the step's last piece
    pl->slab_live = true;
    pl->slab_live_groups = s.groups;
    pl->slab_live_probe = gz.d_probe;
  } else if (gz.d_probe) {
    pl->slab_live = false;
    const long long per = (long long)P * kN2;
    {
      ProfScope ps(pl, kKSlabReduce, st);
      hipLaunchKernelGGL(k_slab_reduce, dim3((unsigned)((per + 255) / 256)), dim3(256), 0, st, pl->sslab, s.groups,
                         per, pl->Gsum);
    }
    launch_probe_fin(pl, a, st, gz.d_probe, P);
  }
  return launch_status("stripe adjoint launch");
}

extern "C" int ptyx_profile_begin(ptyx_plan* pl) {
  g_err.clear();
  if (!pl) return fail(PTYX_EINVAL, "plan is null");
  pl->prof = true;
  return PTYX_OK;
}

extern "C" int ptyx_profile_end(ptyx_plan* pl, ptyx_kernel_stat* out, int32_t cap, int32_t* n_out) {
  g_err.clear();
  if (!pl) return fail(PTYX_EINVAL, "plan is null");
  DeviceGuard dg(pl->device);
  int launches[kKCount] = {0};
  double ms[kKCount] = {0};
  int rc = PTYX_OK;
  for (auto& r : pl->recs) {
    float t = 0.f;
    hipError_t e = hipEventSynchronize(r.b);
    if (e == hipSuccess) e = hipEventElapsedTime(&t, r.a, r.b);
    if (e != hipSuccess && rc == PTYX_OK) rc = hip_fail(e, "hipEventElapsedTime");
    launches[r.kind] += 1;
    ms[r.kind] += t;
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  pl->recs.clear();
  pl->prof = false;
  int n = 0;
  for (int k = 0; k < kKCount; ++k) {
    if (!launches[k]) continue;
    if (out && n < cap) {
      std::snprintf(out[n].name, sizeof(out[n].name), "%s", kKernelNames[k]);
      out[n].launches = launches[k];
      out[n].total_ms = (float)ms[k];
    }
    ++n;
  }
  if (n_out) *n_out = n;
  return rc;
}

// ---------------------------------------------------------------- graph-replayed step bookkeeping
// (ptyrad_amd/stepgraph.py): the step's indices by a device counter, and the flat gradient zeroed,
// in one launch; the loss terms stored and the counter advanced in another.
__global__ void k_step_select(const int32_t* idx_all, const int64_t* istart, const int64_t* cnt, int n,
                              int32_t* idx_out, float* grad, int64_t grad_n, float* const* steps, int n_steps) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (int64_t)gridDim.x * blockDim.x;
  if (t < n) idx_out[t] = idx_all[istart[*cnt] + t];
  if (t < n_steps) {   // the optimizer's step counts (f32, as torch's state_step += 1)
    float* s = steps[t];
    *s = *s + 1.0f;
  }
  // scalar head up to 16-byte alignment, float4 body, scalar tail
  const int64_t head = std::min<int64_t>(grad_n, ((16 - (reinterpret_cast<uintptr_t>(grad) & 15)) & 15) >> 2);
  if (t < head) grad[t] = 0.f;
  float4* g4 = reinterpret_cast<float4*>(grad + head);
  const int64_t n4 = (grad_n - head) >> 2;
  for (int64_t i = t; i < n4; i += stride) g4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t i = head + 4 * n4 + t; i < grad_n; i += stride) grad[i] = 0.f;
}
__global__ __launch_bounds__(256) void k_step_store(const float* terms, int nb, const int64_t* rstart, int64_t* cnt,
                                                    float* terms_all) {
  const int64_t c = *cnt;
  const int64_t r0 = rstart[c];
  for (int i = threadIdx.x; i < nb * 5; i += blockDim.x) terms_all[r0 * 5 + i] = terms[i];
  __syncthreads();   // every thread has read *cnt
  if (threadIdx.x == 0) *cnt = c + 1;
}

static int step_select_check(const int32_t* idx_all, const int64_t* istart, const int64_t* cnt, float* grad,
                             int64_t grad_n, float* const* steps, int32_t n_steps) {
  if (!idx_all || !istart || !cnt || grad_n < 0 || (grad_n && !grad))
    return fail(PTYX_EINVAL, "ptyx_step_select: null pointer or negative size");
  if (n_steps < 0 || n_steps > 256 || (n_steps && !steps))
    return fail(PTYX_EINVAL, "ptyx_step_select: steps must be a device array of at most 256 pointers");
  if (reinterpret_cast<uintptr_t>(grad) % 4)
    return fail(PTYX_EINVAL, "ptyx_step_select: grad must be 4-byte aligned");
  return PTYX_OK;
}

extern "C" int ptyx_step_select(void* stream, const int32_t* idx_all, const int64_t* istart, const int64_t* cnt,
                                int32_t n, int32_t* idx_out, float* grad, int64_t grad_n, float* const* steps,
                                int32_t n_steps) {
  g_err.clear();
  if (!idx_out || n < 0) return fail(PTYX_EINVAL, "ptyx_step_select: null pointer or negative size");
  if (int rc = step_select_check(idx_all, istart, cnt, grad, grad_n, steps, n_steps)) return rc;
  const int64_t work = std::max<int64_t>(n, (grad_n + 3) / 4);
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(4096, (work + 255) / 256));
  hipLaunchKernelGGL(k_step_select, dim3(blocks), dim3(256), 0, (hipStream_t)stream, idx_all, istart, cnt, n,
                     idx_out, grad, grad_n, steps, n_steps);
  return launch_status("k_step_select launch");
}

extern "C" int ptyx_step_store(void* stream, const float* terms, int32_t nb, const int64_t* rstart, int64_t* cnt,
                               float* terms_all) {
  g_err.clear();
  if (!terms || !rstart || !cnt || !terms_all || nb < 0)
    return fail(PTYX_EINVAL, "ptyx_step_store: null pointer or negative size");
  hipLaunchKernelGGL(k_step_store, dim3(1), dim3(256), 0, (hipStream_t)stream, terms, nb, rstart, cnt, terms_all);
  return launch_status("k_step_store launch");
}

extern "C" int ptyx_forward(ptyx_plan* pl, void* stream, const ptyx_inputs* in, const int32_t* idx, int32_t n_idx,
                            float* dp_out) {
  g_err.clear();
  if (!pl) return fail(PTYX_EINVAL, "plan is null");
  if (int rc0 = take_error(pl)) return rc0;
  int rc = check_inputs(pl, in, false);
  if (rc) return rc;
  if (n_idx < 0 || n_idx > pl->d.max_patterns) return fail(PTYX_EINVAL, "n_idx out of range [0, max_patterns]");
  if ((rc = busy(pl))) return rc;
  pl->slots_ready = false;
  if (n_idx == 0) return PTYX_OK;
  if (!idx || !dp_out) return fail(PTYX_EINVAL, "idx / dp_out is null");
  DeviceGuard dg(pl->device);
  pl->prep.valid = false;   // F(P) is rewritten
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  KArgs a = make_args(pl, in, idx, n_idx);
  a.dp_out = dp_out;
  a.psums = nullptr;
  if (a.shift || a.HT) launch_spectrum(pl, a, st);
  launch_forward(pl, a, st);
  return launch_status("ptyx_forward launch");
}

// propagator gradient: validate the request and point the kernels at the plan's slabs
static int setup_prop_grad(const ptyx_plan* pl, const ptyx_grads& gz, KArgs& a) {
  if (!gz.d_H && !gz.d_tilts && !gz.d_dz) return PTYX_OK;
  if (!(pl->d.flags & PTYX_PROP_GRAD))
    return fail(PTYX_EINVAL, "d_H / d_tilts need a plan created with PTYX_PROP_GRAD");
  if ((gz.d_tilts || gz.d_dz) && !a.ptilt) return fail(PTYX_EINVAL, "d_tilts / d_dz need inputs.obj_tilts");
  a.hslab = gz.d_H ? pl->hslab : nullptr;   // null when Nz == 1: H is unused, nothing to add
  a.d_tilts = pl->d.Nz > 1 ? gz.d_tilts : nullptr;
  a.d_dz = pl->d.Nz > 1 ? gz.d_dz : nullptr;
  return PTYX_OK;
}

static int reduce_prop_grad(const ptyx_plan* pl, const KArgs& a, const ptyx_grads& gz, hipStream_t st) {
  if (!gz.d_H || !a.hslab) return PTYX_OK;
  const int n2 = pl->d.N * pl->d.N;
  hipLaunchKernelGGL(k_hslab_reduce, dim3((n2 + 255) / 256), dim3(256), 0, st, pl->hslab, pl->nwg, n2,
                     reinterpret_cast<float2*>(gz.d_H));
  return launch_status("k_hslab_reduce launch");
}

// Validation, argument block and engine choice of one ptyx_forward_loss_grad call.
static int setup_call(ptyx_plan* pl, const ptyx_inputs* in, const int32_t* idx, const int32_t* boff,
                      int32_t n_batches, int32_t n_idx, const ptyx_loss_cfg* cfg, float* dp_out,
                      const ptyx_grads& gz, KArgs* out, int* engine) {
  if (!cfg) return fail(PTYX_EINVAL, "cfg is null");
  int rc = check_inputs(pl, in, true);
  if (rc) return rc;
  if (n_idx < 0 || n_idx > pl->d.max_patterns) return fail(PTYX_EINVAL, "n_idx out of range [0, max_patterns]");
  if (n_batches < 1 || n_batches > n_idx) return fail(PTYX_EINVAL, "need 1 <= n_batches <= n_idx");
  if (!idx || !boff) return fail(PTYX_EINVAL, "idx / batch_offsets is null");
  if (!cfg->single_on && !cfg->poissn_on)
    return fail(PTYX_EINVAL, "at least one data-error loss term (loss_single / loss_poissn) must be on");
  if (cfg->sparse_on && cfg->sparse_n < 1) return fail(PTYX_EINVAL, "sparse_n must be >= 1");
  if ((cfg->prep & ~(PTYX_PREP_DEFER_PROBE | PTYX_PREP_DEFER_GATHER | PTYX_PREP_GRAD_STORE | PTYX_PREP_FUSED_ADAM |
                     PTYX_PREP_SELECT)) > PTYX_PREP_REUSE ||
      cfg->prep < 0)
    return fail(PTYX_EINVAL, "unknown cfg.prep");
  KArgs a = make_args(pl, in, idx, n_idx);
  a.boff = boff;
  a.n_batches = n_batches;
  a.single_on = cfg->single_on;
  a.pois_on = cfg->poissn_on;
  a.sparse_on = cfg->sparse_on;
  a.sparse_n = cfg->sparse_n;
  a.q1 = cfg->single_q;
  a.q2 = cfg->poissn_q;
  a.eps2 = cfg->poissn_eps;
  a.psums = pl->psums;
  a.coef = pl->coef;
  a.dp_out = dp_out;
  a.d_obja = gz.d_obja;
  a.d_objp = gz.d_objp;
  a.d_shifts = gz.d_shifts;
  a.need_probe = gz.d_probe != nullptr;
  if ((rc = setup_prop_grad(pl, gz, a))) return rc;
  // propagator gradients and per-position tilts: general two-pass engine only
  const bool want_H = a.hslab != nullptr || a.d_tilts != nullptr || a.d_dz != nullptr ||
                      (a.ptilt != nullptr && pl->d.Nz > 1);
  a.w1 = cfg->single_w;
  a.w2 = cfg->poissn_w;
  a.ws = cfg->sparse_w;
  a.grad_scale = cfg->grad_scale;
  const bool any_grad = gz.d_obja || gz.d_objp || gz.d_probe || gz.d_shifts || gz.d_H || gz.d_tilts || gz.d_dz;
  const bool one_term = (cfg->single_on != 0) != (cfg->poissn_on != 0);
  const bool single_mode = pl->d.N <= 128 && pl->d.P * pl->d.O * pl->d.Nz == 1;
  const bool slots_fit = n_idx <= pl->og_cap && (long long)n_batches + std::min(pl->nwg3, n_idx) <= pl->seg_cap;
  // register-resident engines: k_fused3 (N = 128, single mode) and k_fused3ms (N = 128, P = O = 1,
  // Nz ≥ 2); f32 DPs, one data term, slots and segment slabs large enough for the call (no
  // co-residency or max_batch condition: they never wait)
  const bool both_terms = cfg->single_on && cfg->poissn_on;
  // (both data terms: two passes around k_finalize, MODE 1 / 2)
  const bool fused3 = any_grad && single_mode && pl->nwg3 > 0 && pl->d.N == 128 && !a.meas_f16 && slots_fit &&
                      (one_term || both_terms);
  const bool fused3ms = any_grad && !want_H && pl->ms3 && pl->nwg3 > 0 && !a.meas_f16 && slots_fit &&
                        (one_term || both_terms);
  // stripe engine (N = 256, Nz = 1, O ≤ 2, shifted probes): either or both data terms (both: k_s3
  // twice, around k_finalize), call within capacity
  const bool stripe = pl->stripe_cap > 0 && n_idx <= pl->stripe_cap && !want_H && a.shift && (one_term || both_terms);
  // mixed-state register engine (N = 128, P > 1, O = 1): either or both data terms (both applied
  // in k_fmm_adj), f32 DPs, the call within the far-field cache its slots live in
  const bool fmm = any_grad && !want_H && pl->fmm && !a.meas_f16 && n_idx <= pl->ffc_cap;   // (either or both terms)
#ifdef PTYX_ONLY_N
  *engine = (fused3 || fused3ms) && PTYX_ONLY_N == 128 ? kEngFused3 : fmm && PTYX_ONLY_N == 128 ? kEngFmm
          : stripe && PTYX_ONLY_N == 256 ? kEngStripe : kEngTwoPass;
#else
  *engine = (fused3 || fused3ms) ? kEngFused3 : fmm ? kEngFmm : stripe ? kEngStripe : kEngTwoPass;
#endif
  // (not with propagator gradients: k_adjoint's recomputed forward is what parks their Xⁿ)
  if (*engine == kEngTwoPass && any_grad && pl->ffc && n_idx <= pl->ffc_cap && !a.hslab && !a.d_tilts && !a.d_dz) {
    a.ffc = pl->ffc;
    a.ffc_per = pl->ffc_per;
  }
  if (pl->slab_live && *engine != kEngStripe)
    return fail(PTYX_EINVAL, "a deferred stripe probe gradient awaits the step's last piece on this plan");
  *out = a;
  return PTYX_OK;
}

// PTYX_PREP_GRAD_STORE: the register engines' gathers overwrite the object gradient (returns
// true: pl->grad_store for the call); any other engine accumulates, so its two arrays are cleared
// on the stream first.
static int grad_store_setup(ptyx_plan* pl, int engine, const ptyx_grads& gz, hipStream_t st, bool* gather_store) {
  *gather_store = false;
  if (engine == kEngFused3 || engine == kEngFmm) {
    *gather_store = true;
    return PTYX_OK;
  }
  const int64_t n = (int64_t)pl->d.O * pl->d.Nz * pl->d.Ny * pl->d.Nx;
  for (float* p : {gz.d_obja, gz.d_objp}) {
    if (!p) continue;
    if (int rc = fill32(p, n, 0u, st)) return rc;
  }
  return PTYX_OK;
}

// PTYX_PREP_REUSE only when the plan's record says a PTYX_PREP_FULL call of the same engine
// prepared the same inputs; otherwise the call prepares in full (a call split into
// pieces can change engine between pieces).  Updates the record.
static void resolve_prep(ptyx_plan* pl, const ptyx_inputs* in, int engine, ptyx_loss_cfg* c) {
  auto& r = pl->prep;
  if (c->prep == PTYX_PREP_REUSE) {
    const bool same = r.valid && r.engine == engine && r.obja == in->obja && r.objp == in->objp &&
                      r.probe == in->probe && r.H == in->H && r.sparse_on == c->sparse_on &&
                      (!c->sparse_on || r.sparse_n == c->sparse_n);
    if (same) return;
    c->prep = PTYX_PREP_FULL;
  }
  if (c->prep == PTYX_PREP_FULL) {
    r.valid = true;
    r.engine = engine;
    r.obja = in->obja; r.objp = in->objp; r.probe = in->probe; r.H = in->H;
    r.sparse_on = c->sparse_on; r.sparse_n = c->sparse_n;
  } else {
    r.valid = false;   // PTYX_PREP_CALL overwrites part of the preparation
  }
}

// The two-pass engine: k_forward (dp, loss partial sums) → k_finalize → k_adjoint.
static int run_two_pass(ptyx_plan* pl, const ptyx_inputs* in, const KArgs& a, const ptyx_loss_cfg* cfg,
                        const ptyx_grads& gz, hipStream_t st, float* loss_terms, int ph, double* bsums) {
  int rc = PTYX_OK;
  // small calls with several probe modes: one job per (pattern, probe mode), so a 32-pattern
  // mini-batch at P = 6 keeps 192 workgroups busy instead of 32 (the default grad_accumulation = 1)
  KArgs b = a;
  if (pl->Imodes && pl->d.P > 1 && a.n_idx <= kModeSplitCap && a.n_idx < pl->nwg) {
    b.msplit = pl->d.P;
    b.Imodes = pl->Imodes;
    b.cslab = a.hslab == nullptr;   // (a propagator slab per workgroup needs every workgroup)
  }
  if (ph != kPhaseEnd) {
    if ((b.shift || b.HT) && cfg->prep != PTYX_PREP_REUSE) launch_spectrum(pl, b, st);
    launch_forward(pl, b, st);
    if ((rc = launch_status("k_forward launch"))) return rc;
    if (b.msplit > 1) {
      ProfScope ps(pl, kKForward, st);
      launch_modesum(pl, b, st);
      if ((rc = launch_status("k_forward_modesum launch"))) return rc;
    }
  }
  FinArgs f{};
  f.boff = a.boff; f.n_batches = a.n_batches; f.N = pl->d.N; f.Nz = pl->d.Nz; f.O = pl->d.O;
  f.psums = pl->psums; f.occu = in->omode_occu;
  f.single_on = cfg->single_on; f.pois_on = cfg->poissn_on; f.sparse_on = cfg->sparse_on;
  f.sparse_n = cfg->sparse_n; f.w1 = cfg->single_w; f.w2 = cfg->poissn_w; f.ws = cfg->sparse_w;
  f.grad_scale = cfg->grad_scale; f.coef = pl->coef; f.loss_terms = loss_terms;
  f.bsums_out = ph == kPhaseBegin ? bsums : nullptr;
  f.bsums_in = ph == kPhaseEnd ? bsums : nullptr;
  {
    ProfScope ps(pl, kKFinalize, st);
    hipLaunchKernelGGL(k_finalize, dim3((a.n_batches + kFinWaves - 1) / kFinWaves), dim3(64 * kFinWaves), 0, st, f);
  }
  if ((rc = launch_status("k_finalize launch")) || ph == kPhaseBegin) return rc;
  const bool any_grad = gz.d_obja || gz.d_objp || gz.d_probe || gz.d_shifts || gz.d_H || gz.d_tilts || gz.d_dz;
  if (!any_grad) return PTYX_OK;
  launch_adjoint(pl, b, st, false);
  if ((rc = launch_status("k_adjoint launch"))) return rc;
  if ((rc = reduce_prop_grad(pl, a, gz, st))) return rc;
  if (gz.d_probe) {
    launch_probe_finalize(pl, a, st, gz.d_probe, adjoint_slabs(pl, b));
    if ((rc = launch_status("probe finalize launch"))) return rc;
  }
  return PTYX_OK;
}

static int run_call(ptyx_plan* pl, const ptyx_inputs* in, const KArgs& a, const ptyx_loss_cfg* cfg,
                    const ptyx_grads& gz, int engine, hipStream_t st, float* loss_terms, int ph, double* bsums,
                    bool defer) {
#if !defined(PTYX_ONLY_N) || PTYX_ONLY_N == 128
  if (engine == kEngFused3) return run_fused3(pl, in, a, cfg, gz, st, loss_terms, ph, bsums);
  if (engine == kEngFmm) return run_fmm(pl, in, a, cfg, gz, st, loss_terms, ph, bsums);
#endif
#if !defined(PTYX_ONLY_N) || PTYX_ONLY_N == 256
  if (engine == kEngStripe) return run_stripe(pl, in, a, cfg, gz, st, loss_terms, ph, bsums, defer);
#endif
  return run_two_pass(pl, in, a, cfg, gz, st, loss_terms, ph, bsums);
}

extern "C" int ptyx_forward_loss_grad(ptyx_plan* pl, void* stream, const ptyx_inputs* in, const int32_t* idx,
                                      const int32_t* boff, int32_t n_batches, int32_t n_idx,
                                      const ptyx_loss_cfg* cfg, float* loss_terms, float* dp_out,
                                      const ptyx_grads* grads) {
  g_err.clear();
  if (!pl) return fail(PTYX_EINVAL, "plan is null");
  if (int rc0 = take_error(pl)) return rc0;
  int rc = busy(pl);
  if (rc) return rc;
  ptyx_grads gz{};
  if (grads) gz = *grads;
  KArgs a{};
  int engine = kEngTwoPass;
  if (cfg && (cfg->prep & PTYX_PREP_DEFER_GATHER))
    return fail(PTYX_EINVAL, "PTYX_PREP_DEFER_GATHER is for ptyx_forward_loss_grad_begin / _end");
  if ((rc = setup_call(pl, in, idx, boff, n_batches, n_idx, cfg, dp_out, gz, &a, &engine))) return rc;
  DeviceGuard dg(pl->device);
  pl->slots_ready = false;
  ptyx_loss_cfg c = *cfg;
  const bool defer = (c.prep & PTYX_PREP_DEFER_PROBE) != 0;
  const bool store = (c.prep & PTYX_PREP_GRAD_STORE) != 0;
  const bool fadam = (c.prep & PTYX_PREP_FUSED_ADAM) != 0;
  const bool sel = (c.prep & PTYX_PREP_SELECT) != 0;
  c.prep &= ~(PTYX_PREP_DEFER_PROBE | PTYX_PREP_GRAD_STORE | PTYX_PREP_FUSED_ADAM | PTYX_PREP_SELECT);
  if (fadam && !pl->fadam_set) return fail(PTYX_EINVAL, "PTYX_PREP_FUSED_ADAM without ptyx_plan_set_adam");
  if (sel && !pl->sel_set) return fail(PTYX_EINVAL, "PTYX_PREP_SELECT without ptyx_plan_set_select");
  resolve_prep(pl, in, engine, &c);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // PTYX_PREP_SELECT: inside the register engines' small-call preparation launch, else first here
  pl->sel_fold = sel && (engine == kEngFused3 || engine == kEngFmm) && a.n_idx <= f3::kSmallCall && pl->bbox &&
                 c.prep == PTYX_PREP_CALL && g_tuning[kTuneSelFold] != 0;
  if (sel) {
    pl->sel_set = false;
    if (!pl->sel_fold) {
      const int64_t work = std::max<int64_t>(n_idx, (pl->sel_grad_n + 3) / 4);
      const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(4096, (work + 255) / 256));
      hipLaunchKernelGGL(k_step_select, dim3(blocks), dim3(256), 0, st, pl->sel_all, pl->sel_start, pl->sel_cnt, n_idx,
                         const_cast<int32_t*>(idx), pl->sel_grad, pl->sel_grad_n, pl->sel_steps, pl->sel_n_steps);
      if ((rc = launch_status("k_step_select launch"))) return rc;
    }
  }
  bool gstore = false;
  if (store && (rc = grad_store_setup(pl, engine, gz, st, &gstore))) return rc;
  pl->grad_store = gstore;
  pl->fadam_on = fadam;
  pl->fadam_done = false;
  rc = run_call(pl, in, a, &c, gz, engine, st, loss_terms, kPhaseAll, nullptr, defer);
  pl->grad_store = false;
  pl->sel_fold = false;
  if (fadam) {   // the registered step, consumed: fused into the epilogue, or its own launch now
    if (!rc && !pl->fadam_done)
      rc = opt::adam_launch(st, pl->fadam_ts, pl->fadam_h, pl->fadam_store ? &pl->fadam_ss : nullptr);
    pl->fadam_on = pl->fadam_set = pl->fadam_done = false;
  }
  return rc;
}

extern "C" int ptyx_plan_set_select(ptyx_plan* pl, const int32_t* idx_all, const int64_t* istart, const int64_t* cnt,
                                    float* grad, int64_t grad_n, float* const* steps, int32_t n_steps) {
  g_err.clear();
  if (!pl) return fail(PTYX_EINVAL, "plan is null");
  if (int rc = step_select_check(idx_all, istart, cnt, grad, grad_n, steps, n_steps)) return rc;
  pl->sel_all = idx_all;
  pl->sel_start = istart;
  pl->sel_cnt = cnt;
  pl->sel_grad = grad;
  pl->sel_grad_n = grad_n;
  pl->sel_steps = steps;
  pl->sel_n_steps = n_steps;
  pl->sel_set = true;
  return PTYX_OK;
}

extern "C" int ptyx_plan_set_adam(ptyx_plan* pl, int32_t n, float* const* params, const float* const* grads,
                                  float* const* exp_avgs, float* const* exp_avg_sqs, const float* const* steps,
                                  const int64_t* numels, const double* lrs, double beta1, double beta2, double eps,
                                  double weight_decay, int32_t flags, const float* terms, int32_t nb,
                                  const int64_t* rstart, int64_t* cnt, float* terms_all) {
  g_err.clear();
  if (!pl) return fail(PTYX_EINVAL, "plan is null");
  if (n < 0 || (n && (!params || !grads || !exp_avgs || !exp_avg_sqs || !steps || !numels || !lrs)))
    return fail(PTYX_EINVAL, "ptyx_plan_set_adam: null array or negative count");
  if (terms && (!rstart || !cnt || !terms_all || nb < 0))
    return fail(PTYX_EINVAL, "ptyx_plan_set_adam: null step-store pointer or negative size");
  std::vector<opt::AdamTensor> ts;
  for (int i = 0; i < n; ++i) {
    if (numels[i] < 0 || (numels[i] && (!params[i] || !grads[i] || !exp_avgs[i] || !exp_avg_sqs[i] || !steps[i])))
      return fail(PTYX_EINVAL, "ptyx_plan_set_adam: null tensor pointer or negative size");
    ts.push_back({params[i], grads[i], exp_avgs[i], exp_avg_sqs[i], steps[i], lrs[i], numels[i]});
  }
  pl->fadam_ts = std::move(ts);
  pl->fadam_h = opt::hyper(beta1, beta2, eps, weight_decay, flags);
  pl->fadam_store = terms != nullptr;
  pl->fadam_ss = opt::StepStore{terms, nb, rstart, cnt, terms_all};
  pl->fadam_set = true;
  return PTYX_OK;
}

extern "C" int ptyx_forward_loss_grad_begin(ptyx_plan* pl, void* stream, const ptyx_inputs* in, const int32_t* idx,
                                            const int32_t* boff, int32_t n_batches, int32_t n_idx,
                                            const ptyx_loss_cfg* cfg, float* dp_out, const ptyx_grads* grads,
                                            double* batch_sums) {
  g_err.clear();
  if (!pl) return fail(PTYX_EINVAL, "plan is null");
  if (int rc0 = take_error(pl)) return rc0;
  int rc = busy(pl);
  if (rc) return rc;
  if (!batch_sums) return fail(PTYX_EINVAL, "batch_sums is null");
  ptyx_grads gz{};
  if (grads) gz = *grads;
  KArgs a{};
  int engine = kEngTwoPass;
  if (cfg && (cfg->prep & (PTYX_PREP_FUSED_ADAM | PTYX_PREP_SELECT)))
    return fail(PTYX_EINVAL, "PTYX_PREP_FUSED_ADAM / PTYX_PREP_SELECT are for ptyx_forward_loss_grad (a split "
                             "step's gradients are complete only after the caller's exchange)");
  if ((rc = setup_call(pl, in, idx, boff, n_batches, n_idx, cfg, dp_out, gz, &a, &engine))) return rc;
  DeviceGuard dg(pl->device);
  ptyx_loss_cfg c = *cfg;
  const bool defer_gather = (c.prep & PTYX_PREP_DEFER_GATHER) != 0;
  const bool store = (c.prep & PTYX_PREP_GRAD_STORE) != 0;
  // a split call is one piece: it closes its own probe gradient
  c.prep &= ~(PTYX_PREP_DEFER_PROBE | PTYX_PREP_DEFER_GATHER | PTYX_PREP_GRAD_STORE);
  if (defer_gather && engine != kEngFused3)
    return fail(PTYX_EUNSUPPORTED, "PTYX_PREP_DEFER_GATHER needs the k_fused3 / k_fused3ms engine "
                                   "(ptyx_plan_slot_floats > 0, f32 DPs, the call within the register capacity)");
  if (defer_gather && store)
    return fail(PTYX_EINVAL, "PTYX_PREP_GRAD_STORE with PTYX_PREP_DEFER_GATHER: the slot gather accumulates");
  bool gstore = false;
  if (store && (rc = grad_store_setup(pl, engine, gz, reinterpret_cast<hipStream_t>(stream), &gstore))) return rc;
  pl->slots_ready = false;
  pl->use_tgt = defer_gather && pl->slot_tgt && n_idx <= pl->slot_tgt_cap;
  resolve_prep(pl, in, engine, &c);
  if ((rc = run_call(pl, in, a, &c, gz, engine, reinterpret_cast<hipStream_t>(stream), nullptr, kPhaseBegin,
                     batch_sums, false))) {
    pl->use_tgt = false;
    pl->slot_tgt = nullptr;
    return rc;
  }
  pl->pend = true;
  pl->pend_in = *in; pl->pend_gz = gz; pl->pend_cfg = c;
  pl->pend_idx = idx; pl->pend_boff = boff; pl->pend_nb = n_batches; pl->pend_n = n_idx;
  pl->pend_dp = dp_out; pl->pend_engine = engine;
  pl->pend_defer_gather = defer_gather;
  pl->pend_store = gstore;
  return PTYX_OK;
}

extern "C" int ptyx_forward_loss_grad_end(ptyx_plan* pl, void* stream, const double* batch_sums, float* loss_terms) {
  g_err.clear();
  if (!pl) return fail(PTYX_EINVAL, "plan is null");
  if (!pl->pend) return fail(PTYX_EINVAL, "no ptyx_forward_loss_grad_begin call is waiting on this plan");
  if (!batch_sums) return fail(PTYX_EINVAL, "batch_sums is null");
  pl->pend = false;
  KArgs a{};
  int engine = kEngTwoPass;
  int rc = setup_call(pl, &pl->pend_in, pl->pend_idx, pl->pend_boff, pl->pend_nb, pl->pend_n, &pl->pend_cfg,
                      pl->pend_dp, pl->pend_gz, &a, &engine);
  if (rc) return rc;
  if (engine != pl->pend_engine) return fail(PTYX_EINVAL, "internal: engine changed between _begin and _end");
  DeviceGuard dg(pl->device);
  pl->gather_deferred = pl->pend_defer_gather;
  pl->grad_store = pl->pend_store;
  rc = run_call(pl, &pl->pend_in, a, &pl->pend_cfg, pl->pend_gz, engine, reinterpret_cast<hipStream_t>(stream),
                loss_terms, kPhaseEnd, const_cast<double*>(batch_sums), false);
  pl->gather_deferred = false;
  pl->grad_store = false;
  if (rc == PTYX_OK && pl->pend_defer_gather) {
    pl->slots_ready = true;
    pl->slots_n = pl->pend_n;
    pl->slots_idx = pl->pend_idx;
    pl->slots_at = pl->use_tgt ? pl->slot_tgt : reinterpret_cast<float*>(pl->ogscr);
  }
  pl->use_tgt = false;
  pl->slot_tgt = nullptr;   // one call's target
  return rc;
}

// ---------------------------------------------------------------- slot exchange (split mini-batches)
constexpr int kSlotMeta = PTYX_SLOT_META;
// A split call with PTYX_PREP_DEFER_GATHER leaves its patterns' unit-coefficient object-gradient
// slots (g_O = conj(ψ⁰)·g, ptyx_gather.hpp), their window origins and mini-batch coefficients in
// the plan.  ptyx_slots_export copies them into caller buffers padded to a common count, the
// caller all-gathers those over the ranks, and ptyx_obj_gather_slots runs the deterministic
// gather over EVERY rank's patterns: each rank forms the whole object gradient itself, bitwise
// the same on every rank, with no object all-reduce.
extern "C" int64_t ptyx_plan_slot_floats(const ptyx_plan* pl) {
  if (!pl || pl->nwg3 <= 0 || pl->og_cap <= 0 || (pl->d.flags & PTYX_MEAS_F16) || pl->d.N != 128 ||
      pl->d.P * pl->d.O != 1)
    return 0;
  return (int64_t)2 * pl->d.Nz * pl->d.N * pl->d.N;
}

// Rank block of the slot exchange (floats): cap slots of sf floats, then cap table rows of
// kSlotMeta floats: geo (2 × int bits), pcoef (2), scan index (int bits), the pattern's
// position-gradient row (2), 0.  Padding rows: geo far outside the object (no tile hits it),
// pcoef 0, index -1.
__global__ void k_slots_meta(const int2* geo, const float2* pcoef, const int32_t* idx, int n, int n_pad,
                             const float* d_shifts, float* meta) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_pad) return;
  float* m = meta + (size_t)j * kSlotMeta;
  if (j < n) {
    const int2 o = geo[j];
    const float2 c = pcoef[j];
    const int s = idx[j];
    m[0] = __int_as_float(o.x); m[1] = __int_as_float(o.y);
    m[2] = c.x; m[3] = c.y;
    m[4] = __int_as_float(s);
    m[5] = d_shifts ? d_shifts[2 * (size_t)s] : 0.f;
    m[6] = d_shifts ? d_shifts[2 * (size_t)s + 1] : 0.f;
  } else {
    m[0] = __int_as_float(-(1 << 29)); m[1] = __int_as_float(-(1 << 29));
    m[2] = 0.f; m[3] = 0.f;
    m[4] = __int_as_float(-1);
    m[5] = 0.f; m[6] = 0.f;
  }
  m[7] = 0.f;
}

__device__ __forceinline__ const float* block_meta(const float* buf, int j, int cap, long long bfl, long long sf) {
  return buf + (size_t)(j / cap) * bfl + (size_t)cap * sf + (size_t)(j % cap) * kSlotMeta;
}

// geo / pcoef columns of every rank block's table rows, for GatherArgs
__global__ void k_slots_unpack(const float* buf, int n, int cap, long long bfl, long long sf, int2* geo,
                               float2* pcoef) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const float* m = block_meta(buf, j, cap, bfl, sf);
  geo[j] = make_int2(__float_as_int(m[0]), __float_as_int(m[1]));
  pcoef[j] = make_float2(m[2], m[3]);
}

// the other ranks' position-gradient rows added to this rank's dense d_shifts (every scan index
// occurs once in a call, so no two threads touch one row; this rank's own block is skipped)
__global__ void k_slots_rows_add(const float* buf, int n, int cap, long long bfl, long long sf, int self,
                                 float* d_shifts) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n || j / cap == self) return;
  const float* m = block_meta(buf, j, cap, bfl, sf);
  const int s = __float_as_int(m[4]);
  if (s < 0) return;
  d_shifts[2 * (size_t)s] += m[5];
  d_shifts[2 * (size_t)s + 1] += m[6];
}

extern "C" int64_t ptyx_slot_block_floats(const ptyx_plan* pl, int32_t cap) {
  const int64_t sf = ptyx_plan_slot_floats(pl);
  return sf > 0 && cap > 0 ? (int64_t)cap * (sf + kSlotMeta) : 0;
}

extern "C" int ptyx_plan_slot_target(ptyx_plan* pl, float* block, int32_t cap) {
  g_err.clear();
  if (!pl) return fail(PTYX_EINVAL, "plan is null");
  if (pl->pend) return fail(PTYX_EINVAL, "a ptyx_forward_loss_grad_begin call is waiting on this plan");
  if (block && ptyx_plan_slot_floats(pl) <= 0) return fail(PTYX_EUNSUPPORTED, "this plan's calls keep no slots");
  if (block && cap < 1) return fail(PTYX_EINVAL, "cap must be >= 1");
  pl->slot_tgt = block;
  pl->slot_tgt_cap = block ? cap : 0;
  return PTYX_OK;
}

extern "C" int ptyx_slots_export(ptyx_plan* pl, void* stream, int32_t use_last, int32_t cap, float* block,
                                 const float* d_shifts) {
  g_err.clear();
  if (!pl) return fail(PTYX_EINVAL, "plan is null");
  if (pl->pend) return fail(PTYX_EINVAL, "a ptyx_forward_loss_grad_begin call is waiting on this plan");
  const int64_t sf = ptyx_plan_slot_floats(pl);
  if (sf <= 0) return fail(PTYX_EUNSUPPORTED, "this plan's calls keep no object-gradient slots");
  if (use_last && !pl->slots_ready) return fail(PTYX_EINVAL, "no split call with PTYX_PREP_DEFER_GATHER to export");
  const int n = use_last ? pl->slots_n : 0;
  if (cap < n || cap < 1) return fail(PTYX_EINVAL, "cap must be >= 1 and cover the call's patterns");
  if (!block) return fail(PTYX_EINVAL, "null output block");
  DeviceGuard dg(pl->device);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n > 0 && pl->slots_at != block) {   // (written in place when the block was the call's target)
    hipError_t e = hipMemcpyAsync(block, pl->slots_at, (size_t)n * sf * sizeof(float), hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpyAsync(slots)");
  }
  hipLaunchKernelGGL(k_slots_meta, dim3((cap + 255) / 256), dim3(256), 0, st, pl->geo, pl->pcoef,
                     use_last ? pl->slots_idx : nullptr, n, cap, d_shifts, block + (size_t)cap * sf);
  return launch_status("k_slots_meta launch");
}

static int gather_slots(ptyx_plan* pl, void* stream, const float* blocks, int32_t n_ranks, int32_t cap,
                        int32_t self_rank, const float* obja, const float* objp, float* d_obja, float* d_objp,
                        int32_t sparse_n, float* d_shifts, bool fadam);

extern "C" int ptyx_obj_gather_slots(ptyx_plan* pl, void* stream, const float* blocks, int32_t n_ranks, int32_t cap,
                                     int32_t self_rank, const float* obja, const float* objp, float* d_obja,
                                     float* d_objp, int32_t sparse_n, float* d_shifts) {
  g_err.clear();
  return gather_slots(pl, stream, blocks, n_ranks, cap, self_rank, obja, objp, d_obja, d_objp, sparse_n, d_shifts,
                      false);
}

extern "C" int ptyx_obj_gather_slots_adam(ptyx_plan* pl, void* stream, const float* blocks, int32_t n_ranks,
                                          int32_t cap, int32_t self_rank, const float* obja, const float* objp,
                                          float* d_obja, float* d_objp, int32_t sparse_n, float* d_shifts) {
  g_err.clear();
  if (pl && !pl->fadam_set) return fail(PTYX_EINVAL, "ptyx_obj_gather_slots_adam without ptyx_plan_set_adam");
  const int rc = gather_slots(pl, stream, blocks, n_ranks, cap, self_rank, obja, objp, d_obja, d_objp, sparse_n,
                              d_shifts, true);
  if (pl) pl->fadam_set = pl->fadam_done = false;
  return rc;
}

static int gather_slots(ptyx_plan* pl, void* stream, const float* blocks, int32_t n_ranks, int32_t cap,
                        int32_t self_rank, const float* obja, const float* objp, float* d_obja, float* d_objp,
                        int32_t sparse_n, float* d_shifts, bool fadam) {
  if (!pl) return fail(PTYX_EINVAL, "plan is null");
  if (pl->pend) return fail(PTYX_EINVAL, "a ptyx_forward_loss_grad_begin call is waiting on this plan");
  const int64_t sf = ptyx_plan_slot_floats(pl);
  if (sf <= 0) return fail(PTYX_EUNSUPPORTED, "this plan's calls keep no object-gradient slots");
  if (n_ranks < 1 || cap < 1 || (int64_t)n_ranks * cap > pl->d.max_patterns)
    return fail(PTYX_EINVAL, "n_ranks x cap must be in [1, max_patterns]");
  if (self_rank < 0 || self_rank >= n_ranks) return fail(PTYX_EINVAL, "self_rank outside [0, n_ranks)");
  if (!blocks || !obja || !objp) return fail(PTYX_EINVAL, "null input");
  const int n = n_ranks * cap;
  const long long bfl = (long long)cap * (sf + kSlotMeta);
  const int sn = sparse_n < 1 ? 1 : sparse_n;
  DeviceGuard dg(pl->device);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // the unpacked table reuses the plan's per-call geo / pcoef arrays (capacity max_patterns)
  hipLaunchKernelGGL(k_slots_unpack, dim3((n + 255) / 256), dim3(256), 0, st, blocks, n, cap, bfl, (long long)sf,
                     pl->geo, pl->pcoef);
  int rc = launch_status("k_slots_unpack launch");
  if (rc) return rc;
  pl->slots_ready = false;
  // (the other ranks' position rows first: with the fused step their Adam runs in the gather's launch)
  if (d_shifts && n_ranks > 1) {
    hipLaunchKernelGGL(k_slots_rows_add, dim3((n + 255) / 256), dim3(256), 0, st, blocks, n, cap, bfl, (long long)sf,
                       self_rank, d_shifts);
    if ((rc = launch_status("k_slots_rows_add launch"))) return rc;
  }
  bool done = false;
  if (d_obja || d_objp) {
#if !defined(PTYX_ONLY_N) || PTYX_ONLY_N == 128
    constexpr int N = 128;
    GatherArgs g{};
    g.ogscr = reinterpret_cast<const float2*>(blocks); g.geo = pl->geo; g.pcoef = pl->pcoef; g.n = n;
    g.blk = cap; g.bstride = bfl / 2;   // (float2 units)
    g.boff = nullptr; g.blist = nullptr; g.bbox = nullptr;
    g.Ny = pl->d.Ny; g.Nx = pl->d.Nx; g.tiles_x = (pl->d.Nx + kGTX - 1) / kGTX; g.sparse_n = sn;
    g.obja = obja; g.objp = objp; g.d_obja = d_obja; g.d_objp = d_objp;
    const int tiles = g.tiles_x * ((pl->d.Ny + kGTY - 1) / kGTY);
    const bool sparse_tiles = (long long)n * BinReach<N>::n < 64LL * tiles;
    g.nz = pl->d.Nz;
    g.zgrid = 1;
    // ptyx_obj_gather_slots_adam: every other gradient is final (the caller all-reduced the probe
    // part): the gather with the optimizer step in one launch (k_gather_adam, no probe-row blocks)
    FusedAdamArgs fz{};
    ptyx_grads gz{};
    gz.d_obja = d_obja;
    gz.d_objp = d_objp;
    const int gform = gather_form(false, n);
    if (fadam && pl->d.Nz == 1 && sparse_tiles && g_tuning[kTuneFuseAdam] != 0 &&
        fused_adam_setup(pl, obja, objp, nullptr, gz, false, g, tiles, &fz)) {
      ProfScope ps(pl, kKGatherAdam, st);
      const dim3 gr(fz.tiles + fz.pblocks + fz.rblocks);
      if (gform == 3) hipLaunchKernelGGL((k_gather_adam_r5<N>), gr, dim3(256), 0, st, fz);
      else if (gform == 2) hipLaunchKernelGGL((k_gather_adam_r4<N>), gr, dim3(256), 0, st, fz);
      else if (gform == 1) hipLaunchKernelGGL((k_gather_adam<N, true, true, 1, false>), gr, dim3(256), 0, st, fz);
      else hipLaunchKernelGGL((k_gather_adam<N, true>), gr, dim3(256), 0, st, fz);
      done = true;
    } else {
      ProfScope ps(pl, kKGather, st);
      launch_gather<N, true, false>(pl, g, tiles, pl->d.Nz, sparse_tiles, st);
    }
    if ((rc = launch_status("k_obj_gather (slots) launch"))) return rc;
#endif
  }
  if (fadam && !done)
    rc = opt::adam_launch(st, pl->fadam_ts, pl->fadam_h, pl->fadam_store ? &pl->fadam_ss : nullptr);
  return rc;
}

extern "C" int ptyx_adjoint_dldi(ptyx_plan* pl, void* stream, const ptyx_inputs* in, const int32_t* idx,
                                 int32_t n_idx, const float* dLdI, float grad_scale, const ptyx_grads* grads) {
  g_err.clear();
  if (!pl) return fail(PTYX_EINVAL, "plan is null");
  if (int rc0 = take_error(pl)) return rc0;
  int rc = check_inputs(pl, in, false);
  if (rc) return rc;
  if (n_idx < 0 || n_idx > pl->d.max_patterns) return fail(PTYX_EINVAL, "n_idx out of range [0, max_patterns]");
  if ((rc = busy(pl))) return rc;
  pl->slots_ready = false;
  if (n_idx == 0 || !grads) return PTYX_OK;
  if (!idx || !dLdI) return fail(PTYX_EINVAL, "idx / dLdI is null");
  pl->prep.valid = false;   // F(P) is rewritten
  const ptyx_grads gz = *grads;
  if (!(gz.d_obja || gz.d_objp || gz.d_probe || gz.d_shifts || gz.d_H || gz.d_tilts || gz.d_dz)) return PTYX_OK;
  DeviceGuard dg(pl->device);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  KArgs a = make_args(pl, in, idx, n_idx);
  a.dLdI_ext = dLdI;
  a.ext_scale = grad_scale;
  a.d_obja = gz.d_obja;
  a.d_objp = gz.d_objp;
  a.d_shifts = gz.d_shifts;
  a.need_probe = gz.d_probe != nullptr;
  if ((rc = setup_prop_grad(pl, gz, a))) return rc;
  if (a.shift || a.HT) launch_spectrum(pl, a, st);
  launch_adjoint(pl, a, st, true);
  if ((rc = launch_status("k_adjoint(ext) launch"))) return rc;
  if ((rc = reduce_prop_grad(pl, a, gz, st))) return rc;
  if (gz.d_probe) {
    launch_probe_finalize(pl, a, st, gz.d_probe, pl->nwg);
    if ((rc = launch_status("probe finalize launch"))) return rc;
  }
  return PTYX_OK;
}

