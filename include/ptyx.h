/* ptyx.h — C ABI of the MI355X-native ptychographic forward/adjoint engine (libptyx.so).
 *
 * Drop-in boundary for PtyRAD's per-mini-batch hot path.  PtyRAD has no
 * FFI of its own; the interfaces each entry point replaces are:
 *
 *   ptyx_forward            PtychoAD.forward(indices) -> dp_fwd      src/ptyrad/models.py:422-436
 *                           (get_obj_ROI :251-265, get_probes :286-298, get_propagators case 4
 *                            :358-360, multislice_forward_model_vec_all src/ptyrad/forward.py:20-80)
 *   ptyx_forward_loss_grad  compute_loss + loss_batch.backward()      src/ptyrad/reconstruction.py:792-806, :750-753
 *                           (CombinedLoss.forward src/ptyrad/losses.py:143-155: loss_single :36-50,
 *                            loss_poissn :52-75, loss_sparse :91-104; autograd adjoint of all of the above)
 *   ptyx_adjoint_dldi       the autograd backward of PtychoAD.forward for an arbitrary downstream
 *                           loss that supplies dL/d(dp_fwd)            src/ptyrad/models.py:422-436
 *
 * Conventions
 *  - All array pointers are DEVICE pointers (HBM), caller-owned, contiguous, row-major, in the
 *    reference's layouts.  They are borrowed for the duration of the call only.
 *  - Complex arrays are interleaved (re, im) float32, i.e. torch.view_as_real layout.
 *  - Every call is asynchronous on `stream` (a hipStream_t; NULL = default stream) and performs
 *    no host<->device synchronisation, no allocation and no host copies, so it can be captured
 *    in a hipGraph.  Loss terms stay on the device.
 *  - Gradients are ACCUMULATED (+=) into caller-zeroed buffers; a NULL gradient pointer means
 *    "not required" (requires_grad False, reconstruction.py:783-790) and its work is skipped.
 *  - Status: 0 on success, a PTYX_E* code otherwise; ptyx_last_error() gives a thread-local
 *    message.  No C++ exception crosses the ABI.
 *  - A plan is bound to one device and one geometry and must not be used by two host threads
 *    concurrently.
 */
#ifndef PTYX_H
#define PTYX_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version: ptyx_dims.abi_version must equal it (ptyx_plan_create rejects a binding built
 * against another revision of this header); ptyx_version() returns it too. */
#define PTYX_ABI_VERSION 210

#define PTYX_OK 0
#define PTYX_EINVAL 1
#define PTYX_ENOMEM 2
#define PTYX_EHIP 3
#define PTYX_EUNSUPPORTED 4

/* loss_cfg.prep: per-call preparation of the object (A e^{iφ}, loss_sparse prefix sums) and of
 * the probe spectrum.  A caller that splits one optimizer step's group of mini-batches into
 * several calls (obja / objp / probe / H unchanged between them) passes PTYX_PREP_FULL on the
 * first call and PTYX_PREP_REUSE on the others. */
#define PTYX_PREP_CALL 0   /* prepare what this call's windows touch                           */
#define PTYX_PREP_FULL 1   /* prepare the whole object, for later PTYX_PREP_REUSE calls          */
#define PTYX_PREP_REUSE 2  /* reuse the previous call's preparation on this plan                */
/* Flag bit, or'ed into loss_cfg.prep by a caller that splits one optimizer step into pieces: this
 * piece may leave its probe-gradient reduction to a later piece (the stripe engine keeps
 * accumulating its per-group k-space partials and runs the reduction and inverse FFT once, on the
 * first later piece without the bit).  Until then d_probe lacks these pieces' contribution, and
 * every call on the plan must pass the same d_probe.  Engines without a deferred epilogue
 * ignore the bit. */
#define PTYX_PREP_DEFER_PROBE 4
/* PTYX_PREP_DEFER_GATHER (ptyx_forward_loss_grad_begin / _end only, ABI 208): the register engines
 * (k_fused3 / k_fused3ms: ptyx_plan_slot_floats > 0) leave the object gradient untouched and keep
 * the call's per-pattern object-gradient slots for ptyx_slots_export; the caller all-gathers them
 * over the ranks and runs ptyx_obj_gather_slots.  Another engine: PTYX_EUNSUPPORTED. */
#define PTYX_PREP_DEFER_GATHER 8
/* PTYX_PREP_GRAD_STORE (ABI 208): the call OVERWRITES d_obja / d_objp with its own object
 * gradient instead of accumulating into them (their content on entry is ignored), so a caller
 * that would zero them first need not: the register engines' gathers store, the other engines
 * clear the two arrays on the stream before they accumulate.  The other gradients accumulate as
 * usual.  (A graph-replayed optimizer step zeroes only the rest of its flat gradient buffer.) */
#define PTYX_PREP_GRAD_STORE 16
/* PTYX_PREP_FUSED_ADAM (ptyx_forward_loss_grad only, ABI 209): the call ends with the optimizer step
 * that ptyx_plan_set_adam registered on the plan (consumed by this call): what ptyx_adam_step (or
 * ptyx_adam_step_store) with those arguments would do right after the call, on the same stream.
 * The k_fused3 engine's small calls (one mini-batch per optimizer step) fold it into their epilogue
 * (k_gather_adam: the object gather, the probe gradient's row pass and the update of every tensor
 * in one launch); any other call issues the ordinary k_adam launch after its own epilogue.  Either
 * way the gradients are written as without the flag, and the results are bitwise the same. */
#define PTYX_PREP_FUSED_ADAM 32
/* PTYX_PREP_SELECT (ptyx_forward_loss_grad only, ABI 210): the call begins with what
 * ptyx_step_select(stream, idx_all, istart, cnt, n_idx, idx, grad, grad_n, steps, n_steps) does,
 * with the arguments ptyx_plan_set_select registered on the plan (consumed by this call) and the
 * call's own idx as idx_out: its pattern indices are picked on the device by the step counter, the
 * gradient buffer zeroed and the step counts advanced before any kernel reads them.  The register
 * engines' small calls do it inside their preparation launch (one launch fewer per graph-replayed
 * step); any other call issues the k_step_select launch first.  The same results either way. */
#define PTYX_PREP_SELECT 64
/* The plan records what a PTYX_PREP_FULL call prepared (engine, input pointers, loss_sparse order).
 * A PTYX_PREP_REUSE call whose engine or inputs do not match that record (or that follows a
 * PTYX_PREP_CALL call, ptyx_forward or ptyx_adjoint_dldi on the plan) prepares in full instead of
 * reusing: REUSE is a hint, never a way to read stale preparation. */

/* dims.flags */
#define PTYX_SHIFT_PROBES 1u /* sub-px Fourier-shifted probes (PtychoAD.shift_probes, models.py:120) */
#define PTYX_MEAS_F16 2u     /* measurements stored as IEEE half (fp16 storage / fp32 accumulate)   */
#define PTYX_PROP_GRAD 4u    /* plan can return dL/dH (optimised tilts / slice thickness, §8f row 4):
                                (Nz-1)·N² extra scratch and an N² slab per persistent workgroup */

typedef struct ptyx_plan ptyx_plan;

typedef struct ptyx_dims {
  int32_t N;            /* probe / DP side: any 2^a 3^b 5^c 7^d in [32, 512] (else EUNSUPPORTED)    */
  int32_t P;            /* probe modes  (opt_probe.shape[0])                               */
  int32_t O;            /* object modes (opt_obja.shape[0])                                */
  int32_t Nz;           /* object slices (opt_obja.shape[1])                               */
  int32_t Ny, Nx;       /* object extent                                                   */
  int32_t n_scans;      /* number of probe positions (crop_pos.shape[0])                   */
  int32_t max_patterns; /* largest number of patterns per call (sizes the workspace)       */
  uint32_t flags;       /* PTYX_SHIFT_PROBES | PTYX_MEAS_F16 | PTYX_PROP_GRAD              */
  int32_t abi_version;  /* = PTYX_ABI_VERSION                                              */
} ptyx_dims;

typedef struct ptyx_inputs {
  const float *obja;       /* (O,Nz,Ny,Nx) f32  PtychoAD.opt_obja                            */
  const float *objp;       /* (O,Nz,Ny,Nx) f32  PtychoAD.opt_objp                            */
  const float *probe;      /* (P,N,N,2)    f32  PtychoAD.opt_probe (view_as_real)            */
  const float *shifts;     /* (n_scans,2)  f32  PtychoAD.opt_probe_pos_shifts (y,x) px       */
  const float *H;          /* (N,N,2)      f32  PtychoAD.H, zero frequency at the corner      */
  const float *omode_occu; /* (O,)         f32                                               */
  const int32_t *crop_pos; /* (n_scans,2)  i32  integer top-left (y,x) of each patch          */
  const void *meas;        /* (rows,N,N) f32 (or f16 with PTYX_MEAS_F16), fftshifted DPs:
                              rows = n_scans, or a rank-local block addressed via meas_rows  */
  /* per-position object tilts (tilt_type 'each', get_propagators models.py:330-356): position s
   * propagates with H ⊙ exp(i dz (Ky tan(θy_s/1e3) + Kx tan(θx_s/1e3))).  NULL = none. */
  const float *obj_tilts;  /* (n_scans,2)  f32  PtychoAD.opt_obj_tilts, mrad                  */
  const float *kvec;       /* (N)          f32  propagator_grid k values (Ky[:,0] = Kx[0,:])  */
  float dz;                /* slice thickness used by the tilt ramps                           */
  /* rank-local measurement storage (the data-parallel driver keeps only the DPs of its own
   * mini-batches): meas_rows[s] = row of `meas` holding scan position s, with
   * 0 <= meas_rows[s] < meas_row_count for every s a call touches.  NULL = row s.             */
  const int32_t *meas_rows; /* (n_scans) i32 device, or NULL                                     */
  int32_t meas_row_count;   /* rows of `meas` when meas_rows is set (>= 1), else ignored         */
} ptyx_inputs;

/* Preconditions on the device arrays of every compute call (ptyx_forward, ptyx_forward_loss_grad
 * (_begin), ptyx_adjoint_dldi), for each pattern j of the call with s = idx[j]:
 *   0 <= s < n_scans;  0 <= crop_pos[s] (y, x) and crop_pos[s] + N <= (Ny, Nx);
 *   0 <= meas_rows[s] < meas_row_count (when meas_rows is set).
 * The engines check them on the device as they read the indices (no host synchronisation): a
 * violation is clamped (no out-of-bounds access) and flagged on the plan, and the NEXT compute call
 * on the plan — or ptyx_plan_check — returns PTYX_EINVAL naming it (the reference raises
 * IndexError from its advanced indexing, models.py:261-264).  ptyx_plan_check reports the flags of
 * every call whose kernels have completed (synchronise the stream first) and clears them. */
int ptyx_plan_check(ptyx_plan *plan);

typedef struct ptyx_grads {
  float *d_obja;   /* (O,Nz,Ny,Nx)  += dL/dobja                 or NULL */
  float *d_objp;   /* (O,Nz,Ny,Nx)  += dL/dobjp                 or NULL */
  float *d_probe;  /* (P,N,N,2)     += dL/dRe + i dL/dIm probe  or NULL */
  float *d_shifts; /* (n_scans,2)   += dL/dshift                or NULL */
  float *d_H;      /* (N,N,2)       += dL/dRe + i dL/dIm H      or NULL: the propagator gradient
                      behind optimised obj_tilts / slice_thickness (get_propagators cases 1, 2A, 3,
                      src/ptyrad/models.py:339-356).  Needs a PTYX_PROP_GRAD plan; runs the general
                      (two-pass) engine; Nz = 1 adds nothing (H is unused). */
  float *d_tilts;  /* (n_scans,2)   += dL/dobj_tilts (per-position tilts, mrad) or NULL; needs
                      inputs.obj_tilts and a PTYX_PROP_GRAD plan (general engine). */
  float *d_dz;     /* (1)           += the per-position tilt ramps' part of dL/d(slice_thickness)
                      (∂/∂dz of exp(i dz (Ky tan θy + Kx tan θx))) or NULL; the part through H
                      comes from d_H.  Same requirements as d_tilts. */
} ptyx_grads;

/* CombinedLoss terms on the hot path (params/loss_params.py defaults in brackets). */
typedef struct ptyx_loss_cfg {
  int32_t single_on;  float single_w, single_q;              /* loss_single [1, 1.0, 0.5]       */
  int32_t poissn_on;  float poissn_w, poissn_q, poissn_eps;  /* loss_poissn [0, 1.0, 1.0, 1e-6] */
  int32_t sparse_on;  float sparse_w; int32_t sparse_n;      /* loss_sparse [1, 0.1, 1]         */
  float grad_scale;   /* multiplies every gradient: 1/grad_accumulation, reconstruction.py:750 */
  int32_t max_batch;  /* largest mini-batch of the call, 0 = unknown (informational: engine
                         choice depends only on the geometry and the call's capacity)      */
  int32_t prep;       /* PTYX_PREP_CALL | PTYX_PREP_FULL | PTYX_PREP_REUSE                   */
} ptyx_loss_cfg;

/* Create a plan: validates dims, allocates the device workspace and twiddle tables.
 * device: HIP device ordinal the plan (and every pointer passed to it) lives on. */
int ptyx_plan_create(ptyx_plan **out, const ptyx_dims *dims, int device);
int ptyx_plan_destroy(ptyx_plan *plan);

/* dp_out (n_idx,N,N) f32 = PtychoAD.forward(idx) for the positions idx[0..n_idx). */
int ptyx_forward(ptyx_plan *plan, void *stream, const ptyx_inputs *in, const int32_t *idx,
                 int32_t n_idx, float *dp_out);

/* Fused forward + loss + adjoint over n_batches mini-batches.
 * idx[batch_offsets[b] .. batch_offsets[b+1]) are the scan indices of mini-batch b (each with its
 * own NRMSE normalisation, losses.py:45-47); gradients of all mini-batches are summed (i.e. the
 * reference's grad_accumulation over these batches, scaled by cfg->grad_scale).
 * loss_terms (n_batches,5) f32 device: [single, poissn, pacbed(=0), sparse, simlar(=0)] per batch,
 * unscaled (the values CombinedLoss returns). dp_out (n_idx,N,N) optional (NULL to skip). */
int ptyx_forward_loss_grad(ptyx_plan *plan, void *stream, const ptyx_inputs *in, const int32_t *idx,
                           const int32_t *batch_offsets, int32_t n_batches, int32_t n_idx,
                           const ptyx_loss_cfg *cfg, float *loss_terms, float *dp_out,
                           const ptyx_grads *grads);

/* The same call in two halves, for a mini-batch whose patterns are split over data-parallel ranks
 * (the reference's split_batches, utils/common.py:63 / reconstruction.py:125-132, with the
 * single-device NRMSE normalisation losses.py:45-47 kept exact).
 *
 *   _begin runs the forward model and the loss partial sums of this rank's patterns and writes,
 *     per mini-batch of the call, PTYX_BATCH_SUMS doubles to batch_sums (n_batches, 37) f64 device:
 *     [pattern count, Σ(I^q-M^q)², ΣM^q (loss_single), Σ(M^q log(I^q+ε)-I^q), ΣM^q (loss_poissn),
 *      Σ|φ|^n per object mode (loss_sparse, 32 slots)].  Every quantity is additive over patterns.
 *   the caller sums batch_sums over the ranks that hold parts of the same mini-batches (one
 *     all-reduce of n_batches·37 doubles), in place,
 *   _end takes the summed batch_sums, writes loss_terms (n_batches,5) for the WHOLE mini-batches
 *     and accumulates this rank's share of the gradients; the ranks' gradients then sum (the
 *     caller's gradient all-reduce) to the single-device gradient of the whole mini-batches.
 *
 * Arguments are those of ptyx_forward_loss_grad; the device arrays passed to _begin (inputs, idx,
 * batch_offsets, gradients, dp_out) must stay valid and unchanged until _end returns, and no other
 * compute call may run on the plan in between (PTYX_EINVAL).  The call must fit the plan in one
 * piece (n_idx <= max_patterns and, for the register engines, <= ptyx_plan_register_capacity).
 * ptyx_forward_loss_grad is _begin + _end with the call's own sums (no collective). */
#define PTYX_BATCH_SUMS 37
int ptyx_forward_loss_grad_begin(ptyx_plan *plan, void *stream, const ptyx_inputs *in, const int32_t *idx,
                                 const int32_t *batch_offsets, int32_t n_batches, int32_t n_idx,
                                 const ptyx_loss_cfg *cfg, float *dp_out, const ptyx_grads *grads,
                                 double *batch_sums);
int ptyx_forward_loss_grad_end(ptyx_plan *plan, void *stream, const double *batch_sums, float *loss_terms);

/* Slot exchange for mini-batches split over ranks (ABI 208; replaces the object part of the DDP
 * gradient all-reduce, reconstruction.py:753, for a split step).  A _begin / _end call with
 * PTYX_PREP_DEFER_GATHER keeps, per pattern, its unit-coefficient object-gradient slot
 * (ptyx_plan_slot_floats floats, an internal row order that ptyx_obj_gather_slots reads back),
 * window origin and mini-batch coefficients.  A rank's block (ptyx_slot_block_floats(cap) floats)
 * holds cap slots, then cap table rows of PTYX_SLOT_META floats (window origin, coefficients, scan
 * index, the pattern's row of the (n_scans, 2) position gradient); rows past the call's patterns
 * are padding (no effect).
 *   ptyx_slots_export: this rank's block from the last such call (use_last 0: padding only, for a
 *     rank with no part in the step); d_shifts (or NULL) is read for the position rows.
 *   ptyx_obj_gather_slots: `blocks` = the n_ranks blocks all-gathered rank by rank.  The object
 *     gradient of all n_ranks x cap rows is accumulated into d_obja / d_objp (deterministic, fixed
 *     order: identical on every rank that passes the same blocks) and the position-gradient rows
 *     of the other ranks' blocks are added into d_shifts. */
#define PTYX_SLOT_META 8
int64_t ptyx_plan_slot_floats(const ptyx_plan *plan);               /* 0: the plan keeps no slots */
int64_t ptyx_slot_block_floats(const ptyx_plan *plan, int32_t cap);  /* floats of one rank's block */
/* ptyx_plan_slot_target: the NEXT _begin / _end call with PTYX_PREP_DEFER_GATHER (of at most cap
 * patterns) writes its slots straight into `block` (this rank's block, e.g. its slice of the
 * all-gather's output: an in-place all-gather), so ptyx_slots_export only adds the table rows.
 * One call's target: cleared when that call ends; NULL clears it. */
int ptyx_plan_slot_target(ptyx_plan *plan, float *block, int32_t cap);
int ptyx_slots_export(ptyx_plan *plan, void *stream, int32_t use_last, int32_t cap, float *block,
                      const float *d_shifts);
int ptyx_obj_gather_slots(ptyx_plan *plan, void *stream, const float *blocks, int32_t n_ranks, int32_t cap,
                          int32_t self_rank, const float *obja, const float *objp, float *d_obja, float *d_objp,
                          int32_t sparse_n, float *d_shifts);
/* ptyx_obj_gather_slots, then the optimizer step ptyx_plan_set_adam registered (consumed), as
 * ptyx_adam_step[_store] would take it right after (ABI 210): the caller has made every other
 * gradient final (the probe part all-reduced).  A k_fused3 plan with one slice folds the step into
 * the gather's launch (k_gather_adam); otherwise a k_adam launch follows.  Bitwise either way. */
int ptyx_obj_gather_slots_adam(ptyx_plan *plan, void *stream, const float *blocks, int32_t n_ranks, int32_t cap,
                               int32_t self_rank, const float *obja, const float *objp, float *d_obja,
                               float *d_objp, int32_t sparse_n, float *d_shifts);

/* Adjoint for an external loss: given dLdI (n_idx,N,N) = dL/d(dp_fwd) for the patterns idx,
 * accumulate the object / probe / position gradients (autograd of PtychoAD.forward). */
int ptyx_adjoint_dldi(ptyx_plan *plan, void *stream, const ptyx_inputs *in, const int32_t *idx,
                      int32_t n_idx, const float *dLdI, float grad_scale, const ptyx_grads *grads);

/* Per-kernel timing for roofline reporting: while profiling is on, every kernel the plan
 * launches is bracketed by HIP events on its stream.  ptyx_profile_end waits for the recorded
 * events, writes up to `cap` {kernel name, launches, total milliseconds} rows and turns
 * profiling off.  (Not for graph capture: it creates events.) */
typedef struct ptyx_kernel_stat {
  char name[32];
  int32_t launches;
  float total_ms;
} ptyx_kernel_stat;
int ptyx_profile_begin(ptyx_plan *plan);
int ptyx_profile_end(ptyx_plan *plan, ptyx_kernel_stat *out, int32_t cap, int32_t *n_out);

/* ---------------------------------------------------------------------------------------------
 * Iteration-wise constraints on the device, replacing the object / probe
 * updates of CombinedConstraint.forward (src/ptyrad/constraints.py:227-246).  Same conventions
 * as above: device pointers, asynchronous on `stream`, no host synchronisation; `ws` is a
 * caller-allocated device workspace of ptyx_constraints_ws_bytes() bytes (8-byte aligned).
 * ------------------------------------------------------------------------------------------- */
typedef struct ptyx_obj_constraints {
  int32_t zblur_a, zblur_p, zblur_ks; float zblur_std;     /* obj_zblur      constraints.py:100-114 */
  int32_t cr_a, cr_p; float cr_alpha1, cr_alpha2;           /* complex_ratio  constraints.py:147-163 */
  int32_t mir_on; float mir_relax, mir_scale, mir_power;     /* mirrored_amp   constraints.py:165-179 */
  int32_t thr_on; float thr_relax, thr_lo, thr_hi;           /* obja_thresh    constraints.py:181-190 */
  int32_t pos_on, pos_subtract_min; float pos_relax;         /* objp_postiv    constraints.py:192-208 */
} ptyx_obj_constraints;

size_t ptyx_constraints_ws_bytes(void);

/* obj_rblur (constraints.py:83-98): torchvision gaussian_blur over the last two axes of
 * n_planes contiguous (Ny, Nx) f32 planes, reflect padding, kernel_size odd ≤ 15, out of place. */
int ptyx_obj_rblur(void *stream, const float *in, float *out, int32_t n_planes, int32_t Ny, int32_t Nx,
                   int32_t kernel_size, float sigma);

/* ---------------------------------------------------------------------------------------------
 * Optional forward stages.  Composed around the engine entry points by the
 * host mirror (ptyrad_amd/stages.py); same conventions as above.
 *   detector_blur_std  PtychoAD.get_forward_meas  src/ptyrad/models.py:375-382
 *                      dp = gaussian_blur(dp, 5, std): ptyx_obj_rblur on the (B,N,N) dp planes,
 *                      backward ptyx_blur_adjoint on dL/d(blurred dp).
 *   obj_preblur_std    PtychoAD.get_obj_patches   src/ptyrad/models.py:267-284
 *                      patches = gaussian_blur(get_obj_ROI(idx), 5, std) per amplitude / phase
 *                      plane: ptyx_patch_gather → ptyx_obj_rblur → engine on the patch stack;
 *                      backward ptyx_blur_adjoint → ptyx_patch_scatter_add.
 * ------------------------------------------------------------------------------------------- */

/* Transpose of ptyx_obj_rblur (reflect-padded separable Gaussian), i.e. the autograd backward
 * of torchvision gaussian_blur: out = B^T in over n_planes (Ny, Nx) f32 planes, out of place,
 * deterministic.  n_planes ≤ 65535. */
int ptyx_blur_adjoint(void *stream, const float *in, float *out, int32_t n_planes, int32_t Ny, int32_t Nx,
                      int32_t kernel_size, float sigma);

/* get_obj_ROI (models.py:251-265) for one (O,Nz,Ny,Nx) f32 plane set: patches (O,Nz,n_idx,N,N)
 * [o,z,b] = obj[o,z, crop_pos[idx[b]] + (0..N, 0..N)].  crop_pos (n_scans,2) int32, idx
 * (n_idx) int32, both device; n_idx ≤ 65535, O·Nz ≤ 65535.  Windows outside the object give 0. */
int ptyx_patch_gather(void *stream, const float *obj, int32_t O, int32_t Nz, int32_t Ny, int32_t Nx,
                      const int32_t *crop_pos, const int32_t *idx, int32_t n_idx, int32_t N, float *patches);

/* Transpose of ptyx_patch_gather: gobj += scatter(gpatches) (f32 atomics; overlapping windows
 * are summed in arrival order).  Same shapes and limits. */
int ptyx_patch_scatter_add(void *stream, const float *gpatches, int32_t O, int32_t Nz, int32_t Ny, int32_t Nx,
                           const int32_t *crop_pos, const int32_t *idx, int32_t n_idx, int32_t N, float *gobj);

/* loss_simlar's core (CombinedLoss.get_loss_simlar, src/ptyrad/losses.py:106-141):
 * x (O, n_planes, n_pix) f32 — the (blurred / resampled) patches of one type, modes outermost —,
 * occ (O) f32.  sums[q] = Σ_pix std_o(occ_o·x[o,q,pix]), the unbiased (correction 1) std over the
 * modes as torch.std(1); per plane a fixed-order reduction (deterministic).  O = 1 gives NaN, as
 * torch does.  n_planes ≤ 2^31 − 1. */
int ptyx_simlar_std(void *stream, const float *x, int32_t O, int64_t n_planes, int32_t n_pix, const float *occ,
                    float *sums);
/* Its backward: gx[o,q,pix] = gsum[q]·occ_o·(w_o − mean_o w)/((O − 1)·std), w = occ·x (torch's
 * std backward; 0/0 where the std is 0, as torch). */
int ptyx_simlar_std_grad(void *stream, const float *x, int32_t O, int64_t n_planes, int32_t n_pix, const float *occ,
                         const float *gsum, float *gx);

/* loss_pacbed (src/ptyrad/losses.py:77-89) per mini-batch, on model intensities dp (n_idx,N,N)
 * (e.g. the dp_out of ptyx_forward_loss_grad): loss_terms[m*5 + 2] = w·sqrt(mse(mean_b dp^q…)) /
 * mean(M^q) written for every batch m; dLdI (n_idx,N,N) = grad_scale · dL/d(dp) (NULL to skip),
 * which ptyx_adjoint_dldi turns into gradients.  meas (n_scans,N,N) f32 / f16 addressed through
 * idx like the engine; batch_offsets device int32.  ws: ptyx_pacbed_ws_bytes(N, n_batches) bytes
 * of device memory, 8-byte aligned; n_batches ≤ 65535; batch_offsets[n_batches] must equal n_idx.
 * Fixed-order fp64 sums (deterministic). */
size_t ptyx_pacbed_ws_bytes(int32_t N, int32_t n_batches);
int ptyx_loss_pacbed(void *stream, const float *dp, const void *meas, int32_t meas_f16, const int32_t *idx,
                     const int32_t *batch_offsets, int32_t n_batches, int32_t n_idx, int32_t N, float weight,
                     float dp_pow, float grad_scale, float *loss_terms, float *dLdI, void *ws);

/* PtychoAD.get_measurements(indices) with on-the-fly padding / resampling (models.py:384-412):
 * out (n_idx,Ho,Wo) f32 = interpolate(paste(canvas, meas[idx[b]] at (h1, w1)), scale, bilinear,
 * align_corners=False) / (scale_y·scale_x).  meas (n_scans,Hm,Wm) f32 (f16 when meas_f16);
 * canvas (Hp,Wp) f32 = on_the_fly_meas_padded, or NULL (no padding: Hp,Wp = Hm,Wm, h1 = w1 = 0);
 * scale 1,1 = no resampling; Ho,Wo = floor(Hp·scale_y), floor(Wp·scale_x).  n_idx ≤ 65535. */
int ptyx_meas_gather(void *stream, const void *meas, int32_t meas_f16, int32_t Hm, int32_t Wm, const int32_t *idx,
                     int32_t n_idx, const float *canvas, int32_t Hp, int32_t Wp, int32_t h1, int32_t w1,
                     double scale_y, double scale_x, int32_t Ho, int32_t Wo, float *out);

/* obj_zblur → complex_ratio → mirrored_amp → obja_thresh → objp_postiv on (O,Nz,Ny,Nx) f32
 * obja / objp, in place, in CombinedConstraint.forward order (kr/kz filters, which sit between
 * zblur and complex_ratio, are the caller's: call once with only zblur, filter, call again). */
int ptyx_obj_constrain(void *stream, float *obja, float *objp, int32_t O, int32_t Nz, int32_t Ny, int32_t Nx,
                       const ptyx_obj_constraints *c, void *ws);

/* fix_probe_int (constraints.py:70-81): probe (P,N,N,2) *= sqrt(*probe_int_sum / Σ|probe|²);
 * probe_int_sum is a device f32 scalar (PtychoAD.probe_int_sum, models.py:122). */
int ptyx_probe_fix_int(void *stream, float *probe, int32_t P, int32_t N, const float *probe_int_sum, void *ws);

/* ortho_pmode (constraints.py:34-41 → orthogonalize_modes_vec :255-291, sort=True): probe modes
 * (P,N,N,2), 1 ≤ P ≤ 64, replaced in place by V^H M sorted by descending power, V the
 * eigenvectors of M M^H (LAPACK geev normalisation).  Eigenvalues (P f64) land in
 * ws + ptyx_constraints_evals_offset(). */
int ptyx_probe_ortho(void *stream, float *probe, int32_t P, int32_t N, void *ws);
size_t ptyx_constraints_evals_offset(void);

/* ---------------------------------------------------------------------------------------------
 * Measurement ingest: load_raw (src/ptyrad/load.py:19-49) and
 * Initializer._process_meas (src/ptyrad/initialization.py:709-752) straight into HBM.
 * ------------------------------------------------------------------------------------------- */
typedef struct ptyx_meas_proc {
  int32_t flipud, fliplr, transpose;                 /* meas_flipT [0,0,0]            :766-792  */
  int32_t crop_ky0, crop_ky1, crop_kx0, crop_kx1;    /* meas_crop ky / kx (after flipT), -1 = whole axis;
                                                        the scan-axis crop is a frame selection  */
  int32_t neg_mode, neg_force; float neg_value;      /* meas_remove_neg_values        :837-890  
                                                        0 clip_neg, 1 subtract_min, 2 clip_value, 3 subtract_value */
  int32_t norm_mode; float norm_value;               /* meas_normalization            :892-935
                                                        0 max_at_one, 1 mean_at_one, 2 sum_to_one, 3 divide_const */
} ptyx_meas_proc;

/* Frames [first, first+count) of an EMPAD-style raw file (offset + file_frames × (H·W·4 + gap)
 * bytes, size checked like load.py:27-31) into dst (count,H,W) f32 on the device, through
 * pinned double buffers and strided DMA (gaps dropped by the copy engine).  Host-blocking. */
int ptyx_raw_read(void *stream, const char *path, int64_t offset, int32_t H, int32_t W, int32_t gap,
                  int64_t file_frames, int64_t first, int64_t count, float *dst);

/* stats (device f64, ptyx_meas_stats_len(Ho,Wo) values = [min, n, Σraw(Ho·Wo), Σapplied(Ho·Wo)],
 * initialised by the caller to {+inf, 0, 0, ...}) += the statistics of n frames raw (n,H,W) f32 after
 * flipT + crop; call once per chunk; across ranks reduce stats[0] with MIN and the rest with SUM.
 * ws: device workspace of ptyx_meas_ws_bytes(Ho,Wo) bytes. */
size_t ptyx_meas_stats_len(int32_t Ho, int32_t Wo);
size_t ptyx_meas_ws_bytes(int32_t Ho, int32_t Wo);
int ptyx_meas_stats(void *stream, const float *raw, int64_t n, int32_t H, int32_t W, const ptyx_meas_proc *p,
                    double *stats, void *ws);
/* dst (n,Ho,Wo) f32 (or IEEE half with dst_f16) = _process_meas of raw, given the complete stats. */
int ptyx_meas_finish(void *stream, const float *raw, int64_t n, int32_t H, int32_t W, const ptyx_meas_proc *p,
                     const double *stats, void *ws, void *dst, int32_t dst_f16);

/* The mean diffraction pattern of the processed (normalised) stack, mean (Ho,Wo) f64, from the
 * complete stats alone (no pass over the frames): the meas.mean(0) that _meas_pad fits its
 * background to (initialization.py:987).  ws as for ptyx_meas_finish. */
int ptyx_meas_mean(void *stream, int32_t H, int32_t W, const ptyx_meas_proc *p, const double *stats, void *ws,
                   double *mean);

/* The reference's f32 mean pattern of the stack after the negative-value rule (normalized = 0),
 * or after normalisation by p's constant (normalized = 1): numpy's meas.mean(0), i.e. a
 * sequential f32 sum over the frames in order, then / n, bit for bit.  mean (Ho,Wo) f32.  The
 * single-rank ingest takes the normalisation constant (max / mean / sum of the first) and
 * meas_pad's fit input (the second) from it; stats as for ptyx_meas_finish (the min). */
int ptyx_meas_mean_seq(void *stream, const float *raw, int64_t n, int32_t H, int32_t W, const ptyx_meas_proc *p,
                       const double *stats, void *ws, int32_t normalized, float *mean);

/* meas_pad's padded background (initialization.py:986-1025), bg (Hp,Wp) f64: the amplitude
 * amp = sqrt(mean) of the (Hm,Wm) mean pattern placed at (h1, w1) and padded by pad_type
 *   0 constant (amp = value), 1 edge, 2 linear_ramp (to value at the canvas border; numpy.pad's
 *   axis order), all three in f32 like the reference's f32 amp_avg;
 *   3 exp  a·exp(-b·r), 4 power  a·r^-b  (f64), r = distance to (Hm/2 + h1, Wm/2 + w1) + 1e-10,
 *   with (a, b) the host's curve_fit of the thresholded mean (image_proc.py:458-492);
 * then squared back to intensity and zeroed under the frame [h1, h1+Hm) × [w1, w1+Wm). */
int ptyx_meas_pad_background(void *stream, const double *mean, int32_t Hm, int32_t Wm, int32_t pad_type, double a,
                             double b, double value, int32_t Hp, int32_t Wp, int32_t h1, int32_t w1, double *bg);

/* meas_pad / meas_resample 'precompute' (initialization.py:1030-1034, 1083-1086) fused into one
 * pass: frame k of the canvas is bg (Hp,Wp) f64 with src frame k (Hm,Wm; f32, or f16 when
 * src_f16) pasted at (h1, w1) — bg NULL = no padding (Hp,Wp = Hm,Wm, h1 = w1 = 0) — and dst
 * (n,Ho,Wo) is that canvas resampled as scipy.ndimage.zoom(order=1, grid_mode=False) does
 * (output pixel o reads input coordinate o·(Hp-1)/(Ho-1)), f64 arithmetic, stored f32 (or f16
 * with dst_f16).  Ho,Wo = Hp,Wp copies the canvas (padding only). */
int ptyx_meas_pad_resample(void *stream, const void *src, int32_t src_f16, int64_t n, int32_t Hm, int32_t Wm,
                           const double *bg, int32_t Hp, int32_t Wp, int32_t h1, int32_t w1, int32_t Ho, int32_t Wo,
                           void *dst, int32_t dst_f16);

/* ---------------------------------------------------------------------------------------------
 * Optimizer-step bookkeeping for graph-replayed recon_step (reconstruction.py:658-781 at
 * grad_accumulation = 1: one step per mini-batch).  A captured step reads its mini-batch through
 * a device step counter, so one hipGraph serves every step of the same shape.
 *   ptyx_step_select: idx_out[i] = idx_all[istart[*cnt] + i] for i < n, zeroes grad[0..grad_n)
 *                     (the flat gradient buffer every trainable parameter's .grad views, or the
 *                     part of it a PTYX_PREP_GRAD_STORE call does not overwrite; any 4-byte
 *                     aligned start), and
 *                     adds 1 to *steps[j] for j < n_steps (steps: a DEVICE array of device f32
 *                     pointers, n_steps ≤ 256 — the optimizer's step counts, torch's
 *                     state_step += 1, so the step's Adam launch needs no increment launch of its
 *                     own; steps may be null with n_steps 0).
 *   ptyx_step_store:  terms_all[rstart[*cnt] + b][k] = terms[b][k] (b < nb, k < 5), then ++*cnt
 *                     (one workgroup: every thread reads *cnt before it is advanced).
 * ------------------------------------------------------------------------------------------- */
int ptyx_step_select(void *stream, const int32_t *idx_all, const int64_t *istart, const int64_t *cnt, int32_t n,
                     int32_t *idx_out, float *grad, int64_t grad_n, float *const *steps, int32_t n_steps);
int ptyx_step_store(void *stream, const float *terms, int32_t nb, const int64_t *rstart, int64_t *cnt,
                    float *terms_all);

/* The optimizer step PtyRAD takes after each accumulated gradient (reconstruction.py:758-760,
 * torch.optim.Adam / AdamW, the schema default optimizer params/recon_params.py) for n tensors in
 * one grid-filling launch (ptyrad_amd.optim): per tensor i (host arrays of device pointers, read
 * during the call only) params[i] -= Adam update from grads[i], exp_avgs[i], exp_avg_sqs[i], the
 * step count *steps[i] (f32 on the device, ALREADY incremented for this step) and lrs[i];
 * numels[i] elements.  flags: 1 = decoupled weight decay (AdamW), 2 = maximize.  torch's
 * single-tensor arithmetic (fp32 elements, fp64 bias corrections). */
int ptyx_adam_step(void *stream, int32_t n, float *const *params, const float *const *grads, float *const *exp_avgs,
                   float *const *exp_avg_sqs, const float *const *steps, const int64_t *numels, const double *lrs,
                   double beta1, double beta2, double eps, double weight_decay, int32_t flags);
/* ptyx_adam_step, then in the same launch what ptyx_step_store does (terms_all[rstart[*cnt] + b][k]
 * = terms[b][k], ++*cnt): a graph-replayed step whose optimizer is the HIP Adam needs no store
 * launch of its own.  Issues one bookkeeping-only launch when no tensor has elements. */
int ptyx_adam_step_store(void *stream, int32_t n, float *const *params, const float *const *grads,
                         float *const *exp_avgs, float *const *exp_avg_sqs, const float *const *steps,
                         const int64_t *numels, const double *lrs, double beta1, double beta2, double eps,
                         double weight_decay, int32_t flags, const float *terms, int32_t nb, const int64_t *rstart,
                         int64_t *cnt, float *terms_all);

/* Registers the step selection the plan's next ptyx_forward_loss_grad call with PTYX_PREP_SELECT
 * takes (arguments as ptyx_step_select's; steps is a DEVICE array of at most 256 pointers). */
int ptyx_plan_set_select(ptyx_plan *plan, const int32_t *idx_all, const int64_t *istart, const int64_t *cnt,
                         float *grad, int64_t grad_n, float *const *steps, int32_t n_steps);

/* Registers the optimizer step the plan's next ptyx_forward_loss_grad call with PTYX_PREP_FUSED_ADAM
 * takes (arguments as ptyx_adam_step's; the host arrays are copied, the device pointers must stay
 * valid until that call).  terms non-NULL: also what ptyx_step_store(stream, terms, nb, rstart,
 * cnt, terms_all) does (ptyx_adam_step_store).  A later ptyx_plan_set_adam replaces it. */
int ptyx_plan_set_adam(ptyx_plan *plan, int32_t n, float *const *params, const float *const *grads,
                       float *const *exp_avgs, float *const *exp_avg_sqs, const float *const *steps,
                       const int64_t *numels, const double *lrs, double beta1, double beta2, double eps,
                       double weight_decay, int32_t flags, const float *terms, int32_t nb, const int64_t *rstart,
                       int64_t *cnt, float *terms_all);

/* Patterns one ptyx_forward_loss_grad call may hold and still run on the plan's fast engine:
 * the register-resident engines' slot capacity (k_fused3 / k_fused3ms / mixed-state), the stripe
 * engine's call size, else the general engine's far-field cache capacity (calls beyond it
 * recompute the forward in k_adjoint).  0 when the plan keeps none of these.  Callers with
 * host-side batch offsets split larger calls at mini-batch boundaries (gradients accumulate). */
int64_t ptyx_plan_register_capacity(const ptyx_plan *plan);

/* Engine-variant selection for tests and A/B measurements (no environment variable changes an
 * engine): key "s3_hold" (0..4: probe/object modes k_s3 keeps in registers), "s_psi0" (0/1: the
 * stripe engine parks ψ⁰ instead of recomputing it), "s_gather" (0/1: stripe object gradient by
 * slots + gather instead of f32 atomics), "s_defer_groups" (0: the stripe engine ignores
 * PTYX_PREP_DEFER_PROBE; n > 0: k_s5 partial groups of deferring calls), "gather_split" (n >= 1:
 * the object-gradient gather splits every tile's candidates over n workgroups; the default splits
 * only grids too small to fill the GPU), "gen_wg_per_cu" (n >= 1: the general engine's persistent
 * workgroups per CU instead of its LDS / thread residency); value -1 restores the measured
 * default.  Process-wide, read by ptyx_plan_create (s_psi0, s_gather, gen_wg_per_cu) and by each
 * call (s3_hold).  Every variant computes
 * the same results.  ptyx_get_tuning returns the current value (-1 default, -2 unknown key). */
int ptyx_set_tuning(const char *key, int64_t value);
int64_t ptyx_get_tuning(const char *key);

/* Bytes of device workspace the plan holds. */
size_t ptyx_plan_workspace_bytes(const ptyx_plan *plan);
/* Last error message of the calling thread ("" if none). */
const char *ptyx_last_error(void);
/* sha1 (40 hex digits) of the sources and flags the library was built from: the loader refuses a
 * library whose id does not match the sources shipped next to it (no silently stale builds). */
const char *ptyx_build_id(void);
/* ABI version (major*100 + minor) = PTYX_ABI_VERSION. */
int ptyx_version(void);
/* sizeof of every struct of this header, in declaration order: ptyx_dims, ptyx_inputs,
 * ptyx_grads, ptyx_loss_cfg, ptyx_kernel_stat, ptyx_obj_constraints, ptyx_meas_proc.  Writes
 * min(cap, 7) values and returns 7; a binding checks its own struct sizes against them. */
int ptyx_abi_struct_sizes(size_t *out, int32_t cap);

#ifdef __cplusplus
}
#endif
#endif /* PTYX_H */
