// ptyx_stripe.hpp — the N = 256 engine (BASELINE c3: P = 8 probe × O = 2 object modes; c5: P = 4,
// fp16 DPs): forward, loss and adjoint of multislice_forward_model_vec_all (forward.py:20-80,
// Nz = 1) + CombinedLoss (losses.py:36-104) + the autograd adjoint as five
// mode-batched STRIPE passes.  Included by ptyx_kernels.hip.
//
// Why not a register-resident 2-D FFT as at N = 128 (ptyx_regfft.hpp): one 256² complex field is
// 512 KiB, exactly the whole vector register file of a CU (4 SIMDs × 512 VGPRs × 64 lanes × 4 B),
// and LDS is 160 KiB, so no CU can hold a field plus working registers.  Every 2-D transform must
// cross HBM (or the 256 MiB Infinity Cache) once.  The engine therefore spends exactly ONE round
// trip per 2-D FFT, by alternating the transform axis between passes (the second half of one 2-D
// FFT and the first half of the next run on the same in-register lines), and batches the probe /
// object modes inside each pass so that the mode sums (Σ occ|Ψ|², Σ_p g·conj(ψ⁰), Σ_o g·conj(O))
// never leave the chip:
//
//   P1  columns  v = F(P_p)·wy  → column IFFT                                     → T1[p]
//   P2  rows     ×wx → row IFFT → ψ⁰_p/N² (kept: PSI0[p]); per o: ψ⁰_p·O_o → row FFT → T23[p,o]
//                (loss_sparse window sums of |φ|ⁿ from the same object rows)
//   P3  columns  per (p,o): column FFT → Ψ = ·/N;  I = Σ occ|Ψ|² + 1e-10 (registers);  DP read,
//                loss partial sums, u = ∂ℓ/∂I per UNIT mini-batch coefficient;  per (p,o):
//                g_Ψ = 2 occ Ψ u → column IFFT                                     → T23[p,o]
//                (Ψ of the first `hold` modes stays in registers, the others' column FFTs are
//                redone; ptyx_set_tuning "s3_hold")
//   --- k_finalize: the mini-batch NRMSE coefficients c_m (losses.py:45-47) ---
//   P4  rows     per p: per o: row IFFT → g/N;  slot_o += g·conj(ψ⁰_p);  gP += g·conj(O_o);
//                row FFT(gP) → T4[p] (= T1's storage);  then dA, dφ (+ the sparse sign term)
//                scaled by c_m, f32 atomics into the object gradient (O = 1), or the slot_o
//                waves stored over T3 fields 0..O-1 for k_obj_gather (O = 2: deterministic)
//   P5  columns  per pattern: column FFT(T4[p]) → G;  slab += c_m conj(W_b) G (registers, the
//                block's stripe of the probe-gradient spectrum across its patterns);  position
//                gradient Σ 2π g·Im(F(P) W conj(G)) per pattern (Parseval, no extra FFT)
//
// A stripe is 16 lines (rows or columns) × 256 points, one 256-thread workgroup: 16 threads per
// line, 16 points per thread.  A 256-point line transform is DFT16 in registers (n = n1 + 16 n2),
// the W256^(n1·k2) twiddles, one 16×16 exchange through LDS, DFT16 again: natural order in and
// out, thread slot t holding points t + 16 r.  Row passes read / write whole 2 KiB rows; column
// passes read / write 128 B row segments (one cache line).  All intermediates are in natural
// (N, N) layout, chunked per call (the host splits calls at mini-batch boundaries:
// ptyx_plan_register_capacity).
#pragma once
#include "ptyx_common.hpp"
#include "ptyx_fused3.hpp"
#include "ptyx_regfft.hpp"

namespace ptyx {
namespace sp {

constexpr int kN = 256, kN2 = kN * kN;
constexpr int kL = 16;                 // lines per stripe
constexpr int kStripes = kN / kL;      // 16
constexpr int kXElems = kL * 272;      // LDS exchange buffer (float2), row stride padded 256 → 272
constexpr int kMaxO = 2;

// Every pass is compiled for two workgroups per CU (256 VGPRs per lane): one workgroup per CU
// measured slower (k_s3 holding 4 modes: 28 vs 21 ms at c5), three spill (k_s5 with F(P) re-read
// from L2 instead of held: 8.9 → 11.9 ms, profiles/r02/ab/r02y_s5_*).
constexpr int kPassWG = 2;

struct SArgs {
  int n, P, O, Ny, Nx, n_scans, meas_f16;
  const int* idx;        // scan index per pattern
  const int* bid;        // mini-batch per pattern
  const int2* geo;       // clamped window origin per pattern
  const float* shifts;   // (n_scans, 2)
  const float2* sxy;     // (n) this call's patterns' (sy, sx), gathered by k_s_table: one load, no
                         // idx → shifts chain in front of the passes' first barrier
  const int* mrow;       // measurement row of a scan index (NULL: the index itself)
  int mrows;             // rows of meas (meas_rows entries are clamped into [0, mrows))
  const float2* Fp;      // (P, N, N) F(probe), natural order
  const float2* oc;      // (O, Ny, Nx) A e^{iφ}
  const float* obja;
  const float* objp;
  const void* meas;
  const float* occu;
  float q, eps2;
  float q2;              // loss_poissn's dp_pow when both data terms are on (k_s3 PH 1 / 2)
  int sparse_on, sparse_n;
  float2* t14;           // (n, P, N²)   T1, later T4
  float2* t4;            // = t14 when P4 writes T4 (probe / position gradients wanted), else NULL
  float2* psi0;          // (n, P, N²) parked ψ⁰, or NULL: P4 recomputes ψ⁰ from T1 (one row IFFT)
  float2* t23;           // (n, P·O, N²) T2, later T3
  float* psum_s;         // (n, kStripes, kNSum) per-stripe loss partial sums
  float* dp_out;         // (n, N, N) or NULL
  const float* coef;     // (batches, kNCoef) from k_finalize
  int ci;                // data-term coefficient index (0 single, 1 poissn; 2: both, applied in k_s3)
  float* d_obja;
  float* d_objp;
  float2* oslot;         // non-NULL: P4 stores the object-gradient waves (unit c_m) as slots over
                         // T3 fields 0..O-1 of each pattern (k_obj_gather), instead of atomics
  float2* slabpart;      // (groups, P, N²) probe-gradient spectrum partials
  int groups;
  int slab_acc;          // 1: add to the partials an earlier call of the step left (deferred epilogue)
  float* dsp;            // (n, kStripes·P, 2) position-gradient partials
  const float2* twg;     // W256^m, m = 0..255 (fp64-rounded)
};

struct Map {
  int line, slot;
};
// COL: thread t owns column line = t & 15 of the stripe and points y = slot + 16 r (slot = t >> 4):
// one register's load is 16 consecutive columns × 4 rows per wave (128 B segments).
// ROW: line = t >> 4 (the wave holds 4 rows), points x = slot + 16 r: 128 B per 16 lanes.
template <bool COL>
__device__ __forceinline__ Map map_of(int t) {
  return COL ? Map{t & 15, t >> 4} : Map{t >> 4, t & 15};
}
// exchange slot of (line, n1, k2); both forms are bank-conflict free for the ds_write_b64 /
// ds_read_b64 lane groups of their mapping (row stride 272: the two lines of a 32-lane read group
// fall in different bank halves; the XOR spreads a 16-lane write group over 16 banks pairs)
template <bool COL>
__device__ __forceinline__ int xidx(int line, int n1, int k2) {
  return COL ? ((n1 << 4) + k2) * 16 + line : line * 272 + (n1 << 4) + (k2 ^ n1);
}

__device__ __forceinline__ int opq(int v) {
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ float opqf(float v) {
  asm volatile("" : "+v"(v));
  return v;
}

// Scheduling fence: everything above is issued before anything below.  Used after a batch of
// loads so that the 16 loads of a register array are all in flight before the first use (left
// alone, the scheduler interleaves load / wait / use one register at a time).
__device__ __forceinline__ void fence_sched() { __builtin_amdgcn_sched_barrier(0); }

// v[r] = p[r·stride] for the 16 points of a thread, all issued before any is used
__device__ __forceinline__ void ld16(float2 (&v)[16], const float2* p, int stride) {
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = p[r * stride];
  fence_sched();
}

// The 16 points of a thread in one field through a buffer resource: the field base is uniform
// (SGPRs), the thread's byte offset one opaque VGPR, the per-point offsets constants.  With plain
// pointers every point of a column access (32 KiB apart, beyond the immediate range) needs its
// own 64-bit address, and those get hoisted out of the mode / pattern loops: 32 VGPRs per array,
// the spills of k_s4.
constexpr unsigned kFieldBytes = kN2 * 8;
constexpr int kColStride = kL * kN * 8;   // column pass: a thread's points are 16 rows apart
constexpr int kRowStride = kL * 8;        // row pass: 16 columns apart
template <int STRIDE>
__device__ __forceinline__ void ldb(float2 (&v)[16], const float2* base, unsigned bytes, int voff) {
  const f3::Rsrc r = f3::rsrc(base, bytes);
  const int vo = opq(voff);
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = f3::ld2(r, vo, k * STRIDE);
  fence_sched();
}
template <int STRIDE>
__device__ __forceinline__ void stb(const float2 (&v)[16], float2* base, unsigned bytes, int voff) {
  const f3::Rsrc r = f3::rsrc(base, bytes);
  const int vo = opq(voff);
#pragma unroll
  for (int k = 0; k < 16; ++k) f3::st2(v[k], r, vo, k * STRIDE);
}
// The same for the per-call intermediate fields (T1…T4, ψ⁰, slots: written once, read once by
// another pass) are marked non-temporal (aux "nt"), so they do not displace the
// lines that are re-read (F(P), the object rows, the twiddles).  Measured (profiles/r02/ab/
// r02y_nt_*): c5 222 → 229 k, c3 72.7 → 75.8 k patterns/s.
constexpr int kStreamAux = 2;
template <int STRIDE>
__device__ __forceinline__ void lds_(float2 (&v)[16], const float2* base, unsigned bytes, int voff) {
  const f3::Rsrc r = f3::rsrc(base, bytes);
  const int vo = opq(voff);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const auto u = __builtin_amdgcn_raw_buffer_load_b64(r, vo + k * STRIDE, 0, kStreamAux);
    v[k] = make_float2(__uint_as_float(u[0]), __uint_as_float(u[1]));
  }
  fence_sched();
}
template <int STRIDE>
__device__ __forceinline__ void sts_(const float2 (&v)[16], float2* base, unsigned bytes, int voff) {
  const f3::Rsrc r = f3::rsrc(base, bytes);
  const int vo = opq(voff);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const __attribute__((ext_vector_type(2))) unsigned u = {__float_as_uint(v[k].x), __float_as_uint(v[k].y)};
    __builtin_amdgcn_raw_buffer_store_b64(u, r, vo + k * STRIDE, 0, kStreamAux);
  }
}
// object window of pattern j (origin g0), mode o: base and byte size
__device__ __forceinline__ const float2* win_base(const SArgs& a, int o, int2 g0) {
  return a.oc + ((size_t)o * a.Ny + g0.x) * a.Nx + g0.y;
}
__device__ __forceinline__ unsigned win_bytes(const SArgs& a) { return (unsigned)(((kN - 1) * a.Nx + kN) * 8); }

// 256-point DFT of every line of the stripe (DIR -1 forward, +1 unnormalised inverse).
template <int DIR, bool COL>
__device__ __forceinline__ void fft_line(float2 (&v)[16], Map m, float2* xb, const float2* tw) {
  float2 w[15];
  // (an opaque slot: the compiler would otherwise hoist these 30 loop-invariant registers out of
  // the mode / pattern loops of the calling pass)
  const int sl = opq(m.slot);
#pragma unroll
  for (int k2 = 1; k2 < 16; ++k2) w[k2 - 1] = tw[(sl * k2) & 255];
  fence_sched();
  rf::dft<16, DIR>(v);   // over n2: v[k2]
#pragma unroll
  for (int k2 = 1; k2 < 16; ++k2) {
    float2 t = w[k2 - 1];
    if (DIR > 0) t.y = -t.y;
    v[k2] = cmul(v[k2], t);
  }
#pragma unroll
  for (int k2 = 0; k2 < 16; ++k2) xb[xidx<COL>(m.line, m.slot, k2)] = v[k2];
  __syncthreads();
#pragma unroll
  for (int n1 = 0; n1 < 16; ++n1) v[n1] = xb[xidx<COL>(m.line, n1, m.slot)];
  __syncthreads();
  rf::dft<16, DIR>(v);   // over n1: v[k1] = X[slot + 16 k1]
}

__device__ __forceinline__ float shift_g(int k) { return (float)((k + kN / 2) & (kN - 1)) * (1.0f / kN); }

// Sub-pixel ramps (image_proc.py:531).  A thread's points are k = slot + 16 r (slot < 16), so
// (k + N/2) mod N wraps exactly at r = 8 for every thread:
//   g(slot + 16 r) = slot/256 + h_r,   h_r = 1/2 + r/16 (r < 8),  (r − 8)/16 (r ≥ 8),
// and cis(−s·g) = cis(−s·slot/256) · cis(−s·h_r): one per-thread factor and 16 factors shared by
// the workgroup (an LDS row written by 16 threads) instead of 16 sin/cos pairs per thread.
__device__ __forceinline__ float ramp_h(int r) { return r < 8 ? 0.5f + (float)r * (1.0f / 16) : (float)(r - 8) * (1.0f / 16); }
// threads 0..15 write the shared factors of shift s into rl[16] (visible after the next barrier)
__device__ __forceinline__ void ramp_row(float2* rl, float s) {
  if (threadIdx.x < 16) rl[threadIdx.x] = f3::cis_rev(-s * ramp_h((int)threadIdx.x));
}
// the per-thread factor cis(−s·slot/256)
__device__ __forceinline__ float2 ramp_t(float s, int slot) { return f3::cis_rev(-s * ((float)slot * (1.0f / kN))); }

__device__ __forceinline__ void load_tw(float2* tw, const float2* twg) {
  for (int i = threadIdx.x; i < kN; i += blockDim.x) tw[i] = twg[i];
}

__device__ __forceinline__ int scan_of(const SArgs& a, int j) { return min(max(a.idx[j], 0), a.n_scans - 1); }

// workgroup (4 waves) sum of NV floats, fixed order, result valid in every thread
template <int NV>
__device__ __forceinline__ void bsum(float (&v)[NV], float* red) {
  f3::block_sum4<NV>(v, red);
}

// ---------------------------------------------------------------------------------- P1
// grid (n, kStripes, P): columns kx of F(P_p)·wy → column IFFT → T1[j][p]
__global__ __launch_bounds__(256, kPassWG) void k_s1(SArgs a) {
  __shared__ float2 xb[kXElems];
  __shared__ float2 tw[kN];
  __shared__ float2 rl[16];
  const int j = blockIdx.x, s = blockIdx.y, p = blockIdx.z;
  const Map m = map_of<true>(opq(threadIdx.x));
  const int kx = s * kL + m.line;
  const int vcol = (m.slot * kN + kx) * 8;
  float2 v[16];
  ldb<kColStride>(v, a.Fp + (size_t)p * kN2, kFieldBytes, vcol);   // (in flight during the setup)
  const float sy = a.sxy[j].x;
  load_tw(tw, a.twg);
  ramp_row(rl, sy);
  __syncthreads();
  const float2 T = ramp_t(sy, m.slot);
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = f3::pcm(v[r], f3::pcm(T, rl[r]));
  fft_line<+1, true>(v, m, xb, tw);
  sts_<kColStride>(v, a.t14 + ((size_t)j * a.P + p) * kN2, kFieldBytes, vcol);
}

// ---------------------------------------------------------------------------------- P2
// grid (n, kStripes): rows y of every probe mode: ×wx → row IFFT → ψ⁰ (PSI0); ×O_o → row FFT → T2
template <int O_>
__global__ __launch_bounds__(256, kPassWG) void k_s2(SArgs a) {
  __shared__ float2 xb[kXElems];
  __shared__ float2 tw[kN];
  __shared__ float red[4 * kMaxO];
  __shared__ float2 rl[16];
  const int j = blockIdx.x, s = blockIdx.y;
  const float sx = a.sxy[j].y;
  load_tw(tw, a.twg);
  ramp_row(rl, sx);
  __syncthreads();
  const Map m = map_of<false>(opq(threadIdx.x));
  const int y = s * kL + m.line;
  const float2 T = ramp_t(sx, m.slot);
  const int2 g0 = a.geo[j];
  const int P = a.P;
  constexpr float inv_n2 = 1.0f / kN2;
  // this stripe of the object window (O_o does not depend on the probe mode: loaded once)
  const int vrow = (y * kN + m.slot) * 8, vwin = (y * a.Nx + m.slot) * 8;
  float2 ob[O_][16];
#pragma unroll
  for (int o = 0; o < O_; ++o) ldb<kRowStride>(ob[o], win_base(a, o, g0), win_bytes(a), vwin);
  // the next probe mode's T1 rows are prefetched during this mode's transforms (O = 1: the
  // registers of a second object mode would not fit beside them)
  constexpr bool PREF = O_ == 1;
  float2 nxt[16];
  if constexpr (PREF) lds_<kRowStride>(nxt, a.t14 + (size_t)j * P * kN2, kFieldBytes, vrow);
  for (int p = 0; p < P; ++p) {
    float2 v[16];
    if constexpr (PREF) {
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = nxt[r];
      if (p + 1 < P) lds_<kRowStride>(nxt, a.t14 + ((size_t)j * P + p + 1) * kN2, kFieldBytes, vrow);
    } else {
      lds_<kRowStride>(v, a.t14 + ((size_t)j * P + p) * kN2, kFieldBytes, vrow);
    }
    const float2* rlo = rl + opq(0);   // (re-read per mode, not hoisted into 32 registers)
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = f3::pcm(v[r], f3::pcm(T, rlo[r]));
    fft_line<+1, false>(v, m, xb, tw);
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = cscale(v[k], inv_n2);
    if (a.psi0) sts_<kRowStride>(v, a.psi0 + ((size_t)j * P + p) * kN2, kFieldBytes, vrow);
    rf::sfor<0, O_>([&](auto OO) {
      constexpr int o = decltype(OO)::value;
      float2 u[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) u[k] = cmul(v[k], ob[o][k]);
      fft_line<-1, false>(u, m, xb, tw);
      sts_<kRowStride>(u, a.t23 + ((size_t)j * P * O_ + p * O_ + o) * kN2, kFieldBytes, vrow);
    });
  }
  // loss_sparse (losses.py:101): Σ |φ|ⁿ over this stripe of the window, per object mode
  float sp[O_];
#pragma unroll
  for (int o = 0; o < O_; ++o) {
    sp[o] = 0.f;
    if (a.sparse_on) {
      const float* prow = a.objp + ((size_t)o * a.Ny + g0.x + y) * a.Nx + g0.y + m.slot;
      float ph[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) ph[k] = prow[16 * k];
      fence_sched();
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const float ap = fabsf(ph[k]);
        sp[o] += a.sparse_n == 1 ? ap : powq(ap, (float)a.sparse_n);
      }
    }
  }
  bsum<O_>(sp, red);
  if (threadIdx.x == 0) {
    float* ps = a.psum_s + ((size_t)j * kStripes + s) * kNSum + kSumBase;
#pragma unroll
    for (int o = 0; o < O_; ++o) ps[o] = sp[o];
  }
}

// ---------------------------------------------------------------------------------- P3
// grid (n, kStripes): columns kx of every mode: column FFT → Ψ, intensity, loss, g_Ψ → column IFFT.
// The first HOLD modes keep Ψ in registers between the two sweeps; the column FFTs of the others
// (P·O − HOLD of them) are redone in the second sweep.
//
// PH (loss_single + loss_poissn together, whose two mini-batch coefficients cannot be factored out
// of one unit-coefficient field): 1 = the loss partial sums of both terms (and dp_out) only, no
// stores to T3;  2 = after k_finalize, g_Ψ with ∂ℓ/∂I = c_single u_single + c_poissn u_poissn of the
// pattern's mini-batch (the later passes then take coefficient 1: SArgs.ci = 2).  0 = one term.
template <bool SINGLE, int QM, int HOLD, int PH = 0>
__global__ __launch_bounds__(256, kPassWG) void k_s3(SArgs a) {
  __shared__ float2 xb[kXElems];
  __shared__ float2 tw[kN];
  __shared__ float red[16];   // 4 waves × up to 4 sums (PH 1)
  load_tw(tw, a.twg);
  __syncthreads();
  const int j = blockIdx.x, s = blockIdx.y;
  const Map m = map_of<true>(opq(threadIdx.x));
  const int kx = s * kL + m.line;
  const int PO = a.P * a.O;   // ≥ HOLD (host)
  const int O = a.O;
  constexpr float inv_n = 1.0f / kN;
  float2* base = a.t23 + (size_t)j * PO * kN2;
  const int vcol = (m.slot * kN + kx) * 8;
  auto far_field = [&](int q, float2 (&v)[16]) {
    ldb<kColStride>(v, base + (size_t)q * kN2, kFieldBytes, vcol);   // (modes past the hold are read again)
    fft_line<-1, true>(v, m, xb, tw);
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = cscale(v[k], inv_n);
  };
  float I[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) I[k] = 0.f;
  float2 hold[HOLD > 0 ? HOLD : 1][16];
  rf::sfor<0, HOLD>([&](auto QQ) {
    constexpr int q = decltype(QQ)::value;
    far_field(q, hold[q]);
    const float occ = a.occu[q % O];
#pragma unroll
    for (int k = 0; k < 16; ++k) I[k] = fmaf(occ, cabs2(hold[q][k]), I[k]);
  });
  for (int q = HOLD; q < PO; ++q) {
    float2 v[16];
    far_field(q, v);
    const float occ = a.occu[q % O];
#pragma unroll
    for (int k = 0; k < 16; ++k) I[k] = fmaf(occ, cabs2(v[k]), I[k]);
  }
  // loss at every point of the stripe (fftshifted DP index), unit-coefficient ∂ℓ/∂I (PH 2: scaled)
  const int sidx = scan_of(a, j);
  const size_t mi = (size_t)meas_row(a.mrow, a.mrows, sidx);
  const int col = (kx + kN / 2) & (kN - 1);
  float Mv[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int e = ((m.slot + 16 * k + kN / 2) & (kN - 1)) * kN + col;
    Mv[k] = a.meas_f16 ? __half2float(reinterpret_cast<const __half*>(a.meas)[mi * kN2 + e])
                       : reinterpret_cast<const float*>(a.meas)[mi * kN2 + e];
  }
  fence_sched();
  float S = 0.f, Ms = 0.f, u[16];
  if constexpr (PH == 1) {   // both terms' partial sums, no ∂ℓ/∂I
    float S2 = 0.f, Ms2 = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int ky = m.slot + 16 * k;
      const int e = ((ky + kN / 2) & (kN - 1)) * kN + col;
      const float Iv = I[k] + kDpEps;
      if (a.dp_out) a.dp_out[(size_t)j * kN2 + e] = Iv;
      (void)f3::loss_point<QM, true>(Iv, Mv[k], a.q, a.eps2, S, Ms);
      (void)f3::loss_point<2, false>(Iv, Mv[k], a.q2, a.eps2, S2, Ms2);
    }
    float v4[4] = {S, Ms, S2, Ms2};
    bsum<4>(v4, red);
    if (threadIdx.x == 0) {
      float* ps = a.psum_s + ((size_t)j * kStripes + s) * kNSum;
#pragma unroll
      for (int i = 0; i < 4; ++i) ps[i] = v4[i];
    }
    return;
  } else if constexpr (PH == 2) {
    const int mb = a.bid[j];
    const float c1 = a.coef[(size_t)mb * kNCoef + 0], c2 = a.coef[(size_t)mb * kNCoef + 1];
    float d0 = 0.f, d1 = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float Iv = I[k] + kDpEps;
      u[k] = fmaf(c1, f3::loss_point<QM, true>(Iv, Mv[k], a.q, a.eps2, d0, d1),
                  c2 * f3::loss_point<2, false>(Iv, Mv[k], a.q2, a.eps2, d0, d1));
    }
  } else {
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int ky = m.slot + 16 * k;
    const int e = ((ky + kN / 2) & (kN - 1)) * kN + col;
    const float Iv = I[k] + kDpEps;
    const float M = Mv[k];
    if (a.dp_out) a.dp_out[(size_t)j * kN2 + e] = Iv;
    u[k] = f3::loss_point<QM, SINGLE>(Iv, M, a.q, a.eps2, S, Ms);
  }
  {
    float v2[2] = {S, Ms};
    bsum<2>(v2, red);
    if (threadIdx.x == 0) {
      float* ps = a.psum_s + ((size_t)j * kStripes + s) * kNSum;
      const int b0 = SINGLE ? 0 : 2;
      ps[b0] = v2[0];
      ps[b0 + 1] = v2[1];
      ps[2 - b0] = 0.f;
      ps[3 - b0] = 0.f;
    }
  }
  }
  // g_Ψ = 2 occ Ψ u → column IFFT, in place over T2
  auto back = [&](int q, float2 (&v)[16]) {
    const float c = 2.0f * a.occu[q % O];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = cscale(v[k], c * u[k]);
    fft_line<+1, true>(v, m, xb, tw);
    sts_<kColStride>(v, base + (size_t)q * kN2, kFieldBytes, vcol);
  };
  for (int q = HOLD; q < PO; ++q) {
    float2 v[16];
    far_field(q, v);
    back(q, v);
  }
  rf::sfor<0, HOLD>([&](auto QQ) {
    constexpr int q = decltype(QQ)::value;
    back(q, hold[q]);
  });
}

// ---------------------------------------------------------------------------------- P4
// grid (n, kStripes): rows y: per p: per o: row IFFT → g;  slot_o += g conj(ψ⁰_p);
// gP += g conj(O_o);  row FFT(gP) → T4.  Then the object gradient (× c_m) by f32 atomics.
// PARK: ψ⁰ was parked by P2 (read once per probe mode; reading it after each object mode's
// transform instead, so that it is not live across the FFTs, measured slower: c3 k_s4 76 → 99 ms);
// else recomputed from T1 (one row IFFT per probe mode).
template <int O_, bool PARK>
__global__ __launch_bounds__(256, kPassWG) void k_s4(SArgs a) {
  __shared__ float2 xb[kXElems];
  __shared__ float2 tw[kN];
  // O_ = 2: the per-probe-mode accumulator gP lives in LDS ([k][thread], conflict free), so the
  // two object-mode slot accumulators fit the registers of two workgroups per CU
  constexpr bool GP_LDS = O_ > 1;
  __shared__ float2 gpl[GP_LDS ? 16 * 256 : 1];
  // O_ = 1: the object stripe is read from HBM once and kept in LDS ([k][thread], each thread
  // reads back only its own points: no barrier) for the P probe modes
  constexpr bool OB_LDS = O_ == 1;
  __shared__ float2 obl[OB_LDS ? 16 * 256 : 1];
  __shared__ float2 rl[16];
  const int j = blockIdx.x, s = blockIdx.y;
  const float sx = a.sxy[j].y;
  load_tw(tw, a.twg);
  if constexpr (!PARK) ramp_row(rl, sx);
  __syncthreads();
  const Map m = map_of<false>(opq(threadIdx.x));
  const int y = s * kL + m.line;
  const int2 g0 = a.geo[j];
  const int P = a.P;
  const int mb = a.bid[j];
  constexpr float inv_n = 1.0f / kN;
  const bool want_t4 = a.t4 != nullptr;
  constexpr float inv_n2 = 1.0f / kN2;
  float2 so[O_][16];
#pragma unroll
  for (int o = 0; o < O_; ++o)
#pragma unroll
    for (int k = 0; k < 16; ++k) so[o][k] = make_float2(0.f, 0.f);
  const int vrow = (y * kN + m.slot) * 8, vwin = (y * a.Nx + m.slot) * 8;
  if constexpr (OB_LDS) {
    float2 ob[16];
    ldb<kRowStride>(ob, win_base(a, 0, g0), win_bytes(a), vwin);
#pragma unroll
    for (int k = 0; k < 16; ++k) obl[k * 256 + threadIdx.x] = ob[k];
  }
  for (int p = 0; p < P; ++p) {
    float2 psr[16];
    if constexpr (PARK) {
      lds_<kRowStride>(psr, a.psi0 + ((size_t)j * P + p) * kN2, kFieldBytes, vrow);
    } else {   // ψ⁰_p = F⁻¹_x(wx · T1_p)/N² again: one row transform instead of a parked field
      lds_<kRowStride>(psr, a.t14 + ((size_t)j * P + p) * kN2, kFieldBytes, vrow);
      const float2 T = ramp_t(opqf(sx), m.slot);
      const float2* rlo = rl + opq(0);
#pragma unroll
      for (int r = 0; r < 16; ++r) psr[r] = f3::pcm(psr[r], f3::pcm(T, rlo[r]));
      fft_line<+1, false>(psr, m, xb, tw);
#pragma unroll
      for (int k = 0; k < 16; ++k) psr[k] = cscale(psr[k], inv_n2);
    }
    float2 gp[GP_LDS ? 1 : 16];
    if constexpr (!GP_LDS) {
#pragma unroll
      for (int k = 0; k < 16; ++k) gp[k] = make_float2(0.f, 0.f);
    }
    rf::sfor<0, O_>([&](auto OO) {
      constexpr int o = decltype(OO)::value;
      float2 v[16], ob[16];
      lds_<kRowStride>(v, a.t23 + ((size_t)j * P * O_ + p * O_ + o) * kN2, kFieldBytes, vrow);
      fft_line<+1, false>(v, m, xb, tw);
      const float2(&psi)[16] = psr;
      if constexpr (OB_LDS) {
        const int t = opq(threadIdx.x);   // (not hoisted out of the p loop: 32 registers)
#pragma unroll
        for (int k = 0; k < 16; ++k) ob[k] = obl[k * 256 + t];
      } else {
        ldb<kRowStride>(ob, win_base(a, o, g0), win_bytes(a), vwin);   // (L2: re-read per p)
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const float2 g = cscale(v[k], inv_n);
        so[o][k] = cadd(so[o][k], cmulc(g, psi[k]));
        const float2 h = cmulc(g, ob[k]);
        if constexpr (GP_LDS) {
          float2& e = gpl[k * 256 + threadIdx.x];
          e = o == 0 ? h : cadd(e, h);
        } else {
          gp[k] = cadd(gp[k], h);
        }
      }
    });
    if (want_t4) {
      float2 gq[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) gq[k] = GP_LDS ? gpl[k * 256 + threadIdx.x] : gp[GP_LDS ? 0 : k];
      fft_line<-1, false>(gq, m, xb, tw);
      sts_<kRowStride>(gq, a.t4 + ((size_t)j * P + p) * kN2, kFieldBytes, vrow);   // over T1_p's rows (read above)
    }
  }
  if (!a.d_obja && !a.d_objp) return;
  if (a.oslot) {
    // slot o of pattern j = T3 field (p = 0, o), whose rows of this stripe were consumed above
    // (no other workgroup touches them): natural (N, N) rows, c_m applied by k_obj_gather
#pragma unroll
    for (int o = 0; o < O_; ++o) sts_<kRowStride>(so[o], a.oslot + ((size_t)j * P * O_ + o) * kN2, kFieldBytes, vrow);
    return;
  }
  // object gradient.  The slot accumulators are re-mapped through the (now free) exchange buffer
  // so that each wave owns 4 whole rows: every atomic / object load is 256 contiguous bytes per
  // wave instruction (the full-rate shape of global float atomics) instead of 4 × 64 B.
  const float c = a.ci == 2 ? 1.f : a.coef[(size_t)mb * kNCoef + a.ci];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int o = 0; o < O_; ++o) {
    const float csp = a.sparse_on ? a.coef[(size_t)mb * kNCoef + 2 + o] : 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) xb[m.line * 272 + m.slot + 16 * k] = so[o][k];
    __syncthreads();
    float Ar[16], Pr[16];
    float2 gv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int r = 4 * wv + (i >> 2), xx = lane + 64 * (i & 3);
      const size_t off = ((size_t)o * a.Ny + g0.x + s * kL + r) * a.Nx + g0.y + xx;
      Ar[i] = a.obja[off];
      Pr[i] = a.objp[off];
      gv[i] = xb[r * 272 + xx];
    }
    fence_sched();
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int r = 4 * wv + (i >> 2), xx = lane + 64 * (i & 3);
      const size_t off = ((size_t)o * a.Ny + g0.x + s * kL + r) * a.Nx + g0.y + xx;
      const float A = Ar[i], ph = Pr[i];
      float sn, cs;
      phase_sincos(ph, &sn, &cs);
      const float2 gO = cscale(gv[i], c);
      if (a.d_obja) atomicAdd(a.d_obja + off, fmaf(gO.x, cs, gO.y * sn));   // Re(g_O e^{-iφ})
      if (a.d_objp) {
        float dph = A * fmaf(gO.y, cs, -gO.x * sn);                          // Im(conj(O) g_O)
        if (csp != 0.f) {
          const float sg = ph > 0.f ? 1.f : (ph < 0.f ? -1.f : 0.f);
          dph += a.sparse_n == 1 ? csp * sg : csp * powq(fabsf(ph), (float)(a.sparse_n - 1)) * sg;
        }
        atomicAdd(a.d_objp + off, dph);
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------- P5
// grid (kStripes, P, groups): block (s, p, g) sweeps patterns g, g + groups, ...: column FFT of
// T4[p] → G;  slab += c_m conj(W_b) G (kept in registers across the sweep);  position-gradient
// partials per pattern.  The slab stripe is written once at the end (k_slab_reduce sums groups);
// with slab_acc it starts from the partial an earlier call of the step stored there.
__global__ __launch_bounds__(256, kPassWG) void k_s5(SArgs a) {
  __shared__ float2 xb[kXElems];
  __shared__ float2 tw[kN];
  __shared__ float red[8];
  __shared__ float2 rl[2][16];   // the shared ramp factors of the pattern in flight (double-buffered)
  load_tw(tw, a.twg);
  __syncthreads();
  const int s = blockIdx.x, p = blockIdx.y, gi = blockIdx.z;
  const Map m = map_of<true>(opq(threadIdx.x));
  const int kx = s * kL + m.line;
  const int P = a.P;
  constexpr float two_pi_n2 = 6.283185307179586f / (float)kN2;
  const int vcol = (m.slot * kN + kx) * 8;
  // F(P)'s stripe is held in 32 VGPRs across the sweep
  float2 acc[16];
  float2 fp[16];
  ldb<kColStride>(fp, a.Fp + (size_t)p * kN2, kFieldBytes, vcol);
  if (a.slab_acc) {
    ldb<kColStride>(acc, a.slabpart + ((size_t)gi * P + p) * kN2, kFieldBytes, vcol);
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) acc[k] = make_float2(0.f, 0.f);
  }
  const float gx = shift_g(kx);
  float2 nxt[16];   // the next pattern's stripe is in flight during this pattern's transform
  if (gi < a.n) lds_<kColStride>(nxt, a.t14 + ((size_t)gi * P + p) * kN2, kFieldBytes, vcol);
  // the next pattern's shifts and mini-batch are loaded one pattern ahead too
  float2 sh_n = gi < a.n ? a.sxy[gi] : make_float2(0.f, 0.f);
  int bid_n = gi < a.n ? a.bid[gi] : 0;
  for (int j = gi, it = 0; j < a.n; j += a.groups, ++it) {
    const float sy = sh_n.x, sx = sh_n.y;
    const float c = a.ci == 2 ? 1.f : a.coef[(size_t)bid_n * kNCoef + a.ci];
    if (j + a.groups < a.n) {
      sh_n = a.sxy[j + a.groups];
      bid_n = a.bid[j + a.groups];
    }
    // (written here, read after fft_line's barriers; the other copy may still be read by threads
    // finishing the previous pattern)
    float2* rlj = rl[it & 1];
    ramp_row(rlj, sy);
    float2 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = nxt[r];
    if (j + a.groups < a.n) lds_<kColStride>(nxt, a.t14 + ((size_t)(j + a.groups) * P + p) * kN2, kFieldBytes, vcol);
    fft_line<-1, true>(v, m, xb, tw);
    const float2 TW = f3::pcm(ramp_t(sy, m.slot), f3::cis_rev(-sx * gx));   // cis(−sy·slot/N)·wx
    float sy_acc = 0.f, sim = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int ky = m.slot + 16 * k;
      const float gyk = shift_g(ky);
      const float2 W = f3::pcm(TW, rlj[k]);
      const float2 FW = cmul(fp[k], W);
      const float im = fmaf(FW.y, v[k].x, -FW.x * v[k].y);   // Im(F(P) W conj(G))
      sy_acc = fmaf(gyk, im, sy_acc);
      sim += im;
      const float2 t = cmulc(v[k], W);                        // G conj(W)
      acc[k].x = fmaf(c, t.x, acc[k].x);
      acc[k].y = fmaf(c, t.y, acc[k].y);
    }
    float ds[2] = {sy_acc, gx * sim};
    bsum<2>(ds, red);
    if (threadIdx.x == 0) {
      float* o = a.dsp + (((size_t)j * kStripes + s) * P + p) * 2;
      o[0] = ds[0] * c * two_pi_n2;
      o[1] = ds[1] * c * two_pi_n2;
    }
  }
  stb<kColStride>(acc, a.slabpart + ((size_t)gi * P + p) * kN2, kFieldBytes, vcol);
}

// ---------------------------------------------------------------------------------- small kernels
// pattern → (mini-batch, clamped window origin)
__global__ void k_s_table(const int* idx, int n, const int* boff, int n_batches, const int* crop, int n_scans, int Ny,
                          int Nx, int* bid, int2* geo, const float* shifts, float2* sxy, int* err, const int* mrow,
                          int mrows) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  check_pattern(err, idx[j], n_scans, crop, Ny, Nx, kN, mrow, mrows);
  int lo = 0, hi = n_batches;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (boff[mid] <= j) lo = mid;
    else hi = mid;
  }
  bid[j] = lo;
  const int s = min(max(idx[j], 0), n_scans - 1);
  geo[j] = make_int2(min(max(crop[2 * s], 0), Ny - kN), min(max(crop[2 * s + 1], 0), Nx - kN));
  sxy[j] = make_float2(shifts[2 * s], shifts[2 * s + 1]);
}

// psums[j][i] = Σ_stripes psum_s[j][s][i]   (fixed order)
__global__ void k_s_psum(const float* psum_s, int n, float* psums) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * kNSum) return;
  const int j = t / kNSum, i = t % kNSum;
  float acc = 0.f;
  for (int s = 0; s < kStripes; ++s) acc += psum_s[((size_t)j * kStripes + s) * kNSum + i];
  psums[(size_t)j * kNSum + i] = acc;
}

// d_shifts[idx[j]] += Σ over the pattern's stripe / mode partials (fixed order)
__global__ void k_s_shift(const float* dsp, int n, int per, const int* idx, int n_scans, float* d_shifts) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  float y = 0.f, x = 0.f;
  for (int i = 0; i < per; ++i) {
    y += dsp[((size_t)j * per + i) * 2];
    x += dsp[((size_t)j * per + i) * 2 + 1];
  }
  const int s = min(max(idx[j], 0), n_scans - 1);
  atomicAdd(d_shifts + 2 * s, y);
  atomicAdd(d_shifts + 2 * s + 1, x);
}

}  // namespace sp
}  // namespace ptyx
