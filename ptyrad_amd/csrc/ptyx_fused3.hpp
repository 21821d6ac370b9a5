// ptyx_fused3.hpp — one-pass forward / loss / adjoint for N = 128, P = O = Nz = 1 (the bench
// configuration c2, and c1) on the register-resident FFT of ptyx_regfft.hpp.  Included by
// ptyx_kernels.hip.
//
// One 256-thread workgroup owns one pattern; two workgroups per CU (64 KiB LDS, ≤ 256 VGPRs
// each), so two patterns are in flight per CU and one hides the other's barrier and memory
// waits.  Per pattern (reference forward.py:20-80, losses.py:36-104, autograd):
//
//   K layout  v = F(P)·W_b                     F(P) K-packed, W_b = exp(-2πi s_b·g) (image_proc.py:531)
//   IFFT  →   ψ⁰ = F⁻¹(v)/N²                   R layout; ψ⁰ parked in this pattern's slot
//             ψ  = ψ⁰·O                        O = A e^{iφ} precomputed per call (k_obj_prep)
//   FFT   →   Ψ  = F(ψ)/N                      the DP streams HBM → LDS (LDS-DMA) meanwhile
//             I  = occ|Ψ|² + 1e-10, loss partial sums, g_Ψ/c_m = 2 occ Ψ ∂ℓ/∂I (unit coefficient)
//   IFFT  →   g  = F⁻¹(g_Ψ)/N                  R layout
//             slot = g·conj(ψ⁰)   (object gradient per unit c_m; k_obj_gather reduces the slots)
//             h    = g·conj(O)
//   FFT   →   G  = F(h)                        K layout
//             slab += G conj(W_b);  d_shift sums += Σ g·Im(F(P) W_b conj(G))   (unit c_m; scaled
//             by c_m after k_finalize: k_segslab_reduce, k_shift_apply)
//
// Every global operand is laid out so that one register's access is contiguous across lanes:
// F(P) and the slab are K-packed ([k][thread]); slots are stored row-permuted
// (row' = 2(y & 63) + (y >> 6)); object rows are read 2 × 256 B per wave instruction; the DP
// lands in LDS through 1 KiB global_load_lds_dwordx4 instructions with an XOR-swizzled source
// so that the K-layout ds_read_b128 of it are bank-conflict free.
// The sparse loss needs no per-pattern FFT work: its window sums come from per-row prefix
// sums (k_obj_prep, k_pattern_table3).
#pragma once
#include "ptyx_common.hpp"
#include "ptyx_regfft.hpp"

namespace ptyx {
namespace f3 {

constexpr int kN = 128, kN2 = kN * kN;

__device__ __forceinline__ int fixed_of(int t) { return ((t & 63) >> 1) | ((t >> 6) << 5); }

// (cos 2πx, sin 2πx) for x in revolutions (v_cos_f32 / v_sin_f32 after reduction to [-1/2, 1/2])
__device__ __forceinline__ float2 cis_rev(float x) {
  const float r = x - rintf(x);
  return make_float2(__builtin_amdgcn_cosf(r), __builtin_amdgcn_sinf(r));
}

struct F3Args {
  int n_idx, n_scans, Ny, Nx;
  const int* idx;          // scan index per pattern
  const int* bid;          // mini-batch per pattern
  const int2* geo;         // clamped window origin (cy, cx) per pattern
  const float* shifts;     // (n_scans, 2)
  const float2* fpk;       // SHIFT: F(probe) K-packed; else the probe R-packed
  const float2* oc;        // A e^{iφ}, (Ny, Nx)
  const float* meas;       // (rows, 128, 128) f32, fftshifted
  const int* mrow;         // measurement row of scan position s (NULL: row s; rank-local blocks)
  int mrows;               // rows of meas (meas_rows entries are clamped into [0, mrows))
  const float* occp;       // omode_occu (device), occ = occp[0]
  float q, eps2;
  float* psums;            // per-pattern loss partial sums (k_finalize)
  float2* slots;           // per-pattern object-gradient slots, unit coefficient (row-permuted)
  float2* segslab;         // per-segment probe-gradient spectra, unit coefficient (K- / R-packed)
  int* segbid;             // mini-batch of each segment (-1: unused id)
  float* dsu;              // per-pattern position-gradient sums, unit coefficient (2 floats)
  int tail;                // probe or position gradient wanted
  float* dp_out;
  // multislice (k_fused3ms): Nz slices, H/N² K-packed; slots hold Nz planes per pattern (slice n
  // at slots + (pat·Nz + n)·N²), oc is (Nz, Ny, Nx)
  int Nz;
  const float2* hpk;
  // both data terms (k_fused3 MODE 1 / 2): loss_poissn's dp_pow, and the per-mini-batch
  // coefficients [c_single, c_poissn] (k_finalize) MODE 2 weights ∂ℓ/∂I with
  float q2 = 1.f;
  const float* coef = nullptr;
};

// Packed layouts (thread t = 0..255, register i = 0..63):
//   K: (row, col) = (ky, kx) = (fixed(t), i + 64·(t & 1))
//   R: (row, col) = (y, x)   = (i + 64·(t & 1), fixed(t))
template <bool KL>
__device__ __forceinline__ int packed_rc(int t, int i) {
  const int f = fixed_of(t), o = i + 64 * (t & 1);
  return KL ? f * kN + o : o * kN + f;
}

// natural (N×N complex) → packed, one element per thread
// (grid.y = mode: plane blockIdx.y of src → plane blockIdx.y of dst)
template <bool KL>
__global__ void k_pack128(const float2* src, float2* dst, float scale = 1.0f) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= kN2) return;
  src += (size_t)blockIdx.y * kN2;
  dst += (size_t)blockIdx.y * kN2;
  const int i = e >> 8, t = e & 255;
  const float2 v = src[packed_rc<KL>(t, i)];
  dst[e] = make_float2(v.x * scale, v.y * scale);
}

// Probe-gradient spectrum: Σ over segments (fixed order) of c_{m(seg)} × the segment's unit
// slab.  Two levels for parallelism: block (x, y) sums segments y, y + SPL, ... of 256 elements
// into part[y]; k_segslab_final adds the SPL partials in order and unpacks to natural order.
constexpr int kSegSplit = 32;
__global__ void k_segslab_reduce(const float2* segslab, const int* segbid, int nseg, const float* coef, int ci,
                                 float2* part) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y;
  float2 acc = make_float2(0.f, 0.f);
  for (int g = y; g < nseg; g += kSegSplit) {
    const int m = segbid[g];
    if (m < 0) continue;
    const float c = ci >= 2 ? 1.f : coef[(size_t)m * kNCoef + ci];   // (ci 2: applied by the kernel)
    const float2 u = segslab[(size_t)g * kN2 + e];
    acc.x = fmaf(c, u.x, acc.x);
    acc.y = fmaf(c, u.y, acc.y);
  }
  part[(size_t)y * kN2 + e] = acc;
}
// (grid.y = mode p: part + p·kSegSplit·N², out + p·N²)
template <bool KL>
__global__ void k_segslab_final(const float2* part, float2* out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  part += (size_t)blockIdx.y * kSegSplit * kN2;
  out += (size_t)blockIdx.y * kN2;
  float2 acc = make_float2(0.f, 0.f);
  for (int y = 0; y < kSegSplit; ++y) acc = cadd(acc, part[(size_t)y * kN2 + e]);
  out[packed_rc<KL>(e & 255, e >> 8)] = acc;
}

// d_shifts[s] += c_{m(pat)} · 2π/N² · dsu[pat]   (position gradient, image_proc.py:531 adjoint)
__global__ void k_shift_apply(const int* idx, int n, int n_scans, const int* bid, const float* coef, int ci,
                              const float* dsu, float* d_shifts) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int s = min(max(idx[j], 0), n_scans - 1);
  const float k = 6.283185307179586f * (ci >= 2 ? 1.f : coef[(size_t)bid[j] * kNCoef + ci]) * (1.0f / kN2);
  atomicAdd(d_shifts + 2 * s, dsu[2 * j] * k);
  atomicAdd(d_shifts + 2 * s + 1, dsu[2 * j + 1] * k);
}

// Small calls (one mini-batch per optimizer step, ≤ kSmallCall patterns): k_segslab_reduce +
// k_segslab_final + k_shift_apply in ONE launch.  Blocks [0, N²/256) sum the segments in exactly
// the two kernels' order (partial y = Σ_{g ≡ y mod kSegSplit} c·u, then the partials in order:
// bit-identical results); the blocks after them apply the position gradient.
// The probe gradient of a small call, inverse-transformed in two launches instead of three: a
// tail block owns columns i and i + 64 of the K-packed spectrum G (element 256 i + t is row
// fixed_of(t), column i + 64(t & 1)), so it transforms those two columns along themselves in LDS
// (tail_cols_ifft) and stores them to tmp in natural order; k_probe_rows_acc then transforms the
// rows and adds F⁻¹(G)/N² to d_probe (k_lines_cols<128, +1, 1>'s epilogue).  Columns before rows
// instead of rows before columns: the same transform up to fp32 rounding.
constexpr int kPrLinesT = 8;   // rows a k_probe_rows_acc block (ptyx_general.hpp kSpecLines)
__device__ __forceinline__ void tail_cols_ifft(float2 acc, int i, const float2* twg, float2* tmp_plane) {
  constexpr int N = kN;
  using LT = LineTile<N, 2>;
  using P1 = Plan1D<N>;
  __shared__ float2 s_tw[N];
  __shared__ float2 T[LT::kElems];
  const int t = threadIdx.x, line = t & 1, f = fixed_of(t);
  for (int k = t; k < N; k += 256) s_tw[k] = twg[k];
  T[LT::off(line, f)] = acc;
  __syncthreads();
  line_pass<N, 256, P1::R1, 1, +1, 2>(T, s_tw, 2);
  line_pass<N, 256, P1::R2, P1::R1, +1, 2>(T, s_tw, 2);
  tmp_plane[f * N + i + 64 * line] = T[LT::off(line, f)];
}
// Rows l0 … l0 + kPrLinesT − 1 of probe plane p (256 threads): g = d_probe + F⁻¹_rows(tmp)/N² per
// element, handed to epi(pointer into d_probe, element index in the plane stack, g), which stores it
// (k_probe_rows_acc) or also takes the optimizer step on it (k_gather_adam, ptyx_stepfuse.hpp).
template <class Epi>
__device__ __forceinline__ void probe_rows_block(const float2* tmp, float2* d_probe, const float2* twg, int l0, int p,
                                                 Epi epi) {
  constexpr int N = kN;
  using LT = LineTile<N, kPrLinesT>;
  using P1 = Plan1D<N>;
  __shared__ float2 s_tw[N];
  __shared__ float2 T[LT::kElems];
  const float2* s = tmp + (size_t)p * N * N;
  float2* d = d_probe + (size_t)p * N * N;
  for (int k = threadIdx.x; k < N; k += 256) s_tw[k] = twg[k];
  for (int e = threadIdx.x; e < kPrLinesT * N; e += 256) T[LT::off(e / N, e % N)] = s[(size_t)(l0 + e / N) * N + e % N];
  __syncthreads();
  line_pass<N, 256, P1::R1, 1, +1, kPrLinesT>(T, s_tw, kPrLinesT);
  line_pass<N, 256, P1::R2, P1::R1, +1, kPrLinesT>(T, s_tw, kPrLinesT);
  constexpr float inv_n2 = 1.0f / (float)(N * N);
  for (int e = threadIdx.x; e < kPrLinesT * N; e += 256) {
    const size_t el = (size_t)(l0 + e / N) * N + e % N;
    float2* dp = d + el;
    const float2 v = T[LT::off(e / N, e % N)];
    epi(dp, (size_t)p * N * N + el, cadd(*dp, make_float2(v.x * inv_n2, v.y * inv_n2)));
  }
}
// grid (N / kPrLinesT, P), block 256: rows l0 … l0 + 7 of plane p, d_probe += F⁻¹_rows(tmp)/N²
__global__ __launch_bounds__(256) void k_probe_rows_acc(const float2* tmp, float2* d_probe, const float2* twg) {
  probe_rows_block(tmp, d_probe, twg, blockIdx.x * kPrLinesT, blockIdx.y,
                   [](float2* dp, size_t, float2 g) { *dp = g; });
}

// The tail's body, workgroup bx, with the mini-batch coefficient coef_of(m) (c of segment / pattern
// batch m for the data term ci; ci 2: already applied): k_small_tail reads it from k_finalize's coef,
// the small calls' k_small_tail_fin (ptyx_kernels.hip) computes it in the workgroup — pre() runs
// once the workgroup's first loads are in flight and before coef_of is first called.
template <bool KL, class CoefOf, class Pre>
__device__ __forceinline__ void small_tail_body(int bx, const float2* segslab, const int* segbid, int nseg,
                                                CoefOf coef_of, Pre pre, float2* out, const int* idx, int n,
                                                int n_scans, const int* bid, const float* dsu, float* d_shifts,
                                                const float2* twg, float2* cols_out) {
  constexpr int kSlabBlocks = kN2 / 256;
  if (bx >= kSlabBlocks) {
    const int j = (bx - kSlabBlocks) * 256 + threadIdx.x;
    const bool on = d_shifts && j < n;
    int s = 0, bj = 0;
    float2 dj = make_float2(0.f, 0.f);
    if (on) {
      s = min(max(idx[j], 0), n_scans - 1);
      bj = bid[j];
      dj = make_float2(dsu[2 * j], dsu[2 * j + 1]);
    }
    pre();
    if (!on) return;
    const float k = 6.283185307179586f * coef_of(bj) * (1.0f / kN2);
    atomicAdd(d_shifts + 2 * s, dj.x * k);
    atomicAdd(d_shifts + 2 * s + 1, dj.y * k);
    return;
  }
  if (!out) {
    pre();
    return;
  }
  // the kSegSplit partial chains are independent: each round issues the loads of all of them, then
  // adds (a missing segment leaves its partial unchanged, as k_segslab_reduce skips it), so the
  // sums and their order are k_segslab_reduce + k_segslab_final's.  The slab loads do not wait for
  // the segment ids: every g < nseg is inside the slab buffer, and an unused segment's value (never
  // written: anything, NaN included) is dropped by the select, never multiplied.
  const int e = bx * 256 + threadIdx.x;
  float2 part[kSegSplit];
#pragma unroll
  for (int y = 0; y < kSegSplit; ++y) part[y] = make_float2(0.f, 0.f);
  for (int g0 = 0; g0 < nseg; g0 += kSegSplit) {
    float2 u[kSegSplit];
    int mm[kSegSplit];
#pragma unroll
    for (int y = 0; y < kSegSplit; ++y) {
      const int g = g0 + y;
      mm[y] = g < nseg ? segbid[g] : -1;
      u[y] = g < nseg ? segslab[(size_t)g * kN2 + e] : make_float2(0.f, 0.f);
    }
    if (g0 == 0) pre();
#pragma unroll
    for (int y = 0; y < kSegSplit; ++y) {
      if (mm[y] >= 0) {
        const float c = coef_of(mm[y]);
        part[y].x = fmaf(c, u[y].x, part[y].x);
        part[y].y = fmaf(c, u[y].y, part[y].y);
      }
    }
  }
  if (nseg <= 0) pre();
  float2 acc = make_float2(0.f, 0.f);
#pragma unroll
  for (int y = 0; y < kSegSplit; ++y) acc = cadd(acc, part[y]);
  if (KL && cols_out) {   // (block-uniform) the column pass of the probe gradient's inverse FFT
    tail_cols_ifft(acc, bx, twg, cols_out);
    return;
  }
  out[packed_rc<KL>(e & 255, e >> 8)] = acc;
}

template <bool KL>
__global__ __launch_bounds__(256) void k_small_tail(const float2* segslab, const int* segbid, int nseg,
                                                    const float* coef, int ci, float2* out, const int* idx, int n,
                                                    int n_scans, const int* bid, const float* dsu, float* d_shifts,
                                                    const float2* twg = nullptr, float2* cols_out = nullptr) {
  small_tail_body<KL>(blockIdx.x, segslab, segbid, nseg,
                      [&](int m) { return ci >= 2 ? 1.f : coef[(size_t)m * kNCoef + ci]; }, [] {}, out, idx, n,
                      n_scans, bid, dsu, d_shifts, twg, cols_out);
}

// Per call: complex object O = A e^{iφ} (the fused kernel then needs no transcendental per
// object point), and — for loss_sparse — per-row fp64 prefix sums of |φ|^n:
// pref[y][x] = Σ_{x' < x} |φ(y, x')|^n, x = 0..Nx.  One workgroup per object row.
__global__ void k_obj_prep(const float* obja, const float* objp, int Ny, int Nx, float2* oc, double* pref,
                           int sparse_n, const int* bbox = nullptr, int rows_per_slice = 0, int win = kN) {
  __shared__ double s_part[256];
  const int y = blockIdx.x;
  if (bbox) {   // rows no window of this call touches are never read (k_fused3*, k_pattern_table3)
    const int r = y % rows_per_slice;
    if (r < bbox[0] || r >= bbox[1] + win) return;
  }
  const float* ar = obja + (size_t)y * Nx;
  const float* pr = objp + (size_t)y * Nx;
  float2* orow = oc + (size_t)y * Nx;
  for (int x = threadIdx.x; x < Nx; x += blockDim.x) {
    float sn, cs;
    phase_sincos(pr[x], &sn, &cs);
    orow[x] = make_float2(ar[x] * cs, ar[x] * sn);
  }
  if (!pref) return;
  // contiguous chunk per thread, exclusive scan of the chunk sums in thread order (fixed order)
  const int per = (Nx + blockDim.x - 1) / blockDim.x;
  const int x0 = threadIdx.x * per, x1 = min(Nx, x0 + per);
  double sum = 0;
  for (int x = x0; x < x1; ++x) {
    const float ap = fabsf(pr[x]);
    sum += sparse_n == 1 ? (double)ap : (double)powq(ap, (float)sparse_n);
  }
  s_part[threadIdx.x] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    double run = 0;
    for (int i = 0; i < (int)blockDim.x; ++i) {
      const double t = s_part[i];
      s_part[i] = run;
      run += t;
    }
  }
  __syncthreads();
  double* prow = pref + (size_t)y * (Nx + 1);
  double run = s_part[threadIdx.x];
  for (int x = x0; x < x1; ++x) {
    prow[x] = run;
    const float ap = fabsf(pr[x]);
    run += sparse_n == 1 ? (double)ap : (double)powq(ap, (float)sparse_n);
  }
  if (x1 == Nx && x0 < x1) prow[Nx] = run;
  if (Nx == 0 && threadIdx.x == 0) prow[0] = 0;
}

// Columns of the row prefix sums → a summed-area table, in place: after k_obj_prep,
// pref[z][y][x] = Σ_{r0 ≤ y' ≤ y} Σ_{x' < x} |φ(z, y', x')|^n over the prepared rows [r0, r1)
// (all rows, or those the call's windows touch: the bbox rule of k_obj_prep).  A window's sum is
// then four lookups per slice (k_pattern_table3) instead of one pair per window row.  fp64, in
// two passes over chunks of kPrefChunk rows (one thread per (slice, chunk, column)): pass 1 scans
// each chunk and keeps its total, pass 2 adds the totals of the chunks above (fixed order).
constexpr int kPrefChunk = 32;
__device__ __forceinline__ void pref_rows(const int* bbox, int Ny, int win, int& r0, int& r1) {
  r0 = bbox ? max(0, bbox[0]) : 0;
  r1 = bbox ? min(Ny, bbox[1] + win) : Ny;
}
__global__ void k_pref_cols1(double* pref, double* tot, int Ny, int Nx, const int* bbox, int win = kN) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, c = blockIdx.y, z = blockIdx.z, nch = gridDim.y;
  if (x > Nx) return;
  int r0, r1;
  pref_rows(bbox, Ny, win, r0, r1);
  const int y0 = r0 + c * kPrefChunk, y1 = min(r1, y0 + kPrefChunk);
  double* col = pref + (size_t)z * Ny * (Nx + 1) + x;
  double acc = 0;
  for (int y = y0; y < y1; ++y) col[(size_t)y * (Nx + 1)] = acc += col[(size_t)y * (Nx + 1)];
  tot[((size_t)z * nch + c) * (Nx + 1) + x] = acc;   // (0 for chunks past r1)
}
__global__ void k_pref_cols2(double* pref, const double* tot, int Ny, int Nx, const int* bbox, int win = kN) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, c = blockIdx.y, z = blockIdx.z, nch = gridDim.y;
  if (x > Nx || c == 0) return;
  int r0, r1;
  pref_rows(bbox, Ny, win, r0, r1);
  const int y0 = r0 + c * kPrefChunk, y1 = min(r1, y0 + kPrefChunk);
  if (y0 >= y1) return;
  double off = 0;
  for (int k = 0; k < c; ++k) off += tot[((size_t)z * nch + k) * (Nx + 1) + x];
  double* col = pref + (size_t)z * Ny * (Nx + 1) + x;
  for (int y = y0; y < y1; ++y) col[(size_t)y * (Nx + 1)] += off;
}

// Bounding box of the call's windows: bbox = {min cy, max cy, min cx, max cx} (clamped origins);
// initialise with k_bbox_init.  Lets k_obj_prep / k_obj_gather skip untouched object rows / tiles.
__global__ void k_bbox_init(int* bbox) {
  if (threadIdx.x == 0) {
    bbox[0] = 0x7fffffff;
    bbox[1] = -0x7fffffff;
    bbox[2] = 0x7fffffff;
    bbox[3] = -0x7fffffff;
  }
}
// Grid-stride over the patterns (launch with at most kBboxBlocks blocks of 256 threads): wave
// reduction, then one set of four atomics per workgroup (contended atomics on four addresses
// from every wave cost ≈ 50 µs at 65,536 patterns).
constexpr int kBboxBlocks = 64;
__global__ __launch_bounds__(256) void k_bbox(const int* idx, int n, const int* crop, int n_scans, int Ny, int Nx,
                                              int* bbox, int win = kN) {
  __shared__ int red[4][4];
  int a = 0x7fffffff, b = -0x7fffffff, c = 0x7fffffff, d = -0x7fffffff;
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    const int s = min(max(idx[j], 0), n_scans - 1);
    const int cy = min(max(crop[2 * s], 0), Ny - win), cx = min(max(crop[2 * s + 1], 0), Nx - win);
    a = min(a, cy);
    b = max(b, cy);
    c = min(c, cx);
    d = max(d, cx);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    a = min(a, __shfl_xor(a, o, 64));
    b = max(b, __shfl_xor(b, o, 64));
    c = min(c, __shfl_xor(c, o, 64));
    d = max(d, __shfl_xor(d, o, 64));
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[wv][0] = a;
    red[wv][1] = b;
    red[wv][2] = c;
    red[wv][3] = d;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
      a = min(a, red[w][0]);
      b = max(b, red[w][1]);
      c = min(c, red[w][2]);
      d = max(d, red[w][3]);
    }
    atomicMin(bbox + 0, a);
    atomicMax(bbox + 1, b);
    atomicMin(bbox + 2, c);
    atomicMax(bbox + 3, d);
  }
}

// Small calls (≤ kSmallCall patterns, e.g. one 32-pattern mini-batch per optimizer step at the
// reference's default grad_accumulation = 1): the bounding box in ONE workgroup (no init launch,
// no atomics), which also clears the call's segment table (no memset launch).
constexpr int kSmallCall = 256;
__device__ __forceinline__ void k_bbox_small_body(const int* idx, int n, const int* crop, int n_scans, int Ny,
                                                  int Nx, int* bbox, int win, int* segbid, int nseg) {
  __shared__ int red[4][4];
  int a = 0x7fffffff, b = -0x7fffffff, c = 0x7fffffff, d = -0x7fffffff;
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    const int s = min(max(idx[j], 0), n_scans - 1);
    const int cy = min(max(crop[2 * s], 0), Ny - win), cx = min(max(crop[2 * s + 1], 0), Nx - win);
    a = min(a, cy);
    b = max(b, cy);
    c = min(c, cx);
    d = max(d, cx);
  }
  for (int i = threadIdx.x; i < nseg; i += blockDim.x) segbid[i] = -1;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    a = min(a, __shfl_xor(a, o, 64));
    b = max(b, __shfl_xor(b, o, 64));
    c = min(c, __shfl_xor(c, o, 64));
    d = max(d, __shfl_xor(d, o, 64));
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[wv][0] = a;
    red[wv][1] = b;
    red[wv][2] = c;
    red[wv][3] = d;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
      a = min(a, red[w][0]);
      b = max(b, red[w][1]);
      c = min(c, red[w][2]);
      d = max(d, red[w][3]);
    }
    bbox[0] = a;
    bbox[1] = b;
    bbox[2] = c;
    bbox[3] = d;
  }
}
__global__ __launch_bounds__(256) void k_bbox_small(const int* idx, int n, const int* crop, int n_scans, int Ny,
                                                    int Nx, int* bbox, int win, int* segbid, int nseg) {
  k_bbox_small_body(idx, n, crop, n_scans, Ny, Nx, bbox, win, segbid, nseg);
}

// pattern → (mini-batch, clamped window origin) and, with pref (the summed-area table of
// k_pref_cols1/2), the loss_sparse window sum Σ_{window} |φ|^n into psums[kSumBase]: four fp64
// lookups per slice, lane z per slice, fixed-order wave sum.  bbox: the table's first row is
// bbox[0] (PTYX_PREP_CALL), else row 0.  One wave per pattern.
struct TableCheck {   // input validation of the call's patterns (check_pattern)
  int* err;
  const int* mrow;
  int mrows;
};
__global__ void k_pattern_table3(const int* idx, int n, const int* boff, int n_batches, const int* crop,
                                 int n_scans, int Ny, int Nx, int* bid, int2* geo, const double* pref,
                                 float* psums, int Nz, const int* bbox, TableCheck tc) {
  const int j = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (j >= n) return;
  const int s = min(max(idx[j], 0), n_scans - 1);
  const int cy = min(max(crop[2 * s], 0), Ny - kN), cx = min(max(crop[2 * s + 1], 0), Nx - kN);
  if (lane == 0) {
    check_pattern(tc.err, idx[j], n_scans, crop, Ny, Nx, kN, tc.mrow, tc.mrows);
    int lo = 0, hi = n_batches;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (boff[mid] <= j) lo = mid;
      else hi = mid;
    }
    bid[j] = lo;
    geo[j] = make_int2(cy, cx);
  }
  if (!pref) return;
  const int r0 = bbox ? max(0, bbox[0]) : 0;
  double acc = 0;
  for (int z = lane; z < Nz; z += 64) {
    const double* ps = pref + (size_t)z * Ny * (Nx + 1);
    const double* lo = ps + (size_t)(cy + kN - 1) * (Nx + 1);   // rows r0 .. cy + N - 1
    acc += lo[cx + kN] - lo[cx];
    if (cy > r0) {                                              // minus rows r0 .. cy - 1
      const double* hi = ps + (size_t)(cy - 1) * (Nx + 1);
      acc -= hi[cx + kN] - hi[cx];
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) psums[(size_t)j * kNSum + kSumBase] = (float)acc;
}

// Small calls (PTYX_PREP_CALL, ≤ kSmallCall patterns): k_pattern_table3's entries with the
// loss_sparse window sum Σ_window |φ|^n read straight from objp — no summed-area table to build.
// One workgroup per pattern: wave w sums rows w, w + 4, … of every slice, a lane two columns, a
// slice's 32 rows per round (64 loads in flight: one round trip a slice); fp64 lane sums,
// fixed-order wave reduction, waves added in order through LDS (deterministic).
// one pattern's table entry (mini-batch by binary search over boff, clamped window origin) and
// its input validation
__device__ __forceinline__ void table_entry(int j, const int* idx, const int* boff, int n_batches, const int* crop,
                                            int n_scans, int Ny, int Nx, int* bid, int2* geo, TableCheck tc) {
  const int s = min(max(idx[j], 0), n_scans - 1);
  const int cy = min(max(crop[2 * s], 0), Ny - kN), cx = min(max(crop[2 * s + 1], 0), Nx - kN);
  check_pattern(tc.err, idx[j], n_scans, crop, Ny, Nx, kN, tc.mrow, tc.mrows);
  int lo = 0, hi = n_batches;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (boff[mid] <= j) lo = mid;
    else hi = mid;
  }
  bid[j] = lo;
  geo[j] = make_int2(cy, cx);
}
__device__ __forceinline__ void k_pattern_table_direct_body(int j, const int* idx, int n, const int* boff,
                                                            int n_batches, const int* crop, int n_scans, int Ny,
                                                            int Nx, int* bid, int2* geo, const float* objp,
                                                            int sparse_n, float* psums, int Nz, TableCheck tc) {
  __shared__ double s_w[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int s = min(max(idx[j], 0), n_scans - 1);
  const int cy = min(max(crop[2 * s], 0), Ny - kN), cx = min(max(crop[2 * s + 1], 0), Nx - kN);
  if (threadIdx.x == 0) table_entry(j, idx, boff, n_batches, crop, n_scans, Ny, Nx, bid, geo, tc);
  double acc = 0;
  for (int z = 0; z < Nz; ++z) {
    // the wave's 32 rows of the slice in one round (64 loads in flight), summed in row order
    const float* ph = objp + ((size_t)z * Ny + cy + wave) * Nx + cx + lane;
    float v[64];
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      v[2 * k] = ph[(size_t)(4 * k) * Nx];
      v[2 * k + 1] = ph[(size_t)(4 * k) * Nx + 64];
    }
#pragma unroll
    for (int k = 0; k < 64; ++k) {
      const float a = fabsf(v[k]);
      acc += sparse_n == 1 ? (double)a : (double)powq(a, (float)sparse_n);
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) s_w[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) psums[(size_t)j * kNSum + kSumBase] = (float)(((s_w[0] + s_w[1]) + s_w[2]) + s_w[3]);
}
__global__ __launch_bounds__(256) void k_pattern_table_direct(const int* idx, int n, const int* boff, int n_batches,
                                                              const int* crop, int n_scans, int Ny, int Nx, int* bid,
                                                              int2* geo, const float* objp, int sparse_n, float* psums,
                                                              int Nz, TableCheck tc) {
  k_pattern_table_direct_body(blockIdx.x, idx, n, boff, n_batches, crop, n_scans, Ny, Nx, bid, geo, objp, sparse_n,
                              psums, Nz, tc);
}

// Small calls with PTYX_PREP_CALL (one mini-batch per optimizer step): k_pattern_table_direct,
// k_obj_prep and k_bbox_small as ONE launch of independent block roles —
//   blocks [0, n)            the pattern table (+ the loss_sparse window sums when SPARSE; with
//                            PrepExtra::zsum n·Nz blocks, one (pattern, slice) sum each);
//   blocks [n, n + R)        O = A e^{iφ} for kPrepRows object rows (of the Nz·Ny) each, those any
//                            window of the call covers (decided from the ≤ 256 windows directly,
//                            not the bbox); R = ⌈Nz·Ny / kPrepRows⌉ (small_prep_blocks);
//   block n + R              the bounding box (k_obj_gather) and the segment-table clear.
// Same outputs as the three kernels (the rows no window touches are never read under PREP_CALL).
constexpr int kPrepRows = 4;
// zs (multislice calls with loss_sparse): the pattern blocks are n·Nz, one (pattern, slice) each
__host__ __device__ constexpr int small_prep_blocks(int n, int Nz, int Ny, bool zs = false) {
  return (zs ? n * Nz : n) + (Nz * Ny + kPrepRows - 1) / kPrepRows + 1;
}
// Work of the call's probe preparation that rides in k_small_prep's launch as further block roles
// (independent of the table / object rows): the row pass of F(P_p) (k_lines_rows<128, −1>, the
// same code: its column pass, k_lines_cols, follows as the next launch) and the K-packing of H/N²
// (k_pack128<true>).  probe / H null: that role is absent.
constexpr int kPrLines = 8;   // lines a row block (ptyx_general.hpp kSpecLines)
struct PrepExtra {
  const float2* probe = nullptr;
  int P = 0;
  float2* tmp = nullptr;       // (P, N, N) row-pass output
  const float2* twg = nullptr;
  const float2* H = nullptr;
  float2* hpk = nullptr;
  float hscale = 1.0f;
  double* zsum = nullptr;      // per-(pattern, slice) loss_sparse window sums (else psums, per pattern)
  float2* fpk = nullptr;       // non-null: F(P_p) straight to the K-packed fpk, one leading workgroup a
                               // mode (probe_spectrum_reg), instead of the row pass into tmp
  // PTYX_PREP_SELECT folded in (a graph-replayed step's ptyx_step_select): the call's indices are
  // sel_all[sel_start[*sel_cnt] + j], which the pattern workgroups also store to sel_out (the call's
  // idx, read by the later launches); sel workgroups zero zero[0, zero_n) and advance *steps[t]
  const int32_t* sel_all = nullptr;
  const int64_t* sel_start = nullptr;
  const int64_t* sel_cnt = nullptr;
  int32_t* sel_out = nullptr;
  float* zero = nullptr;
  long long zero_n = 0;
  float* const* steps = nullptr;
  int n_steps = 0;
  __host__ __device__ int lead_blocks() const { return probe && fpk ? P : 0; }
  __host__ __device__ int sel_blocks() const {
    if (!sel_all) return 0;
    const long long zb = (zero_n + 4095) / 4096;
    return (int)(zb < 1 ? 1 : zb > 64 ? 64 : zb);
  }
  __host__ __device__ int row_blocks() const { return probe && !fpk ? (kN / kPrLines) * P : 0; }
  __host__ __device__ int h_blocks() const { return H ? kN2 / 256 : 0; }
};
__device__ __forceinline__ void probe_rows_body(int bx, int p, const float2* src, float2* tmp, const float2* twg) {
  constexpr int N = kN;
  using LT = LineTile<N, kPrLines>;
  using P1 = Plan1D<N>;
  __shared__ float2 s_tw[N];
  __shared__ float2 T[LT::kElems];
  const int l0 = bx * kPrLines;
  const float2* s = src + (size_t)p * N * N;
  float2* d = tmp + (size_t)p * N * N;
  for (int i = threadIdx.x; i < N; i += 256) s_tw[i] = twg[i];
  const int nl = min(kPrLines, N - l0);
  for (int e = threadIdx.x; e < nl * N; e += 256) T[LT::off(e / N, e % N)] = s[(size_t)(l0 + e / N) * N + e % N];
  __syncthreads();
  line_pass<N, 256, P1::R1, 1, -1, kPrLines>(T, s_tw, nl);
  line_pass<N, 256, P1::R2, P1::R1, -1, kPrLines>(T, s_tw, nl);
  for (int e = threadIdx.x; e < nl * N; e += 256) d[(size_t)(l0 + e / N) * N + e % N] = T[LT::off(e / N, e % N)];
}
// The shifted probe's spectrum F(P) of a small call in ONE workgroup: the register-resident 2-D FFT
// (ptyx_regfft.hpp) from the natural probe straight to the K-packed layout the register engines
// read (fpk[256 k + t] = F[ky][k + 64 l0] of thread t, as k_lines_cols packs it), instead of a row
// pass here and a column launch (k_lines_cols) after.  Same transform up to fp32 rounding.
__device__ __forceinline__ void probe_spectrum_reg(const float2* probe, float2* fpk) {
  using namespace rf;
  __shared__ float2 buf[kLdsElems];
  const Coord cd = coord(threadIdx.x);
  const LaneCtx lc = lane_ctx(cd.lane);
  float2 v[64];
#pragma unroll
  for (int j = 0; j < 64; ++j) v[j] = probe[(size_t)(j + 64 * cd.l0) * kN + cd.fixed];
  fft_fwd(v, buf, lc, cd.wsign);
#pragma unroll
  for (int k = 0; k < 64; ++k) fpk[(size_t)k * 256 + threadIdx.x] = v[k];
}
// one (pattern, slice)'s loss_sparse window sum: the slice pass of k_pattern_table_direct_body,
// its fp64 wave sums added in wave order, to zsum[j·Nz + z] (k_finalize adds the slices in order)
__device__ __forceinline__ void slice_window_sum(int j, int z, const int* idx, const int* crop, int n_scans, int Ny,
                                                 int Nx, const float* objp, int sparse_n, int Nz, double* zsum) {
  __shared__ double s_z[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int s = min(max(idx[j], 0), n_scans - 1);
  const int cy = min(max(crop[2 * s], 0), Ny - kN), cx = min(max(crop[2 * s + 1], 0), Nx - kN);
  const float* ph = objp + ((size_t)z * Ny + cy + wave) * Nx + cx + lane;
  float v[64];
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    v[2 * k] = ph[(size_t)(4 * k) * Nx];
    v[2 * k + 1] = ph[(size_t)(4 * k) * Nx + 64];
  }
  double acc = 0;
#pragma unroll
  for (int k = 0; k < 64; ++k) {
    const float a = fabsf(v[k]);
    acc += sparse_n == 1 ? (double)a : (double)powq(a, (float)sparse_n);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) s_z[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) zsum[(size_t)j * Nz + z] = ((s_z[0] + s_z[1]) + s_z[2]) + s_z[3];
}
template <bool SPARSE>
__global__ __launch_bounds__(256) void k_small_prep(const int* idx, int n, const int* boff, int n_batches,
                                                    const int* crop, int n_scans, int Ny, int Nx, int* bid, int2* geo,
                                                    const float* obja, const float* objp, int sparse_n, float* psums,
                                                    int Nz, TableCheck tc, float2* oc, int* bbox, int* segbid,
                                                    int nseg, PrepExtra ex) {
  if ((int)blockIdx.x < ex.lead_blocks()) {   // (first: the longest chain of the launch starts first)
    probe_spectrum_reg(ex.probe + (size_t)blockIdx.x * kN2, ex.fpk + (size_t)blockIdx.x * kN2);
    return;
  }
  if ((int)blockIdx.x < ex.lead_blocks() + ex.sel_blocks()) {   // the folded step selection
    const int sb = (int)blockIdx.x - ex.lead_blocks(), nsb = ex.sel_blocks();
    if (sb == 0 && (int)threadIdx.x < ex.n_steps) {   // the optimizer's step counts (torch's state_step += 1)
      float* s = ex.steps[threadIdx.x];
      *s = *s + 1.0f;
    }
    // scalar head up to 16-byte alignment, float4 body, scalar tail (as k_step_select)
    float* g = ex.zero;
    const long long n = ex.zero_n, t = (long long)sb * 256 + threadIdx.x, stride = (long long)nsb * 256;
    const long long head = min(n, (long long)(((16 - (reinterpret_cast<uintptr_t>(g) & 15)) & 15) >> 2));
    if (t < head) g[t] = 0.f;
    float4* g4 = reinterpret_cast<float4*>(g + head);
    const long long n4 = (n - head) >> 2;
    for (long long i = t; i < n4; i += stride) g4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (long long i = head + 4 * n4 + t; i < n; i += stride) g[i] = 0.f;
    return;
  }
  const int b = blockIdx.x - ex.lead_blocks() - ex.sel_blocks();
  if (ex.sel_all) idx = ex.sel_all + ex.sel_start[*ex.sel_cnt];
  const bool zs = SPARSE && ex.zsum != nullptr;
  const int np = zs ? n * Nz : n;                         // pattern blocks
  const int bx = b - small_prep_blocks(n, Nz, Ny, zs);   // the PrepExtra roles
  if (bx >= 0) {
    if (bx < ex.row_blocks()) {
      probe_rows_body(bx % (kN / kPrLines), bx / (kN / kPrLines), ex.probe, ex.tmp, ex.twg);
      return;
    }
    const int e = (bx - ex.row_blocks()) * 256 + (int)threadIdx.x;   // H/N² K-packed
    const float2 h = ex.H[packed_rc<true>(e & 255, e >> 8)];
    ex.hpk[e] = make_float2(h.x * ex.hscale, h.y * ex.hscale);
    return;
  }
  if (b < np) {
    if (zs) {   // (pattern j, slice z): z = 0 also writes the table entry
      const int j = b / Nz, z = b - j * Nz;
      if (z == 0 && threadIdx.x == 0) table_entry(j, idx, boff, n_batches, crop, n_scans, Ny, Nx, bid, geo, tc);
      if (z == 0 && threadIdx.x == 0 && ex.sel_out) ex.sel_out[j] = idx[j];
      slice_window_sum(j, z, idx, crop, n_scans, Ny, Nx, objp, sparse_n, Nz, ex.zsum);
    } else if constexpr (SPARSE) {
      if (threadIdx.x == 0 && ex.sel_out) ex.sel_out[b] = idx[b];
      k_pattern_table_direct_body(b, idx, n, boff, n_batches, crop, n_scans, Ny, Nx, bid, geo, objp, sparse_n, psums,
                                  Nz, tc);
    } else if (threadIdx.x == 0) {
      if (ex.sel_out) ex.sel_out[b] = idx[b];
      table_entry(b, idx, boff, n_batches, crop, n_scans, Ny, Nx, bid, geo, tc);
    }
    return;
  }
  const int nrb = (Nz * Ny + kPrepRows - 1) / kPrepRows;
  if (b == np + nrb) {
    k_bbox_small_body(idx, n, crop, n_scans, Ny, Nx, bbox, kN, segbid, nseg);
    return;
  }
  // kPrepRows consecutive object rows (flattened z·Ny + r): which of them any window covers, then
  // their loads issued together
  const int y0 = (b - np) * kPrepRows;
  int cy = -(1 << 29);
  if ((int)threadIdx.x < n) {
    const int s = min(max(idx[threadIdx.x], 0), n_scans - 1);
    cy = min(max(crop[2 * s], 0), Ny - kN);
  }
  bool hit[kPrepRows];
#pragma unroll
  for (int k = 0; k < kPrepRows; ++k) {
    const int r = (y0 + k) % Ny;
    hit[k] = __syncthreads_or(y0 + k < Nz * Ny && r >= cy && r < cy + kN) != 0;
  }
  for (int x0 = 0; x0 < Nx; x0 += 256) {
    const int x = x0 + (int)threadIdx.x;
    float av[kPrepRows], pv[kPrepRows];
#pragma unroll
    for (int k = 0; k < kPrepRows; ++k)
      if (hit[k] && x < Nx) {
        av[k] = obja[(size_t)(y0 + k) * Nx + x];
        pv[k] = objp[(size_t)(y0 + k) * Nx + x];
      }
#pragma unroll
    for (int k = 0; k < kPrepRows; ++k)
      if (hit[k] && x < Nx) {
        float sn, cs;
        phase_sincos(pv[k], &sn, &cs);
        oc[(size_t)(y0 + k) * Nx + x] = make_float2(av[k] * cs, av[k] * sn);
      }
  }
}

// Far-field loss at one point, branch-free.  Returns u = ∂ℓ/∂I per unit mini-batch coefficient
// and accumulates the partial sums (S, ΣM^q):
//   SINGLE: ℓ ∝ Σ(I^q − M^q)²          (losses.py:45-47),  u = (I^q − M^q)·q·I^q/I
//   else:   ℓ ∝ Σ(M^q ln(I^q+ε) − I^q) (losses.py:70-72),  u = (M^q/(I^q+ε) − 1)·q·I^q/I
// QM: 0 → q = 1/2 (sqrt / rsqrt), 1 → q = 1, 2 → general q (exp2(q·log2 x)); I ≥ 1e-10 > 0.
// (The kernel is instantiated for QM 0 and 2 only: q = 1 runs the general form.)
template <int QM, bool SINGLE>
__device__ __forceinline__ float loss_point(float I, float M, float q, float eps2, float& S, float& Ms) {
  float Iq, Mq, qIqI;   // qIqI = q·I^q/I
  if constexpr (QM == 0) {
    const float r = __builtin_amdgcn_rsqf(I);
    Iq = I * r;
    Mq = __builtin_amdgcn_sqrtf(M);
    qIqI = 0.5f * r;
  } else if constexpr (QM == 1) {
    Iq = I;
    Mq = M;
    qIqI = 1.0f;
  } else {
    Iq = __builtin_amdgcn_exp2f(q * __builtin_amdgcn_logf(I));
    Mq = M > 0.f ? __builtin_amdgcn_exp2f(q * __builtin_amdgcn_logf(M)) : (q > 0.f ? 0.f : __builtin_inff());
    qIqI = q * Iq * __builtin_amdgcn_rcpf(I);
  }
  Ms += Mq;
  if constexpr (SINGLE) {
    const float d = Iq - Mq;
    S = fmaf(d, d, S);
    return d * qIqI;
  } else {
    const float ip = Iq + eps2;
    S += Mq * fast_ln(ip) - Iq;
    return fmaf(Mq, __builtin_amdgcn_rcpf(ip), -1.0f) * qIqI;
  }
}

// Buffer-resource access with 32-bit VGPR offsets (base + per-register constant, one v_add each;
// soffset 0).  Plain global loads would need a 64-bit address VGPR pair per register once the
// offsets pass the 4 KiB immediate range, and per-register SGPR soffsets get hoisted out of the
// pattern loop by MachineLICM (≈200 SGPRs, spilled).
using Rsrc = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ Rsrc rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float2 ld2(Rsrc r, int voff, int off) {
  const auto u = __builtin_amdgcn_raw_buffer_load_b64(r, voff + off, 0, 0);
  return make_float2(__uint_as_float(u[0]), __uint_as_float(u[1]));
}
__device__ __forceinline__ void st2(float2 v, Rsrc r, int voff, int off) {
  const __attribute__((ext_vector_type(2))) unsigned u = {__float_as_uint(v.x), __float_as_uint(v.y)};
  __builtin_amdgcn_raw_buffer_store_b64(u, r, voff + off, 0, 0);
}
// Non-temporal (aux = 2, "nt") for the streams read once much later or never again in this kernel
// (final slot stores, the DP), so they do not evict the park / slab / object / F(P) lines the next
// passes re-read from L2.
constexpr int kNtAux = 2;
__device__ __forceinline__ void st2_stream(float2 v, Rsrc r, int voff, int off) {
  const __attribute__((ext_vector_type(2))) unsigned u = {__float_as_uint(v.x), __float_as_uint(v.y)};
  __builtin_amdgcn_raw_buffer_store_b64(u, r, voff + off, 0, kNtAux);
}

// Wave sum in a fixed order, result in every lane: DPP adds within each 16-lane row
// (pairs, quads, half-rows, rows), then the four row sums via v_readlane.  No ds_bpermute,
// no per-step lane-index arithmetic (which spills beside 128 live data VGPRs).
template <int CTRL>
__device__ __forceinline__ float dppmov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum(float x) {
  x += dppmov<0xB1>(x);    // quad_perm [1,0,3,2]
  x += dppmov<0x4E>(x);    // quad_perm [2,3,0,1]
  x += dppmov<0x141>(x);   // row_half_mirror
  x += dppmov<0x140>(x);   // row_mirror
  const float a0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 0));
  const float a1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 16));
  const float a2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 32));
  const float a3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 48));
  return (a0 + a1) + (a2 + a3);
}
// Workgroup (4 waves) sum of NV floats in a fixed order; result valid in every thread.
template <int NV>
__device__ __forceinline__ void block_sum4(float (&v)[NV], float* red) {
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = wave_sum(v[i]);
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) red[wv * NV + i] = v[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = (red[i] + red[NV + i]) + (red[2 * NV + i] + red[3 * NV + i]);
  __syncthreads();
}

// Pin a value at this point of the program (empty volatile asm that "redefines" it): the
// compiler can no longer sink its computation towards a later use, which otherwise keeps every
// intermediate of a 64-register pass live across barriers and spills.
__device__ __forceinline__ void pin(float2& v) { asm volatile("" : "+v"(v.x), "+v"(v.y)); }

// Software-pipelined pass over the 64 registers in NC chunks: the global loads of chunks
// c+1 … c+D are in flight while chunk c is consumed, and a scheduling barrier after every chunk
// keeps the compiler from hoisting all 64 loads at once (which would need 128+ extra VGPRs and
// spill).  D = 1 (deeper measured no faster at 256 VGPRs).
template <int NC, class Ld, class Use>
__device__ __forceinline__ void pipeline(Ld&& ld, Use&& use) {
  constexpr int D = 1;
  using T = decltype(ld(std::integral_constant<int, 0>{}));
  T ring[D + 1];
  rf::sfor<0, D>([&](auto I) {
    constexpr int i = decltype(I)::value;
    if constexpr (i < NC) ring[i] = ld(std::integral_constant<int, i>{});
  });
  rf::sfor<0, NC>([&](auto C) {
    constexpr int c = decltype(C)::value;
    if constexpr (c + D < NC) ring[(c + D) % (D + 1)] = ld(std::integral_constant<int, c + D>{});
    use(C, ring[c % (D + 1)]);
    __builtin_amdgcn_sched_barrier(0);
  });
}
struct Ch8 {
  float2 x[8];
};
struct Ch4x2 {
  float2 x[4], y[4];
};

// ------------------------------------------------------------------ packed complex arithmetic
// Two v_pk instructions per complex product (the scalar cmul / cmulc of ptyx_fft.hpp take four
// VALU instructions); operand halves are routed by op_sel / neg modifiers.
//   pcm(a, b)  = a·b        = (a.x b.x − a.y b.y, a.x b.y + a.y b.x)
//   pcmc(a, b) = a·conj(b)  = (a.x b.x + a.y b.y, a.y b.x − a.x b.y)
__device__ __forceinline__ float2 pcm(float2 a, float2 b) {
  rf::v2f t, r;
  asm("v_pk_mul_f32 %0, %2, %3 op_sel_hi:[0,1]\n\t"
      "v_pk_fma_f32 %1, %2, %3, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
      : "=&v"(t), "=v"(r)
      : "v"(rf::pv(a)), "v"(rf::pv(b)));
  return rf::pf(r);
}
__device__ __forceinline__ float2 pcmc(float2 a, float2 b) {
  rf::v2f t, r;
  asm("v_pk_mul_f32 %0, %2, %3 op_sel_hi:[1,0]\n\t"
      "v_pk_fma_f32 %1, %2, %3, %0 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[0,1,0]"
      : "=&v"(t), "=v"(r)
      : "v"(rf::pv(a)), "v"(rf::pv(b)));
  return rf::pf(r);
}
__device__ __forceinline__ float2 pscale(float2 a, float s) { return rf::pf(rf::pv(a) * (rf::v2f){s, s}); }
__device__ __forceinline__ float2 padd2(float2 a, float2 b) { return rf::pf(rf::pv(a) + rf::pv(b)); }

// ------------------------------------------------------------------ LDS-DMA operand ring
// The operands of the point-wise passes of the shifted-probe kernels (object window, ψ⁰ park, F(P), segment
// slab) stream HBM/L2 → LDS by buffer_load_dwordx4 … lds into a per-wave ring in the (then free)
// exchange buffer, D register pairs ahead of their use, and are read back with ds_read_b64.  No
// VGPRs are held by loads in flight, so a pass keeps 8-16 KiB per wave (64-128 KiB per CU) of
// operands in flight instead of the one 4-register chunk the register pipeline could afford; the
// first D pairs are issued during the second half of the preceding FFT.
//
// The DMA is emitted as inline asm: issued through the builtin, the compiler would put a
// vmcnt(0) in front of every later LDS read of the buffer (it cannot tell the ring slots apart),
// which serialises the ring.  The waits are explicit (vm_wait, counts from ring_wait_count), M0 is
// saved and restored inside the asm, and every asm carries a memory clobber so no compiler memory
// access moves across it.  Per wave the ring is 16 KiB: wave w owns bytes [16 KiB·w, 16 KiB·(w+1))
// of the exchange buffer, and each wave DMAs exactly the operands its own threads read, so the
// ring needs no workgroup barrier.
typedef unsigned v4u __attribute__((ext_vector_type(4)));
// buffer descriptor as four SGPRs (raw, stride 0; word 3 as rsrc())
__device__ __forceinline__ v4u srd(const void* base, unsigned bytes) {
  const unsigned long long p = (unsigned long long)base;
  return v4u{(unsigned)p, (unsigned)(p >> 32) & 0xffffu, bytes, 0x00020000u};
}
// 16 B per lane: LDS[m0 + 16·lane] ← mem[r + voff + SOFF]
template <int SOFF>
__device__ __forceinline__ void dma_c(v4u r, int voff, int m0) {
  int t, s;
  asm volatile(
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_mov_b32 %1, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_mov_b32 %0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %4, %5, %0 offen lds\n\t"
      "s_mov_b32 m0, %1"
      : "=&s"(t), "=&s"(s)
      : "s"(m0), "i"(SOFF), "v"(voff), "s"(r)
      : "memory");
}
// the same with soffset = J·os (object rows: os = 8·Nx bytes)
template <int J>
__device__ __forceinline__ void dma_m(v4u r, int voff, int m0, int os) {
  int t, s;
  asm volatile(
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_mov_b32 %1, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_mul_i32 %0, %3, %4\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %5, %6, %0 offen lds\n\t"
      "s_mov_b32 m0, %1"
      : "=&s"(t), "=&s"(s)
      : "s"(m0), "s"(os), "i"(J), "v"(voff), "s"(r)
      : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
// Vector-memory instructions a wave has issued after the DMAs of register pair Q, at the wait of
// pair Q: D pairs are issued ahead (A DMAs each); iteration P then does S stores and the DMAs of
// pair P + D (if any) into the slot pair P just freed.  The passes call it with S = 0: vmcnt
// retires loads in order among themselves, but a store may be acknowledged before an older load
// returns, so only the loads issued after pair Q's DMAs may be left outstanding.
//
// A wave's ring lies in the exchange buffer, which the next FFT's exchange overwrites across all
// waves: a workgroup barrier separates the last ring read of every wave from that exchange.
constexpr int ring_wait_count(int Q, int A, int S, int D) {
  int n = 0;
  if (Q < D) {
    n = (D - 1 - Q) * A;
    for (int P = 0; P < Q; ++P) n += S + (P + D < 32 ? A : 0);
  } else {
    for (int P = Q - D + 1; P < Q; ++P) n += S + (P + D < 32 ? A : 0);
  }
  return n;
}
// Per-lane DMA source offsets (μ = lane; the two halves of a wave fetch register pair (2q, 2q+1)).
//   K-packed arrays (F(P), slab: element (t, k) at 8t + 2048k) and the ψ⁰ park: LDS image of a
//   register = thread λ at 8λ.  Object window (element (λ, j) at row j + 64·l0, column 32w + λ/2):
//   LDS image pos(λ) = 256(f>>4) + 32((f&15)>>1) + 16·l0 + 8(f&1), f = λ>>1 (conflict-free
//   ds_read_b64, 16-B DMA granules = two adjacent columns of one row).
__device__ __forceinline__ int dma_off_k(int mu, int w) { return ((mu >> 5) << 11) + (w << 9) + ((mu & 31) << 4); }
__device__ __forceinline__ int dma_off_park(int mu, int w) {
  return ((mu >> 5) << 11) + (((mu >> 4) & 1) << 10) + (w << 8) + ((mu & 15) << 4);
}
__device__ __forceinline__ int dma_off_obj(int mu, int w, int os) {
  const int nu = mu & 31, l0 = nu & 1, i = ((nu >> 4) << 3) | ((nu >> 1) & 7);
  return ((mu >> 5) + 64 * l0) * os + (w << 8) + (i << 4);
}
// ψ⁰ park store offset of thread λ (within wave w's slot bytes of each register row)
__device__ __forceinline__ int park_off(int lam, int w) { return ((lam >> 5) << 10) + (w << 8) + ((lam & 31) << 3); }
// float2 index of thread λ's object element in a register's LDS image
__device__ __forceinline__ int obj_img(int lam) {
  const int f = lam >> 1;
  return ((f >> 4) << 5) + (((f & 15) >> 1) << 2) + ((lam & 1) << 1) + (f & 1);
}

// Park stores: k_fused3 reads its ψ⁰ park two transforms later, partly from L2, so it stores
// them plainly (non-temporal measured 11.35-11.56 → 11.66-11.68 ms, profiles/r02/ab/r02y_pnt_*);
// k_fused3ms reads slice n's park 2·(Nz − n) transforms later and stores them non-temporal
// (c4 2.672 → 2.641 s per step).  A pattern's scalars come from the previous pattern's post4 pass.

// Per-pattern scalars.
struct PatInfo {
  int m, cy, cx, sidx, mi;   // mini-batch, window origin, scan index, measurement row
  float sy, sx;
};
// Per-pattern scalars through the scalar cache (s_load, counted by lgkmcnt).  A plain load of
// these read-only tables is a vector load here (the kernel stores to global memory, so the
// compiler cannot prove them unwritten), and its vmcnt(0) wait would also wait for every slot /
// slab / park store still in flight.  Uniform addresses only.
__device__ __forceinline__ int s_ld(const int* p) {
  int v;
  asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return v;
}
__device__ __forceinline__ void s_ld3(const int* pb, const int2* pg, const int* pi, int& b, int2& g, int& i) {
  unsigned long long gg;
  asm volatile(
      "s_load_dword %0, %3, 0x0\n\t"
      "s_load_dwordx2 %1, %4, 0x0\n\t"
      "s_load_dword %2, %5, 0x0\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&s"(b), "=&s"(gg), "=&s"(i)
      : "s"(pb), "s"(pg), "s"(pi)
      : "memory");
  g = make_int2((int)(unsigned)gg, (int)(unsigned)(gg >> 32));
}
__device__ __forceinline__ float2 s_ldf2(const float* p) {
  unsigned long long v;
  asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return make_float2(__uint_as_float((unsigned)v), __uint_as_float((unsigned)(v >> 32)));
}
template <bool SHIFT>
__device__ __forceinline__ PatInfo pat_info(const F3Args& a, int pat) {
  PatInfo p;
  const int pp = min(pat, a.n_idx - 1);   // (a past-the-end "next" pattern reads a valid slot)
  int2 g;
  int si;
  s_ld3(a.bid + pp, a.geo + pp, a.idx + pp, p.m, g, si);
  p.cy = g.x;
  p.cx = g.y;
  p.sidx = min(max(si, 0), a.n_scans - 1);
  p.mi = a.mrow ? min(max(s_ld(a.mrow + p.sidx), 0), a.mrows - 1) : p.sidx;
  if constexpr (SHIFT) {
    const float2 s = s_ldf2(a.shifts + 2 * p.sidx);
    p.sy = s.x;
    p.sx = s.y;
  } else {
    p.sy = p.sx = 0.f;
  }
  return p;
}

// W_b(ky, kx) = exp(-2πi (sy gy + sx gx)), g = ((k + 64) mod 128)/128 (image_proc.py:531 on the
// ifftshifted grid of models.py:179).  K layout: ky = this thread's row, kx = 4qq + r + 64 l0,
// factored as A(qq)·B(r) so a 64-register pass needs 16 + 4 sin/cos pairs.
struct Ramp {
  float2 B[4];
  float sy, sx, gy;
  int l0;
  __device__ __forceinline__ void init(float sy_, float sx_, float gy_, int l0_) {
    sy = rf::opaquef(sy_);
    sx = rf::opaquef(sx_);
    gy = gy_;
    l0 = l0_;
#pragma unroll
    for (int r = 0; r < 4; ++r) B[r] = cis_rev(-sx * (float)r * (1.0f / kN));
  }
  __device__ __forceinline__ float2 a(int qq) const {
    return cis_rev(-fmaf(sy, gy, sx * (float)(4 * qq + 64 * (1 - l0)) * (1.0f / kN)));
  }
};

// QM: 0 → dp_pow q = 1/2 (sqrt / rsqrt), 2 → general q (see loss_point)
//
// Work split: workgroup w owns the contiguous pattern range [w·n/G, (w+1)·n/G).  Everything that
// depends on a mini-batch's NRMSE coefficient c_m (losses.py:45-47) is accumulated with a unit
// coefficient and scaled after k_finalize: the object-gradient slots (k_obj_gather), the
// position-gradient sums (k_shift_apply) and the probe-gradient spectrum, which is kept per
// SEGMENT = maximal run of the range inside one mini-batch (id m + w, unique because every
// segment boundary advances m or w), reduced by k_segslab_reduce.  So no workgroup ever waits
// for another: no arrival counters, no co-residency requirement, any grid size.
//
// Per pattern: IFFT · park ψ⁰, ×O · FFT (DP → LDS meanwhile) · loss partial sums, g_Ψ ·
// IFFT · slot, ×conj(O) · FFT (probe-gradient spectrum) · one pass: segment slab += conj(W) G,
// position-gradient sums, and v = F(P)·W for the next pattern (F(P) read once per pattern).
//
// Two workgroups per CU (≤ 256 VGPRs).  Holding ψ⁰ and the segment slab in AGPRs at one workgroup
// per CU instead of the park and the slab read-modify-write measured the same time
// (profiles/r02/ab/r02l_c2hold: 12.29 vs 12.16 ms), so the kernel parks them.
// MODE (loss_single + loss_poissn, whose mini-batch coefficients are known only after
// k_finalize): 1 = forward and both terms' loss partial sums only (no park, no adjoint; the next
// pattern's v formed right after the sums), 2 = the full pass with ∂ℓ/∂I = c_single u_single +
// c_poissn u_poissn of the pattern's mini-batch (slots / slabs / position sums then carry the
// coefficients; no partial sums written).  0 = one data term, unit coefficient (the c2 kernel).
// HOLD (small calls, at most one workgroup a CU; shifted probes): ψ⁰ stays in registers from the
// first transform to the slot instead of the park round trip (one workgroup a CU leaves the
// register file to it).
template <bool SHIFT, bool SINGLE, int QM, int MODE = 0, bool HOLD = false>
__global__ __launch_bounds__(256, HOLD ? 1 : 2) void k_fused3(F3Args a) {
  static_assert(!HOLD || (SHIFT && MODE == 0), "HOLD: the shifted-probe ring path, one data term");
  using namespace rf;
  __shared__ float2 buf[kLdsElems];
  __shared__ float s_red[4 * 2];
  const Coord cd = coord(threadIdx.x);
  const LaneCtx lc = lane_ctx(cd.lane);
  constexpr float inv_n = 1.0f / kN, inv_n2 = 1.0f / kN2;
  const int w = blockIdx.x, G = gridDim.x;
  const int p0 = (int)((long long)w * a.n_idx / G), p1 = (int)((long long)(w + 1) * a.n_idx / G);
  if (p0 >= p1) return;
  const float occ = a.occp[0], q = a.q;
  const bool tail = a.tail != 0;   // (uniform)
  const int Nx = a.Nx;
  const Rsrc r_fpk = rsrc(a.fpk, kN2 * 8);
  const float gy = (float)((cd.fixed + 64) & 127) * inv_n;   // ifftshifted grid of this thread's ky

  // ---------------------------------------------------------------- prologue: v for the first pattern
  constexpr bool kRing = SHIFT;
  const int lds0 = (int)(size_t)(__attribute__((address_space(3))) float2*)buf;   // LDS byte address
  float2 v[64];
  {
    const int tid = rf::opaque(threadIdx.x);
    const int vpk = 8 * tid;
    const PatInfo pi0 = pat_info<SHIFT>(a, p0);
    Ramp rp;
    rp.init(pi0.sy, pi0.sx, gy, tid & 1);
    pipeline<16>(
        [&](auto C) {
          Ch4x2 t;
#pragma unroll
          for (int r = 0; r < 4; ++r) t.x[r] = ld2(r_fpk, vpk, 2048 * (4 * C + r));
          return t;
        },
        [&](auto C, const Ch4x2& t) {
          const float2 A = rp.a(C);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            // (the same arithmetic as the post4 pass that forms every later pattern's v)
            if constexpr (kRing) v[4 * C + r] = pcm(t.x[r], pcm(A, rp.B[r]));
            else v[4 * C + r] = SHIFT ? cmul(t.x[r], cmul(A, rp.B[r])) : t.x[r];
            pin(v[4 * C + r]);
          }
        });
  }

  // the pattern's scalars are carried over from the previous pattern's post4 pass (which loads
  // them for the next v), and its mini-batch for the segment test: no scalar-load round trips at
  // the top of a pattern
  PatInfo p_nxt = pat_info<SHIFT>(a, p0);
  int m_prev = 0;
  for (int pat = p0; pat < p1; ++pat) {
    // per-thread bases re-derived from an opaque thread id each pattern and pass: keeps LICM /
    // CSE from holding 64 per-register offsets live across the transforms (they would spill)
    const int tid = rf::opaque(threadIdx.x);
    const int fx = fixed_of(tid);
    const int l0 = tid & 1;
    const PatInfo p = p_nxt;
    float2 hold[HOLD ? 64 : 1];   // HOLD: ψ⁰
    // slot (row-permuted): element (y = j + 64 l0, x = fx) at row 2j + l0 → offset 2048·j
    const Rsrc r_slot = rsrc(a.slots + (size_t)pat * kN2, kN2 * 8);
    const int vslot0 = 8 * (l0 * kN + fx);
    // object window: element (j + 64 l0, fx) → offset vobj + 8·Nx·j
    const Rsrc r_obj = rsrc(a.oc + (size_t)p.cy * Nx + p.cx, (unsigned)(((kN - 1) * Nx + kN) * 8));
    const int vobj0 = 8 * (64 * l0 * Nx + fx);
    const int ostr0 = 8 * Nx;
    // ring (kRing): this wave's 16 KiB of the exchange buffer, descriptors of the streamed operands
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int m0w = lds0 + (wv << 14);
    const float2* ringw = buf + (wv << 11);
    const v4u s_obj = srd(a.oc + (size_t)p.cy * Nx + p.cx, (unsigned)(((kN - 1) * Nx + kN) * 8));
    const v4u s_park = srd(a.slots + (size_t)pat * kN2, kN2 * 8);
    const int os = __builtin_amdgcn_readfirstlane(ostr0);
    // post1 ring: the object window, 16 register pairs ahead (A = 1, S = 2 park stores per pair)
    auto issue1 = [&](auto Q, int voff) {
      constexpr int q = decltype(Q)::value;
      dma_m<2 * q>(s_obj, voff, m0w + (q % 16) * 1024, os);
    };
    // ------------------------------------------------ ψ⁰ = F⁻¹(F(P)·W_b)  (R layout)
    if constexpr (SHIFT) {
      fft_inv(v, buf, lc, cd.wsign, [&] {
        if constexpr (kRing) {
          const int vo = dma_off_obj(rf::opaque(tid) & 63, wv, os);
          rf::sfor<0, 16>([&](auto Q) { issue1(Q, vo); });
        }
      });
#pragma unroll
      for (int j = 0; j < 64; ++j) v[j] = pscale(v[j], inv_n2);
    }
    // ------------------------------------------------ park ψ⁰; ψ = ψ⁰·O
    if constexpr (kRing) {
      const int lam = rf::opaque(tid) & 63;
      const int vo = dma_off_obj(lam, wv, os);
      const int vpark = park_off(lam, wv);
      const int io = obj_img(lam);
      const Rsrc r_park = rsrc(a.slots + (size_t)pat * kN2, kN2 * 8);
      rf::sfor<0, 32>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        vm_wait<ring_wait_count(q, 1, 0, 16)>();
        const float2* sl = ringw + (q % 16) * 128;
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          const int j = 2 * q + rb;
          const float2 O = sl[rb * 64 + io];
          if constexpr (HOLD) hold[j] = v[j];
          else if constexpr (MODE != 1) st2(v[j], r_park, vpark, 2048 * j);
          v[j] = pcm(v[j], O);
          pin(v[j]);
        }
        if constexpr (q + 16 < 32) issue1(std::integral_constant<int, q + 16>{}, vo);
        __builtin_amdgcn_sched_barrier(0);
      });
    } else {
      const int vslot = rf::opaque(vslot0), vobj = rf::opaque(vobj0), ostr = rf::opaque(ostr0);
      pipeline<8>(
          [&](auto C) {
            Ch8 t;
#pragma unroll
            for (int r = 0; r < 8; ++r)
              t.x[r] = ld2(r_obj, vobj, ostr * (8 * C + r));
            return t;
          },
          [&](auto C, const Ch8& t) {
#pragma unroll
            for (int r = 0; r < 8; ++r) {
              const int j = 8 * C + r;
              if constexpr (MODE != 1) st2(v[j], r_slot, vslot, 2048 * j);
              v[j] = cmul(v[j], t.x[r]);
              pin(v[j]);
            }
          });
    }
    // ------------------------------------------------ far field; DP → LDS during the row DFTs
    const float* dp = a.meas + (size_t)p.mi * kN2;
    if constexpr (kRing) __syncthreads();   // every wave is done with its ring before the exchange
    fft_fwd(v, buf, lc, cd.wsign, [&] {
      const int lane = cd.lane;
      const int wv = __builtin_amdgcn_readfirstlane(cd.wave);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int gi = wv * 16 + i;                // rows 2gi, 2gi+1 (1 KiB)
        const int r = 2 * gi + (lane >> 5);
        const int sl = lane & 31;
        const int c4 = sl ^ ((r & 7) | ((sl >> 4) << 3));
        __builtin_amdgcn_global_load_lds(dp + r * kN + 4 * c4,
                                         (__attribute__((address_space(3))) void*)((char*)buf + gi * 1024), 16, 0,
                                         kNtAux);
      }
    });
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    float S = 0.f, Ms = 0.f, S2 = 0.f, Ms2 = 0.f;
    const float occ_n2 = occ * inv_n2, occ2_n = 2.0f * occ * inv_n;
    float2 cc = make_float2(0.f, 0.f);   // MODE 2: (c_single, c_poissn) of the pattern's mini-batch
    if constexpr (MODE == 2) cc = s_ldf2(a.coef + (size_t)p.m * kNCoef);
    {
      const int r = (fx + 64) & 127;               // fftshifted DP row of ky
      const int b = 1 - l0;                        // fftshifted column half of kx = k + 64 l0
      const float4* row4 = reinterpret_cast<const float4*>(buf) + r * 32;
      // dp_out through a buffer resource with num_records 0 when not requested: the stores are
      // dropped by the hardware bounds check, so the loop has no branch
      const Rsrc r_dp = rsrc(a.dp_out ? a.dp_out + (size_t)pat * kN2 : a.psums, a.dp_out ? kN2 * 4 : 0);
      const int vdp = 4 * (r * kN + 64 * b);
#pragma unroll
      for (int kq = 0; kq < 16; ++kq) {
        const float4 M4 = row4[(kq + 16 * b) ^ ((r & 7) | (b << 3))];
        const float Mv[4] = {M4.x, M4.y, M4.z, M4.w};
        float Iv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = 4 * kq + e;
          // Ψ = v/N with N a power of two: |Ψ|² occ = |v|² (occ/N²) and g_Ψ = v (2 occ u / N) exactly
          Iv[e] = fmaf(occ_n2, cabs2(v[k]), kDpEps);
          if constexpr (MODE == 1) {
            (void)loss_point<QM, true>(Iv[e], Mv[e], q, a.eps2, S, Ms);
            (void)loss_point<2, false>(Iv[e], Mv[e], a.q2, a.eps2, S2, Ms2);
          } else if constexpr (MODE == 2) {
            const float u = fmaf(cc.x, loss_point<QM, true>(Iv[e], Mv[e], q, a.eps2, S, Ms),
                                 cc.y * loss_point<2, false>(Iv[e], Mv[e], a.q2, a.eps2, S2, Ms2));
            v[k] = pscale(v[k], occ2_n * u);
            pin(v[k]);
          } else {
            const float u = loss_point<QM, SINGLE>(Iv[e], Mv[e], q, a.eps2, S, Ms);
            v[k] = pscale(v[k], occ2_n * u);
            pin(v[k]);
          }
        }
        {
          const __attribute__((ext_vector_type(4))) float i4 = {Iv[0], Iv[1], Iv[2], Iv[3]};
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, i4),
                                                 r_dp, vdp + 16 * kq, 0, 0);
        }
        if (kq & 1) __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (MODE == 1) {
      // both terms' sums, then the next pattern's v (the prologue's arithmetic) and no adjoint
      float v4[4] = {S, Ms, S2, Ms2};
      block_sum4<4>(v4, s_red);
      if (threadIdx.x == 0) {
        float* ps = a.psums + (size_t)pat * kNSum;
#pragma unroll
        for (int i = 0; i < 4; ++i) ps[i] = v4[i];
      }
      const PatInfo pn = pat_info<SHIFT>(a, min(pat + 1, p1 - 1));
      p_nxt = pn;
      const int vpk = rf::opaque(8 * tid);
      Ramp rp;
      rp.init(pn.sy, pn.sx, gy, rf::opaque(tid) & 1);
      pipeline<16>(
          [&](auto C) {
            Ch4x2 t;
#pragma unroll
            for (int r = 0; r < 4; ++r) t.x[r] = ld2(r_fpk, vpk, 2048 * (4 * C + r));
            return t;
          },
          [&](auto C, const Ch4x2& t) {
            const float2 A = rp.a(C);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if constexpr (kRing) v[4 * C + r] = pcm(t.x[r], pcm(A, rp.B[r]));
              else v[4 * C + r] = SHIFT ? cmul(t.x[r], cmul(A, rp.B[r])) : t.x[r];
              pin(v[4 * C + r]);
            }
          });
      continue;
    } else {
      // (block_sum4's first barrier also retires every wave's DP reads before the next exchange)
      float v2[2] = {S, Ms};
      block_sum4<2>(v2, s_red);
      if (MODE == 0 && threadIdx.x == 0) {
        float* ps = a.psums + (size_t)pat * kNSum;
        const int base = SINGLE ? 0 : 2;
        ps[base] = v2[0];
        ps[base + 1] = v2[1];
        ps[2 - base] = 0.f;
        ps[3 - base] = 0.f;
      }
    }
    // ------------------------------------------------ back to real space
    // post3 ring: ψ⁰ park + object window, 8 register pairs ahead (A = 2, S = 2 slot stores)
    auto issue3 = [&](auto Q, int vpo, int voo) {
      constexpr int q = decltype(Q)::value;
      if constexpr (!HOLD) dma_c<4096 * q>(s_park, vpo, m0w + (q % 8) * 2048);
      dma_m<2 * q>(s_obj, voo, m0w + (q % 8) * 2048 + 1024, os);
    };
    fft_inv(v, buf, lc, cd.wsign, [&] {
      if constexpr (kRing) {
        const int lam = rf::opaque(tid) & 63;
        const int vpo = dma_off_park(lam, wv), voo = dma_off_obj(lam, wv, os);
        rf::sfor<0, 8>([&](auto Q) { issue3(Q, vpo, voo); });
      }
    });
    if constexpr (kRing) {
      const int lam = rf::opaque(tid) & 63;
      const int vpo = dma_off_park(lam, wv), voo = dma_off_obj(lam, wv, os);
      const int io = obj_img(lam);
      const int vslot = rf::opaque(vslot0);
      rf::sfor<0, 32>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        vm_wait<ring_wait_count(q, HOLD ? 1 : 2, 0, 8)>();
        const float2* sl = ringw + (q % 8) * 256;
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          const int j = 2 * q + rb;
          float2 ps;
          if constexpr (HOLD) ps = hold[j];
          else ps = sl[rb * 64 + lam];
          const float2 O = sl[128 + rb * 64 + io];
          const float2 gv = pscale(v[j], inv_n);
          // g_O / c_m = g·conj(ψ⁰); HOLD (a small call: the gather reads the slots next) keeps them in L2
          if constexpr (HOLD) st2(pcmc(gv, ps), r_slot, vslot, 2048 * j);
          else st2_stream(pcmc(gv, ps), r_slot, vslot, 2048 * j);
          v[j] = pcmc(gv, O);                                                          // g·conj(O)
          pin(v[j]);
        }
        if constexpr (q + 8 < 32) issue3(std::integral_constant<int, q + 8>{}, vpo, voo);
        __builtin_amdgcn_sched_barrier(0);
      });
    } else {
      const int vslot = rf::opaque(vslot0), vobj = rf::opaque(vobj0), ostr = rf::opaque(ostr0);
      pipeline<16>(
          [&](auto C) {
            Ch4x2 t;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int j = 4 * C + r;
              t.x[r] = ld2(r_slot, vslot, 2048 * j);
              t.y[r] = ld2(r_obj, vobj, ostr * j);
            }
            return t;
          },
          [&](auto C, const Ch4x2& t) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int j = 4 * C + r;
              const float2 gv = cscale(v[j], inv_n);
              st2_stream(cmulc(gv, t.x[r]), r_slot, vslot, 2048 * j);   // g_O / c_m = g·conj(ψ⁰)
              v[j] = cmulc(gv, t.y[r]);                  // g·conj(O)
              pin(v[j]);
            }
          });
    }
    // ------------------------------------------------ probe / position gradient, next pattern's v
    // Segment of this pattern: the run of the range inside mini-batch m, id m + w.  The first
    // pattern of a segment reads its slab through a zero-length buffer resource (loads return 0)
    // and so initialises it; later patterns accumulate.  Without probe/position gradients (tail
    // false) the same pass runs without the FFT and its slab / sums are never used.
    const PatInfo pn = pat_info<SHIFT>(a, min(pat + 1, p1 - 1));
    const bool first = pat == p0 || m_prev != p.m;   // (uniform)
    m_prev = p.m;
    p_nxt = pn;
    const int seg = p.m + w;
    float2* segs = a.segslab + (size_t)seg * kN2;
    const Rsrc r_slab_ld = rsrc(segs, first ? 0u : (unsigned)(kN2 * 8));
    const Rsrc r_slab_st = rsrc(segs, kN2 * 8);
    if (first && threadIdx.x == 0) a.segbid[seg] = p.m;
    if constexpr (kRing) {
      // post4 ring: F(P) + the segment slab, 8 register pairs ahead (A = 2, S = 2 slab stores).
      // The first pattern of a segment streams F(P) in the slab's place (finite) and scales it by
      // zero, which initialises the slab.
      const v4u s_fpk = srd(a.fpk, kN2 * 8);
      const v4u s_slab = first ? s_fpk : srd(segs, kN2 * 8);
      const float keep = first ? 0.f : 1.f;
      auto issue4 = [&](auto Q, int vk) {
        constexpr int q = decltype(Q)::value;
        dma_c<4096 * q>(s_fpk, vk, m0w + (q % 8) * 2048);
        dma_c<4096 * q>(s_slab, vk, m0w + (q % 8) * 2048 + 1024);
      };
      auto pre4 = [&] {
        const int vk = dma_off_k(rf::opaque(tid) & 63, wv);
        rf::sfor<0, 8>([&](auto Q) { issue4(Q, vk); });
      };
      __syncthreads();   // every wave is done with its post3 ring before the exchange
      // G = F(h), K layout (unconditional here: a branch around the FFT spills the 64 points;
      // without probe / position gradients the slab and sums are simply never read)
      fft_fwd(v, buf, lc, cd.wsign, pre4);
      const int lam = rf::opaque(tid) & 63;
      const int vk = dma_off_k(lam, wv);
      const int vpk = rf::opaque(8 * tid);
      const int l0b = rf::opaque(tid) & 1;
      Ramp rc, rn;
      rc.init(p.sy, p.sx, gy, l0b);
      rn.init(pn.sy, pn.sx, gy, l0b);
      float sim = 0.f, kim = 0.f;
      float2 A = make_float2(0.f, 0.f), An = A;
      rf::sfor<0, 32>([&](auto Q) {
        constexpr int q = decltype(Q)::value;
        vm_wait<ring_wait_count(q, 2, 0, 8)>();
        const float2* sl = ringw + (q % 8) * 256;
        if constexpr ((q & 1) == 0) {
          A = rc.a(q >> 1);
          An = rn.a(q >> 1);
        }
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          const int k = 2 * q + rb;
          const int r = k & 3;
          const float2 F = sl[rb * 64 + lam];
          const float2 W = pcm(A, rc.B[r]);
          const float2 FW = pcm(F, W);
          const float im = fmaf(FW.y, v[k].x, -FW.x * v[k].y);     // Im(F(P) W conj(G))
          sim += im;
          kim = fmaf((float)k, im, kim);                          // Σ k·im (k literal)
          {
            const float2 so = sl[128 + rb * 64 + lam];
            const float2 gw = pcmc(v[k], W);                      // + conj(W) G (unit)
            const float2 sn = rf::pf(__builtin_elementwise_fma((rf::v2f){keep, keep}, rf::pv(so), rf::pv(gw)));
            st2(sn, r_slab_st, vpk, 2048 * k);
          }
          v[k] = pcm(F, pcm(An, rn.B[r]));                        // next pattern: F(P)·W_next
          pin(v[k]);
        }
        if constexpr (q + 8 < 32) issue4(std::integral_constant<int, q + 8>{}, vk);
        __builtin_amdgcn_sched_barrier(0);
      });
      {
        float ds[2] = {gy * sim, fmaf(kim, inv_n, 0.5f * (float)(1 - l0b) * sim)};
        block_sum4<2>(ds, s_red);
        if (threadIdx.x == 0) {
          a.dsu[2 * pat] = ds[0];
          a.dsu[2 * pat + 1] = ds[1];
        }
      }
    } else if constexpr (SHIFT) {
      if (tail) fft_fwd(v, buf, lc, cd.wsign);        // G = F(h), K layout
      const int vpk = rf::opaque(8 * tid);
      const int l0b = rf::opaque(tid) & 1;
      Ramp rc, rn;
      rc.init(p.sy, p.sx, gy, l0b);
      rn.init(pn.sy, pn.sx, gy, l0b);
      float sim = 0.f, kim = 0.f;
      pipeline<16>(
          [&](auto C) {
            Ch4x2 t;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int k = 4 * C + r;
              t.x[r] = ld2(r_fpk, vpk, 2048 * k);
              t.y[r] = ld2(r_slab_ld, vpk, 2048 * k);
            }
            return t;
          },
          [&](auto C, const Ch4x2& t) {
            const float2 A = rc.a(C), An = rn.a(C);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int k = 4 * C + r;
              const float2 W = cmul(A, rc.B[r]);
              const float2 FW = cmul(t.x[r], W);
              const float im = fmaf(FW.y, v[k].x, -FW.x * v[k].y);     // Im(F(P) W conj(G))
              sim += im;
              kim = fmaf((float)k, im, kim);                          // Σ k·im (k literal)
              st2(cadd(t.y[r], cmulc(v[k], W)), r_slab_st, vpk, 2048 * k);   // + conj(W) G (unit)
              v[k] = cmul(t.x[r], cmul(An, rn.B[r]));                 // next pattern: F(P)·W_next
              pin(v[k]);
            }
          });
      {
        // Always reduced (a conditional consumer lets the compiler sink all 64 im products into
        // the branch and keep F(P)·W and G live, which spills).
        // Σ g_y·im and Σ g_x·im with g_x = (k + 64(1 − l0))/128
        float ds[2] = {gy * sim, fmaf(kim, inv_n, 0.5f * (float)(1 - l0b) * sim)};
        block_sum4<2>(ds, s_red);
        if (threadIdx.x == 0) {
          a.dsu[2 * pat] = ds[0];
          a.dsu[2 * pat + 1] = ds[1];
        }
      }
    } else {
      const int vpk = rf::opaque(8 * tid);
      pipeline<16>(
          [&](auto C) {
            Ch4x2 t;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              t.x[r] = ld2(r_fpk, vpk, 2048 * (4 * C + r));
              t.y[r] = ld2(r_slab_ld, vpk, 2048 * (4 * C + r));
            }
            return t;
          },
          [&](auto C, const Ch4x2& t) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int j = 4 * C + r;
              st2(cadd(t.y[r], v[j]), r_slab_st, vpk, 2048 * j);   // + h (unit, R layout)
              v[j] = t.x[r];                                       // next pattern: the probe
              pin(v[j]);
            }
          });
    }
  }
}


// ================================================================================= multislice
// k_fused3ms: the same one-pass forward / loss / adjoint for Nz ≥ 2 slices (P = O = 1), the
// c4 shape.  multislice_forward_model_vec_all (forward.py:50-80) and its adjoint:
//   forward   ψ⁰ = F⁻¹(F(P)·W_b)/N²;  for n < Nz:  park ψⁿ in slot plane n;  u = ψⁿ·O_n;
//             n < Nz−1:  ψⁿ⁺¹ = F⁻¹(H ⊙ F(u))/N²           (FFT, ×H/N² in K layout, IFFT)
//   far field Ψ = F(u_{Nz−1})/N, loss, g_Ψ per unit mini-batch coefficient (as k_fused3)
//   adjoint   g = F⁻¹(g_Ψ)/N;  for n = Nz−1 … 0:  slot plane n = g·conj(ψⁿ);  g ← g·conj(O_n);
//             n > 0:  g ← F⁻¹(conj(H) ⊙ F(g))/N²            (the propagator's adjoint)
//   then the probe / position pass on g = ∂ℓ/∂ψ⁰ exactly as k_fused3.
// 4·Nz FFTs per pattern, the algorithmic count: no forward is recomputed.  Each slot plane
// first parks ψⁿ and is overwritten by slice n's object gradient.  With shifts (kRing) the 2·Nz
// per-slice point-wise passes stream their operands through k_fused3's LDS-DMA ring: slice n's
// object window (forward; ψⁿ parked in the ring's park layout) or its park + object window
// (backward) are issued during the preceding inverse FFT, D register pairs ahead of their use.
// MODE: as k_fused3 (1: forward through every slice + both terms' sums, no parks, no adjoint;
// 2: the full pass with both mini-batch coefficients applied; 0: one term, unit coefficient).
template <bool SHIFT, bool SINGLE, int QM, int MODE = 0>
__global__ __launch_bounds__(256, 2) void k_fused3ms(F3Args a) {
  using namespace rf;
  __shared__ float2 buf[kLdsElems];
  __shared__ float s_red[4 * 2];
  const Coord cd = coord(threadIdx.x);
  const LaneCtx lc = lane_ctx(cd.lane);
  constexpr float inv_n = 1.0f / kN, inv_n2 = 1.0f / kN2;
  const int w = blockIdx.x, G = gridDim.x;
  const int p0 = (int)((long long)w * a.n_idx / G), p1 = (int)((long long)(w + 1) * a.n_idx / G);
  if (p0 >= p1) return;
  const float occ = a.occp[0], q = a.q;
  const bool tail = a.tail != 0;
  const int Nx = a.Nx, Nz = a.Nz;
  const size_t plane = (size_t)a.Ny * a.Nx;
  const Rsrc r_fpk = rsrc(a.fpk, kN2 * 8);
  const Rsrc r_hpk = rsrc(a.hpk, kN2 * 8);
  const float gy = (float)((cd.fixed + 64) & 127) * inv_n;
  constexpr bool kRing = SHIFT;
  const int lds0 = (int)(size_t)(__attribute__((address_space(3))) float2*)buf;   // LDS byte address

  float2 v[64];
  {
    const int tid = rf::opaque(threadIdx.x);
    const int vpk = 8 * tid;
    const PatInfo pi0 = pat_info<SHIFT>(a, p0);
    Ramp rp;
    rp.init(pi0.sy, pi0.sx, gy, tid & 1);
    pipeline<16>(
        [&](auto C) {
          Ch4x2 t;
#pragma unroll
          for (int r = 0; r < 4; ++r) t.x[r] = ld2(r_fpk, vpk, 2048 * (4 * C + r));
          return t;
        },
        [&](auto C, const Ch4x2& t) {
          const float2 A = rp.a(C);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[4 * C + r] = SHIFT ? pcm(t.x[r], pcm(A, rp.B[r])) : t.x[r];
            pin(v[4 * C + r]);
          }
        });
  }

  // K-layout pass: v ← v ⊙ (H or conj(H)) / N²  (hpk holds H/N², packed by the host: exact, N² is
  // a power of two)
  auto prop_k = [&](bool conj_h) {
    const int vpk = rf::opaque(8 * rf::opaque(threadIdx.x));
    pipeline<16>(
        [&](auto C) {
          Ch4x2 t;
#pragma unroll
          for (int r = 0; r < 4; ++r) t.x[r] = ld2(r_hpk, vpk, 2048 * (4 * C + r));
          return t;
        },
        [&](auto C, const Ch4x2& t) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int k = 4 * C + r;
            v[k] = conj_h ? pcmc(v[k], t.x[r]) : pcm(v[k], t.x[r]);
            pin(v[k]);
          }
        });
  };

  PatInfo p_nxt = pat_info<SHIFT>(a, p0);   // (carried over as in k_fused3)
  int m_prev = 0;
  for (int pat = p0; pat < p1; ++pat) {
    const int tid = rf::opaque(threadIdx.x);
    const int fx = fixed_of(tid);
    const int l0 = tid & 1;
    const PatInfo p = p_nxt;
    // ring (kRing): this wave's 16 KiB of the exchange buffer; slice n's operand descriptors
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int m0w = lds0 + (wv << 14);
    const float2* ringw = buf + (wv << 11);
    const int os = __builtin_amdgcn_readfirstlane(8 * Nx);
    const unsigned obytes = (unsigned)(((kN - 1) * Nx + kN) * 8);
    auto s_obj = [&](int n) { return srd(a.oc + n * plane + (size_t)p.cy * Nx + p.cx, obytes); };
    auto s_park = [&](int n) { return srd(a.slots + ((size_t)pat * Nz + n) * kN2, kN2 * 8); };
    // forward ring: the object window, 16 register pairs ahead (A = 1)
    auto issue1 = [&](auto Q, const v4u& so, int voff) {
      constexpr int q = decltype(Q)::value;
      dma_m<2 * q>(so, voff, m0w + (q % 16) * 1024, os);
    };
    auto pre1 = [&](int n) {   // (mid() of the inverse FFT before slice n's pass)
      if constexpr (kRing) {
        const v4u so = s_obj(n);
        const int vo = dma_off_obj(rf::opaque(tid) & 63, wv, os);
        rf::sfor<0, 16>([&](auto Q) { issue1(Q, so, vo); });
      }
    };
    // backward ring: slice n's park + object window, 8 register pairs ahead (A = 2)
    auto issue3 = [&](auto Q, const v4u& sp, const v4u& so, int vpo, int voo) {
      constexpr int q = decltype(Q)::value;
      dma_c<4096 * q>(sp, vpo, m0w + (q % 8) * 2048);
      dma_m<2 * q>(so, voo, m0w + (q % 8) * 2048 + 1024, os);
    };
    auto pre3 = [&](int n) {
      if constexpr (kRing) {
        const v4u sp = s_park(n), so = s_obj(n);
        const int lam = rf::opaque(tid) & 63;
        const int vpo = dma_off_park(lam, wv), voo = dma_off_obj(lam, wv, os);
        rf::sfor<0, 8>([&](auto Q) { issue3(Q, sp, so, vpo, voo); });
      }
    };
    if constexpr (SHIFT) {
      fft_inv(v, buf, lc, cd.wsign, [&] { pre1(0); });
#pragma unroll
      for (int j = 0; j < 64; ++j) v[j] = pscale(v[j], inv_n2);
    }
    // ------------------------------------------------ slices: park ψⁿ, ×O_n, propagate
    for (int n = 0; n < Nz; ++n) {
      const Rsrc r_slot = rsrc(a.slots + ((size_t)pat * Nz + n) * kN2, kN2 * 8);
      const Rsrc r_obj = rsrc(a.oc + n * plane + (size_t)p.cy * Nx + p.cx, obytes);
      if constexpr (kRing) {
        const v4u so = s_obj(n);
        const int lam = rf::opaque(tid) & 63;
        const int vo = dma_off_obj(lam, wv, os);
        const int vpark = park_off(lam, wv);
        const int io = obj_img(lam);
        rf::sfor<0, 32>([&](auto Q) {
          constexpr int q = decltype(Q)::value;
          vm_wait<ring_wait_count(q, 1, 0, 16)>();
          const float2* sl = ringw + (q % 16) * 128;
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) {
            const int j = 2 * q + rb;
            const float2 O = sl[rb * 64 + io];
            if constexpr (MODE != 1) st2_stream(v[j], r_slot, vpark, 2048 * j);   // ψⁿ park (ring layout: read back by pre3)
            v[j] = pcm(v[j], O);
            pin(v[j]);
          }
          if constexpr (q + 16 < 32) issue1(std::integral_constant<int, q + 16>{}, so, vo);
          __builtin_amdgcn_sched_barrier(0);
        });
        __syncthreads();   // every wave is done with its ring before the next exchange
      } else {
        const int tq = rf::opaque(threadIdx.x);
        const int vslot = 8 * ((tq & 1) * kN + fixed_of(tq)), vobj = 8 * (64 * (tq & 1) * Nx + fixed_of(tq));
        const int ostr = rf::opaque(8 * Nx);
        pipeline<8>(
            [&](auto C) {
              Ch8 t;
#pragma unroll
              for (int r = 0; r < 8; ++r) t.x[r] = ld2(r_obj, vobj, ostr * (8 * C + r));
              return t;
            },
            [&](auto C, const Ch8& t) {
#pragma unroll
              for (int r = 0; r < 8; ++r) {
                const int j = 8 * C + r;
                if constexpr (MODE != 1) st2(v[j], r_slot, vslot, 2048 * j);
                v[j] = pcm(v[j], t.x[r]);
                pin(v[j]);
              }
            });
      }
      if (n + 1 < Nz) {
        fft_fwd(v, buf, lc, cd.wsign);
        prop_k(false);
        fft_inv(v, buf, lc, cd.wsign, [&] { pre1(n + 1); });
      }
    }
    // ------------------------------------------------ far field; DP → LDS during the row DFTs
    const float* dp = a.meas + (size_t)p.mi * kN2;
    fft_fwd(v, buf, lc, cd.wsign, [&] {
      const int lane = cd.lane;
      const int wv = __builtin_amdgcn_readfirstlane(cd.wave);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int gi = wv * 16 + i;
        const int r = 2 * gi + (lane >> 5);
        const int sl = lane & 31;
        const int c4 = sl ^ ((r & 7) | ((sl >> 4) << 3));
        __builtin_amdgcn_global_load_lds(dp + r * kN + 4 * c4,
                                         (__attribute__((address_space(3))) void*)((char*)buf + gi * 1024), 16, 0,
                                         kNtAux);
      }
    });
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    float S = 0.f, Ms = 0.f, S2 = 0.f, Ms2 = 0.f;
    const float occ_n2 = occ * inv_n2, occ2_n = 2.0f * occ * inv_n;
    float2 cc = make_float2(0.f, 0.f);   // MODE 2: (c_single, c_poissn) of the pattern's mini-batch
    if constexpr (MODE == 2) cc = s_ldf2(a.coef + (size_t)p.m * kNCoef);
    {
      const int r = (fx + 64) & 127;
      const int b = 1 - l0;
      const float4* row4 = reinterpret_cast<const float4*>(buf) + r * 32;
      const Rsrc r_dp = rsrc(a.dp_out ? a.dp_out + (size_t)pat * kN2 : a.psums, a.dp_out ? kN2 * 4 : 0);
      const int vdp = 4 * (r * kN + 64 * b);
#pragma unroll
      for (int kq = 0; kq < 16; ++kq) {
        const float4 M4 = row4[(kq + 16 * b) ^ ((r & 7) | (b << 3))];
        const float Mv[4] = {M4.x, M4.y, M4.z, M4.w};
        float Iv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = 4 * kq + e;
          // Ψ = v/N with N a power of two: occ|Ψ|² = |v|²·(occ/N²) and g_Ψ = v·(2 occ u/N), exactly
          Iv[e] = fmaf(occ_n2, cabs2(v[k]), kDpEps);
          if constexpr (MODE == 1) {
            (void)loss_point<QM, true>(Iv[e], Mv[e], q, a.eps2, S, Ms);
            (void)loss_point<2, false>(Iv[e], Mv[e], a.q2, a.eps2, S2, Ms2);
          } else if constexpr (MODE == 2) {
            const float u = fmaf(cc.x, loss_point<QM, true>(Iv[e], Mv[e], q, a.eps2, S, Ms),
                                 cc.y * loss_point<2, false>(Iv[e], Mv[e], a.q2, a.eps2, S2, Ms2));
            v[k] = pscale(v[k], occ2_n * u);
            pin(v[k]);
          } else {
            const float u = loss_point<QM, SINGLE>(Iv[e], Mv[e], q, a.eps2, S, Ms);
            v[k] = pscale(v[k], occ2_n * u);
            pin(v[k]);
          }
        }
        {
          const __attribute__((ext_vector_type(4))) float i4 = {Iv[0], Iv[1], Iv[2], Iv[3]};
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, i4),
                                                 r_dp, vdp + 16 * kq, 0, 0);
        }
        if (kq & 1) __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (MODE == 1) {
      // both terms' sums, then the next pattern's v (the prologue's arithmetic) and no adjoint
      float v4[4] = {S, Ms, S2, Ms2};
      block_sum4<4>(v4, s_red);
      if (threadIdx.x == 0) {
        float* ps = a.psums + (size_t)pat * kNSum;
#pragma unroll
        for (int i = 0; i < 4; ++i) ps[i] = v4[i];
      }
      const PatInfo pn = pat_info<SHIFT>(a, min(pat + 1, p1 - 1));
      p_nxt = pn;
      const int vpk = rf::opaque(8 * tid);
      Ramp rp;
      rp.init(pn.sy, pn.sx, gy, rf::opaque(tid) & 1);
      pipeline<16>(
          [&](auto C) {
            Ch4x2 t;
#pragma unroll
            for (int r = 0; r < 4; ++r) t.x[r] = ld2(r_fpk, vpk, 2048 * (4 * C + r));
            return t;
          },
          [&](auto C, const Ch4x2& t) {
            const float2 A = rp.a(C);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[4 * C + r] = SHIFT ? pcm(t.x[r], pcm(A, rp.B[r])) : t.x[r];
              pin(v[4 * C + r]);
            }
          });
      continue;
    } else {
      float v2[2] = {S, Ms};
      block_sum4<2>(v2, s_red);
      if (MODE == 0 && threadIdx.x == 0) {
        float* ps = a.psums + (size_t)pat * kNSum;
        const int base = SINGLE ? 0 : 2;
        ps[base] = v2[0];
        ps[base + 1] = v2[1];
        ps[2 - base] = 0.f;
        ps[3 - base] = 0.f;
      }
    }
    fft_inv(v, buf, lc, cd.wsign, [&] { pre3(Nz - 1); });
    // ------------------------------------------------ slices backwards
    for (int n = Nz - 1; n >= 0; --n) {
      const Rsrc r_slot = rsrc(a.slots + ((size_t)pat * Nz + n) * kN2, kN2 * 8);
      const Rsrc r_obj = rsrc(a.oc + n * plane + (size_t)p.cy * Nx + p.cx, obytes);
      const float sc = n == Nz - 1 ? inv_n : 1.0f;   // far-field ortho scale once; propagation scaled in K
      if constexpr (kRing) {
        const v4u sp = s_park(n), so = s_obj(n);
        const int lam = rf::opaque(tid) & 63;
        const int vpo = dma_off_park(lam, wv), voo = dma_off_obj(lam, wv, os);
        const int io = obj_img(lam);
        const int vslot = 8 * ((rf::opaque(tid) & 1) * kN + fixed_of(rf::opaque(tid)));
        rf::sfor<0, 32>([&](auto Q) {
          constexpr int q = decltype(Q)::value;
          vm_wait<ring_wait_count(q, 2, 0, 8)>();
          const float2* sl = ringw + (q % 8) * 256;
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) {
            const int j = 2 * q + rb;
            const float2 ps = sl[rb * 64 + lam];
            const float2 O = sl[128 + rb * 64 + io];
            const float2 gv = pscale(v[j], sc);
            st2_stream(pcmc(gv, ps), r_slot, vslot, 2048 * j);   // slice n: g·conj(ψⁿ)
            v[j] = pcmc(gv, O);                                  // g·conj(O_n)
            pin(v[j]);
          }
          if constexpr (q + 8 < 32) issue3(std::integral_constant<int, q + 8>{}, sp, so, vpo, voo);
          __builtin_amdgcn_sched_barrier(0);
        });
        __syncthreads();   // every wave is done with its ring before the next exchange
      } else {
        const int tq = rf::opaque(threadIdx.x);
        const int vslot = 8 * ((tq & 1) * kN + fixed_of(tq)), vobj = 8 * (64 * (tq & 1) * Nx + fixed_of(tq));
        const int ostr = rf::opaque(8 * Nx);
        pipeline<16>(
            [&](auto C) {
              Ch4x2 t;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int j = 4 * C + r;
                t.x[r] = ld2(r_slot, vslot, 2048 * j);
                t.y[r] = ld2(r_obj, vobj, ostr * j);
              }
              return t;
            },
            [&](auto C, const Ch4x2& t) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int j = 4 * C + r;
                const float2 gv = pscale(v[j], sc);
                st2_stream(pcmc(gv, t.x[r]), r_slot, vslot, 2048 * j);   // slice n: g·conj(ψⁿ)
                v[j] = pcmc(gv, t.y[r]);                                  // g·conj(O_n)
                pin(v[j]);
              }
            });
      }
      if (n > 0) {
        fft_fwd(v, buf, lc, cd.wsign);
        prop_k(true);
        fft_inv(v, buf, lc, cd.wsign, [&] { pre3(n - 1); });
      }
    }
    // ------------------------------------------------ probe / position gradient, next pattern's v
    const PatInfo pn = pat_info<SHIFT>(a, min(pat + 1, p1 - 1));
    const bool first = pat == p0 || m_prev != p.m;
    m_prev = p.m;
    p_nxt = pn;
    const int seg = p.m + w;
    float2* segs = a.segslab + (size_t)seg * kN2;
    const Rsrc r_slab_ld = rsrc(segs, first ? 0u : (unsigned)(kN2 * 8));
    const Rsrc r_slab_st = rsrc(segs, kN2 * 8);
    if (first && threadIdx.x == 0) a.segbid[seg] = p.m;
    if constexpr (SHIFT) {
      if (tail) fft_fwd(v, buf, lc, cd.wsign);
      const int vpk = rf::opaque(8 * tid);
      const int l0b = rf::opaque(tid) & 1;
      Ramp rc, rn;
      rc.init(p.sy, p.sx, gy, l0b);
      rn.init(pn.sy, pn.sx, gy, l0b);
      float sim = 0.f, kim = 0.f;
      pipeline<16>(
          [&](auto C) {
            Ch4x2 t;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int k = 4 * C + r;
              t.x[r] = ld2(r_fpk, vpk, 2048 * k);
              t.y[r] = ld2(r_slab_ld, vpk, 2048 * k);
            }
            return t;
          },
          [&](auto C, const Ch4x2& t) {
            const float2 A = rc.a(C), An = rn.a(C);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int k = 4 * C + r;
              const float2 W = pcm(A, rc.B[r]);
              const float2 FW = pcm(t.x[r], W);
              const float im = fmaf(FW.y, v[k].x, -FW.x * v[k].y);
              sim += im;
              kim = fmaf((float)k, im, kim);
              st2(padd2(t.y[r], pcmc(v[k], W)), r_slab_st, vpk, 2048 * k);
              v[k] = pcm(t.x[r], pcm(An, rn.B[r]));
              pin(v[k]);
            }
          });
      {
        float ds[2] = {gy * sim, fmaf(kim, inv_n, 0.5f * (float)(1 - l0b) * sim)};
        block_sum4<2>(ds, s_red);
        if (threadIdx.x == 0) {
          a.dsu[2 * pat] = ds[0];
          a.dsu[2 * pat + 1] = ds[1];
        }
      }
    } else {
      const int vpk = rf::opaque(8 * tid);
      pipeline<16>(
          [&](auto C) {
            Ch4x2 t;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              t.x[r] = ld2(r_fpk, vpk, 2048 * (4 * C + r));
              t.y[r] = ld2(r_slab_ld, vpk, 2048 * (4 * C + r));
            }
            return t;
          },
          [&](auto C, const Ch4x2& t) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int j = 4 * C + r;
              st2(cadd(t.y[r], v[j]), r_slab_st, vpk, 2048 * j);
              v[j] = t.x[r];
              pin(v[j]);
            }
          });
    }
  }
}

}  // namespace f3
}  // namespace ptyx
