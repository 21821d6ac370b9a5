// ptyx_regfft.hpp — register-resident 128×128 complex fp32 2-D FFT for gfx950 (CDNA4).
//
// One 256-thread workgroup (4 waves) owns one N = 128 pattern; every thread keeps 64 of the
// 16,384 points in registers (128 VGPRs) for the whole forward/adjoint chain, so point-wise
// model work between transforms is plain register arithmetic and the data never round-trips
// through LDS except once per 2-D transform (the row↔column exchange).  Two such workgroups
// fit one CU (64 KiB LDS + ≤ 256 VGPRs each): two patterns in flight per CU, two waves per
// SIMD, so one pattern's barrier / memory waits overlap the other's butterflies.
//
// Index bits.  A point (y, x) has 7 + 7 bits; a thread holds 6 of them in its register index
// and the 8 thread bits (6 lane + 2 wave) hold the rest.  Lane bit 0 ("l0") always carries one
// bit of the dimension being transformed; that radix-2 step runs across the lane pair with a
// DPP quad_perm exchange (no LDS), the other 6 bits run as an in-register DFT64 (radix 8×8,
// compile-time twiddles, no table lookups).
//
//   R layout (real space)   thread: x = (lane>>1) | wave<<5      register j: y = j + 64·l0
//   K layout (k space)      thread: ky = (lane>>1) | wave<<5     register k: kx = k + 64·l0
//
//   fft_fwd  R → K :  F1  column DFT128 over y (DIF: lane radix-2 on y6, then DFT64)  → ky = 2k + l0
//                     T   LDS exchange (two 64 KiB halves)
//                     F2  row DFT128 over x (DIT: DFT64 over x = 2m + l0, then lane radix-2)
//   fft_inv  K → R :  the exact reverse (G2, T⁻¹, G1) with conjugate twiddles; unnormalised.
//
// Both layouts give every thread one fixed coordinate along a row (x or ky) and 64 points of
// a column; the global operands of the point-wise steps are stored (or packed) so that one
// register's load is contiguous across lanes.
//
// Replaces the torch.fft.fft2/ifft2 calls of src/ptyrad/forward.py:63,79 and
// src/ptyrad/utils/image_proc.py:532 for N = 128 (the BASELINE c1/c2/c4 probe size).
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

// Scheduling barrier after every 8-register group of the FFT (keeps the machine scheduler from
// interleaving all 64 registers' work, which needs ~70 extra VGPRs).
#define PTYX_RF_SB() __builtin_amdgcn_sched_barrier(0)

namespace ptyx {
namespace rf {

constexpr int kN = 128;
constexpr int kNT = 256;    // threads per pattern
constexpr int kR = 64;      // complex points per thread
constexpr int kLdsElems = 64 * 128;   // one 64 KiB exchange half (float2)

template <int I, int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

// ------------------------------------------------------------------ compile-time trig
constexpr double kPiD = 3.14159265358979323846264338327950288;
// sin / cos of 2π k / M, argument reduced to (-π, π], Taylor series (error < 1e-15)
constexpr double sin2pi(int k, int M) {
  k = ((k % M) + M) % M;
  if (2 * k > M) k -= M;
  const double x = 2.0 * kPiD * (double)k / (double)M;
  double t = x, s = x;
  for (int i = 1; i < 30; ++i) {
    t *= -x * x / ((2.0 * i) * (2.0 * i + 1.0));
    s += t;
  }
  return s;
}
constexpr double cos2pi(int k, int M) {
  k = ((k % M) + M) % M;
  if (2 * k > M) k -= M;
  const double x = 2.0 * kPiD * (double)k / (double)M;
  double t = 1.0, s = 1.0;
  for (int i = 1; i < 30; ++i) {
    t *= -x * x / ((2.0 * i - 1.0) * (2.0 * i));
    s += t;
  }
  return s;
}

// v · exp(DIR·2πi·K/M), trivial angles without multiplies (DIR = -1 forward, +1 inverse)
template <int M, int K, int DIR>
__device__ __forceinline__ float2 rot(float2 v) {
  constexpr int k = ((K % M) + M) % M;
  if constexpr (k == 0) {
    return v;
  } else if constexpr (4 * k == M) {            // DIR·i
    return DIR < 0 ? make_float2(v.y, -v.x) : make_float2(-v.y, v.x);
  } else if constexpr (2 * k == M) {
    return make_float2(-v.x, -v.y);
  } else if constexpr (4 * k == 3 * M) {        // -DIR·i
    return DIR < 0 ? make_float2(-v.y, v.x) : make_float2(v.y, -v.x);
  } else if constexpr ((8 * k) % M == 0) {      // odd multiples of π/4: (±1 ± i)/√2
    constexpr float h = 0.70710678118654752f;
    constexpr float c = cos2pi(k, M) > 0 ? 1.f : -1.f;
    constexpr float s = (sin2pi(k, M) > 0 ? 1.f : -1.f) * (float)DIR;
    return make_float2(h * (c * v.x - s * v.y), h * (s * v.x + c * v.y));
  } else {
    constexpr float c = (float)cos2pi(k, M);
    constexpr float s = (float)(DIR * sin2pi(k, M));
    return make_float2(fmaf(v.x, c, -v.y * s), fmaf(v.x, s, v.y * c));
  }
}

// v · (lf ? exp(DIR·2πi·K/M) : 1) for lf ∈ {0, 1} (per-lane select of a compile-time twiddle):
// v + lf·v·(W − 1), six VALU ops, no branch.
template <int M, int K, int DIR>
__device__ __forceinline__ float2 rot_sel(float2 v, float lf) {
  constexpr int k = ((K % M) + M) % M;
  if constexpr (k == 0) {
    return v;
  } else {
    constexpr float c1 = (float)(cos2pi(k, M) - 1.0);
    constexpr float s = (float)(DIR * sin2pi(k, M));
    const float ux = fmaf(v.x, c1, -v.y * s);
    const float uy = fmaf(v.x, s, v.y * c1);
    return make_float2(fmaf(lf, ux, v.x), fmaf(lf, uy, v.y));
  }
}

// ------------------------------------------------------------------ in-register DFTs
__device__ __forceinline__ float2 add2(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 sub2(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }

// Packed f32 butterflies (v_pk_add/mul/fma_f32: one instruction per complex add, two per complex
// twiddle multiply, the ±i and odd-π/4 swaps folded into op_sel / neg modifiers).
typedef float v2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v2f pv(float2 a) { return __builtin_bit_cast(v2f, a); }
__device__ __forceinline__ float2 pf(v2f a) { return __builtin_bit_cast(float2, a); }
__device__ __forceinline__ float2 padd(float2 a, float2 b) { return pf(pv(a) + pv(b)); }
__device__ __forceinline__ float2 psub(float2 a, float2 b) { return pf(pv(a) - pv(b)); }
// e + i·o = (e.x − o.y, e.y + o.x)  and  e − i·o = (e.x + o.y, e.y − o.x), one instruction each
__device__ __forceinline__ float2 padd_i(float2 e, float2 o) {
  v2f r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(pv(e)), "v"(pv(o)));
  return pf(r);
}
__device__ __forceinline__ float2 psub_i(float2 e, float2 o) {
  v2f r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(pv(e)), "v"(pv(o)));
  return pf(r);
}
// v·(DIR·i): DIR < 0 → (v.y, −v.x); DIR > 0 → (−v.y, v.x)
template <int DIR>
__device__ __forceinline__ float2 pmul_i(float2 v) {
  v2f r;
  if constexpr (DIR < 0)
    asm("v_pk_add_f32 %0, 0, %1 op_sel:[0,1] op_sel_hi:[0,0] neg_hi:[0,1]" : "=v"(r) : "v"(pv(v)));
  else
    asm("v_pk_add_f32 %0, 0, %1 op_sel:[0,1] op_sel_hi:[0,0] neg_lo:[0,1]" : "=v"(r) : "v"(pv(v)));
  return pf(r);
}
// u = (C·x − S·y, S·x + C·y) for C, S ∈ {±1}: one v_pk_add_f32 (odd multiples of π/4 before √½)
template <int C, int S>
__device__ __forceinline__ v2f prot45(float2 v) {
  v2f r;
  if constexpr (C > 0 && S > 0)
    asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(pv(v)));
  else if constexpr (C > 0 && S < 0)
    asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(pv(v)));
  else if constexpr (C < 0 && S > 0)
    asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[1,1] neg_hi:[1,0]" : "=v"(r) : "v"(pv(v)));
  else
    asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[1,0] neg_hi:[1,1]" : "=v"(r) : "v"(pv(v)));
  return r;
}
// v·(c + i s) for compile-time c, s (bit patterns CB, SB): v_pk_mul (c·x, c·y), then v_pk_fma
// with the swapped v.  The two constants are materialised INSIDE the asm (s_mov_b64 of a
// 32-bit literal; both halves read the low word through op_sel_hi = 0), so the compiler cannot
// hoist ~100 distinct twiddles out of the pattern loop into SGPRs (which spills).
template <int CB, int SB>
__device__ __forceinline__ float2 pcmul_k(float2 v) {
  v2f r;
  unsigned long long k0, k1;
  asm("s_mov_b64 %1, %4\n\t"
      "s_mov_b64 %2, %5\n\t"
      "v_pk_mul_f32 %0, %3, %1 op_sel_hi:[1,0]\n\t"
      "v_pk_fma_f32 %0, %3, %2, %0 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_lo:[0,1,0]"
      : "=&v"(r), "=&s"(k0), "=&s"(k1)
      : "v"(pv(v)), "i"(CB), "i"(SB));
  return pf(r);
}
template <int M, int K, int DIR>
__device__ __forceinline__ float2 prot(float2 v) {
  constexpr int k = ((K % M) + M) % M;
  if constexpr (k == 0) {
    return v;
  } else if constexpr (4 * k == M) {
    return pmul_i<DIR>(v);
  } else if constexpr (2 * k == M) {
    return pf(-pv(v));
  } else if constexpr (4 * k == 3 * M) {
    return pmul_i<-DIR>(v);
  } else if constexpr ((8 * k) % M == 0) {
    constexpr int C = cos2pi(k, M) > 0 ? 1 : -1;
    constexpr int S = (sin2pi(k, M) > 0 ? 1 : -1) * DIR;
    constexpr float h = 0.70710678118654752f;
    return pf(prot45<C, S>(v) * (v2f){h, h});
  } else {
    constexpr float c = (float)cos2pi(k, M);
    constexpr float sn = (float)(DIR * sin2pi(k, M));
    return pcmul_k<__builtin_bit_cast(int, c), __builtin_bit_cast(int, sn)>(v);
  }
}
// butterfly (e + W o, e − W o) with W = exp(DIR·2πi·K/M)
template <int M, int K, int DIR>
__device__ __forceinline__ void pbfly(float2 e, float2 o, float2& a, float2& b) {
  constexpr int k = ((K % M) + M) % M;
  if constexpr (k == 0) {
    a = padd(e, o);
    b = psub(e, o);
  } else if constexpr (4 * k == M) {       // W = DIR·i
    if constexpr (DIR < 0) { a = psub_i(e, o); b = padd_i(e, o); }
    else { a = padd_i(e, o); b = psub_i(e, o); }
  } else if constexpr (2 * k == M) {
    a = psub(e, o);
    b = padd(e, o);
  } else if constexpr (4 * k == 3 * M) {   // W = −DIR·i
    if constexpr (DIR < 0) { a = padd_i(e, o); b = psub_i(e, o); }
    else { a = psub_i(e, o); b = padd_i(e, o); }
  } else if constexpr ((8 * k) % M == 0) {
    constexpr int C = cos2pi(k, M) > 0 ? 1 : -1;
    constexpr int S = (sin2pi(k, M) > 0 ? 1 : -1) * DIR;
    constexpr float h = 0.70710678118654752f;
    const v2f u = prot45<C, S>(o);
    a = pf(__builtin_elementwise_fma(u, (v2f){h, h}, pv(e)));
    b = pf(__builtin_elementwise_fma(u, (v2f){-h, -h}, pv(e)));
  } else {
    const float2 t = prot<M, K, DIR>(o);
    a = padd(e, t);
    b = psub(e, t);
  }
}

// DFT of size R ∈ {2, 4, 8}, natural order in and out (radix-2 DIT recursion)
template <int R, int DIR>
__device__ __forceinline__ void dft(float2 (&v)[R]) {
  if constexpr (R == 2) {
    const float2 a = v[0], b = v[1];
    v[0] = padd(a, b);
    v[1] = psub(a, b);
  } else {
    float2 e[R / 2], o[R / 2];
#pragma unroll
    for (int i = 0; i < R / 2; ++i) {
      e[i] = v[2 * i];
      o[i] = v[2 * i + 1];
    }
    dft<R / 2, DIR>(e);
    dft<R / 2, DIR>(o);
    sfor<0, R / 2>([&](auto kk) {
      constexpr int k = decltype(kk)::value;
      pbfly<R, k, DIR>(e[k], o[k], v[k], v[k + R / 2]);
    });
  }
}

// DFT64 in registers: n = n1 + 8·n2, k = k2 + 8·k1 (radix 8×8, compile-time twiddles W64^(n1·k2))
template <int DIR>
__device__ __forceinline__ void dft64(float2 (&v)[64]) {
  sfor<0, 8>([&](auto I1) {
    constexpr int n1 = decltype(I1)::value;
    float2 t[8];
#pragma unroll
    for (int n2 = 0; n2 < 8; ++n2) t[n2] = v[n1 + 8 * n2];
    dft<8, DIR>(t);
    sfor<0, 8>([&](auto K2) {
      constexpr int k2 = decltype(K2)::value;
      v[n1 + 8 * k2] = prot<64, n1 * k2, DIR>(t[k2]);
    });
    PTYX_RF_SB();
  });
  float2 o[64];
#pragma unroll
  for (int k2 = 0; k2 < 8; ++k2) {
    float2 t[8];
#pragma unroll
    for (int n1 = 0; n1 < 8; ++n1) t[n1] = v[n1 + 8 * k2];
    dft<8, DIR>(t);
#pragma unroll
    for (int k1 = 0; k1 < 8; ++k1) o[k2 + 8 * k1] = t[k1];
    PTYX_RF_SB();
  }
#pragma unroll
  for (int i = 0; i < 64; ++i) v[i] = o[i];
}

// ------------------------------------------------------------------ lane-pair radix-2 (DPP)
// value of the same register in lane ^ 1 (quad_perm [1,0,3,2])
__device__ __forceinline__ float xl1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}

struct LaneCtx {
  float sgn;   // +1 on even lanes, -1 on odd lanes
  float lf;    // 0 on even lanes, 1 on odd lanes
};
__device__ __forceinline__ LaneCtx lane_ctx(int lane) {
  const float lf = (float)(lane & 1);
  return LaneCtx{1.0f - 2.0f * lf, lf};
}

// v·(lf ? W : 1) packed: u = v·(W − 1) (two instructions), v + lf·u (one)
template <int M, int K, int DIR>
__device__ __forceinline__ float2 prot_sel(float2 v, float lf) {
  constexpr int k = ((K % M) + M) % M;
  if constexpr (k == 0) {
    return v;
  } else {
    constexpr float c1 = (float)(cos2pi(k, M) - 1.0);
    constexpr float sn = (float)(DIR * sin2pi(k, M));
    const float2 u = pcmul_k<__builtin_bit_cast(int, c1), __builtin_bit_cast(int, sn)>(v);
    return pf(__builtin_elementwise_fma((v2f){lf, lf}, pv(u), pv(v)));
  }
}
// sgn·m + (m of lane ^ 1), one v_pk_fma after the two DPP moves
__device__ __forceinline__ float2 plane_mix(float2 m, float sgn) {
  const v2f x = {xl1(m.x), xl1(m.y)};
  return pf(__builtin_elementwise_fma((v2f){sgn, sgn}, pv(m), x));
}

// DIF step: even lane a = x0 + x1, odd lane b = (x0 − x1)·W128^(DIR·j), j = register index
template <int DIR>
__device__ __forceinline__ void lane_pre(float2 (&v)[64], LaneCtx c) {
  sfor<0, 64>([&](auto J) {
    constexpr int j = decltype(J)::value;
    const float2 m = v[j];
    v[j] = prot_sel<128, j, DIR>(plane_mix(m, c.sgn), c.lf);
    if constexpr ((j & 7) == 7) PTYX_RF_SB();
  });
}
// DIT step: odd lane twiddles its value by W128^(DIR·j), then even lane E + WO, odd lane E − WO
template <int DIR>
__device__ __forceinline__ void lane_post(float2 (&v)[64], LaneCtx c) {
  sfor<0, 64>([&](auto J) {
    constexpr int j = decltype(J)::value;
    v[j] = plane_mix(prot_sel<128, j, DIR>(v[j], c.lf), c.sgn);
    if constexpr ((j & 7) == 7) PTYX_RF_SB();
  });
}

// ------------------------------------------------------------------ LDS exchange
// Half c of the exchange holds the points with ky6 ^ x6 = c, addressed (row = ky & 63, x):
//   float2 index = row·128 + (x ^ (π(row & 15) << 1)),  π(r) = r1 | r2<<1 | r0<<2 | (r0^r3)<<3.
// The XOR swizzle keeps both sides' ds_write_b64 (16-lane groups) and ds_read_b64 (32-lane
// groups) free of bank conflicts with no padding.
//   column layout (F1 out / G1 in; register k: ky = 2k + l0, thread x): row = 2(k & 31) + l0
//   row layout    (F2 in / G2 out; register m: x = 2m + l0, thread ky):  row = ky & 63
// Logical register k (or m) with bit 5 = h belongs to half h ^ w1 (w1 = wave bit 1 = the
// thread's x6 or ky6).  So that every wave moves the same PHYSICAL registers in round c, waves
// with w1 = 1 keep the two layouts above with register bit 5 flipped (physical p = k ^ 32):
// an in-register DFT64 maps "input sign-flipped on odd n" to "output index + 32", and
// "input index + 32" to "output sign-flipped on odd k" (W64^32 = −1), so flip_odd() before the
// DFT64 that produces the column/row layout and after the one that consumes it is all the
// permutation costs (64 VALU multiplies per flip).  Uniform rounds: no divergent branches, the
// exchange is in place, 64 live points per thread throughout.
__device__ __forceinline__ int swz(int r) {
  return ((r >> 1) & 1) | (((r >> 2) & 1) << 1) | ((r & 1) << 2) | (((r ^ (r >> 3)) & 1) << 3);
}

// v[odd] *= s  (s = −1 on waves with w1 = 1, +1 otherwise; wave-uniform)
__device__ __forceinline__ void flip_odd(float2 (&v)[64], float s) {
#pragma unroll
  for (int i = 1; i < 64; i += 2) {
    v[i] = pf(pv(v[i]) * (v2f){s, s});
  }
}

struct XAddr {
  int col[8];    // column side: float2 index minus (p & 31)·256, for p & 7 = 0..7
  int row[16];   // row side: float2 index minus 2·(p & 16), for p & 15, round 0 (round 1: +64 or −64)
  int rdelta;    // row side: index change from round 0 to round 1 (±64: logical x6 flips)
};

// tid must be opaque to the compiler (keeps the bases inside the caller's pattern loop)
__device__ __forceinline__ XAddr xaddr(int tid) {
  XAddr a;
  const int lane = tid & 63, wave = tid >> 6, l0 = lane & 1, w1 = wave >> 1;
  // column side: x = (lane >> 1) | wave << 5;  r = row & 15 = ((p & 7) << 1) | l0
  const int x = (lane >> 1) | (wave << 5);
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int r = ((p << 1) | l0) & 15;
    a.col[p] = l0 * 128 + (x ^ (swz(r) << 1));
  }
  // row side: row = (lane >> 1) | (wave & 1) << 5; logical m = p ^ 32·w1, x = 2m + l0;
  // index = row·128 + l0 + 2·(m ^ π) = row·128 + l0 + 2·((p & 15) ^ π) + 2·(p & 16) + 64·m5
  const int row = (lane >> 1) | ((wave & 1) << 5);
  const int pr = swz(row & 15);
#pragma unroll
  for (int q = 0; q < 16; ++q) a.row[q] = row * 128 + l0 + 2 * (q ^ pr) + 64 * w1;
  a.rdelta = 64 - 128 * w1;
  return a;
}

template <int H>
__device__ __forceinline__ void x_put_cols(const float2 (&v)[64], float2* buf, const XAddr& a) {
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int p = H * 32 + i;
    buf[a.col[p & 7] + (p & 31) * 256] = v[p];
  }
}
template <int H>
__device__ __forceinline__ void x_get_cols(float2 (&v)[64], const float2* buf, const XAddr& a) {
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int p = H * 32 + i;
    v[p] = buf[a.col[p & 7] + (p & 31) * 256];
  }
}
template <int H>
__device__ __forceinline__ void x_put_rows(const float2 (&v)[64], float2* buf, const XAddr& a) {
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int p = H * 32 + i;
    buf[a.row[p & 15] + (H ? a.rdelta : 0) + 2 * (p & 16)] = v[p];
  }
}
template <int H>
__device__ __forceinline__ void x_get_rows(float2 (&v)[64], const float2* buf, const XAddr& a) {
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int p = H * 32 + i;
    v[p] = buf[a.row[p & 15] + (H ? a.rdelta : 0) + 2 * (p & 16)];
  }
}

__device__ __forceinline__ int opaque(int t) {
  asm volatile("" : "+v"(t));
  return t;
}
__device__ __forceinline__ float opaquef(float t) {
  asm volatile("" : "+v"(t));
  return t;
}

// column layout (F1 output) → row layout (F2 input).  Ends with a workgroup barrier, after which
// the exchange buffer is free.
__device__ __forceinline__ void exchange_fwd(float2 (&v)[64], float2* buf) {
  const XAddr a = xaddr(opaque(threadIdx.x));
  x_put_cols<0>(v, buf, a);
  __syncthreads();
  x_get_rows<0>(v, buf, a);
  __syncthreads();
  x_put_cols<1>(v, buf, a);
  __syncthreads();
  x_get_rows<1>(v, buf, a);
  __syncthreads();
}
// row layout → column layout
__device__ __forceinline__ void exchange_inv(float2 (&v)[64], float2* buf) {
  const XAddr a = xaddr(opaque(threadIdx.x));
  x_put_rows<0>(v, buf, a);
  __syncthreads();
  x_get_cols<0>(v, buf, a);
  __syncthreads();
  x_put_rows<1>(v, buf, a);
  __syncthreads();
  x_get_cols<1>(v, buf, a);
  __syncthreads();
}

// ------------------------------------------------------------------ 2-D transforms
// s = −1 on waves 2-3 (w1 = 1), +1 on waves 0-1: the layout permutation sign of flip_odd.
// Unnormalised forward DFT (exp(-2πi…)), R layout in, K layout out.
// mid() runs right after the exchange (the LDS buffer is free from there to the next exchange).
template <class Mid>
__device__ __forceinline__ void fft_fwd(float2 (&v)[64], float2* buf, LaneCtx c, float s, Mid&& mid) {
  lane_pre<-1>(v, c);
  flip_odd(v, s);
  dft64<-1>(v);
  exchange_fwd(v, buf);
  mid();
  dft64<-1>(v);
  flip_odd(v, s);
  lane_post<-1>(v, c);
}
__device__ __forceinline__ void fft_fwd(float2 (&v)[64], float2* buf, LaneCtx c, float s) {
  fft_fwd(v, buf, c, s, [] {});
}
// Unnormalised inverse DFT (exp(+2πi…)), K layout in, R layout out.
template <class Mid>
__device__ __forceinline__ void fft_inv(float2 (&v)[64], float2* buf, LaneCtx c, float s, Mid&& mid) {
  lane_pre<+1>(v, c);
  flip_odd(v, s);
  dft64<+1>(v);
  exchange_inv(v, buf);
  mid();
  dft64<+1>(v);
  flip_odd(v, s);
  lane_post<+1>(v, c);
}
__device__ __forceinline__ void fft_inv(float2 (&v)[64], float2* buf, LaneCtx c, float s) {
  fft_inv(v, buf, c, s, [] {});
}

// Thread coordinates.  R layout: (y = j + 64·l0, x = fixed); K layout: (ky = fixed, kx = k + 64·l0).
struct Coord {
  int lane, wave, l0, w1;
  float wsign;   // flip_odd sign: −1 on waves with w1 = 1
  int fixed;   // x (R layout) = ky (K layout) = (lane >> 1) | wave << 5
};
__device__ __forceinline__ Coord coord(int tid) {
  Coord c;
  c.lane = tid & 63;
  c.wave = tid >> 6;
  c.l0 = c.lane & 1;
  c.w1 = __builtin_amdgcn_readfirstlane(c.wave >> 1);
  c.wsign = c.w1 ? -1.0f : 1.0f;
  c.fixed = (c.lane >> 1) | (c.wave << 5);
  return c;
}

}  // namespace rf
}  // namespace ptyx
