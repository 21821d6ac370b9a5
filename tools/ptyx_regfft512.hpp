// ptyx_regfft512.hpp — register-resident 128×128 complex fp32 2-D FFT on 512 threads (gfx950).
//
// The 256-thread transform of ptyx_regfft.hpp keeps 64 points a thread (128 VGPRs).  This one
// spreads the same field over 512 threads, 32 points each (64 VGPRs): a pattern then fills a CU
// with 8 waves on its own — half the per-wave work per transform (the latency of a lone pattern:
// the reference's default cadence, one 32-pattern mini-batch per optimizer step) and 64 more
// registers a thread for state that would otherwise round-trip HBM.
//
// Index bits.  A thread holds 5 bits of a point in its register index; of its 9 thread bits the
// two lowest lane bits (l0, l1, a DPP quad) carry two bits of the dimension being transformed and
// the other 7 ((lane >> 2) | wave << 4 = the "fixed" coordinate) the other dimension:
//   R layout (real space)  thread: x = fixed      register j: y = j + 32·l0 + 64·l1
//   K layout (k space)     thread: ky = fixed     register k: kx = 4k + 2·l0 + l1
// fft_fwd R → K: column DFT128 over y by decimation in frequency — lane radix-2 on y6 (partner
//   lane ^ 2, twiddle W128^(y mod 64)), lane radix-2 on y5 (lane ^ 1, W64^(y mod 32)), DFT32 in
//   registers (radix 4×8) — leaves ky = 4k + 2·l0 + l1; ONE LDS exchange (the whole 128 KiB
//   field at once: one workgroup a CU); the same row DFT128 over x.
// fft_inv K → R: the exact reverse with conjugate twiddles (decimation in time), unnormalised.
//
// The exchange.  LDS float2 index = ky·128 + (x ^ m), m a 5-bit function of ky's low bits and
// x5, x6 (an in-row permutation, no padding), chosen so that every access is bank-conflict free:
// ds_write_b64 serves 4 groups of 16 lanes (bank (a/4) mod 32: the 16 lanes' idx mod 16 must
// differ), ds_read_b64 2 groups of 32 (bank (a/4) mod 64: idx mod 32 must differ) —
//   forward  (columns write, rows read)  m_A = x5 | x6<<1 | ky0<<2 | ky1<<3 | ky2<<4
//   inverse  (rows write, columns read)  m_B = x5 | x6<<1 | ky1<<2 | ky0<<3 | ky1<<4
// On the column side (x fixed, ky = 4k + 2·l0 + l1) m is a thread constant except for m_A's ky2 =
// k & 1, so addresses are a base plus an immediate; on the row side (ky fixed) register j lands
// at (j ^ m) + 32·l0 + 64·l1, addressed through a 4 + 8 entry table (one add a register).
//
// Replaces the torch.fft calls of src/ptyrad/forward.py:63,79 and
// src/ptyrad/utils/image_proc.py:532 for N = 128 (the BASELINE c1/c2/c4 probe size).
#pragma once
#include "ptyx_regfft.hpp"

namespace ptyx {
namespace rf2 {

using rf::pf;
using rf::pv;
using rf::v2f;

constexpr int kN = 128;
constexpr int kNT = 512;            // threads per pattern
constexpr int kR = 32;              // complex points per thread
constexpr int kLdsElems = 128 * 128;   // the whole field (128 KiB of float2)

struct Coord {
  int lane, wave, l0, l1;
  int fixed;          // x (R layout) = ky (K layout) = (lane >> 2) | wave << 4
  float lf0, lf1;     // l0, l1 as 0 / 1
  float sg0, sg1;     // +1 / −1 for l0, l1 = 0 / 1
  float lf01;         // l0·l1
};
__device__ __forceinline__ Coord coord(int tid) {
  Coord c;
  c.lane = tid & 63;
  c.wave = tid >> 6;
  c.l0 = c.lane & 1;
  c.l1 = (c.lane >> 1) & 1;
  c.fixed = (c.lane >> 2) | (c.wave << 4);
  c.lf0 = (float)c.l0;
  c.lf1 = (float)c.l1;
  c.sg0 = 1.0f - 2.0f * c.lf0;
  c.sg1 = 1.0f - 2.0f * c.lf1;
  c.lf01 = c.lf0 * c.lf1;
  return c;
}

// ------------------------------------------------------------------ in-register DFT32
// n = n1 + 4·n2, k = k2 + 8·k1: 4 DFT8 over n2, twiddles W32^(n1·k2), 8 DFT4 over n1
template <int DIR>
__device__ __forceinline__ void dft32(float2 (&v)[32]) {
  rf::sfor<0, 4>([&](auto I1) {
    constexpr int n1 = decltype(I1)::value;
    float2 t[8];
#pragma unroll
    for (int n2 = 0; n2 < 8; ++n2) t[n2] = v[n1 + 4 * n2];
    rf::dft<8, DIR>(t);
    rf::sfor<0, 8>([&](auto K2) {
      constexpr int k2 = decltype(K2)::value;
      v[n1 + 4 * k2] = rf::prot<32, n1 * k2, DIR>(t[k2]);
    });
    PTYX_RF_SB();
  });
  float2 o[32];
#pragma unroll
  for (int k2 = 0; k2 < 8; ++k2) {
    float2 t[4];
#pragma unroll
    for (int n1 = 0; n1 < 4; ++n1) t[n1] = v[n1 + 4 * k2];
    rf::dft<4, DIR>(t);
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) o[k2 + 8 * k1] = t[k1];
    PTYX_RF_SB();
  }
#pragma unroll
  for (int i = 0; i < 32; ++i) v[i] = o[i];
}

// ------------------------------------------------------------------ lane radix-2 steps (DPP quad)
__device__ __forceinline__ float xl1(float v) {   // lane ^ 1
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float xl2(float v) {   // lane ^ 2
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
}
// sg·m + (m of the partner lane)
template <int P>
__device__ __forceinline__ float2 mix(float2 m, float sg) {
  const v2f x = P == 1 ? (v2f){xl1(m.x), xl1(m.y)} : (v2f){xl2(m.x), xl2(m.y)};
  return pf(__builtin_elementwise_fma((v2f){sg, sg}, pv(m), x));
}
// v·(DIR·i) on the lanes with l0 = l1 = 1 (the W128^32 = DIR·i factor of stage A), else v
template <int DIR>
__device__ __forceinline__ float2 quarter_sel(float2 v, float lf01) {
  const float2 r = rf::pmul_i<DIR>(v);
  return pf(__builtin_elementwise_fma((v2f){lf01, lf01}, pv(r) - pv(v), pv(v)));
}

// decimation in frequency, stage A (the top bit, partner lane ^ 2): lane l1 = 0 keeps
// x0 + x1, lane l1 = 1 gets (x0 − x1)·W128^(DIR·(j + 32·l0))
template <int DIR>
__device__ __forceinline__ void dif_a(float2 (&v)[32], const Coord& c) {
  rf::sfor<0, 32>([&](auto J) {
    constexpr int j = decltype(J)::value;
    v[j] = quarter_sel<DIR>(rf::prot_sel<128, j, DIR>(mix<2>(v[j], c.sg1), c.lf1), c.lf01);
    if constexpr ((j & 7) == 7) PTYX_RF_SB();
  });
}
// stage B (partner lane ^ 1): l0 = 1 gets (x0 − x1)·W64^(DIR·j)
template <int DIR>
__device__ __forceinline__ void dif_b(float2 (&v)[32], const Coord& c) {
  rf::sfor<0, 32>([&](auto J) {
    constexpr int j = decltype(J)::value;
    v[j] = rf::prot_sel<64, j, DIR>(mix<1>(v[j], c.sg0), c.lf0);
    if constexpr ((j & 7) == 7) PTYX_RF_SB();
  });
}
// decimation in time (the inverse steps, DIR = +1 for the inverse transform): twiddle, then mix
template <int DIR>
__device__ __forceinline__ void dit_b(float2 (&v)[32], const Coord& c) {
  rf::sfor<0, 32>([&](auto J) {
    constexpr int j = decltype(J)::value;
    v[j] = mix<1>(rf::prot_sel<64, j, DIR>(v[j], c.lf0), c.sg0);
    if constexpr ((j & 7) == 7) PTYX_RF_SB();
  });
}
template <int DIR>
__device__ __forceinline__ void dit_a(float2 (&v)[32], const Coord& c) {
  rf::sfor<0, 32>([&](auto J) {
    constexpr int j = decltype(J)::value;
    v[j] = mix<2>(quarter_sel<DIR>(rf::prot_sel<128, j, DIR>(v[j], c.lf1), c.lf01), c.sg1);
    if constexpr ((j & 7) == 7) PTYX_RF_SB();
  });
}

// ------------------------------------------------------------------ LDS exchange
__device__ __forceinline__ int opaque(int t) {
  asm volatile("" : "+v"(t));
  return t;
}

// byte addresses (LDS offsets) a thread's 32 points use on each side of an exchange
struct ColAddr {           // column side: x = fixed, register k → ky = 4k + 2·l0 + l1
  int b[4];                // bases of k < 16 even / odd, k ≥ 16 even / odd
};
struct RowAddr {           // row side: ky = fixed, register j → x = (j ^ m) + 32·l0 + 64·l1
  int hi[4];               // 8·(row·128 + 32·l0 + 64·l1) + 64·((j >> 3) ^ (m >> 3))
  int lo[8];               // 8·((j & 7) ^ (m & 7))
};

// m_A (forward) for the point (ky, x): x5 | x6<<1 | ky0<<2 | ky1<<3 | ky2<<4
__device__ __forceinline__ int m_fwd(int ky, int x) { return ((x >> 5) & 3) | ((ky & 7) << 2); }
// m_B (inverse): x5 | x6<<1 | ky1<<2 | ky0<<3 | ky1<<4
__device__ __forceinline__ int m_inv(int ky, int x) {
  return ((x >> 5) & 3) | (((ky >> 1) & 1) << 2) | ((ky & 1) << 3) | (((ky >> 1) & 1) << 4);
}

template <bool FWD>
__device__ __forceinline__ ColAddr col_addr(int tid) {
  const int lane = tid & 63, x = (lane >> 2) | ((tid >> 6) << 4);
  const int c = 2 * (lane & 1) + ((lane >> 1) & 1);   // ky & 3
  ColAddr a;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int odd = 0; odd < 2; ++odd) {
      const int ky = 4 * (16 * h + odd) + c;
      const int m = FWD ? m_fwd(ky, x) : m_inv(ky, x);
      // the address of register k = 16h + odd; register k adds 4096·(k & 14) as an immediate
      // (ky·128·8 = 4096·k + 1024·c)
      a.b[2 * h + odd] = 8 * (ky * 128 + (x ^ m));
    }
  return a;
}

template <bool FWD>
__device__ __forceinline__ RowAddr row_addr(int tid) {
  const int lane = tid & 63, ky = (lane >> 2) | ((tid >> 6) << 4);
  const int l0 = lane & 1, l1 = (lane >> 1) & 1;
  const int m = FWD ? m_fwd(ky, 32 * l0 + 64 * l1) : m_inv(ky, 32 * l0 + 64 * l1);
  RowAddr a;
#pragma unroll
  for (int h = 0; h < 4; ++h) a.hi[h] = 8 * (ky * 128 + 32 * l0 + 64 * l1) + 64 * (h ^ (m >> 3));
#pragma unroll
  for (int l = 0; l < 8; ++l) a.lo[l] = 8 * (l ^ (m & 7));
  return a;
}

__device__ __forceinline__ void lds_st(char* base, int off, float2 v) {
  *reinterpret_cast<float2*>(base + off) = v;
}
__device__ __forceinline__ float2 lds_ld(const char* base, int off) {
  return *reinterpret_cast<const float2*>(base + off);
}

// column side → LDS (register k at ky = 4k + c)
__device__ __forceinline__ void put_cols(const float2 (&v)[32], float2* buf, const ColAddr& a) {
  char* b = reinterpret_cast<char*>(buf);
#pragma unroll
  for (int k = 0; k < 32; ++k) lds_st(b, a.b[2 * (k >> 4) + (k & 1)] + 4096 * (k & 14), v[k]);
}
__device__ __forceinline__ void get_cols(float2 (&v)[32], const float2* buf, const ColAddr& a) {
  const char* b = reinterpret_cast<const char*>(buf);
#pragma unroll
  for (int k = 0; k < 32; ++k) v[k] = lds_ld(b, a.b[2 * (k >> 4) + (k & 1)] + 4096 * (k & 14));
}
__device__ __forceinline__ void put_rows(const float2 (&v)[32], float2* buf, const RowAddr& a) {
  char* b = reinterpret_cast<char*>(buf);
#pragma unroll
  for (int j = 0; j < 32; ++j) lds_st(b, a.hi[j >> 3] + a.lo[j & 7], v[j]);
}
__device__ __forceinline__ void get_rows(float2 (&v)[32], const float2* buf, const RowAddr& a) {
  const char* b = reinterpret_cast<const char*>(buf);
#pragma unroll
  for (int j = 0; j < 32; ++j) v[j] = lds_ld(b, a.hi[j >> 3] + a.lo[j & 7]);
}

// column layout → row layout; ends with a workgroup barrier (the buffer is free afterwards)
__device__ __forceinline__ void exchange_fwd(float2 (&v)[32], float2* buf) {
  const int tid = opaque(threadIdx.x);
  put_cols(v, buf, col_addr<true>(tid));
  __syncthreads();
  get_rows(v, buf, row_addr<true>(tid));
  __syncthreads();
}
// row layout → column layout
__device__ __forceinline__ void exchange_inv(float2 (&v)[32], float2* buf) {
  const int tid = opaque(threadIdx.x);
  put_rows(v, buf, row_addr<false>(tid));
  __syncthreads();
  get_cols(v, buf, col_addr<false>(tid));
  __syncthreads();
}

// ------------------------------------------------------------------ 2-D transforms
// Unnormalised forward DFT (exp(−2πi…)), R layout in, K layout out.  mid() runs right after the
// exchange (the LDS buffer is free from there to the next exchange).
template <class Mid>
__device__ __forceinline__ void fft_fwd(float2 (&v)[32], float2* buf, const Coord& c, Mid&& mid) {
  dif_a<-1>(v, c);
  dif_b<-1>(v, c);
  dft32<-1>(v);
  exchange_fwd(v, buf);
  mid();
  dif_a<-1>(v, c);
  dif_b<-1>(v, c);
  dft32<-1>(v);
}
__device__ __forceinline__ void fft_fwd(float2 (&v)[32], float2* buf, const Coord& c) {
  fft_fwd(v, buf, c, [] {});
}
// Unnormalised inverse DFT (exp(+2πi…)), K layout in, R layout out.
template <class Mid>
__device__ __forceinline__ void fft_inv(float2 (&v)[32], float2* buf, const Coord& c, Mid&& mid) {
  dft32<+1>(v);
  dit_b<+1>(v, c);
  dit_a<+1>(v, c);
  exchange_inv(v, buf);
  mid();
  dft32<+1>(v);
  dit_b<+1>(v, c);
  dit_a<+1>(v, c);
}
__device__ __forceinline__ void fft_inv(float2 (&v)[32], float2* buf, const Coord& c) {
  fft_inv(v, buf, c, [] {});
}

}  // namespace rf2
}  // namespace ptyx
