// ptyx_fft.hpp — workgroup-resident 2-D complex FFTs for gfx950 (CDNA4), fp32.
//
// One workgroup transforms one N×N complex64 array.  The array lives either in LDS
// (N ≤ 128: 128·136·8 B = 136 KiB, in place) or in a per-workgroup global scratch pair
// (N = 256, ping-pong).  Each 1-D pass is a Stockham radix-R iteration (natural order in
// and out; Govindaraju et al. 2008 indexing, checked against numpy in tests): every thread
// loads R points of one line, applies the stage twiddles (fp64-rounded table in LDS),
// runs an in-register DFT_R and stores R points.  Rows are transformed first, then
// columns.  Point-wise work that sits between FFTs in the ptychography model (probe
// shift ramps, object multiply, propagator, |·|², loss gradient, scatter-add) is fused
// into the first stage's loads ("pre") and the last stage's stores ("post"), so data
// makes one trip through LDS per stage and none through HBM.
//
// Replaces the torch.fft calls of src/ptyrad/forward.py:63,79 and
// src/ptyrad/utils/image_proc.py:532 (pocketfft on CPU / hipFFT on GPU in the reference).
#pragma once
#include <hip/hip_runtime.h>
#include <type_traits>

namespace ptyx {

// ---------------------------------------------------------------- complex helpers
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}
// a * conj(b)
__device__ __forceinline__ float2 cmulc(float2 a, float2 b) {
  return make_float2(fmaf(a.x, b.x, a.y * b.y), fmaf(a.y, b.x, -a.x * b.y));
}
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
__device__ __forceinline__ float cabs2(float2 a) { return fmaf(a.x, a.x, a.y * a.y); }

// cos/sin(2πk/16), correctly rounded to fp32
__device__ constexpr float kCos16[16] = {
    1.0f, 0.92387953251128674f, 0.70710678118654752f, 0.38268343236508977f,
    0.0f, -0.38268343236508977f, -0.70710678118654752f, -0.92387953251128674f,
    -1.0f, -0.92387953251128674f, -0.70710678118654752f, -0.38268343236508977f,
    0.0f, 0.38268343236508977f, 0.70710678118654752f, 0.92387953251128674f};
__device__ constexpr float kSin16[16] = {
    0.0f, 0.38268343236508977f, 0.70710678118654752f, 0.92387953251128674f,
    1.0f, 0.92387953251128674f, 0.70710678118654752f, 0.38268343236508977f,
    0.0f, -0.38268343236508977f, -0.70710678118654752f, -0.92387953251128674f,
    -1.0f, -0.92387953251128674f, -0.70710678118654752f, -0.38268343236508977f};

// v · exp(DIR·2πi·K/R), trivial rotations without multiplies (DIR = -1 forward, +1 inverse)
template <int R, int K, int DIR>
__device__ __forceinline__ float2 twmul(float2 v) {
  constexpr int k16 = (K * (16 / R)) & 15;
  if constexpr (k16 == 0) {
    return v;
  } else if constexpr (k16 == 4) {  // DIR·i
    return DIR < 0 ? make_float2(v.y, -v.x) : make_float2(-v.y, v.x);
  } else if constexpr (k16 == 8) {
    return make_float2(-v.x, -v.y);
  } else if constexpr (k16 == 12) {  // -DIR·i
    return DIR < 0 ? make_float2(-v.y, v.x) : make_float2(v.y, -v.x);
  } else {
    return cmul(v, make_float2(kCos16[k16], DIR * kSin16[k16]));
  }
}

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// compile-time sin / cos of 2πk/M (argument reduced to (-π, π], Taylor series, error < 1e-15)
constexpr double ct_sin2pi(int k, int M) {
  k = ((k % M) + M) % M;
  if (2 * k > M) k -= M;
  const double x = 2.0 * 3.14159265358979323846264338327950288 * (double)k / (double)M;
  double t = x, s = x;
  for (int i = 1; i < 30; ++i) {
    t *= -x * x / ((2.0 * i) * (2.0 * i + 1.0));
    s += t;
  }
  return s;
}
constexpr double ct_cos2pi(int k, int M) {
  k = ((k % M) + M) % M;
  if (2 * k > M) k -= M;
  const double x = 2.0 * 3.14159265358979323846264338327950288 * (double)k / (double)M;
  double t = 1.0, s = 1.0;
  for (int i = 1; i < 30; ++i) {
    t *= -x * x / ((2.0 * i - 1.0) * (2.0 * i));
    s += t;
  }
  return s;
}

// v · exp(DIR·2πi·E/R) with compile-time constants; the quarter-turn rotations without multiplies.
template <int R, int E, int DIR>
__device__ __forceinline__ float2 ctwmul(float2 v) {
  constexpr int e = E % R;
  if constexpr (e == 0) {
    return v;
  } else if constexpr (4 * e == R) {   // DIR·i
    return DIR < 0 ? make_float2(v.y, -v.x) : make_float2(-v.y, v.x);
  } else if constexpr (2 * e == R) {
    return make_float2(-v.x, -v.y);
  } else if constexpr (4 * e == 3 * R) {
    return DIR < 0 ? make_float2(-v.y, v.x) : make_float2(v.y, -v.x);
  } else {
    constexpr float c = (float)ct_cos2pi(e, R), s = (float)((double)DIR * ct_sin2pi(e, R));
    return make_float2(fmaf(v.x, c, -v.y * s), fmaf(v.x, s, v.y * c));
  }
}

constexpr int ct_smallest_factor(int R) {
  for (int f = 2; f * f <= R; ++f)
    if (R % f == 0) return f;
  return R;
}

// Direct DFT of a prime size (radix 3, 5, 7 of mixed-radix N): X[k] = Σ_n v[n] exp(DIR·2πi nk/R),
// compile-time twiddles, (R-1)² complex multiply-adds.
template <int R, int DIR>
__device__ __forceinline__ void dft_direct(float2 (&v)[R]) {
  float2 out[R];
  static_for<0, R>([&](auto KK) {
    constexpr int k = decltype(KK)::value;
    float2 acc = v[0];
    static_for<1, R>([&](auto NN) {
      constexpr int n = decltype(NN)::value;
      acc = cadd(acc, ctwmul<R, n * k, DIR>(v[n]));
    });
    out[k] = acc;
  });
#pragma unroll
  for (int k = 0; k < R; ++k) v[k] = out[k];
}

// In-register DFT of size R, natural order in and out.  Powers of two: radix-2 DIT recursion;
// composite R = F·M (F its smallest prime factor): decimation in time, F sub-DFTs of size M over
// n ≡ n1 (mod F), twiddles W_R^{n1·k1}, then M DFTs of size F (X[k1 + M·k2]); prime R: direct.
template <int R, int DIR>
struct DFT {
  __device__ __forceinline__ static void run(float2 (&v)[R]) {
    constexpr int F = ct_smallest_factor(R);
    if constexpr ((R & (R - 1)) == 0) {
      run_pow2(v);
    } else if constexpr (F == R) {
      dft_direct<R, DIR>(v);
    } else {
      constexpr int M = R / F;
      float2 sub[F][M];
#pragma unroll
      for (int n1 = 0; n1 < F; ++n1)
#pragma unroll
        for (int n2 = 0; n2 < M; ++n2) sub[n1][n2] = v[n1 + F * n2];
      static_for<0, F>([&](auto N1) {
        constexpr int n1 = decltype(N1)::value;
        DFT<M, DIR>::run(sub[n1]);
        static_for<1, M>([&](auto K1) {
          constexpr int k1 = decltype(K1)::value;
          sub[n1][k1] = ctwmul<R, n1 * k1, DIR>(sub[n1][k1]);
        });
      });
#pragma unroll
      for (int k1 = 0; k1 < M; ++k1) {
        float2 t[F];
#pragma unroll
        for (int n1 = 0; n1 < F; ++n1) t[n1] = sub[n1][k1];
        DFT<F, DIR>::run(t);
#pragma unroll
        for (int k2 = 0; k2 < F; ++k2) v[k1 + M * k2] = t[k2];
      }
    }
  }
  __device__ __forceinline__ static void run_pow2(float2 (&v)[R]) {
    float2 e[R / 2], o[R / 2];
#pragma unroll
    for (int i = 0; i < R / 2; ++i) {
      e[i] = v[2 * i];
      o[i] = v[2 * i + 1];
    }
    DFT<R / 2, DIR>::run(e);
    DFT<R / 2, DIR>::run(o);
    static_for<0, R / 2>([&](auto kk) {
      constexpr int k = decltype(kk)::value;
      // (the 16-entry table covers R ≤ 16; R = 32, the first pass of N = 512, takes ctwmul)
      float2 t;
      if constexpr (R <= 16) t = twmul<R, k, DIR>(o[k]);
      else t = ctwmul<R, k, DIR>(o[k]);
      v[k] = cadd(e[k], t);
      v[k + R / 2] = csub(e[k], t);
    });
  }
};
template <int DIR>
struct DFT<2, DIR> {
  __device__ __forceinline__ static void run(float2 (&v)[2]) {
    const float2 a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
  }
};
template <int DIR>
struct DFT<4, DIR> {
  __device__ __forceinline__ static void run(float2 (&v)[4]) {
    const float2 a0 = cadd(v[0], v[2]), a1 = csub(v[0], v[2]);
    const float2 a2 = cadd(v[1], v[3]), a3 = twmul<4, 1, DIR>(csub(v[1], v[3]));
    v[0] = cadd(a0, a2);
    v[2] = csub(a0, a2);
    v[1] = cadd(a1, a3);
    v[3] = csub(a1, a3);
  }
};

// ---------------------------------------------------------------- radix plans
// Per-dimension Stockham radices: N = R1·R2 (R2 = 1 ⇒ one pass per dimension).  Powers of two
// keep their measured plans; every other 2·3·5·7-smooth N ≤ 256 takes the largest R1 ≤ 16 with
// N / R1 ≤ 16, else the smallest R1 ≤ 49 with N / R1 ≤ 16 (125, 162, 175, 189, 200, 216, 243,
// 245 = 35·7, 250); N in (256, 512] the smallest divisor R1 ≥ √N (512 = 32·16, 441 = 21·21,
// 343 = 49·7).  Radix 7 (and 14, 21, 28, 35, 49) runs as a direct DFT (dft_direct) or by
// decimation in time inside DFT<R>.
constexpr int kMaxRadix = 49;   // largest Stockham radix (points a thread holds in one pass)
constexpr bool is_smooth235(int n) {
  if (n < 1) return false;
  for (int f : {2, 3, 5, 7})
    while (n % f == 0) n /= f;
  return n == 1;
}
constexpr int plan_r1(int N) {
  switch (N) {
    case 16: return 16;
    case 32: return 8;
    case 64: return 8;
    case 128: return 16;
    case 256: return 16;
    default: break;
  }
  if (N > 256) {   // the smallest divisor ≥ √N: the most balanced two-pass split (R1 ≤ 49: 343 = 49·7)
    for (int r = 2; r <= N; ++r)
      if (N % r == 0 && r * r >= N) return r <= kMaxRadix ? r : 0;
    return 0;
  }
  for (int r = 16; r >= 2; --r)
    if (N % r == 0 && N / r <= 16) return r;
  for (int r = 17; r <= 27; ++r)
    if (N % r == 0 && N / r <= 16) return r;
  for (int r = 28; r <= kMaxRadix; ++r)   // 245 = 35·7
    if (N % r == 0 && N / r <= 16) return r;
  return 0;
}
template <int N>
struct Plan1D {
  static_assert(is_smooth235(N) && plan_r1(N) > 0, "N must be 2·3·5·7-smooth with a two-pass plan");
  static constexpr int R1 = plan_r1(N), R2 = N / plan_r1(N);
};

// ---------------------------------------------------------------- array views
// LDS view, in place.  Row stride N + N/16 and one pad point per 16 spreads the
// strided Stockham accesses over the banks (ds_read_b64 / ds_write_b64).
template <int N>
struct LdsArray {
  static constexpr bool kInPlace = true;
  static constexpr int kRowStride = N + N / 16;
  static constexpr int kElems = N * kRowStride;
  float2* p;
  __device__ __forceinline__ int off(int y, int x) const { return y * kRowStride + x + (x >> 4); }
  __device__ __forceinline__ float2 ld(int y, int x) const { return p[off(y, x)]; }
  __device__ __forceinline__ void st(int y, int x, float2 v) const { p[off(y, x)] = v; }
};

// Global scratch pair for arrays that do not fit LDS (N = 256); ping-pong between a and b.
// lds: the workgroup's line-block tile (kG256Elems float2) when the two-stage path is used.
template <int N>
struct GlobalPair {
  static constexpr bool kInPlace = false;
  float2* a;
  float2* b;
  float2* lds = nullptr;
  __device__ __forceinline__ float2 ld(int y, int x) const { return a[y * N + x]; }
  __device__ __forceinline__ void st(int y, int x, float2 v) const { a[y * N + x] = v; }
};
template <int N>
struct GlobalView {
  float2* p;
  __device__ __forceinline__ float2 ld(int y, int x) const { return p[y * N + x]; }
  __device__ __forceinline__ void st(int y, int x, float2 v) const { p[y * N + x] = v; }
};

// stage kinds
enum : int { kMid = 0, kFirst = 1, kLast = 2 };

// Fused pre/post element group size between scheduling barriers.  Without it hipcc hoists every element's global loads of a 16-point
// epilogue ahead of the arithmetic and spills at 128 VGPRs (1024-thread workgroups).
constexpr int kFuseGroup = 4;

// twiddle table tw[m] = exp(-2πi m / N) (fp64 rounded), conj for inverse
template <int DIR>
__device__ __forceinline__ float2 twiddle(const float2* tw, int m) {
  const float2 w = tw[m];
  return DIR < 0 ? w : make_float2(w.x, -w.y);
}

// pre/post hooks come in two forms: (y, x, v) and slot-aware (y, x, v, slot), where slot =
// kb·R + r enumerates a thread's points of the pass (see PassMap).  Slot-aware hooks read
// values the caller prefetched into registers for exactly those points, so they carry no
// global-memory latency and are scheduled freely.
template <class F>
constexpr bool kSlotPre = std::is_invocable_v<F&, int, int, float2, int>;
template <class F>
constexpr bool kSlotPost = std::is_invocable_v<F&, int, int, float2&, int>;

template <class F>
__device__ __forceinline__ float2 call_pre(F& f, int y, int x, float2 v, int slot) {
  if constexpr (kSlotPre<F>) return f(y, x, v, slot);
  else return f(y, x, v);
}
template <class F>
__device__ __forceinline__ bool call_post(F& f, int y, int x, float2& v, int slot) {
  if constexpr (kSlotPost<F>) return f(y, x, v, slot);
  else return f(y, x, v);
}

// Points (y, x) a thread owns in the first (row, radix R1) and last (column) pass of fft2d on
// an LDS array: the same formulas as stockham_pass, for register prefetch outside the FFT.
template <int N, int NT>
struct PassMap {
  using P1 = Plan1D<N>;
  static constexpr int R1 = P1::R1;
  static constexpr int RL = P1::R2 == 1 ? P1::R1 : P1::R2;   // radix of the last pass
  static constexpr int NSL = P1::R2 == 1 ? 1 : P1::R1;        // its Stockham span
  static constexpr int KBF = (N * N / R1 + NT - 1) / NT;
  static constexpr int KBL = (N * N / RL + NT - 1) / NT;
  static constexpr int kFirstSlots = KBF * R1;
  static constexpr int kLastSlots = KBL * RL;
  // Idle slots (only when NT does not divide the butterfly count) are clamped onto a valid
  // point so that register prefetches can be unconditional: a conditionally written register
  // array becomes loop-carried and stays live across the whole pattern loop.
  __device__ __forceinline__ static void first(int tid, int slot, int& y, int& x) {
    const int kb = slot / R1, r = slot % R1;
    const int bf = min(tid + kb * NT, N * N / R1 - 1);
    y = bf / (N / R1);
    x = bf % (N / R1) + r * (N / R1);
  }
  __device__ __forceinline__ static void last(int tid, int slot, int& y, int& x) {
    const int kb = slot / RL, r = slot % RL;
    const int bf = min(tid + kb * NT, N * N / RL - 1);
    const int j = bf / N;
    x = bf % N;
    y = (j / NSL) * NSL * RL + (j % NSL) + r * NSL;
  }
  __device__ __forceinline__ static bool last_active(int tid, int slot) {
    return tid + (slot / RL) * NT < N * N / RL;
  }
};

// One Stockham pass of radix R over all N lines.  ROW: lines are rows (x varies).
//  PRELOAD (first pass only): whether to load the source before calling pre(y,x,v).
//  post(y,x,v) (last pass only) may modify v and returns true if v must be stored.
template <int N, int NT, int R, int NS, bool ROW, int DIR, int KIND, bool PRELOAD, bool INPLACE, class Src,
          class Dst, class Pre, class Post>
__device__ __forceinline__ void stockham_pass(const Src& src, const Dst& dst, const float2* tw, Pre& pre,
                                              Post& post) {
  constexpr int NB = N * N / R;           // butterflies in this pass
  constexpr int L = N / R;                // butterflies per line
  constexpr int TWS = N / (NS * R);       // twiddle table stride
  // Opaque copy of threadIdx.x: keeps hipcc from hoisting every pass's per-element LDS
  // addresses out of the persistent pattern loop (loop-invariant code motion of ~300 address
  // registers, all spilled at the 128-VGPR cap).  Recomputing them is a few VALU ops per point.
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  if constexpr (INPLACE) {
    constexpr int KB = (NB + NT - 1) / NT;
    float2 v[KB][R];
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const int bf = tid + kb * NT;
      if ((NB % NT) == 0 || bf < NB) {
        const int line = ROW ? bf / L : bf % N;
        const int j = ROW ? bf % L : bf / N;
        const int k = j % NS;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int e = j + r * L;
          const int y = ROW ? line : e, x = ROW ? e : line;
          float2 val;
          if constexpr (KIND & kFirst) {
            if constexpr (PRELOAD) val = call_pre(pre, y, x, src.ld(y, x), kb * R + r);
            else val = call_pre(pre, y, x, make_float2(0.f, 0.f), kb * R + r);
            if constexpr (kFuseGroup > 0 && !kSlotPre<Pre>) {
              if ((r + 1) % kFuseGroup == 0) __builtin_amdgcn_sched_barrier(0);
            }
          } else {
            val = src.ld(y, x);
          }
          if constexpr (NS > 1) {
            if (r > 0) val = cmul(val, twiddle<DIR>(tw, k * r * TWS));
          }
          v[kb][r] = val;
        }
        DFT<R, DIR>::run(v[kb]);
      }
    }
    __syncthreads();
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const int bf = tid + kb * NT;
      if ((NB % NT) == 0 || bf < NB) {
        const int line = ROW ? bf / L : bf % N;
        const int j = ROW ? bf % L : bf / N;
        const int k = j % NS;
        const int d0 = (j / NS) * NS * R + k;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int e = d0 + r * NS;
          const int y = ROW ? line : e, x = ROW ? e : line;
          float2 val = v[kb][r];
          if constexpr (KIND & kLast) {
            if (call_post(post, y, x, val, kb * R + r)) dst.st(y, x, val);
            // bound the compiler's hoisting of the fused epilogue's global loads
            if constexpr (kFuseGroup > 0 && !kSlotPost<Post>) {
              if ((r + 1) % kFuseGroup == 0) __builtin_amdgcn_sched_barrier(0);
            }
          } else {
            dst.st(y, x, val);
          }
        }
      }
    }
    __syncthreads();
  } else {
    for (int bf = tid; bf < NB; bf += NT) {
      const int line = ROW ? bf / L : bf % N;
      const int j = ROW ? bf % L : bf / N;
      const int k = j % NS;
      float2 v[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int e = j + r * L;
        const int y = ROW ? line : e, x = ROW ? e : line;
        float2 val;
        if constexpr (KIND & kFirst) {
          if constexpr (PRELOAD) val = call_pre(pre, y, x, src.ld(y, x), r);
          else val = call_pre(pre, y, x, make_float2(0.f, 0.f), r);
        } else {
          val = src.ld(y, x);
        }
        if constexpr (NS > 1) {
          if (r > 0) val = cmul(val, twiddle<DIR>(tw, k * r * TWS));
        }
        v[r] = val;
      }
      DFT<R, DIR>::run(v);
      const int d0 = (j / NS) * NS * R + k;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int e = d0 + r * NS;
        const int y = ROW ? line : e, x = ROW ? e : line;
        float2 val = v[r];
        if constexpr (KIND & kLast) {
          if (call_post(post, y, x, val, r)) dst.st(y, x, val);
        } else {
          dst.st(y, x, val);
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- N = 256, two stages
// A 256² complex array (512 KiB) does not fit one CU, so each 2-D FFT makes ONE round trip
// through the workgroup's global scratch instead of one per Stockham pass: stage 1 transforms
// 32-row blocks (512 threads, 16 a row; ≈ 78 KiB of LDS, two workgroups a CU) entirely on chip (DFT16 over n2, twiddle W256^(n1·k2), LDS exchange, DFT16
// over n1) and stores the block TRANSPOSED, so stage 2 is the same row kernel on the
// transposed array, whose transposed store restores the natural orientation.  Both stores go
// through an LDS tile and leave as 32 consecutive points (256 B) per line.  The multislice
// chains fuse the stages of consecutive transforms further (g256_fstage).
constexpr int kG256Threads = 512;                       // workgroup size of the N = 256 kernels
constexpr int kG256Rows = kG256Threads / 16;            // rows per block: 16 threads a row
constexpr int kG256RowStride = 16 * 17;                 // [row][k2][n1], one pad per 16
constexpr int kG256Tile = kG256Rows + 1;                // transposed tile [256][rows + 1]
constexpr int kG256Elems = kG256Rows * kG256RowStride > 256 * kG256Tile ? kG256Rows * kG256RowStride : 256 * kG256Tile;

// One length-256 DFT along a block row held by its 16 threads: thread q holds the points
// q + 16·n2 (n2 = 0..15) in v[n2] and gets back X[q + 16·k1] in v[k1] — the same layout, so two
// row DFTs can follow each other with a point-wise step in between.
template <int DIR>
__device__ __forceinline__ void g256_row_dft(float2 (&v)[16], float2* lds, int lr, int q, const float2* tw) {
  DFT<16, DIR>::run(v);
#pragma unroll
  for (int k2 = 1; k2 < 16; ++k2) v[k2] = cmul(v[k2], twiddle<DIR>(tw, q * k2));
#pragma unroll
  for (int k2 = 0; k2 < 16; ++k2) lds[lr * kG256RowStride + k2 * 17 + q] = v[k2];
  // the exchange stays inside the wave (its 4 rows): LDS ops retired, no workgroup barrier
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xc07f);
  asm volatile("" ::: "memory");
#pragma unroll
  for (int n1 = 0; n1 < 16; ++n1) v[n1] = lds[lr * kG256RowStride + q * 17 + n1];
  DFT<16, DIR>::run(v);                       // X[row][q + 16·k1] = v[k1]
}

struct NoMid {
  __device__ __forceinline__ void operator()(int, int, float2&) const {}
};

// One N = 256 stage over the 64-row blocks of src: [pre] → row DFT (DIR1; 0 = none) → mid(y, x, v)
// → row DFT (DIR2; 0 = none) → transposed store into dst (STORE), post(y, x, v) on the way out
// (POST).  SRC_T: src holds the transposed array (its rows are columns of the natural one); pre,
// mid and post always see natural coordinates.  A 2-D FFT is two stages; between an FFT and the
// next inverse FFT of the multislice chain the point-wise step (×H, ×Oⁿ, the slice adjoint)
// runs between the two row DFTs of ONE stage (the second axis of one transform and the first
// axis of the next are the same rows), so the chain makes one round trip per transform instead
// of two (forward_far_g256 / k_adjoint).
template <int DIR1, int DIR2, bool SRC_T, bool FIRST, bool PRELOAD, bool STORE, bool POST, class Pre, class Mid,
          class Post>
__device__ __forceinline__ void g256_fstage(const float2* __restrict__ src, float2* __restrict__ dst, float2* lds,
                                            const float2* tw, Pre& pre, Mid& mid, Post& post) {
  constexpr int N = 256;
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int lr = tid >> 4, q = tid & 15;   // block row, n1 (step 1) / k2 (step 2)
  for (int r0 = 0; r0 < N; r0 += kG256Rows) {
    const int row = r0 + lr;
    float2 v[16];
#pragma unroll
    for (int n2 = 0; n2 < 16; ++n2) {
      const int j = q + 16 * n2;
      const int y = SRC_T ? j : row, x = SRC_T ? row : j;
      if constexpr (FIRST) {
        if constexpr (PRELOAD) v[n2] = call_pre(pre, y, x, src[row * N + j], n2);
        else v[n2] = call_pre(pre, y, x, make_float2(0.f, 0.f), n2);
        if constexpr (kFuseGroup > 0 && !kSlotPre<Pre>) {
          if ((n2 + 1) % kFuseGroup == 0) __builtin_amdgcn_sched_barrier(0);
        }
      } else {
        v[n2] = src[row * N + j];
      }
    }
    if constexpr (DIR1 != 0) g256_row_dft<DIR1>(v, lds, lr, q, tw);
    if constexpr (!std::is_same_v<Mid, NoMid>) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int j = q + 16 * k;
        mid(SRC_T ? j : row, SRC_T ? row : j, v[k]);
        if constexpr (kFuseGroup > 0) {
          if ((k + 1) % kFuseGroup == 0) __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    if constexpr (DIR2 != 0) g256_row_dft<DIR2>(v, lds, lr, q, tw);
    if constexpr (STORE) {
      __syncthreads();
#pragma unroll
      for (int k1 = 0; k1 < 16; ++k1) lds[(q + 16 * k1) * kG256Tile + lr] = v[k1];
      __syncthreads();
      // transposed store: dst[k][r0 + c] for k = 0..255, c < kG256Rows consecutive per line
#pragma unroll 4
      for (int i = 0; i < 16; ++i) {
        const int e = tid + kG256Threads * i, k = e / kG256Rows, c = e % kG256Rows;
        float2 val = lds[k * kG256Tile + c];
        if constexpr (POST) {
          if (call_post(post, SRC_T ? k : r0 + c, SRC_T ? r0 + c : k, val, i)) dst[k * N + r0 + c] = val;
        } else {
          dst[k * N + r0 + c] = val;
        }
      }
      __syncthreads();
    }
  }
  if constexpr (!STORE) __syncthreads();
}

template <int DIR, bool FIRST, bool LAST, bool PRELOAD, class Pre, class Post>
__device__ __forceinline__ void g256_stage(const float2* __restrict__ src, float2* __restrict__ dst, float2* lds,
                                           const float2* tw, Pre& pre, Post& post) {
  NoMid nm;
  g256_fstage<DIR, 0, LAST, FIRST, PRELOAD, true, LAST>(src, dst, lds, tw, pre, nm, post);
}

// ---------------------------------------------------------------- 128 < N ≤ 512: line blocks
// A field that does not fit LDS (and is not 256², which has its own stages above) transforms in
// TWO global round trips: stage 1 takes blocks of kLines rows through LDS (pre hook on the loads,
// both Stockham passes of the row DFT in LDS, stored to the pair's b), stage 2 blocks of kLines
// columns (128-B row segments in, both passes, post hook on the way out to a).  32 lines a block
// up to N = 256, 16 above (a 512-point line block is 70 KiB of LDS).
template <int N, int L = (N > 256 ? 16 : 32)>
struct LineTile {
  static constexpr int kLines = L;
  static constexpr int kStride = N + N / 16;                 // one pad point per 16 (LdsArray's rule)
  static constexpr int kElems = kLines * kStride;
  __device__ __forceinline__ static int off(int line, int x) { return line * kStride + x + (x >> 4); }
};

// One in-place Stockham pass of radix R (span NS) along `lines` lines of a LineTile<N, L>.
template <int N, int NT, int R, int NS, int DIR, int LINES = LineTile<N>::kLines>
__device__ __forceinline__ void line_pass(float2* tile, const float2* tw, int lines) {
  using LT = LineTile<N, LINES>;
  constexpr int L = N / R;                 // butterflies per line
  constexpr int TWS = N / (NS * R);        // twiddle table stride
  constexpr int KB = (LT::kLines * L + NT - 1) / NT;
  const int NB = lines * L;
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  float2 v[KB][R];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    const int bf = tid + kb * NT;
    if (bf < NB) {
      const int line = bf / L, j = bf % L, k = j % NS;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        float2 val = tile[LT::off(line, j + r * L)];
        if constexpr (NS > 1) {
          if (r > 0) val = cmul(val, twiddle<DIR>(tw, k * r * TWS));
        }
        v[kb][r] = val;
      }
      DFT<R, DIR>::run(v[kb]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    const int bf = tid + kb * NT;
    if (bf < NB) {
      const int line = bf / L, j = bf % L, k = j % NS;
      const int d0 = (j / NS) * NS * R + k;
#pragma unroll
      for (int r = 0; r < R; ++r) tile[LT::off(line, d0 + r * NS)] = v[kb][r];
    }
  }
  __syncthreads();
}

template <int N, int NT, int DIR, bool PRELOAD, class Pre, class Post>
__device__ __forceinline__ void fft2d_lines(const GlobalPair<N>& arr, const float2* tw, Pre& pre, Post& post) {
  using LT = LineTile<N>;
  using P1 = Plan1D<N>;
  constexpr int B = LT::kLines;
  float2* T = arr.lds;
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  for (int l0 = 0; l0 < N; l0 += B) {          // rows of a → b
    const int nl = N - l0 < B ? N - l0 : B;
    for (int e = tid; e < nl * N; e += NT) {
      const int r = e / N, x = e % N, y = l0 + r;
      float2 val;
      if constexpr (PRELOAD) val = call_pre(pre, y, x, arr.a[y * N + x], 0);
      else val = call_pre(pre, y, x, make_float2(0.f, 0.f), 0);
      T[LT::off(r, x)] = val;
    }
    __syncthreads();
    line_pass<N, NT, P1::R1, 1, DIR>(T, tw, nl);
    line_pass<N, NT, P1::R2, P1::R1, DIR>(T, tw, nl);
    for (int e = tid; e < nl * N; e += NT) {
      const int r = e / N, x = e % N;
      arr.b[(l0 + r) * N + x] = T[LT::off(r, x)];
    }
    __syncthreads();
  }
  for (int c0 = 0; c0 < N; c0 += B) {          // columns of b → a
    const int nc = N - c0 < B ? N - c0 : B;
    for (int e = tid; e < nc * N; e += NT) {
      const int y = e / nc, c = e % nc;
      T[LT::off(c, y)] = arr.b[y * N + c0 + c];
    }
    __syncthreads();
    line_pass<N, NT, P1::R1, 1, DIR>(T, tw, nc);
    line_pass<N, NT, P1::R2, P1::R1, DIR>(T, tw, nc);
    for (int e = tid; e < nc * N; e += NT) {
      const int y = e / nc, c = e % nc, x = c0 + c;
      float2 val = T[LT::off(c, y)];
      if (call_post(post, y, x, val, 0)) arr.a[y * N + x] = val;
    }
    __syncthreads();
  }
}

template <int DIR, bool PRELOAD, class Pre, class Post>
__device__ __forceinline__ void fft2d_g256(const GlobalPair<256>& arr, const float2* tw, Pre& pre, Post& post) {
  g256_stage<DIR, true, false, PRELOAD>(arr.a, arr.b, arr.lds, tw, pre, post);
  g256_stage<DIR, false, true, false>(arr.b, arr.a, arr.lds, tw, pre, post);
}

// Unnormalised 2-D DFT of the array (DIR = -1 forward, +1 inverse), rows then columns.
// Result left in the array (for GlobalPair: in .a after an even number of passes).
template <int N, int NT, int DIR, bool PRELOAD, class Arr, class Pre, class Post>
__device__ __forceinline__ void fft2d(const Arr& arr, const float2* tw, Pre&& pre, Post&& post) {
  using P1 = Plan1D<N>;
  constexpr int R1 = P1::R1, R2 = P1::R2;
  if constexpr (Arr::kInPlace) {
    if constexpr (R2 == 1) {
      stockham_pass<N, NT, R1, 1, true, DIR, kFirst, PRELOAD, true>(arr, arr, tw, pre, post);
      stockham_pass<N, NT, R1, 1, false, DIR, kLast, false, true>(arr, arr, tw, pre, post);
    } else {
      stockham_pass<N, NT, R1, 1, true, DIR, kFirst, PRELOAD, true>(arr, arr, tw, pre, post);
      stockham_pass<N, NT, R2, R1, true, DIR, kMid, false, true>(arr, arr, tw, pre, post);
      stockham_pass<N, NT, R1, 1, false, DIR, kMid, false, true>(arr, arr, tw, pre, post);
      stockham_pass<N, NT, R2, R1, false, DIR, kLast, false, true>(arr, arr, tw, pre, post);
    }
  } else {
    static_assert(R2 != 1, "global ping-pong needs two passes per dimension");
    if constexpr (N == 256 && NT == kG256Threads) {
      fft2d_g256<DIR, PRELOAD>(arr, tw, pre, post);
    } else {
      fft2d_lines<N, NT, DIR, PRELOAD>(arr, tw, pre, post);
    }
  }
}


// LDS (float2) a general-engine kernel declares for its N×N transforms: the whole field (N ≤ 128),
// N = 256's stage tile, or the line-block tile (128 < N < 256)
template <int N, bool LDS>
constexpr int kFieldLds = LDS ? LdsArray<N>::kElems : N == 256 ? kG256Elems : LineTile<N>::kElems;

}  // namespace ptyx
