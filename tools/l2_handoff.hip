// l2_handoff.hip — can a stripe-pass intermediate be handed from producer to consumer through one
// XCD's L2 instead of HBM?  (DESIGN §4c "Per-XCD L2 residency".)
//
// Models the k_s1 → k_s2 dependency of the N = 256 stripe engine (ptyx_stripe.hpp): per task
// (= one pattern) 16 producer items each write one column-stripe chunk of W/16 bytes (k_s1: P
// fields × 16 columns × 256 rows × 8 B), and 16 consumer items each read 1/16 of EVERY producer's
// chunk (k_s2: a row stripe needs all 16 column stripes).  W = P × 512 KiB: 2 MiB at c5 (P = 4),
// 4 MiB at c3 (P = 8, T1), 8 MiB for c3's T2 (P·O = 16).
//
//   fused<SHIFT>: one persistent launch; each workgroup reads its XCD (HW_REG_XCC_ID) and dequeues
//     items from that XCD's queue.  Queue x holds, in task order, the producers of tasks t ≡ x and
//     the consumers of tasks t ≡ x − SHIFT (mod 8): SHIFT 0 = consumer on the producer's XCD (its
//     L2 holds the chunk if it has not been evicted), SHIFT 1 = always another XCD.  Hand-off per
//     MI355X_MICROARCH.md §Workgroup dispatch: plain stores → vmcnt(0) → barrier → lane-0 agent
//     release → vmcnt(0) → relaxed agent flag add; consumer: relaxed poll → agent acquire →
//     vmcnt(0) → barrier → plain loads.  Producers never wait and every queue is dequeued in task
//     order, so every consumer's producers are dequeued before it (no deadlock, any residency).
//   two-kernel: all producers, kernel boundary, all consumers (the engine today).
//
// Every consumer checks every word it reads.  Output: one JSON line per (W, variant) with GB/s of
// payload moved (written + read) and the consumer-read rate; run under rocprofv3 --pmc
// (FETCH_SIZE; WRITE_SIZE + TCC_HIT_sum + TCC_MISS_sum) with --once for per-dispatch counters.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/l2_handoff tools/l2_handoff.hip
//   tools/l2_handoff [--once]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

constexpr int kNT = 256;       // threads per workgroup (the stripe passes' shape)
constexpr int kParts = 16;     // producers and consumers per task (stripes)

struct Args {
  float4* pay;      // T × W bytes
  int* flag;        // T producer arrival counters
  int* head;        // 8 per-XCD queue heads (fused) / 1 grid-stride head unused
  int* bad;         // words that failed the check
  float* out;       // T × 16 consumer checksums
  long long W;      // bytes per task
  int T;            // tasks (multiple of 8)
};

__device__ __forceinline__ int xcc_id() {
  // HW_REG_XCC_ID: hwreg 20, bits [3:0]
  return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)) & 7;
}

__device__ __forceinline__ float4 word(int t, int p, long long i) {
  return make_float4((float)t, (float)p, (float)(i & 0xffff), 1.f);
}

__device__ __forceinline__ void produce(const Args& a, int t, int p) {
  const long long C = a.W / kParts / 16;   // float4 per chunk
  float4* dst = a.pay + ((long long)t * kParts + p) * C;
  for (long long i = threadIdx.x; i < C; i += kNT) dst[i] = word(t, p, i);
}

__device__ __forceinline__ void consume(const Args& a, int t, int c) {
  const long long C = a.W / kParts / 16, S = C / kParts;   // float4 per chunk / per sub-chunk
  float acc = 0.f;
  int bad = 0;
  for (int p = 0; p < kParts; ++p) {
    const float4* src = a.pay + ((long long)t * kParts + p) * C + (long long)c * S;
    for (long long i = threadIdx.x; i < S; i += kNT) {
      const float4 v = src[i];
      const float4 w = word(t, p, (long long)c * S + i);
      bad += (v.x != w.x) | (v.y != w.y) | (v.z != w.z) | (v.w != w.w);
      acc += v.w;
    }
  }
  if (bad) atomicAdd(a.bad, bad);
  if (threadIdx.x == 0) a.out[t * kParts + c] = acc;
}

template <int SHIFT>
__global__ __launch_bounds__(kNT, 2) void k_fused(Args a) {
  __shared__ int s_q;
  const int x = xcc_id();
  const int per_queue = (a.T / 8) * 2 * kParts;
  for (;;) {
    if (threadIdx.x == 0) s_q = atomicAdd(a.head + x, 1);
    __syncthreads();
    const int q = s_q;
    __syncthreads();
    if (q >= per_queue) break;
    const int k = q / (2 * kParts), r = q % (2 * kParts);
    if (r < kParts) {
      const int t = 8 * k + x;
      produce(a, t, r);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(a.flag + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {
      const int t = 8 * k + ((x - SHIFT) & 7);
      if (threadIdx.x == 0) {
        while (__hip_atomic_load(a.flag + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < kParts)
          __builtin_amdgcn_s_sleep(2);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      consume(a, t, r - kParts);
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(kNT, 2) void k_produce_all(Args a) {
  for (int it = blockIdx.x; it < a.T * kParts; it += gridDim.x) produce(a, it / kParts, it % kParts);
}
__global__ __launch_bounds__(kNT, 2) void k_consume_all(Args a) {
  for (int it = blockIdx.x; it < a.T * kParts; it += gridDim.x) consume(a, it / kParts, it % kParts);
}

int main(int argc, char** argv) {
  const bool once = argc > 1 && std::strcmp(argv[1], "--once") == 0;
  int dev = 0, cu = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev));
  const int grid = 2 * cu;   // two 256-thread workgroups per CU, as the stripe passes
  const long long total = 2LL << 30;   // payload bytes per run
  const long long Ws[] = {256LL << 10, 512LL << 10, 1LL << 20, 2LL << 20, 4LL << 20, 8LL << 20};
  Args a{};
  CHECK(hipMalloc(&a.pay, total));
  const int Tmax = (int)(total / Ws[0]);
  CHECK(hipMalloc(&a.flag, sizeof(int) * Tmax));
  CHECK(hipMalloc(&a.head, sizeof(int) * 8));
  CHECK(hipMalloc(&a.bad, sizeof(int)));
  CHECK(hipMalloc(&a.out, sizeof(float) * Tmax * kParts));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int reps = once ? 1 : 5;
  for (long long W : Ws) {
    a.W = W;
    a.T = (int)(total / W) / 8 * 8;
    for (int v = 0; v < 3; ++v) {   // 0 fused same-XCD, 1 fused cross-XCD, 2 two kernels
      float best = 1e30f;
      int bad_total = 0;
      for (int r = 0; r < reps + (once ? 0 : 1); ++r) {
        CHECK(hipMemset(a.flag, 0, sizeof(int) * a.T));
        CHECK(hipMemset(a.head, 0, sizeof(int) * 8));
        CHECK(hipMemset(a.bad, 0, sizeof(int)));
        CHECK(hipMemset(a.pay, 0, total));
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0, 0));
        if (v == 0) hipLaunchKernelGGL(k_fused<0>, dim3(grid), dim3(kNT), 0, 0, a);
        else if (v == 1) hipLaunchKernelGGL(k_fused<1>, dim3(grid), dim3(kNT), 0, 0, a);
        else {
          hipLaunchKernelGGL(k_produce_all, dim3(grid), dim3(kNT), 0, 0, a);
          hipLaunchKernelGGL(k_consume_all, dim3(grid), dim3(kNT), 0, 0, a);
        }
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        int bad = 0;
        CHECK(hipMemcpy(&bad, a.bad, sizeof(int), hipMemcpyDeviceToHost));
        bad_total += bad;
        if (r > 0 || once) best = ms < best ? ms : best;
      }
      const double bytes = 2.0 * (double)a.T * (double)W;
      std::printf("{\"W_bytes\": %lld, \"tasks\": %d, \"variant\": \"%s\", \"ms\": %.3f, \"GBps_moved\": %.1f, "
                  "\"bad_words\": %d, \"grid\": %d}\n",
                  W, a.T, v == 0 ? "fused_same_xcd" : v == 1 ? "fused_cross_xcd" : "two_kernels", best,
                  bytes / (best * 1e6), bad_total, grid);
      std::fflush(stdout);
    }
  }
  return 0;
}
