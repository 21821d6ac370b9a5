// ptyx_stepfuse.hpp — the optimizer step fused into a small call's epilogue (PTYX_PREP_FUSED_ADAM,
// include/ptyx.h).  Included by ptyx_kernels.hip inside namespace ptyx, after ptyx_gather.hpp.
//
// At the reference's default cadence (grad_accumulation = 1, reconstruction.py:741-760) every
// 32-pattern mini-batch ends with loss.backward() and optimizer.step().  ptyx's k_fused3 path ends
// a call with the object gather (k_obj_gather: 1,105 tiles at c2 that write the whole 8.5 MB object
// gradient), the probe gradient's row IFFT (k_probe_rows_acc), and then the HIP Adam launch reads
// every gradient back with p, m, v.  k_gather_adam does all three in ONE launch:
//   blocks [0, tiles)                    one object tile each: the gather's sums, then per pixel
//                                        the gradient (stored, as the gather does) and the Adam
//                                        step of obja and objp on it — the gradient, the object
//                                        and its moments are each touched once;
//   blocks [tiles, tiles + N/kPrLinesT)  the probe gradient's rows (k_probe_rows_acc), then the
//                                        Adam step of those probe elements;
//   the rest                             k_adam's chunks over every other tensor (positions ...),
//                                        whose gradients are complete before the launch.
// (Role order; with f.lead the probe-row and rest blocks take the first block indices.)
// Same arithmetic as the unfused path (gather_apply's expressions, ptyx_adam.hpp's element update),
// so the trajectory is bitwise the gather + rows + k_adam one (tests/test_gpu_stepgraph.py).

struct FusedAdamArgs {
  GatherArgs ga;           // the object gather of the call
  opt::AdamHyper h;
  int tiles;               // object tile blocks: ptiles tiles of each of the nz object planes
  int ptiles;
  float* op[2];            // obja (0) / objp (1) as Adam parameters (= ga.obja / ga.objp) with their
  float* om[2];            // state; om[i] null: that plane takes no step here
  float* ov[2];
  const float* ostep[2];
  double olr[2];
  int pblocks;             // probe-row blocks (N / kPrLinesT a probe mode), 0: no probe gradient
  const float2* ptmp;      // the probe gradient's column-transformed spectrum (k_small_tail)
  float2* d_probe;
  const float2* twg;
  float* pp;               // Adam state of the probe (as floats); null: no step here
  float* pm;
  float* pv;
  const float* pstep;
  double plr;
  opt::AdamArgs rest;      // every other tensor (and the step bookkeeping in rest.scnt)
  int rblocks;
  int lead;                // 1: the probe-row and rest blocks take the launch's first block indices
                           // (dispatched first: their chains overlap the tile rounds instead of
                           // trailing them); 0: tiles first
};

// One object tile: the gather's sums, then gradient + Adam per pixel (thread e, e + 256, ...).
template <int N, bool ROWPERM>
__device__ __forceinline__ void gather_adam_tile(const FusedAdamArgs& f, int b) {
  __shared__ float2 s_acc[kGTY * kGTX];
  __shared__ float s_cnt[kGTY * kGTX];
  __shared__ float s_ns[2], s_bc[2];
  const GatherArgs ga = f.ga;   // (a copy: a reference into the kernel argument put the whole struct in scratch)
  const int tyi = b / ga.tiles_x, txi = b % ga.tiles_x;
  const int ty = tyi * kGTY, tx = txi * kGTX;
  constexpr int PX = kGTY * kGTX / 256;   // pixels a thread
  if (threadIdx.x == 0 && f.om[0]) opt::adam_step_scalars(f.h, f.olr[0], *f.ostep[0], &s_ns[0], &s_bc[0]);
  if (threadIdx.x == 64 && f.om[1]) opt::adam_step_scalars(f.h, f.olr[1], *f.ostep[1], &s_ns[1], &s_bc[1]);
  // the epilogue's operands, loaded before the candidate scan (only this workgroup touches them)
  float A[PX], ph[PX], ma[PX], va[PX], mp[PX], vp[PX], ga0[PX], gp0[PX];
#pragma unroll
  for (int k = 0; k < PX; ++k) {
    const int e = threadIdx.x + 256 * k;
    const int y = ty + e / kGTX, x = tx + e % kGTX;
    A[k] = ph[k] = ma[k] = va[k] = mp[k] = vp[k] = ga0[k] = gp0[k] = 0.f;
    if (y < ga.Ny && x < ga.Nx) {
      const size_t off = (size_t)y * ga.Nx + x;
      A[k] = ga.obja[off];
      ph[k] = ga.objp[off];
      if (f.om[0]) {
        ma[k] = f.om[0][off];
        va[k] = f.ov[0][off];
      }
      if (f.om[1]) {
        mp[k] = f.om[1][off];
        vp[k] = f.ov[1][off];
      }
      if (!ga.store) {
        if (ga.d_obja) ga0[k] = ga.d_obja[off];
        if (ga.d_objp) gp0[k] = ga.d_objp[off];
      }
    }
  }
  const bool skip = ga.bbox && (ty + kGTY <= ga.bbox[0] || ty >= ga.bbox[1] + N || tx + kGTX <= ga.bbox[2] ||
                                tx >= ga.bbox[3] + N);
  if (!skip) {
    gather_tile_sums<N, ROWPERM, 4, false, false>(ga, tyi, txi, 0, s_acc, s_cnt);
  } else {
    __syncthreads();   // (the step scalars)
  }
  const float dec0 = (float)(1.0 - f.olr[0] * (double)f.h.wd), dec1 = (float)(1.0 - f.olr[1] * (double)f.h.wd);
#pragma unroll
  for (int k = 0; k < PX; ++k) {
    const int e = threadIdx.x + 256 * k;
    const int y = ty + e / kGTX, x = tx + e % kGTX;
    if (y >= ga.Ny || x >= ga.Nx) continue;
    const size_t off = (size_t)y * ga.Nx + x;
    // gather_apply's expressions
    const float2 S = skip ? make_float2(0.f, 0.f) : s_acc[e];
    const float C = skip ? 0.f : s_cnt[e];
    float sn, cs;
    phase_sincos(ph[k], &sn, &cs);
    if (ga.d_obja) {
      // (a skipped tile: zeros in store mode, else the gradient as it was — k_obj_gather's early exit)
      const float g = skip ? (ga.store ? 0.f : ga0[k]) : ga0[k] + fmaf(S.x, cs, S.y * sn);
      ga.d_obja[off] = g;
      if (f.om[0]) {
        float p = A[k];
        opt::adam_elem(f.h, s_ns[0], s_bc[0], dec0, g, p, ma[k], va[k]);
        f.op[0][off] = p;
        f.om[0][off] = ma[k];
        f.ov[0][off] = va[k];
      }
    }
    if (ga.d_objp) {
      float g;
      if (skip) {
        g = ga.store ? 0.f : gp0[k];
      } else {
        float dph = A[k] * fmaf(S.y, cs, -S.x * sn);
        if (C != 0.f) {
          const float sg = ph[k] > 0.f ? 1.f : (ph[k] < 0.f ? -1.f : 0.f);
          dph += ga.sparse_n == 1 ? C * sg : C * powq(fabsf(ph[k]), (float)(ga.sparse_n - 1)) * sg;
        }
        g = gp0[k] + dph;
      }
      ga.d_objp[off] = g;
      if (f.om[1]) {
        float p = ph[k];
        opt::adam_elem(f.h, s_ns[1], s_bc[1], dec1, g, p, mp[k], vp[k]);
        f.op[1][off] = p;
        f.om[1][off] = mp[k];
        f.ov[1][off] = vp[k];
      }
    }
  }
}

// The same for the mixed-state engine's row-split gather (k_obj_gather_rows, 4 waves, the probe
// modes' slot planes summed): tile b % ptiles of object plane (slice) b / ptiles.
template <int N, bool ROWPERM, bool MP, int HU>
__device__ __forceinline__ void gather_rows_adam_tile(const FusedAdamArgs& f, int b) {
  constexpr int GW = 4, RW = kGTY / GW;
  __shared__ float s_ns[2], s_bc[2];
  const GatherArgs ga = f.ga;   // (a copy, as gather_adam_tile)
  const int tile = b % f.ptiles, z = b / f.ptiles;
  const int tyi = tile / ga.tiles_x, txi = tile % ga.tiles_x;
  const int ty = tyi * kGTY, tx = txi * kGTX;
  const size_t zoff = (size_t)z * ga.Ny * ga.Nx;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int x = tx + lane, r0 = ty + wave * RW;
  if (threadIdx.x == 0 && f.om[0]) opt::adam_step_scalars(f.h, f.olr[0], *f.ostep[0], &s_ns[0], &s_bc[0]);
  if (threadIdx.x == 64 && f.om[1]) opt::adam_step_scalars(f.h, f.olr[1], *f.ostep[1], &s_ns[1], &s_bc[1]);
  float pa[RW], pp[RW], pga[RW], pgp[RW], ma[RW], va[RW], mp[RW], vp[RW];
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    pa[r] = pp[r] = pga[r] = pgp[r] = ma[r] = va[r] = mp[r] = vp[r] = 0.f;
    if (r0 + r < ga.Ny && x < ga.Nx) {
      const size_t off = zoff + (size_t)(r0 + r) * ga.Nx + x;
      pa[r] = ga.obja[off];
      pp[r] = ga.objp[off];
      if (ga.d_obja && !ga.store) pga[r] = ga.d_obja[off];
      if (ga.d_objp && !ga.store) pgp[r] = ga.d_objp[off];
      if (f.om[0]) {
        ma[r] = f.om[0][off];
        va[r] = f.ov[0][off];
      }
      if (f.om[1]) {
        mp[r] = f.om[1][off];
        vp[r] = f.ov[1][off];
      }
    }
  }
  const bool skip = ga.bbox && (ty + kGTY <= ga.bbox[0] || ty >= ga.bbox[1] + N || tx + kGTX <= ga.bbox[2] ||
                                tx >= ga.bbox[3] + N);
  float2 acc[RW];
  float cnt[RW];
  if (!skip) {
    gather_rows_sums<N, ROWPERM, GW, MP, HU>(ga, tyi, txi, z, acc, cnt);
  } else {
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      acc[r] = make_float2(0.f, 0.f);
      cnt[r] = 0.f;
    }
  }
  __syncthreads();   // (the step scalars)
  const float dec0 = (float)(1.0 - f.olr[0] * (double)f.h.wd), dec1 = (float)(1.0 - f.olr[1] * (double)f.h.wd);
#pragma unroll
  for (int r = 0; r < RW; ++r) {   // k_obj_gather_rows' epilogue, then the Adam step on its gradient
    const int y = r0 + r;
    if (y >= ga.Ny || x >= ga.Nx) continue;
    const size_t off = zoff + (size_t)y * ga.Nx + x;
    float sn, cs;
    phase_sincos(pp[r], &sn, &cs);
    if (ga.d_obja) {
      const float g = skip ? (ga.store ? 0.f : pga[r]) : pga[r] + fmaf(acc[r].x, cs, acc[r].y * sn);
      ga.d_obja[off] = g;
      if (f.om[0]) {
        float p = pa[r];
        opt::adam_elem(f.h, s_ns[0], s_bc[0], dec0, g, p, ma[r], va[r]);
        f.op[0][off] = p;
        f.om[0][off] = ma[r];
        f.ov[0][off] = va[r];
      }
    }
    if (ga.d_objp) {
      float g;
      if (skip) {
        g = ga.store ? 0.f : pgp[r];
      } else {
        float dph = pa[r] * fmaf(acc[r].y, cs, -acc[r].x * sn);
        if (cnt[r] != 0.f) {
          const float ph = pp[r];
          const float sg = ph > 0.f ? 1.f : (ph < 0.f ? -1.f : 0.f);
          dph += ga.sparse_n == 1 ? cnt[r] * sg : cnt[r] * powq(fabsf(ph), (float)(ga.sparse_n - 1)) * sg;
        }
        g = pgp[r] + dph;
      }
      ga.d_objp[off] = g;
      if (f.om[1]) {
        float p = pp[r];
        opt::adam_elem(f.h, s_ns[1], s_bc[1], dec1, g, p, mp[r], vp[r]);
        f.op[1][off] = p;
        f.om[1][off] = mp[r];
        f.ov[1][off] = vp[r];
      }
    }
  }
}

// ROWS: the tile blocks are gather_rows_adam_tile's (mixed-state engine; HU hits in flight a wave;
// MP false: one slot plane a hit, the single-state engine's row-split gather), else gather_adam_tile's.
template <int N, bool ROWPERM, bool ROWS, int HU, bool MP>
__device__ __forceinline__ void gather_adam_body(const FusedAdamArgs& f) {
  int b = blockIdx.x;   // the block's role index: tiles, then probe rows, then rest
  if (f.lead) {
    const int nl = f.pblocks + f.rblocks;
    b = b < nl ? f.tiles + b : b - nl;
  }
  if (blockIdx.x == 0 && f.rest.scnt) {   // as k_step_store: every thread reads *scnt before it advances
    const int64_t c = *f.rest.scnt;
    const int64_t r0 = f.rest.srstart[c];
    for (int i = threadIdx.x; i < f.rest.snb * 5; i += blockDim.x) f.rest.sterms_all[r0 * 5 + i] = f.rest.sterms[i];
    __syncthreads();
    if (threadIdx.x == 0) *f.rest.scnt = c + 1;
  }
  if (b < f.tiles) {
    if constexpr (ROWS) gather_rows_adam_tile<N, ROWPERM, MP, HU>(f, b);
    else gather_adam_tile<N, ROWPERM>(f, b);
    return;
  }
  if (b < f.tiles + f.pblocks) {
    __shared__ float s_pns, s_pbc;
    if (threadIdx.x == 0 && f.pp) opt::adam_step_scalars(f.h, f.plr, *f.pstep, &s_pns, &s_pbc);
    __syncthreads();
    const float ns = s_pns, bc = s_pbc;
    const float dec = (float)(1.0 - f.plr * (double)f.h.wd);
    float* pp = f.pp;
    float* pm = f.pm;
    float* pv = f.pv;
    const opt::AdamHyper h = f.h;
    constexpr int kRowBlocks = N / f3::kPrLinesT;   // a probe mode's
    const int pb = b - f.tiles;
    f3::probe_rows_block(f.ptmp, f.d_probe, f.twg, (pb % kRowBlocks) * f3::kPrLinesT, pb / kRowBlocks,
                         [&](float2* dp, size_t el, float2 g) {
                           *dp = g;
                           if (!pp) return;
                           float2 p = reinterpret_cast<float2*>(pp)[el];
                           float2 m = reinterpret_cast<float2*>(pm)[el];
                           float2 v = reinterpret_cast<float2*>(pv)[el];
                           opt::adam_elem(h, ns, bc, dec, g.x, p.x, m.x, v.x);
                           opt::adam_elem(h, ns, bc, dec, g.y, p.y, m.y, v.y);
                           reinterpret_cast<float2*>(pp)[el] = p;
                           reinterpret_cast<float2*>(pm)[el] = m;
                           reinterpret_cast<float2*>(pv)[el] = v;
                         });
    return;
  }
  __shared__ float s_nstep[opt::kMaxT], s_bc2s[opt::kMaxT];
  if (threadIdx.x < (unsigned)f.rest.nt)
    opt::adam_step_scalars(f.h, f.rest.lr[threadIdx.x], *f.rest.step[threadIdx.x], &s_nstep[threadIdx.x],
                           &s_bc2s[threadIdx.x]);
  __syncthreads();
  opt::adam_chunks(f.rest, s_nstep, s_bc2s, b - f.tiles - f.pblocks, f.rblocks);
}
template <int N, bool ROWPERM, bool ROWS = false, int HU = 1, bool MP = true>
__global__ __launch_bounds__(256) void k_gather_adam(FusedAdamArgs f) {
  gather_adam_body<N, ROWPERM, ROWS, HU, MP>(f);
}
// The one-plane row form held to 128 VGPRs: four workgroups a CU instead of three (tuning
// gather_rows 2; 131 VGPRs unconstrained)
template <int N>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_gather_adam_r4(FusedAdamArgs f) {
  gather_adam_body<N, true, true, 1, false>(f);
}
// ... and to 96 VGPRs: five workgroups a CU, every tile of a c2 call in one round (gather_rows 3)
template <int N>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void k_gather_adam_r5(FusedAdamArgs f) {
  gather_adam_body<N, true, true, 1, false>(f);
}
