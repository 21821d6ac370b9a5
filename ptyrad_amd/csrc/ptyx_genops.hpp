// ptyx_genops.hpp — the general engine's per-N launch table.
//
// The general engine's kernels are instantiated once per supported N in the ptyx_gen.hip
// translation units (ptyx_general.hpp's GenLaunch<N>), which register one GenOps each at load
// time; ptyx_kernels.hip (plans, engine selection, the C ABI) looks the table up by N and never
// instantiates those kernels itself.  Supported N = the sizes registered: every 2·3·5·7-smooth N
// in [32, 512] (src/ptyrad/params/init_params.py:53, 340, 361: meas_crop / meas_resample /
// meas_pad produce them; the reference transforms them with torch's mixed-radix FFT).
#pragma once
#include <hip/hip_runtime.h>

namespace ptyx {

struct KArgs;

struct GenOps {
  int N, nt;
  bool lds;            // the N×N wave in LDS (N ≤ 128), else in the per-workgroup scratch pair
  int blocks_per_cu;   // LDS / thread-limited residency of the FFT kernels
  void (*spectrum)(const KArgs& a, int nblk, float2* Fp, hipStream_t st);
  // one_mode: P·O = 1;  single: P·O·Nz = 1
  void (*forward)(const KArgs& a, int grid, bool one_mode, bool single, hipStream_t st);
  void (*modesum)(const KArgs& a, hipStream_t st);
  void (*adjoint)(const KArgs& a, int grid, bool one_mode, bool single, bool ext, hipStream_t st);
  void (*probe_finalize)(const KArgs& a, int nblk, const float2* G, float2* d_probe, hipStream_t st);
  // two-launch row / column forms (N/8 workgroups a mode each; tmp: P·N² float2 of scratch):
  // F(P) → Fp (+ the N = 128 K-packed fpk), and d_probe += F⁻¹(G)/N² (no probe shift: not used)
  void (*spectrum_lines)(const float2* probe, int P, float2* Fp, float2* fpk, float2* tmp, const float2* twg,
                         hipStream_t st);
  void (*probe_finalize_lines)(const float2* G, int P, float2* d_probe, float2* tmp, const float2* twg,
                               hipStream_t st);
  // the column launch of spectrum_lines alone (its row pass ran inside another launch: the
  // register engines' k_small_prep)
  void (*spectrum_cols)(const float2* tmp, int P, float2* Fp, float2* fpk, const float2* twg, hipStream_t st);
};

// registry (ptyx_kernels.hip): gen_register is called from the size groups' static initialisers
void gen_register(const GenOps* ops);
const GenOps* gen_ops(int N);

}  // namespace ptyx
