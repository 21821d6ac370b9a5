// ptyx_gen.hip — one size group of the general engine: GenLaunch<N> for every N in
// PTYX_GEN_SIZES (set by the build, e.g. -DPTYX_GEN_SIZES=96,160), registered with the launch
// table of ptyx_genops.hpp when libptyx.so loads.  The build compiles this file once per group,
// in parallel (ptyrad_amd/csrc/build.py GEN_GROUPS).
#include "ptyx_general.hpp"

#ifndef PTYX_GEN_SIZES
#error "PTYX_GEN_SIZES (the N of this size group) is set by build.py"
#endif

namespace ptyx {
namespace {
template <int... Ns>
struct GenGroup {
  GenGroup() { (gen_register(GenLaunch<Ns>::ops()), ...); }
};
const GenGroup<PTYX_GEN_SIZES> kGroup;
}  // namespace
}  // namespace ptyx
