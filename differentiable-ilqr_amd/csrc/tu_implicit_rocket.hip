// tu_implicit_rocket.hip — the DiLQR implicit backward for rocket
// (16 lanes per problem, dilqr_implicit_group.h; rocket.py:263-323, 541-820).
#include "dilqr_common.h"
#include "dilqr_implicit_group.h"
#include "dilqr_launch.h"

namespace dilqr {

int implicit_rocket_ws_floats() { return ImplicitGroupWs<Rocket>::REC; }

// DILQR_IMPL_SPLIT (default 0): passes B, C and D as three launches (each at
// 3 waves per SIMD, dilqr_implicit_group.h PASSES) instead of one launch at 2.
// Measured at config 3 (B = 32 768, T = 30): one launch 1.353-1.364 ms; three
// at 3 waves 1.655-1.741 (pass D then spills); pass D at 2 waves 1.362-1.408 —
// the extra waves of passes B and C buy nothing, the kernel is bound by its
// per-step dependent chain, not by latency hiding across problems
// (profiles/r06/ab_implicit_rocket_pass_launches.txt).  Bit-identical either way.
#ifndef DILQR_IMPL_SPLIT
#define DILQR_IMPL_SPLIT 0
#endif
int launch_implicit_rocket(const ImplicitArgs& a) {
#define IMPL_LAUNCH(MODE_, PASSES_)                                                                         \
  k_implicit_backward_group<Rocket, gen::RocketD2, MODE_, PASSES_><<<grid_group(a.B), 64, 0, a.stream>>>(  \
      a.T, a.B, a.theta, a.C, a.c, a.x, a.u, a.K, a.dl_dx, a.dl_du, a.bd, a.ws, a.dC, a.dc, a.dtheta)
#define IMPL_ALL(MODE_)                                                                                     \
  do {                                                                                                      \
    if (DILQR_IMPL_SPLIT) {                                                                                 \
      IMPL_LAUNCH(MODE_, 1);                                                                                \
      IMPL_LAUNCH(MODE_, 2);                                                                                \
      IMPL_LAUNCH(MODE_, 4);                                                                                \
    } else {                                                                                                \
      IMPL_LAUNCH(MODE_, 7);                                                                                \
    }                                                                                                       \
  } while (0)
  if (a.bd.mode == DILQR_BOUNDS_NONE) IMPL_ALL(GAIN_UNC);
  else IMPL_ALL(GAIN_ZERO_I);
#undef IMPL_ALL
#undef IMPL_LAUNCH
  return launched();
}

}  // namespace dilqr
