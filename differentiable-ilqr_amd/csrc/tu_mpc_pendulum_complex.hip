// tu_mpc_pendulum_complex.hip — the fused iteration kernels instantiated for the
// 5-parameter pendulum (env_dx/pendulum.py simple=False, n=3 m=1).
#include "dilqr_fused.h"

namespace dilqr {
int launch_mpc_step_pendulum_complex(const MpcStepArgs& a) { return launch_mpc_step_tpp<PendulumComplex>(a); }
int launch_ilqr_iterate_pendulum_complex(const IlqrIterArgs& a) { return launch_ilqr_iterate_tpp<PendulumComplex>(a); }
int launch_mpc_solve_pendulum_complex(const MpcSolveArgs& a) { return launch_mpc_solve_tpp<PendulumComplex>(a); }
int launch_mpc_solve_small_pendulum_complex(const MpcSolveArgs& a, float eps, int lim) {
  return launch_mpc_solve_small_tpp<PendulumComplex>(a, eps, lim);
}
}  // namespace dilqr
