// tu_mpc_pendulum.hip — the fused iteration kernels instantiated for the
// pendulum (env_dx/pendulum.py, n=3 m=1).
#include "dilqr_fused.h"

namespace dilqr {
int launch_mpc_step_pendulum(const MpcStepArgs& a) { return launch_mpc_step_tpp<Pendulum>(a); }
int launch_ilqr_iterate_pendulum(const IlqrIterArgs& a) { return launch_ilqr_iterate_tpp<Pendulum>(a); }
int launch_mpc_solve_pendulum(const MpcSolveArgs& a) { return launch_mpc_solve_tpp<Pendulum>(a); }
int launch_mpc_solve_small_pendulum(const MpcSolveArgs& a, float eps, int lim) {
  return launch_mpc_solve_small_tpp<Pendulum>(a, eps, lim);
}
}  // namespace dilqr
