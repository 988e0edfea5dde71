// tu_mpc_cartpole.hip — the fused iteration kernels instantiated for cartpole
// (env_dx/cartpole.py, n=5 m=1): the headline kernel k_mpc_iterate<Cartpole,...>.
#include "dilqr_fused.h"

namespace dilqr {
int launch_mpc_step_cartpole(const MpcStepArgs& a) { return launch_mpc_step_tpp<Cartpole>(a); }
int launch_ilqr_iterate_cartpole(const IlqrIterArgs& a) { return launch_ilqr_iterate_tpp<Cartpole>(a); }
int launch_mpc_solve_cartpole(const MpcSolveArgs& a) { return launch_mpc_solve_tpp<Cartpole>(a); }
int launch_mpc_solve_small_cartpole(const MpcSolveArgs& a, float eps, int lim) {
  return launch_mpc_solve_small_tpp<Cartpole>(a, eps, lim);
}
}  // namespace dilqr

#ifdef DILQR_STAMPS
// diagnostic build only: copy the phase stamps of the last fused MPC iteration
// (the stamps of this unit's kernels: cartpole, the model the tools stamp)
extern "C" int dilqr_debug_stamps(unsigned long long* host, int n) {
  using namespace dilqr;
  if (n > kStampWaves * kStampSlots) n = kStampWaves * kStampSlots;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0 : -1;
}
#endif
