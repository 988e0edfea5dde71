// dilqr_launch.h — launchers that live in one translation unit and are called
// from the C-ABI entry points of another (the per-model fused-iteration and
// implicit-backward instantiations compile in their own units, see Makefile).
// Host-side only; every launcher returns the C-ABI status (0 or -hipError).
#pragma once
#include <hip/hip_runtime.h>

#include "dilqr_device.h"

namespace dilqr {

// One fused MPC iteration launch (dilqr_mpc_step_f32 / _iterate_fixed_f32).
struct MpcStepArgs {
  int T, B;
  const float *theta, *x_init, *C, *c;
  Bounds bd;
  float decay;
  int max_ls, iteration;
  float best_cost_eps, eps;
  int lim, G;                   // G < 0: fixed-count solve (no stop-rule prologue)
  dilqr_mpc_state st;
  hipStream_t stream;
};

// A whole fixed-count solve in one launch (dilqr_mpc_solve_fixed_f32; the
// thread-per-problem models).
struct MpcSolveArgs {
  int T, B;
  const float *theta, *x_init, *u_init, *C, *c;
  Bounds bd;
  float decay;
  int max_ls, iters;
  float best_cost_eps;
  dilqr_mpc_state st;
  hipStream_t stream;
};

// One standalone fused iteration (dilqr_ilqr_iterate_f32).
struct IlqrIterArgs {
  int T, B;
  const float *theta, *x_init, *C, *c, *x, *u;
  Bounds bd;
  float decay;
  int max_ls;
  float *ws, *x_out, *u_out, *cost, *du_sq, *alpha;
  const dilqr_mpc_ctrl* ctrl;
  hipStream_t stream;
};

int launch_mpc_step_pendulum(const MpcStepArgs& a);
int launch_mpc_step_cartpole(const MpcStepArgs& a);
int launch_mpc_step_rocket(const MpcStepArgs& a);
int launch_mpc_step_pendulum_complex(const MpcStepArgs& a);
int launch_mpc_solve_pendulum(const MpcSolveArgs& a);
int launch_mpc_solve_cartpole(const MpcSolveArgs& a);
int launch_mpc_solve_pendulum_complex(const MpcSolveArgs& a);
int launch_mpc_solve_small_pendulum(const MpcSolveArgs& a, float eps, int lim);
int launch_mpc_solve_small_cartpole(const MpcSolveArgs& a, float eps, int lim);
int launch_mpc_solve_small_pendulum_complex(const MpcSolveArgs& a, float eps, int lim);
int launch_ilqr_iterate_pendulum(const IlqrIterArgs& a);
int launch_ilqr_iterate_cartpole(const IlqrIterArgs& a);
int launch_ilqr_iterate_rocket(const IlqrIterArgs& a);
int launch_ilqr_iterate_pendulum_complex(const IlqrIterArgs& a);

// rocket implicit backward (dilqr_implicit_group.h)
struct ImplicitArgs {
  int T, B;
  const float *theta, *C, *c, *x, *u, *K, *dl_dx, *dl_du;
  Bounds bd;
  float *ws, *dC, *dc, *dtheta;
  hipStream_t stream;
};
int launch_implicit_rocket(const ImplicitArgs& a);
int implicit_rocket_ws_floats();

}  // namespace dilqr
