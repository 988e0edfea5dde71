/*
 * dilqr.h — C-ABI of the MI355X-native batched differentiable-iLQR hot path.
 *
 * The reference (josef-w/Differentiable-iLQR) is pure PyTorch; its "FFI" for
 * this path is the Python autograd surface  MPC / LQRStep / pnqp / dynamics.
 * Each entry point below replaces one reference function (cited) and is what
 * the reference-side binding (ctypes) calls.
 *
 * Conventions (all entry points):
 *   - every pointer is a caller-owned DEVICE buffer, fp32, contiguous, in the
 *     reference's time-major layout: C [T,B,d,d], c [T,B,d], F [T-1,B,n,d],
 *     f [T-1,B,n], x [T,B,n], u [T,B,m], K [T,B,m,n], k [T,B,m]; x_init [B,n];
 *     per-problem vectors [B];  d = n + m;
 *   - gains are written in NATURAL time order (K[t] is the gain of step t);
 *   - pointers must be 16-byte aligned (torch allocations are);
 *   - `stream` is a hipStream_t passed as void* (0 = legacy default stream);
 *   - no allocation, no host synchronisation: every call is capturable in a
 *     hipGraph; all work is enqueued on `stream`;
 *   - return value: 0 = ok, >0 = invalid argument (DILQR_E_*), <0 = -(hipError_t).
 *   - reentrant, no global state: independent calls on different streams or
 *     devices are safe.
 *
 * Semantics are per problem (one problem per GPU lane); see DESIGN.md for the
 * three places where the reference couples problems of a batch (pnqp's
 * batch-max Armijo exit, pnqp's all-converged early return, and the MPC stop
 * rule — the last one IS reproduced on device).
 */
#ifndef DILQR_H
#define DILQR_H

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes ------------------------------------------------------- */
#define DILQR_OK 0
#define DILQR_E_SHAPE 1      /* unsupported (n, m) / model combination        */
#define DILQR_E_ARG 2        /* null or misaligned pointer, bad size          */
#define DILQR_E_MODE 3       /* unsupported option combination                */

/* ---- dynamics models (env_dx/ *.py) --------------------------------------- */
#define DILQR_MODEL_LINDX 0      /* x' = F_t [x;u] + f_t  (definitions.py LinDx) */
#define DILQR_MODEL_PENDULUM 1   /* env_dx/pendulum.py   n=3  m=1 p=3            */
#define DILQR_MODEL_CARTPOLE 2   /* env_dx/cartpole.py   n=5  m=1 p=4            */
#define DILQR_MODEL_ROCKET 3     /* env_dx/rocket.py     n=13 m=3 p=5            */
#define DILQR_MODEL_PENDULUM_COMPLEX 4  /* env_dx/pendulum.py simple=False: n=3 m=1
                                    p=5 (g, m, l, damping, gravity bias); its
                                    Jacobian is the autograd one (the clamp's
                                    gate applied), no second-order terms: the
                                    implicit backward, get_matrices, grad_input
                                    and the dynamics VJP return DILQR_E_SHAPE */

/* ---- control bounds (MPC u_lower/u_upper: float or [T,B,m] tensor) -------- */
#define DILQR_BOUNDS_NONE 0
#define DILQR_BOUNDS_SCALAR 1    /* lo/hi are floats                              */
#define DILQR_BOUNDS_TENSOR 2    /* lo_t/hi_t are [T,B,m] device tensors          */

/* ---- m>1 unconstrained gain solve ---------------------------------------- */
#define DILQR_SOLVE_INV 0        /* lqr_step_explicit.py:90-96 pinverse (=inverse
                                    for nonsingular Q_uu)                         */
#define DILQR_SOLVE_CHOL 1       /* lqr_step_backup.py:199-208 chol(Q_uu+1e-6 I)  */

typedef struct dilqr_bounds {
  int mode;                      /* DILQR_BOUNDS_*                               */
  float lo, hi;                  /* scalar bounds                                */
  const float* lo_t;             /* [T,B,m] or NULL                              */
  const float* hi_t;             /* [T,B,m] or NULL                              */
} dilqr_bounds;

/* Library version (for the loader's sanity check): 8. */
int dilqr_version(void);

/* Build id: the first 16 hex digits of the sha256 of the sources the library
   was built from (differentiable-ilqr_amd/Makefile BUILD_ID; the loader
   dilqr/_native.py recomputes it from the tree and refuses a mismatch). */
const char* dilqr_build_id(void);

/* Number of parameters theta of a model (4 for cartpole), or -1. */
int dilqr_model_num_params(int model);
int dilqr_model_num_ctrl(int model);

/* x' = f(x, u; theta) for N independent rows.  Replaces the models' forward():
   cartpole.py:64-97, pendulum.py:60-95, rocket.py:82-164.
   x [N,n], u [N,m], theta [p] device, out [N,n]. */
int dilqr_dynamics_f32(int model, int N, const float* theta, const float* x,
                       const float* u, float* out, void* stream);

/* Vector-Jacobian product of dilqr_dynamics_f32 (the reference obtains it from
   autograd through forward(), e.g. the sysid loss, il_exp.py:338-347): per row
   gtheta [N,p] = gout^T df/dtheta (per row; sum over rows for the parameter
   gradient), gx [N,n] = gout^T df/dx, gu [N,m] = gout^T df/du (0 where the
   model's control clamp is active), each at the clamped u.  gx, gu nullable.
   Models: pendulum, cartpole. */
int dilqr_dynamics_vjp_f32(int model, int N, const float* theta, const float* x,
                           const float* u, const float* gout, float* gtheta, float* gx,
                           float* gu, void* stream);
/* D = d f / d [x;u] at the unclamped u, [N,n,n+m].  Replaces get_linear_dyn:
   cartpole.py:790-839, pendulum.py:444-475, rocket.py:324-426. */
int dilqr_linear_dyn_f32(int model, int N, const float* theta, const float* x,
                         const float* u, float* D, void* stream);

/* Rollout x_{t+1} = f(x_t, u_t) from x_init; util.get_traj (util.py:104-127).
   For DILQR_MODEL_LINDX pass F [T-1,B,n,d] and f [T-1,B,n] (f may be NULL). */
int dilqr_rollout_f32(int model, int n, int m, int T, int B, const float* theta,
                      const float* F, const float* f, const float* x_init,
                      const float* u, float* x_out, void* stream);

/* Linearisation around (x,u): F = D(x_t,u_t), f = f(x_t,u_t) - F [x_t;u_t],
   t < T-1.  MPC.linearize_dynamics ANALYTIC, mpc_explicit.py:516-546. */
int dilqr_linearize_f32(int model, int T, int B, const float* theta, const float* x,
                        const float* u, float* F, float* f, void* stream);

/* Backward Riccati sweep in delta space: lqr_backward, lqr_step_explicit.py:54-162
   (with the c_back of 630-636 fused: c_back_t = C_t [x_t;u_t] + c_t; pass
   x = NULL to give c_back directly in c — u may then still be given, it only
   shifts the box bounds (lb = lower - u_t); with u = NULL too the bounds are
   taken as already relative, lb = lower: the delta_u trust region clips them
   to +-delta_u, lqr_step_explicit.py:132-135).  Bounded problems
   run pnqp (pnqp.py:5-82) per step, warm-started from the later step.
   u_zero_I [T,B,m] (uint8, nullable): the masked solve of
   lqr_step_backup.py:210-232 used by the adjoint engines.
   n_qp_iter [B] (nullable): per-problem sum of 1+pnqp iterations.
   n_qp_step [T] (nullable, zeroed by the caller): per step, the largest pnqp
   iteration count over the batch (atomic max) — the reference's batched pnqp
   runs until its slowest problem converges, so its n_total_qp_iter
   (lqr_step_explicit.py:148-150) is sum_t (1 + n_qp_step[t]). */
int dilqr_lqr_backward_f32(int n, int m, int T, int B, const float* C, const float* c,
                           const float* x, const float* u, const float* F,
                           dilqr_bounds bounds, const unsigned char* u_zero_I,
                           int m_solver, float* K, float* k, int* n_qp_iter,
                           int* n_qp_step, void* stream);

/* Rollout with per-problem backtracking line search: lqr_forward,
   lqr_step_explicit.py:166-263.  `model` gives the true dynamics (F/f for
   LINDX).  Outputs: new x/u, cost [B] (final pass), du_sq [T,m,B] =
   (u - new_u)^2 of the FIRST pass laid out [T,m,B] (input of
   dilqr_quirk_norm_f32), alpha [B] = the alpha of the final pass.
   old_cost [B] (nullable): the current trajectory's cost when the caller has
   it (an MPC loop: its previous line search's value for the accepted
   candidate), else formed from x, u (lqr_step_explicit.py:171); one lane per
   problem models and LINDX d <= 8 only (DILQR_E_MODE otherwise).  old_cost
   may alias cost (each problem's old cost is read before its new cost is
   written). */
int dilqr_lqr_forward_f32(int model, int n, int m, int T, int B, const float* theta,
                          const float* F, const float* f, const float* x_init,
                          const float* C, const float* c, const float* x,
                          const float* u, const float* K, const float* k,
                          dilqr_bounds bounds, const unsigned char* u_zero_I,
                          float linesearch_decay, int max_linesearch_iter,
                          float* x_out, float* u_out, float* cost, float* du_sq,
                          float* alpha, const float* old_cost, void* stream);

/* The reference's batch-mixing norm (lqr_step_explicit.py:245-247):
   (u-new_u).transpose(1,2).contiguous().view(B,-1).norm(2,1), i.e. row r is
   the 2-norm of elements [r*T*m, (r+1)*T*m) of the [T,m,B] buffer du_sq
   (already squared).  out [B]. */
int dilqr_quirk_norm_f32(int T, int m, int B, const float* du_sq, float* out,
                         void* stream);

/* ---- the iLQR outer loop (mpc_explicit.py:182-358) ------------------------ */

/* Device-resident loop state; zero it (hipMemsetAsync) before iteration 0. */
typedef struct dilqr_mpc_ctrl {
  int iter;              /* iterations executed                          */
  int stopped;           /* 1 once the stop rule fired                   */
  int n_not_improved;    /* mpc_explicit.py:264, 279                     */
  int any_improved;      /* scratch for the current iteration            */
  unsigned max_du_bits;  /* float bits of max(full_du_norm) this iter    */
  int pad[3];
} dilqr_mpc_ctrl;

/* Projected-Newton box QP, pnqp.py:5-82, per problem (the reference at batch
   size 1; its batched call couples the Armijo exits across the batch):
   min 1/2 x^T H x + q^T x, lower <= x <= upper.  H [B,m,m], q [B,m], bounds
   scalar or [B,m] (mode NONE is an error), x_init [B,m] nullable (then the
   unconstrained solve, pnqp.py:14-19).  Outputs x [B,m]; If [B,m] free mask,
   Hfree [B,m,m] the masked matrix of the last iteration (pnqp.py:44-48; the
   reference returns it for m=1 and its LU for m>1) and n_iter [B] the iteration
   index at exit (pnqp.py:59/82), each nullable.  m <= 4. */
int dilqr_pnqp_f32(int m, int B, const float* H, const float* q, dilqr_bounds bounds,
                   const float* x_init, float* x, float* If, float* Hfree, int* n_iter,
                   void* stream);

/* One fused iLQR iteration for a model (not LINDX): linearise on the fly,
   Riccati sweep (+pnqp), old cost, line-search rollout.  Reads the current
   trajectory (x,u), writes the new one (x_out,u_out), cost [B], du_sq [T,m,B],
   alpha [B].  The line search rolls passes 2r and 2r+1 out together and keeps
   the first accepted (the sequential search's result).  ws_gains: workspace
   of T*B*(ceil4(m*n+m+1) + n + m) floats (gain records + the second
   candidate's trajectory).  No-op when ctrl->stopped. */
int dilqr_ilqr_iterate_f32(int model, int T, int B, const float* theta,
                           const float* x_init, const float* C, const float* c,
                           const float* x, const float* u, dilqr_bounds bounds,
                           float linesearch_decay, int max_linesearch_iter,
                           float* ws_gains, float* x_out, float* u_out, float* cost,
                           float* du_sq, float* alpha, dilqr_mpc_ctrl* ctrl,
                           void* stream);

/* Best-iterate bookkeeping + stop rule of one MPC iteration
   (mpc_explicit.py:264-299): full_du_norm from du_sq (quirk layout), per
   problem "cost <= best + best_cost_eps" -> copy (x,u,cost,du) into best;
   then n_not_improved / stopped.  first != 0 for iteration 0.
   No-op when ctrl->stopped. */
int dilqr_mpc_update_best_f32(int n, int m, int T, int B, int first,
                              float best_cost_eps, float eps, int not_improved_lim,
                              const float* x, const float* u, const float* cost,
                              const float* du_sq, float* full_du_norm,
                              float* best_x, float* best_u, float* best_cost,
                              float* best_du, dilqr_mpc_ctrl* ctrl, void* stream);

/* ---- backward passes -------------------------------------------------------- */

/* Classic differentiable-LQR adjoint, lqr_step.py:312-407: r = [dl_dx;dl_du],
   active set |u - bound| <= 1e-8, one adjoint LQR solve (u_zero_I masked, m_solver
   as the engine), costates, outer products.  Outputs dx_init [B,n], dC, dc,
   dF [T-1,B,n,d], df [T-1,B,n] (df nullable).  ws: T*B*(m*n+m) floats. */
int dilqr_lqr_adjoint_f32(int n, int m, int T, int B, const float* C, const float* c,
                          const float* F, const float* x, const float* u,
                          const float* dl_dx, const float* dl_du, dilqr_bounds bounds,
                          int m_solver, float* ws, float* dx_init, float* dC, float* dc,
                          float* dF, float* df, void* stream);

/* DiLQR implicit backward through the iLQR fixed point: LQRStepFn.backward
   (lqr_step_explicit.py:653-712) with fix_point_equ (458-598) and the model's
   grad_input (cartpole.py:717-788, pendulum.py:383-443).  Inputs: the solution
   (x, u), its Riccati gains K [T,B,m,n] in NATURAL order (the kernel applies the
   reference's reversed-stack indexing itself), C, c, theta, dl_dx, dl_du, the
   box bounds (active set |u - bound| <= 1e-8).  Outputs dC [T,B,d,d], dc [T,B,d],
   dtheta [B,p] (per problem; the autograd caller sums over the batch).
   ws: T*B*dilqr_implicit_ws_floats(model) floats.  Models: pendulum, cartpole (one lane per
   problem), rocket (16 lanes per problem, rocket.py:263-323 and its builder
   tables 541-820). */
int dilqr_implicit_ws_floats(int model);
int dilqr_implicit_backward_f32(int model, int T, int B, const float* theta,
                                const float* C, const float* c, const float* x,
                                const float* u, const float* K, const float* dl_dx,
                                const float* dl_du, dilqr_bounds bounds, float* ws,
                                float* dC, float* dc, float* dtheta, void* stream);

/* ---- the model protocol's second-order API (not on the solver's path) ---- */

/* get_matrices: cartpole.py:105-716, pendulum.py:152-382, rocket.py:258-261
   (+ its build_batched_* tables, 541-820).  Per row of x [N,n], u [N,m] (the
   unclamped u): D [N,n,d] (= get_linear_dyn), D_params [N,n,d,p], D_x
   [N,n,d,n], D_u [N,n,d,m], x_theta [N,n,p], x_xtm1 [N,n,n], x_utm1 [N,n,m],
   with the reference's closed forms where they differ from the derivative
   (cartpole: D_params[4,3..5,*] and x_xtm1[0,0] = 0; rocket: the builder
   tables).  Zero-fills the sparse arrays on `stream` first. */
int dilqr_get_matrices_f32(int model, int N, const float* theta, const float* x,
                           const float* u, float* D, float* Dp, float* Dx, float* Du,
                           float* x_theta, float* x_xtm1, float* x_utm1, void* stream);

/* grad_input: cartpole.py:717-788, pendulum.py:383-443, rocket.py:263-323.
   X [T,B,n], U [T,B,m], K [T,B,m,n] consumed as K[t] (NULL = zeros), and
   dilqr_get_matrices_f32's outputs for the T*B rows.  Outputs grad_D
   [T-1,B,n,d,p], grad_d [T-1,B,n,p], d_x = -D_x tau [T-1,B,n,n], d_u = -D_u tau
   [T-1,B,n,m] (the 7-tuple's other members are get_matrices' D_x, D_u, D). */
int dilqr_grad_input_f32(int model, int T, int B, const float* X, const float* U,
                         const float* K, const float* D, const float* Dp, const float* Dx,
                         const float* Du, const float* x_theta, const float* x_xtm1,
                         const float* x_utm1, float* grad_D, float* grad_d, float* d_x,
                         float* d_u, void* stream);

/* ---- the device-resident MPC loop with per-problem trajectory slots ------ */
/* Caller-owned device buffers of one solve.  Xs and Us hold four trajectories
   per problem: for the pendulum and cartpole Xs is [4,T,B,n+m] records
   [x_t; u_t] (a lane moves its record with two wide accesses) and Us is unused
   (pass Xs); for rocket Xs is [4,T,B,n] and Us [4,T,B,m].  begin writes slot
   0 itself (see dilqr_mpc_begin_f32).  slot [2,B] (uint8) the indices of each
   problem's current and best one.  The line search's two candidates roll out
   into the two free slots, so accepting a step size or taking an iterate as
   the new best (mpc_explicit.py:277-283) moves no data.
   ws: T*B*ceil4(m*n+m+1) floats.  done_counter: the stop rule's sync area of
   16 + 4*ceil(B/64) uints.  ctrl: two dilqr_mpc_ctrl (ping-pong, zeroed by begin).
   Cpk (nullable) + cost_sym [B] (uint8): the solve's packed copy of a
   symmetric cost, T*B*dilqr_mpc_packed_cost_floats(n,m) floats (diag of C_t,b,
   then c_t,b, then the strict upper triangle row-major; component-major).
   From iteration 1 on, the fused kernel takes the current trajectory's cost
   (the line search's old cost) from cost[B], which the previous iteration's
   line search wrote for the accepted candidate, instead of summing it again.
   Iteration 0 (first != 0) reads C, c and writes the copy and, per problem,
   flags: bit 0 all its C_t bitwise symmetric, bit 1 all off-diagonals +0.0 too.
   Later iterations of flagged problems read the copy: 27 instead of 42 floats
   per step at d=6, or 12 for a diagonal cost (diag(q), the reference's own
   callers, il_env.py:159-162); identical arithmetic.  The cost passed to the
   iterations of one solve must not change.  For the lane-group models
   (rocket) Cpk holds B*2d floats instead: iteration 0 sets cost_sym[b]
   = 7 when problem b's cost is diagonal (off-diagonal entries +0.0) and the
   same at every t, and stores its diag and c [B][2d]; later iterations of
   such problems hold them in registers and read no cost at all.
   Invariant: every trajectory held in a slot is a rollout of the model, i.e.
   x_{t+1} == forward(x_t, u_t) bit for bit with u_t as stored (already
   clamped to the box) — begin and the line search write only such
   trajectories.  The fused sweep relies on it: models whose Jacobian needs the
   integrated angle's cos/sin (cartpole) take them from x_{t+1} instead of
   recomputing them from x_t.  Do not write into Xs/Us from outside. */
typedef struct dilqr_mpc_state {
  float* Xs; float* Us; unsigned char* slot; float* best_cost; float* best_du;
  int* improved; float* cost; float* alpha; float* du_sq; float* full_du_norm;
  float* ws; dilqr_mpc_ctrl* ctrl; unsigned* done_counter; float* Cpk;
  unsigned char* cost_sym;
  int* best_iter;        /* [B], fixed-count solves only (NULL otherwise) */
} dilqr_mpc_state;

/* Start a solve: slot 0 = (get_traj(u), u) with u = u_init or zeros when
   u_init is NULL; slots/ctrl reset (mpc_explicit.py:228-249, util.py:104-127).
   u_init: the caller's controls, fp32 [T,B,m] contiguous (time-major, the
   reference's layout), read once with scalar loads, so 4-byte alignment
   suffices (checked; the 16-byte rule above does not apply to it). */
int dilqr_mpc_packed_cost_floats(int n, int m);
int dilqr_mpc_begin_f32(int model, int T, int B, const float* theta, const float* x_init,
                        const float* u_init, dilqr_mpc_state st, void* stream);

/* One MPC iteration (mpc_explicit.py:246-299), iteration = 0, 1, ... of the
   solve.  Two launches: (1) the stop rule for iteration-1 (mpc_explicit.py:264,
   279, 297-299: max full_du_norm < eps or n_not_improved > not_improved_lim) as
   the prologue of the fused linearise + Riccati (+pnqp) + line-search kernel on
   each problem's current slot with the best-iterate slot update; (2) the quirk
   full_du_norm rows, best_du and per-workgroup partials of this iteration for
   the next prologue.  Once stopped, iterations are no-ops.  The control state
   after the decisions for iterations 0..k-1 is in ctrl[k&1] (ctrl points to two
   dilqr_mpc_ctrl).  = dilqr_mpc_step_f32 + dilqr_mpc_stop_rule_f32. */
int dilqr_mpc_iterate_f32(int model, int T, int B, const float* theta, const float* x_init,
                          const float* C, const float* c, dilqr_bounds bounds,
                          float linesearch_decay, int max_linesearch_iter, int iteration,
                          float best_cost_eps, float eps, int not_improved_lim,
                          dilqr_mpc_state st, void* stream);
/* Iterations first_iteration .. first_iteration+count-1 of the same solve in
   one call (ABI 7): dilqr_mpc_iterate_f32 for each, in order — the host
   launches a run of iterations between two polls of the stop flag without a
   foreign-function round trip per iteration (iterations after a stop are
   device no-ops either way). */
int dilqr_mpc_iterate_range_f32(int model, int T, int B, const float* theta, const float* x_init,
                                const float* C, const float* c, dilqr_bounds bounds,
                                float linesearch_decay, int max_linesearch_iter,
                                int first_iteration, int count, float best_cost_eps, float eps,
                                int not_improved_lim, dilqr_mpc_state st, void* stream);
/* its two launches, separately (profiling) */
int dilqr_mpc_step_f32(int model, int T, int B, const float* theta, const float* x_init,
                       const float* C, const float* c, dilqr_bounds bounds,
                       float linesearch_decay, int max_linesearch_iter, int iteration,
                       float best_cost_eps, float eps, int not_improved_lim,
                       dilqr_mpc_state st, void* stream);
int dilqr_mpc_stop_rule_f32(int T, int m, int B, int iteration, dilqr_mpc_state st,
                            void* stream);

/* Fixed-count solves: eps <= 0 and not_improved_lim >= the number of
   iterations, so the stop rule (mpc_explicit.py:297-299) can never fire and
   the solve runs all of them (the reference's loop does exactly that).  Each
   iteration is ONE launch — the fused kernel with no stop-rule prologue — that
   writes its du rows into plane `iteration` of du_sq (then [iters,T,m,B]) and
   keeps in best_iter[B] the last iteration that took the best-iterate branch
   (mpc_explicit.py:277-283).  dilqr_mpc_finish_fixed_f32 then forms best_du
   from those planes (the quirk rows, lqr_step_explicit.py:245-247, bit for bit
   the per-iteration rule's values), full_du_norm from the last iteration's
   plane (what the per-iteration rule leaves there) and sets ctrl[].iter. */
int dilqr_mpc_iterate_fixed_f32(int model, int T, int B, const float* theta, const float* x_init,
                                const float* C, const float* c, dilqr_bounds bounds,
                                float linesearch_decay, int max_linesearch_iter, int iteration,
                                float best_cost_eps, dilqr_mpc_state st, void* stream);
int dilqr_mpc_finish_fixed_f32(int T, int m, int B, int iterations, dilqr_mpc_state st,
                               void* stream);

/* A whole fixed-count solve in one call (ABI 6): begin (u_init as in
   dilqr_mpc_begin_f32), `iterations` iterations, finish — the same results,
   bit for bit, as dilqr_mpc_begin_f32 + dilqr_mpc_iterate_fixed_f32 per
   iteration + dilqr_mpc_finish_fixed_f32.  Pendulum and cartpole run begin
   and every iteration in ONE launch (each lane iterates its own problem; no
   problem couples to another until best_du), then the finish launch; rocket
   keeps its per-iteration launches (the 8-lane sweep, then the lane-pair
   line search, each in one instantiation per cost kind).  st.du_sq must hold iterations*T*m*B
   floats and st.best_iter must be set. */
int dilqr_mpc_solve_fixed_f32(int model, int T, int B, const float* theta, const float* x_init,
                              const float* u_init, const float* C, const float* c,
                              dilqr_bounds bounds, float linesearch_decay,
                              int max_linesearch_iter, int iterations, float best_cost_eps,
                              dilqr_mpc_state st, void* stream);

/* A whole stop-rule solve in one launch for a small batch (ABI 9): begin (u_init
   as in dilqr_mpc_begin_f32), then up to `iterations` iterations with the stop
   rule (mpc_explicit.py:264-299: max full_du_norm < eps or n_not_improved >
   not_improved_lim) applied after each, inside ONE workgroup holding every
   problem — the rule's batch-mixing rows and reductions need a barrier, not a
   launch, and the host polls nothing.  The same iterates, costs, best_du,
   full_du_norm and stop iteration as dilqr_mpc_begin_f32 +
   dilqr_mpc_iterate_f32 per iteration; ctrl[0] = ctrl[1] = the control word
   those launches leave: {iter, stopped, n_not_improved, max_du_bits} with iter
   = the iterations run and max_du_bits that of the last one when the rule
   stopped the solve, else iter = iterations - 1 and the max of the iteration
   before the last (the last iteration's rule is never applied).  B <= 256 and the thread-per-problem
   models (pendulum, cartpole, 5-parameter pendulum); DILQR_E_SHAPE otherwise.
   Replaces the per-iteration loop of MPC.forward for the IL loop's batches
   (il_exp.py:44 n_batch = 32, il_env.py:153-188). */
int dilqr_mpc_solve_small_f32(int model, int T, int B, const float* theta, const float* x_init,
                              const float* u_init, const float* C, const float* c,
                              dilqr_bounds bounds, float linesearch_decay,
                              int max_linesearch_iter, int iterations, float best_cost_eps,
                              float eps, int not_improved_lim, dilqr_mpc_state st, void* stream);

/* Materialise each problem's best trajectory into x_out [T,B,n], u_out [T,B,m]. */
int dilqr_mpc_gather_best_f32(int n, int m, int T, int B, dilqr_mpc_state st, float* x_out,
                              float* u_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DILQR_H */
