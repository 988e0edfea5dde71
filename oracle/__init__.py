"""CPU oracle for the batched differentiable-iLQR hot path.

TEST INFRASTRUCTURE ONLY.  This package is a from-scratch numpy restatement of
the reference algorithm (josef-w/Differentiable-iLQR).  Every function cites
the reference file:line it restates.  It is pinned against golden vectors that
the reference itself produced (tests/golden/*.npz, made by
tests/golden/gen_golden.py) and against the reference's own known-answer
datasets (data/cartpole.pkl, data/pendulum.pkl, parsed statically).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
it, and only as the checker or the CPU baseline — never as the thing measured
or shipped.  The product path (differentiable-ilqr_amd/dilqr) never imports
this package and fails loudly when its HIP library is missing.

Modules:
  models   dynamics (forward / get_linear_dyn / get_matrices / grad_input)
  lqr      Riccati sweep, pnqp box QP, rollout + line search
  mpc      the iLQR outer loop (mpc_explicit.MPC.forward)
  adjoint  classic adjoint (lqr_step.py backward) and the DiLQR implicit
           backward (lqr_step_explicit.py backward + fix_point_equ)
"""
