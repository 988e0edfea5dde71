"""Functional layer over the C-ABI: allocate outputs, launch on the current
stream.  Every function here is one (or a few) libdilqr.so calls; nothing
computes on the host.
"""
import collections
import os

import torch

from . import _native as N


def _f32(t):
    if t is None:
        return None
    if t.dtype != torch.float32:
        raise TypeError(f"dilqr computes in fp32; got {t.dtype}")
    return t.detach().contiguous()


def model_id_of(dx):
    from .definitions import LinDx
    if isinstance(dx, LinDx):
        return N.MODEL_LINDX
    mid = getattr(dx, "model_id", None)
    if mid is None:
        raise NotImplementedError(
            "dilqr: dynamics must be a dilqr.env_dx model or a LinDx "
            "(generic autograd/finite-difference dynamics are not on the HIP path)")
    return mid


def generic_model_id(dx):
    """model_id_of, or None for a dynamics Module the HIP kernels do not model
    (the caller then runs it in torch)."""
    from .definitions import LinDx
    if isinstance(dx, LinDx):
        return N.MODEL_LINDX
    return getattr(dx, "model_id", None)


def theta_of(dx, like):
    return dx._theta(like)


def rollout(model_id, theta, x_init, u, F=None, f=None):
    """util.get_traj (util.py:104-127)."""
    T, B, m = u.shape
    n = x_init.shape[1]
    x_init, u, F, f = _f32(x_init), _f32(u), _f32(F), _f32(f)
    x = torch.empty(T, B, n, device=u.device)
    N.call("dilqr_rollout_f32", model_id, n, m, T, B, N.ptr(theta), N.ptr(F), N.ptr(f), N.ptr(x_init), N.ptr(u),
           N.ptr(x), N.stream(u.device))
    return x


def linearize(model_id, theta, x, u):
    """MPC.linearize_dynamics ANALYTIC (mpc_explicit.py:516-546)."""
    T, B, n = x.shape
    m = u.shape[2]
    x, u = _f32(x), _f32(u)
    F = torch.empty(max(T - 1, 0), B, n, n + m, device=x.device)
    f = torch.empty(max(T - 1, 0), B, n, device=x.device)
    N.call("dilqr_linearize_f32", model_id, T, B, N.ptr(theta), N.ptr(x), N.ptr(u), N.ptr(F), N.ptr(f),
           N.stream(x.device))
    return F, f


def zero_mask(u_zero_I, T, B, m, device):
    """u_zero_I as the kernels read it: uint8 [T,B,m] on `device` (the kernels
    index it (t*B + b)*m + a for every t and b, so any other shape is refused
    here rather than read out of bounds on the device)."""
    if u_zero_I is None:
        return None
    if tuple(u_zero_I.shape) != (T, B, m):
        raise ValueError(f"u_zero_I: expected [T, B, m] = {(T, B, m)}, got {tuple(u_zero_I.shape)}")
    return u_zero_I.to(device=device, dtype=torch.uint8).contiguous()


def lqr_backward(C, c, F, n, m, x=None, u=None, u_lower=None, u_upper=None, u_zero_I=None,
                 m_solver=N.SOLVE_INV, want_nqp=False, qp_total=False):
    """lqr_backward (lqr_step_explicit.py:54-162) with the fused delta-space c_back.
    Returns K [T,B,m,n], k [T,B,m] (natural time order), and n_qp [B] (the
    per-problem sums of 1 + pnqp iterations) with want_nqp, or with qp_total
    the reference's n_total_qp_iter (lqr_step_explicit.py:148-150: its batched
    pnqp runs each step until the slowest problem converges, so the count is
    sum_t (1 + max over problems of that step's iterations); 0 unbounded)."""
    T, B = C.shape[:2]
    C, c, F, x, u = _f32(C), _f32(c), _f32(F), _f32(x), _f32(u)
    bounds, keep = N.make_bounds(u_lower, u_upper)
    zI = zero_mask(u_zero_I, T, B, m, C.device)
    K = torch.empty(T, B, m, n, device=C.device)
    k = torch.empty(T, B, m, device=C.device)
    nqp = torch.zeros(B, dtype=torch.int32, device=C.device) if want_nqp else None
    step = torch.zeros(T, dtype=torch.int32, device=C.device) if qp_total else None
    N.call("dilqr_lqr_backward_f32", n, m, T, B, N.ptr(C), N.ptr(c), N.ptr(x), N.ptr(u), N.ptr(F), bounds,
           N.ptr(zI), m_solver, N.ptr(K), N.ptr(k), N.ptr(nqp), N.ptr(step), N.stream(C.device))
    del keep
    if qp_total:
        return K, k, (int(step.sum().item()) + T if bounds.mode != N.BOUNDS_NONE else 0)
    return K, k, nqp


def c_back(C, c, x, u):
    """Delta-space linear term C_t tau_t + c_t (lqr_step_explicit.py:630-636),
    for the callers that hand the sweep relative bounds (delta_u)."""
    tau = torch.cat((x, u), -1)
    return (C @ tau.unsqueeze(-1)).squeeze(-1) + c


def _full(v, like):
    return v if isinstance(v, torch.Tensor) else torch.full_like(like, float(v))


def delta_u_sweep_bounds(u_lower, u_upper, u, delta_u):
    """The sweep's box in delta space with the delta_u trust region,
    lqr_step_explicit.py:132-135: lb = lower - u_t, ub = upper - u_t, then
    lb[lb < -delta_u] = -delta_u, ub[ub > delta_u] = delta_u (exact values)."""
    lb = _full(u_lower, u) - u
    ub = _full(u_upper, u) - u
    lb = torch.where(lb < -delta_u, torch.full_like(lb, -delta_u), lb)
    ub = torch.where(ub > delta_u, torch.full_like(ub, delta_u), ub)
    return lb.contiguous(), ub.contiguous()


def delta_u_rollout_bounds(u_lower, u_upper, u, delta_u):
    """The rollout's clamp with the delta_u trust region, lqr_step_explicit.py:
    205-213: lb = u_t - delta_u raised to lower, ub = u_t + delta_u cut to upper."""
    lb = u - delta_u
    ub = u + delta_u
    lo, hi = _full(u_lower, u), _full(u_upper, u)
    lb = torch.where(lb < lo, lo, lb)
    ub = torch.where(ub > hi, hi, ub)
    return lb.contiguous(), ub.contiguous()


def lqr_forward(model_id, theta, x_init, C, c, x, u, K, k, F=None, f=None, u_lower=None, u_upper=None,
                u_zero_I=None, linesearch_decay=0.2, max_linesearch_iter=10):
    """lqr_forward (lqr_step_explicit.py:166-263): returns new_x, new_u, costs [B],
    du_sq [T,m,B] (first pass), alphas [B] (final pass)."""
    T, B, n = x.shape
    m = u.shape[2]
    x_init, C, c, x, u, K, k, F, f = map(_f32, (x_init, C, c, x, u, K, k, F, f))
    bounds, keep = N.make_bounds(u_lower, u_upper)
    zI = zero_mask(u_zero_I, T, B, m, x.device)
    dev = x.device
    nx, nu = torch.empty_like(x), torch.empty_like(u)
    cost, alpha = torch.empty(B, device=dev), torch.empty(B, device=dev)
    du_sq = torch.empty(T, m, B, device=dev)
    N.call("dilqr_lqr_forward_f32", model_id, n, m, T, B, N.ptr(theta), N.ptr(F), N.ptr(f), N.ptr(x_init),
           N.ptr(C), N.ptr(c), N.ptr(x), N.ptr(u), N.ptr(K), N.ptr(k), bounds, N.ptr(zI),
           float(linesearch_decay), int(max_linesearch_iter), N.ptr(nx), N.ptr(nu), N.ptr(cost), N.ptr(du_sq),
           N.ptr(alpha), None, N.stream(dev))
    del keep
    return nx, nu, cost, du_sq, alpha


def pnqp(H, q, lower, upper, x_init=None):
    """pnqp.py:5-82 per problem -> (x [B,m], H_ [B,m,m], If [B,m], n_iter [B]).
    lower/upper: floats or [B,m] tensors.  The reference's batched call couples
    the Armijo loop across the batch; this is the reference at batch size 1."""
    B, m = q.shape
    H, q, x_init = _f32(H), _f32(q), _f32(x_init)
    bounds, keep = N.make_bounds(lower, upper)
    x = torch.empty(B, m, device=q.device)
    If = torch.empty(B, m, device=q.device)
    Hf = torch.empty(B, m, m, device=q.device)
    it = torch.empty(B, dtype=torch.int32, device=q.device)
    N.call("dilqr_pnqp_f32", m, B, N.ptr(H), N.ptr(q), bounds, N.ptr(x_init), N.ptr(x), N.ptr(If), N.ptr(Hf),
           N.ptr(it), N.stream(q.device))
    del keep
    return x, Hf, If, it


def quirk_norm(du_sq):
    """lqr_step_explicit.py:245-247 norm over the re-viewed [T,m,B] buffer."""
    T, m, B = du_sq.shape
    out = torch.empty(B, device=du_sq.device)
    N.call("dilqr_quirk_norm_f32", T, m, B, N.ptr(du_sq), N.ptr(out), N.stream(du_sq.device))
    return out


def grec_floats(n, m):
    return ((m * n + m + 1) + 3) // 4 * 4


def ilqr_ws_floats(n, m):
    """Per-(t,b) workspace of dilqr_ilqr_iterate_f32: gain record + the line
    search's second candidate (x, u)."""
    return grec_floats(n, m) + n + m


class MPCWorkspace:
    """Device buffers of one MPC solve (reused across iterations)."""

    def __init__(self, T, B, n, m, device, packed_cost=True):
        dev = device
        self.xa = torch.empty(T, B, n, device=dev)
        self.ua = torch.empty(T, B, m, device=dev)
        self.xb = torch.empty(T, B, n, device=dev)
        self.ub = torch.empty(T, B, m, device=dev)
        self.ws = torch.empty(T * B * grec_floats(n, m), device=dev)
        self.cost = torch.empty(B, device=dev)
        self.alpha = torch.empty(B, device=dev)
        self.du_sq = torch.empty(T, m, B, device=dev)
        self.fdn = torch.empty(B, device=dev)
        self.best_x = torch.empty(T, B, n, device=dev)
        self.best_u = torch.empty(T, B, m, device=dev)
        self.best_cost = torch.empty(B, device=dev)
        self.best_du = torch.empty(B, device=dev)
        self.ctrl = torch.zeros(N.CTRL_INTS, dtype=torch.int32, device=dev)


class MPCSolve:
    """Device state of one fused MPC solve (dilqr_mpc_state): three trajectory
    slots per problem (current, best, two line-search candidates), per-problem
    best bookkeeping, the loop control block."""

    def __init__(self, T, B, n, m, device, packed_cost=True, fixed_iters=None):
        """fixed_iters: a fixed-count solve of that many iterations (the stop rule
        cannot fire: eps <= 0, not_improved_lim >= iterations) — one launch per
        iteration (iterate_fixed) and finish_fixed at the end; du_sq keeps one
        [T,m,B] plane per iteration."""
        dev = device
        self.T, self.B, self.n, self.m = T, B, n, m
        self.fixed_iters = fixed_iters
        # slots: [4,T,B,n+m] records [x_t; u_t] for the thread-per-problem models
        # (Us aliases Xs, unused by the kernels), the caller's [4,T,B,n] and
        # [4,T,B,m] for rocket
        self.rec = n + m <= 8
        if self.rec:
            self.Xs = torch.zeros((4, T, B, n + m), device=dev)
            self.Us = self.Xs
        else:
            self.Xs = torch.empty((4, T, B, n), device=dev)
            self.Us = torch.zeros((4, T, B, m), device=dev)
        self.slot = torch.zeros(2, B, dtype=torch.uint8, device=dev)
        self.best_cost = torch.empty(B, device=dev)
        self.best_du = torch.empty(B, device=dev)
        self.improved = torch.zeros(B, dtype=torch.int32, device=dev)
        self.cost = torch.empty(B, device=dev)
        self.alpha = torch.empty(B, device=dev)
        self.du_sq = torch.empty((fixed_iters or 1) * T, m, B, device=dev)
        self.best_iter = torch.zeros(B, dtype=torch.int32, device=dev) if fixed_iters else None
        self.full_du_norm = torch.empty(B, device=dev)
        self.ws = torch.empty(T * B * ilqr_ws_floats(n, m), device=dev)
        self.ctrl = torch.zeros(2 * N.CTRL_INTS, dtype=torch.int32, device=dev)   # ping-pong control state
        self.last_iteration = -1
        # stop-rule sync area: 16 words + two planes of per-workgroup partials (<= ceil(B/64))
        self.counter = torch.zeros(16 + 4 * ((B + 63) // 64), dtype=torch.int32, device=dev)
        # the solve's copy of its cost: packed symmetric records for the thread-per-
        # problem fused kernels (d <= 8), one [2d] row record per problem (a
        # time-invariant diagonal cost) for the 16-lane ones
        pk = N.lib().dilqr_mpc_packed_cost_floats(n, m)
        if not packed_cost:
            self.Cpk = None
        elif n + m <= 8:
            self.Cpk = torch.empty(T * B * pk, device=dev)
        else:
            self.Cpk = torch.empty(B * 2 * (n + m), device=dev)
        self.cost_sym = torch.zeros(B, dtype=torch.uint8, device=dev) if self.Cpk is not None else None
        self.state = N.MpcState(*[t.data_ptr() if t is not None else None for t in (
            self.Xs, self.Us, self.slot, self.best_cost, self.best_du, self.improved, self.cost, self.alpha,
            self.du_sq, self.full_du_norm, self.ws, self.ctrl, self.counter, self.Cpk, self.cost_sym,
            self.best_iter)])

    def _u_init(self, u_init):
        if u_init is None:
            return None
        u0 = u_init.to(device=self.Xs.device, dtype=torch.float32)
        if u0.ndimension() == 2:
            u0 = u0.unsqueeze(1).expand(self.T, self.B, self.m)
        u0 = u0.contiguous()
        if tuple(u0.shape) != (self.T, self.B, self.m):
            raise ValueError(f"u_init: expected [T, B, m] = {(self.T, self.B, self.m)} or [T, m], got "
                             f"{tuple(u_init.shape)}")
        return u0

    def begin(self, model_id, theta, x_init, u_init=None):
        """x = get_traj(u_init or 0) into slot 0; reset slots and the control block."""
        u0 = self._u_init(u_init)
        N.call("dilqr_mpc_begin_f32", model_id, self.T, self.B, N.ptr(theta), N.ptr(x_init),
               None if u0 is None else N.ptr(u0), self.state, N.stream(x_init.device))
        self._u0 = u0                       # alive until the launch has read it

    def solve_fixed(self, model_id, theta, x_init, C, c, bounds, decay, max_ls, best_cost_eps, u_init=None):
        """A whole fixed-count solve of fixed_iters iterations in one call
        (dilqr_mpc_solve_fixed_f32: begin + every iteration in one launch for
        the single-lane models, then finish); the same bits as begin +
        iterate_fixed per iteration + finish_fixed."""
        if not self.fixed_iters:
            raise ValueError("solve_fixed: solve not built for a fixed count")
        u0 = self._u_init(u_init)
        N.call("dilqr_mpc_solve_fixed_f32", model_id, self.T, self.B, N.ptr(theta), N.ptr(x_init),
               None if u0 is None else N.ptr(u0), N.ptr(C), N.ptr(c), bounds, float(decay), int(max_ls),
               int(self.fixed_iters), float(best_cost_eps), self.state, N.stream(x_init.device))
        self._u0 = u0
        self.last_iteration = self.fixed_iters - 1

    def solve_small(self, model_id, theta, x_init, C, c, bounds, decay, max_ls, iterations, best_cost_eps, eps,
                    not_improved_lim, u_init=None):
        """A whole stop-rule solve in one launch (dilqr_mpc_solve_small_f32: B <=
        SMALL_BATCH_MAX, one workgroup, the rule applied in-kernel after each
        iteration); the same bits as begin + iterate per iteration."""
        u0 = self._u_init(u_init)
        N.call("dilqr_mpc_solve_small_f32", model_id, self.T, self.B, N.ptr(theta), N.ptr(x_init),
               None if u0 is None else N.ptr(u0), N.ptr(C), N.ptr(c), bounds, float(decay), int(max_ls),
               int(iterations), float(best_cost_eps), float(eps), int(min(not_improved_lim, 2 ** 31 - 1)),
               self.state, N.stream(x_init.device))
        self._u0 = u0
        self.small = True
        self.last_iteration = iterations - 1

    def iterate(self, model_id, theta, x_init, C, c, bounds, decay, max_ls, iteration, best_cost_eps, eps,
                not_improved_lim):
        """Iteration `iteration` (0, 1, ...) of the solve started by begin()."""
        if isinstance(iteration, bool):
            raise TypeError("iteration is the 0-based iteration index")
        N.call("dilqr_mpc_iterate_f32", model_id, self.T, self.B, N.ptr(theta), N.ptr(x_init), N.ptr(C),
               N.ptr(c), bounds, float(decay), int(max_ls), int(iteration), float(best_cost_eps), float(eps),
               int(min(not_improved_lim, 2 ** 31 - 1)), self.state, N.stream(x_init.device))
        self.last_iteration = int(iteration)

    def iterate_range(self, model_id, theta, x_init, C, c, bounds, decay, max_ls, first, count, best_cost_eps, eps,
                      not_improved_lim):
        """Iterations first .. first+count-1 in one library call (the same
        launches as iterate() for each)."""
        N.call("dilqr_mpc_iterate_range_f32", model_id, self.T, self.B, N.ptr(theta), N.ptr(x_init), N.ptr(C),
               N.ptr(c), bounds, float(decay), int(max_ls), int(first), int(count), float(best_cost_eps), float(eps),
               int(min(not_improved_lim, 2 ** 31 - 1)), self.state, N.stream(x_init.device))
        if count > 0:
            self.last_iteration = int(first + count - 1)

    def iterate_fixed(self, model_id, theta, x_init, C, c, bounds, decay, max_ls, iteration, best_cost_eps):
        """Iteration `iteration` of a fixed-count solve (one launch, no stop rule)."""
        if not self.fixed_iters or not 0 <= iteration < self.fixed_iters:
            raise ValueError("iterate_fixed: solve not built for a fixed count, or iteration out of range")
        N.call("dilqr_mpc_iterate_fixed_f32", model_id, self.T, self.B, N.ptr(theta), N.ptr(x_init), N.ptr(C),
               N.ptr(c), bounds, float(decay), int(max_ls), int(iteration), float(best_cost_eps), self.state,
               N.stream(x_init.device))
        self.last_iteration = int(iteration)

    def finish_fixed(self, iterations):
        """best_du of a fixed-count solve after `iterations` iterations."""
        N.call("dilqr_mpc_finish_fixed_f32", self.T, self.m, self.B, int(iterations), self.state,
               N.stream(self.Xs.device))

    def poll_buffer(self, i):
        """Pinned host buffer i (a small ring) for mpc_solve's non-blocking stop
        polls; a buffer is reused only after its poll was read."""
        if not hasattr(self, "_polls"):
            self._polls = [torch.empty(N.CTRL_INTS, dtype=torch.int32, pin_memory=True)
                           for _ in range(POLL_AHEAD + 2)]
        return self._polls[i % len(self._polls)]

    def _ctrl_now(self):
        k = max(self.last_iteration, 0)
        return self.ctrl.view(2, N.CTRL_INTS)[k & 1]        # solve_small writes both words

    def gather_best(self):
        x = torch.empty(self.T, self.B, self.n, device=self.Xs.device)
        u = torch.empty(self.T, self.B, self.m, device=self.Xs.device)
        N.call("dilqr_mpc_gather_best_f32", self.n, self.m, self.T, self.B, self.state, N.ptr(x), N.ptr(u),
               N.stream(x.device))
        return x, u

    @property
    def stopped(self):
        """True once the stop rule fired (the device skips later iterations); the
        rule for the last launched iteration is applied by the next one."""
        return bool(int(self._ctrl_now()[1].item()))

    @property
    def iterations(self):
        """The iterations that ran: the device's count when the stop rule fired
        (published by the prologue after the iteration that met it), else every
        launched iteration (the rule of the last one is never applied, so the
        device word then reads one less; every solve path leaves the same word)."""
        ctrl = self._ctrl_now()
        if int(ctrl[1].item()):
            return int(ctrl[0].item())
        return self.last_iteration + 1


# runs of the stop-rule loop queued behind the oldest unread stop-flag copy
# (mpc_solve): the host waits for a poll only this far behind the device
# (DILQR_POLL_AHEAD=0: a blocking poll after every run, the round-5 loop)
POLL_AHEAD = int(os.environ.get("DILQR_POLL_AHEAD", "2"))

# dilqr_mpc_solve_small_f32: batches one workgroup holds, thread-per-problem models
SMALL_BATCH_MAX = 256
SMALL_BATCH_MODELS = (N.MODEL_PENDULUM, N.MODEL_CARTPOLE, N.MODEL_PENDULUM_COMPLEX)


def mpc_solve(model_id, theta, x_init, C, c, T, u_init=None, u_lower=None, u_upper=None, lqr_iter=10,
              eps=1e-7, linesearch_decay=0.2, max_linesearch_iter=10, not_improved_lim=5, best_cost_eps=1e-4,
              check_every=8, verbose=0):
    """The iLQR outer loop of mpc_explicit.MPC.forward (mpc_explicit.py:228-299)
    entirely on device (fused iterate kernel + norm/stop kernel per iteration);
    the host only polls the stop flag every `check_every` iterations.
    Returns (best_x, best_u, best_cost, best_du, solve).

    verbose > 0: the same launches one iteration per library call, each
    followed by reductions queued on the stream (mean best cost, max
    full_du_norm, mean step size: the reference's table row, mpc_explicit.py:
    285-295) into a device array; `solve.log` holds them for util.print_solve_log
    (no host sync inside the loop)."""
    B, n = x_init.shape
    m = C.shape[-1] - n
    x_init, C, c = _f32(x_init), _f32(C), _f32(c)
    # the stop rule (max full_du_norm < eps or n_not_improved > lim) cannot fire:
    # one launch per iteration, best_du formed at the end (same values).  The
    # per-iteration du planes are kept, so this mode is taken only while they
    # stay small: at most 1/16 of the free device memory and 2 GiB
    plane_bytes = 4 * lqr_iter * T * m * B
    fixed = (lqr_iter >= 1 and eps <= 0 and not_improved_lim >= lqr_iter
             and plane_bytes <= min(2 ** 31, torch.cuda.mem_get_info(x_init.device)[0] // 16))
    sv = MPCSolve(T, B, n, m, x_init.device, fixed_iters=lqr_iter if fixed else None)
    bounds, keep = N.make_bounds(u_lower, u_upper)
    if verbose > 0:
        _mpc_solve_logged(sv, model_id, theta, x_init, C, c, u_init, bounds, u_lower is None, lqr_iter, eps,
                          linesearch_decay, max_linesearch_iter, not_improved_lim, best_cost_eps)
        del keep
        x, u = sv.gather_best()
        return x, u, sv.best_cost, sv.best_du, sv
    if fixed:
        sv.solve_fixed(model_id, theta, x_init, C, c, bounds, linesearch_decay, max_linesearch_iter, best_cost_eps,
                       u_init)
        del keep
        x, u = sv.gather_best()
        return x, u, sv.best_cost, sv.best_du, sv
    if B <= SMALL_BATCH_MAX and model_id in SMALL_BATCH_MODELS and lqr_iter >= 1:
        # the whole stop-rule loop in one launch (one workgroup holds the batch)
        sv.solve_small(model_id, theta, x_init, C, c, bounds, linesearch_decay, max_linesearch_iter, lqr_iter,
                       best_cost_eps, eps, not_improved_lim, u_init)
        del keep
        x, u = sv.gather_best()
        return x, u, sv.best_cost, sv.best_du, sv
    sv.begin(model_id, theta, x_init, u_init)
    # runs of check_every iterations per library call (iterations after a stop
    # are device no-ops).  The stop flag is polled without stalling the device:
    # after each run the control word is copied to pinned host memory behind an
    # event, and the host only waits for the copy of a run once POLL_AHEAD runs
    # are queued behind it — so the GPU never drains while the host looks (a
    # blocking poll every 8 iterations idled it once per poll), and at most
    # POLL_AHEAD runs of no-op launches follow a stop.
    step = check_every if check_every else max(lqr_iter, 1)
    polls = collections.deque()
    n_polls = 0
    stream = torch.cuda.current_stream(x_init.device)
    for i0 in range(0, lqr_iter, step):
        sv.iterate_range(model_id, theta, x_init, C, c, bounds, linesearch_decay, max_linesearch_iter, i0,
                         min(step, lqr_iter - i0), best_cost_eps, eps, not_improved_lim)
        if i0 + step >= lqr_iter:
            break
        host = sv.poll_buffer(n_polls)            # a ring longer than the polls in flight
        n_polls += 1
        host.copy_(sv._ctrl_now(), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
        polls.append((ev, host))
        stopped = False
        while polls and (len(polls) > POLL_AHEAD or polls[0][0].query()):
            ev0, host0 = polls.popleft()
            ev0.synchronize()
            if int(host0[1]):
                stopped = True
                break
        if stopped:
            break
    del keep
    x, u = sv.gather_best()
    return x, u, sv.best_cost, sv.best_du, sv


def quad_traj_cost(x, u, C, c):
    """util.get_cost for a quadratic cost (util.py:130-153): per problem,
    sum_t 0.5 tau_t^T C_t tau_t + c_t^T tau_t, in torch on the device (the
    verbose report's initial cost only)."""
    tau = torch.cat((x, u), -1)
    return (0.5 * torch.einsum("tbi,tbij,tbj->tb", tau, C, tau) + (tau * c).sum(-1)).sum(0)


def _mpc_solve_logged(sv, model_id, theta, x_init, C, c, u_init, bounds, unbounded, lqr_iter, eps, decay, max_ls,
                      not_improved_lim, best_cost_eps):
    """mpc_solve with verbose > 0: the same kernels, one iteration per call,
    the table row's reductions queued after each on the launch stream."""
    dev = x_init.device
    stats = torch.zeros(max(lqr_iter, 1), 3, device=dev)
    sv.begin(model_id, theta, x_init, u_init)
    x0, u0 = sv.gather_best()                               # slot 0: get_traj(u_init)
    initial = quad_traj_cost(x0, u0, C, c).mean()
    T, m, B = sv.T, sv.m, sv.B
    for i in range(lqr_iter):
        if sv.fixed_iters:
            sv.iterate_fixed(model_id, theta, x_init, C, c, bounds, decay, max_ls, i, best_cost_eps)
            fdn = quirk_norm(sv.du_sq[i * T:(i + 1) * T])
        else:
            sv.iterate(model_id, theta, x_init, C, c, bounds, decay, max_ls, i, best_cost_eps, eps, not_improved_lim)
            fdn = sv.full_du_norm
        stats[i, 0] = sv.best_cost.mean()
        stats[i, 1] = fdn.max()
        stats[i, 2] = sv.alpha.mean()
    if sv.fixed_iters:
        sv.finish_fixed(lqr_iter)
    # the iterations that ran: the rule after iteration k is applied by
    # iteration k+1's prologue, which then publishes iter = k+1 with the stop
    # flag (dilqr_fused.h mpc_decide); a solve that never stopped ran them all
    ran = sv.iterations
    # total_qp_iters: 0 without bounds, as the reference (pnqp runs only with
    # bounds, lqr_step_explicit.py:137-150); the fused kernels do not count the
    # batch-coupled pnqp iterations the reference reports with bounds
    sv.log = {"initial_mean_cost": initial, "stats": stats, "iterations": ran, "qp_iters": 0 if unbounded else None}


def lqr_adjoint(C, c, F, x, u, dl_dx, dl_du, u_lower=None, u_upper=None, m_solver=N.SOLVE_INV, want_df=True):
    """Classic adjoint (lqr_step.py:312-407) -> dx_init, dC, dc, dF, df."""
    T, B, n = x.shape
    m = u.shape[2]
    d = n + m
    C, c, F, x, u, dl_dx, dl_du = map(_f32, (C, c, F, x, u, dl_dx, dl_du))
    bounds, keep = N.make_bounds(u_lower, u_upper)
    dev = C.device
    ws = torch.empty(T * B * (m * n + m), device=dev)
    dx0 = torch.empty(B, n, device=dev)
    dC = torch.empty(T, B, d, d, device=dev)
    dc = torch.empty(T, B, d, device=dev)
    dF = torch.empty(max(T - 1, 0), B, n, d, device=dev)
    df = torch.empty(max(T - 1, 0), B, n, device=dev) if want_df else None
    N.call("dilqr_lqr_adjoint_f32", n, m, T, B, N.ptr(C), N.ptr(c), N.ptr(F), N.ptr(x), N.ptr(u), N.ptr(dl_dx),
           N.ptr(dl_du), bounds, m_solver, N.ptr(ws), N.ptr(dx0), N.ptr(dC), N.ptr(dc), N.ptr(dF), N.ptr(df),
           N.stream(dev))
    del keep
    return dx0, dC, dc, dF, df


def mpc_solve_unfused(model_id, theta, x_init, C, c, T, F=None, f=None, u_init=None, u_lower=None,
                      u_upper=None, lqr_iter=10, eps=1e-7, linesearch_decay=0.2, max_linesearch_iter=10,
                      not_improved_lim=5, best_cost_eps=1e-4, check_every=8, u_zero_I=None, verbose=0):
    """The same outer loop with the unfused kernels (linearise -> F in HBM ->
    Riccati -> rollout/line search).  Used for LinDx dynamics (classic mpc.MPC,
    the adjoint engines), MPC(u_zero_I=...) and to cross-check the fused
    iteration.  u_zero_I [T,B,m] (bool): controls held at zero — the sweep's
    masked solve when unconstrained (lqr_step_explicit.py:98-129; with bounds
    the reference's pnqp branch ignores the mask) and zeroed in every rollout
    before the clamp (199-200).

    The host polls the stop flag every `check_every` iterations: up to
    check_every - 1 iterations after the stop rule fired still run their
    linearise, sweep and line-search launches (these kernels carry no stop
    guard); their results are discarded by k_mpc_best, which leaves the best
    iterate, best_du and the control word as they were at the stop."""
    B, n = x_init.shape
    m = C.shape[-1] - n
    dev = x_init.device
    x_init, C, c, F, f = _f32(x_init), _f32(C), _f32(c), _f32(F), _f32(f)
    ws = MPCWorkspace(T, B, n, m, dev)
    if u_init is None:
        ws.ua.zero_()
    else:
        u0 = u_init.to(device=dev, dtype=torch.float32)
        if u0.ndimension() == 2:
            u0 = u0.unsqueeze(1).expand(T, B, m)
        ws.ua.copy_(u0)
    s = N.stream(dev)
    zI = zero_mask(u_zero_I, T, B, m, dev)
    N.call("dilqr_rollout_f32", model_id, n, m, T, B, N.ptr(theta), N.ptr(F), N.ptr(f), N.ptr(x_init),
           N.ptr(ws.ua), N.ptr(ws.xa), s)
    stats = None
    if verbose > 0:                        # the table rows, reduced on the stream (util.print_solve_log)
        stats = torch.zeros(max(lqr_iter, 1), 3, device=dev)
        initial = quad_traj_cost(ws.xa, ws.ua, C, c).mean()
    ran = 0
    for i in range(lqr_iter):
        if model_id == N.MODEL_LINDX:
            Fi, fi = F, f
        else:
            Fi, fi = linearize(model_id, theta, ws.xa, ws.ua)
        K, k, _ = lqr_backward(C, c, Fi, n, m, x=ws.xa, u=ws.ua, u_lower=u_lower, u_upper=u_upper,
                               u_zero_I=zI if u_lower is None else None)
        bounds, keep = N.make_bounds(u_lower, u_upper)
        # from iteration 1 the old cost is the previous line search's value for
        # the accepted candidate (ws.cost), as the fused MPC kernel takes it
        prev = (N.ptr(ws.cost) if i > 0 and model_id in (N.MODEL_PENDULUM, N.MODEL_CARTPOLE) else None)
        N.call("dilqr_lqr_forward_f32", model_id, n, m, T, B, N.ptr(theta), N.ptr(F), N.ptr(f),
               N.ptr(x_init), N.ptr(C), N.ptr(c), N.ptr(ws.xa), N.ptr(ws.ua), N.ptr(K), N.ptr(k), bounds, N.ptr(zI),
               float(linesearch_decay), int(max_linesearch_iter), N.ptr(ws.xb), N.ptr(ws.ub), N.ptr(ws.cost),
               N.ptr(ws.du_sq), N.ptr(ws.alpha), prev, s)
        N.call("dilqr_mpc_update_best_f32", n, m, T, B, int(i == 0), float(best_cost_eps), float(eps),
               int(min(not_improved_lim, 2 ** 31 - 1)), N.ptr(ws.xb), N.ptr(ws.ub), N.ptr(ws.cost),
               N.ptr(ws.du_sq), N.ptr(ws.fdn), N.ptr(ws.best_x), N.ptr(ws.best_u), N.ptr(ws.best_cost),
               N.ptr(ws.best_du), N.ptr(ws.ctrl), s)
        del keep
        if stats is not None:
            stats[i, 0] = ws.best_cost.mean()
            stats[i, 1] = ws.fdn.max()
            stats[i, 2] = ws.alpha.mean()
        ran = i + 1
        ws.xa, ws.xb = ws.xb, ws.xa
        ws.ua, ws.ub = ws.ub, ws.ua
        # once the stop rule fired, k_mpc_best ignores further iterations (the
        # best iterate, its cost, best_du and the control word stay as they
        # were), so the loop can run on past the stop: the host polls the flag
        # only every check_every iterations, like mpc_solve
        if check_every and (i + 1) % check_every == 0 and i + 1 < lqr_iter and int(ws.ctrl[1].item()):
            break
    if stats is not None:
        # k_mpc_control counts the iterations that ran (ctrl[0]) and stops counting
        # once the rule fired (ctrl[1])
        if int(ws.ctrl[1].item()):
            ran = min(ran, int(ws.ctrl[0].item()))
        ws.log = {"initial_mean_cost": initial, "stats": stats, "iterations": ran,
                  "qp_iters": 0 if u_lower is None else None}
    return ws
