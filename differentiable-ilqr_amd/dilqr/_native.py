"""ctypes binding of libdilqr.so (the C-ABI declared in include/dilqr.h).

This is the binding a maintainer of the reference would add:
torch tensors are passed as raw device pointers plus sizes, the current HIP
stream as a void*.  There is NO fallback: if the library is missing, or a tensor
is not on the GPU, every call raises.
"""
import ctypes
import glob
import hashlib
import os

import torch  # noqa: F401  (must be imported first: libdilqr.so then binds to torch's HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DILQR_LIB", os.path.join(_HERE, "libdilqr.so"))
ABI_VERSION = 9
_PKG = os.path.dirname(_HERE)          # differentiable-ilqr_amd/ (the Makefile's directory)

MODEL_LINDX, MODEL_PENDULUM, MODEL_CARTPOLE, MODEL_ROCKET, MODEL_PENDULUM_COMPLEX = 0, 1, 2, 3, 4
BOUNDS_NONE, BOUNDS_SCALAR, BOUNDS_TENSOR = 0, 1, 2
SOLVE_INV, SOLVE_CHOL = 0, 1
ERRORS = {1: "unsupported shape/model", 2: "invalid argument", 3: "unsupported option combination"}


class Bounds(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int), ("lo", ctypes.c_float), ("hi", ctypes.c_float),
                ("lo_t", ctypes.c_void_p), ("hi_t", ctypes.c_void_p)]


CTRL_INTS = 8          # sizeof(dilqr_mpc_ctrl) / 4


class MpcState(ctypes.Structure):
    """dilqr_mpc_state: device pointers of one MPC solve (include/dilqr.h)."""
    _fields_ = [(name, ctypes.c_void_p) for name in
                ("Xs", "Us", "slot", "best_cost", "best_du", "improved", "cost", "alpha", "du_sq",
                 "full_du_norm", "ws", "ctrl", "done_counter", "Cpk", "cost_sym", "best_iter")]

_vp, _i, _f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
SIGNATURES = {
    "dilqr_version": ([], _i),
    "dilqr_build_id": ([], ctypes.c_char_p),
    "dilqr_model_num_params": ([_i], _i),
    "dilqr_model_num_ctrl": ([_i], _i),
    "dilqr_dynamics_f32": ([_i, _i, _vp, _vp, _vp, _vp, _vp], _i),
    "dilqr_dynamics_vjp_f32": ([_i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], _i),
    "dilqr_linear_dyn_f32": ([_i, _i, _vp, _vp, _vp, _vp, _vp], _i),
    "dilqr_rollout_f32": ([_i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp], _i),
    "dilqr_linearize_f32": ([_i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp], _i),
    "dilqr_lqr_backward_f32": ([_i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, Bounds, _vp, _i, _vp, _vp, _vp,
                                _vp, _vp], _i),
    "dilqr_lqr_forward_f32": ([_i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, Bounds,
                               _vp, _f, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp], _i),
    "dilqr_pnqp_f32": ([_i, _i, _vp, _vp, Bounds, _vp, _vp, _vp, _vp, _vp, _vp], _i),
    "dilqr_quirk_norm_f32": ([_i, _i, _i, _vp, _vp, _vp], _i),
    "dilqr_ilqr_iterate_f32": ([_i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, Bounds, _f, _i, _vp, _vp, _vp, _vp,
                                _vp, _vp, _vp, _vp], _i),
    "dilqr_mpc_update_best_f32": ([_i, _i, _i, _i, _i, _f, _f, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _vp, _vp, _vp], _i),
    "dilqr_lqr_adjoint_f32": ([_i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, Bounds, _i, _vp, _vp, _vp,
                               _vp, _vp, _vp, _vp], _i),
    "dilqr_implicit_ws_floats": ([_i], _i),
    "dilqr_mpc_packed_cost_floats": ([_i, _i], _i),
    "dilqr_mpc_begin_f32": ([_i, _i, _i, _vp, _vp, _vp, MpcState, _vp], _i),
    "dilqr_mpc_iterate_f32": ([_i, _i, _i, _vp, _vp, _vp, _vp, Bounds, _f, _i, _i, _f, _f, _i, MpcState, _vp], _i),
    "dilqr_mpc_step_f32": ([_i, _i, _i, _vp, _vp, _vp, _vp, Bounds, _f, _i, _i, _f, _f, _i, MpcState, _vp], _i),
    "dilqr_mpc_iterate_range_f32": ([_i, _i, _i, _vp, _vp, _vp, _vp, Bounds, _f, _i, _i, _i, _f, _f, _i, MpcState,
                                     _vp], _i),
    "dilqr_mpc_stop_rule_f32": ([_i, _i, _i, _i, MpcState, _vp], _i),
    "dilqr_mpc_iterate_fixed_f32": ([_i, _i, _i, _vp, _vp, _vp, _vp, Bounds, _f, _i, _i, _f, MpcState, _vp], _i),
    "dilqr_mpc_finish_fixed_f32": ([_i, _i, _i, _i, MpcState, _vp], _i),
    "dilqr_mpc_solve_fixed_f32": ([_i, _i, _i, _vp, _vp, _vp, _vp, _vp, Bounds, _f, _i, _i, _f, MpcState, _vp],
                                  _i),
    "dilqr_mpc_solve_small_f32": ([_i, _i, _i, _vp, _vp, _vp, _vp, _vp, Bounds, _f, _i, _i, _f, _f, _i, MpcState,
                                   _vp], _i),
    "dilqr_mpc_gather_best_f32": ([_i, _i, _i, _i, MpcState, _vp, _vp, _vp], _i),
    "dilqr_get_matrices_f32": ([_i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], _i),
    "dilqr_grad_input_f32": ([_i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                              _vp], _i),
    "dilqr_implicit_backward_f32": ([_i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, Bounds, _vp, _vp, _vp,
                                     _vp, _vp], _i),
}

_lib = None


def tree_build_id():
    """The Makefile's BUILD_ID recomputed from the sources in this tree: sha256
    of csrc/*.hip, csrc/*.h and ../include/dilqr.h concatenated in byte-sorted
    path order, first 16 hex digits.  None when the sources are not present."""
    names = [os.path.relpath(f, _PKG) for f in glob.glob(os.path.join(_PKG, "csrc", "*.hip"))
             + glob.glob(os.path.join(_PKG, "csrc", "*.h"))]
    names.append(os.path.join("..", "include", "dilqr.h"))
    if not all(os.path.exists(os.path.join(_PKG, n)) for n in names) or len(names) < 2:
        return None
    h = hashlib.sha256()
    for n in sorted(names):
        with open(os.path.join(_PKG, n), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def lib():
    """Load libdilqr.so once; raise if it is missing (no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"dilqr: HIP library not found at {LIB_PATH}; build it with "
                "`python __graft_entry__.py` (or `make -C differentiable-ilqr_amd`). "
                "There is no CPU fallback.")
        handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (args, res) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.argtypes = args
            fn.restype = res
        v = handle.dilqr_version()
        if v != ABI_VERSION:
            raise RuntimeError(f"dilqr: library ABI {v} != expected {ABI_VERSION}")
        built = handle.dilqr_build_id().decode()
        tree = tree_build_id()
        if tree is not None and built != tree and not os.environ.get("DILQR_SKIP_BUILD_ID"):
            raise RuntimeError(
                f"dilqr: {LIB_PATH} was built from other sources (build id {built}, tree {tree}); "
                "rebuild it with `make -C differentiable-ilqr_amd`")
        _lib = handle
    return _lib


def exported_symbols():
    return list(SIGNATURES)


def check(rc, name):
    if rc != 0:
        what = ERRORS.get(rc, f"HIP error {-rc}" if rc < 0 else f"code {rc}")
        raise RuntimeError(f"dilqr: {name} failed: {what}")


def ptr(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("dilqr: tensor is not on the GPU (this library has no CPU path)")
    if t.dtype not in (torch.float32, torch.int32, torch.uint8):
        raise TypeError(f"dilqr: unsupported dtype {t.dtype}")
    if not t.is_contiguous():
        raise ValueError("dilqr: tensors must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


def stream(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def make_bounds(lo, hi):
    """MPC's u_lower/u_upper: None, python floats, or [T,B,m] device tensors."""
    if lo is None:
        return Bounds(BOUNDS_NONE, 0.0, 0.0, None, None), ()
    if isinstance(lo, (int, float)) and isinstance(hi, (int, float)):
        return Bounds(BOUNDS_SCALAR, float(lo), float(hi), None, None), ()
    lo_t = lo.contiguous().float()
    hi_t = hi.contiguous().float()
    return Bounds(BOUNDS_TENSOR, 0.0, 0.0, ptr(lo_t).value, ptr(hi_t).value), (lo_t, hi_t)


def call(name, *args):
    check(getattr(lib(), name)(*args), name)
