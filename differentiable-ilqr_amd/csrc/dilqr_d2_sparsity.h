// dilqr_d2_sparsity.h — the structural zeros of the generated second-order
// pieces (dilqr_models_gen.h, tools/gen_model_derivs.py): the entries of
// lag_hess (d x d), lag_dparam (d x p) and f_theta_cs (n x p) the generated
// code writes as a literal 0.0f.  The implicit backward skips the products with
// them at compile time, as the sweeps skip the Jacobian's structural zeros
// (Model::FSparsity): an exact zero term changes no nonzero sum.  Plain
// constexpr C++ (host and device), so tests/test_models_gen.py checks these
// tables against the generated functions on the host.
#pragma once

namespace dilqr {
namespace gen {

struct PendulumD2Z {                 // every entry is a function of the state
  static constexpr bool hess_nz(int, int) { return true; }
  static constexpr bool dparam_nz(int, int) { return true; }
  static constexpr bool ftheta_nz(int, int) { return true; }
};

struct CartpoleD2Z {
  // second derivatives only in (cos, sin, dth, u) = 2..5, and none of u with
  // sin, dth, u (cartpole.py:64-97: u enters x' and dth' through cart_in)
  static constexpr bool hess_nz(int i, int j) { return i >= 2 && j >= 2 && !(i == 5 && j >= 3) && !(j == 5 && i >= 3); }
  static constexpr bool dparam_nz(int i, int k) { return i >= 2 && !(i >= 4 && k == 0); }
  static constexpr bool ftheta_nz(int i, int) { return i == 1 || i == 4; }
};

}  // namespace gen
}  // namespace dilqr
