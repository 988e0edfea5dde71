// tu_implicit_rocket.hip — the DiLQR implicit backward for rocket
// (16 lanes per problem, dilqr_implicit_group.h; rocket.py:263-323, 541-820).
#include "dilqr_common.h"
#include "dilqr_implicit_group.h"
#include "dilqr_launch.h"

namespace dilqr {

int implicit_rocket_ws_floats() { return ImplicitGroupWs<Rocket>::REC; }

int launch_implicit_rocket(const ImplicitArgs& a) {
  if (a.bd.mode == DILQR_BOUNDS_NONE)
    k_implicit_backward_group<Rocket, gen::RocketD2, GAIN_UNC><<<grid_group(a.B), 64, 0, a.stream>>>(
        a.T, a.B, a.theta, a.C, a.c, a.x, a.u, a.K, a.dl_dx, a.dl_du, a.bd, a.ws, a.dC, a.dc, a.dtheta);
  else
    k_implicit_backward_group<Rocket, gen::RocketD2, GAIN_ZERO_I><<<grid_group(a.B), 64, 0, a.stream>>>(
        a.T, a.B, a.theta, a.C, a.c, a.x, a.u, a.K, a.dl_dx, a.dl_du, a.bd, a.ws, a.dC, a.dc, a.dtheta);
  return launched();
}

}  // namespace dilqr
