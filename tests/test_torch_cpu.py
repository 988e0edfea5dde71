"""The CPU baseline's restatement (oracle/torch_cpu.py, fp32 torch with the
reference's op structure) pinned to the reference's own fp32 output: the
cart_unc MPC golden (tests/golden/gen_golden.py case E, fp32, B=64) — costs to
1e-5 relative (measured 2.6e-7), controls and states to 2e-4 of their max
magnitude (measured: |du| 3.1e-3 on one of the 64 problems, whose controls
reach ~36; the cartpole problems are chaotic, so summation-order differences
grow)."""
import numpy as np
import torch

from oracle import torch_cpu as tc


def test_torch_cpu_restatement_matches_reference_f32(golden):
    g = golden("mpc_f32")
    x0 = g["cart_unc_x0"]
    B, T = x0.shape[0], 25
    q = torch.tensor([0.1, 0.1, 1., 1., 0.1, 0.001])
    p = torch.tensor([0., 0., -1., 0., 0., 0.])
    C = torch.diag(q).expand(T, B, 6, 6).contiguous()
    c = p.expand(T, B, 6).contiguous()
    with torch.no_grad():
        x, u, cost = tc.mpc_forward(torch.tensor(x0, dtype=torch.float32), C, c, T, 10)
    ref = g["cart_unc_costs"]
    cerr = np.abs(cost.numpy() - ref) / np.maximum(1.0, np.abs(ref))
    print(f"restatement vs reference fp32: max rel cost err {cerr.max():.2e}, "
          f"max |du| {np.abs(u.numpy() - g['cart_unc_u']).max():.2e}")
    assert cerr.max() < 1e-5
    rel = lambda a, b: np.abs(a - b).max() / max(1.0, np.abs(b).max())  # noqa: E731
    print(f"controls {rel(u.numpy(), g['cart_unc_u']):.2e}, states {rel(x.numpy(), g['cart_unc_x']):.2e}")
    assert rel(u.numpy(), g["cart_unc_u"]) < 2e-4
    assert rel(x.numpy(), g["cart_unc_x"]) < 2e-4


def test_torch_cpu_jacobian_is_the_derivative():
    """cartpole_jacobian equals autograd of cartpole_forward at the unclamped u."""
    rng = np.random.RandomState(4)
    th = rng.uniform(-np.pi, np.pi, 8)
    x = torch.tensor(np.stack([rng.uniform(-1, 1, 8), rng.uniform(-1, 1, 8), np.cos(th), np.sin(th),
                               rng.uniform(-1, 1, 8)], 1), dtype=torch.float64)
    u = torch.tensor(rng.uniform(-5, 5, (8, 1)), dtype=torch.float64)
    D = tc.cartpole_jacobian(x, u)
    J = torch.autograd.functional.jacobian(lambda xu: tc.cartpole_forward(xu[:, :5], xu[:, 5:]),
                                           torch.cat((x, u), 1))
    Jd = torch.stack([J[i, :, i, :] for i in range(8)])
    assert torch.allclose(D, Jd, atol=1e-10)
