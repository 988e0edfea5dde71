"""The IL loop counterpart (SURVEY.md §8 f #1-2): dataset I/O without
unpickling, IL_Env.mpc / populate_data, and the sysid / empc training steps."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

CART_PKL = os.path.join(GOLDEN, "cartpole_dataset.pkl")      # the reference's data/cartpole.pkl
PEND_PKL = os.path.join(GOLDEN, "pendulum_dataset.pkl")      # the reference's data/pendulum.pkl


@pytest.mark.parametrize("env,path", [("cartpole", CART_PKL), ("pendulum", PEND_PKL)])
def test_dataset_loader_matches_golden(golden, env, path):
    """load_il_dataset walks the pickle opcodes (nothing is unpickled) and
    returns the same arrays the golden generator extracted."""
    from dilqr import il
    d = il.load_il_dataset(path)
    g = golden("datasets")
    assert d["env"] == env
    for k in ("train_data", "val_data", "test_data", "params"):
        np.testing.assert_array_equal(d[k].numpy(), g[f"{env}_{k}"].astype(np.float32))
    for k in ("lqr_iter", "mpc_T", "linesearch_decay", "max_linesearch_iter", "mpc_eps", "lower", "upper"):
        assert float(d[k]) == float(g[f"{env}_{k}"]), k


@pytest.mark.gpu
def test_il_env_reproduces_dataset():
    """IL_Env.mpc from the dataset's own initial states reproduces the expert
    controls of data/cartpole.pkl (T=35, lqr_iter=100, eps=1e-4, bounds 100)."""
    from dilqr import il
    env = il.IL_Env.from_dataset(CART_PKL, device="cuda")
    data = torch.cat([env.train_data, env.val_data, env.test_data]).cuda()
    n = env.true_dx.n_state
    q, p = env.true_dx.get_true_obj()
    with torch.no_grad():
        x, u = env.mpc(env.true_dx, data[:, 0, :n].contiguous(), q.cuda(), p.cuda())
    ref_u = data[:, :, n:].transpose(0, 1)
    err = (u - ref_u).abs().max() / ref_u.abs().max()
    print(f"\n[il dataset] max |u - expert| / max |expert| {float(err):.2e}")
    assert float(err) < 1e-4, float(err)


@pytest.mark.gpu
def test_dynamics_vjp_vs_finite_differences():
    """Autograd through HipDynamics.forward (dilqr_dynamics_vjp_f32) vs central
    differences of the fp64 oracle model, incl. rows with a clamped control."""
    from dilqr.env_dx.cartpole import CartpoleDx
    from oracle import models as om
    rng = np.random.RandomState(0)
    N = 64
    th = rng.uniform(-np.pi, np.pi, N)
    x = np.stack([rng.normal(size=N), rng.normal(size=N), np.cos(th), np.sin(th), rng.normal(size=N)], 1)
    u = rng.uniform(-150, 150, (N, 1))                   # some beyond the +-100 clamp
    w = rng.normal(size=(N, 5))
    params = torch.tensor((9.8, 1.0, 0.1, 0.5), device="cuda", requires_grad=True)
    xt = torch.tensor(x, dtype=torch.float32, device="cuda", requires_grad=True)
    ut = torch.tensor(u, dtype=torch.float32, device="cuda", requires_grad=True)
    loss = (CartpoleDx(params)(xt, ut) * torch.tensor(w, dtype=torch.float32, device="cuda")).sum()
    loss.backward()
    p0 = np.array((9.8, 1.0, 0.1, 0.5))

    def L(pp, xx, uu):
        return float((om.Cartpole.forward(xx, uu, pp) * w).sum())
    eps = 1e-6
    g_fd = np.array([(L(p0 + eps * e, x, u) - L(p0 - eps * e, x, u)) / (2 * eps) for e in np.eye(4)])
    assert np.allclose(params.grad.cpu().numpy(), g_fd, rtol=2e-3, atol=1e-3)
    gu_fd = np.array([(L(p0, x, u + eps * np.eye(1)[0]) - L(p0, x, u - eps * np.eye(1)[0])) / (2 * eps)])
    assert abs(float(ut.grad.sum()) - gu_fd[0]) < 1e-2 * max(1.0, abs(gu_fd[0]))
    assert float(ut.grad[np.abs(u[:, 0]) > 100].abs().max()) == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("mode,kw", [("sysid", {}), ("empc", {"learn_dx": True}), ("empc", {"learn_cost": True})])
def test_il_trainer_runs_and_learns(mode, kw):
    """A few epochs of the reference's training loop on data/pendulum.pkl
    (20 training trajectories): finite losses, the learned parameters move, the
    sysid loss falls."""
    from dilqr import il
    env = il.IL_Env.from_dataset(PEND_PKL, device="cuda")
    env.lqr_iter = 30
    tr = il.ILTrainer(env, mode=mode, n_batch=10, n_train=20, **kw)
    h = tr.fit(6)
    train = np.array(h["train"])
    assert np.isfinite(train).all() and np.isfinite(np.array(h["val_test"])).all() and len(h["val_test"]) == 6
    if kw.get("learn_cost"):
        assert np.abs(h["cost"][-1] - h["cost"][0]).max() > 0
    else:
        assert np.abs(h["params"][-1] - h["params"][0]).max() > 1e-3
    if mode == "sysid":
        assert train[-2:, 2].mean() < train[:2, 2].mean()


def test_il_golden_records_reference_behaviour(golden):
    """The generator ran the reference's IL_Exp.run for sysid and for both empc
    variants (empc through the SURVEY.md §8(c) recipe: the closing
    linearisation on the detached best iterate, which avoids torch 2.10's
    leaf-variable error without changing any gradient that reaches the
    parameters; gen_golden.py case_il)."""
    g = golden("il")
    assert "pend_sysid_train" in g and "pend_sysid_dx_hist" in g
    for k in ("pend_empc_dx_train", "pend_empc_dx_val_test", "pend_empc_dx_dx_hist", "pend_empc_cost_train",
              "pend_empc_cost_val_test", "pend_empc_cost_cost_hist", "cart_empc_dx_train", "cart_empc_dx_val_test",
              "cart_empc_dx_dx_hist"):
        assert k in g and np.isfinite(g[k]).all(), k
    assert not any(k.endswith("_error") for k in g)


# case: (dataset, lqr_iter override, n_batch, n_train, n_epoch) — gen_golden.py IL_CASES
EMPC_CASES = {"pend_empc_dx": (PEND_PKL, 30, 5, 10, 2), "pend_empc_cost": (PEND_PKL, 30, 5, 10, 2),
              "cart_empc_dx": (CART_PKL, None, 2, 2, 4)}


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(EMPC_CASES))
def test_il_empc_matches_reference_curve(golden, case):
    """ILTrainer(mode='empc') reproduces the reference IL_Exp.run's
    train_losses.csv (im_loss through the MPC + the DiLQR implicit backward),
    val_test_losses.csv and dx_hist.csv / cost_hist.csv: the parameter steps
    are RMSprop steps on the implicit gradients, so the histories pin dtheta
    (learn_dx) and dC, dc through q, p (learn_cost) end to end.  On
    data/pendulum.pkl: n_train=10, n_batch=5, 2 epochs, lqr_iter 30, seed 5.
    On data/cartpole.pkl (the north-star model, T=35, lqr_iter 100 from the
    dataset, bounds +-100): its 2 training trajectories, n_batch=2, 4 epochs."""
    from dilqr import il
    g = golden("il")
    path, lqr_iter, n_batch, n_train, n_epoch = EMPC_CASES[case]
    env = il.IL_Env.from_dataset(path, device="cuda")
    if lqr_iter:
        env.lqr_iter = lqr_iter
    kw = {"learn_cost": True} if case.endswith("_cost") else {"learn_dx": True}
    tr = il.ILTrainer(env, mode="empc", n_batch=n_batch, n_train=n_train, seed=5, **kw)
    h = tr.fit(n_epoch)
    train = np.array(h["train"])
    ref = g[f"{case}_train"]
    print(f"{case}: train {train.tolist()}\n  ref {ref.tolist()}")
    assert train.shape == ref.shape
    np.testing.assert_allclose(train[:, 0], ref[:, 0])
    np.testing.assert_allclose(train[:, 1:], ref[:, 1:], rtol=2e-3, atol=1e-5)
    if "learn_dx" in kw:
        hist, ghist = np.array(h["params"]), g[f"{case}_dx_hist"][1:]
    else:
        hist, ghist = np.array(h["cost"]), g[f"{case}_cost_hist"][1:]
    print(f"  hist {hist.tolist()}\n  ref {ghist.tolist()}")
    np.testing.assert_allclose(hist, ghist, rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(np.array(h["val_test"]), g[f"{case}_val_test"], rtol=2e-3, atol=1e-5)


@pytest.mark.gpu
def test_il_sysid_matches_reference_curve(golden):
    """ILTrainer(mode='sysid') on data/pendulum.pkl (n_train=10, n_batch=5, 3
    epochs, seed 5) reproduces the reference IL_Exp.run's train_losses.csv
    (im_loss through the MPC, sysid_loss through the dynamics' gradient),
    val_test_losses.csv and dx_hist.csv."""
    from dilqr import il
    g = golden("il")
    env = il.IL_Env.from_dataset(PEND_PKL, device="cuda")
    tr = il.ILTrainer(env, mode="sysid", n_batch=5, n_train=10, seed=5)
    h = tr.fit(3)
    train = np.array(h["train"])
    ref = g["pend_sysid_train"]
    assert train.shape == ref.shape
    np.testing.assert_allclose(train[:, 0], ref[:, 0])
    np.testing.assert_allclose(train[:, 2], ref[:, 2], rtol=1e-3)            # sysid loss
    np.testing.assert_allclose(train[:, 1], ref[:, 1], rtol=2e-3, atol=1e-5)  # im loss (MPC solutions)
    np.testing.assert_allclose(np.array(h["params"]), g["pend_sysid_dx_hist"][1:], rtol=1e-4)
    vt = np.array(h["val_test"])
    np.testing.assert_allclose(vt, g["pend_sysid_val_test"], rtol=2e-3, atol=1e-5)
