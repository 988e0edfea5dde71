"""Multi-process (world_size 2, gloo, CPU) coverage of the batch-sharded path
that bench.py runs on N GPUs: shard boundaries, the per-shard problem set, the
max-over-ranks timing reduction, that solving each shard independently gives
the same per-problem result as solving the whole batch for fixed-count solves
(so no collective is needed in the data path), and what a sharded stop-rule
(eps > 0) solve returns: one reference call per shard.  The
per-shard solver here is the CPU oracle; on the GPU box the same shards go
through the HIP library."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, B_per, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from oracle import models as om
    from oracle import mpc as ompc
    B_total = B_per * world
    x0_all, q, p = bench.make_problems(B_total)
    lo, hi = bench.shard_rows(B_total, world, rank)
    assert hi - lo == B_per
    x0 = x0_all[lo:hi].astype(np.float64)
    T = 6
    C, c = ompc.expand_cost(np.diag(q).astype(np.float64), p.astype(np.float64), T, B_per)
    _, u, costs, _ = ompc.mpc_forward(om.Cartpole, x0, C, c, T, lqr_iter=3, eps=0.0, not_improved_lim=10 ** 9,
                                      linesearch_decay=0.5, max_linesearch_iter=2)
    np.save(os.path.join(out_dir, f"u_{rank}.npy"), u)
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    assert t.item() == float(world)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_solve_matches_whole_batch(tmp_path):
    world, B_per = 2, 8
    port = _free_port()
    mp.spawn(_worker, args=(world, port, B_per, str(tmp_path)), nprocs=world, join=True)
    import bench
    from oracle import models as om
    from oracle import mpc as ompc
    x0_all, q, p = bench.make_problems(B_per * world)
    T = 6
    C, c = ompc.expand_cost(np.diag(q).astype(np.float64), p.astype(np.float64), T, B_per * world)
    _, u_all, _, _ = ompc.mpc_forward(om.Cartpole, x0_all.astype(np.float64), C, c, T, lqr_iter=3, eps=0.0,
                                      not_improved_lim=10 ** 9, linesearch_decay=0.5, max_linesearch_iter=2)
    u_sharded = np.concatenate([np.load(tmp_path / f"u_{r}.npy") for r in range(world)], axis=1)
    np.testing.assert_allclose(u_sharded, u_all, rtol=0, atol=1e-12)


STOP_CASE = dict(T=8, B_per=8, seed=3, lqr_iter=40, eps=1e-2, not_improved_lim=5)


def _stop_rule_solve(x0, T, lqr_iter, eps, not_improved_lim, q, p):
    from oracle import models as om
    from oracle import mpc as ompc
    C, c = ompc.expand_cost(np.diag(q).astype(np.float64), p.astype(np.float64), T, x0.shape[0])
    _, u, costs, info = ompc.mpc_forward(om.Cartpole, x0.astype(np.float64), C, c, T, lqr_iter=lqr_iter, eps=eps,
                                         not_improved_lim=not_improved_lim, linesearch_decay=0.5,
                                         max_linesearch_iter=2)
    return u, costs, info["full_du_norm"], info["n_iters"]


def _stop_rule_worker(rank, world, port, out_dir):
    """One rank of a sharded eps > 0 solve: the rank's MPC call over its own
    contiguous shard, nothing exchanged but the iteration counts (reported)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    k = STOP_CASE
    B_total = k["B_per"] * world
    x0_all, q, p = bench.make_problems(B_total, seed=k["seed"])
    lo, hi = bench.shard_rows(B_total, world, rank)
    u, costs, du, iters = _stop_rule_solve(x0_all[lo:hi], k["T"], k["lqr_iter"], k["eps"],
                                           k["not_improved_lim"], q, p)
    np.savez(os.path.join(out_dir, f"stop_{rank}.npz"), u=u, costs=costs, du=du)
    its = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(its, torch.tensor([iters]))
    if rank == 0:
        np.save(os.path.join(out_dir, "stop_iters.npy"), np.array([int(t.item()) for t in its]))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_stop_rule_is_per_shard(tmp_path):
    """an eps > 0 solve sharded over N ranks is N independent
    reference MPC calls, one per shard.  The stop rule (mpc_explicit.py:297-299:
    max full_du_norm < eps or n_not_improved > lim) and the batch-mixing
    full_du_norm rows (lqr_step_explicit.py:245-247) are evaluated per call, so
    they are per shard: rank r returns exactly the reference's result for its
    shard alone, which differs from the whole-batch call wherever the shard's
    stop fires at another iteration than the whole batch's.  No collective is
    in the data path."""
    world = 2
    k = STOP_CASE
    mp.spawn(_stop_rule_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    import bench
    B_total = k["B_per"] * world
    x0_all, q, p = bench.make_problems(B_total, seed=k["seed"])
    args = (k["T"], k["lqr_iter"], k["eps"], k["not_improved_lim"], q, p)
    iters = np.load(tmp_path / "stop_iters.npy")
    per_shard = []
    for r in range(world):
        lo, hi = bench.shard_rows(B_total, world, r)
        got = np.load(tmp_path / f"stop_{r}.npz")
        want = _stop_rule_solve(x0_all[lo:hi], *args)
        for a, b in zip((got["u"], got["costs"], got["du"]), want[:3]):
            np.testing.assert_array_equal(a, b)          # the rank's result = the call on its shard alone
        assert iters[r] == want[3]
        per_shard.append(got)
    u_w, c_w, du_w, it_w = _stop_rule_solve(x0_all, *args)
    # this case pins the difference: shard 0 stops with the whole batch (8
    # iterations), shard 1 one iteration earlier (7)
    assert list(iters) == [8, 7] and it_w == 8
    lo, hi = bench.shard_rows(B_total, world, 0)
    np.testing.assert_array_equal(per_shard[0]["u"], u_w[:, lo:hi])   # same iterations: same iterates
    np.testing.assert_array_equal(per_shard[0]["costs"], c_w[lo:hi])
    lo, hi = bench.shard_rows(B_total, world, 1)
    assert np.abs(per_shard[1]["u"] - u_w[:, lo:hi]).max() > 1e-3    # stopped earlier: a different iterate
    # best_du is a quirk row of the call's own [T, m, B] buffer: per shard
    assert not np.array_equal(np.concatenate([s["du"] for s in per_shard]), du_w)


def _rank_record_worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["LOCAL_RANK"] = str(rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import json
    import types
    import bench
    fake = lambda dev: types.SimpleNamespace(  # noqa: E731  (a device per rank, as the driver's N-GPU node)
        name="AMD Instinct MI355X", gcnArchName="gfx950:sramecc+:xnack-", pci_domain_id=0, pci_bus_id=0x10 + rank,
        pci_device_id=0, uuid=f"GPU-{rank:04d}")
    lo, hi = bench.shard_rows(64 * world, world, rank)
    rec = bench.rank_records(dist, f"cuda:{rank}", 0.5 + rank, lo, hi, props=fake)
    if rank == 0:
        with open(os.path.join(out_dir, "ranks.json"), "w") as f:
            json.dump(rec, f)
    dist.barrier()
    dist.destroy_process_group()


def test_rank_records_gloo_world2(tmp_path):
    """bench.py's self-verifying N > 1 record (outside the timed region): the
    process group's world size, one entry per rank with its device, PCI
    location, shard rows and own elapsed time, and the min/max spread."""
    import json
    world = 2
    mp.spawn(_rank_record_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    rec = json.load(open(tmp_path / "ranks.json"))
    assert rec["world_size"] == world and rec["backend"] == "gloo" and rec["distinct_devices"] == world
    assert [r["rank"] for r in rec["per_rank"]] == [0, 1]
    assert [r["pci"] for r in rec["per_rank"]] == ["0000:10:00", "0000:11:00"]
    assert rec["rows_cover"] and rec["per_rank"][1]["rows"] == [64, 128]
    assert rec["elapsed_min_s"] == 0.5 and rec["elapsed_max_s"] == 1.5
    assert rec["spread"] == pytest.approx(1.0 / 1.5)


def test_shard_rows_cover_batch():
    import bench
    for world in (1, 2, 4, 8):
        rows = [bench.shard_rows(65536 * world, world, r) for r in range(world)]
        assert rows[0][0] == 0 and rows[-1][1] == 65536 * world
        assert all(a[1] == b[0] for a, b in zip(rows, rows[1:]))


@pytest.mark.gpu
def test_bench_sharded_hip_path_equals_whole_batch(tmp_path):
    """bench.py's N > 1 path on the HIP library: two ranks (torchrun, gloo for the
    timing reduction, both on cuda:0) each solve their contiguous shard of the
    generated batch; the shards' best trajectories and costs equal, bit for bit,
    the whole-batch solve of the same problems (problems are independent, so no
    collective is needed in the data path)."""
    import subprocess
    import sys
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    world, B_per, it = 2, 1024, 10
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", str(world), "--batch", str(B_per), "--steps", "2", "--warmup", "0", "--lqr-iter", str(it),
           "--no-secondary", "--no-cpu-baseline", "--dump", str(tmp_path)]
    r = subprocess.run(cmd, env=env, cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    import json
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    rk = line["ranks"]                      # the self-verifying record (both ranks share cuda:0 here)
    assert line["n_gpus"] == world and rk["world_size"] == world and rk["backend"] == "gloo"
    assert [p["rank"] for p in rk["per_rank"]] == list(range(world)) and rk["distinct_devices"] == 1
    assert rk["rows_cover"] and rk["per_rank"][-1]["rows"][1] == B_per * world
    assert rk["elapsed_max_s"] == pytest.approx(line["ms_per_step"] * line["steps"] / 1e3, rel=1e-9)
    assert all(p["gcn_arch"].startswith("gfx950") and p["pci"] for p in rk["per_rank"])
    import bench
    from dilqr import ops
    from dilqr import _native as N
    x0_all, q, p = bench.make_problems(B_per * world)
    dev = torch.device("cuda:0")
    T, B = bench.T_HORIZON, B_per * world
    x0 = torch.tensor(x0_all, device=dev)
    C = torch.diag(torch.tensor(q)).repeat(T, B, 1, 1).to(dev).contiguous()
    c = torch.tensor(p).repeat(T, B, 1).to(dev).contiguous()
    theta = torch.tensor([9.8, 1.0, 0.1, 0.5], device=dev)
    x, u, cost, _, _ = ops.mpc_solve(N.MODEL_CARTPOLE, theta, x0, C, c, T, lqr_iter=it, eps=0.0,
                                     linesearch_decay=0.5, max_linesearch_iter=2, not_improved_lim=10 ** 9)
    for rank in range(world):
        sh = torch.load(tmp_path / f"shard{rank}.pt", weights_only=True)
        lo, hi = sh["rows"]
        assert (lo, hi) == bench.shard_rows(B, world, rank)
        assert torch.equal(sh["u"], u[:, lo:hi].cpu()) and torch.equal(sh["x"], x[:, lo:hi].cpu())
        assert torch.equal(sh["cost"], cost[lo:hi].cpu())


@pytest.mark.gpu
def test_bench_rccl_path_runs(tmp_path):
    """bench.py's RCCL branch — init_process_group("nccl"), the barriers around
    the timed region and the max-over-ranks timing all-reduce on the device —
    under torchrun with one rank on cuda:0 (one GPU per rank: a second rank
    would need a second GPU), and its JSON line is well formed."""
    import json
    import subprocess
    import sys
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "1", "--batch", "4096", "--steps", "3", "--warmup", "1", "--no-secondary", "--no-cpu-baseline"]
    env = dict(os.environ)
    env.pop("BENCH_DIST_BACKEND", None)
    r = subprocess.run(cmd, env=env, cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["value"] > 0 and line["config"]["global_batch"] == 4096
    rk = line["ranks"]
    assert rk["world_size"] == 1 and rk["backend"] == "nccl" and rk["distinct_devices"] == 1
    assert rk["per_rank"][0]["rows"] == [0, 4096] and rk["per_rank"][0]["gcn_arch"].startswith("gfx950")
    assert rk["elapsed_min_s"] == rk["elapsed_max_s"] > 0
