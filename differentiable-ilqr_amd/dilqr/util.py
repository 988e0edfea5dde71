"""The reference's per-iteration progress table (util.py:80-101, table_log) and
the MPC classes' `verbose > 0` report (mpc_explicit.py:236-241, 285-295;
mpc.py:270-275, 368-379).

The solve records its per-iteration figures on the device (ops.mpc_solve,
`verbose > 0`: a few reductions queued on the launch stream after each
iteration, no host sync inside the loop); the table is printed once the solve
is done, one row per iteration the solve actually ran (the reference breaks out
of its loop after printing the row of the iteration whose stop rule fired).
"""

_seen_tables = set()


def table_log(tag, rows):
    """util.py:80-101: print the header the first time a table `tag` is seen,
    then one row.  `rows` is a sequence of (name, value) or (name, value, fmt)."""
    def line(cells):
        print("| " + " | ".join(cells) + " |")
    if tag not in _seen_tables:
        line([r[0] for r in rows])
        _seen_tables.add(tag)
    cells = []
    for r in rows:
        if len(r) not in (2, 3):
            raise ValueError("table_log: each entry is (name, value) or (name, value, fmt)")
        cells.append(r[2].format(r[1]) if len(r) == 3 else str(r[1]))
    line(cells)


def print_solve_log(log):
    """Print what ops.mpc_solve recorded with verbose > 0: the initial mean cost
    (mpc_explicit.py:236-241) and the 'lqr' table rows (285-295)."""
    print("Initial mean(cost): {:.4e}".format(float(log["initial_mean_cost"])))
    stats = log["stats"].cpu()
    qp = log.get("qp_iters")
    for i in range(int(log["iterations"])):
        table_log("lqr", (
            ("iter", i),
            ("mean(cost)", float(stats[i, 0]), "{:.4e}"),
            ("||full_du||_max", float(stats[i, 1]), "{:.2e}"),
            ("mean(alphas)", float(stats[i, 2]), "{:.2e}"),
            ("total_qp_iters", "-" if qp is None else int(qp)),
        ))
