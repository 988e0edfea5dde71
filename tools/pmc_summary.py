#!/usr/bin/env python3
"""Summarise the PMC passes of tools/profile_pmc.sh into profiles/<round>/pmc_summary.json
and profiles/pmc_traffic.json (read by bench.py for roofline.traffic).

HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB counters).  The factor 2:
on gfx950 FETCH_SIZE reports half the bytes of wide streaming reads
(MI355X_MICROARCH.md §HBM); calibrated here on k_lqr_backward<5,1,UNC>, whose
reads are known exactly (C, c_back, F = 7,080 B/problem): FETCH_SIZE*1024/reads = 0.50."""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    for key in ("k_mpc_iterate", "k_ilqr_iterate", "k_lqr_backward", "k_mpc_norm_control", "k_implicit_backward",
                "k_lqr_forward", "k_lqr_adjoint"):
        if key in name:
            return key + ("<box>" if "Li3EE" in name else "")
    return None


def main(pmc_dir, round_tag):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in sorted(os.listdir(pmc_dir)):
        f = os.path.join(pmc_dir, p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in agg.items():
        out[k] = {c: sorted(v)[len(v) // 2] for c, v in cs.items()}   # median launch
        if "FETCH_SIZE" in out[k] and "WRITE_SIZE" in out[k]:
            out[k]["hbm_bytes_per_launch"] = (2 * out[k]["FETCH_SIZE"] + out[k]["WRITE_SIZE"]) * 1024
    os.makedirs(os.path.join(ROOT, "profiles", round_tag), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "profiles", round_tag, "pmc_summary.json"), "w"), indent=1)
    t = {"note": "HBM bytes per launch = (2*FETCH_SIZE + WRITE_SIZE)*1024 from rocprofv3 --pmc, "
                 f"profiles/{round_tag}/pmc_summary.json; cartpole T=25 B=65536"}
    for k in ("k_ilqr_iterate", "k_mpc_iterate", "k_lqr_backward"):
        if k in out and "hbm_bytes_per_launch" in out[k]:
            t[k + "_bytes_per_launch"] = out[k]["hbm_bytes_per_launch"]
    json.dump(t, open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(t, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc"),
         sys.argv[2] if len(sys.argv) > 2 else "r01")
