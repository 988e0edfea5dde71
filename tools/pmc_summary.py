#!/usr/bin/env python3
"""Summarise the PMC passes of tools/profile_pmc.sh into profiles/<round>/pmc_summary.json
and profiles/pmc_traffic.json (read by bench.py for roofline.traffic).

Fabric bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB counters).  The
factors are calibrated, per access pattern, by tools/microbench/fetch_calib.hip
(tools/fetch_calib.sh; profiles/r02/pmc_calibration.json): FETCH_SIZE = 0.50 x
bytes for 4-B/lane coalesced, 16-B/lane coalesced and 144-B-record-per-lane
reads, WRITE_SIZE = 1.00 x bytes for 4-B and 16-B/lane stores — the patterns of
the hot kernels (the MPC slots' component planes, the float4 planes, the
caller's C records).  The counters sit on the L2's memory side, so MALL
(Infinity Cache) hits are included: the figure is L2-miss traffic, an upper
bound on HBM traffic.  Raw counters are kept next to the corrected figure."""
import subprocess
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
            if key == "k_mpc_iterate" and name.split("(")[0].rstrip().endswith("true>"):
                key += "<first>"                      # iteration 0's own instantiation (FIRST = true)
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
            out[k]["fetch_bytes_raw"] = out[k]["FETCH_SIZE"] * 1024
            out[k]["write_bytes_raw"] = out[k]["WRITE_SIZE"] * 1024
            out[k]["hbm_bytes_per_launch"] = (2 * out[k]["FETCH_SIZE"] + out[k]["WRITE_SIZE"]) * 1024
    os.makedirs(os.path.join(ROOT, "profiles", round_tag), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "profiles", round_tag, "pmc_summary.json"), "w"), indent=1)
    try:
        head = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                              text=True).stdout.strip()
    except OSError:
        head = "?"
    t = {"note": "L2-miss (fabric) bytes per launch = (2*FETCH_SIZE + WRITE_SIZE)*1024 from rocprofv3 --pmc "
                 "(factors calibrated per access pattern: profiles/r02/pmc_calibration.json), "
                 f"profiles/{round_tag}/pmc_summary.json; cartpole T=25 B=65536",
         "measured_at_commit": head}
    for k in ("k_ilqr_iterate", "k_mpc_iterate", "k_lqr_backward"):
        if k in out and "hbm_bytes_per_launch" in out[k]:
            t[k + "_bytes_per_launch"] = out[k]["hbm_bytes_per_launch"]
            t[k + "_raw"] = {"FETCH_SIZE_KiB": out[k]["FETCH_SIZE"], "WRITE_SIZE_KiB": out[k]["WRITE_SIZE"]}
            if "SQ_WAVE_CYCLES" in out[k] and "SQ_ACTIVE_INST_VALU" in out[k]:
                w = out[k]["SQ_WAVE_CYCLES"]
                t[k + "_issue"] = {"valu_busy": out[k]["SQ_ACTIVE_INST_VALU"] / w,
                                   "waitcnt_stall": out[k].get("SQ_WAIT_ANY", 0.0) / w,
                                   "valu_instr_per_wave": out[k]["SQ_INSTS_VALU"] / out[k]["SQ_WAVES"]}
    json.dump(t, open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(t, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc"),
         sys.argv[2] if len(sys.argv) > 2 else "r02")
