#!/usr/bin/env python3
"""Summarise the PMC passes of tools/profile_pmc.sh into
profiles/<round>/pmc_summary.json (every kernel instantiation seen, median
launch per counter) and profiles/pmc_traffic.json (read by bench.py for each
roofline's `traffic`).

HBM-side bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB counters).  On
gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads
(MI355X_MICROARCH.md, HBM section); tools/microbench/fetch_calib.hip measured
the same 0.50 for the 4-B/lane, 16-B/lane and 144-B-record-per-lane reads of
these kernels and WRITE_SIZE = 1.00 x bytes for their stores
(profiles/r02/pmc_calibration.json).  The counters sit on the L2's memory side,
so Infinity-Cache hits count: an upper bound on HBM traffic.  SQ_* cycle
counters are quad-cycles per wave; ratios to SQ_WAVE_CYCLES are fractions of
wave lifetime."""
import collections
import csv
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def signature(name):
    """'void dilqr::k_mpc_iterate<dilqr::Cartpole, 0, true, false>(int, ...)' ->
    'k_mpc_iterate<Cartpole, 0, true, false>' (one key per instantiation)."""
    head = name.split("(")[0].strip()
    head = re.sub(r"^void\s+", "", head).replace("dilqr::gen::", "").replace("dilqr::", "")
    return head


def derived(c):
    out = {}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        out["fetch_bytes_raw"] = c["FETCH_SIZE"] * 1024
        out["write_bytes_raw"] = c["WRITE_SIZE"] * 1024
        out["hbm_bytes_per_launch"] = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
    w = c.get("SQ_WAVE_CYCLES")
    if w:
        for k, name in (("SQ_ACTIVE_INST_VALU", "valu_busy"), ("SQ_WAIT_ANY", "waitcnt_stall"),
                        ("SQ_WAIT_INST_ANY", "issue_stall"), ("SQ_ACTIVE_INST_VMEM", "vmem_busy"),
                        ("SQ_ACTIVE_INST_LDS", "lds_busy")):
            if k in c:
                out[name] = c[k] / w
    if c.get("SQ_WAVES"):
        for k, name in (("SQ_INSTS_VALU", "valu_instr_per_wave"), ("SQ_INSTS_LDS", "lds_instr_per_wave"),
                        ("SQ_INSTS_SALU", "salu_instr_per_wave"), ("SQ_INSTS_VMEM_RD", "vmem_rd_instr_per_wave")):
            if k in c:
                out[name] = c[k] / c["SQ_WAVES"]
    return out


def main(pmc_dir, round_tag):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in sorted(os.listdir(pmc_dir)):
        d = os.path.join(pmc_dir, p)
        if not os.path.isdir(d):
            continue
        for f in (os.path.join(d, "run_counter_collection.csv"),):
            if not os.path.exists(f):
                continue
            for r in csv.DictReader(open(f)):
                agg[signature(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in sorted(agg.items()):
        med = {c: sorted(v)[len(v) // 2] for c, v in cs.items()}        # median launch
        med["launches"] = max(len(v) for v in cs.values())
        med.update(derived(med))
        out[k] = med
    try:
        head = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                              text=True).stdout.strip()
    except OSError:
        head = "?"
    for v in out.values():
        v["measured_at"] = head
    # merge: kernels of the families not profiled in this run keep their entries
    # (each tagged with the commit it was measured at)
    os.makedirs(os.path.join(ROOT, "profiles", round_tag), exist_ok=True)
    summ_path = os.path.join(ROOT, "profiles", round_tag, "pmc_summary.json")
    try:
        old_summ = json.load(open(summ_path))
    except (OSError, ValueError):
        old_summ = {}
    json.dump({**old_summ, **out}, open(summ_path, "w"), indent=1)
    keep = ("hbm_bytes_per_launch", "fetch_bytes_raw", "write_bytes_raw", "valu_busy", "waitcnt_stall", "issue_stall",
            "lds_busy", "valu_instr_per_wave", "lds_instr_per_wave", "salu_instr_per_wave", "measured_at")
    traffic_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        old_t = json.load(open(traffic_path))
    except (OSError, ValueError):
        old_t = {}
    old_k = old_t.get("kernels", {})
    for v in old_k.values():
        v.setdefault("measured_at", old_t.get("measured_at_commit", "?"))
    t = {"note": "per kernel instantiation, median launch: HBM-side bytes per launch = (2*FETCH_SIZE + "
                 "WRITE_SIZE)*1024 (gfx950 FETCH_SIZE = half the bytes, MI355X_MICROARCH.md; "
                 "profiles/r02/pmc_calibration.json), issue fractions of SQ_WAVE_CYCLES; profiles/<round>/"
                 "pmc_summary.json; measured_at: the commit each kernel's counters were taken at",
         "measured_at_commit": head,
         "kernels": {**old_k, **{k: {f: v[f] for f in keep if f in v} for k, v in out.items()}}}
    json.dump(t, open(traffic_path, "w"), indent=1)
    for k, v in t["kernels"].items():
        print(k, json.dumps({f: round(x, 4) if isinstance(x, float) and x < 100 else x for f, x in v.items()}))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc"),
         sys.argv[2] if len(sys.argv) > 2 else "r03")
