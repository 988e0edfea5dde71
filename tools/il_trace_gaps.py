"""GPU busy time vs span of one IL training step, from a rocprofv3 kernel trace
of `tools/il_small_batch.py 32`: the kernels of one step period (from the
second-to-last k_mpc_solve_small launch to the last one), each with its start
offset and duration, then busy / span and the largest idle gaps — what the host
(Python, autograd, allocation) costs between the launches.

  rocprofv3 --kernel-trace -d gpurun_out/iltrace -o run --output-format csv -- python3 tools/il_small_batch.py 32
  python tools/il_trace_gaps.py gpurun_out/iltrace
"""
import csv
import glob
import os
import sys


def main(d):
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    solves = [i for i, k in enumerate(ks) if "k_mpc_solve_small" in k[2]]
    if len(solves) < 2:
        print("fewer than two small-batch solves in the trace")
        return
    a, b = solves[-2], solves[-1]
    # one step period: from the second-to-last solve's start to the last one's
    # (that solve, its post-processing, the backward, the next step's set-up)
    step = ks[a:b]
    t0 = step[0][0]
    busy = 0
    prev_end = t0
    gaps = []
    for s, e, n in step:
        busy += e - s
        gaps.append((s - prev_end, n))
        prev_end = max(prev_end, e)
        print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  {n.split('(')[0][:90]}")
    gaps.append((ks[b][0] - prev_end, ks[b][2]))
    span = ks[b][0] - t0
    print(f"kernels {len(step)}, busy {busy / 1e3:.1f} us, span {span / 1e3:.1f} us")
    for g, n in sorted(gaps, reverse=True)[:8]:
        print(f"  gap {g / 1e3:8.1f} us before {n.split('(')[0][:80]}")


if __name__ == "__main__":
    main(sys.argv[1])
