"""Summarise tools/ab.sh output (bench JSON lines) per variant: median ms/step,
fused-iteration and sweep launch ms."""
import json
import statistics
import sys
from collections import defaultdict

rows = defaultdict(list)
for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab.log"):
    v, _, j = line.partition(" ")
    try:
        d = json.loads(j)
    except ValueError:
        continue
    if "ms_per_step" in d:
        rows[v].append((d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["riccati_roofline"]["avg_launch_ms"]))
    else:
        rows[v].append((d.get("iter_ms", 0.0), d.get("iter_ms", 0.0), d.get("sweep_ms", 0.0)))
for v, r in sorted(rows.items()):
    med = [statistics.median(c) for c in zip(*r)]
    print(f"{v:12s} n={len(r)} step {med[0]:.4f} ms  iter {med[1]:.4f} ms  sweep {med[2]:.4f} ms")
