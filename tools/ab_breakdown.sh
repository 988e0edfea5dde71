#!/usr/bin/env bash
# A/B of prebuilt library variants (ab/libdilqr_<V>.so) on whole headline
# solves: tools/step_breakdown.py per variant, alternating, then a table of
# iteration 0 / steady iteration / whole-solve microseconds per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB_CMD=tools/step_breakdown.py bash tools/ab.sh ${1:-3} > gpurun_out/ab.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/ab.log | python -c "
import sys, json
for l in sys.stdin:
    v, _, j = l.partition(' ')
    d = json.loads(j)
    print(v, 'iter0', round(d['iter0'] * 1e3, 1), 'iterk', round(d['iterk'] * 1e3, 1), 'solve', round(d['solve_iterate'] * 1e3, 1))"
