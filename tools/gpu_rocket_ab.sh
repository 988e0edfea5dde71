#!/usr/bin/env bash
# rocket parity tests on the in-tree library, then A/B of ab/libdilqr_*.so on
# the config-3 kernels (tools/ab_rocket.py) and per-kernel rocprof stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rfE -s --timeout 300 --timeout-method thread \
    -k "rock or Rock or fixed_count or packed or dist" > gpurun_out/pytest_rocket.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_rocket.log
[ $rc -le 1 ] || exit $rc
AB_CMD="tools/ab_rocket.py" timeout -k 10 600 bash tools/ab.sh 3; rc=$?
[ $rc -eq 0 ] || exit $rc
PSET=rocket timeout -k 10 300 bash tools/gpu_prof_set.sh | grep -E "rc=|k_mpc"
