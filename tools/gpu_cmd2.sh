#!/usr/bin/env bash
# round-6 scratch GPU session: rocket implicit + MPC tests, then two A/B sets
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "rocket" \
    > gpurun_out/pytest_rocket.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_rocket.log; [ $rc -eq 0 ] || exit $rc
AB_GLOB="libdilqr_[br]*.so" AB_CMD=tools/ab_implicit_rocket.py timeout -k 10 600 bash tools/ab.sh 3 > gpurun_out/ab1.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/ab1.txt; [ $rc -eq 0 ] || exit $rc
AB_GLOB="libdilqr_[bg]*.so" AB_CMD=tools/ab_rocket_dense.py timeout -k 10 600 bash tools/ab.sh 2 > gpurun_out/ab2.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/ab2.txt; exit $rc
