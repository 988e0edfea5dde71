#!/usr/bin/env bash
# round-6 scratch GPU session: implicit tests on the in-tree library, then A/B of ab/ variants
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${PYTEST:-1}" = 1 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-implicit or end_to_end or il_}" \
    > gpurun_out/pytest_implicit.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_implicit.log; [ $rc -eq 0 ] || exit $rc
fi
AB_CMD="${AB_CMD:-tools/ab_implicit.py}" timeout -k 10 600 bash tools/ab.sh ${AB_ROUNDS:-3} > gpurun_out/ab.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/ab.txt; exit $rc
