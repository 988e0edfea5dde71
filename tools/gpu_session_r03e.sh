#!/usr/bin/env bash
# implicit parity tests on the in-tree build + implicit A/B of ab/ variants
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rfE -s --timeout 300 --timeout-method thread \
    -k "implicit or il_ or end_to_end" > gpurun_out/pytest_sub.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/pytest_sub.log | tail -5
[ $rc -le 1 ] || exit $rc
AB_CMD="bench.py --kernels-only --profile-set implicit" timeout -k 10 600 bash tools/ab.sh ${ROUNDS:-3} || exit 1
