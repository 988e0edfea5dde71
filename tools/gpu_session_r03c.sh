#!/usr/bin/env bash
# Round-3 session: parity subset (fused/fixed/whole/implicit), A/B of ab/
# variants on the headline solve and on both implicit backwards.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rfE -s --timeout 300 --timeout-method thread \
    -k "fused or packed or fixed or whole or mpc_solve or dataset or lqr_step or full_size or implicit or il_" > gpurun_out/pytest_sub.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/pytest_sub.log | tail -5
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 bash tools/ab.sh ${ROUNDS:-3} || exit 1
AB_CMD="bench.py --kernels-only --profile-set implicit" timeout -k 10 600 bash tools/ab.sh 2 || exit 1
