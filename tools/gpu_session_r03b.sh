#!/usr/bin/env bash
# Round-3 session: phase stamps of the whole-solve launch, A/B of ab/ variants
# (bench --kernels-only: solve, steady iteration and sweep times), parity subset.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rfE -s --timeout 300 --timeout-method thread \
    -k "fused or packed or fixed or whole or mpc_solve or dataset or lqr_step or full_size" > gpurun_out/pytest_sub.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/pytest_sub.log | tail -5
[ $rc -le 1 ] || exit $rc
DILQR_SKIP_BUILD_ID=1 timeout -k 10 200 python tools/phase_stamps.py solve > gpurun_out/stamps_solve.json || exit 1
echo "stamps: $(cat gpurun_out/stamps_solve.json)"
timeout -k 10 900 bash tools/ab.sh ${ROUNDS:-3} || exit 1
