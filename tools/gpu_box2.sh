#!/usr/bin/env bash
# box path: parity subset, A/B (config 4 steady kernel), pnqp counts, phase stamps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rfE -s --timeout 300 --timeout-method thread \
    -k "box or Box or pnqp or fused or packed or fixed_count or lqr_step or implicit or rock or golden" > gpurun_out/pytest_sub.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/pytest_sub.log | tail -5
[ $rc -le 1 ] || exit $rc
AB_CMD="bench.py --kernels-only --profile-set box" timeout -k 10 600 bash tools/ab.sh 3 || exit 1
timeout -k 10 200 python tools/box_nqp.py 100 5 | cut -c1-300 || exit 1
export DILQR_SKIP_BUILD_ID=1
BOUNDS=100 timeout -k 10 200 python tools/phase_stamps.py 5 > gpurun_out/stamps_b100.json || exit 1
cat gpurun_out/stamps_b100.json
