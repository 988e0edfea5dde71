#!/usr/bin/env bash
# box-path parity tests, A/B of ab/libdilqr_*.so on the config-4 steady kernel,
# phase stamps (diagnostic build) for config 2 and config 4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rfE -s --timeout 300 --timeout-method thread \
    -k "box or Box or pnqp or fused or packed or fixed_count or lqr_step" > gpurun_out/pytest_box.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_box.log
[ $rc -le 1 ] || exit $rc
AB_CMD="bench.py --kernels-only --profile-set box" timeout -k 10 600 bash tools/ab.sh 3 || exit 1
export DILQR_SKIP_BUILD_ID=1
for b in 0 100 10; do
  BOUNDS=$b timeout -k 10 200 python tools/phase_stamps.py 5 > gpurun_out/stamps_b$b.json || exit 1
  echo "stamps bounds=$b"; cat gpurun_out/stamps_b$b.json
done
