#!/usr/bin/env bash
# GPU tests with the in-place library, then A/B of the prebuilt ab/ variants:
# cartpole (bench --kernels-only) and rocket (tools/ab_rocket.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
      > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 900 bash tools/ab.sh ${AB_ROUNDS:-2} > gpurun_out/ab.log 2>&1 || { echo "ab failed"; tail -5 gpurun_out/ab.log; exit 1; }
python tools/ab_summary.py gpurun_out/ab.log 2>/dev/null || cat gpurun_out/ab.log
if [ "${SKIP_ROCKET:-0}" != 1 ]; then
  AB_CMD=tools/ab_rocket.py timeout -k 10 900 bash tools/ab.sh 1 > gpurun_out/ab_rocket.log 2>&1 || { echo "ab rocket failed"; tail -5 gpurun_out/ab_rocket.log; exit 1; }
  cat gpurun_out/ab_rocket.log
fi
echo AB_DONE
