#!/usr/bin/env bash
# Round-4 GPU session: build in-tree, GPU tests (PYTEST_K filters them; "all"
# runs every -m gpu test), then optional timing commands.  Every GPU step has
# its own time limit; a failure ends the script.
#   PYTEST_K   pytest -k expression ("" skips the tests, "all" = no filter)
#   EXTRA      a command run after the tests (e.g. bench.py --kernels-only ...)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
make -C differentiable-ilqr_amd -j16 > $OUT/build.log 2>&1 || { echo "build failed"; tail -20 $OUT/build.log; exit 1; }
if [ -n "${PYTEST_K:-}" ]; then
  if [ "$PYTEST_K" = "all" ]; then K=(); else K=(-k "$PYTEST_K"); fi
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -rfE -s --timeout 300 --timeout-method thread "${K[@]}" \
      > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/pytest_gpu.log | tail -40
  [ $rc -le 1 ] || exit $rc
fi
if [ -n "${EXTRA:-}" ]; then
  timeout -k 10 600 bash -c "$EXTRA" > $OUT/extra.log 2>&1; rc=$?
  echo "extra rc=$rc"; tail -20 $OUT/extra.log
  [ $rc -eq 0 ] || exit $rc
fi
echo SESSION_DONE
