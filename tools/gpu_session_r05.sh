#!/usr/bin/env bash
# Round-5 GPU session: the in-tree libdilqr.so built here travels with the
# snapshot (no rebuild on the box; _native.py refuses a stale library), then
# the GPU tests (PYTEST_K filters them; "all" = every -m gpu test; "" skips),
# then an optional command.  Every GPU step has its own time limit; a failure
# ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
test -f differentiable-ilqr_amd/dilqr/libdilqr.so || { echo "libdilqr.so missing"; exit 1; }
if [ -n "${PYTEST_K:-}" ]; then
  if [ "$PYTEST_K" = "all" ]; then K=(); else K=(-k "$PYTEST_K"); fi
  timeout -k 10 600 python -u -m pytest tests -m gpu -v -rfE -s --timeout 180 --timeout-method thread "${K[@]}" \
      > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest_gpu.log | tail -30
  [ $rc -le 1 ] || exit $rc
fi
if [ -n "${EXTRA:-}" ]; then
  timeout -k 10 900 bash -c "$EXTRA" > $OUT/extra.log 2>&1; rc=$?
  echo "extra rc=$rc"; tail -30 $OUT/extra.log
  [ $rc -eq 0 ] || exit $rc
fi
echo SESSION_DONE
