#!/usr/bin/env bash
# round-6 scratch: stop-rule MPC tests, then the IL step at 4096 / 1024 problems with blocking (DILQR_POLL_AHEAD=0) vs pipelined polls
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "mpc or il_ or stop" \
    > gpurun_out/pytest_poll.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_poll.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for pa in 0 2; do
    DILQR_POLL_AHEAD=$pa timeout -k 10 300 python tools/il_small_batch.py 4096 1024 > gpurun_out/il_poll_$pa.json 2>&1 || exit 1
    echo "poll_ahead=$pa $(grep -v amdgpu gpurun_out/il_poll_$pa.json)" | cut -c1-600
  done
done
