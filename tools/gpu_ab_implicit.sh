#!/usr/bin/env bash
# implicit-backward parity tests on the in-tree library, then A/B of
# ab/libdilqr_*.so on the config-4 cartpole implicit backward (tools/ab_implicit.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "implicit" \
    > gpurun_out/pytest_implicit.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_implicit.log; [ $rc -le 1 ] || exit $rc
AB_CMD="tools/ab_implicit.py" timeout -k 10 900 bash tools/ab.sh ${AB_ROUNDS:-4}
