#!/usr/bin/env bash
# round-6 scratch: the full GPU suite on the in-tree library, then the headline A/B of ab/ variants
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
    > gpurun_out/pytest_all.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_all.log; [ $rc -eq 0 ] || exit $rc
AB_CMD="bench.py --no-secondary --no-cpu-baseline --steps 40" timeout -k 10 900 bash tools/ab.sh ${AB_ROUNDS:-4} > gpurun_out/ab_headline.log 2>&1; rc=$?
grep -E "^[a-z0-9_]+ \{" gpurun_out/ab_headline.log | sed -E "s/ \{.*\"value\": ([0-9.]+).*/ \1/"; exit $rc
