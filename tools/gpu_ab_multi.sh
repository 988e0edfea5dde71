#!/usr/bin/env bash
# A/B of ab/libdilqr_*.so: rocket (tools/ab_rocket.py) and config-4 box
# (bench --kernels-only --profile-set box) timings, alternating variants
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AB_CMD="tools/ab_rocket.py" timeout -k 10 600 bash tools/ab.sh ${ROUNDS:-3} || exit 1
AB_CMD="bench.py --kernels-only --profile-set box" timeout -k 10 600 bash tools/ab.sh ${ROUNDS:-3} || exit 1
