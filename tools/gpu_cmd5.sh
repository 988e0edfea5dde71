#!/usr/bin/env bash
# round-6 scratch: bit-identity tests of the ab/ variants, then an A/B with AB_CMD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_TEST_K="${AB_TEST_K}" timeout -k 10 900 bash tools/ab_variants_tests.sh || exit 1
timeout -k 10 900 bash tools/ab.sh ${AB_ROUNDS:-3} > gpurun_out/ab.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/ab.txt; exit $rc
