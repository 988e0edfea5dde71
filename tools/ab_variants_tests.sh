#!/usr/bin/env bash
# The bit-identity GPU tests against every ab/libdilqr_<V>.so variant (the
# variants are built from other sources on purpose: DILQR_SKIP_BUILD_ID), then
# the in-tree library restored.  Stops at the first failing variant.
set -o pipefail
export DILQR_SKIP_BUILD_ID=1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=differentiable-ilqr_amd/dilqr/libdilqr.so
cp $L ab/.inplace.so
K=${AB_TEST_K:-"fused_iteration_equals_unfused or whole_solve or fixed_count or packed_cost or small_batch or mpc_solve_vs_oracle"}
rc=0
for f in ab/${AB_GLOB:-libdilqr_*.so}; do
  v=${f#ab/libdilqr_}; v=${v%.so}
  cp $f $L
  timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "$K" \
      > gpurun_out/abtest_$v.log 2>&1; rc=$?
  echo "$v tests rc=$rc: $(tail -1 gpurun_out/abtest_$v.log)"
  [ $rc -eq 0 ] || break
done
cp ab/.inplace.so $L
exit $rc
