#!/usr/bin/env bash
# PMC passes (tools/profile_pmc.sh, PMC_SETS) over every ab/libdilqr_<V>.so
# variant in turn, each into gpurun_out/pmc_<V>; the in-tree library restored.
set -o pipefail
export DILQR_SKIP_BUILD_ID=1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=differentiable-ilqr_amd/dilqr/libdilqr.so
cp $L ab/.inplace.so
rc=0
for f in ab/libdilqr_*.so; do
  v=${f#ab/libdilqr_}; v=${v%.so}
  cp $f $L
  rm -rf gpurun_out/pmc
  bash tools/profile_pmc.sh > gpurun_out/pmc_$v.log 2>&1; rc=$?
  mv gpurun_out/pmc gpurun_out/pmc_$v
  echo "$v pmc rc=$rc"
  [ $rc -eq 0 ] || break
done
cp ab/.inplace.so $L
exit $rc
