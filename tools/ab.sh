#!/usr/bin/env bash
# A/B timing of prebuilt libdilqr.so variants on the same box (ab/libdilqr_<V>.so,
# every variant present), alternating, bench --kernels-only by default.
# Usage: bash tools/ab.sh [rounds]; AB_CMD overrides the timed command, AB_GLOB
# picks a subset of ab/ (default libdilqr_*.so).
set -o pipefail
export DILQR_SKIP_BUILD_ID=1   # the variants are built from other sources on purpose
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=differentiable-ilqr_amd/dilqr/libdilqr.so
cp $L ab/.inplace.so
for r in $(seq ${1:-3}); do
  for f in ab/${AB_GLOB:-libdilqr_*.so}; do
    v=${f#ab/libdilqr_}; v=${v%.so}
    cp $f $L
    out=$(timeout -k 10 300 python ${AB_CMD:-bench.py --kernels-only ${BENCH_ARGS:-}} | tail -1) || exit 1
    echo "$v $out"
  done
done
cp ab/.inplace.so $L
