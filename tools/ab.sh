#!/usr/bin/env bash
# A/B timing of two prebuilt libdilqr.so variants on the same box (ab/libdilqr_{A,B}.so),
# alternating, bench --kernels-only.  Usage: bash tools/ab.sh [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=differentiable-ilqr_amd/dilqr/libdilqr.so
for r in $(seq ${1:-3}); do
  for v in A B; do
    cp ab/libdilqr_$v.so $L
    out=$(timeout -k 10 300 python ${AB_CMD:-bench.py --kernels-only ${BENCH_ARGS:-}} | tail -1) || exit 1
    echo "$v $out"
  done
done
