#!/usr/bin/env bash
# FETCH_SIZE / WRITE_SIZE calibration passes (one counter per pass, kernel
# trace only) over tools/microbench/fetch_calib; summary by tools/pmc_calib.py.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/gpurun_out/calib
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c -d $OUT/$c -o run --output-format csv -- \
      $R/tools/microbench/fetch_calib > $OUT/$c.log 2>&1
  rc=$?; echo "calib $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
echo CALIB_DONE
