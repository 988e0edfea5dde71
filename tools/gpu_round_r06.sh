#!/usr/bin/env bash
# Round-6 full GPU session on the in-tree library (no rebuild on the box):
# GPU tests, smoke, bench (the JSON line), rocprof kernel stats of bench and of
# the kernels-only launch set, then the PMC passes (tools/profile_pmc.sh).
# STEPS selects (test smoke bench prof pmc; default all).  Every GPU step has
# its own time limit; a failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
STEPS="${STEPS:-all}"
test -f differentiable-ilqr_amd/dilqr/libdilqr.so || { echo "libdilqr.so missing"; exit 1; }
has() { [[ "$STEPS" == *all* || "$STEPS" == *$1* ]]; }
if has test; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v -rfE -s --timeout 180 --timeout-method thread \
      > $OUT/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest_gpu.log | tail -5
  [ $rc -le 1 ] || exit $rc
fi
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if has bench; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -c 600 $OUT/bench.log; echo; [ $rc -eq 0 ] || exit $rc
fi
if has prof; then
  R=$(pwd)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof -o run --output-format csv -- \
      python3 $R/bench.py --no-cpu-baseline > $R/$OUT/prof.log 2>&1; rc=$?
  echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_k -o run --output-format csv -- \
      python3 $R/bench.py --kernels-only > $R/$OUT/prof_k.log 2>&1; rc=$?
  echo "rocprof kernels-only rc=$rc"; tail -1 $R/$OUT/prof_k.log; [ $rc -eq 0 ] || exit $rc
  cd $R
fi
if has pmc; then
  PMC_SETS="${PMC_SETS:-headline box rocket implicit}" bash tools/profile_pmc.sh > $OUT/pmc.log 2>&1; rc=$?
  echo "pmc rc=$rc"; tail -3 $OUT/pmc.log; [ $rc -eq 0 ] || exit $rc
fi
echo ALL_DONE
