#!/usr/bin/env bash
# One GPU-box session: build, GPU parity tests, smoke, bench, rocprof kernel stats.
# Every GPU step has its own time limit; a crash/timeout ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
STEPS="${STEPS:-all}"
make -C differentiable-ilqr_amd -j16 > $OUT/build.log 2>&1 || { echo "build failed"; tail -20 $OUT/build.log; exit 1; }
if [[ "$STEPS" == *all* || "$STEPS" == *test* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -rfE -s --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
      > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -30 $OUT/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [[ "$STEPS" == *all* || "$STEPS" == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -5 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if [[ "$STEPS" == *all* || "$STEPS" == *bench* ]]; then
  timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -3 $OUT/bench.log; [ $rc -eq 0 ] || exit $rc
fi
if [[ "$STEPS" == *all* || "$STEPS" == *prof* ]]; then
  R=$(pwd)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof -o run --output-format csv -- \
      python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/$OUT/prof.log 2>&1; rc=$?
  echo "rocprof rc=$rc"; tail -3 $R/$OUT/prof.log; [ $rc -eq 0 ] || exit $rc
  # the roofline kernel alone (bench --kernels-only: the steady-state fused
  # iteration's launches are exactly the ones bench.py times with HIP events)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_k -o run --output-format csv -- \
      python3 $R/bench.py --kernels-only > $R/$OUT/prof_k.log 2>&1; rc=$?
  echo "rocprof kernels-only rc=$rc"; tail -1 $R/$OUT/prof_k.log; [ $rc -eq 0 ] || exit $rc
  cd $R
fi
echo ALL_DONE
