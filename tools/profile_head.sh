#!/usr/bin/env bash
# Every profile the bench line cites, from one tree: build in-tree, rocprof
# kernel statistics of the default bench run and of the kernels-only run, then
# the PMC passes of every kernel family (tools/profile_pmc.sh).  Each GPU step
# has its own time limit and a failure ends the script.  Afterwards, here:
#   python tools/pmc_summary.py gpurun_out/pmc <round>
#   cp gpurun_out/stats/bench/run_kernel_stats.csv profiles/<round>/kernel_stats_bench.csv
#   cp gpurun_out/stats/kern/run_kernel_stats.csv profiles/<round>/kernel_stats_kernels_only.csv
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/gpurun_out
mkdir -p $OUT/stats
make -C $R/differentiable-ilqr_amd -j16 > $OUT/build.log 2>&1 || { echo "build failed"; tail -20 $OUT/build.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/stats/bench -o run --output-format csv -- \
    python3 $R/bench.py > $OUT/stats/bench.log 2>&1
rc=$?; echo "stats bench rc=$rc"; tail -1 $OUT/stats/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats/kern -o run --output-format csv -- \
    python3 $R/bench.py --kernels-only > $OUT/stats/kern.log 2>&1
rc=$?; echo "stats kernels-only rc=$rc"; [ $rc -eq 0 ] || exit $rc
find $OUT/stats -name '*kernel_stats.csv' | sed 's/^/  /'
bash $R/tools/profile_pmc.sh
