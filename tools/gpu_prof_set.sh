#!/usr/bin/env bash
# rocprofv3 kernel trace + stats of one bench --kernels-only profile set
#   PSET=rocket bash tools/gpu_prof_set.sh
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${PSET} -o run --output-format csv -- \
    python3 $R/bench.py --kernels-only --profile-set ${PSET} > $R/gpurun_out/prof_${PSET}.log 2>&1; rc=$?
echo "rocprof $PSET rc=$rc"; tail -2 $R/gpurun_out/prof_${PSET}.log
find $R/gpurun_out/prof_${PSET} -name "*kernel_stats.csv" -exec cat {} \;
exit $rc
