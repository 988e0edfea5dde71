#!/usr/bin/env bash
# rocprof kernel stats of one timing command for each ab/ variant matching
# AB_GLOB (the variant copied over the in-tree library, restored after):
# per-kernel times that the variant's changed iterates do not confound
set -o pipefail
export DILQR_SKIP_BUILD_ID=1
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
L=differentiable-ilqr_amd/dilqr/libdilqr.so
cp $L ab/.inplace.so
for f in ab/${AB_GLOB:-libdilqr_*.so}; do
  v=${f#ab/libdilqr_}; v=${v%.so}
  cp $f $L
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pv_$v -o run \
      --output-format csv -- python3 $R/${PROF_CMD:-tools/ab_rocket_dense.py} > $R/gpurun_out/pv_$v.log 2>&1) || { cp ab/.inplace.so $L; exit 1; }
  echo "== $v"; f2=$(find gpurun_out/pv_$v -name "*kernel_stats.csv" | head -1); head -12 "$f2" | cut -d, -f1-4
done
cp ab/.inplace.so $L
