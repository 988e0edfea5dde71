#!/usr/bin/env bash
# Do more waves per SIMD buy issue throughput for the fused cartpole iteration?
# The build with gain records in HBM (ab_exp/libdilqr_nolds.so, -DDILQR_NO_LDS_GAINS=1:
# eight workgroups fit a CU) at B = 65536 (1 wave per SIMD) and 131072 (2 per
# SIMD): steady kernel time (bench --kernels-only) and PMC issue counters.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export DILQR_SKIP_BUILD_ID=1 DILQR_LIB=$R/ab_exp/libdilqr_nolds.so
OUT=$R/gpurun_out/waves
mkdir -p $OUT
for B in 65536 131072; do
  timeout -k 10 200 python3 $R/bench.py --kernels-only --batch $B > $OUT/k_$B.log 2>&1 || exit 1
  echo "B=$B $(tail -1 $OUT/k_$B.log | cut -c1-400)"
done
cd /tmp && export TMPDIR=/tmp
for B in 65536 131072; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/b${B}_p$i -o run --output-format csv -- \
        python3 $R/bench.py --kernels-only --batch $B > $OUT/b${B}_p$i.log 2>&1 || exit 1
  done
done
echo WAVES_DONE
