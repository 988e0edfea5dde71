#!/usr/bin/env bash
# LDS / issue counters of one kernel family (PSET, default rocket) for the
# in-tree library and every ab/libdilqr_<V>.so variant: one counter group per
# pass, kernel trace only (PMCS_VARIANTS=0: the in-tree library only).
# Output: gpurun_out/pmcs/<variant>_p<i>/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/gpurun_out/pmcs
mkdir -p $OUT
export DILQR_SKIP_BUILD_ID=1
L=$R/differentiable-ilqr_amd/dilqr/libdilqr.so
cp $L $OUT/.inplace.so
cd /tmp && export TMPDIR=/tmp
GROUPS_=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS"
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL"
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_CMD_FIFO_FULL SQ_LDS_UNALIGNED_STALL"
         "SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_INST_LEVEL_LDS")
VARIANTS=$R/ab/libdilqr_*.so
[ "${PMCS_VARIANTS:-1}" = "0" ] && VARIANTS=
for f in $OUT/.inplace.so $VARIANTS; do
  [ -f "$f" ] || continue
  v=$(basename $f .so); v=${v#libdilqr_}; [ "$v" = ".inplace" ] && v=inplace
  cp $f $L
  i=0
  for grp in "${GROUPS_[@]}"; do
    i=$((i+1))
    timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/${v}_p$i -o run --output-format csv -- \
        python3 $R/bench.py --kernels-only --profile-set ${PSET:-rocket} > $OUT/${v}_p$i.log 2>&1
    rc=$?; echo "$v pass $i rc=$rc"
    [ $rc -eq 0 ] || { cp $OUT/.inplace.so $L; exit $rc; }
  done
done
cp $OUT/.inplace.so $L
echo PMCS_DONE
