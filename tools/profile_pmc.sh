#!/usr/bin/env bash
# PMC passes over bench.py --kernels-only, one counter group per pass and one
# kernel family per run (PMC_SETS: headline box rocket implicit), kernel trace
# only: never combined with sys/runtime tracing.  Summarise with
#   python tools/pmc_summary.py gpurun_out/pmc <round>
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
GROUPS_=("FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_INSTS_VALU"
         "SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE")
# counters this ROCm/GPU offers: drop any of the optional last group it lacks
timeout -k 10 -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
opt=""
for c in ${GROUPS_[4]}; do grep -qw "$c" $OUT/avail.txt && opt="$opt $c"; done
GROUPS_[4]="${opt# }"
echo "optional group: ${GROUPS_[4]}"
for set in ${PMC_SETS:-headline box rocket implicit}; do
  i=0
  for grp in "${GROUPS_[@]}"; do
    i=$((i+1))
    [ -n "$grp" ] || continue
    timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/${set}_p$i -o run --output-format csv -- \
        python3 $R/bench.py --kernels-only --profile-set $set > $OUT/${set}_p$i.log 2>&1
    rc=$?; echo "set $set pass $i ($grp) rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
echo PMC_DONE
