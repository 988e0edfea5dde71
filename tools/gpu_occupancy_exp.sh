#!/usr/bin/env bash
# Do two co-resident waves per SIMD raise the issue rate of the whole-solve
# kernel ("Two lanes per problem")?  Variants in ab/ (built by
# tools/build_variant.sh): base (the shipped library), diagonly (only the
# time-invariant diagonal cost path compiled: 240 VGPRs, no AGPRs) and
# diag_half2 (the same with 32 problems per wave and a 2-waves-per-SIMD launch
# bound: 2048 waves, two co-resident per SIMD, gain records in LDS).  Times
# (bench --kernels-only) and the issue counters of each, kernel trace only.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export DILQR_SKIP_BUILD_ID=1
OUT=$R/gpurun_out/occ
mkdir -p $OUT
for v in ${VARIANTS:-base diagonly diag_half2}; do
  DILQR_LIB=$R/ab/libdilqr_$v.so timeout -k 10 200 python3 $R/bench.py --kernels-only > $OUT/k_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 $OUT/k_$v.log)"
done
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-base diagonly diag_half2}; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_INSTS_VALU" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    DILQR_LIB=$R/ab/libdilqr_$v.so timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/${v}_p$i -o run \
        --output-format csv -- python3 $R/bench.py --kernels-only > $OUT/${v}_p$i.log 2>&1 || exit 1
  done
  echo "pmc $v done"
done
echo OCC_DONE
