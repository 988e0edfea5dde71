#!/usr/bin/env bash
# Build an A/B variant of libdilqr.so into ab/libdilqr_<name>.so: the listed
# translation units recompiled with extra flags, every other unit taken from
# the in-tree build (make first).  Usage:
#   bash tools/build_variant.sh <name> "<extra hipcc flags>" tu_mpc_cartpole [tu_...]
# tools/ab.sh then times every ab/libdilqr_*.so on one box.
set -e -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
P=$R/differentiable-ilqr_amd
NAME=$1; FLAGS=$2; shift 2
make -s -C $P -j8
mkdir -p $R/ab /tmp/abv/$NAME
OBJS=()
for o in $P/build/tu_*.o; do
  tu=$(basename $o .o)
  if [[ " $* " == *" $tu "* ]]; then
    # the unit's own flags from the Makefile (TUFLAGS_<unit> := ...), as the
    # in-tree build compiles it, then the variant's
    TUF=$(sed -n "s/^TUFLAGS_$tu := //p" $P/Makefile)
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -ffp-contract=on \
        $TUF $FLAGS -c -o /tmp/abv/$NAME/$tu.o $P/csrc/$tu.hip
    OBJS+=(/tmp/abv/$NAME/$tu.o)
  else
    OBJS+=($o)
  fi
done
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -o $R/ab/libdilqr_$NAME.so "${OBJS[@]}"
echo "built ab/libdilqr_$NAME.so ($FLAGS: $*; unit flags from the Makefile)"
