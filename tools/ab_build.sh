#!/bin/bash
# Build the product library of another git revision (an A/B arm) into OUT, from the tree's history:
#   tools/ab_build.sh REV OUT.so [XFLAGS]
# e.g. tools/ab_build.sh a53f363 alt/libspartan_hip_r05.so  (round 5's HEAD: rocPRIM radix sort)
# The arm then runs through SPX_LIB_PATH (tools/ab_bench.sh, tools/ab_vrank.sh).
set -e
REV="$1"; OUT=$(realpath -m "$2"); XF="${3:-}"
D=$(mktemp -d /tmp/abbuild.XXXXXX)
git archive "$REV" r1cs-spartan_amd include | tar -x -C "$D"
mkdir -p "$(dirname "$OUT")"
make -s -j"${MAX_JOBS:-8}" -C "$D/r1cs-spartan_amd/csrc" OUT="$OUT" OBJDIR="$D/obj" XFLAGS="$XF"
rm -rf "$D"
echo "built $REV -> $OUT"
