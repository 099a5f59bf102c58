#!/bin/bash
# Round-5 call 1: K3r clamp-free blocks (tests + c5fir A/B), then KF2's VALU by phase (SQ passes of the
# diagnostic builds, tools/build_variant.sh).  Every step has its own limit; the first failure stops.
bash tools/k3r_ab.sh || exit $?
export TMPDIR=/tmp
LIBS="libicw.so libicw_cut1.so libicw_cut2.so" W=c2fir TAG=r5kf2 FRAMES=262144 bash tools/pmc_variants.sh || exit $?
echo all-ok
