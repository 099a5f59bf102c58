#!/bin/bash
# Round-5 profile pass: kernel-trace stats + FETCH/WRITE/SQ passes per workload (tools/profile_round.sh),
# then KF2's phase split on c2fir (tools/r5_kf2_pmc.sh: full build and the diagnostic cuts)
WLS=${WLS:-"c2fir c4fir c3fir c5fir"} bash tools/profile_round.sh || exit $?
TAG=r5kf2q bash tools/r5_kf2_pmc.sh || exit $?
echo all-ok
