#!/bin/bash
# A/B build of a committed revision: tools/ab_rev.sh <name> [<rev>=HEAD] -> in_cwave_amd/<name>.so
# (git-ignored, travels to the GPU box; select it with ICW_LIB=<name>.so)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; rev=${2:-HEAD}
D=$(mktemp -d /tmp/icw_rev.XXXX)
git -C "$R" archive "$rev" in_cwave_amd/csrc include | tar -x -C "$D"
make -s -j8 -C "$D/in_cwave_amd/csrc" OUT="$R/in_cwave_amd/$name.so" > /dev/null
rm -rf "$D"
echo "built in_cwave_amd/$name.so from $(git -C "$R" rev-parse --short "$rev")"
