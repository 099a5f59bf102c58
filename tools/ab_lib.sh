#!/bin/bash
# A/B build: tools/ab_lib.sh <name> [<icw_iir.hip variant>] -> in_cwave_amd/<name>.so (git-ignored,
# travels to the GPU box; select it with ICW_LIB=<name>.so).  The variant replaces the kernel file
# of the current tree; everything else is the working tree.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; var=$2
D=$(mktemp -d /tmp/icw_ab.XXXX)
mkdir -p "$D/in_cwave_amd" "$D/include"
cp -r "$R/in_cwave_amd/csrc" "$D/in_cwave_amd/"
cp "$R"/include/*.h "$D/include/"
rm -f "$D"/in_cwave_amd/csrc/*.o
[ -n "$var" ] && cp "$var" "$D/in_cwave_amd/csrc/icw_iir.hip"
make -s -j8 -C "$D/in_cwave_amd/csrc" OUT="$R/in_cwave_amd/$name.so" > /dev/null
rm -rf "$D"
echo "built in_cwave_amd/$name.so"
