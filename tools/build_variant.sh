#!/bin/bash
# An in-tree A/B build of the WORKING TREE with extra compile flags (diagnostic variants):
#   tools/build_variant.sh <name> "<EXTRA flags>"  ->  in_cwave_amd/<name>.so (git-ignored; ICW_LIB=<name>.so)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; extra=$2
D=$(mktemp -d /tmp/icw_var.XXXX)
mkdir -p "$D/pkg" "$D/include"
cp -r "$R/in_cwave_amd/csrc" "$D/pkg/csrc"
cp "$R"/include/*.h "$D/include/"
rm -f "$D"/pkg/csrc/*.o
make -s -j4 -C "$D/pkg/csrc" EXTRA="$extra" OUT="$R/in_cwave_amd/$name.so" > /dev/null
rm -rf "$D"
echo "built in_cwave_amd/$name.so ($extra)"
