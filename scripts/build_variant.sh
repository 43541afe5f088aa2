#!/bin/bash
# Build an A/B variant of libmmre_hip.so from the in-tree sources with one sed edit applied.
# usage: scripts/build_variant.sh <name> <csrc file> <sed expression>  ->  abl/<name>.so
# Every build appends its name, file, sed expression and source revision (with a "+dirty" mark
# when the tree had uncommitted changes) to scripts/variants.txt, which is committed: an A/B
# library must be reproducible from the record (round 4's abl/norescore.so was not).
set -e
name=$1; file=$2; expr=$3
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=/tmp/mmre_variant_$name
rm -rf $tmp && mkdir -p $tmp/pkg $tmp/include
cp -r $root/multimodal-relation-extrapolation_amd/csrc $root/multimodal-relation-extrapolation_amd/Makefile $tmp/pkg/
cp $root/include/*.h $tmp/include/
before=$(md5sum $tmp/pkg/csrc/$file | cut -d' ' -f1)
sed -i "$expr" $tmp/pkg/csrc/$file
[ "$(md5sum $tmp/pkg/csrc/$file | cut -d' ' -f1)" != "$before" ] || { echo "sed changed nothing"; exit 1; }
make -C $tmp/pkg -j8 mmre/lib/libmmre_hip.so > $tmp/build.log 2>&1 || { tail -20 $tmp/build.log; exit 1; }
mkdir -p $root/abl && cp $tmp/pkg/mmre/lib/libmmre_hip.so $root/abl/$name.so
rev=$(git -C $root rev-parse --short HEAD)$(git -C $root diff --quiet HEAD -- multimodal-relation-extrapolation_amd/csrc include || echo +dirty)
printf '%s\t%s\t%s\t%s\t%s\n' "$(date -u +%FT%TZ)" "$name" "$file" "$rev" "$expr" >> $root/scripts/variants.txt
echo "abl/$name.so"
