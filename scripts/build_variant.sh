#!/bin/bash
# Build an A/B variant of libmmre_hip.so from the in-tree sources with one sed edit applied.
# usage: scripts/build_variant.sh <name> <csrc file> <sed expression>  ->  abl/<name>.so
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
echo "abl/$name.so"
