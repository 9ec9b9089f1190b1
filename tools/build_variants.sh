#!/bin/bash
# Build tuning variants of librt_mi355x.so under buas-pathtracer_amd/lib/variants/<name>/.
# usage: tools/build_variants.sh name1 "flags1" name2 "flags2" ...
set -e
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  make -s -C buas-pathtracer_amd/csrc OUTDIR=$PWD/buas-pathtracer_amd/lib/variants/$name \
       BUILD=$PWD/buas-pathtracer_amd/build/variants/$name EXTRA="$flags" >/dev/null
  echo "built $name ($flags)"
done
