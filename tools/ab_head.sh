#!/bin/bash
# Build the committed kernel source as variant "head" for an A/B run against the working tree.
set -e
cd "$(dirname "$0")/.."
rm -rf buas-pathtracer_amd/lib/variants/head buas-pathtracer_amd/build/variants/head
cp buas-pathtracer_amd/csrc/rt_kernels.hip /tmp/rt_cur_ab.hip
git show HEAD:buas-pathtracer_amd/csrc/rt_kernels.hip > buas-pathtracer_amd/csrc/rt_kernels.hip
tools/build_variants.sh head "" || true
cp /tmp/rt_cur_ab.hip buas-pathtracer_amd/csrc/rt_kernels.hip
touch buas-pathtracer_amd/csrc/rt_kernels.hip
make -s -C buas-pathtracer_amd/csrc
