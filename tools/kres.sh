#!/bin/bash
# Register / LDS / scratch use of every kernel in a built rt_kernels.o (or any HIP object):
#   tools/kres.sh [buas-pathtracer_amd/build/rt_kernels.o] [kernel-name-regex]
obj=${1:-buas-pathtracer_amd/build/rt_kernels.o}
pat=${2:-.}
tmp=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section .hip_fatbin=$tmp/fb "$obj"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
    --input=$tmp/fb --output=$tmp/co --unbundle
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $tmp/co | python3 -c '
import sys, re
txt = sys.stdin.read()
pat = re.compile(sys.argv[1])
for blk in txt.split("  - .agpr_count")[1:]:
    def g(k):
        m = re.search(r"\.%s:\s+(\S+)" % re.escape(k), blk)
        return m.group(1) if m else "?"
    name = g("name")
    if not pat.search(name): continue
    print("%-60s vgpr %4s sgpr %4s lds %6s scratch %5s" % (name[:60], g("vgpr_count"), g("sgpr_count"),
          g("group_segment_fixed_size"), g("private_segment_fixed_size")))
' "$pat"
rm -rf $tmp
