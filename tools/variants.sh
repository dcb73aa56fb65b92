#!/bin/bash
# Build gen_bench (bench/gen_bench.cpp) against compile-time variants of one
# kernel source, for interleaved A/B runs on the GPU (tools/ab.sh):
#
#   tools/variants.sh csrc/kernels/binary_gs.hip "pd1:-DPGA_TP_PD=1" "t:-DPGA_TP_TIMING"
#   -> build/variants/gen_<name>
#
# binary_gs.hip (the BINARY launchers, one object per group size) is rebuilt
# for the headline group size 8 only; the other group sizes link from the
# regular build.  Needs the regular build first (tools/build.py): the other
# kernels, the engine and the CPU backend link from build/obj.  Nothing here
# is shipped.
set -e
cd "$(dirname "$0")/.."
src=$1; shift
base=$(basename "$src" .hip)
O=build/obj
mkdir -p build/variants
flags="-O3 -std=c++17 -Icsrc/include -Iinclude -x hip --offload-arch=gfx950 -munsafe-fp-atomics -ffp-contract=fast"
/opt/rocm/bin/hipcc $flags -c bench/gen_bench.cpp -o build/variants/gen_bench.o
others=""
for k in binary binary_batch real_batch perm qubo real util compat sort; do
  [ "$k" = "$base" ] || others="$others $O/csrc_kernels_$k.k.o"
done
extra=""
if [ "$base" = binary_gs ]; then
  extra="-DPGA_BIN_GS=8"
  for g in 1 2 4 16 32 64; do others="$others $O/csrc_kernels_binary_gs.gs$g.k.o"; done
else
  for g in 1 2 4 8 16 32 64; do others="$others $O/csrc_kernels_binary_gs.gs$g.k.o"; done
fi
for spec in "$@"; do
  name=${spec%%:*}
  defs=${spec#*:}
  (
    /opt/rocm/bin/hipcc $flags $extra $defs -c "$src" -o "build/variants/${base}_$name.o" &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -o "build/variants/gen_$name" build/variants/gen_bench.o \
      "build/variants/${base}_$name.o" $others $O/csrc_engine_*.h.o $O/csrc_cpu_*.h.o -lpthread -ldl
  ) &
done
wait
ls build/variants/gen_*
