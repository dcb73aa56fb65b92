#!/bin/bash
# build/micro/gen_v<i> from binary.hip with VAR<i> flags
set -e
cd /root/repo
F="-O3 -std=c++17 -Icsrc/include --offload-arch=gfx950"
common="build/obj/csrc_kernels_util.k.o build/obj/csrc_kernels_real.k.o build/obj/csrc_kernels_perm.k.o build/obj/csrc_engine_island.h.o build/obj/csrc_cpu_cpu_ops.h.o build/obj/csrc_cpu_cpu_real.h.o build/obj/csrc_cpu_cpu_perm.h.o build/obj/csrc_engine_jit.h.o build/obj/csrc_engine_trace.h.o build/obj/csrc_kernels_compat.k.o build/obj/csrc_kernels_qubo.k.o -lhiprtc -L/opt/rocm/lib -lroctx64"
i=0
for v in "$@"; do
  (hipcc $F -x hip $v -c csrc/kernels/binary.hip -o build/micro/bin_v$i.o && hipcc --offload-arch=gfx950 -o build/micro/gen_v$i build/micro/gen_bench.o build/micro/bin_v$i.o $common) &
  i=$((i+1))
done
wait
