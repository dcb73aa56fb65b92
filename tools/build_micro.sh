#!/bin/bash
# Diagnostic ablation binaries: bench/micro/gen_abl<N> with -DPGA_ABL=N
# (1 = no crossover RNG, 2 = no pool RNG, 4 = no mutation, 8 = no parent gather).
set -e
cd "$(dirname "$0")/.."
python tools/build.py build/libpga.so >/dev/null 2>&1 || true
F="-O3 -std=c++17 -Icsrc/include --offload-arch=gfx950"
mkdir -p build/micro
common="build/obj/csrc_kernels_util.k.o build/obj/csrc_kernels_real.k.o build/obj/csrc_kernels_perm.k.o build/obj/csrc_engine_island.h.o build/obj/csrc_cpu_cpu_ops.h.o build/obj/csrc_cpu_cpu_real.h.o build/obj/csrc_cpu_cpu_perm.h.o build/obj/csrc_engine_jit.h.o build/obj/csrc_engine_trace.h.o build/obj/csrc_kernels_compat.k.o build/obj/csrc_kernels_qubo.k.o -lhiprtc -L/opt/rocm/lib -lroctx64"
hipcc $F -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -c bench/gen_bench.cpp -o build/micro/gen_bench.o
for n in ${ABL:-0 1 2 4 8 7 15}; do
  hipcc $F -x hip -DPGA_ABL=$n ${EXTRA:-} -c csrc/kernels/binary.hip -o build/micro/binary_abl$n.o &
done
wait
for n in ${ABL:-0 1 2 4 8 7 15}; do
  hipcc --offload-arch=gfx950 -o build/micro/gen_abl$n build/micro/gen_bench.o build/micro/binary_abl$n.o $common
done
ls build/micro/gen_abl*
