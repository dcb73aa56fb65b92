#!/bin/bash
# Host-side AddressSanitizer + UndefinedBehaviorSanitizer build of the C API
# and CPU backend, then the native C API test on the CPU backend (no GPU).
# Device code is compiled normally: -fsanitize goes to the host only
# (-Xarch_host on .hip lines, -fno-gpu-sanitize on host-only lines).
# SURVEY.md §5.2 / §4.2 item 5.
set -eo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
O=build/asan
mkdir -p $O
HIPCC=/opt/rocm/bin/hipcc
CLANG=/opt/rocm/llvm/bin/clang
SAN="-fsanitize=address -fsanitize=undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined"
COMMON="-O1 -g -fPIC -std=c++17 -Icsrc/include -Iinclude"
objs=()
# an object is fresh only if newer than its source AND every header it may include
HDR=$(ls -t csrc/include/pga/*.hpp include/*.h | sed -n 1p)
for s in csrc/kernels/binary.hip csrc/kernels/real.hip csrc/kernels/perm.hip csrc/kernels/util.hip csrc/kernels/compat.hip; do
  o=$O/$(basename $s .hip).o; objs+=($o)
  [ $o -nt $s ] && [ $o -nt $HDR ] || echo "$HIPCC --offload-arch=gfx950 $COMMON -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer -c $s -o $o"
done > $O/cmds.txt
for s in csrc/engine/island.cpp csrc/engine/trace.cpp csrc/engine/jit.cpp csrc/cpu/cpu_ops.cpp csrc/cpu/cpu_real.cpp \
         csrc/cpu/cpu_perm.cpp csrc/cpu/parallel.cpp csrc/capi/pga_capi.cpp csrc/capi/comm_rccl.cpp; do
  o=$O/$(basename $s .cpp).o; objs+=($o)
  [ $o -nt $s ] && [ $o -nt $HDR ] || echo "$HIPCC -x c++ -D__HIP_PLATFORM_AMD__=1 -I/opt/rocm/include $COMMON $SAN -fno-gpu-sanitize -Wno-unused-command-line-argument -c $s -o $o"
done >> $O/cmds.txt
xargs -P ${ASAN_JOBS:-6} -I{} bash -c "{}" < $O/cmds.txt
$HIPCC --offload-arch=gfx950 -shared -o $O/libpga_asan.so "${objs[@]}" $SAN -fno-gpu-sanitize -shared-libsan \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
$CLANG -O1 -g $SAN -shared-libsan -Iinclude -o $O/capi_cpu tests/native/capi_cpu.c $O/libpga_asan.so -lm \
  -Wl,-rpath,"$R/$O" -Wl,-rpath,$($CLANG -print-resource-dir)/lib/linux -Wl,-rpath,/opt/rocm/lib
# leaks inside the HIP runtime's own initialisation are not ours
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 $O/capi_cpu $O/capi_cpu.ckpt
