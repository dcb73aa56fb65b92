#!/usr/bin/env python3
"""Build every native artefact of the framework for gfx950, in-tree.

Outputs
  libpga_amd/_C.so      torch extension (Island runtime + kernels + CPU backend)
  build/libpga.so       reference-compatible C API (include/pga.h), no torch
  build/libpga.a        same, relocatable device code (-fgpu-rdc) so user
                        __device__ objective/crossover/mutate function pointers
                        link into the library kernels (reference Makefile:2-3 uses
                        nvcc -dc for the same reason)
  build/examples/*      reference examples E1/E2/E3 rewritten against pga.h

Drives hipcc through a generated ninja file (parallel, incremental).  No
hipify, no torch cpp_extension JIT: the .so files live in the tree so they
travel with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "build")
ARCH = os.environ.get("PGA_ARCH", "gfx950")

# kernel sources built once per -D variant (tag, flags): the BINARY launchers
# per group size, so the heaviest instantiation sets compile in parallel
SPLIT = {"csrc/kernels/binary_gs.hip": [(f"gs{g}", f"-DPGA_BIN_GS={g}") for g in (1, 2, 4, 8, 16, 32, 64)]}
KERNELS = ["csrc/kernels/binary.hip", "csrc/kernels/real.hip", "csrc/kernels/perm.hip",
           "csrc/kernels/util.hip", "csrc/kernels/compat.hip", "csrc/kernels/qubo.hip",
           "csrc/kernels/sort.hip", "csrc/kernels/binary_batch.hip", "csrc/kernels/real_batch.hip"]
HOST = ["csrc/engine/island.cpp", "csrc/engine/trace.cpp", "csrc/engine/jit.cpp", "csrc/cpu/cpu_ops.cpp", "csrc/cpu/cpu_real.cpp", "csrc/cpu/cpu_perm.cpp", "csrc/cpu/parallel.cpp"]
CAPI = ["csrc/capi/pga_capi.cpp", "csrc/capi/comm.cpp", "csrc/capi/comm_rccl.cpp"]
COMPAT = []
BINDINGS = ["csrc/python/bindings.cpp", "csrc/python/comm_bind.cpp"]


def torch_paths():
    import torch  # noqa: WPS433
    from torch.utils import cpp_extension
    inc = cpp_extension.include_paths()
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def pybind_includes():
    import pybind11
    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


def obj_path(src: str, tag: str) -> str:
    base = os.path.splitext(src.replace("/", "_"))[0]
    return os.path.join("build", "obj", f"{base}.{tag}.o")


def write_ninja(opt: str, with_torch: bool) -> str:
    common = f"-O{opt} -fPIC -std=c++17 -Icsrc/include -Iinclude -Wall -Wno-unused-function -Wno-unused-variable"
    hip_flags = f"{common} -x hip --offload-arch={ARCH} -munsafe-fp-atomics -ffp-contract=fast"
    rdc_flags = f"{hip_flags} -fgpu-rdc"
    host_flags = f"{common} -x c++ -D__HIP_PLATFORM_AMD__=1 -I/opt/rocm/include"
    lines = [
        "ninja_required_version = 1.3",
        "hipcc = /opt/rocm/bin/hipcc",
        f"hip_flags = {hip_flags}",
        f"rdc_flags = {rdc_flags}",
        f"host_flags = {host_flags}",
        "rule hip",
        "  command = $hipcc $hip_flags $extra -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIP $in",
        "rule rdc",
        "  command = $hipcc $rdc_flags $extra -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIP-RDC $in",
        "rule jitbc",
        "  command = $hipcc $hip_flags -Xclang -disable-llvm-passes -fgpu-rdc --cuda-device-only -emit-llvm $extra -c $in -o $out",
        "  description = HIP-BC $out",
        "rule host",
        "  command = $hipcc $host_flags $extra -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "rule link_so",
        f"  command = $hipcc --offload-arch={ARCH} -shared -o $out $in $ldflags",
        "  description = LINK $out",
        "rule link_rdc_so",
        f"  command = $hipcc --offload-arch={ARCH} -fgpu-rdc --hip-link -shared -o $out $in $ldflags",
        "  description = LINK-RDC $out",
        "rule ar",
        "  command = rm -f $out && /opt/rocm/lib/llvm/bin/llvm-ar rcs $out $in",
        "  description = AR $out",
        "rule cc",
        "  command = gcc -O2 -o $out $in",
        "  description = CC $out",
        "rule cexe",
        "  command = gcc -O2 -Iinclude -o $out $in -Lbuild -lpga -Wl,-rpath,'$$ORIGIN/..'",
        "  description = CC $out",
        "rule link_exe",
        f"  command = $hipcc --offload-arch={ARCH} $extra -o $out $in $ldflags",
        "  description = LINK $out",
    ]
    core_objs = []
    for s in KERNELS:
        o = obj_path(s, "k")
        lines.append(f"build {o}: hip {s}")
        core_objs.append(o)
    split_rdc = []
    for s, variants in SPLIT.items():
        for tag, flags in variants:
            o = obj_path(s, f"{tag}.k")
            lines.append(f"build {o}: hip {s}")
            lines.append(f"  extra = {flags}")
            core_objs.append(o)
            o = obj_path(s, f"{tag}.rdc")
            lines.append(f"build {o}: rdc {s}")
            lines.append(f"  extra = {flags}")
            split_rdc.append(o)
    for s in HOST:
        o = obj_path(s, "h")
        lines.append(f"build {o}: host {s}")
        core_objs.append(o)

    # C API shared library (non-rdc: built-in objectives and host-side logic)
    capi_objs = []
    for s in CAPI:
        o = obj_path(s, "h")
        lines.append(f"build {o}: host {s}")
        capi_objs.append(o)
    compat_objs = []
    for s in COMPAT:
        o = obj_path(s, "k")
        lines.append(f"build {o}: hip {s}")
        compat_objs.append(o)
    lines.append(f"build build/libpga.so: link_so {' '.join(core_objs + capi_objs + compat_objs)}")
    lines.append("  ldflags = -Wl,-soname,libpga.so -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib")

    # static rdc library for user device function pointers
    rdc_objs = list(split_rdc)
    for s in KERNELS + COMPAT:
        o = obj_path(s, "rdc")
        lines.append(f"build {o}: rdc {s}")
        rdc_objs.append(o)
    lines.append(f"build build/libpga.a: ar {' '.join(rdc_objs + [obj_path(s, 'h') for s in HOST + CAPI])}")

    # examples
    ex = []
    for name in ("e1_onemax_float", "e2_knapsack", "e3_tsp", "onemax_bits"):
        src = f"examples/{name}.hip"
        if not os.path.exists(os.path.join(ROOT, src)):
            continue
        o = obj_path(src, "rdc")
        lines.append(f"build {o}: rdc {src}")
        exe = f"build/examples/{name}"
        lines.append(f"build {exe}: link_exe {o} build/libpga.a")
        lines.append(f"  extra = -fgpu-rdc --hip-link")
        lines.append("  ldflags = -lpthread -L/opt/rocm/lib -lrccl")
        ex.append(exe)
    for name in ("onemax_bits", "islands_multi_gpu", "islands_multiproc"):
        src = f"examples/{name}.c"
        if not os.path.exists(os.path.join(ROOT, src)):
            continue
        exe = f"build/examples/{name}"
        lines.append(f"build {exe}: cexe {src} | build/libpga.so")
        ex.append(exe)
    if os.path.exists(os.path.join(ROOT, "examples/gen_tsp.c")):
        lines.append("build build/examples/gen_tsp: cc examples/gen_tsp.c")
        ex.append("build/examples/gen_tsp")

    # reference-semantics baseline (bench/refsem.hip)
    if os.path.exists(os.path.join(ROOT, "bench/refsem.hip")):
        o = obj_path("bench/refsem.hip", "k")
        lines.append(f"build {o}: hip bench/refsem.hip")
        lines.append(f"build build/bench/refsem: link_exe {o}")
        lines.append("  ldflags = ")
        ex.append("build/bench/refsem")

    # the hot BINARY generation kernel as LLVM bitcode, one file per variant,
    # for linking hipRTC-compiled user objectives into it at run time (jit.cpp)
    jit_bc = []
    for gs in (1, 2, 4, 8, 16, 32, 64):
        for full in (0, 1):
            for dense in (0, 1):
                out = f"build/jit/gen_{gs}_{full}_{dense}.bc"
                # no depfile from a device-only bitcode compile: the headers are listed
                hdrs = " ".join(f"csrc/include/pga/{h}.hpp" for h in ("binary_dev", "tp", "core", "device", "ops"))
                lines.append(f"build {out}: jitbc csrc/kernels/jitgen.hip | {hdrs}")
                lines.append(f"  extra = -DPGA_JIT_GS={gs} -DPGA_JIT_FULL={full} -DPGA_JIT_DENSE={dense}")
                jit_bc.append(out)
        out = f"build/jit/gen_real_{gs}.bc"
        hdrs = " ".join(f"csrc/include/pga/{h}.hpp" for h in ("real_dev", "real_ops", "tp", "core", "device", "ops"))
        lines.append(f"build {out}: jitbc csrc/kernels/jitgen_real.hip | {hdrs}")
        lines.append(f"  extra = -DPGA_JIT_GS={gs}")
        jit_bc.append(out)

    defaults = ["build/libpga.so", "build/libpga.a"] + ex + jit_bc
    if with_torch:
        inc, lib, abi = torch_paths()
        tflags = " ".join(f"-isystem {p}" for p in inc + pybind_includes())
        bind_objs = []
        for s in BINDINGS:
            o = obj_path(s, "t")
            lines.append(f"build {o}: host {s}")
            lines.append(f"  extra = {tflags} -DTORCH_EXTENSION_NAME=_C -DTORCH_API_INCLUDE_EXTENSION_H "
                         f"-D_GLIBCXX_USE_CXX11_ABI={abi} -Wno-deprecated-declarations")
            bind_objs.append(o)
        # the engine's RCCL transport (comm_bind.cpp): librccl.so.1 resolves to
        # the copy torch has already loaded (same soname), one RCCL per process
        comm_objs = [obj_path(s, "h") for s in ("csrc/capi/comm.cpp", "csrc/capi/comm_rccl.cpp")]
        lines.append(f"build libpga_amd/_C.so: link_so {' '.join(core_objs + bind_objs + comm_objs)}")
        lines.append(f"  ldflags = -L{lib} -Wl,-rpath,{lib} -lc10 -lc10_hip -ltorch -ltorch_cpu -ltorch_hip "
                     f"-ltorch_python -L/opt/rocm/lib -lrccl")
        defaults.insert(0, "libpga_amd/_C.so")
    lines.append("default " + " ".join(defaults))
    path = os.path.join(BUILD, "build.ninja")
    os.makedirs(os.path.join(BUILD, "obj"), exist_ok=True)
    os.makedirs(os.path.join(BUILD, "examples"), exist_ok=True)
    os.makedirs(os.path.join(BUILD, "jit"), exist_ok=True)
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return path


def build(jobs: int | None = None, opt: str = "3", with_torch: bool = True, targets=()) -> None:
    path = write_ninja(opt, with_torch)
    ninja = shutil.which("ninja") or "ninja"
    cmd = [ninja, "-f", path, "-C", ROOT]
    if jobs:
        cmd += ["-j", str(jobs)]
    cmd += list(targets)
    subprocess.run(cmd, check=True, cwd=ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 8))
    ap.add_argument("-O", "--opt", default="3")
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("targets", nargs="*")
    a = ap.parse_args()
    build(a.jobs, a.opt, not a.no_torch, a.targets)


if __name__ == "__main__":
    sys.exit(main())
