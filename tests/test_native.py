"""The C API as a plain C consumer sees it (tests/native/capi_cpu.c on the CPU
backend), normally and under host AddressSanitizer + UBSan."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_capi_cpu_plain_c(tmp_path):
    lib = os.path.join(ROOT, "build", "libpga.so")
    if not os.path.exists(lib):
        pytest.skip("build/libpga.so not built")
    exe = tmp_path / "capi_cpu"
    subprocess.run(["gcc", "-O1", "-Wall", "-Werror", "-Iinclude", "-o", str(exe), "tests/native/capi_cpu.c",
                    "-Lbuild", "-lpga", f"-Wl,-rpath,{ROOT}/build", "-lm"], cwd=ROOT, check=True)
    r = subprocess.run([str(exe), str(tmp_path / "c.ckpt")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "capi_cpu ok" in r.stdout, r.stdout + r.stderr


def test_capi_cpu_under_asan_ubsan():
    r = subprocess.run(["bash", "tools/asan_host.sh"], cwd=ROOT, capture_output=True, text=True, timeout=1800)
    assert r.returncode == 0 and "capi_cpu ok" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
