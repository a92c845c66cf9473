"""The debug modes of the HIP path on the CPU (SURVEY.md §5 "race detection / sanitizers"):
(1) the C-ABI's host code under AddressSanitizer + UndefinedBehaviorSanitizer — a host-only sanitized
copy of libdasa_hip driven through every pre-launch path by tools/asan_host_check.cpp (no kernel is
launched); (2) the DASA_CHECK_FINITE output check (dasa_amd/debug.py) and its wrapping of dasa_amd.ops;
(3) the device-check library flavour compiles (DASA_DCHECK in common.h)."""
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_host_code_under_asan_ubsan():
    from dasa_amd import build
    lib = build.build_debug(host_only=True)
    d = os.path.dirname(lib)
    exe = os.path.join(d, "asan_host_check")
    r = subprocess.run(["/opt/rocm/lib/llvm/bin/clang++", "-std=c++17", "-g", "-fsanitize=address,undefined",
                        "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined",
                        "-I" + os.path.join(ROOT, "include"), os.path.join(ROOT, "tools", "asan_host_check.cpp"),
                        "-L" + d, "-ldasa_hip_hostsan", "-Wl,-rpath," + d, "-o", exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "0 failed" in r.stdout and "Sanitizer" not in r.stderr, r.stderr[-4000:]
    n = int(r.stdout.split("asan_host_check:")[1].split()[0])
    assert n > 10000, n


def test_check_finite_outputs():
    from dasa_amd import debug
    from dasa_amd._lib import DasaError
    ok = (torch.tensor([1.0, -float("inf")]), torch.zeros(3, dtype=torch.int64))
    assert debug.check_outputs("x", ok, strict=False) is ok          # -inf is the reference's mask value
    with pytest.raises(DasaError, match="non-finite output of ops.x"):
        debug.check_outputs("x", ok, strict=True)
    with pytest.raises(DasaError, match=r"output 1, .*nan at \[2\]"):
        debug.check_outputs("x", [torch.ones(2), torch.tensor([0.0, 1.0, float("nan")])], strict=False)
    with pytest.raises(DasaError):
        debug.check_outputs("x", {"a": torch.tensor([float("inf")])}, strict=False)


def test_check_finite_wraps_ops_in_a_fresh_process():
    code = ("import dasa_amd.ops as o, dasa_amd.graph as g; "
            "assert getattr(o.linear, '__dasa_checked__', False) and getattr(o.softdot_fwd, '__dasa_checked__', False); "
            "assert not getattr(o.check_device_errors, '__dasa_checked__', False); assert not g.ENABLED; print('ok')")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, DASA_CHECK_FINITE="1"))
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def test_device_check_flavour_compiles():
    """One translation unit of the DASA_DEBUG device build (the DCHECKs of the policy head)."""
    from dasa_amd import build
    out = os.path.join(build.BUILD_DIR, "debug_probe_policy.o")
    os.makedirs(build.BUILD_DIR, exist_ok=True)
    r = subprocess.run([build.HIPCC] + build.DEBUG_FLAGS + ["-c", os.path.join(build.CSRC, "policy.hip"), "-o", out],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
