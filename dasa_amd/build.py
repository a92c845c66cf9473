"""Build libdasa_hip.so (gfx950) in-tree with hipcc.

Every HIP source under dasa_amd/csrc is compiled for --offload-arch=gfx950 and linked into
dasa_amd/libdasa_hip.so, whose C-ABI is include/dasa_hip.h. The .so is git-ignored but travels to
the GPU box with the repo snapshot.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libdasa_hip.so")
BUILD_DIR = os.path.join(HERE, "build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# -fno-slp-vectorize -fno-vectorize and the packed-fp32-ops target feature off (device; the host compile ignores
# it with a warning): no packed-FP32 VALU (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32) anywhere. r05 traced the
# r04 row-split attention failure to them: with an MFMA-dense bf16x6 GEMM workgroup starting on the same CU,
# the LOW half of a packed result came back wrong on lanes 48-63 (profiles/r05/rowsplit_diag_b_m*.log: every
# bad partial is an even row of a compiler-packed row pair, lanes 48-63); built without them the same stress
# has 0 bad calls in 200 for either load form and every hand-off kernel stays bitwise reproducible
# (rowsplit_diag_c_noslp_m*.log, stress_c_noslp_all_mode1.log), at equal iteration time (bench_c_*.log).
# tests/test_host_cpu.py::test_no_packed_fp32 scans the built library's device code for them.
FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-pass-failed", "-Wno-inline-asm",
         "-fno-slp-vectorize", "-fno-vectorize", "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops",
         "-I" + os.path.join(os.path.dirname(HERE), "include")]


# Debug builds (SURVEY.md §5 "race detection / sanitizers"):
#  * `python -m dasa_amd.build --debug` -> libdasa_hip_debug.so, loaded instead of the release library when
#    DASA_DEBUG=1: device code with the DASA_DCHECK input checks compiled in (common.h; a failed check sets
#    a bit in the error word that ops.check_device_errors() raises on), host code at -O1 -g. It carries no
#    host ASan: a python process would need the ASan runtime preloaded, and GPU-side ASan / xnack builds are
#    not available on the GPU pool.
#  * `python -m dasa_amd.build --debug --host-only` -> a HOST-ONLY (--cuda-host-only: no device code, so
#    seconds to build, kernels never launched) copy of the same sources under AddressSanitizer +
#    UndefinedBehaviorSanitizer, driven by tools/asan_host_check.cpp — an executable built with
#    -fsanitize=address, so the runtime comes first — through every host-side entry point (argument
#    validation, workspace sizing, the GEMM / attention / bi-LSTM planners): tests/test_debug_cpu.py.
#  * DASA_CHECK_FINITE=1 (dasa_amd/debug.py): NaN / +Inf check of every op's outputs (release or debug lib).
OUT_DEBUG = os.path.join(HERE, "libdasa_hip_debug.so")
SAN = ["-Xarch_host", "-fsanitize=address,undefined", "-Xarch_host", "-fno-omit-frame-pointer",
       "-Xarch_host", "-fno-sanitize-recover=undefined"]
_INC = ["-I" + os.path.join(os.path.dirname(HERE), "include")]
DEBUG_FLAGS = ["-O3", "-Xarch_host", "-O1", "-g", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}",
               "-Wno-pass-failed", "-Wno-inline-asm", "-fno-slp-vectorize", "-fno-vectorize", "-Xclang", "-target-feature", "-Xclang",
               "-packed-fp32-ops", "-DDASA_DEBUG=1"] + _INC
HOSTSAN_FLAGS = ["-O1", "-g", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "--cuda-host-only",
                 "-Wno-pass-failed", "-Wno-inline-asm", "-DDASA_DEBUG=1"] + _INC + SAN
HOSTSAN_OUT = os.path.join(BUILD_DIR, "hostsan", "libdasa_hip_hostsan.so")


def build_variant(out, flags, build_dir, link_extra=(), jobs=8):
    """Compile every source with `flags` into `build_dir` and link `out` (no up-to-date checks)."""
    os.makedirs(build_dir, exist_ok=True)

    def compile_one(src):
        obj = os.path.join(build_dir, os.path.basename(src) + ".o")
        r = subprocess.run([HIPCC] + list(flags) + ["-c", src, "-o", obj], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
        return obj

    with ThreadPoolExecutor(max_workers=min(jobs, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(compile_one, sources()))
    if "--cuda-host-only" in flags:
        objs.append(_fatbin_stub(objs, build_dir))
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out] + list(link_extra) + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    return out


def _fatbin_stub(objs, build_dir):
    """A host-only object still references each translation unit's device image (__hip_fatbin_<hash>);
    define each as an empty offload bundle (the magic string, no entries) so the host code links and
    loads. Nothing in the host-sanitizer run launches a kernel."""
    names = set()
    for o in objs:
        r = subprocess.run(["nm", o], capture_output=True, text=True)
        names.update(ln.split()[-1] for ln in r.stdout.splitlines() if ln.split()[-1].startswith("__hip_fatbin_")
                     and ln.split()[0] == "U")
    src = os.path.join(build_dir, "fatbin_stub.c")
    with open(src, "w") as f:
        for n in sorted(names):
            f.write(f'__attribute__((aligned(4096))) const char {n}[32] = "__CLANG_OFFLOAD_BUNDLE__";\n')
    obj = src[:-2] + ".o"
    r = subprocess.run(["gcc", "-c", "-fPIC", src, "-o", obj], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr)
    return obj


def build_debug(host_only=False):
    """The debug library (device DCHECKs), or with host_only=True the host-sanitizer copy."""
    if host_only:
        return build_variant(HOSTSAN_OUT, HOSTSAN_FLAGS, os.path.join(BUILD_DIR, "hostsan"), link_extra=SAN[:2])
    return build_variant(OUT_DEBUG, DEBUG_FLAGS, os.path.join(BUILD_DIR, "debug"))


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _includes(path, seen=None):
    """The quoted #include files `path` pulls in, transitively (dependency check of build())."""
    import re
    seen = set() if seen is None else seen
    for name in re.findall(r'^#include "([^"]+)"', open(path).read(), flags=re.M):
        dep = os.path.normpath(os.path.join(os.path.dirname(path), name))
        if dep not in seen and os.path.exists(dep):
            seen.add(dep)
            _includes(dep, seen)
    return sorted(seen)


def _needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = sources() + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    deps.append(os.path.join(os.path.dirname(HERE), "include", "dasa_hip.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=True):
    if not force and not _needs_build():
        return OUT
    os.makedirs(BUILD_DIR, exist_ok=True)

    def compile_one(src):
        obj = os.path.join(BUILD_DIR, os.path.basename(src) + ".o")
        if (not force and os.path.exists(obj)
                and os.path.getmtime(obj) > max(os.path.getmtime(d) for d in [src] + _includes(src))):
            return obj        # up to date with the source and every header it includes
        cmd = [HIPCC] + FLAGS + ["-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
        return obj

    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(compile_one, sources()))
    tmp = OUT + ".tmp"
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(tmp, OUT)
    if verbose:
        print(f"[dasa_amd] built {OUT}", file=sys.stderr)
    return OUT


if __name__ == "__main__":
    if "--debug" in sys.argv:
        print(build_debug(host_only="--host-only" in sys.argv), file=sys.stderr)
    else:
        build(force="--force" in sys.argv)
