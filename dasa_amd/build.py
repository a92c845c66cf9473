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
FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-pass-failed", "-Wno-inline-asm",
         "-I" + os.path.join(os.path.dirname(HERE), "include")]


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


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

    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    headers.append(os.path.join(os.path.dirname(HERE), "include", "dasa_hip.h"))
    newest_header = max(os.path.getmtime(h) for h in headers)

    def compile_one(src):
        obj = os.path.join(BUILD_DIR, os.path.basename(src) + ".o")
        if (not force and os.path.exists(obj) and os.path.getmtime(obj) > os.path.getmtime(src)
                and os.path.getmtime(obj) > newest_header):
            return obj        # up to date (every source includes the headers, so a header edit rebuilds all)
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
    build(force="--force" in sys.argv)
