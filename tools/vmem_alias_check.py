"""Static scan of gfx950 kernel assembly for the load pattern behind r04's row-split attention failure
(profiles/r05/rowsplit_diag_a.log): a vector-memory load whose DESTINATION registers overlap the ADDRESS
registers of an older load that may still be in flight (no covering s_waitcnt vmcnt in between), or its
own address. hipcc emits it freely (the ISA reads address operands at issue), but the r04 row-split
SoftDot kernel, whose row loads were allocated this way, returned wrong data on lanes 48-63 of one row's
load under concurrent GEMM start-up, and the same kernel with one shared offset VGPR per load did not.

    python tools/vmem_alias_check.py [file.hip ...]       (default: every dasa_amd/csrc/*.hip)

Compiles each source to assembly (hipcc --cuda-device-only -S, the build's flags) and prints, per kernel,
the number of such loads (younger-load overlaps / self overlaps); exit code 0 always (a report)."""
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
VMEM = re.compile(r"^\s*(global|buffer|flat)_(load|store|atomic)\w*\s+(.*)$")
WAIT = re.compile(r"s_waitcnt\s+.*?vmcnt\((\d+)\)")
REG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)\b")


def regs(tok):
    m = REG.match(tok.strip())
    if not m:
        return set()
    if m.group(1) is not None:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return {int(m.group(3))}


def scan(asm):
    out = {}
    fn = None
    inflight = []      # address register sets of outstanding VMEM ops, oldest first
    for line in asm.splitlines():
        if re.match(r"^[_A-Za-z][\w.$]*:\s*(;.*)?$", line) and not line.startswith("."):
            name = line.split(":")[0]
            if name.startswith("_Z") or name.startswith("dasa"):
                fn = name
                out.setdefault(fn, [0, 0, 0])
                inflight = []
            continue
        if fn is None:
            continue
        if "s_endpgm" in line:
            inflight = []
            continue
        w = WAIT.search(line)
        if w:
            n = int(w.group(1))
            inflight = inflight[len(inflight) - n:] if n < len(inflight) else inflight
            continue
        m = VMEM.match(line)
        if not m:
            continue
        ops = [o.strip() for o in m.group(3).split(",")]
        kind = m.group(2)
        out[fn][0] += 1
        if kind == "load" and "lds" not in line.split()[0]:
            dst, addr = regs(ops[0]), regs(ops[1]) if len(ops) > 1 else set()
            if any(dst & a for a in inflight):
                out[fn][1] += 1
            if dst & addr:
                out[fn][2] += 1
        else:
            addr = regs(ops[0]) if kind == "store" and False else regs(ops[1] if kind != "store" else ops[0])
        inflight.append(addr)
    return out


def main():
    srcs = sys.argv[1:] or sorted(glob.glob(os.path.join(ROOT, "dasa_amd", "csrc", "*.hip")))
    flags = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-Wno-pass-failed", "-Wno-inline-asm",
             "-I" + os.path.join(ROOT, "include"), "--cuda-device-only", "-S"]
    total = 0
    for src in srcs:
        with tempfile.TemporaryDirectory() as d:
            s = os.path.join(d, "k.s")
            r = subprocess.run([HIPCC] + flags + [src, "-o", s], capture_output=True, text=True)
            if r.returncode != 0:
                print(f"{src}: compile failed\n{r.stderr[-1000:]}")
                continue
            res = scan(open(s).read())
        for fn, (nv, younger, self_) in sorted(res.items()):
            if younger or self_:
                total += 1
                print(f"{os.path.basename(src):18s} {fn[:90]:90s} vmem {nv:4d}  dst-over-inflight-addr {younger:3d}  "
                      f"dst-over-own-addr {self_:3d}")
    print(f"kernels with the pattern: {total}")


if __name__ == "__main__":
    main()
