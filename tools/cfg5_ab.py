"""A/B of the configs[4] leg under forced bf16 GEMM tile forms (tuning): runs bench.cfg5_leg once per
form, in alternating order, and prints decisions/s and the gemm_bf16 family line of each.

    python tools/cfg5_ab.py [form ...]      (form -1 = the default plan)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main(forms):
    import torch
    from dasa_amd import _lib
    torch.cuda.set_device(0)
    forms_argv, sys.argv = sys.argv[1:], [sys.argv[0]]
    a = bench.parse()
    del forms_argv
    L = _lib.lib()
    for f in forms + forms[::-1]:
        L.dasa_gemm_force_config(-1 if f < 0 else (1 << 20) + f)
        r = bench.cfg5_leg(a)
        g = r["bf16"]["kernels"].get("gemm_bf16", {})
        print(json.dumps({"form": f, "bf16": r["bf16"]["value"], "fp32": r["fp32"]["value"],
                          "gemm_bf16": {k: g.get(k) for k in ("launches", "device_ms", "avg_launch_us", "achieved")}}),
              flush=True)
    L.dasa_gemm_force_config(-1)


if __name__ == "__main__":
    main([int(v) for v in sys.argv[1:]] or [-1, 2, 9])
