"""Phase clocks of the persistent bi-LSTM forward (dasa_persist_stamps): per timestep, workgroup 0's
s_memtime at step start, after the recurrent MFMAs, after the partial-sum exchange, after the cell update
and after the direction barrier; prints the median cycles of each phase and the launch time.

    python tools/lstm_stamps.py [B ...]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dasa_amd import _lib, ops  # noqa: E402


def run(B, L=80, H=1024, E=768):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(B)
    xproj = torch.randn(B, L, 2, 4 * H, device=dev, generator=g) * 0.1
    whh_f = torch.randn(4 * H, H, device=dev, generator=g) * 0.02
    whh_b = torch.randn(4 * H, H, device=dev, generator=g) * 0.02
    lens = torch.full((B,), L, dtype=torch.int32, device=dev)
    buf = torch.zeros(8 * L, dtype=torch.int64, device=dev)
    L_ = _lib.lib()
    for _ in range(3):
        ops.bilstm_fwd(xproj, whh_f, whh_b, lens, H)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        ops.bilstm_fwd(xproj, whh_f, whh_b, lens, H)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 5 * 1e3
    L_.dasa_persist_stamps(ctypes_ptr(buf))
    ops.bilstm_fwd(xproj, whh_f, whh_b, lens, H)
    torch.cuda.synchronize()
    L_.dasa_persist_stamps(None)
    st = buf.view(L, 8).cpu().numpy().astype(np.int64)
    ph = {"mfma+hload": st[1:, 1] - st[1:, 0], "exchange": st[1:, 2] - st[1:, 1], "cell+store": st[1:, 3] - st[1:, 2],
          "barrier": st[1:L - 1, 4] - st[1:L - 1, 3], "step": st[2:, 0] - st[1:-1, 0]}
    print(f"B={B}: {us:.0f} us/launch ({us / L:.2f} us/step); median cycles per phase: "
          + ", ".join(f"{k} {int(np.median(v))}" for k, v in ph.items()), flush=True)


def ctypes_ptr(t):
    import ctypes
    return ctypes.c_void_p(t.data_ptr())


if __name__ == "__main__":
    for b in ([int(v) for v in sys.argv[1:]] or [20, 160]):
        run(b)
