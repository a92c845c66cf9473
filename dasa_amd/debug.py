"""NaN / Inf check mode of the HIP path (SURVEY.md §5 "race detection / sanitizers": the debug build's
NaN/Inf check; dasa_amd/build.py has the device-check and host-sanitizer libraries).

DASA_CHECK_FINITE=1 wraps every tensor-producing entry point of `dasa_amd.ops` (the one place the product
calls the C-ABI): after each call its outputs are checked on the device and a NaN or +Inf raises DasaError
naming the op and the first bad element — so a kernel that writes garbage is caught at the launch that
wrote it, not 35 decision steps later in a loss. -Inf is allowed (the reference's own mask value:
model.py:284 masked_fill(-inf), agent_dg.py:841 candidate logits, the policy head's log-probabilities);
DASA_CHECK_FINITE=strict rejects it too. Each check synchronises the stream, so hipGraph capture and replay
are switched off while the mode is on (graph.ENABLED, the agent's step / training graphs) and the mode is
for debugging runs only, never for timing."""
import functools
import os

import torch

MODE = os.environ.get("DASA_CHECK_FINITE", "0").strip().lower()

# ops functions that produce no device output (settings, hooks, host reads)
_SKIP = {"check", "check_device_errors", "attn_set_mode", "attn_debug_buffer", "set_gemm_emulation",
         "register_concurrent_stream", "force_persist_timeout", "bf16_matmul"}


def active():
    return MODE not in ("", "0", "off", "false")


def _tensors(x):
    if isinstance(x, torch.Tensor):
        yield x
    elif isinstance(x, (tuple, list)):
        for y in x:
            yield from _tensors(y)
    elif isinstance(x, dict):
        for y in x.values():
            yield from _tensors(y)


def check_outputs(name, out, strict=None):
    """Raise DasaError if a floating-point tensor in `out` holds a NaN or +Inf (any non-finite value with
    strict). Skipped while a stream is being captured (no sync possible there)."""
    from ._lib import DasaError
    strict = (MODE == "strict") if strict is None else strict
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        return out
    for i, t in enumerate(_tensors(out)):
        if not t.is_floating_point() or t.numel() == 0:
            continue
        bad = ~torch.isfinite(t) if strict else (torch.isnan(t) | torch.isposinf(t))
        if bool(bad.any()):
            idx = torch.nonzero(bad)[0].tolist()
            raise DasaError(f"non-finite output of ops.{name} (output {i}, shape {tuple(t.shape)}): "
                            f"{t[tuple(idx)].item()} at {idx}")
    return out


def _wrap(name, fn):
    @functools.wraps(fn)
    def checked(*a, **k):
        return check_outputs(name, fn(*a, **k))
    checked.__dasa_checked__ = True
    return checked


def install(module):
    """Wrap the module's public functions (dasa_amd.ops) with the output check."""
    for name in dir(module):
        fn = getattr(module, name)
        if name.startswith("_") or name in _SKIP or not callable(fn) or isinstance(fn, type):
            continue
        if getattr(fn, "__module__", None) != module.__name__ or getattr(fn, "__dasa_checked__", False):
            continue
        setattr(module, name, _wrap(name, fn))
