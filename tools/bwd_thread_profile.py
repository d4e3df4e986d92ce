"""Debug hook (SCALING_AMD_DEBUG_HOOKS=tools/bwd_thread_profile.py): cProfile of the autograd device thread, where the
backward's Python (custom autograd functions, hooks) runs -- a main-thread profile only sees ``run_backward``.  The
profiler is switched on for that thread by the first embedding backward (the last node of a step's backward), so it
covers every later backward; rank 0 writes gpurun_out/bwd_thread.prof at exit."""
import atexit
import cProfile
import os
import threading

from scaling_amd.ops import embedding

_main = threading.get_ident()
_prof = {}
_orig = embedding._Embed.backward


def _backward(ctx, dy):
    if threading.get_ident() != _main and "p" not in _prof:
        _prof["p"] = cProfile.Profile()
        _prof["p"].enable()
    return _orig(ctx, dy)


embedding._Embed.backward = staticmethod(_backward)


def _dump() -> None:
    if "p" in _prof and os.environ.get("RANK", "0") == "0":
        os.makedirs("gpurun_out", exist_ok=True)
        _prof["p"].dump_stats("gpurun_out/bwd_thread.prof")


atexit.register(_dump)
