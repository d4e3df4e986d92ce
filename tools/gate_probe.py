"""Probe of the stream-gate primitive (hipStreamWaitValue32 on a host-written flag word) behind the asynchronous
rehearsal collectives: a stream must hold its later work until the host writes the flag, then run it.
    python tools/gate_probe.py        (flag words in coherent pinned host memory)"""
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scaling_amd.ops._ext import ext  # noqa: E402

x = torch.zeros(1, device="cuda")
s = torch.cuda.Stream()
base = ext().gate_flags_alloc(4)
print(f"flags at {base:#x}, read {ext().gate_flag_read(base, 0)}", flush=True)
ev = torch.cuda.Event()
with torch.cuda.stream(s):
    x.fill_(1)
    ext().gate_stream_wait(base, 0, 1)
    x.add_(1)
    ev.record(s)
t0 = time.time()
threading.Timer(0.3, lambda: ext().gate_flag_write(base, 0, 1)).start()
time.sleep(0.1)
early = ev.query()
s.synchronize()
dt = time.time() - t0
print(f"done before the flag: {early}; released after {dt:.3f} s; x = {x.item()}", flush=True)
ok = (not early) and dt >= 0.29 and x.item() == 2.0
# a second gate on the same word at a higher generation, released at once
with torch.cuda.stream(s):
    ext().gate_stream_wait(base, 0, 2)
    x.add_(1)
ext().gate_flag_write(base, 0, 2)
s.synchronize()
ok = ok and x.item() == 3.0
print(f"{'OK' if ok else 'FAILED'}", flush=True)
sys.exit(0 if ok else 1)
