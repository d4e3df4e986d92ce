import os
import random
import socket
from contextlib import closing


def _ephemeral_range() -> tuple[int, int]:
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            lo, hi = (int(x) for x in f.read().split()[:2])
        return lo, hi
    except (OSError, ValueError):
        return 32768, 60999


def _bindable(port: int) -> bool:
    with closing(socket.socket(socket.AF_INET, socket.SOCK_STREAM)) as s:
        try:
            s.bind(("127.0.0.1", port))
        except OSError:
            return False
    return True


def find_free_port() -> int:
    """A free localhost port for a rendezvous store (reference ``utils/port.py:12``).

    Picked OUTSIDE the kernel's ephemeral range: a port that ``bind(0)`` handed out and released can be taken by any
    outgoing connection -- gloo and the other ranks open many -- before the store binds it (EADDRINUSE on a busy box).
    Falls back to ``bind(0)`` if no port below / above the range is free."""
    lo, hi = _ephemeral_range()
    rng = random.Random(os.getpid() ^ random.SystemRandom().getrandbits(32))
    spans = [(s, e) for s, e in ((20000, lo), (hi + 1, 65536)) if e - s > 256]
    for _ in range(64):
        if not spans:
            break
        s, e = spans[rng.randrange(len(spans))]
        port = rng.randrange(s, e)
        if _bindable(port):
            return port
    with closing(socket.socket(socket.AF_INET, socket.SOCK_STREAM)) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])
