import socket
from contextlib import closing


def find_free_port() -> int:
    """Bind port 0 on localhost and return the chosen free port (reference ``utils/port.py:12``)."""
    with closing(socket.socket(socket.AF_INET, socket.SOCK_STREAM)) as s:
        s.bind(("127.0.0.1", 0))
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        return int(s.getsockname()[1])
