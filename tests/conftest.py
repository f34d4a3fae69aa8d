import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built extension")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")


def free_port() -> int:
    """A free TCP port for a rendezvous, drawn OUTSIDE the kernel's ephemeral range (32768+):
    an ephemeral port found free here can be taken by any outgoing connection on the box before
    the store binds it (EADDRINUSE flake seen on a shared GPU box)."""
    import random
    rng = random.Random()
    for _ in range(200):
        p = rng.randrange(15000, 30000)
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def port():
    return free_port()
