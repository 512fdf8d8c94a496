"""Rendezvous ports for the multi-process tests. A port the kernel hands out for bind(0) comes from
the ephemeral range, where any outgoing connection (a previous launcher's sockets, RCCL's own) may
take it again before the launcher binds it (EADDRINUSE). These ports come from below that range
(20000-32767), picked at random and checked free."""
import random
import socket


def free_port() -> int:
    rng = random.SystemRandom()
    for _ in range(200):
        p = rng.randrange(20000, 32000)
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
        except OSError:
            continue
        finally:
            s.close()
        return p
    raise RuntimeError("no free port in 20000-32000")
