"""One process per GPU without torchrun: the launcher behind ``bench.py --gpus N``.

Pure Python (no torch import): the parent must not touch a GPU, because the ranks it starts are the
only processes that may (one HIP context per GPU, RCCL between them).  Each rank gets the environment
torch.distributed.run would give it -- RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR
(127.0.0.1: the container hostname may not resolve) and a free MASTER_PORT -- and the parent only
waits: the ranks write their own output, and a rank that fails stops the others (their exact PIDs;
their collectives would otherwise wait for it forever).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import time


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(rank: int, world: int, port: int, base=None) -> dict:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    return env


def stop_ranks(procs, grace_s: float = 10.0) -> None:
    """SIGTERM every rank still running, wait up to grace_s, then SIGKILL the ones left (a rank stuck in an RCCL
    collective may ignore SIGTERM) and reap them: no orphan keeps a GPU."""
    live = [p for p in procs if p.poll() is None]
    for p in live:
        p.send_signal(signal.SIGTERM)
    deadline = time.monotonic() + grace_s
    for p in live:
        try:
            p.wait(timeout=max(0.0, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def launch_ranks(n: int, argv, poll_s: float = 0.2, grace_s: float = 10.0) -> int:
    """Start ``argv`` once per rank 0..n-1 and wait; returns 0, or the first failing rank's exit status
    (a rank killed by a signal reports 128 + signal, as a shell would).  On a failing rank, an exception or
    Ctrl-C in this parent, the remaining ranks are stopped (stop_ranks) before it returns or re-raises."""
    port = free_port()
    procs = []
    rc = 0
    try:
        for r in range(n):
            procs.append(subprocess.Popen(list(argv), env=rank_env(r, n, port)))
        live = list(procs)
        while live:
            time.sleep(poll_s)
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    stop_ranks(live, grace_s)
    finally:
        stop_ranks(procs, grace_s)
    return rc
