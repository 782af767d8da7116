"""Self-launch of N rank processes for ``bench.py --gpus N`` (one process per
GPU, ballots sharded, partial tallies all-gathered over RCCL).

When a program is started without a launcher (no ``WORLD_SIZE`` in the environment) and
asks for N > 1 ranks, it re-runs itself as N child processes with the variables
``torch.distributed.run`` would set (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE,
MASTER_ADDR=127.0.0.1, MASTER_PORT).  This module imports nothing GPU-related: the parent
must not initialise HIP before it starts the children (it never execs; it waits for them
and returns the worst exit status).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from typing import List, Optional, Sequence


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_env(rank: int, world: int, port: int, base: Optional[dict] = None) -> dict:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    return env


def run_ranks(script: str, argv: Sequence[str], world: int, timeout: Optional[float] = None,
              env: Optional[dict] = None, poll_s: float = 0.2) -> int:
    """Run `python script argv...` as `world` rank processes; -> 0 when every rank succeeds,
    else the exit status of the FIRST rank that failed.  Every child is polled: as soon as one
    exits non-zero the others are killed (a dead rank would otherwise leave its peers blocked
    in a collective until the watchdog fires), so the caller sees the failing rank's status at
    once.  Ranks still running after `timeout` seconds are killed and 124 is returned."""
    port = free_port()
    procs: List[subprocess.Popen] = []
    for r in range(world):
        procs.append(subprocess.Popen([sys.executable, script, *argv], env=rank_env(r, world, port, env)))
    deadline = None if timeout is None else time.monotonic() + timeout
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if deadline is not None and time.monotonic() > deadline:
                rc = 124
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for p in procs:
            p.wait()
    return rc


def launched_world() -> Optional[int]:
    """WORLD_SIZE set by a launcher (torch.distributed.run or run_ranks), else None."""
    w = os.environ.get("WORLD_SIZE")
    return int(w) if w else None
