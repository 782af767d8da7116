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
              env: Optional[dict] = None) -> int:
    """Run `python script argv...` as `world` rank processes; -> the first non-zero exit
    status (0 when all ranks succeed).  A rank that fails makes the others' collectives
    error out; any rank still running after `timeout` seconds is killed."""
    port = free_port()
    procs: List[subprocess.Popen] = []
    for r in range(world):
        procs.append(subprocess.Popen([sys.executable, script, *argv], env=rank_env(r, world, port, env)))
    deadline = None if timeout is None else time.monotonic() + timeout
    rc = 0
    try:
        for p in procs:
            left = None if deadline is None else max(1.0, deadline - time.monotonic())
            code = p.wait(timeout=left)
            if code != 0 and rc == 0:
                rc = code
    except subprocess.TimeoutExpired:
        rc = 124
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def launched_world() -> Optional[int]:
    """WORLD_SIZE set by a launcher (torch.distributed.run or run_ranks), else None."""
    w = os.environ.get("WORLD_SIZE")
    return int(w) if w else None
