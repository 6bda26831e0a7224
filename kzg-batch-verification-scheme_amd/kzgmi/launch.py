"""Process-per-GPU launcher: `python bench.py --gpus N` without torchrun.

The multi-GPU path (kzgmi/distributed.py) runs one process per GPU with the torchrun
environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT).  When a script is
started directly with N > 1 ranks requested and no WORLD_SIZE in its environment, `launch`
starts N copies of it with that environment set (rank r on local device r) and waits:

- rank 0's stdout is the parent's stdout (the one JSON line bench.py prints); the other
  ranks' stdout is discarded, every rank's stderr is inherited;
- the first rank that fails ends the job: the others are terminated (a rank left waiting in a
  collective would otherwise hang) and the parent returns that rank's exit status;
- the parent never touches a GPU (it must not: it spawns the processes that do), so it is
  called before torch or libkzgmi initialise HIP.

Rendezvous is on 127.0.0.1 (the container hostname may not resolve).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from typing import List, Optional, Sequence


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(base: dict, rank: int, world: int, port: int) -> dict:
    env = dict(base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    return env


def launch(argv: Sequence[str], nprocs: int, port: Optional[int] = None, poll_s: float = 0.2,
           stop_grace_s: float = 10.0) -> int:
    """Run `python argv...` as nprocs ranks; return 0 if every rank exits 0, else the first
    failing rank's exit status (a signal death -s maps to 128 + s)."""
    if nprocs < 1:
        raise ValueError("nprocs must be >= 1")
    port = port or free_port()
    procs: List[subprocess.Popen] = []
    for r in range(nprocs):
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=rank_env(os.environ, r, nprocs, port),
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    failed = None
    try:
        while True:
            alive = False
            for r, p in enumerate(procs):
                rc = p.poll()
                if rc is None:
                    alive = True
                elif rc != 0 and failed is None:
                    failed = (r, rc)
            if failed is not None or not alive:
                break
            time.sleep(poll_s)
    finally:
        if failed is not None or any(p.poll() is None for p in procs):
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            deadline = time.time() + stop_grace_s
            for p in procs:
                try:
                    p.wait(timeout=max(0.0, deadline - time.time()))
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
    if failed is None:
        return 0
    r, rc = failed
    sys.stderr.write("[launch] rank %d exited with status %d; stopped the other ranks\n" % (r, rc))
    return rc if rc > 0 else 128 - rc


def maybe_launch(argv: Sequence[str], gpus: int) -> Optional[int]:
    """If `gpus` > 1 ranks are asked for and this process is not itself a rank (no WORLD_SIZE),
    run the ranks and return the job's exit status; otherwise None (this process is a rank)."""
    if gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    return launch(argv, gpus)
