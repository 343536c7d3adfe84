"""Self-launch of N rank processes (one per GPU) for a script invoked as `script --gpus N`.

The driver may start `bench.py --gpus N` directly, without torch.distributed.run.  Then the
first process (which must not have touched a GPU yet: no HIP call, no torch.cuda query that
initialises the runtime) starts `python -m torch.distributed.run --nproc-per-node N` as a CHILD
process with the same arguments, waits for it and returns its exit code -- no exec of the
current process, so nothing GPU-initialised is ever replaced.  The ranks find WORLD_SIZE set
and run normally.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def needs_spawn(n_procs: int) -> bool:
    return n_procs > 1 and "WORLD_SIZE" not in os.environ


def spawn(n_procs: int, script: str, argv: list, env_extra: dict | None = None, timeout: float | None = None) -> int:
    """Run `script argv` as n_procs ranks under torch.distributed.run (127.0.0.1 rendezvous);
    returns the launcher's exit code.  Rank 0's stdout passes through unchanged."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n_procs}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), script, *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts
    if env_extra:
        env.update(env_extra)
    return subprocess.run(cmd, env=env, timeout=timeout).returncode
