"""Process groups for multi-process tests: spawn `nprocs` workers on a fresh
127.0.0.1 rendezvous port.  A port picked free can still be taken before the
rank-0 store binds it (the kernel hands the same ephemeral ports to outgoing
gloo connections), so a group that dies with EADDRINUSE is started again on
another port instead of failing the test."""
import socket

import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_group(fn, nprocs: int, make_args, attempts: int = 3) -> None:
    """mp.start_processes(fn, args=make_args(port), nprocs) with a retry on a
    rendezvous port that was taken in between (workers must be idempotent)."""
    for k in range(attempts):
        try:
            mp.start_processes(fn, args=make_args(free_port()), nprocs=nprocs, start_method="spawn",
                               join=True)
            return
        except mp.ProcessRaisedException as e:
            if "EADDRINUSE" not in str(e) or k == attempts - 1:
                raise
