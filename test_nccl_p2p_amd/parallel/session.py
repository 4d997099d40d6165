"""Native sessions wired up from a torch.distributed-style environment.

Control plane: ``torch.distributed`` (gloo, CPU) carries only the bootstrap
port of the native TCP star; the native engine then creates its own RCCL
communicator (ncclGetUniqueId on rank 0, broadcast over that star,
ncclCommInitRankConfig) and drives ncclSend/ncclRecv over xGMI itself.  This
replaces the reference's MPI_Bcast of the ncclUniqueId
(/root/reference/p2p_matrix.cc:115-120) for torchrun-launched jobs.
"""

from __future__ import annotations

import datetime
import os
from typing import NamedTuple, Optional

import torch.distributed as dist

from .._native import require_native


class DistEnv(NamedTuple):
    rank: int
    world: int
    local_rank: int
    master_addr: str


def dist_env() -> DistEnv:
    return DistEnv(
        int(os.environ.get("RANK", 0)),
        int(os.environ.get("WORLD_SIZE", 1)),
        int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", 0))),
        os.environ.get("MASTER_ADDR", "127.0.0.1"),
    )


def init_control_plane(backend: str = "gloo", timeout_s: float = 600.0) -> DistEnv:
    """Initialises torch.distributed (env://) when world > 1."""
    env = dist_env()
    if env.world > 1 and not dist.is_initialized():
        dist.init_process_group(backend=backend, rank=env.rank, world_size=env.world,
                                timeout=datetime.timedelta(seconds=timeout_s))
    return env


def create_session(transport: str = "rccl", device: Optional[int] = None, timeout_s: float = 300.0):
    """Returns a native ``Session``; collective over the torch.distributed group."""
    n = require_native()
    env = init_control_plane()
    dev = env.local_rank if device is None else device
    if env.world == 1:
        return n.Session(0, 1, device=dev, transport=transport, timeout_s=timeout_s)
    listener = n.TcpListener(0) if env.rank == 0 else None
    box = [listener.port if listener is not None else None]
    dist.broadcast_object_list(box, src=0)
    return n.Session(env.rank, env.world, host=env.master_addr, port=int(box[0]), device=dev,
                     transport=transport, timeout_s=timeout_s, listener=listener)
