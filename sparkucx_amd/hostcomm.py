"""Host collectives for the exchange's host backend (sgx_comm_init_host, include/sgx.h).

The engine runs the whole exchange -- counts all-gather, sgx_plan_exchange, the all-to-all
of the partition-contiguous map output into the [source rank][my reducers] receive layout,
block fetches from HBM -- and calls back into these two functions for the byte movement
between processes.  ``TorchDistributedCollectives`` implements them over a
``torch.distributed`` process group (gloo on the host): the path for ranks that share one
GPU (RCCL refuses two ranks on one device) and the fake backend of SURVEY §4.  On one GPU per
rank the engine's RCCL backend (``ShuffleEngine.comm_init``) moves the bytes over xGMI
instead; both produce the same blocks.
"""
from __future__ import annotations

import ctypes
import sys
import traceback

import numpy as np

from . import _lib


def _view(addr: int, nbytes: int) -> np.ndarray:
    """A writable uint8 view of host memory at ``addr`` (no copy)."""
    if nbytes <= 0:
        return np.zeros(0, dtype=np.uint8)
    return np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(addr))


class TorchDistributedCollectives:
    """all-gather / all-to-all-v of raw bytes over a torch.distributed group (gloo)."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def allgather(self, send: np.ndarray) -> np.ndarray:
        import torch

        t = torch.from_numpy(np.ascontiguousarray(send))
        outs = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(outs, t, group=self.group)
        return torch.cat(outs).numpy()

    def alltoallv(self, send: np.ndarray, send_counts, recv_counts) -> np.ndarray:
        import torch

        out = torch.empty(int(sum(recv_counts)), dtype=torch.uint8)
        self.dist.all_to_all_single(out, torch.from_numpy(np.ascontiguousarray(send)),
                                    output_split_sizes=[int(x) for x in recv_counts],
                                    input_split_sizes=[int(x) for x in send_counts], group=self.group)
        return out.numpy()


class HostCommBinding:
    """The C callbacks handed to sgx_comm_init_host (kept alive as long as the engine)."""

    def __init__(self, collectives):
        self.coll = collectives

        def allgather(user, send, nbytes, recv):
            try:
                got = self.coll.allgather(_view(send, nbytes).copy())
                dst = _view(recv, got.nbytes)
                dst[:] = got
                return 0
            except Exception:  # noqa: BLE001 - reported to the engine as SGX_ERR_COMM
                traceback.print_exc(file=sys.stderr)
                return 1

        def alltoallv(user, send, scounts, sdispls, recv, rcounts, rdispls):
            try:
                P = self.coll.world
                sc = [scounts[j] for j in range(P)]
                sd = [sdispls[j] for j in range(P)]
                rc = [rcounts[j] for j in range(P)]
                rd = [rdispls[j] for j in range(P)]
                total = sum(sc)
                src = _view(send, sd[-1] + sc[-1] if P else 0)
                # segments in destination order (the engine's plan lays them out contiguously)
                packed = np.concatenate([src[sd[j]:sd[j] + sc[j]] for j in range(P)]) if total else \
                    np.zeros(0, np.uint8)
                got = self.coll.alltoallv(packed, sc, rc)
                dst = _view(recv, rd[-1] + rc[-1] if P else 0)
                pos = 0
                for j in range(P):
                    dst[rd[j]:rd[j] + rc[j]] = got[pos:pos + rc[j]]
                    pos += rc[j]
                return 0
            except Exception:  # noqa: BLE001
                traceback.print_exc(file=sys.stderr)
                return 1

        self._ag = _lib.ALLGATHER_FN(allgather)
        self._a2a = _lib.ALLTOALLV_FN(alltoallv)
        self.struct = _lib.HostCommStruct(None, self._ag, self._a2a)
