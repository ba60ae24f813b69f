"""In-process collective layer for ranks that are threads of one process
(the interface of pypardis_amd.distributed's comms), so the threaded
multi-device runner can be tested on the CPU.  Test infrastructure only."""
from __future__ import annotations

import threading

import numpy as np
import torch


class _Shared(object):
    def __init__(self, world):
        self.barrier = threading.Barrier(world, timeout=120)
        self.slots = [None] * world


class LocalComm(object):
    device = torch.device("cpu")

    def __init__(self, shared, world, rank):
        self.sh = shared
        self.world = world
        self.rank = rank

    def _exchange(self, value):
        self.sh.slots[self.rank] = value
        self.sh.barrier.wait()
        vals = list(self.sh.slots)
        self.sh.barrier.wait()
        return vals

    def abort(self):
        """pd_comm_abort's role: release every rank blocked on the group."""
        self.sh.barrier.abort()

    def all_reduce_t(self, t, op):
        vals = torch.stack(self._exchange(t.clone()))
        return {"sum": vals.sum(0), "max": vals.max(0).values,
                "min": vals.min(0).values}[op].to(t.dtype)

    def all_gather_t(self, t):
        return torch.stack(self._exchange(t.clone()))

    def exchange(self, sends, recvs, send_counts, recv_counts, skip_self=True):
        me = self.rank
        sc = [int(c) for c in send_counts]
        if skip_self:
            sc[me] = 0
        blocks = [list(torch.split(s, sc)) for s in sends]
        vals = self._exchange(blocks)
        ro = np.concatenate([[0], np.cumsum(np.asarray(recv_counts, np.int64))])
        for f, rcv in enumerate(recvs):
            for src in range(self.world):
                if skip_self and src == me:
                    continue
                b = vals[src][f][me]
                assert b.shape[0] == int(recv_counts[src])
                rcv[int(ro[src]):int(ro[src]) + b.shape[0]] = b

    def to(self, t):
        return t.to(self.device)

    def all_reduce(self, arr, op):
        vals = np.stack(self._exchange(np.asarray(arr)))
        return vals.max(0) if op == "max" else vals.sum(0)

    def all_gather_np(self, arr):
        return np.stack(self._exchange(np.asarray(arr).copy()))

    def all_gather_var(self, t):
        return torch.cat(self._exchange(t.clone()))

    def all_to_all_v(self, send, send_counts, recv_counts):
        chunks = list(torch.split(send, [int(c) for c in send_counts]))
        vals = self._exchange(chunks)
        out = torch.cat([vals[src][self.rank] for src in range(self.world)])
        assert out.shape[0] == int(np.sum(recv_counts))
        return out


def local_comms(world):
    sh = _Shared(world)
    return [LocalComm(sh, world, r) for r in range(world)]
