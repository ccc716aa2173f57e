"""An in-process transport for libwost's distributed protocol (wost_distributed_run):
R threads play R ranks, the collectives meet at a barrier. Lets one process (and one
GPU) run the real C++ agreement / gather / merge of an R-rank solve."""
from __future__ import annotations

import threading

import numpy as np


class RankThreads:
    def __init__(self, n_ranks: int):
        self.R = int(n_ranks)
        self.bar = threading.Barrier(self.R, timeout=120)
        self.slots = [None] * self.R

    def transport(self, rank: int):
        def exchange(a):
            self.slots[rank] = np.array(a, np.float64, copy=True)
            self.bar.wait()
            out = np.stack(self.slots)
            self.bar.wait()
            return out

        def allreduce(a, op):
            st = exchange(a)
            return st.max(0) if op == "max" else st.sum(0)

        return allreduce, exchange

    def run(self, fn):
        """fn(rank, allreduce, allgather) on R threads -> [result or exception per rank]."""
        res = [None] * self.R

        def body(r):
            try:
                res[r] = fn(r, *self.transport(r))
            except Exception as e:   # noqa: BLE001 -- returned to the test
                res[r] = e

        th = [threading.Thread(target=body, args=(r,)) for r in range(self.R)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=300)
        return res
