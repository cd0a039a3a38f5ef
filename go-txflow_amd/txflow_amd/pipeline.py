"""Pipelined device-resident AddVote steps with the per-batch commit-state exchange of the
sharded path -- the step path bench.py times and the multi-rank GPU tests run.

A step is one batch through the whole AddVote chain of txv_run_staged (TxFlow.addVote for a
batch: txflow/service.go:192-234 -> types/vote_set.go:81-166), optionally on a fresh TxFlow
(txv_reset_flow) as bench.py replays its workload.  Batches sit in `depth` device slots; up to
`depth` steps are enqueued, so step k+1's verify chain runs beside step k's tally.

At world > 1 every step's packed commit state -- written by the device into the slot's commit
sink at the end of the step's TxFlow chain (txv_set_commit_sink) -- is all-gathered across
ranks:
  nccl (RCCL over xGMI): the all-gather is enqueued on the context's FLOW stream right behind
        the step's chain (txv_flow_stream via torch.cuda.ExternalStream), so it reads the sink
        after the pack, the next step's TxFlow chain (which rewrites nothing the gather reads
        until the slot comes round again) queues behind it, and no host thread waits for it;
  gloo  (CPU rehearsal): after the step's results are fetched (the sink is complete then), the
        sink goes to the host and is gathered there.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np

from . import EVENT_DTYPE, Context, VoteBatch, commit_state_bytes, commit_state_unpack


class PipelinedSteps:
    def __init__(self, ctx: Context, batches: Sequence[VoteBatch], *, depth: int = 3, fresh_flow: bool = True,
                 dist=None, n_sets_cap: int = 0, device: int = 0, ev_cap: int = 0):
        """batches: one per slot step k runs batches[k % len(batches)] (staged once into
        slot k % depth; len(batches) must divide depth or be 1).  dist: torch.distributed with an
        initialised process group, or None (no exchange)."""
        assert 2 <= depth <= 4 and (len(batches) == 1 or depth % len(batches) == 0)
        self.ctx, self.depth, self.fresh, self.dist, self.device = ctx, depth, fresh_flow, dist, device
        self.batches = [batches[sl % len(batches)] for sl in range(depth)]
        for sl in range(depth):
            ctx.stage(sl, self.batches[sl])
        nmax = max(b.n for b in self.batches)
        self.st_buf = [np.zeros(max(b.n, 1), np.uint8) for b in self.batches]   # reused every step
        self.ev_cap = ev_cap or nmax
        self.ev_buf = [np.zeros(self.ev_cap, EVENT_DTYPE) for _ in range(depth)]
        self.cap = n_sets_cap
        self.state = self.gathered = None
        self.world, self.gloo, self._ext = 1, False, None
        if dist is not None:
            import torch
            self.world = dist.get_world_size()
            self.gloo = dist.get_backend() == "gloo"
            assert n_sets_cap > 0
            words = commit_state_bytes(n_sets_cap) // 4
            self.state = [torch.zeros(words, dtype=torch.int32, device=f"cuda:{device}") for _ in range(depth)]
            for sl in range(depth):
                ctx.set_commit_sink(sl, self.state[sl].data_ptr(), n_sets_cap)
            self.gathered = torch.zeros(self.world * words, dtype=torch.int32,
                                        device="cpu" if self.gloo else f"cuda:{device}")
            if not self.gloo:
                self._ext = torch.cuda.ExternalStream(ctx.flow_stream(), device=f"cuda:{device}")

    def close(self):
        if self.state is not None:
            for sl in range(self.depth):
                self.ctx.set_commit_sink(sl, None)
            self.state = None

    def launch(self, k: int):
        """enqueue step k (a fresh TxFlow first, in flow-stream order after step k-1) and, over
        RCCL, its commit-state all-gather on the flow stream behind it"""
        sl = k % self.depth
        if self.fresh:
            self.ctx.reset_flow()
        self.ctx.run_staged(sl)
        if self._ext is not None:
            import torch
            with torch.cuda.stream(self._ext):
                self.dist.all_gather_into_tensor(self.gathered, self.state[sl])

    def finish(self, k: int):
        """statuses + commit events of step k (waits for its chain); gloo: gather its sink"""
        sl = k % self.depth
        st, ev = self.ctx.fetch_staged(sl, self.batches[sl].n, ev_cap=self.ev_cap, out=self.st_buf[sl],
                                       evs=self.ev_buf[sl])
        if self.gloo:
            self.dist.all_gather(list(self.gathered.chunk(self.world)), self.state[sl].cpu())
        return st, ev

    def run(self, m: int, on_finish=None):
        """m steps, up to `depth` enqueued: launch k before waiting for k - depth + 1.
        on_finish(k, st, ev) is called as each step's results arrive; returns the last step's"""
        out = None
        for k in range(m):
            self.launch(k)
            if k >= self.depth - 1:
                j = k - self.depth + 1
                out = self.finish(j)
                if on_finish:
                    on_finish(j, *out)
        for j in range(max(0, m - self.depth + 1), m):
            out = self.finish(j)
            if on_finish:
                on_finish(j, *out)
        return out

    def gathered_states(self) -> Optional[List[tuple]]:
        """the last all-gathered states, unpacked per rank: [(committed bool[], sums i64[])]
        (waits for the flow stream)"""
        if self.gathered is None:
            return None
        self.ctx.sync()
        g = self.gathered.cpu().numpy().view(np.uint8).reshape(self.world, -1)
        return [commit_state_unpack(g[r], self.cap) for r in range(self.world)]
