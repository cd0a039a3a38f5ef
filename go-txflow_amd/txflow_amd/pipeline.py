"""Pipelined device-resident AddVote steps with the per-batch commit-state exchange of the
sharded path -- the step path bench.py times and the multi-rank GPU tests run.

A step is one batch through the whole AddVote chain of txv_run_staged (TxFlow.addVote for a
batch: txflow/service.go:192-234 -> types/vote_set.go:81-166), optionally on a fresh TxFlow
(txv_reset_flow) as bench.py replays its workload.  Batches sit in `depth` device slots; up to
`depth` steps are enqueued, so step k+1's verify chain runs beside step k's tally.

At world > 1 every step's packed commit state -- written by the device into the slot's commit
sink at the end of the step's TxFlow chain (txv_set_commit_sink) -- is all-gathered across
ranks:
  nccl (RCCL over xGMI): the all-gather runs on an exchange stream of its own, after an event
        recorded on the context's FLOW stream (txv_flow_stream via torch.cuda.ExternalStream)
        behind the step's chain, so it reads the sink after the pack while the next steps'
        TxFlow chains go on -- a rank's chain does not wait for the other ranks (the collective
        is the only cross-rank point); the flow stream waits for a slot's previous all-gather
        only when that slot is launched again (its sink is rewritten then), and no host thread
        waits for it;
  gloo  (CPU rehearsal): after the step's results are fetched (the sink is complete then), the
        sink goes to the host and is gathered there.
Every slot has a gathered buffer of its own, so step k's all-gathered global state (the commit
set and stakes of every shard as of step k, which the reference's per-vote commit side effects
act on: txflow/service.go:216-232) survives steps k+1 .. k+depth-1 and is read after finish(k)
by gathered_state(k) -- also while later steps are enqueued.  Over RCCL a timing event pair on
the exchange stream brackets each step's all-gather (exchange_ms: the per-step exchange cost,
including the wait for the slowest rank).
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
        self.slot_step = [-1] * depth       # the step whose gathered state slot sl holds
        self.finished = -1                  # newest step finished
        self._ev = None                     # RCCL: per slot, events around its step's all-gather
        self._ready = None                  # RCCL: per slot, the step's chain done (flow stream)
        self._xs = None                     # RCCL: the exchange stream
        self._gathering = [False] * depth   # an all-gather of the slot was enqueued
        if dist is not None:
            import torch
            self.world = dist.get_world_size()
            self.gloo = dist.get_backend() == "gloo"
            assert n_sets_cap > 0
            words = commit_state_bytes(n_sets_cap) // 4
            # device "cpu": a host-only rehearsal of the ring (gloo; tests/test_dist_gloo.py)
            sdev = "cpu" if device == "cpu" else f"cuda:{device}"
            assert sdev != "cpu" or self.gloo
            self.state = [torch.zeros(words, dtype=torch.int32, device=sdev) for _ in range(depth)]
            for sl in range(depth):
                ctx.set_commit_sink(sl, self.state[sl].data_ptr(), n_sets_cap)
            gdev = "cpu" if self.gloo else f"cuda:{device}"
            self.gathered = [torch.zeros(self.world * words, dtype=torch.int32, device=gdev) for _ in range(depth)]
            if not self.gloo:
                self._ext = torch.cuda.ExternalStream(ctx.flow_stream(), device=f"cuda:{device}")
                self._ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                            for _ in range(depth)]
                self._ready = [torch.cuda.Event() for _ in range(depth)]
                self._xs = torch.cuda.Stream(device=f"cuda:{device}")

    def close(self):
        if self._xs is not None:
            self._xs.synchronize()          # the all-gathers read the sinks
        if self.state is not None:
            for sl in range(self.depth):
                self.ctx.set_commit_sink(sl, None)
            self.state = None

    def launch(self, k: int):
        """enqueue step k (a fresh TxFlow first, in flow-stream order after step k-1) and, over
        RCCL, its commit-state all-gather on the exchange stream once the step's chain is done,
        into slot k % depth's gathered buffer (step k - depth's state there was finished and
        read before; its all-gather, which read the slot's sink, is done before the chain
        rewrites the sink)"""
        sl = k % self.depth
        if self._ext is not None and self._gathering[sl]:
            self._ext.wait_event(self._ev[sl][1])
        if self.fresh:
            self.ctx.reset_flow()
        self.ctx.run_staged(sl)
        self.slot_step[sl] = k
        if self._ext is not None:
            import torch
            self._ready[sl].record(self._ext)
            with torch.cuda.stream(self._xs):
                self._xs.wait_event(self._ready[sl])
                self._ev[sl][0].record(self._xs)
                self.dist.all_gather_into_tensor(self.gathered[sl], self.state[sl])
                self._ev[sl][1].record(self._xs)
            self._gathering[sl] = True

    def finish(self, k: int):
        """statuses + commit events of step k (waits for its chain); gloo: gather its sink"""
        sl = k % self.depth
        assert self.slot_step[sl] == k, "step k's slot was relaunched before step k was finished"
        st, ev = self.ctx.fetch_staged(sl, self.batches[sl].n, ev_cap=self.ev_cap, out=self.st_buf[sl],
                                       evs=self.ev_buf[sl])
        if self.gloo:
            self.dist.all_gather(list(self.gathered[sl].chunk(self.world)), self.state[sl].cpu())
        self.finished = k                   # the newest finished step (steps finish in order)
        return st, ev

    def run(self, m: int, on_finish=None):
        """m steps, up to `depth` enqueued: launch k before waiting for k - depth + 1.
        on_finish(k, st, ev) is called as each step's results arrive (gathered_state(k) is valid
        inside it); returns the last step's"""
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

    def gathered_state(self, k: Optional[int] = None) -> Optional[List[tuple]]:
        """step k's all-gathered state (default: the newest finished step), unpacked per rank:
        [(committed bool[], sums i64[], digests [n, 16] u8)] -- each set named by tx_digest(TxHash).  Valid from finish(k) until step k + depth is launched;
        waits for step k's all-gather only (later steps may still run)."""
        if self.gathered is None:
            return None
        k = self.finished if k is None else k
        sl = k % self.depth
        assert self.slot_step[sl] == k, "step k's slot was reused"
        if self._ev is not None:
            self._ev[sl][1].synchronize()
        g = self.gathered[sl].cpu().numpy().view(np.uint8).reshape(self.world, -1)
        return [commit_state_unpack(g[r], self.cap) for r in range(self.world)]

    def gathered_states(self) -> Optional[List[tuple]]:
        """the newest finished step's gathered state (waits for the flow stream and its all-gather)"""
        if self.gathered is None:
            return None
        self.ctx.sync()
        return self.gathered_state()

    def step_exchange_ms(self, k: int) -> Optional[float]:
        """RCCL: device time of step k's all-gather on the exchange stream (waits for it)"""
        if self._ev is None:
            return None
        sl = k % self.depth
        assert self.slot_step[sl] == k
        self._ev[sl][1].synchronize()
        return self._ev[sl][0].elapsed_time(self._ev[sl][1])
