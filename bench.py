#!/usr/bin/env python3
"""bench.py — verified+tallied TxVotes/sec on MI355X (BASELINE.json metric).

Workload: per GPU, 100 validators (power 1, quorum 67) x 10,000 txs
= 1,000,000 ed25519-signed TxVotes in shuffled arrival order (config C2 at N=1).  At N>1 each
rank holds its shard (SHA-256(TxHash)[0] mod N, txv_shard_of) of N x 20,000 txs: the C3 layout
(16M votes at N = 8, ~2M per GPU), weak scaling.  Signatures come from the device signer.

One step = one pass of the hot path over the batch, inputs resident in HBM: a fresh TxFlow
(txv_reset_flow), then the whole AddVote kernel chain of txv_run_staged -- TxHash routing to
TxVoteSets (device hash table, first-seen ids), validator lookup and pre-checks, SignBytes,
K1a/K1b verify, the first-accepted resolution, stake sums and 2/3 crossings -- and the per-vote
statuses + commit events in host memory; at N>1 also the packed per-shard commit state
all-gathered over RCCL.  Steps run pipelined (slots 0-2 hold the same staged batch, up to three
enqueued): step k+1's verify chain runs while step k's TxFlow chain tallies, as consecutive
batches of a node do.  value = votes processed by all ranks / max-over-ranks time.

Beside it: the end-to-end rate from the caller's host SoA columns (txv_submit_votes /
txv_wait_votes, three batches in flight: staging copy + PCIe upload + kernels + results), the
CPU baseline (the oracle's C restatement on every allowed host core, and 1 thread), the
TxVoteMessage wire-decode leg and the C5 streaming leg.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)
"""
import argparse
import json
import math
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "go-txflow_amd"))

import numpy as np  # noqa: E402

# Roofline of the verify pair (K1a + K1b), integer VALU.  Peak = 256 CU x 4 SIMD x 32 lanes/clk x
# 2.4 GHz (MI355X_MICROARCH.md: "issues each VALU instruction over 2 cycles (32 lanes/cycle)").
VALU_PEAK = 256 * 4 * 32 * 2.4e9
# Algorithmic HBM bytes per verified vote of the verify pair: 23 table entries of
# 128 B (11 base-point + 13 validator positions - 1 starting entry), the signature (64 B), the
# SignBytes words (2 SHA-512 blocks' worth of message, 128 B), k written and read (2 x 32 B), the
# parked points of V = 8 (7/8 of a vote parks 128 B, written and read back), the verdict (1 B)
VERIFY_ALG_BYTES = 23 * 128 + 64 + 128 + 2 * 32 + 7 / 8 * 2 * 128 + 1
# Algorithmic int32 lane-ops per verified vote of the algorithm that runs (the
# one roofline definition, also BASELINE.md "Roofline as measured"):
#   SHA-512 of R||A||SignBytes, 2 blocks + ScReduce                                1.1e4
#   [s]B + [k](-A) over fixed-base tables: 11 + 13 = 24 entries -> the first is the
#   starting point (1 FM for its T), then 23 mixed additions x 7 FM, the last without T (6)  161 FM
#   encode (2 FM), Montgomery batch inverse (3 FM / vote), divstep inverse / 8 (~8 FM-eq)     13 FM
#   at 100 lane-ops per 255-bit field multiply (SURVEY.md §8d cost model)  -> 1.74e4
W_FM = 1 + 22 * 7 + 6 + 2 + 3 + 8
W_ALG = 1.1e4 + W_FM * 100.0


def table_positions(w: int) -> int:
    """table positions (one entry read per position and vote) of a radix-2^w table: ceil(256/w),
    12 for the long-top radix-2^21 layout (ed25519_dev.h Tab<21>)"""
    return 12 if w == 21 else -(-256 // w)


def w_alg_for(wb: int, wa: int) -> float:
    """W_ALG of the same algorithm for other table windows (C5's 1000 validators run W_A = 16:
    11 + 16 = 27 entries): the same terms with nT = positions(wb) + positions(wa) entries"""
    nt = table_positions(wb) + table_positions(wa)
    return 1.1e4 + (1 + (nt - 2) * 7 + 6 + 2 + 3 + 8) * 100.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cores() -> int:
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU quota if one is set"""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
        if q != "max":
            n = min(n, max(1, math.ceil(int(q) / int(p))))
    except Exception:
        pass
    return max(1, n)


def cpu_baseline(wl, threads: int, serial_votes: int, parallel_votes: int):
    """The oracle's C restatement of the reference path on this host (kind "port": the Go
    reference cannot be built here): TxFlow.addVote over the same SoA batch -- SignBytes, ed25519
    Verify on `threads` host threads, then the sequential tally (txflow/service.go:192-234) -- and
    the 1-thread form (the reference's single checkMaj23Routine goroutine, service.go:123-166)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.build()
    out = {}
    for name, m, th in (("parallel", min(parallel_votes, wl.n), threads), ("serial", min(serial_votes, wl.n), 1)):
        flow = O.Flow(wl.pubs, wl.powers, b"test_chain_id")
        b = wl.head(m)
        t0 = time.perf_counter()
        st, _, _ = flow.add_batch(b, th)
        secs = time.perf_counter() - t0
        assert (st == 0).all(), "CPU baseline: a valid vote was not ADDED"
        out[name] = (m, secs)
    (mp, sp), (ms, ss) = out["parallel"], out["serial"]
    return dict(value=round(mp / sp, 1), unit="votes/s", cores=threads, kind="port",
                sample=f"first {mp} votes of the same workload through the oracle's TxFlow.addVote "
                       f"(SignBytes + Verify on {threads} threads + sequential tally, {sp:.2f}s); "
                       f"1 thread on the first {ms} votes = {ms / ss:.1f} votes/s",
                serial_value=round(ms / ss, 1), serial_cores=1)


def c1_leg(device: int, threads: int):
    """C1 (BASELINE.json configs[0]): 4 validators, 10k signed TxVotes (2,500 txs x 4), the
    reference's own CPU config: the oracle on 1 thread and on every core, and the same batch
    end to end on the GPU (txv_add_votes: host SoA in, statuses and events out)."""
    import txflow_amd as T
    from txflow_amd.workload import Workload, SEEDS
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.build()
    ctx = T.Context(device=device, max_batch=16384, max_txs=4096, max_validators=8)
    wl = Workload(ctx, 4, 2500, SEEDS["c1"])
    res = {}
    for name, th in (("serial", 1), ("parallel", threads)):
        flow = O.Flow(wl.pubs, wl.powers, b"test_chain_id")
        t0 = time.perf_counter()
        ost, _, ofired = flow.add_batch(wl.batch, th)
        res[name] = wl.n / (time.perf_counter() - t0)
    exp = ost.astype(np.uint8) | (ofired.astype(np.uint8) << 7)
    st, ev = ctx.add_votes(wl.batch)
    ctx.reset_flow()
    reps, t0 = 20, time.perf_counter()
    for _ in range(reps):
        st, ev = ctx.add_votes(wl.batch)
        ctx.reset_flow()
    gpu = wl.n * reps / (time.perf_counter() - t0)
    ok = bool(np.array_equal(st, exp)) and len(ev) == wl.n_txs
    ctx.close()
    return {"workload": "C1: 4 validators x 2,500 txs = 10,000 signed TxVotes", "correct": ok,
            "cpu_serial_votes_per_s": round(res["serial"], 1),
            "cpu_parallel_votes_per_s": round(res["parallel"], 1), "cpu_cores": threads,
            "gpu_end_to_end_votes_per_s": round(gpu, 1)}


def end_to_end_leg(ctx, wl, steps: int, registered: bool):
    """Host SoA -> statuses + commit events: txv_reset_flow + txv_submit_votes per step, three steps
    in flight (step k+1's upload overlaps step k's kernels, step k+2's host pass and staging copy
    step k+1's upload), txv_wait_votes."""
    import txflow_amd as T
    b = wl.batch
    cols = [b.height, b.ts_sec, b.ts_nanos, b.txhash_off, b.txhash_len, b.addr, b.addr_len, b.sig, b.sig_len,
            b.txhash_arena] + ([b.txkey] if b.txkey is not None else [])
    if registered:
        for a in cols:
            ctx.host_register(a)
    col_bytes = sum(a.nbytes for a in cols)
    # the library fills uniform height / seconds / length columns on the device and decodes the
    # TxKey column from the TxHashes that spell it instead of uploading them (txv_staged_bytes)
    up_bytes = None
    inflight, lat, ok = [], [], True
    st_buf = None

    def drain():
        nonlocal ok
        t_sub, tk = inflight.pop(0)
        st, ev = ctx.wait_votes(tk, ev_cap=wl.n_txs + 1)
        lat.append((time.perf_counter() - t_sub) * 1e3)
        ok = ok and len(ev) == wl.n_txs and int(np.count_nonzero((st & 0x7F) == T.ADDED)) == wl.n

    for _ in range(2):                      # warm-up: first touch of the staging buffers
        ctx.reset_flow()
        inflight.append((time.perf_counter(), ctx.submit_votes(b)))
        up_bytes = ctx.staged_bytes()
        drain()
    lat.clear()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.reset_flow()
        if len(inflight) == E2E_INFLIGHT:
            drain()
        inflight.append((time.perf_counter(), ctx.submit_votes(b)))
    while inflight:
        drain()
    el = time.perf_counter() - t0
    if registered:
        for a in cols:
            ctx.host_unregister(a)
    del st_buf
    return {"votes_per_s": round(wl.n * steps / el, 1), "ms_per_step": round(el / steps * 1e3, 3),
            "p50_batch_ms": round(float(np.median(lat)), 3), "host_bytes_per_step": col_bytes,
            "uploaded_bytes_per_step": up_bytes, "uploaded_bytes_per_vote": round(up_bytes / wl.n, 1),
            "pcie_GBps": round(up_bytes * steps / el / 1e9, 2), "correct": ok}


E2E_INFLIGHT = 3        # end-to-end leg: steps in flight (of the library's four-slot submit ring)
C5_REPLAY = 0.05        # 5% exact replays in the stream
C5_CACHE = 10000        # TxVotePool CacheSize: tendermint's default (config.DefaultMempoolConfig)


def c5_expected_pool(wl, cache_size: int):
    """the oracle pool's CheckTx verdicts for the stream, batch by batch (checker, untimed)"""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.build()
    op = O.Pool(size=wl.n + 1, cache_size=cache_size, max_txs_bytes=1 << 40)
    return [op.check_batch(b) for b in wl.batches]


C5_INFLIGHT = int(os.environ.get("TXV_C5_INFLIGHT", "4"))   # TxFlow batches in flight in the C5 leg (<= 4, the submit ring)
# TxVotePool Size cap of the C5 legs: committed votes leave the pool through Update, so the pool
# holds what CheckTx admitted ahead of the commits (~8 batches in the pipelines below) -- not the
# stream (2.15M votes)
C5_POOL_SIZE = 1 << 20
C5_PASSES = 5           # timed passes of the C5 SoA (device cache) and wire legs: the median is reported
C5_CHECKED = os.environ.get("TXV_C5_CHECKED", "1") != "0"   # C5 SoA: txv_submit_checked (0: statuses waited first)
WIRE_INFLIGHT = int(os.environ.get("TXV_WIRE_INFLIGHT", "3"))   # wire batches between decode and wait (<= 3, the ingest ring)
C5_LONG_POOL_SIZE = 1 << 23     # c5_long: leaked replay entries accumulate over 16M votes (see c5_long)
# TXV_C5_NO_UPDATE=1 (experiment: the "without Update" figure of the same build): no Update calls,
# and a Size cap above the stream so nothing fills
C5_NO_UPDATE = bool(os.environ.get("TXV_C5_NO_UPDATE"))
if C5_NO_UPDATE:
    C5_POOL_SIZE = 1 << 23


def c5_commit_updates(wl, added_slots, fired_slots):
    """TxFlow's commit side effect on the pool, per batch (txflow/service.go:216-227 ->
    TxVotePool.Update, txvotepool.go:329-359).  The reference calls Update(height, set.GetVotes())
    after EVERY fired vote (an ADDED vote of a set with 2/3: the crossing vote and each later
    ADDED one), each time with the set's whole vote list.  A key's last push decides its LRU place
    and removals are idempotent, so that sequence leaves the pool exactly as this one does, issued
    once per batch: the sets that fired in the batch, ordered by their last fired vote, each set's
    accepted votes so far in one block (GetVotes iterates a Go map, so the reference's order inside
    a block is unspecified; arrival order is one of its orders).  tests/test_update_cadence.py
    checks the equivalence on the oracle pool.  added_slots / fired_slots: stream indices of the
    ADDED / fired votes (an untimed pass).  Returns one VoteBatch (or None) per batch, gathered
    from the stream's columns."""
    import txflow_amd as T
    B = wl.batch_size
    cols = {c: np.concatenate([getattr(b, c) for b in wl.batches]) for c in
            ("height", "txhash_off", "txhash_len", "ts_sec", "ts_nanos", "addr", "addr_len", "sig", "sig_len")}
    added_slots = np.sort(added_slots)
    atx = wl.tx_of[added_slots]
    by_tx = np.argsort(atx, kind="stable")               # each tx's ADDED votes, in stream order
    tcut = np.searchsorted(atx[by_tx], np.arange(wl.n_txs + 1))
    fired_slots = np.sort(fired_slots)
    fb = fired_slots // B
    out = []
    for k in range(len(wl.batches)):
        f = fired_slots[(fb == k)] if len(fired_slots) else fired_slots
        if not len(f):
            out.append(None)
            continue
        ftx = wl.tx_of[f]
        last = {}
        for g_, t_ in zip(f.tolist(), ftx.tolist()):      # the set's last fired vote in the batch
            last[t_] = g_
        end = (k + 1) * B
        blocks = []
        for t_ in sorted(last, key=last.get):
            v = added_slots[by_tx[tcut[t_]:tcut[t_ + 1]]]
            blocks.append(v[v < end])
        idx = np.concatenate(blocks)
        a20 = (idx[:, None] * 20 + np.arange(20)).reshape(-1)
        a64 = (idx[:, None] * 64 + np.arange(64)).reshape(-1)
        out.append(T.VoteBatch(len(idx), height=cols["height"][idx], txhash_arena=wl.batches[0].txhash_arena,
                               txhash_off=cols["txhash_off"][idx], txhash_len=cols["txhash_len"][idx],
                               ts_sec=cols["ts_sec"][idx], ts_nanos=cols["ts_nanos"][idx], addr=cols["addr"][a20],
                               addr_len=cols["addr_len"][idx], sig=cols["sig"][a64], sig_len=cols["sig_len"][idx]))
    return out


def c5_prepare_updates(ctx, wl):
    """the commit-driven Updates (untimed): the ADDED votes and each tx's commit batch from one pass
    of the stream through TxFlow with the oracle pool's admissions (an unbounded pool: the ADDED
    votes are the first occurrence of each distinct vote, whatever the LRU state)"""
    import txflow_amd as T
    expect = c5_expected_pool(wl, C5_CACHE)
    B = wl.batch_size
    added, fired = [], []
    for k, b in enumerate(wl.batches):
        b.is_nil = (expect[k] != T.POOL_OK).astype(np.uint8)
        st, ev = ctx.add_votes(b, ev_cap=b.n)
        added.append(k * B + np.nonzero((st & 0x7F) == T.ADDED)[0])
        fired.append(k * B + np.nonzero(st & T.STATUS_FIRED)[0])
        b.is_nil = None
    ctx.reset_flow()
    upd = c5_commit_updates(wl, np.concatenate(added), np.concatenate(fired))
    if C5_NO_UPDATE:
        upd = [None] * len(upd)
    for u in upd:                      # the Updates' columns registered too (DMA'd by the pool engine)
        if u is not None:
            for col in (u.sig, u.sig_len):
                ctx.host_register(col)
    return upd, sum(u.n for u in upd if u is not None)


def c5_pool_replay(wl, order, upd, got, cache_size, pool_size: int = C5_POOL_SIZE):
    """the oracle pool run through the same CheckTx batches and Updates in the order the pool took
    them (recorded under the callers' lock): every batch's statuses must equal (checker, untimed)"""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.build()
    op = O.Pool(size=pool_size, cache_size=cache_size, max_txs_bytes=1 << 40)
    ok = True
    for kind, k in order:
        if kind == "c":
            ok = ok and bool(np.array_equal(op.check_batch(wl.batches[k]), got[k]))
        elif upd[k] is not None:
            op.update_batch(1, upd[k])
    return ok


def c5_pass(ctx, wl, pool, upd, device_cache: bool, batch: int, n_vals: int, label: str = "", collect_dev: bool = False,
            pool_size: int = C5_POOL_SIZE):
    """One pipelined pass of the C5 stream (c5_streaming's timed pass, c5_long's one long pass):
    CheckTx -> TryAddVote -> Update on the node's threads, C5_INFLIGHT TxFlow batches in flight.  Returns the
    pass's report, the per-batch device stage times (collect_dev) and per-batch wall times
    (submission and completion of every batch, for deciles / percentiles over a long pass)."""
    import queue
    import threading
    import txflow_amd as T
    n_upd = sum(u.n for u in upd if u is not None)
    submit, done, commit_t = [], [], {}
    added = [0]

    # Threads as a node's goroutines: Reactor.Receive -> CheckTx (prepare; with the device cache
    # txv_pool_check_submit), the checkMaj23Routine submitting each checked batch (main;
    # txv_submit_checked with the device cache), the statuses' collection (txv_pool_check_wait,
    # off the TryAddVote path), and a drain thread waiting each ticket in order as soon as it is
    # submitted (commit events reported when the device is done) and issuing the Update.  At most
    # C5_INFLIGHT TxFlow batches in flight; ctypes releases the GIL inside every call.
    import queue
    import threading
    checked = queue.Queue(maxsize=2)
    tickets = queue.Queue()
    slots = threading.Semaphore(C5_INFLIGHT)
    pool_st = [None] * len(wl.batches)
    dev_ms, dev_split = [], []        # per batch in the pipeline: slot events (HIP, per stream)
    # CheckTx batches and Updates reach the pool from different threads (as the reactor's
    # and TxFlow's goroutines do): the order the pool took them in is recorded for the
    # oracle's replay
    order, order_mu, max_size, upd_ms = [], threading.Lock(), [0], []

    # CheckTx in two stages on two threads (txv_pool_prepare: keys on the GPU + TxVote.Size;
    # txv_pool_check_keys: the order-dependent LRU / pool admission), so batch k+1's keys are
    # hashed while batch k is admitted
    prepared = queue.Queue(maxsize=2)
    prep_ms, admit_ms = [], []
    # TXV_C5_TRACE=path (debugging aid): every thread's stage intervals of the pass, as JSON
    trace = [] if os.environ.get("TXV_C5_TRACE") else None

    def mark(what, k, a, b):
        if trace is not None:
            trace.append((what, k, round((a - t0) * 1e3, 4), round((b - t0) * 1e3, 4)))

    # checked: the TxFlow submit of a device CheckTx batch (txv_submit_checked) does not wait for
    # its statuses -- the AddVote chain reads them (and the signatures the CheckTx uploaded) in HBM
    # behind the decisions; a status thread collects them for the report meanwhile
    checked_mode = device_cache and C5_CHECKED
    status_q = queue.Queue()
    if checked_mode:                             # no host nil column: TxFlow takes the pool's from HBM
        for b in wl.batches:
            b.is_nil = None

    def prepare():
        for k, b in enumerate(wl.batches):
            ts = time.perf_counter()
            if device_cache:                     # CheckTx submitted: decided on the GPU in order
                with order_mu:
                    tk = pool.check_submit(b)
                    order.append(("c", k))
                mark("check_submit", k, ts, time.perf_counter())
                if checked_mode:
                    status_q.put((k, ts, time.perf_counter(), tk))
                    checked.put((k, ts, time.perf_counter(), tk))
                    continue
                prepared.put((k, ts, time.perf_counter(), None, tk))
            else:
                keys, sizes = pool.prepare(b)
                prepared.put((k, ts, time.perf_counter(), keys, sizes))
        if checked_mode:
            status_q.put(None)
            checked.put(None)
        else:
            prepared.put(None)

    def statuses():                              # checked mode: the pool's statuses, for the report
        while True:
            item = status_q.get()
            if item is None:
                return
            k, ts, tq, tk = item
            tc = time.perf_counter()
            pool_st[k] = pool.check_wait(tk)
            tp = time.perf_counter()
            mark("check_wait", k, tc, tp)
            prep_ms.append((tq - ts) * 1e3)
            admit_ms.append((tp - tc) * 1e3)

    def ingest():
        while True:
            item = prepared.get()
            if item is None:
                break
            k, ts, tq, keys, sizes = item
            tc = time.perf_counter()
            if keys is None:                     # the submitted batch's statuses
                ps = pool.check_wait(sizes)
            else:
                with order_mu:
                    ps = pool.check_keys(keys, sizes)
                    order.append(("c", k))
            tp = time.perf_counter()
            mark("check_wait", k, tc, tp)
            b = wl.batches[k]
            b.is_nil = (ps != T.POOL_OK).view(np.uint8)    # not admitted: never reaches TxFlow
            pool_st[k] = ps
            prep_ms.append((tq - ts) * 1e3)
            admit_ms.append((tp - tc) * 1e3)
            checked.put((k, ts, tp))
        checked.put(None)

    def drain():
        while True:
            item = tickets.get()
            if item is None:
                return
            k, tk = item
            tw = time.perf_counter()
            st, ev = ctx.wait_votes(tk, ev_cap=wl.batches[k].n)
            te = time.perf_counter()
            mark("wait_votes", k, tw, te)
            if collect_dev:               # the batch's stage times, before its ring slot is reused
                dev_ms.append(ctx.slot_kernel_ms((tk - 1) % T.SUBMIT_RING))
                sp = verify_split(ctx, (tk - 1) % T.SUBMIT_RING)
                if sp:
                    dev_split.append(sp)
            slots.release()
            if upd[k] is not None:        # TxVotePool.Update with the batch's committed votes
                tu = time.perf_counter()
                with order_mu:
                    pool.update_submit(1, upd[k])
                    order.append(("u", k))
                mark("update_submit", k, tu, time.perf_counter())
                upd_ms.append((time.perf_counter() - tu) * 1e3)
                max_size[0] = max(max_size[0], pool.Size())
            done.append(te)
            added[0] += int(np.count_nonzero((st & 0x7F) == T.ADDED))
            for e in ev:
                tx = int(wl.tx_of[k * batch + int(e["vote_index"])])
                assert tx not in commit_t, "tx committed twice"
                commit_t[tx] = te

    t0 = time.perf_counter()
    tpp = threading.Thread(target=prepare, daemon=True)
    th = threading.Thread(target=statuses if checked_mode else ingest, daemon=True)
    td = threading.Thread(target=drain, daemon=True)
    tpp.start()
    th.start()
    td.start()
    while True:
        item = checked.get()
        if item is None:
            break
        if checked_mode:
            k, ts, tp, ptk = item
        else:
            k, ts, tp = item
        ta = time.perf_counter()
        slots.acquire()
        tb = time.perf_counter()
        submit.append(ts)
        tickets.put((k, ctx.submit_checked(wl.batches[k], pool, ptk) if checked_mode else ctx.submit_votes(wl.batches[k])))
        mark("slot_wait", k, ta, tb)
        mark("submit_votes", k, tb, time.perf_counter())
    tpp.join()
    th.join()
    tickets.put(None)
    td.join()
    added = added[0]
    total = time.perf_counter() - t0
    if trace is not None:
        with open(os.environ["TXV_C5_TRACE"] + f".{label.replace(' ', '_')}.json", "w") as f:
            json.dump([("t0", -1, t0, t0)] + trace, f)
    pool.sync()
    pool_ok = c5_pool_replay(wl, order, upd, pool_st, C5_CACHE, pool_size)
    ok = pool_ok and added == wl.n_unique and len(commit_t) == wl.n_txs
    lat = np.array([commit_t[t] - submit[wl.first_batch[t]] for t in commit_t]) * 1e3
    bl = (np.array(done) - np.array(submit)) * 1e3
    allst = np.concatenate(pool_st)
    stages = ("two pipelined stages with the LRU cache in HBM (TXV_POOL_DEVICE_CACHE) -- "
              "txv_pool_check_submit (Size on the host; keys, stack-distance decisions, the new cache and "
              "the pool list in HBM -- the staged Update's pushes and removals first, then the batch's "
              "appends -- enqueued on the GPU, one thread) and txv_pool_check_wait (the statuses, "
              "another); p50_pool_check_ms = their sum per batch" if device_cache else
              "two pipelined stages -- txv_pool_prepare (keys on the GPU + Size, one thread) and "
              "txv_pool_check_keys (LRU + pool on the host, another); p50_pool_check_ms = their sum per batch")
    out = {"workload": f"C5: {n_vals} validators (power 1 + rand mod 1e6), {wl.n_unique} votes + "
                       f"{wl.n - wl.n_unique} exact replays ({C5_REPLAY:.0%}, Appendix C) in {batch}-vote batches "
                       f"through TxVotePool.CheckTx (CacheSize {C5_CACHE}) in {stages} -- + "
                       f"{'txv_submit_checked (TxFlow.TryAddVote enqueued behind the device CheckTx, the pool rejections as nil entries read in HBM)' if checked_mode else 'txv_submit_votes (TxFlow.TryAddVote for the admitted votes)'} / "
                       f"txv_wait_votes ({C5_INFLIGHT} batches in flight, each waited by a drain thread as soon as submitted) + TxVotePool.Update "
                       f"(txv_pool_update_submit, on the drain thread) after each batch's commit events, with the whole "
                       f"vote list of every set that fired in the batch, by last fired vote ({n_upd} votes per pass; "
                       f"the reference's Update(GetVotes()) per fired vote, txflow/service.go:216-227, leaves the same "
                       f"pool: tests/test_update_cadence.py), pool Size cap "
                       f"{pool_size}; pool statuses checked against the oracle pool replaying the CheckTx "
                       f"batches and Updates in the order the pool took them",
           "correct": ok, "pool_matches_oracle": pool_ok, "votes_per_s": round(wl.n / total, 1),
           "pool_size_cap": pool_size, "pool_size_max": max_size[0],
           "p50_pool_update_ms": round(float(np.median(upd_ms)), 3) if upd_ms else None,
           "pool_status_counts": {"ok": int((allst == T.POOL_OK).sum()),
                                  "in_cache": int((allst == T.POOL_ERR_IN_CACHE).sum()),
                                  "full": int((allst == T.POOL_ERR_FULL).sum())},
           "p50_pool_check_ms": round(float(np.median(np.array(prep_ms) + np.array(admit_ms))), 3),
           "p50_pool_prepare_ms": round(float(np.median(prep_ms)), 3),
           "p50_pool_admit_ms": round(float(np.median(admit_ms)), 3),
           "p50_batch_ms": round(float(np.median(bl)), 3), "p99_batch_ms": round(float(np.percentile(bl, 99)), 3),
           "p50_commit_latency_ms": round(float(np.median(lat)), 3) if len(lat) else None,
           "p99_commit_latency_ms": round(float(np.percentile(lat, 99)), 3) if len(lat) else None,
           "table_window": ctx.table_w, "base_window": ctx.base_w}
    log(f"[c5] {'device' if device_cache else 'host'} cache {label}: "
        f"{out['votes_per_s'] / 1e6:.1f}M votes/s, "
        f"correct {ok} (pool {pool_ok}, added {added}/{wl.n_unique}, commits {len(commit_t)}/{wl.n_txs}, "
        f"statuses {out['pool_status_counts']}, max Size {max_size[0]}; p50 ms prepare {out['p50_pool_prepare_ms']} "
        f"admit {out['p50_pool_admit_ms']} update {out['p50_pool_update_ms']} batch {out['p50_batch_ms']})")
    return out, dev_ms, dev_split, {"submit": submit, "done": done, "lat": lat, "bl": bl}


def c5_streaming(device: int, n_vals: int, n_txs: int, batch: int):
    """C5: 1000 weighted validators, the stream (with Appendix C's 5% exact
    replays) cut into `batch`-vote batches fed through the pool ingest (txv_pool_check:
    SHA-256(Signature) keys on the GPU, LRU of tendermint's default 10000 entries + pool list on the
    host) and txv_submit_votes / txv_wait_votes (columns staged + uploaded on the copy stream, the
    whole AddVote chain on the GPU, statuses and commit events back), C5_INFLIGHT batches in flight.  The
    votes CheckTx rejects (ErrTxInCache) never reach TxFlow: they travel as nil entries of the
    batch, which AddVote drops before any state (is_nil column).  Latency-to-commit of a tx =
    return of the call that reported its commit event - submission of the batch holding its first
    vote."""
    import txflow_amd as T
    from txflow_amd.workload import StreamWorkload, SEEDS
    ctx = T.Context(device=device, max_batch=batch, max_txs=n_txs + 64, max_validators=n_vals)
    ctx.bind_host_numa()
    wl = StreamWorkload(ctx, n_vals, n_txs, SEEDS["c5"], batch, replay=C5_REPLAY)
    upd, n_upd = c5_prepare_updates(ctx, wl)
    log(f"[c5] stream ready: {wl.n} votes, {n_upd} committed votes for Update per pass")
    # the batches' columns pinned once (txv_host_register, a node's receive buffers): the key
    # upload of txv_pool_prepare and txv_submit_votes DMA them without a staging copy
    seen = set()
    for b in wl.batches:
        for col in (b.height, b.ts_sec, b.ts_nanos, b.txhash_off, b.txhash_len, b.addr, b.addr_len, b.sig,
                    b.sig_len, b.txhash_arena, b.txkey):
            if col is not None and col.nbytes and col.ctypes.data not in seen:   # the arena is shared
                seen.add(col.ctypes.data)
                ctx.host_register(col)
    # Reactor.Receive -> TxVotePool.CheckTxWithInfo -> TxFlow.TryAddVote, with the pool's LRU cache
    # in HBM (TXV_POOL_DEVICE_CACHE: keys, decisions, the new cache and the pool list's appends and
    # Update removals in one GPU chain per batch) -- the reported mode -- and,
    # beside it, on the host (keys on the GPU, stack-distance decisions on the host threads, the
    # two halves pipelined on two threads)
    def run_mode(device_cache: bool):
        pool = T.TxVotePool(ctx, size=C5_POOL_SIZE, cache_size=C5_CACHE, max_txs_bytes=1 << 40, device_cache=device_cache)
        runs = run_passes(pool, device_cache)
        return pool, runs

    def run_passes(pool, device_cache):
        for w in range(2):          # warm-up pass: first-touch of host tables and pinned buffers
            for k, b in enumerate(wl.batches):
                b.is_nil = (pool.check_batch(b) != T.POOL_OK).astype(np.uint8)
                ctx.add_votes(b, ev_cap=b.n)
                if upd[k] is not None:
                    pool.update(1, upd[k])
            ctx.reset_flow()
            pool.flush()
            log(f"[c5] {'device' if device_cache else 'host'} cache warm-up pass {w} done")
        # a pipelined warm-up pass (the engine's buffers reach the sizes the fused Update batches
        # need), then C5_PASSES timed passes over the same stream (reset between; three for the host
        # cache): a 2M-vote pass lasts ~15-45 ms, so a single host stall (5-10 ms ones are seen on
        # some boxes) moves it; the median pass is reported, every pass beside it
        runs = []
        n_pass = C5_PASSES if device_cache else 3
        for rep in range(-1, n_pass):
            out, dev_ms, dev_split, _ = c5_pass(ctx, wl, pool, upd, device_cache, batch, n_vals,
                                                label=("pass %d" % rep) if rep >= 0 else "pipelined warm-up",
                                                collect_dev=rep == n_pass - 1)
            if rep >= 0:
                runs.append(out)
            ctx.reset_flow()
            pool.flush()
        return runs, dev_ms, dev_split

    if os.environ.get("TXV_C5_DEVICE_ONLY"):   # experiments: the reported mode only
        runs_h = None
    else:
        pool_h, (runs_h, _, _) = run_mode(False)
        pool_h.close()
    pool, (runs, dev_ms, dev_split) = run_mode(True)
    # unloaded latency: one batch at a time (CheckTx -> submit -> wait before the next batch's
    # CheckTx), so a batch's latency is its own chain, with no queueing behind others
    one_start, one_ms, one_commit, one_ps = [], [], {}, []
    t0 = time.perf_counter()
    for k, b in enumerate(wl.batches):
        ts = time.perf_counter()
        one_start.append(ts)
        ps = pool.check_batch(b)
        b.is_nil = (ps != T.POOL_OK).view(np.uint8)
        st, ev = ctx.wait_votes(ctx.submit_votes(b), ev_cap=b.n)
        te = time.perf_counter()
        one_ms.append((te - ts) * 1e3)
        one_ps.append(ps)
        for e in ev:
            one_commit[int(wl.tx_of[k * batch + int(e["vote_index"])])] = te
        if upd[k] is not None:
            pool.update_submit(1, upd[k])
    one_total = time.perf_counter() - t0
    pool.sync()
    one_ok = c5_pool_replay(wl, [(x, k) for k in range(len(wl.batches)) for x in ("c", "u")], upd, one_ps, C5_CACHE)
    one_lat = np.array([te - one_start[wl.first_batch[t]] for t, te in one_commit.items()]) * 1e3
    ctx.reset_flow()
    pool.flush()
    pool.close()
    # the reported pass: the device cache's (one GPU round trip per CheckTx batch, submitted and
    # waited on two threads); the host cache's two-stage pipeline beside it
    runs.sort(key=lambda r: r["votes_per_s"])
    out = dict(runs[len(runs) // 2])
    out["passes"] = len(runs)
    out["votes_per_s_passes"] = [r["votes_per_s"] for r in runs]
    if runs_h:
        runs_h.sort(key=lambda r: r["votes_per_s"])
        out["host_cache"] = {k: runs_h[1][k] for k in ("votes_per_s", "correct", "p50_pool_check_ms", "p50_pool_prepare_ms",
                                                        "p50_pool_admit_ms", "p50_batch_ms", "p50_commit_latency_ms",
                                                        "p99_commit_latency_ms")}
        out["host_cache"]["votes_per_s_passes"] = [r["votes_per_s"] for r in runs_h]
        out["host_cache"]["note"] = ("the same stream with the cache on the host: txv_pool_prepare (keys on the GPU + "
                                     "Size) and txv_pool_check_keys (stack-distance decisions on the host threads) on "
                                     "two threads")
    out["unloaded"] = {
        "note": "one batch at a time: txv_pool_check (device cache) -> txv_submit_votes -> txv_wait_votes before the "
                "next batch's CheckTx",
        "votes_per_s": round(wl.n / one_total, 1),
        "p50_batch_ms": round(float(np.median(one_ms)), 3),
        "p99_batch_ms": round(float(np.percentile(one_ms, 99)), 3),
        "p50_commit_latency_ms": round(float(np.median(one_lat)), 3) if len(one_lat) else None,
        "p99_commit_latency_ms": round(float(np.percentile(one_lat, 99)), 3) if len(one_lat) else None,
        "correct": one_ok and len(one_commit) == wl.n_txs}
    out["correct"] = (all(r["correct"] for r in runs) and out["unloaded"]["correct"] and
                      all(r["correct"] for r in runs_h or []))
    # where a 64k batch's device time goes: the stage times of every batch of the last
    # pass inside the pipeline, and of one batch run alone on a fresh TxFlow (staged slot 0: the
    # submit ring is idle now), with the verify pair's VALU roofline at this batch size
    b0 = wl.batches[0]
    b0.is_nil = None
    ctx.stage(0, b0)
    solo, solo_sp = [], []
    for _ in range(4):
        ctx.reset_flow()
        solo.append(ctx.run_staged(0, timed=True))
        sp = verify_split(ctx, 0)
        if sp:
            solo_sp.append(sp)
        ctx.fetch_staged(0, b0.n, ev_cap=b0.n)
    med = lambda xs, j: round(statistics.median(x[j] for x in xs), 4) if xs else None  # noqa: E731
    w_c5 = w_alg_for(ctx.base_w, ctx.table_w)
    v_solo = med(solo[1:], 1)
    out["device_ms_batch"] = {
        "votes": b0.n,
        "in_pipeline_p50": {"prep": med(dev_ms, 0), "verify": med(dev_ms, 1), "k1a": med(dev_split, 0),
                            "k1b": med(dev_split, 1), "tally_after_verify": med(dev_ms, 2), "chain": med(dev_ms, 3)},
        "standalone": {"prep": med(solo[1:], 0), "verify": v_solo, "k1a": med(solo_sp[1:], 0),
                       "k1b": med(solo_sp[1:], 1), "tally": med(solo[1:], 2), "chain": med(solo[1:], 3)},
        "k1b_kernel": "txv_k_scalarmult_split (4 lanes per vote) + txv_k_batch_encode (K1c)" if b0.n < (3 << 18)
                      else "txv_k_scalarmult_dyn",
        "roofline": {"bound": "valu", "alg_lane_ops_per_vote": w_c5,
                     "achieved": round(b0.n * w_c5 / (v_solo * 1e-3) / 1e12, 3) if v_solo else None,
                     "peak": round(VALU_PEAK / 1e12, 3), "unit": "Tlane-op/s",
                     "frac": round(b0.n * w_c5 / (v_solo * 1e-3) / VALU_PEAK, 4) if v_solo else None,
                     "note": f"standalone K1a + K1b of one batch; W_alg for windows {ctx.base_w}/{ctx.table_w} "
                             f"(bench.w_alg_for: {table_positions(ctx.base_w) + table_positions(ctx.table_w)} table entries)"}}
    ctx.close()
    return out


def c5_long(device: int, n_vals: int, n_txs: int, batch: int):
    """C5 as ONE long-running TxFlow (VERDICT r5 missing 3): the reference keeps every TxVoteSet for
    the life of the node (TxVoteSets map, txflow/service.go:27, 200-209) and fires the commit side
    effects on every later ADDED vote of a committed set (:216-232).  Here one context and one pool
    take the whole stream -- `n_txs` x `n_vals` votes (+ Appendix C's 5% replays) in `batch`-vote
    batches -- in one pipelined pass (c5_pass: CheckTx in HBM -> TryAddVote -> Update, two batches
    in flight) with no txv_reset_flow: the set table, the cells and the accepted-vote arena keep
    every set, sized up front (max_txs = n_txs + 64, max_accepted = min(max_txs x n_vals, 2^26)).
    Reported: the pass's rate, p50 / p99 batch and commit latency over all its batches, the rate of
    each tenth of the pass (flat = per-batch cost independent of the sets accumulated), and the
    same size-independent checks as C5 (every distinct vote ADDED once, every tx committed once,
    pool statuses equal to the oracle pool replaying the calls)."""
    import txflow_amd as T
    from txflow_amd.workload import StreamWorkload, SEEDS
    t_gen = time.perf_counter()
    ctx = T.Context(device=device, max_batch=batch, max_txs=n_txs + 64, max_validators=n_vals)
    ctx.bind_host_numa()
    wl = StreamWorkload(ctx, n_vals, n_txs, SEEDS["c5"] + 0x10, batch, replay=C5_REPLAY)
    upd, n_upd = c5_prepare_updates(ctx, wl)
    seen = set()
    for b in wl.batches:
        for col in (b.height, b.ts_sec, b.ts_nanos, b.txhash_off, b.txhash_len, b.addr, b.addr_len, b.sig,
                    b.sig_len, b.txhash_arena, b.txkey):
            if col is not None and col.nbytes and col.ctypes.data not in seen:
                seen.add(col.ctypes.data)
                ctx.host_register(col)
    log(f"[c5-long] stream ready: {wl.n} votes in {len(wl.batches)} batches, {wl.n_txs} txs, {n_upd} committed votes "
        f"for Update ({time.perf_counter() - t_gen:.1f} s)")
    # the pool's Size cap above the long pass's need: a replay admitted again after its key left the
    # cache is a second list element that txsMap no longer indexes, so Update never removes it (the
    # reference's clist + txsMap.Store, txvotepool.go:265-270, 339-344): the pool keeps growing by
    # ~3% of the stream over the pass, and a cap that could bind sends batches to the host path
    pool = T.TxVotePool(ctx, size=C5_LONG_POOL_SIZE, cache_size=C5_CACHE, max_txs_bytes=1 << 40, device_cache=True)
    for k in range(min(8, len(wl.batches))):        # warm-up: buffers and host tables, then a fresh flow and pool
        b = wl.batches[k]
        b.is_nil = (pool.check_batch(b) != T.POOL_OK).astype(np.uint8)
        ctx.add_votes(b, ev_cap=b.n)
        if upd[k] is not None:
            pool.update(1, upd[k])
    ctx.reset_flow()
    pool.flush()
    out, _, _, per = c5_pass(ctx, wl, pool, upd, True, batch, n_vals, label="one long pass", pool_size=C5_LONG_POOL_SIZE)
    n_sets = ctx.num_tx_sets()
    pool.close()
    ctx.close()
    submit, done = np.array(per["submit"]), np.array(per["done"])
    sizes = np.array([b.n for b in wl.batches], np.int64)
    nb = len(done)
    edges = [round(nb * d / 10) for d in range(11)]
    dec = []
    for d in range(10):
        lo, hi = edges[d], edges[d + 1]
        t0 = done[lo - 1] if lo > 0 else submit[0]
        dec.append(round(float(sizes[lo:hi].sum() / (done[hi - 1] - t0)), 1))
    bl = np.array(per["bl"])
    res = {k: out[k] for k in ("correct", "pool_matches_oracle", "votes_per_s", "p50_batch_ms", "p99_batch_ms",
                               "p50_commit_latency_ms", "p99_commit_latency_ms", "pool_size_max", "p50_pool_check_ms",
                               "pool_status_counts", "table_window", "base_window")}
    res.update({
        "workload": f"C5 as one TxFlow: {n_vals} validators (power 1 + rand mod 1e6), {wl.n_unique} votes + "
                    f"{wl.n - wl.n_unique} exact replays in {nb} batches of {batch}, one pass, no txv_reset_flow; "
                    f"TxVotePool.CheckTx in HBM + TryAddVote + Update (as c5_streaming)",
        "passes": 1, "votes": int(wl.n), "batches": nb, "tx_sets_at_end": int(n_sets),
        "votes_per_s_by_decile": dec,
        "decile_min_over_max": round(min(dec) / max(dec), 3),
        "p90_batch_ms": round(float(np.percentile(bl, 90)), 3),
        "slowest_batches_ms": {int(k): round(float(bl[k]), 3) for k in np.argsort(bl)[::-1][:6]},
        "flow_sizing": {"max_txs": n_txs + 64, "max_accepted": int(min((n_txs + 64) * n_vals, 1 << 26)),
                        "note": "the reference never prunes TxVoteSets; here the flow holds max_txs sets and "
                                "max_accepted accepted votes (sized for the node's horizon: 1M sets x 100 "
                                "validators = 10 GB of HBM), and a batch that would exceed either fails with "
                                "TXV_ECAPACITY and stops the flow until txv_reset_flow (DESIGN.md §3)"}})
    res["correct"] = bool(res["correct"] and n_sets == wl.n_txs)
    return res


def owner_route_leg(device: int, n_vals: int, n_txs: int, batch: int, n_ranks: int = 8):
    """The multi-GPU ingest's owner rank on one GPU: every C5 batch
    through TxVotePool.CheckTx with the cache in HBM (txv_pool_check_submit / _wait) and its
    admitted votes packed for `n_ranks` ranks on the device from the pool's statuses in HBM
    (txv_route_checked), on two threads (batch k+1's CheckTx enqueued while batch k is routed).  Its rate bounds what a node of
    n_ranks GPUs can admit when one owner runs CheckTx for all of them; the ranks' scatter and
    TxFlow chains are not in it.  Checked: every admitted vote routed exactly once (the metas sum
    to the admitted count), one batch's device buffers byte-identical to txv_route_pack_host."""
    import queue
    import threading
    import torch
    import txflow_amd as T
    from txflow_amd.workload import StreamWorkload, SEEDS
    ctx = T.Context(device=device, max_batch=batch, max_txs=64, max_validators=n_vals)
    ctx.bind_host_numa()
    wl = StreamWorkload(ctx, n_vals, n_txs, SEEDS["c5"], batch, replay=C5_REPLAY)
    seen = set()
    for b in wl.batches:
        b.is_nil = None
        for col in (b.height, b.ts_sec, b.ts_nanos, b.txhash_off, b.txhash_len, b.addr, b.addr_len, b.sig,
                    b.sig_len, b.txhash_arena, b.txkey):
            if col is not None and col.nbytes and col.ctypes.data not in seen:
                seen.add(col.ctypes.data)
                ctx.host_register(col)
    stride = max(T.route_stride(b) for b in wl.batches)
    buf = torch.zeros(n_ranks * stride, dtype=torch.uint8, device=f"cuda:{device}")
    # no Update here (the ranks' commits are not in this leg): a Size cap above the stream
    pool = T.TxVotePool(ctx, size=C5_LONG_POOL_SIZE, cache_size=C5_CACHE, max_txs_bytes=1 << 40, device_cache=True)
    # parity of one batch: device route == host route (untimed)
    st0 = pool.check_batch(wl.batches[0])
    m0 = ctx.route_admitted(wl.batches[0], st0, n_ranks, buf.data_ptr(), stride)
    hb, hm = T.route_pack_host(wl.batches[0], st0, n_ranks)
    db = buf.view(n_ranks, stride).cpu().numpy()
    same = bool(np.array_equal(m0, hm)) and all(np.array_equal(db[r, :int(hm[r]["bytes"])], hb[r, :int(hm[r]["bytes"])])
                                                 for r in range(n_ranks))
    pool.flush()
    runs = []
    for rep in range(3):
        tickets = queue.Queue(maxsize=2)
        routed, admitted, route_ms = [0], [0], []

        def submit():
            for b in wl.batches:
                tickets.put((b, pool.check_submit(b)))
            tickets.put(None)

        t0 = time.perf_counter()
        th = threading.Thread(target=submit, daemon=True)
        th.start()
        while True:
            item = tickets.get()
            if item is None:
                break
            b, tk = item
            tr = time.perf_counter()
            # the route kernels read the batch's statuses (and the signatures the CheckTx uploaded)
            # in HBM behind the pool's decisions: txv_route_checked; the statuses come back after
            m = ctx.route_checked(b, pool, tk, n_ranks, buf.data_ptr(), stride)
            route_ms.append((time.perf_counter() - tr) * 1e3)
            ps = pool.check_wait(tk)
            routed[0] += int(m["n"].sum())
            admitted[0] += int((ps == T.POOL_OK).sum())
        th.join()
        total = time.perf_counter() - t0
        runs.append({"votes_per_s": round(wl.n / total, 1), "p50_route_ms": round(float(np.median(route_ms)), 3),
                     "routed": routed[0], "admitted": admitted[0]})
        pool.flush()
    pool.close()
    ctx.close()
    runs.sort(key=lambda r: r["votes_per_s"])
    out = dict(runs[1])
    out.update({"workload": f"owner rank: the C5 stream ({wl.n} votes, {batch}-vote batches, {n_vals} validators) "
                            f"through TxVotePool.CheckTx (cache in HBM) + txv_route_checked to {n_ranks} ranks",
                "n_ranks": n_ranks, "votes_per_s_passes": [r["votes_per_s"] for r in runs],
                "device_route_equals_host": same,
                "correct": same and all(r["routed"] == r["admitted"] for r in runs)})
    return out


def c5_wire_leg(device: int, n_vals: int, n_txs: int, batch: int):
    """C5 from received wire bytes (SURVEY.md §8f.3 + §8a a15): the C5 stream as TxVoteMessage
    bytes (the sender's cdc.MarshalBinaryBare, txv_encode_msgs) per 64k-message batch through
    txv_ingest_decode (Reactor.Receive / decodeMsg on the GPU, keys and sizes computed there from
    the decoded records), txv_ingest_admit_submit (CheckTxWithInfo handed to the device: the LRU
    cache and pool list in HBM, decided behind the decode), txv_ingest_admit_finish (the statuses;
    TryAddVote for the admitted votes built on the device from the same records, enqueued) and
    txv_ingest_wait, on four threads with up to three batches in flight: the wire bytes cross PCIe
    once, and batch k+2 decodes while k+1 is checked and k's TxFlow chain runs (reactor.go:170-190 ->
    txvotepool.go:187-261 -> txflow/service.go:123-166).  Latency-to-commit of a tx = return of
    the wait that reported its commit event - the decode's start for the batch holding its first
    vote."""
    import queue
    import threading
    import txflow_amd as T
    from txflow_amd.workload import StreamWorkload, SEEDS
    ctx = T.Context(device=device, max_batch=batch, max_txs=n_txs + 64, max_validators=n_vals)
    ctx.bind_host_numa()
    wl = StreamWorkload(ctx, n_vals, n_txs, SEEDS["c5"], batch, replay=C5_REPLAY)
    upd, n_upd = c5_prepare_updates(ctx, wl)
    wbs = [T.encode_msgs(b, b.txkey) for b in wl.batches]
    wire_bytes = sum(w.nbytes for w in wbs)
    for w in wbs:          # the receive buffers, pinned once (txv_host_register): DMA'd without a staging copy
        ctx.host_register(w.wire)
    pool = T.TxVotePool(ctx, size=C5_POOL_SIZE, cache_size=C5_CACHE, max_txs_bytes=1 << 40, device_cache=True)
    for k, w in enumerate(wbs):                     # warm-up pass
        pool.ingest(w)
        if upd[k] is not None:
            pool.update(1, upd[k])
    ctx.reset_flow()
    pool.flush()
    runs = []
    for rep in range(-1, C5_PASSES):   # a pipelined warm-up pass, then C5_PASSES timed passes
        start, dec_ms, adm_ms, commit_t = [], [], [], {}
        state = {"added": 0, "ok": True}
        got, order, order_mu = [None] * len(wbs), [], threading.Lock()
        decoded, submitted, admitted = queue.Queue(), queue.Queue(), queue.Queue()
        slots = threading.Semaphore(WIRE_INFLIGHT)  # within the library's ingest ring
        sub_ms = []
        trace = [] if os.environ.get("TXV_C5_TRACE") else None

        def mark(what, k, a, b):
            if trace is not None:
                trace.append((what, k, round((a - t0) * 1e3, 4), round((b - t0) * 1e3, 4)))

        # four goroutine-like stages: Receive (decode) -> CheckTx handed to the device
        # (txv_ingest_admit_submit) -> its statuses + the TxFlow chain enqueued
        # (txv_ingest_admit_finish) -> the commit drain (wait)
        def admit():
            while True:
                item = decoded.get()
                if item is None:
                    submitted.put(None)
                    return
                k, tk = item
                ta = time.perf_counter()
                with order_mu:
                    pool.ingest_admit_submit(tk)
                    order.append(("c", k))
                sub_ms.append((time.perf_counter() - ta) * 1e3)
                mark("admit_submit", k, ta, time.perf_counter())
                submitted.put((k, tk))

        def finish():
            while True:
                item = submitted.get()
                if item is None:
                    admitted.put(None)
                    return
                k, tk = item
                ta = time.perf_counter()
                pool.ingest_admit_finish(tk)
                adm_ms.append((time.perf_counter() - ta) * 1e3)
                mark("admit_finish", k, ta, time.perf_counter())
                admitted.put((k, tk))

        def drain():
            while True:
                item = admitted.get()
                if item is None:
                    return
                k, tk = item
                tw = time.perf_counter()
                ws, ps, fs, ev = pool.ingest_wait(tk)
                te = time.perf_counter()
                mark("ingest_wait", k, tw, te)
                slots.release()
                if upd[k] is not None:            # TxVotePool.Update with the batch's committed votes
                    with order_mu:
                        pool.update_submit(1, upd[k])
                        order.append(("u", k))
                    mark("update_submit", k, te, time.perf_counter())
                got[k] = ps
                state["ok"] = state["ok"] and bool((ws == T.WIRE_OK).all())
                state["added"] += int(np.count_nonzero((fs & 0x7F) == T.ADDED))
                for e in ev:
                    commit_t[int(wl.tx_of[k * batch + int(e["vote_index"])])] = te

        ta_, td_ = threading.Thread(target=admit, daemon=True), threading.Thread(target=drain, daemon=True)
        tf_ = threading.Thread(target=finish, daemon=True)
        t0 = time.perf_counter()
        ta_.start()
        tf_.start()
        td_.start()
        for k, w in enumerate(wbs):
            tq = time.perf_counter()
            slots.acquire()
            ts = time.perf_counter()
            start.append(ts)
            tk = pool.ingest_decode(w)
            dec_ms.append((time.perf_counter() - ts) * 1e3)
            mark("slot_wait", k, tq, ts)
            mark("decode", k, ts, time.perf_counter())
            decoded.put((k, tk))
        decoded.put(None)
        ta_.join()
        tf_.join()
        td_.join()
        total = time.perf_counter() - t0
        if trace is not None:
            with open(os.environ["TXV_C5_TRACE"] + f".wire_{rep}.json", "w") as f:
                json.dump(trace, f)
        pool.sync()
        pool_ok = c5_pool_replay(wl, order, upd, got, C5_CACHE)
        lat = np.array([commit_t[t] - start[wl.first_batch[t]] for t in commit_t]) * 1e3
        log(f"[c5 wire] {'pass %d' % rep if rep >= 0 else 'pipelined warm-up'}: {wl.n / total / 1e6:.1f}M votes/s, "
            f"pool {pool_ok}")
        if rep < 0:
            ctx.reset_flow()
            pool.flush()
            continue
        runs.append({"votes_per_s": round(wl.n / total, 1), "pool_matches_oracle": pool_ok,
                     "correct": pool_ok and state["ok"] and state["added"] == wl.n_unique and len(commit_t) == wl.n_txs,
                     "p50_decode_ms": round(float(np.median(dec_ms)), 3),
                     "p50_admit_submit_ms": round(float(np.median(sub_ms)), 3),
                     "p50_admit_ms": round(float(np.median(adm_ms)), 3),
                     "p50_commit_latency_ms": round(float(np.median(lat)), 3) if len(lat) else None,
                     "p99_commit_latency_ms": round(float(np.percentile(lat, 99)), 3) if len(lat) else None})
        ctx.reset_flow()
        pool.flush()
    # unloaded latency: the same stream one batch at a time (decode -> admit -> wait before the
    # next batch's decode), so a batch's latency is its own chain, with no queueing behind others
    one_start, one_ms, one_commit, one_ok, one_ps = [], [], {}, True, []
    t0 = time.perf_counter()
    for k, w in enumerate(wbs):
        ts = time.perf_counter()
        one_start.append(ts)
        tk = pool.ingest_decode(w)
        pool.ingest_admit(tk)
        ws, ps, fs, ev = pool.ingest_wait(tk)
        te = time.perf_counter()
        one_ms.append((te - ts) * 1e3)
        one_ok = one_ok and bool((ws == T.WIRE_OK).all())
        one_ps.append(ps)
        for e in ev:
            one_commit[int(wl.tx_of[k * batch + int(e["vote_index"])])] = te
        if upd[k] is not None:
            pool.update_submit(1, upd[k])
    one_total = time.perf_counter() - t0
    pool.sync()
    one_ok = one_ok and c5_pool_replay(wl, [(x, k) for k in range(len(wbs)) for x in ("c", "u")], upd, one_ps, C5_CACHE)
    one_lat = np.array([te - one_start[wl.first_batch[t]] for t, te in one_commit.items()]) * 1e3
    ctx.reset_flow()
    pool.flush()
    pool.close()
    ctx.close()
    runs.sort(key=lambda r: r["votes_per_s"])
    out = dict(runs[len(runs) // 2])
    out["unloaded"] = {"note": "one batch at a time: txv_ingest_decode -> _admit -> _wait before the next decode",
                       "votes_per_s": round(wl.n / one_total, 1),
                       "p50_batch_ms": round(float(np.median(one_ms)), 3),
                       "p99_batch_ms": round(float(np.percentile(one_ms, 99)), 3),
                       "p50_commit_latency_ms": round(float(np.median(one_lat)), 3) if len(one_lat) else None,
                       "p99_commit_latency_ms": round(float(np.percentile(one_lat, 99)), 3) if len(one_lat) else None,
                       "correct": one_ok and len(one_commit) == wl.n_txs}
    out.update(workload=f"C5 as wire bytes: {n_vals} validators, {wl.n} TxVoteMessages ({wire_bytes / wl.n:.1f} B avg; "
                        f"{wl.n - wl.n_unique} exact replays, CacheSize {C5_CACHE}) in {batch}-message batches through "
                        f"txv_ingest_decode / txv_ingest_admit_submit / _admit_finish / txv_ingest_wait on four threads (decode -> "
                        f"pool + TxFlow enqueued together -> statuses -> commit events, device-resident, up to three batches in flight; receive buffers registered with "
                        f"txv_host_register, so the wire bytes are DMA'd without a staging copy; the pool's LRU cache "
                        f"in HBM, TXV_POOL_DEVICE_CACHE: CheckTx decided on the GPU from the decoded keys; "
                        f"p50_decode_ms = the upload + decode enqueue, p50_admit_ms = keys wait + CheckTx + TxFlow "
                        f"enqueue) + TxVotePool.Update (txv_pool_update_submit) with each batch's committed votes after "
                        f"its commit events ({n_upd} votes per pass), pool Size cap {C5_POOL_SIZE}",
               passes=len(runs), votes_per_s_passes=[r["votes_per_s"] for r in runs],
               correct=all(r["correct"] for r in runs) and out["unloaded"]["correct"],
               pcie_bytes_per_vote_up=round(wire_bytes / wl.n + 16, 1), pcie_bytes_per_vote_down=38)
    return out


WIRE_OUT_BYTES = 160   # per decoded message: one record (status, height, ts, offsets, lengths, TxKey, addr, sig)


def wire_decode_leg(ctx, wl, cpu: bool, reps: int = 20):
    """Reactor.Receive's decodeMsg for the C2 votes as received TxVoteMessage wire
    bytes (txv_encode_msgs = the sender's MarshalBinaryBare), decoded on the GPU (txv_k_decode_msgs)
    from a batch resident in HBM.  Roofline: HBM, algorithmic bytes = wire bytes + 12 B of offset /
    length per message read + a 160 B record written.  Also the host-inclusive rate (upload,
    decode, results copied into the caller's arrays) and the oracle's C decoder on one host thread."""
    import txflow_amd as T
    wb = T.encode_msgs(wl.batch, wl.batch.txkey)
    ctx.decode_stage(wb)
    ctx.decode_run(reps=2)
    kms = ctx.decode_run(reps=reps)
    d = ctx.decode_fetch(wb)
    n = wb.n
    b = wl.batch
    ok = bool((d.status[:n] == T.WIRE_OK).all() and (d.height[:n] == b.height).all() and
              (d.ts_sec[:n] == b.ts_sec).all() and (d.ts_nanos[:n] == b.ts_nanos).all() and
              (d.sig[:n].reshape(-1) == b.sig).all() and (d.addr[:n].reshape(-1) == b.addr).all() and
              (d.txhash_len[:n] == b.txhash_len).all() and (d.sig_len[:n] == b.sig_len).all() and
              (d.txkey[:n].reshape(-1) == b.txkey).all())
    alg = wb.nbytes + n * (12 + WIRE_OUT_BYTES)
    traffic, pmc_src = None, None   # HBM bytes per launch from the committed PMC passes of this kernel
    pmc = os.path.join(ROOT, "profiles", "pmc_wire.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as f:
                pj = json.load(f)
            if pj.get("msgs_per_launch") == n and pj.get("wire_bytes") in (None, wb.nbytes):
                traffic, pmc_src = pj.get("traffic"), pj.get("source")
        except Exception:
            pass
    t0 = time.perf_counter()
    for _ in range(3):
        ctx.decode_msgs(wb)
    host_s = (time.perf_counter() - t0) / 3
    out = {"workload": f"C2 votes as {n} TxVoteMessage wire messages ({wb.nbytes / n:.1f} B avg), batch resident in HBM",
           "correct": ok, "msgs_per_s": round(n / (kms * 1e-3), 1), "kernel_ms": round(kms, 4),
           "roofline": {"bound": "hbm", "achieved": round(alg / (kms * 1e-3) / 1e9, 1), "peak": 8000.0,
                        "unit": "GB/s", "frac": round(alg / (kms * 1e-3) / 1e9 / 8000.0, 4),
                        "alg_bytes_per_launch": alg, "traffic": traffic, "pmc_source": pmc_src,
                        "kernel": "txv_k_decode_msgs"},
           "host_inclusive_msgs_per_s": round(n / host_s, 1)}
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        m = min(n, 500_000)
        secs, st = O.wire_decode_many(wb.wire, wb.off[:m], wb.len[:m])
        out["cpu_baseline"] = {"value": round(m / secs, 1), "unit": "msgs/s", "cores": 1, "kind": "port",
                               "sample": f"first {m} messages, oracle/wire.c decoder on one thread"}
        out["correct"] = ok and bool((st == 0).all())
    return out


def verify_split(ctx, slot: int):
    """(K1a, K1b) ms of the slot's last run, or None where the library predates the split
    (experiment builds of an older ABI) or the call fails: the split is reported, never required"""
    try:
        return ctx.slot_verify_ms(slot)
    except Exception as e:                     # noqa: BLE001 -- measurement only
        log(f"K1a/K1b split unavailable: {e}")
        return None


def load_pmc(table_w: int, base_w: int, n_votes: int):
    """executed VALU lane-slots / vote and HBM bytes / launch of the verify pair from the committed
    PMC passes (profiles/pmc_verify.json), when they were taken on this kernel configuration"""
    pmc = os.path.join(ROOT, "profiles", "pmc_verify.json")
    if not os.path.exists(pmc):
        return None, None, None, None, None
    try:
        with open(pmc) as f:
            pj = json.load(f)
    except Exception:
        return None, None, None, None, None
    if pj.get("table_window") != table_w or pj.get("base_window", 24) != base_w:
        return None, None, None, None, None
    same = pj.get("votes_per_launch", n_votes) == n_votes
    traffic = pj.get("hbm_bytes_per_launch") if same else None
    tally = pj.get("tally_hbm_bytes_per_launch") if same else None
    return pj.get("verify_w_exec_lane_slots_per_vote"), traffic, pj.get("source"), tally, pj.get("k1b_valu_issue_busy")


TALLY_ALG_VOTE = 16       # B per vote the tally must move
TALLY_ALG_ADDED = 244     # B per ADDED vote: 128-byte accepted row written + 116 source bytes read
# B per vote when its 16-byte (set, validator) cell costs the whole 128-byte line a random access
# moves (tools/microbench/tally_calib.hip: 103 B of line traffic per random 16-B cell load,
# profiles/r03/tally_calib) + the 16 algorithmic bytes
TALLY_LINE_VOTE = 128 + 16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 30 steps by default: the timed region starts from an empty pipeline and ends drained, and
    # that fill / drain (about one batch's latency) is amortised over the steps (48 ms in all)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--validators", type=int, default=100)
    ap.add_argument("--txs-per-gpu", type=int, default=0,
                    help="0 = 10,000 at N=1 (C2) / 20,000 at N>1 (C3: 160k txs at N=8)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every host core this process may use")
    # the C2 context's validator tables: radix 2^21 in the 12-position long-top layout (1.70 GB per
    # validator, 170 GB for C2's 100; 21 mixed additions per verify with the radix-2^26 base table
    # instead of 22): 738-743M vs 717-721M votes/s at radix 2^20 on one box (profiles/r05/w21)
    ap.add_argument("--table-w", type=int, default=21, choices=(0, 4, 8, 10, 12, 14, 16, 18, 20, 21),
                    help="fixed-base window of the C2 context; 0 = auto (largest whose tables fit the HBM "
                         "budget); 21 = 12-position tables, 1.70 GB per validator")
    # the C2 context's base-point table: radix 2^26 (43 GB of HBM, one per process and device; 22
    # mixed additions per verify instead of 23): +3.0 % on one box (688.3M vs 668.3M votes/s,
    # profiles/r05/val1).  The library's default stays radix 2^24 (11.8 GB): a test session holds
    # several contexts.  The other legs' contexts take the library default.
    ap.add_argument("--base-w", type=int, default=26, choices=(0, 4, 8, 10, 12, 14, 16, 20, 22, 24, 26),
                    help="base-point table window of the C2 context (0 = library default: 24)")
    ap.add_argument("--lane-votes", type=int, default=0, choices=(0, 1, 2, 4, 8),
                    help="votes per lane sharing one inversion in the W>=8 verify kernel (0 = library default)")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 streaming-latency leg")
    ap.add_argument("--no-c1", action="store_true", help="skip the C1 leg")
    ap.add_argument("--no-route", action="store_true", help="skip the owner-rank CheckTx + ingest-route leg")
    ap.add_argument("--no-wire", action="store_true", help="skip the TxVoteMessage wire-decode leg")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (host SoA) leg")
    ap.add_argument("--c5-txs", type=int, default=2048)
    ap.add_argument("--c5-long-txs", type=int, default=16384,
                    help="txs of the one-long-TxFlow C5 pass (x 1000 validators: 16.4M votes by default; 0 = skip)")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl = RCCL over xGMI (the measured path); gloo = CPU-side rehearsal of the N>1 "
                         "code path (with --same-gpu, several ranks on one GPU)")
    ap.add_argument("--same-gpu", action="store_true", help="every rank uses device 0 (rehearsal only)")
    ap.add_argument("--cpu-serial-votes", type=int, default=100_000)
    ap.add_argument("--cpu-parallel-votes", type=int, default=1_000_000)
    ap.add_argument("--c5-only", action="store_true",
                    help="profiling aid: run only the C5 legs (SoA and wire) and print them as one JSON line")
    ap.add_argument("--c5-long-only", action="store_true", help="profiling aid: only the one-long-TxFlow C5 leg")
    ap.add_argument("--c5-wire-only", action="store_true", help="profiling aid: only the C5 wire-bytes leg")
    ap.add_argument("--route-only", action="store_true", help="profiling aid: only the owner-rank route leg")
    args = ap.parse_args()
    if os.environ.get("TXV_BENCH_WATCHDOG"):   # debugging aid: every thread's stack on stderr periodically
        import faulthandler
        faulthandler.dump_traceback_later(int(os.environ["TXV_BENCH_WATCHDOG"]), repeat=True, file=sys.stderr)

    if args.route_only:
        import torch
        torch.cuda.init()
        print(json.dumps({"owner_route": owner_route_leg(0, 1000, args.c5_txs, 65536)}), flush=True)
        return
    if args.c5_wire_only:
        print(json.dumps({"c5_wire": c5_wire_leg(0, 1000, args.c5_txs, 65536)}), flush=True)
        return
    if args.c5_long_only:
        print(json.dumps({"c5_long": c5_long(0, 1000, args.c5_long_txs, 65536)}), flush=True)
        return
    if args.c5_only:
        out = {"c5_streaming": c5_streaming(0, 1000, args.c5_txs, 65536)}
        if not args.no_wire:
            out["c5_wire"] = c5_wire_leg(0, 1000, args.c5_txs, 65536)
        if args.c5_long_txs:
            out["c5_long"] = c5_long(0, 1000, args.c5_long_txs, 65536)
        print(json.dumps(out), flush=True)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.same_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and not args.no_route:
        # torch's HIP runtime first, before any txv context (the route leg's device buffers are
        # torch tensors; tests/conftest.py, the N>1 path: the same order)
        import torch
        torch.cuda.init()
    txs_per_gpu = args.txs_per_gpu or (10_000 if world == 1 else 20_000)
    dist = None
    gloo = args.dist_backend == "gloo"
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(args.dist_backend)   # nccl = RCCL over xGMI

    import txflow_amd as T
    from txflow_amd.workload import Workload, SEEDS

    n_txs_global = txs_per_gpu * world
    t_setup = time.perf_counter()
    exp_votes = txs_per_gpu * args.validators
    max_batch = exp_votes if world == 1 else int(exp_votes * 1.25) + 4096   # shards are ~equal
    max_txs = (txs_per_gpu if world == 1 else int(txs_per_gpu * 1.25) + 64) + 64
    ctx = T.Context(device=local, max_batch=max_batch, max_txs=max_txs, max_validators=max(args.validators, 1),
                    table_w=args.table_w or None, lane_votes=args.lane_votes, base_w=args.base_w)
    numa = ctx.bind_host_numa()     # host threads + pinned buffers next to this GPU's PCIe root
    wl = Workload(ctx, args.validators, n_txs_global, SEEDS["c3" if world > 1 else "c2"],
                  shard=rank, n_shards=world)
    # the same batch in the three device slots: step k runs in slot k % 3 with up to three steps
    # enqueued, so step k+1's prep runs beside step k's K1b and its K1a/K1b beside step k's tally
    # (txv_run_staged returns as soon as the chain is enqueued).  At N>1 each step's packed
    # per-shard commit state ([n_sets][bitmap][sums], written by the device into the
    # slot's commit sink) is all-gathered over RCCL on an exchange stream after the step's chain
    # (txflow_amd/pipeline.py): the next chains do not queue behind it, no host thread waits.
    from txflow_amd.pipeline import PipelinedSteps
    DEPTH = int(os.environ.get("TXV_BENCH_DEPTH", "3"))   # 2..4 staged slots
    n_cap = max_txs
    steps_rt = PipelinedSteps(ctx, [wl.batch], depth=DEPTH, fresh_flow=True, dist=dist, n_sets_cap=n_cap,
                              device=local, ev_cap=wl.n_txs + 1)
    log(f"[rank {rank}] {ctx.device_name()}: {wl.n} votes ({wl.n_txs} txs x {args.validators} validators) "
        f"staged in {time.perf_counter() - t_setup:.1f}s")
    red_dev = "cpu" if gloo else f"cuda:{local}"

    step_ms, route_ms, verify_ms, tally_ms, k1a_ms, k1b_ms = [], [], [], [], [], []
    t_launch = {}
    launch0 = steps_rt.launch

    def launch(k: int):
        t_launch[k] = time.perf_counter()
        launch0(k)
    steps_rt.launch = launch

    def record(k, st, ev):
        step_ms.append((time.perf_counter() - t_launch[k]) * 1e3)
        ms = ctx.slot_kernel_ms(k % DEPTH)
        route_ms.append(ms[0]); verify_ms.append(ms[1]); tally_ms.append(ms[2])
        split = verify_split(ctx, k % DEPTH)
        if split:
            k1a_ms.append(split[0]); k1b_ms.append(split[1])

    steps_rt.run(args.warmup)
    # correctness gate on the timed workload: every vote valid -> ADDED; every tx commits once,
    # with exactly n_vals - quorum + 1 fired votes per tx
    st, ev = steps_rt.run(1)
    n_added = int(np.count_nonzero((st & 0x7F) == T.ADDED))
    n_fired = int(np.count_nonzero(st & 0x80))
    quorum = ctx.total_power() * 2 // 3 + 1
    exp_fired = wl.n_txs * (args.validators - quorum + 1)
    if n_added != wl.n or len(ev) != wl.n_txs or n_fired != exp_fired or ctx.num_tx_sets() != wl.n_txs:
        log(f"[rank {rank}] CORRECTNESS FAILURE: added {n_added}/{wl.n}, events {len(ev)}/{wl.n_txs}, "
            f"fired {n_fired}/{exp_fired}, sets {ctx.num_tx_sets()}/{wl.n_txs}")
        sys.exit(2)

    if dist is not None:
        import torch
        # the gathered global state (unpacked with the C-ABI's own layout): every tx of every shard
        # committed with the full stake
        bits = full = 0
        names = set()
        for com, sums, dig in steps_rt.gathered_states():
            bits += int(com.sum())
            full += int((sums == ctx.total_power()).sum())
            names.update(bytes(d) for d in dig[com])
        # the gathered rows name every rank's sets: this rank's own txs among them by digest
        mine = set(T.tx_digest(h.tobytes()) for h in wl.hashes)
        if not mine <= names or len(names) != bits:
            log(f"[rank {rank}] GATHER CHECK FAILURE: {len(mine - names)} own txs not named in the gathered state")
            sys.exit(3)
        nt = torch.tensor([wl.n_txs], dtype=torch.int64, device=red_dev)
        dist.all_reduce(nt)
        if bits != int(nt.item()) or full != bits:
            log(f"[rank {rank}] GATHER CHECK FAILURE: {bits} commit bits / {full} full sums for {int(nt.item())} txs")
            sys.exit(3)
        dist.barrier()
        torch.cuda.synchronize()
    ctx.sync()
    t0 = time.perf_counter()
    steps_rt.run(args.steps, record)
    ctx.sync()
    if dist is not None:
        torch.cuda.synchronize()
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # RCCL: the per-step commit-state all-gather's device time on the exchange stream (events around
    # it, txflow_amd/pipeline.py), for the timed region's last `depth` steps (their slots' events)
    gather_ms = None
    if dist is not None and not gloo:
        gx = [steps_rt.step_exchange_ms(k) for k in range(max(0, args.steps - DEPTH), args.steps)]
        gather_ms = round(statistics.median(gx), 4)
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        nv = torch.tensor([wl.n], dtype=torch.int64, device=red_dev)
        dist.all_reduce(nv)
        total_votes = int(nv.item())
    else:
        total_votes = wl.n

    value = total_votes * args.steps / elapsed
    r_ms, v_ms, t_ms = statistics.median(route_ms), statistics.median(verify_ms), statistics.median(tally_ms)
    # the same chain run alone (one step at a time, nothing beside it): per-stage device times
    # without the pipeline's co-running kernels (the tally's HBM rate uses these)
    solo, solo_split = [], []
    for _ in range(3):
        ctx.reset_flow()
        solo.append(ctx.run_staged(0, timed=True))
        split = verify_split(ctx, 0)
        if split:
            solo_split.append(split)
        ctx.fetch_staged(0, steps_rt.batches[0].n, ev_cap=steps_rt.ev_cap, out=steps_rt.st_buf[0], evs=steps_rt.ev_buf[0])
    s_ms = [statistics.median(x[j] for x in solo) for j in range(4)]
    s_split = [statistics.median(x[j] for x in solo_split) if solo_split else float("nan") for j in range(2)]
    if rank == 0:
        # roofline.achieved = algorithmic lane-ops of the verify pair per launch (W_ALG x votes) /
        # the pair's launch time (HIP events on the compute stream); the executed VALU lane-slots
        # (PMC SQ_INSTS_VALU pass of this build, profiles/pmc_verify.json) give exec_frac
        w_exec, traffic, pmc_src, tally_bytes, k1b_busy = load_pmc(ctx.table_w, ctx.base_w, wl.n)
        w_alg = w_alg_for(ctx.base_w, ctx.table_w)   # the algorithm that runs: its table entries
        achieved = wl.n * w_alg / (v_ms * 1e-3)
        exec_rate = wl.n * w_exec / (v_ms * 1e-3) if w_exec else None
        threads = args.cpu_threads or host_cores()
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(wl, threads, args.cpu_serial_votes, args.cpu_parallel_votes)
        out = {
            "metric": "verified+tallied TxVotes/sec",
            "value": round(value, 1),
            "unit": "votes/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: device-signed ed25519 TxVotes (RFC 8032), SURVEY.md §8d seeds",
            "config": {"workload": ("C2: 100 validators x 10k txs = 1M votes on one MI355X" if world == 1 else
                                    f"C3 layout: {n_txs_global} txs x {args.validators} validators = "
                                    f"{n_txs_global * args.validators} votes sharded by SHA-256(TxHash)[0] mod {world} "
                                    f"(~{exp_votes} per GPU), RCCL all-gather of the packed commit state"),
                       "validators": args.validators, "table_window": ctx.table_w, "base_window": ctx.base_w,
                       "votes_per_gpu": wl.n, "txs_per_gpu": wl.n_txs, "parallelism": f"shard{world}",
                       "host_numa_bound": numa,
                       "step": "reset_flow + device TxHash routing/pre-checks/SignBytes + verify + tally + "
                               "statuses/events to host" + (" + RCCL all-gather" if world > 1 else "") +
                               "; up to three steps enqueued (step k+1's verify overlaps step k's tally)"},
            "p50_batch_ms": round(statistics.median(step_ms), 3),
            "gather_ms": gather_ms,
            "device_ms_p50": {"prep": round(r_ms, 3), "verify": round(v_ms, 3), "k1a": round(statistics.median(k1a_ms), 3) if k1a_ms else None,
                              "k1b": round(statistics.median(k1b_ms), 3) if k1b_ms else None, "tally_after_verify": round(t_ms, 3),
                              "note": "in the timed pipeline (HIP events on each stream): prep + SignBytes, K1a + K1b, "
                                      "verify end -> tally end (includes waiting for the flow stream)"},
            "device_ms_standalone": {"prep": round(s_ms[0], 3), "verify": round(s_ms[1], 3), "k1a": round(s_split[0], 3) if solo_split else None,
                                     "k1b": round(s_split[1], 3) if solo_split else None, "tally": round(s_ms[2], 3),
                                     "chain": round(s_ms[3], 3),
                                     "note": "one step alone after the timed region (no co-running kernels)"},
            "roofline": {"bound": "valu", "achieved": round(achieved / 1e12, 3), "peak": round(VALU_PEAK / 1e12, 3),
                         "unit": "Tlane-op/s (int32 VALU issue)", "frac": round(achieved / VALU_PEAK, 4),
                         "traffic": traffic, "kernel": "txv_k_challenge + txv_k_scalarmult_dyn (verify pair; txv_k_scalarmult_multi when TXV_K1B_DYNAMIC=0)",
                         "alg_bytes_per_launch": round(wl.n * VERIFY_ALG_BYTES),
                         "traffic_over_alg_bytes": None if not traffic else round(traffic / (wl.n * VERIFY_ALG_BYTES), 3),
                         "alg_lane_ops_per_vote": w_alg,
                         "alg_source": f"DESIGN.md §4: SHA-512 2 blocks + ScReduce + field multiplies x 100 for "
                                       f"{table_positions(ctx.base_w) + table_positions(ctx.table_w)} table entries (windows "
                                       f"{ctx.base_w}/{ctx.table_w}; bench.w_alg_for)",
                         "k1b_valu_issue_busy": None if k1b_busy is None else round(k1b_busy, 3),
                         "valu_busy_note": "K1b wave-instructions x issue cycles (64-bit class 4, others 2) / SIMD-cycles "
                                           "of the dispatch (GRBM_GUI_ACTIVE), from the committed PMC pass; "
                                           "SQ_ACTIVE_INST_VALU / SQ_THREAD_CYCLES_VALU count instructions on this "
                                           "stack; the pure-VALU issue probe reads 0.81-0.85 on the same metric",
                         "exec_lane_slots_per_vote": w_exec,
                         "exec_achieved": None if exec_rate is None else round(exec_rate / 1e12, 3),
                         "exec_frac": None if exec_rate is None else round(exec_rate / VALU_PEAK, 4),
                         "pmc_source": pmc_src,
                         "standalone": {"verify_ms": round(s_ms[1], 3),
                                        "achieved": round(wl.n * w_alg / (s_ms[1] * 1e-3) / 1e12, 3),
                                        "frac": round(wl.n * w_alg / (s_ms[1] * 1e-3) / VALU_PEAK, 4),
                                        "note": "the same pair run alone after the timed region (no co-running "
                                                "flow kernels)"},
                         "peak_source": "MI355X_MICROARCH.md: 256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz"},
            "cpu_baseline": cpu,
            # the tally chain after verify (HBM-bound per BASELINE.md): bytes per launch from the same
            # PMC passes (2 x FETCH_SIZE + WRITE_SIZE of its kernels) over the standalone tally time
            # algorithmic bytes: 16 B per vote (set id, validator, verdict, pre-check,
            # status, cell) + 244 B per ADDED vote (its 128-byte accepted-vote row written, the 116
            # bytes of signature / height / time / TxKey it is made of read); every C2 vote is ADDED
            "tally": {"ms": round(s_ms[2], 3), "hbm_bytes_per_launch": tally_bytes,
                      "alg_bytes_per_launch": TALLY_ALG_VOTE * wl.n + TALLY_ALG_ADDED * wl.n,
                      "alg_GBps": round((TALLY_ALG_VOTE + TALLY_ALG_ADDED) * wl.n / (s_ms[2] * 1e-3) / 1e9, 1),
                      "alg_frac_of_8TBps": round((TALLY_ALG_VOTE + TALLY_ALG_ADDED) * wl.n / (s_ms[2] * 1e-3) / 8e12, 3),
                      "traffic_over_alg": None if not tally_bytes else
                      round(tally_bytes / ((TALLY_ALG_VOTE + TALLY_ALG_ADDED) * wl.n), 3),
                      "line_bound_bytes_per_launch": (TALLY_LINE_VOTE + TALLY_ALG_ADDED) * wl.n,
                      "traffic_over_line_bound": None if not tally_bytes else
                      round(tally_bytes / ((TALLY_LINE_VOTE + TALLY_ALG_ADDED) * wl.n), 3),
                      "GBps": None if not tally_bytes else round(tally_bytes / (s_ms[2] * 1e-3) / 1e9, 1),
                      "frac_of_8TBps": None if not tally_bytes else round(tally_bytes / (s_ms[2] * 1e-3) / 8e12, 3),
                      "note": "hbm_bytes_per_launch from the committed PMC passes (2 x FETCH_SIZE + WRITE_SIZE of "
                              "the tally kernels; the x2 holds for its 1- to 16-byte column reads and its random "
                              "cell accesses too: profiles/r03/tally_calib); alg = 16 B/vote + 244 B per ADDED vote "
                              "(BASELINE.md); line bound = the same with the vote's (set, validator) cell moved as "
                              "the 128-B line a random access costs (C2's arrival order is shuffled)"},
        }
        if world == 1 and not args.no_e2e:
            out["end_to_end"] = {
                "note": "host SoA columns -> statuses + commit events (staging copy, PCIe upload, kernels, "
                        "results), txv_submit_votes/txv_wait_votes with three steps in flight",
                "pageable": end_to_end_leg(ctx, wl, max(3, args.steps), registered=False),
                "registered": end_to_end_leg(ctx, wl, max(3, args.steps), registered=True)}
        if world == 1 and not args.no_wire:
            out["wire_decode"] = wire_decode_leg(ctx, wl, not args.no_cpu_baseline)
        if world == 1 and not args.no_c5:
            ctx.close()
            out["c5_streaming"] = c5_streaming(local, 1000, args.c5_txs, 65536)
            out["c5_wire"] = c5_wire_leg(local, 1000, args.c5_txs, 65536)
            if args.c5_long_txs:
                out["c5_long"] = c5_long(local, 1000, args.c5_long_txs, 65536)
        if world == 1 and not args.no_route:
            out["owner_route"] = owner_route_leg(local, 1000, args.c5_txs, 65536)
        if world == 1 and not args.no_c1:
            out["c1"] = c1_leg(local, threads)
        print(json.dumps(out), flush=True)
    steps_rt.close()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
