#!/usr/bin/env python3
"""bench.py — verified+tallied TxVotes/sec on MI355X (BASELINE.json metric).

Workload: per GPU, 100 validators (power 1, quorum 67) x 10,000 txs
= 1,000,000 ed25519-signed TxVotes in shuffled arrival order (config C2 at N=1; at N>1 each
rank holds its shard = SHA-256(TxHash)[0] mod N of N x 10,000 txs, the C3 layout, weak
scaling).  Signatures come from the device signer; inputs are staged in HBM before timing.

One step = one pass of the hot path over the resident batch: empty all TxVoteSets
(device memsets), K1 verify every vote, K2 tally (first-accepted resolution, stake sums,
2/3 crossings, commit bitmap), read back per-vote statuses; at N>1 also an RCCL all-gather
of the per-shard commit bitmaps.  value = votes processed by all ranks / max-over-ranks time.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "go-txflow_amd"))

import numpy as np  # noqa: E402

W_ALG = 2.5e5   # int32 VALU lane-ops per verified vote, SURVEY.md §8d (Straus reference algorithm)
TALLY_BYTES_PER_VOTE = 16.0   # SURVEY.md §8d algorithmic tally traffic


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(wl, threads: int, serial_votes: int, parallel_votes: int):
    """The oracle's C restatement of the reference path on this host (kind "port"):
    serial = TxFlow.addVote loop with verification inside (1 goroutine, txflow/service.go:123-166);
    parallel = verify on `threads` host threads + the sequential tally with those verdicts."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.build()
    n = wl.n
    # serial: sequential AddVote with verification
    idx = np.arange(min(serial_votes, n))
    votes = [wl.vote(int(i)) for i in idx]
    flow = O.Flow(wl.pubs, wl.powers, b"test_chain_id")
    flow.add_votes(votes)
    ts = flow.last_seconds
    serial_rate = len(votes) / ts
    # parallel verify + sequential tally
    m = min(parallel_votes, n)
    msgs = [O.signbytes(1, wl.batch.txhash(i), int(wl.batch.ts_sec[i]), int(wl.batch.ts_nanos[i]), b"test_chain_id")
            for i in range(m)]
    arena = np.frombuffer(b"".join(msgs), np.uint8)
    lens = np.array([len(x) for x in msgs], np.uint16)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint32)
    pubs = np.frombuffer(b"".join(wl.pubs), np.uint8)
    tv, ok = O.verify_many(pubs, wl.val_of[:m], arena, offs, lens, wl.batch.sig[:64 * m], threads)
    flow2 = O.Flow(wl.pubs, wl.powers, b"test_chain_id")
    pv = [wl.vote(i) for i in range(m)]
    flow2.add_votes(pv, verdicts=ok)
    tt = flow2.last_seconds
    par_rate = m / (tv + tt)
    assert ok.all()
    return dict(value=round(par_rate, 1), unit="votes/s", cores=threads, kind="port",
                sample=f"first {m} votes of the same workload: {threads}-thread oracle ed25519 verify "
                       f"({tv:.2f}s) + sequential TxFlow.addVote tally ({tt:.2f}s); "
                       f"serial 1-thread verify-inside-AddVote on {len(votes)} votes = {serial_rate:.1f} votes/s",
                serial_value=round(serial_rate, 1), serial_cores=1)


def c5_streaming(device: int, n_vals: int, n_txs: int, batch: int):
    """C5: 1000 weighted validators, the stream cut into `batch`-vote batches fed
    through the pool ingest (txv_pool_check: SHA-256(Signature) keys on the GPU, LRU + pool list on
    the host) and txv_submit_votes / txv_wait_votes (host amino + routing + pack, H2D on the copy
    stream, verify + tally kernels, statuses and commit events back), two batches in flight so the
    host work of batch k+1 overlaps the kernels of batch k.  Latency-to-commit of a tx = return of the call that reported its commit
    event - submission of the batch holding its first vote."""
    import txflow_amd as T
    from txflow_amd.workload import StreamWorkload, SEEDS
    ctx = T.Context(device=device, max_batch=batch, max_txs=n_txs + 64, max_validators=n_vals,
                    max_accepted=n_txs * n_vals + 4 * batch)
    ctx.bind_host_numa()
    wl = StreamWorkload(ctx, n_vals, n_txs, SEEDS["c5"], batch)
    # Reactor.Receive -> TxVotePool.CheckTxWithInfo (GPU keys + host LRU) -> TxFlow.TryAddVote
    pool = T.TxVotePool(ctx, size=wl.n + 1, cache_size=wl.n + 1, max_txs_bytes=1 << 40)
    for _ in range(2):          # warm-up pass: first-touch of host tables and pinned buffers
        for b in wl.batches:
            pool.check_batch(b)
            ctx.add_votes(b, ev_cap=b.n)
        ctx.reset_flow()
        pool.flush()
    submit, done, commit_t, added, pool_ms = [], [], {}, 0, []
    inflight = []     # (batch index, ticket): at most two batches in flight (txv_submit_votes)

    def drain_one():
        nonlocal added
        k, tk = inflight.pop(0)
        st, ev = ctx.wait_votes(tk, ev_cap=wl.batches[k].n)
        te = time.perf_counter()
        done.append(te)
        added += int(np.count_nonzero((st & 0x7F) == T.ADDED))
        for e in ev:
            tx = int(wl.tx_of[k * batch + int(e["vote_index"])])
            assert tx not in commit_t, "tx committed twice"
            commit_t[tx] = te

    # Reactor.Receive -> CheckTx runs on its own thread (the reference's per-peer Receive goroutines)
    # while the main thread drives TxFlow (checkMaj23Routine): batch k+1's pool check overlaps
    # batch k's pack / kernels.  ctypes releases the GIL inside both calls.
    import queue
    import threading
    checked = queue.Queue(maxsize=2)
    pool_err = []

    def ingest():
        for k, b in enumerate(wl.batches):
            ts = time.perf_counter()
            ps = pool.check_batch(b)
            tp = time.perf_counter()
            if not (ps == T.POOL_OK).all():
                pool_err.append(k)
            checked.put((k, ts, tp))
        checked.put(None)

    t0 = time.perf_counter()
    th = threading.Thread(target=ingest, daemon=True)
    th.start()
    while True:
        item = checked.get()
        if item is None:
            break
        k, ts, tp = item
        if len(inflight) == 2:
            drain_one()
        submit.append(ts)
        inflight.append((k, ctx.submit_votes(wl.batches[k])))
        pool_ms.append((tp - ts) * 1e3)
    th.join()
    if pool_err:
        raise RuntimeError("C5: pool rejected a unique vote")
    while inflight:
        drain_one()
    total = time.perf_counter() - t0
    ok = added == wl.n and len(commit_t) == wl.n_txs
    lat = np.array([commit_t[t] - submit[wl.first_batch[t]] for t in commit_t]) * 1e3
    bl = (np.array(done) - np.array(submit)) * 1e3
    ok = ok and pool.Size() == wl.n
    pool.close()
    out = {"workload": f"C5: {n_vals} validators (power 1 + rand mod 1e6), {wl.n} votes in {batch}-vote batches "
                       f"through txv_pool_check (TxVotePool.CheckTx, on an ingest thread) + txv_submit_votes/txv_wait_votes "
                       f"(TxFlow.TryAddVote, two batches in flight)",
           "correct": ok, "votes_per_s": round(wl.n / total, 1),
           "p50_pool_check_ms": round(float(np.median(pool_ms)), 3),
           "p50_batch_ms": round(float(np.median(bl)), 3), "p99_batch_ms": round(float(np.percentile(bl, 99)), 3),
           "p50_commit_latency_ms": round(float(np.median(lat)), 3) if len(lat) else None,
           "p99_commit_latency_ms": round(float(np.percentile(lat, 99)), 3) if len(lat) else None,
           "table_window": ctx.table_w, "base_window": ctx.base_w}
    ctx.close()
    return out


WIRE_OUT_BYTES = 160   # per decoded message: one record (status, height, ts, offsets, lengths, TxKey, addr, sig)


def wire_decode_leg(ctx, wl, cpu: bool, reps: int = 20):
    """Reactor.Receive's decodeMsg for the C2 votes as received TxVoteMessage wire
    bytes (txv_encode_msgs = the sender's MarshalBinaryBare), decoded on the GPU (txv_k_decode_msgs)
    from a batch resident in HBM.  Roofline: HBM, algorithmic bytes = wire bytes + 12 B of offset /
    length per message read + a 160 B record written.  Also the host-inclusive rate (upload,
    decode, results copied into the caller's arrays) and the oracle's C decoder on one host thread."""
    import txflow_amd as T
    wb = T.encode_msgs(wl.batch)
    ctx.decode_stage(wb)
    ctx.decode_run(reps=2)
    kms = ctx.decode_run(reps=reps)
    d = ctx.decode_fetch(wb)
    n = wb.n
    b = wl.batch
    ok = bool((d.status[:n] == T.WIRE_OK).all() and (d.height[:n] == b.height).all() and
              (d.ts_sec[:n] == b.ts_sec).all() and (d.ts_nanos[:n] == b.ts_nanos).all() and
              (d.sig[:n].reshape(-1) == b.sig).all() and (d.addr[:n].reshape(-1) == b.addr).all() and
              (d.txhash_len[:n] == b.txhash_len).all() and (d.sig_len[:n] == b.sig_len).all())
    alg = wb.nbytes + n * (12 + WIRE_OUT_BYTES)
    traffic, pmc_src = None, None   # HBM bytes per launch from the committed PMC passes of this kernel
    pmc = os.path.join(ROOT, "profiles", "pmc_wire.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as f:
                pj = json.load(f)
            if pj.get("msgs_per_launch") == n:
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--validators", type=int, default=100)
    ap.add_argument("--txs-per-gpu", type=int, default=10_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--table-w", type=int, default=0, choices=(0, 4, 8, 10, 12, 14, 16, 18, 20),
                    help="fixed-base window; 0 = auto (largest whose tables fit the HBM budget)")
    ap.add_argument("--base-w", type=int, default=0, choices=(0, 4, 8, 10, 12, 14, 16, 20, 22, 24),
                    help="base-point table window (0 = library default)")
    ap.add_argument("--lane-votes", type=int, default=0, choices=(0, 1, 2, 4, 8),
                    help="votes per lane sharing one inversion in the W>=8 verify kernel (0 = library default)")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 streaming-latency leg")
    ap.add_argument("--no-wire", action="store_true", help="skip the TxVoteMessage wire-decode leg")
    ap.add_argument("--c5-txs", type=int, default=2048)
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl = RCCL over xGMI (the measured path); gloo = CPU-side rehearsal of the N>1 "
                         "code path (with --same-gpu, several ranks on one GPU)")
    ap.add_argument("--same-gpu", action="store_true", help="every rank uses device 0 (rehearsal only)")
    ap.add_argument("--cpu-serial-votes", type=int, default=150_000)
    ap.add_argument("--cpu-parallel-votes", type=int, default=500_000)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.same_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    gloo = args.dist_backend == "gloo"
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(args.dist_backend)   # nccl = RCCL over xGMI

    import txflow_amd as T
    from txflow_amd.workload import Workload, SEEDS

    n_txs_global = args.txs_per_gpu * world
    t_setup = time.perf_counter()
    max_txs = n_txs_global if world > 1 else args.txs_per_gpu
    ctx = T.Context(device=local, max_batch=2 * args.txs_per_gpu * args.validators, max_txs=max_txs + 64,
                    max_validators=max(args.validators, 1), table_w=args.table_w or None,
                    lane_votes=args.lane_votes, base_w=args.base_w)
    numa = ctx.bind_host_numa()     # host threads + pinned buffers next to this GPU's PCIe root
    wl = Workload(ctx, args.validators, n_txs_global, SEEDS["c3" if world > 1 else "c2"],
                  shard=rank, n_shards=world)
    ctx.stage(0, wl.batch)
    log(f"[rank {rank}] {ctx.device_name()}: {wl.n} votes ({wl.n_txs} txs x {args.validators} validators) "
        f"staged in {time.perf_counter() - t_setup:.1f}s")

    # per-shard commit state all-gathered every step: the commit bitmap of the shard's
    # set ids and their stake sums, packed in one buffer -> one RCCL all-gather over xGMI
    bm_ptr, bm_bytes = ctx.commit_bitmap()
    gathered = None
    if dist is not None:
        import torch
        cap = 2 * args.txs_per_gpu                    # local set ids (shards are ~txs_per_gpu each)
        bm_words = (cap + 31) // 32
        state = torch.zeros(bm_words + 2 * cap, dtype=torch.int32, device=f"cuda:{local}")
        gathered = torch.zeros(world * state.numel(), dtype=torch.int32, device="cpu" if gloo else f"cuda:{local}")
    red_dev = "cpu" if gloo else f"cuda:{local}"

    def all_gather_bitmaps():
        """per-shard commit bitmap + stake sums -> every rank (RCCL all-gather; gloo: host tensors)"""
        ctx.copy_commit_bitmap(state.data_ptr(), 4 * bm_words)
        ctx.copy_set_sums(state.data_ptr() + 4 * bm_words, cap)
        if gloo:
            torch.cuda.synchronize()
            dist.all_gather(list(gathered.chunk(world)), state.cpu())
        else:
            dist.all_gather_into_tensor(gathered, state)
            torch.cuda.synchronize()

    step_ms, verify_ms, tally_ms = [], [], []

    phases = {"reset": [], "run": [], "fetch": [], "gather": []}
    st_buf = np.zeros(wl.n, np.uint8)          # result buffers reused every step
    ev_buf = np.zeros(wl.n_txs + 1, T.EVENT_DTYPE)

    def step(record: bool):
        t0 = time.perf_counter()
        ctx.reset_tally()
        t1 = time.perf_counter()
        ms = ctx.run_staged(0, timed=True)
        t2 = time.perf_counter()
        st, ev = ctx.fetch_staged(0, wl.n, ev_cap=wl.n_txs + 1, out=st_buf, evs=ev_buf)
        t3 = time.perf_counter()
        if dist is not None:
            all_gather_bitmaps()
        t4 = time.perf_counter()
        if record:
            step_ms.append((t4 - t0) * 1e3)
            verify_ms.append(ms[0])
            tally_ms.append(ms[1])
            for k, a_, b_ in (("reset", t0, t1), ("run", t1, t2), ("fetch", t2, t3), ("gather", t3, t4)):
                phases[k].append((b_ - a_) * 1e3)
        return st, ev

    for _ in range(args.warmup):
        st, ev = step(False)
    # correctness gate on the timed workload: every vote valid -> ADDED; every tx commits once
    st, ev = step(False)
    n_added = int(np.count_nonzero((st & 0x7F) == T.ADDED))
    n_fired = int(np.count_nonzero(st & 0x80))
    quorum = ctx.total_power() * 2 // 3 + 1
    exp_fired = wl.n_txs * (args.validators - quorum + 1)
    if n_added != wl.n or len(ev) != wl.n_txs or n_fired != exp_fired:
        log(f"[rank {rank}] CORRECTNESS FAILURE: added {n_added}/{wl.n}, events {len(ev)}/{wl.n_txs}, "
            f"fired {n_fired}/{exp_fired}")
        sys.exit(2)

    if dist is not None:
        # the gathered global state: every tx of every shard committed with the full stake
        g = gathered.cpu().view(world, -1)
        bits = int(sum(bin(int(w) & 0xFFFFFFFF).count("1") for w in g[:, :bm_words].flatten().tolist()))
        sums = g[:, bm_words:].contiguous().view(torch.int64)
        nt = torch.tensor([wl.n_txs], dtype=torch.int64, device=red_dev)
        dist.all_reduce(nt)
        committed_sums = int((sums == ctx.total_power()).sum())
        if bits != int(nt.item()) or committed_sums != bits:
            log(f"[rank {rank}] GATHER CHECK FAILURE: {bits} commit bits / {committed_sums} full sums for {int(nt.item())} txs")
            sys.exit(3)
        dist.barrier()
        torch.cuda.synchronize()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    ctx.sync()
    if dist is not None:
        torch.cuda.synchronize()
        dist.barrier()
    elapsed = time.perf_counter() - t0
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
    v_ms = statistics.median(verify_ms)
    t_ms = statistics.median(tally_ms)
    if rank == 0:
        add_rate, mad_rate = ctx.valu_probe()
        peak = add_rate / 1e12
        # roofline.achieved = algorithmic work per launch / verify launch time: SURVEY.md §8d's
        # W_alg = 2.5e5 int32 lane-ops per verified vote x votes per launch / (K1a+K1b) HIP-event
        # time.  The executed work (rocprofv3 PMC pass of this kernel build, committed in
        # profiles/pmc_verify.json: SQ_INSTS_VALU with 64-bit-class ops counted twice, in
        # full-rate lane-op issue slots) is reported beside it as exec_*; traffic = HBM bytes
        # per launch from FETCH_SIZE (x2 gfx950 correction) + WRITE_SIZE.
        w_exec, traffic, pmc_src, pmc_w = None, None, None, None
        pmc = os.path.join(ROOT, "profiles", "pmc_verify.json")
        if os.path.exists(pmc):
            try:
                with open(pmc) as f:
                    pj = json.load(f)
                pmc_w = pj.get("table_window")
                if pmc_w == ctx.table_w:
                    w_exec = pj.get("verify_w_exec_lane_slots_per_vote")
                    traffic = pj.get("hbm_bytes_per_launch")
                    pmc_src = pj.get("source")
            except Exception:
                pass
        achieved = wl.n * W_ALG / (v_ms * 1e-3) / 1e12
        exec_rate = wl.n * w_exec / (v_ms * 1e-3) / 1e12 if w_exec else None
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            threads = min(args.cpu_threads, os.cpu_count() or 1)
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
                                    f"C3 layout: {world} x 10k txs sharded by SHA-256(TxHash)[0] mod {world}, "
                                    f"100 validators, ~1M votes/GPU, RCCL all-gather of commit bitmaps + stake sums"),
                       "validators": args.validators, "table_window": ctx.table_w, "base_window": ctx.base_w, "votes_per_gpu": wl.n, "txs_per_gpu": wl.n_txs,
                       "parallelism": f"shard{world}", "host_numa_bound": numa},
            "p50_batch_ms": round(statistics.median(step_ms), 3),
            "step_phases_ms_p50": {k: round(statistics.median(v), 3) for k, v in phases.items() if v},
            "verify_kernel_ms": round(v_ms, 3),
            "tally_kernels_ms": round(t_ms, 3),
            "roofline": {"bound": "valu", "achieved": round(achieved, 3), "peak": round(peak, 3),
                         "unit": "Tlane-op/s (int32 VALU)", "frac": round(achieved / peak, 4), "traffic": traffic,
                         "kernel": "txv_k_challenge + txv_k_scalarmult (verify pair)",
                         "alg_lane_ops_per_vote": W_ALG, "alg_source": "SURVEY.md §8d W_alg (Straus, w=8 NAF)",
                         "exec_lane_slots_per_vote": w_exec,
                         "exec_achieved": None if exec_rate is None else round(exec_rate, 3),
                         "exec_frac": None if exec_rate is None else round(exec_rate / peak, 4),
                         "pmc_source": pmc_src,
                         "peak_source": "live v_add_u32 issue-rate probe (txv_valu_probe)",
                         "mad_u64_u32_peak": round(mad_rate / 1e12, 3),
                         "tally_GBps": round(wl.n * TALLY_BYTES_PER_VOTE / (t_ms * 1e-3) / 1e9, 1)},
            "cpu_baseline": cpu,
        }
        if world == 1 and not args.no_wire:
            out["wire_decode"] = wire_decode_leg(ctx, wl, not args.no_cpu_baseline)
        if world == 1 and not args.no_c5:
            ctx.close()
            out["c5_streaming"] = c5_streaming(local, 1000, args.c5_txs, 65536)
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
