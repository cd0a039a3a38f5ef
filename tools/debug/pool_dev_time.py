"""Per-call time of TxVotePool CheckTx on 64k-vote batches (5 % exact replays, CacheSize 10000),
with the cache on the host (txv_pool_prepare + txv_pool_check_keys, and txv_pool_check) and in
HBM (TXV_POOL_DEVICE_CACHE, txv_pool_check), the GPU otherwise idle.  Run under
TXV_PROFILE_HOST=1 for the device path's enqueue / device / out split, or under rocprofv3
--kernel-trace --stats for its kernels."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, "go-txflow_amd")
import txflow_amd as T  # noqa: E402


def batches(n_batches, n, seed=5):
    rng = np.random.default_rng(seed)
    hist = []
    out = []
    for b in range(n_batches):
        sigs = rng.integers(0, 256, size=(n, 64), dtype=np.uint8)
        for i in range(n):
            if hist and rng.random() < 0.05:
                sigs[i] = hist[int(rng.integers(0, len(hist)))]
        hist.extend(list(sigs[:: 16]))
        votes = [T.TxVote(Height=1, TxHash="AB" * 32, Timestamp=(1_700_000_000, 1 + i), ValidatorAddress=b"\1" * 20,
                          Signature=sigs[i].tobytes()) for i in range(n)]
        out.append(T.VoteBatch.from_votes(votes))
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    ctx = T.Context(max_batch=n, max_txs=1024, max_validators=8)
    bs = batches(nb, n)
    res = {}
    for mode in ("host_check", "host_halves", "device"):
        pool = T.TxVotePool(ctx, size=1 << 24, cache_size=10000, max_txs_bytes=1 << 40, device_cache=mode == "device")
        ms = []
        for rep in range(2):
            for b in bs:
                t0 = time.perf_counter()
                if mode == "host_halves":
                    keys, sizes = pool.prepare(b)
                    pool.check_keys(keys, sizes)
                else:
                    pool.check_batch(b)
                ms.append((time.perf_counter() - t0) * 1e3)
            pool.flush()
        pool.close()
        res[mode] = {"p50_ms": round(float(np.median(ms[nb:])), 3), "min_ms": round(min(ms[nb:]), 3)}
        print(mode, res[mode], file=sys.stderr, flush=True)
    ctx.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
