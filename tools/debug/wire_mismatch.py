"""Prints the first messages where txv_decode_msgs and the oracle disagree (debug aid)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "go-txflow_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np
import txflow_amd as T
import oracle as O
import wire_gen as G

mx = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
msgs = G.messages(40000, seed=2024 + mx)
wb = T.WireBatch(msgs)
ctx = T.Context(max_batch=1 << 16, max_txs=1 << 12, max_validators=16, table_w=4)
d = ctx.decode_msgs(wb, mx)
shown = 0
blocks = {}
for i, m in enumerate(msgs):
    st, f = O.wire_decode(m, mx)
    o = int(wb.off[i])
    bad = int(d.status[i]) != st
    if not bad and st == 0:
        got = dict(height=int(d.height[i]), th=(int(d.txhash_off[i]) - o, int(d.txhash_len[i])), key=d.txkey[i].tobytes(),
                   ts=(int(d.ts_sec[i]), int(d.ts_nanos[i])), al=int(d.addr_len[i]), addr=d.addr[i].tobytes(),
                   sl=int(d.sig_len[i]), so=int(d.sig_off[i]) - o, sig=d.sig[i].tobytes())
        al, sl = len(f["addr"]), len(f["sig"])
        exp = dict(height=f["height"], th=(f["txhash_off"], len(f["txhash"])), key=f["txkey"], ts=(f["ts_sec"], f["ts_nanos"]),
                   al=al, addr=f["addr"][:20] + bytes(20 - min(al, 20)), sl=sl, so=f["sig_off"] if sl else 0,
                   sig=f["sig"][:64] + bytes(64 - min(sl, 64)))
        diff = {k: (got[k], exp[k]) for k in got if got[k] != exp[k]}
        bad = bool(diff)
    else:
        diff = {"status": (int(d.status[i]), st)}
    if bad:
        blocks[i // 256] = blocks.get(i // 256, 0) + 1
        if shown < 8:
            shown += 1
            print(f"msg {i} (block {i // 256}, off {o}, len {len(m)}): {diff}")
            print("   hex", m[:120].hex())
print("mismatches per block:", blocks)
spans = {}
for b in blocks:
    idx = [i for i in range(b * 256, min(len(msgs), b * 256 + 256)) if 0 < len(msgs[i]) <= mx]
    lo = min(int(wb.off[i]) for i in idx) & ~15
    hi = max(int(wb.off[i]) + len(msgs[i]) for i in idx)
    spans[b] = hi - lo
print("block spans:", spans)
