"""Per-stream occupancy of a rocprofv3 kernel + memory-copy trace (csv) over three consecutive
batches of one timed pass.  Usage: stream_timeline.py TRACE_DIR PASS [x] [ANCHOR]
  TRACE_DIR  directory holding kt_kernel_trace.csv and kt_memory_copy_trace.csv
  PASS       which run of 33 anchor launches (one per 64k batch) to look at
  x          also list every kernel / copy of the window with its start and duration
  ANCHOR     a kernel name fragment launched once per batch (default decode_msgs)
Prints each pass's span, the busy fraction of every stream / HW queue (S<stream>/Q<queue> for
kernels, S<stream>/copy for copies) in the window, and the largest per-batch costs."""
import csv, sys, collections
d = sys.argv[1]
K = list(csv.DictReader(open(d + "/kt_kernel_trace.csv")))
M = list(csv.DictReader(open(d + "/kt_memory_copy_trace.csv")))
ev = []
for r in K:
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "S%s/Q%s" % (r["Stream_Id"], r["Queue_Id"]), r["Kernel_Name"][:40]))
for r in M:
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "S%s/copy" % r["Stream_Id"], r["Direction"][12:] ))
ev.sort()
t0 = ev[0][0]
# find the decode kernels (one per batch) to locate passes
ANCHOR = sys.argv[4] if len(sys.argv) > 4 else "decode_msgs"
dec = [e for e in ev if ANCHOR in e[3]]
print("anchor launches", len(dec))
gaps = [(dec[i + 1][0] - dec[i][0]) / 1e3 for i in range(len(dec) - 1)]
# passes: runs of 33 decodes
for p in range(len(dec) // 33):
    a, b = dec[33 * p][0], dec[33 * p + 32][1]
    print("pass", p, "span ms", round((b - a) / 1e6, 2), "median decode gap us", sorted(gaps[33 * p:33 * p + 32])[16] if 33 * p + 32 <= len(gaps) else None)
P = int(sys.argv[2]) if len(sys.argv) > 2 else 3
a, b = dec[33 * P + 10][0], dec[33 * P + 13][0]
busy = collections.defaultdict(float)
names = collections.defaultdict(float)
for s, e, st, nm in ev:
    lo, hi = max(s, a), min(e, b)
    if hi > lo:
        busy[st] += hi - lo
        names[(st, nm)] += hi - lo
print("window us", (b - a) / 1e3, "(3 batches)")
for k, v in sorted(busy.items()):
    print(k, round(v / (b - a), 3))
for k, v in sorted(names.items(), key=lambda x: -x[1])[:30]:
    print(k, round(v / 3e3, 1), "us/batch")
if len(sys.argv) > 3 and sys.argv[3] == "x":
    for s, e, st, nm in ev:
        if s >= a and s < b:
            print(f"{(s - a) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {st:10s} {nm}")
