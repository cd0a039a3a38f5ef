"""Print a window of a rocprofv3 kernel trace as a per-stream timeline (usage: timeline.py CSV
[start_dispatch_name_substring] [occurrence] [n_rows]).  Times in us relative to the first row."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
anchor = sys.argv[2] if len(sys.argv) > 2 else None
occ = int(sys.argv[3]) if len(sys.argv) > 3 else 0
nrows = int(sys.argv[4]) if len(sys.argv) > 4 else 80
i0 = 0
if anchor:
    hits = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    i0 = hits[min(occ, len(hits) - 1)]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i0 + nrows]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    nm = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-48:]
    print(f"q{r['Queue_Id']:>2} s{r['Stream_Id']:>3} {s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:7.1f}  {nm}  grid={r['Grid_Size_X']}")
