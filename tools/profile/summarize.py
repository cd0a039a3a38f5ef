#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel trace + PMC passes) for the verify/tally kernels.

usage: python tools/profile/summarize.py gpurun_out/<tag> [--votes N] [--out profiles/<name>.json]

HBM traffic follows MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KB per dispatch;
on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, so the corrected read
bytes are 2 x FETCH_SIZE x 1024 (the raw value is kept beside it).  The same factor holds for
the verify kernels' scattered 16-byte table gathers: tools/microbench/gather_calib.hip measures
2 x FETCH_SIZE x 1024 = the bytes of distinct 128-B lines touched within 2.5 %
(profiles/r01/fetch_calibration.json).
"""
import argparse
import csv
import glob
import json
import os
import statistics
from collections import defaultdict


def rows(path_glob):
    out = []
    for p in glob.glob(path_glob, recursive=True):
        with open(p) as f:
            out.extend(csv.DictReader(f))
    return out


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    base = name.split("(")[0].replace("void ", "").strip()
    if "Pred" in base:   # the scan kernels by predicate: txv_k_scan_apply<AddedPred, AddedAct> -> <AddedPred>
        base = base.split(",")[0].rstrip(">") + ">"
    return base


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--votes", type=float, default=1e6)
    ap.add_argument("--out")
    a = ap.parse_args()
    res = {"source": a.root, "votes_per_launch": a.votes, "kernels": {}}
    bj = os.path.join(a.root, "bench_kt.json")
    if os.path.exists(bj):
        with open(bj) as f:
            line = [x for x in f.read().splitlines() if x.startswith("{")]
        if line:
            b = json.loads(line[-1])
            res["table_window"] = b["config"].get("table_window")
            res["base_window"] = b["config"].get("base_window")
            res["bench_line_under_profiler"] = {k: b[k] for k in ("value", "ms_per_step", "verify_kernel_ms",
                                                                  "tally_kernels_ms") if k in b}
    kt = rows(os.path.join(a.root, "kt", "**", "*kernel_stats.csv"))
    for r in kt:
        res["kernels"].setdefault(short(r["Name"]), {}).update(
            calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]), pct=float(r["Percentage"]))
    pmc = defaultdict(lambda: defaultdict(list))
    for r in rows(os.path.join(a.root, "pmc_*", "**", "*counter_collection.csv")):
        pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in pmc.items():
        d = res["kernels"].setdefault(k, {})
        for c, vals in cs.items():
            d[c] = statistics.median(vals)
    for k, d in res["kernels"].items():
        if "FETCH_SIZE" in d:
            d["hbm_read_bytes_raw"] = d["FETCH_SIZE"] * 1024
            d["hbm_read_bytes_corrected"] = 2 * d["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in d:
            d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
        if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d and d["SQ_WAVES"]:
            d["valu_insts_per_wave"] = d["SQ_INSTS_VALU"] / d["SQ_WAVES"]
        # On this stack (ROCm 7.2, gfx950) SQ_ACTIVE_INST_VALU equals SQ_INSTS_VALU and
        # SQ_THREAD_CYCLES_VALU equals 64 x SQ_INSTS_VALU for every kernel, including the issue-rate
        # probe whose v_mad_u64_u32 takes twice a v_add_u32's time (profiles/r03/prof_head/
        # probe_*): they count instructions, not cycles.  VALU issue-busy is therefore derived:
        # wave-instructions x their issue cycles on a SIMD-32 (64-bit class 4, others 2;
        # MI355X_MICROARCH.md) over the SIMD-cycles of the dispatch (GRBM_GUI_ACTIVE summed over
        # the 8 XCDs = 8 x the dispatch's cycles; 1024 SIMDs).  The probe itself reads 0.81 (adds)
        # and 0.85 (mads): loop SALU and launch / drain are the rest.
        if all(c in d for c in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_INT64", "GRBM_GUI_ACTIVE")) and d["GRBM_GUI_ACTIVE"]:
            cyc = 4.0 * d["SQ_INSTS_VALU_INT64"] + 2.0 * (d["SQ_INSTS_VALU"] - d["SQ_INSTS_VALU_INT64"])
            d["valu_issue_busy"] = cyc / (1024.0 * d["GRBM_GUI_ACTIVE"] / 8.0)
            d["dispatch_cycles"] = d["GRBM_GUI_ACTIVE"] / 8.0
        if all(c in d for c in ("SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")) and d["SQ_WAVE_CYCLES"]:
            d["wave_frac_active"] = d["SQ_ACTIVE_INST_ANY"] / d["SQ_WAVE_CYCLES"]
            d["wave_frac_wait_issue"] = d["SQ_WAIT_INST_ANY"] / d["SQ_WAVE_CYCLES"]
            if "SQ_WAIT_ANY" in d:
                d["wave_frac_wait_mem"] = d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"]
        if "SQ_BUSY_CYCLES" in d and "GRBM_GUI_ACTIVE" in d:
            d["note"] = "SQ_* cycle counters are per-SE sums in quad-cycles (MI355X_MICROARCH.md)"
        if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d and (d["TCC_HIT_sum"] + d["TCC_MISS_sum"]):
            d["l2_hit_rate"] = d["TCC_HIT_sum"] / (d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
    # the verify pair: K1a (challenge) + K1b (scalar mult), per launch of 1 batch
    pair = [d for k, d in res["kernels"].items() if k.startswith(("txv_k_challenge", "txv_k_scalarmult"))]
    if pair and all("SQ_INSTS_VALU" in d and "SQ_INSTS_VALU_INT64" in d for d in pair):
        # issue slots in full-rate lane-op units: 64-bit-class VALU ops (v_mad_u64_u32,
        # 64-bit shifts/adds) issue at half rate, so they count twice
        slots = sum((d["SQ_INSTS_VALU"] + d["SQ_INSTS_VALU_INT64"]) * 64 for d in pair)
        res["verify_w_exec_lane_slots_per_vote"] = slots / a.votes
        res["verify_valu_lane_insts_per_vote"] = sum(d["SQ_INSTS_VALU"] * 64 for d in pair) / a.votes
    k1b = [d for k, d in res["kernels"].items() if k.startswith("txv_k_scalarmult")]
    if k1b and "valu_issue_busy" in k1b[0]:
        res["k1b_valu_issue_busy"] = k1b[0]["valu_issue_busy"]
    if pair and all("hbm_read_bytes_corrected" in d and "hbm_write_bytes" in d for d in pair):
        res["hbm_bytes_per_launch"] = sum(d["hbm_read_bytes_corrected"] + d["hbm_write_bytes"] for d in pair)
        res["hbm_bytes_per_launch_raw_fetch"] = sum(d["hbm_read_bytes_raw"] + d["hbm_write_bytes"] for d in pair)
    # the tally chain after verify (kernels_flow.hip): HBM bytes per launch from the same passes
    tally_names = ("txv_k_tally_part", "txv_k_tally_min_x", "txv_k_tally_min", "txv_k_tally_resolve", "txv_k_tally_cross", "txv_k_status_out", "txv_k_event_top",
                   "txv_k_scan_count<AddedPred>", "txv_k_scan_apply<AddedPred>", "txv_k_scan_count<TouchedPred>",
                   "txv_k_scan_apply<TouchedPred>", "txv_k_scan_count<EventPred>", "txv_k_scan_apply<EventPred>")
    tk = [res["kernels"][k] for k in tally_names if k in res["kernels"]]
    if tk and all("hbm_read_bytes_corrected" in d and "hbm_write_bytes" in d for d in tk):
        res["tally_hbm_bytes_per_launch"] = sum(d["hbm_read_bytes_corrected"] + d["hbm_write_bytes"] for d in tk)
        res["tally_kernel_ns_per_launch"] = sum(d.get("avg_ns", 0.0) for d in tk)
        res["tally_kernels"] = [k for k in tally_names if k in res["kernels"]]
    txt = json.dumps(res, indent=1, sort_keys=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
