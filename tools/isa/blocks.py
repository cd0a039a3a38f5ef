#!/usr/bin/env python3
"""Per-basic-block instruction mix of one kernel in a hipcc -S listing (gfx950).

usage: python tools/isa/blocks.py file.s <kernel-substring> [--top N]
Prints each block's size and class counts, marks loop back-edges."""
import collections
import re
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\w+:\s*(;.*)?$", l)]
    st = next(i for i in starts if key in lines[i])
    en = next((i for i in starts if i > st), len(lines))
    blocks, cur, name = [], [], "entry"
    for l in lines[st:en]:
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            blocks.append((name, cur)); name, cur = m.group(1), []
            continue
        t = l.strip()
        if not t or t.startswith((";", ".", "//")):
            continue
        cur.append(t.split()[0])
    blocks.append((name, cur))
    order = {n: k for k, (n, _) in enumerate(blocks)}
    tot = collections.Counter()
    for k, (n, ins) in enumerate(blocks):
        c = collections.Counter(ins)
        tot.update(c)
        back = [i for i in ins if i.startswith("s_cbranch") or i == "s_branch"]
        cls = collections.Counter()
        for i, v in c.items():
            if i.startswith("v_mad_u64_u32"): cls["mad64"] += v
            elif i.startswith(("v_add_co", "v_addc", "v_sub_co", "v_subb", "v_add_u32", "v_sub_u32", "v_add3", "v_lshl_add", "v_add_lshl")): cls["add"] += v
            elif i.startswith(("v_mov", "v_cndmask")): cls["mov/sel"] += v
            elif i.startswith("v_"): cls["valu_other"] += v
            elif i.startswith("s_nop"): cls["nop"] += v
            elif i.startswith(("global_", "buffer_", "flat_")): cls["vmem"] += v
            elif i.startswith("ds_"): cls["lds"] += v
            elif i.startswith("s_"): cls["salu"] += v
        if len(ins) > 40:
            print(f"{n:>14} {len(ins):6d}  " + " ".join(f"{a}={b}" for a, b in sorted(cls.items())))
    print("TOTAL", sum(tot.values()))
    for i, v in tot.most_common(40):
        print(f"  {i:28s} {v}")


if __name__ == "__main__":
    main()
