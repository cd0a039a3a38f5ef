#!/usr/bin/env python3
"""Generates go-txflow_amd/csrc/fe_asm.h: the device bodies of the hot GF(2^255-19)
primitives (multiply, square, add, sub) as single inline-asm blocks for gfx950.

Why one block per primitive: hipcc's hazard recognizer assumes every inline-asm statement
may carry a dst-forwarding hazard and pads an `s_nop 0` between two adjacent asm statements
that share a register.  A multiply written as 64 small `mac` statements therefore carried
~40 nops.  Inside one block the sequence is ours: the mad -> addc carry hand-off through an
SGPR pair is interlocked by the hardware (the compiler emits the same back-to-back pairs).

Register plan inside the blocks (clobbered scratch, never live across a block):
  X = v[S+4:S+5], Y = v[S+6:S+7]  alternating 64-bit column accumulators; the overflow word of
                                  the column accumulating in one pair grows in the other
                                  pair's high half, so moving to the next column is one mov
  F = v[S+0:S+1]                  reduction carry (high half stays 0)
  Z = v[S+2:S+3]                  mad temporary
with S = TXV_ASM_SCRATCH (120: the top 8 VGPRs of a 128-VGPR / 4-waves-per-SIMD budget).

usage: python tools/gen/gen_fe_asm.py > go-txflow_amd/csrc/fe_asm.h
"""
S = 120
X = (S + 4, S + 5)
Y = (S + 6, S + 7)
F = (S + 0, S + 1)
Z = (S + 2, S + 3)


def pair(p):
    return f"v[{p[0]}:{p[1]}]"


def v(i):
    return f"v{i}"


class Asm:
    def __init__(self):
        self.lines = []

    def __call__(self, s):
        self.lines.append(s)

    def text(self):
        return "".join(f'      "{l}\\n\\t"\n' for l in self.lines)


def product_columns(asm, a, b, prods, out_word, fold=None):
    """Column-scanning 16-word product of the given (i, j) pairs into out_word(k) for
    k < 8 (a mov) and fold(k, reg) for k >= 8.  prods(k) -> list of (ai, bj) operand names.
    Column k accumulates in P = X or Y (by parity); its overflow word is the other pair's
    high half, which is exactly the next column's accumulator high word."""
    pairs = [X, Y]
    first = True
    for k in range(16):
        P = pairs[k % 2]
        Q = pairs[(k + 1) % 2]
        ps = prods(k)
        if k == 0:
            # column 0: a single product, no carry possible
            assert len(ps) == 1
            ai, bj = ps[0]
            asm(f"v_mad_u64_u32 {pair(P)}, %[cc], {ai}, {bj}, 0")
            asm(f"v_mov_b32 {v(Q[1])}, 0")
        else:
            for n, (ai, bj) in enumerate(ps):
                asm(f"v_mad_u64_u32 {pair(P)}, %[cc], {ai}, {bj}, {pair(P)}")
                if n == 0:
                    asm(f"v_addc_co_u32 {v(Q[1])}, %[cc], 0, 0, %[cc]")
                else:
                    asm(f"v_addc_co_u32 {v(Q[1])}, %[cc], {v(Q[1])}, 0, %[cc]")
            if not ps:
                # no product in this column: the carry-forward is the column value itself
                asm(f"v_mov_b32 {v(Q[1])}, 0")
        # column k word = P.lo ; next column accumulator = (P.hi, Q.hi)
        if k < 8:
            out_word(k, v(P[0]))
        else:
            fold(k, v(P[0]))
        if k < 15:
            asm(f"v_mov_b32 {v(Q[0])}, {v(P[1])}")


def emit_fold_init(asm):
    asm(f"v_mov_b64 {pair(F)}, 0")


def emit_fold(asm, h, k, w):
    """R'[k-8] = low word of (38 * w + c), c = high word of the previous fold (F.lo; F.hi = 0).
    One mad per high column; the low words are added to r by one chain at the end."""
    asm(f"v_mad_u64_u32 {pair(Z)}, %[cc], {w}, 38, {pair(F)}")
    asm(f"v_mov_b32 {h[k - 8]}, {v(Z[0])}")
    asm(f"v_mov_b32 {v(F[0])}, {v(Z[1])}")


def emit_final_fold(asm, r, h):
    """r += R' (one carry chain), top = last fold carry + chain carry (<= 39), r += 38 * top,
    then one more conditional +38 for a wrap past 2^256"""
    asm(f"v_add_co_u32 {r[0]}, %[cc], {r[0]}, {h[0]}")
    for i in range(1, 8):
        asm(f"v_addc_co_u32 {r[i]}, %[cc], {r[i]}, {h[i]}, %[cc]")
    asm(f"v_addc_co_u32 {v(F[0])}, %[cc], {v(F[0])}, 0, %[cc]")
    asm(f"v_mul_u32_u24 {v(Z[0])}, {v(F[0])}, 38")
    asm(f"v_add_co_u32 {r[0]}, %[cc], {r[0]}, {v(Z[0])}")
    for i in range(1, 8):
        asm(f"v_addc_co_u32 {r[i]}, %[cc], {r[i]}, 0, %[cc]")
    asm(f"v_cndmask_b32 {v(Z[0])}, 0, 38, %[cc]")
    asm(f"v_add_u32 {r[0]}, {r[0]}, {v(Z[0])}")


def gen_mul():
    asm = Asm()
    r = [f"%[r{i}]" for i in range(8)]
    a = [f"%[a{i}]" for i in range(8)]
    b = [f"%[b{i}]" for i in range(8)]
    h = [f"%[h{i}]" for i in range(8)]
    emit_fold_init(asm)

    def prods(k):
        return [(a[i], b[k - i]) for i in range(max(0, k - 7), min(k, 7) + 1)]

    product_columns(asm, a, b, prods, lambda k, w: asm(f"v_mov_b32 {r[k]}, {w}"),
                    lambda k, w: emit_fold(asm, h, k, w))
    emit_final_fold(asm, r, h)
    outs = ", ".join(f'[r{i}] "=&v"(r.v[{i}])' for i in range(8)) + ", " + \
        ", ".join(f'[h{i}] "=&v"(h[{i}])' for i in range(8)) + ', [cc] "=&s"(cc)'
    ins = ", ".join(f'[a{i}] "v"(a.v[{i}])' for i in range(8)) + ", " + \
        ", ".join(f'[b{i}] "v"(b.v[{i}])' for i in range(8))
    return asm.text(), outs, ins


def gen_sq():
    """t = 2U + sum a_i^2 2^(64i), U = sum_{i<j} a_i a_j 2^(32(i+j)); low 8 words of t in
    r[], high 8 in h[]; then the 38-fold of h into r."""
    asm = Asm()
    r = [f"%[r{i}]" for i in range(8)]
    h = [f"%[h{i}]" for i in range(8)]
    a = [f"%[a{i}]" for i in range(8)]
    t = r + h

    def prods(k):
        return [(a[i], a[k - i]) for i in range(max(0, k - 7), (k + 1) // 2) if i < k - i]

    # U by column scanning (column 0 and 15 empty); product_columns needs a product at
    # column 0, so scan U from column 1 and set t0 = 0 explicitly.
    pairs = [X, Y]
    asm(f"v_mov_b64 {pair(Y)}, 0")          # column-1 accumulator (lo, ovf-hi) = 0
    for k in range(1, 16):
        P = pairs[k % 2]
        Q = pairs[(k + 1) % 2]
        ps = prods(k)
        for n, (ai, bj) in enumerate(ps):
            asm(f"v_mad_u64_u32 {pair(P)}, %[cc], {ai}, {bj}, {pair(P)}")
            if n == 0:
                asm(f"v_addc_co_u32 {v(Q[1])}, %[cc], 0, 0, %[cc]")
            else:
                asm(f"v_addc_co_u32 {v(Q[1])}, %[cc], {v(Q[1])}, 0, %[cc]")
        if not ps:
            asm(f"v_mov_b32 {v(Q[1])}, 0")
        asm(f"v_mov_b32 {t[k]}, {v(P[0])}")
        if k < 15:
            asm(f"v_mov_b32 {v(Q[0])}, {v(P[1])}")
    # Y above: column 1 accumulates in pairs[1] = Y, so Y must start as 0 (done).
    # t = 2U: shift left by one across 16 words (t0 = 0)
    for j in range(15, 0, -1):
        lo = t[j - 1] if j > 1 else None
        if lo is None:
            asm(f"v_lshlrev_b32 {t[1]}, 1, {t[1]}")
        else:
            asm(f"v_alignbit_b32 {t[j]}, {t[j]}, {t[j - 1]}, 31")
    # + diagonal squares, one carry chain over 16 words (mad carry-outs go to cc2)
    for i in range(8):
        asm(f"v_mad_u64_u32 {pair(Z)}, %[cc2], {a[i]}, {a[i]}, 0")
        if i == 0:
            asm(f"v_mov_b32 {t[0]}, {v(Z[0])}")
            asm(f"v_add_co_u32 {t[1]}, %[cc], {t[1]}, {v(Z[1])}")
        else:
            asm(f"v_addc_co_u32 {t[2 * i]}, %[cc], {t[2 * i]}, {v(Z[0])}, %[cc]")
            asm(f"v_addc_co_u32 {t[2 * i + 1]}, %[cc], {t[2 * i + 1]}, {v(Z[1])}, %[cc]")
    emit_fold_init(asm)
    for k in range(8, 16):
        emit_fold(asm, h, k, h[k - 8])
    emit_final_fold(asm, r, h)
    outs = ", ".join(f'[r{i}] "=&v"(r.v[{i}])' for i in range(8)) + ", " + \
        ", ".join(f'[h{i}] "=&v"(h[{i}])' for i in range(8)) + ', [cc] "=&s"(cc), [cc2] "=&s"(cc2)'
    ins = ", ".join(f'[a{i}] "v"(a.v[{i}])' for i in range(8))
    return asm.text(), outs, ins


def gen_addsub(op):
    asm = Asm()
    first, rest = ("v_add_co_u32", "v_addc_co_u32") if op == "add" else ("v_sub_co_u32", "v_subb_co_u32")
    asm(f"{first} %[r0], %[cc], %[a0], %[b0]")
    for i in range(1, 8):
        asm(f"{rest} %[r{i}], %[cc], %[a{i}], %[b{i}], %[cc]")
    asm("v_cndmask_b32 %[w], 0, 38, %[cc]")
    asm(f"{first} %[r0], %[cc], %[r0], %[w]")
    for i in range(1, 8):
        asm(f"{rest} %[r{i}], %[cc], %[r{i}], 0, %[cc]")
    asm("v_cndmask_b32 %[w], 0, 38, %[cc]")
    asm(f"{'v_add_u32' if op == 'add' else 'v_sub_u32'} %[r0], %[r0], %[w]")
    outs = ", ".join(f'[r{i}] "=&v"(r.v[{i}])' for i in range(8)) + ', [w] "=&v"(w), [cc] "=&s"(cc)'
    ins = ", ".join(f'[a{i}] "v"(a.v[{i}])' for i in range(8)) + ", " + \
        ", ".join(f'[b{i}] "v"(b.v[{i}])' for i in range(8))
    return asm.text(), outs, ins


CLOBBER = ", ".join(f'"v{S + i}"' for i in range(8))

HDR = f"""// fe_asm.h — GENERATED by tools/gen/gen_fe_asm.py; do not edit by hand.
//
// Device bodies of fe_mul / fe_sq / fe_add / fe_sub for gfx950 as single inline-asm
// blocks (see the generator's docstring for the register plan and why).  Included by fe.h
// inside namespace txv for the device compile only.
#pragma once
#define TXV_ASM_SCRATCH {S}
"""


def fn(name, sig, decls, body, outs, ins, clobber=True):
    cl = f" : {CLOBBER}" if clobber else ""
    return (f"__device__ __forceinline__ void {name}({sig}) {{\n{decls}"
            f"  asm volatile(\n{body}      : {outs}\n      : {ins}{cl});\n}}\n")


def main():
    out = [HDR]
    body, outs, ins = gen_mul()
    out.append(fn("fe_mul_dev", "fe& r, const fe& a, const fe& b", "  uint32_t h[8]; uint64_t cc;\n", body, outs, ins))
    body, outs, ins = gen_sq()
    out.append(fn("fe_sq_dev", "fe& r, const fe& a", "  uint32_t h[8]; uint64_t cc, cc2;\n", body, outs, ins))
    for op in ("add", "sub"):
        body, outs, ins = gen_addsub(op)
        out.append(fn(f"fe_{op}_dev", "fe& r, const fe& a, const fe& b", "  uint32_t w; uint64_t cc;\n",
                      body, outs, ins, clobber=False))
    print("\n".join(out))


if __name__ == "__main__":
    main()
