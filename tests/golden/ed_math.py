"""Tiny pure-Python edwards25519 arithmetic used only to CRAFT adversarial inputs
(torsion points, non-canonical encodings, forged signatures) for the golden fixtures.
Verdicts are never computed here: they come from the oracle and are cross-checked with
OpenSSL.  Test infrastructure only."""
P = 2 ** 255 - 19
L = 2 ** 252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
I = pow(2, (P - 1) // 4, P)


def inv(x):
    return pow(x, P - 2, P)


def add(p, q):
    x1, y1 = p
    x2, y2 = q
    t = D * x1 * x2 * y1 * y2 % P
    x3 = (x1 * y2 + x2 * y1) * inv(1 + t) % P
    y3 = (y1 * y2 + x1 * x2) * inv(1 - t) % P
    return (x3, y3)


def mul(k, p):
    r = (0, 1)
    while k:
        if k & 1:
            r = add(r, p)
        p = add(p, p)
        k >>= 1
    return r


def recover_x(y, sign):
    """x for y (mod p) with parity sign, or None"""
    y %= P
    x2 = (y * y - 1) * inv(D * y * y + 1) % P
    if x2 == 0:
        return 0
    x = pow(x2, (P + 3) // 8, P)
    if (x * x - x2) % P:
        x = x * I % P
    if (x * x - x2) % P:
        return None
    if (x & 1) != sign:
        x = P - x
    return x


def encode(p):
    x, y = p
    return (y | ((x & 1) << 255)).to_bytes(32, "little")


def encode_raw(y_int, sign):
    return (y_int | (sign << 255)).to_bytes(32, "little")


B = (recover_x(4 * inv(5) % P, 0), 4 * inv(5) % P)


def order(p):
    for k in (1, 2, 4, 8):
        if mul(k, p) == (0, 1):
            return k
    return None


def torsion_points():
    """all 8 points of E[8]"""
    pts = set()
    import random
    rnd = random.Random(8)
    while len(pts) < 8:
        y = rnd.randrange(P)
        x = recover_x(y, rnd.randrange(2))
        if x is None:
            continue
        t = mul(L, (x, y))
        pts.add(t)
        for k in range(8):
            pts.add(mul(k, t))
    return sorted(pts)
