#!/usr/bin/env python3
"""Generate raikv_amd/csrc/bs_aes.hpp: a bitsliced AESDEC round for CDNA4.

Why: the T-table round (meow_dev.hpp) costs 16 LDS lookups per key-round and
the Meow kernels sit at the LDS lookup ceiling.  A bitsliced
round costs only VALU (gfx950 v_bitop3_b32: any 3-input boolean function in
one op), so a share of the keys can be hashed without touching the LDS.

Layout ("8 keys per lane, byte lane = column"): register R[8r + i] holds, in
byte lane c (bits 8c..8c+7), bit i of state byte (row r, column c) of the
lane's 8 keys (key j in bit j of the byte lane).  Then
  * InvSubBytes is one 8-input circuit per row (4 columns x 8 keys at once),
  * InvShiftRows is a rotation of row r's registers by 8r bits,
  * InvMixColumns + basis changes are ONE 32x32 GF(2) matrix applied to the
    32 registers lane-parallel (every column, every key).

Math.  AESDEC(z, k) = InvMixColumns(InvSubBytes(InvShiftRows(z))) ^ k
(Intel _mm_aesdec_si128, used by /root/reference/src/key_hash.c:1075-1088).
Per byte InvS(z) = inv(f(z)) with f affine (f(z) = Ainv(z ^ 0x63)).  With the
GF(2^8) inversion done in a tower field GF(((2^2)^2)^2) through the field
isomorphism X:
    u  = X f(z)            ("pre-inversion form" of the state)
    v  = tinv(u)           (the nonlinear core, per byte)
    z' = InvMix(X^-1 v) ^ k
and the next round's u' = X f(z') = L v ^ kappa(k) where
    L = blockdiag(X Ainv) . InvMix . blockdiag(X^-1)    (per column, 32x32)
    kappa(k) = blockdiag(X Ainv) k ^ X f(0)             (per byte)
The state is carried in u-form across rounds; the last round uses
    Lout = InvMix . blockdiag(X^-1)   and   out = Lout v ^ k.
Keys enter as u1 = X f(F ^ K) = M1 K ^ X f(F) (M1 = X Ainv).

Every generated circuit is checked here, bit-exactly, against a direct
AESDEC over random states, and the whole 16-byte Meow chain against the
README known-answer vector (README.md:134) before the header is written.

usage: python3 tools/gen_bitslice.py [--out raikv_amd/csrc/bs_aes.hpp] [--tries N]
"""
from __future__ import annotations

import argparse
import os
import random
import sys

# ------------------------------------------------------------ GF(2^8), AES
def gmul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        if a & 0x100:
            a ^= 0x11B
        b >>= 1
    return r


def ginv(a):
    if a == 0:
        return 0
    r, e, x = 1, 254, a
    while e:
        if e & 1:
            r = gmul(r, x)
        x = gmul(x, x)
        e >>= 1
    return r


def rotl8(x, s):
    return ((x << s) | (x >> (8 - s))) & 0xFF


SBOX = [0] * 256
for _x in range(256):
    _b = ginv(_x)
    SBOX[_x] = _b ^ rotl8(_b, 1) ^ rotl8(_b, 2) ^ rotl8(_b, 3) ^ rotl8(_b, 4) ^ 0x63
INV_SBOX = [0] * 256
for _x in range(256):
    INV_SBOX[SBOX[_x]] = _x
IMC = [0x0E, 0x0B, 0x0D, 0x09]


def aesdec(s, k):
    """Intel AESDEC on 16-byte lists (byte 4c+r = row r, column c)."""
    t = [0] * 16
    for c in range(4):
        for r in range(4):
            t[4 * c + r] = INV_SBOX[s[4 * ((c - r) % 4) + r]]
    o = [0] * 16
    for c in range(4):
        for r in range(4):
            v = 0
            for q in range(4):
                v ^= gmul(IMC[(q - r) % 4], t[4 * c + q])
            o[4 * c + r] = v ^ k[4 * c + r]
    return o


# --------------------------------------------------------- tower field
def t4mul(a, b):  # GF(4) = GF(2)[w]/(w^2+w+1), element a1 w + a0 as 2 bits
    a0, a1, b0, b1 = a & 1, a >> 1, b & 1, b >> 1
    p, q = a1 & b1, a0 & b0
    r = (a1 ^ a0) & (b1 ^ b0)
    return ((r ^ q) << 1) | (p ^ q)


def mk16(phi):
    def mul(A, B):  # GF(16) = GF(4)[z]/(z^2+z+phi)
        A0, A1, B0, B1 = A & 3, A >> 2, B & 3, B >> 2
        hh = t4mul(A1, B1)
        ll = t4mul(A0, B0)
        mm = t4mul(A1 ^ A0, B1 ^ B0)
        return ((mm ^ ll) << 2) | (t4mul(phi, hh) ^ ll)
    return mul


def mk256(mul16, lam):
    def mul(A, B):  # GF(256) = GF(16)[y]/(y^2+y+lam)
        A0, A1, B0, B1 = A & 15, A >> 4, B & 15, B >> 4
        hh = mul16(A1, B1)
        ll = mul16(A0, B0)
        mm = mul16(A1 ^ A0, B1 ^ B0)
        return ((mm ^ ll) << 4) | (mul16(lam, hh) ^ ll)
    return mul


def find_tower():
    for phi in (2, 3):  # need z^2+z+phi irreducible over GF(4)
        if any(t4mul(z, z) ^ z ^ phi == 0 for z in range(4)):
            continue
        m16 = mk16(phi)
        for lam in range(1, 16):
            if any(m16(y, y) ^ y ^ lam == 0 for y in range(16)):
                continue
            m256 = mk256(m16, lam)
            for r in range(2, 256):  # root of x^8+x^4+x^3+x+1
                pw = [1]
                for _ in range(8):
                    pw.append(m256(pw[-1], r))
                if pw[8] ^ pw[4] ^ pw[3] ^ pw[1] ^ pw[0] == 0:
                    iso = [0] * 256
                    for x in range(256):
                        v = 0
                        for i in range(8):
                            if (x >> i) & 1:
                                v ^= pw[i]
                        iso[x] = v
                    if len(set(iso)) != 256:
                        continue
                    return phi, lam, m16, m256, iso
    raise RuntimeError("no tower")


PHI, LAM, M16, M256, ISO = find_tower()
ISO_INV = [0] * 256
for _x in range(256):
    ISO_INV[ISO[_x]] = _x
for _a in range(0, 256, 7):
    for _b in range(256):
        assert ISO[gmul(_a, _b)] == M256(ISO[_a], ISO[_b])


def tinv(u):
    return ISO[ginv(ISO_INV[u])]


def f_aff(z):  # InvS(z) = ginv(f(z))
    return ginv(INV_SBOX[z])


F0 = f_aff(0)


def lin_matrix(fn, nin, nout):
    """rows[k] = bitmask over inputs of output bit k, for a GF(2)-linear fn."""
    cols = [fn(1 << i) for i in range(nin)]
    assert fn(0) == 0
    return [sum(((cols[i] >> k) & 1) << i for i in range(nin)) for k in range(nout)]


def m1(z):  # X Ainv: linear part of z -> X f(z)
    return ISO[f_aff(z)] ^ ISO[F0]


def col_apply(fn_byte_in, fn_byte_out, x32):
    """column (4 bytes packed little-endian) -> InvMix over per-byte maps"""
    b = [fn_byte_in((x32 >> (8 * r)) & 0xFF) for r in range(4)]
    o = 0
    for r in range(4):
        v = 0
        for q in range(4):
            v ^= gmul(IMC[(q - r) % 4], b[q])
        o |= fn_byte_out(v) << (8 * r)
    return o


L_ROWS = lin_matrix(lambda x: col_apply(lambda b: ISO_INV[b], m1, x), 32, 32)
LOUT_ROWS = lin_matrix(lambda x: col_apply(lambda b: ISO_INV[b], lambda b: b, x), 32, 32)
M1_ROWS = lin_matrix(m1, 8, 8)


# ------------------------------------------------------------- circuits
class Circ:
    """2-input XOR/AND DAG with structural hashing; inputs are named."""

    def __init__(self):
        self.nodes = []  # (op, a, b) ; op in {'in', '^', '&'}
        self.names = []
        self.h = {}

    def inp(self, name):
        self.nodes.append(("in", None, None))
        self.names.append(name)
        return len(self.nodes) - 1

    def g(self, op, a, b):
        if a > b:
            a, b = b, a
        key = (op, a, b)
        if key in self.h:
            return self.h[key]
        self.nodes.append(key)
        self.names.append(None)
        self.h[key] = len(self.nodes) - 1
        return self.h[key]

    def x(self, a, b):
        return self.g("^", a, b)

    def a(self, a, b):
        return self.g("&", a, b)

    def xs(self, sigs):
        sigs = list(sigs)
        assert sigs
        r = sigs[0]
        for s in sigs[1:]:
            r = self.x(r, s)
        return r

    def eval(self, vals):
        """vals: dict input-node -> int (bit-parallel)."""
        out = {}
        for i, (op, a, b) in enumerate(self.nodes):
            if op == "in":
                out[i] = vals[i]
            elif op == "^":
                out[i] = out[a] ^ out[b]
            else:
                out[i] = out[a] & out[b]
        return out


# GF(4)/GF(16)/GF(256) element = tuple of signal ids, bit 0 first
def c4mul(C, a, b):
    p = C.a(a[1], b[1])
    q = C.a(a[0], b[0])
    r = C.a(C.x(a[1], a[0]), C.x(b[1], b[0]))
    return (C.x(p, q), C.x(r, q))


def c4add(C, a, b):
    return (C.x(a[0], b[0]), C.x(a[1], b[1]))


def c4sq(C, a):  # (a1 w + a0)^2 = a1 w + (a1 + a0)
    return (C.x(a[1], a[0]), a[1])


def c4const(C, k, a):  # multiply by constant k in GF(4) (linear)
    if k == 1:
        return a
    if k == 2:  # w: (a1+a0) w + a1
        return (a[1], C.x(a[1], a[0]))
    if k == 3:  # w^2 = w+1: a0 w + (a1+a0)
        return (C.x(a[1], a[0]), a[0])
    raise ValueError


def c16mul(C, A, B):
    A0, A1, B0, B1 = A[:2], A[2:], B[:2], B[2:]
    hh = c4mul(C, A1, B1)
    ll = c4mul(C, A0, B0)
    mm = c4mul(C, c4add(C, A1, A0), c4add(C, B1, B0))
    return c4add(C, c4const(C, PHI, hh), ll) + c4add(C, mm, ll)


def c16inv(C, A):
    A0, A1 = A[:2], A[2:]
    d = c4add(C, c4add(C, c4const(C, PHI, c4sq(C, A1)), c4mul(C, A1, A0)), c4sq(C, A0))
    e = c4sq(C, d)
    return c4mul(C, c4add(C, A1, A0), e) + c4mul(C, A1, e)


def c16lin(C, fn, A):
    """GF(2)-linear map on a GF(16) element via its matrix."""
    rows = lin_matrix(fn, 4, 4)
    out = []
    for r in rows:
        sigs = [A[i] for i in range(4) if (r >> i) & 1]
        out.append(C.xs(sigs) if sigs else None)
    assert all(o is not None for o in out)
    return tuple(out)


def c256inv(C, B):
    B0, B1 = B[:4], B[4:]
    # d = lam*B1^2 + B1*B0 + B0^2 ; the squares and the lam product are linear
    sq_lam = c16lin(C, lambda x: M16(LAM, M16(x, x)), B1)
    sq0 = c16lin(C, lambda x: M16(x, x), B0)
    d = tuple(C.x(C.x(p, q), r) for p, q, r in zip(sq_lam, c16mul(C, B1, B0), sq0))
    e = c16inv(C, d)
    s = tuple(C.x(p, q) for p, q in zip(B1, B0))
    return c16mul(C, s, e) + c16mul(C, B1, e)


def build_inv():
    C = Circ()
    ins = [C.inp("u%d" % i) for i in range(8)]
    outs = list(c256inv(C, tuple(ins)))
    # verify exhaustively (bit-parallel over the 256 inputs)
    vals = {ins[i]: sum(((x >> i) & 1) << x for x in range(256)) for i in range(8)}
    ev = C.eval(vals)
    for x in range(256):
        y = sum(((ev[outs[i]] >> x) & 1) << i for i in range(8))
        assert y == tinv(x), (x, y, tinv(x))
    return C, ins, outs


def build_linear(rows, nin, extra, rng, mode):
    """XOR network for out_k = parity(rows[k] & in) ^ extra_k (Paar-style
    greedy pair extraction with random tie-breaks).  extra: list of lists
    of extra input names per output (round keys: never shared)."""
    C = Circ()
    ins = [C.inp("v%d" % i) for i in range(nin)]
    sets = [set(ins[i] for i in range(nin) if (r >> i) & 1) for r in rows]
    if mode == "paar":
        while True:
            cnt = {}
            for s in sets:
                ls = sorted(s)
                for i in range(len(ls)):
                    for j in range(i + 1, len(ls)):
                        cnt[(ls[i], ls[j])] = cnt.get((ls[i], ls[j]), 0) + 1
            if not cnt:
                break
            best = max(cnt.values())
            if best < 2:
                break
            cands = [p for p, c in cnt.items() if c == best]
            a, b = rng.choice(cands)
            n = C.x(a, b)
            for s in sets:
                if a in s and b in s:
                    s.discard(a)
                    s.discard(b)
                    s.add(n)
    outs = []
    for k, s in enumerate(sets):
        ls = list(s)
        rng.shuffle(ls)
        ex = [C.inp(nm) for nm in extra[k]]
        outs.append(C.xs(ls + ex))
    return C, ins, outs


# ------------------------------------------------------------- LUT3 mapping
def lut3_map(C, outs):
    """Greedy mapping of the 2-input DAG onto 3-input LUT nodes.
    Returns list of (node, inputs(list of <=3 node ids), truth table byte)
    in topological order; `outs` nodes are always materialised."""
    n = len(C.nodes)
    fan = [0] * n
    for op, a, b in C.nodes:
        if op != "in":
            fan[a] += 1
            fan[b] += 1
    for o in outs:
        fan[o] += 1
    # cone[i]: (inputs tuple, function over those inputs as python callable via tt)
    cone = {}

    def tt_of(inputs, fn):
        t = 0
        k = len(inputs)
        for idx in range(1 << k):
            bits = [(idx >> (k - 1 - q)) & 1 for q in range(k)]  # inputs[0] = MSB
            if fn(dict(zip(inputs, bits))):
                t |= 1 << idx
        return t

    def leaf(i):
        return C.nodes[i][0] == "in"

    # represent each node's implemented function as (inputs, tt with k inputs)
    impl = {}
    for i, (op, a, b) in enumerate(C.nodes):
        if op == "in":
            continue
        # candidate absorptions: a child may be absorbed if it is a gate with fanout 1
        best = None
        opts = []
        ca = impl.get(a) if (not leaf(a) and fan[a] == 1) else None
        cb = impl.get(b) if (not leaf(b) and fan[b] == 1) else None
        for ua in ([False, True] if ca else [False]):
            for ub in ([False, True] if cb else [False]):
                ins_a = list(ca[0]) if ua else [a]
                ins_b = list(cb[0]) if ub else [b]
                ins = []
                for s in ins_a + ins_b:
                    if s not in ins:
                        ins.append(s)
                if len(ins) > 3:
                    continue
                opts.append((ua, ub, ins))
        # prefer absorbing more (fewer materialised nodes), then fewer inputs
        opts.sort(key=lambda o: (-(o[0] + o[1]), len(o[2])))
        ua, ub, ins = opts[0]

        def val(s, env, absorbed, child):
            if absorbed:
                cins, ctt = child
                k = len(cins)
                idx = 0
                for q, cs in enumerate(cins):
                    idx |= env[cs] << (k - 1 - q)
                return (ctt >> idx) & 1
            return env[s]

        def fn(env, op=op, a=a, b=b, ua=ua, ub=ub, ca=ca, cb=cb):
            x = val(a, env, ua, ca)
            y = val(b, env, ub, cb)
            return x ^ y if op == "^" else x & y

        impl[i] = (tuple(ins), tt_of(ins, fn), ua, ub)
        impl[i] = (impl[i][0], impl[i][1])
        # record absorption so children are not materialised
        if ua:
            fan[a] = -1  # absorbed
        if ub:
            fan[b] = -1
    # materialise: every non-leaf node with fan != -1 that is reachable
    need = set()
    stack = list(outs)
    while stack:
        s = stack.pop()
        if s in need or leaf(s):
            continue
        need.add(s)
        for x in impl[s][0]:
            stack.append(x)
    prog = [(i, list(impl[i][0]), impl[i][1]) for i in sorted(need)]
    return prog


def check_prog(C, prog, ins, outs, trials=64, rng=None):
    rng = rng or random.Random(1)
    vals = {i: rng.getrandbits(64) for i in range(len(C.nodes)) if C.nodes[i][0] == "in"}
    ref = C.eval(vals)
    got = dict(vals)
    for node, pins, tt in prog:
        k = len(pins)
        r = 0
        for bit in range(64):
            idx = 0
            for q, s in enumerate(pins):
                idx |= ((got[s] >> bit) & 1) << (k - 1 - q)
            r |= ((tt >> idx) & 1) << bit
        got[node] = r
    for o in outs:
        assert got[o] == ref[o]


def ops_of(prog):
    return len(prog)


# ------------------------------------------------------------- emission
def tt3(tt, k):
    """expand a k-input table (inputs MSB-first) to the 3-input bitop3 table
    with unused trailing operands."""
    if k == 3:
        return tt
    t = 0
    for idx in range(8):
        sub = idx >> (3 - k)
        if (tt >> sub) & 1:
            t |= 1 << idx
    return t


def emit_prog(lines, prog, C, name_of, out_names, indent="  "):
    tmp = {}
    for node, pins, tt in prog:
        args = [name_of(p) if C.nodes[p][0] == "in" else tmp[p] for p in pins]
        k = len(args)
        nm = "t%d" % node
        tmp[node] = nm
        if k == 1:
            # identity / not
            if tt == 0b10:
                expr = args[0]
            elif tt == 0b01:
                expr = "~%s" % args[0]
            else:
                raise ValueError(tt)
        elif k == 2 and tt == 0b0110:
            expr = "%s ^ %s" % tuple(args)
        elif k == 2 and tt == 0b1000:
            expr = "%s & %s" % tuple(args)
        else:
            a3 = args + [args[-1]] * (3 - k)
            expr = "bop3<0x%02x>(%s, %s, %s)" % (tt3(tt, k), a3[0], a3[1], a3[2])
        lines.append("%sconst uint32_t %s = %s;" % (indent, nm, expr))
    return tmp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                               "raikv_amd", "csrc", "bs_aes.hpp"))
    ap.add_argument("--tries", type=int, default=200)
    a = ap.parse_args()
    rng = random.Random(12345)

    Ci, ins_i, outs_i = build_inv()
    prog_i = lut3_map(Ci, outs_i)
    check_prog(Ci, prog_i, ins_i, outs_i)
    nand = sum(1 for op, _, _ in Ci.nodes if op == "&")
    nxor = sum(1 for op, _, _ in Ci.nodes if op == "^")
    print("tower phi=%d lam=%d; inversion: %d AND + %d XOR gates -> %d LUT3 ops" %
          (PHI, LAM, nand, nxor, len(prog_i)), file=sys.stderr)

    def best_linear(rows, nin, extra, tag):
        best = None
        for t in range(a.tries):
            C, ins, outs = build_linear(rows, nin, extra, rng, "paar")
            prog = lut3_map(C, outs)
            if best is None or len(prog) < len(best[3]):
                best = (C, ins, outs, prog)
        C, ins, outs, prog = best
        check_prog(C, prog, ins, outs)
        print("%s: %d LUT3 ops" % (tag, len(prog)), file=sys.stderr)
        return best

    key1 = [["k%d" % k] for k in range(32)]
    Lk = best_linear(L_ROWS, 32, key1, "L (+ round key)")
    Lo = best_linear(LOUT_ROWS, 32, key1, "Lout (+ key)")
    Mk = best_linear(M1_ROWS, 8, [["k%d" % k] for k in range(8)], "M1 (+ const)")

    # ---------------- end-to-end check of the bitsliced round in python
    def bs_round_py(u_bytes, kappa, lin_rows):
        v = [tinv(x) for x in u_bytes]
        # InvShiftRows on v (state-byte index 4c+r)
        w = [0] * 16
        for c in range(4):
            for r in range(4):
                w[4 * c + r] = v[4 * ((c - r) % 4) + r]
        out = []
        for c in range(4):
            x = w[4 * c] | (w[4 * c + 1] << 8) | (w[4 * c + 2] << 16) | (w[4 * c + 3] << 24)
            y = 0
            for k, row in enumerate(lin_rows):
                y |= (bin(row & x).count("1") & 1) << k
            out += [(y >> (8 * r)) & 0xFF for r in range(4)]
        return [o ^ q for o, q in zip(out, kappa)]

    def u_form(z):
        return [ISO[f_aff(b)] for b in z]

    def kappa(k):
        return [m1(b) ^ ISO[F0] for b in k]

    r2 = random.Random(7)
    for _ in range(200):
        z = [r2.randrange(256) for _ in range(16)]
        k = [r2.randrange(256) for _ in range(16)]
        ref = aesdec(z, k)
        assert bs_round_py(u_form(z), kappa(k), L_ROWS) == u_form(ref)
        assert bs_round_py(u_form(z), k, LOUT_ROWS) == ref

    # ---------------- write the header
    L = []
    L.append("// bs_aes.hpp -- GENERATED by tools/gen_bitslice.py; do not edit.")
    L.append("// Bitsliced AESDEC for CDNA4 (see the generator's docstring for the math).")
    L.append("// Register R[8r+i], byte lane c, bit j: bit i of state byte (row r, column c)")
    L.append("// of the lane's key j, in 'u-form' (pre-inversion tower-field basis).")
    L.append("// tower: GF(4)=GF(2)[w]/(w^2+w+1), GF(16)=GF(4)[z]/(z^2+z+%d), GF(256)=GF(16)[y]/(y^2+y+%d)" %
             (PHI, LAM))
    L.append("// ops: inversion %d, L %d, Lout %d, M1 %d (v_bitop3_b32 / v_xor / v_and)" %
             (len(prog_i), len(Lk[3]), len(Lo[3]), len(Mk[3])))
    L.append("// Needs KVH_BS_DEV (function qualifiers) and bop3<TT>(a, b, c) (v_bitop3_b32,")
    L.append("// truth-table index a*4+b*2+c) from bs_prelude.hpp (device) or a host test prelude.")
    L.append("#pragma once")
    L.append("#include <stdint.h>")
    L.append("namespace kvh { namespace bs {")
    L.append("")
    L.append("// u-form of a standard state byte: kappa(z) = X f(z) = M1 z ^ X f(0); the round-key")
    L.append("// term of a round with key k is kappa(k) as well (same affine map)")
    L.append("constexpr uint8_t kKappa[256] = {%s};" % ", ".join("%d" % ISO[f_aff(z)] for z in range(256)))
    L.append("")
    # inversion
    L.append("// v[0..7] = tower inverse of u[0..7] (one S-box row: 4 columns x 8 keys)")
    L.append("KVH_BS_DEV void inv8(const uint32_t* u, uint32_t* v) {")
    names = {ins_i[i]: "u[%d]" % i for i in range(8)}
    tmp = emit_prog(L, prog_i, Ci, lambda p: names[p], None)
    for i, o in enumerate(outs_i):
        L.append("  v[%d] = %s;" % (i, tmp[o] if o in tmp else names[o]))
    L.append("}")
    L.append("")

    def emit_lin(fname, best, sig, nin, keynames):
        C, ins, outs, prog = best
        L.append("KVH_BS_DEV void %s(%s) {" % (fname, sig))
        nm = {ins[i]: "v[%d]" % i for i in range(nin)}
        for i, (op, _, _) in enumerate(C.nodes):
            if op == "in" and i not in nm:
                nm[i] = keynames(C.names[i])
        tmp = emit_prog(L, prog, C, lambda p: nm[p], None)
        for k, o in enumerate(outs):
            L.append("  u[%d] = %s;" % (k, tmp[o] if o in tmp else nm[o]))
        L.append("}")
        L.append("")

    kn = lambda s: ("k[%s]" % s[1:]) if s[0] == "k" else ("q[%s]" % s[1:])
    L.append("// u[k] = (L v)[k] ^ k[k]: InvMixColumns between basis changes, next round's u-form")
    emit_lin("lin", Lk, "const uint32_t* v, const uint32_t* k, uint32_t* u", 32, kn)
    L.append("// u[k] = (Lout v)[k] ^ k[k]: last round, standard byte basis")
    emit_lin("lin_out", Lo, "const uint32_t* v, const uint32_t* k, uint32_t* u", 32, kn)
    L.append("// u[k] = (M1 v)[k] ^ k[k]: standard byte -> u-form linear part (data key)")
    emit_lin("m1", Mk, "const uint32_t* v, const uint32_t* k, uint32_t* u", 8, kn)
    L.append("}}  // namespace kvh::bs")
    src = "\n".join(L) + "\n"
    with open(a.out, "w") as fh:
        fh.write(src)
    print("wrote %s" % a.out, file=sys.stderr)


if __name__ == "__main__":
    main()
