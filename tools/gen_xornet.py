#!/usr/bin/env python3
"""Generate rustfs_amd/csrc/rs84_xornet.h (the RS(8,4) bit-sliced encode as a
short straight-line program of three-input XORs, v_bitop3_b32) and
rs164_xornet.h (RS(16,4): two networks over data shards 0-7 and 8-15, the
second XOR-accumulating into the first's output planes, so a lane needs only
64 input planes live at a time).

The bit-sliced encoder (gf_bitslice.h) computes each of the 32 output planes
(4 parity rows x 8 bits) as the XOR of the input planes (8 data shards x 8
bits) selected by the 32 x 64 GF(2) matrix of the RS(8,4) encode rows
(the reference's Vandermonde construction, erasure.rs:448-470 via
rustfs-erasure-codec).  Folding every output plane separately costs 504
three-input XORs for RS(8,4)'s 1040 ones.  Output planes share many sub-sums,
so a greedy common-subexpression search (Paar's heuristic, extended to
triples: repeatedly materialise the pair or triple of variables whose shared
use saves the most ops, counting ceil((t-1)/2) ops for a t-term row) finds a
network about half that size.  The search is seeded and deterministic; the
program is checked here on random planes against the plain matrix product.

Usage: python tools/gen_xornet.py [seeds]  (writes both headers)
"""
import collections
import itertools
import os
import random
import sys

K, M = 8, 4


def gmul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        b >>= 1
        a = ((a << 1) ^ (0x1D if a & 0x80 else 0)) & 0xFF
    return r


def gpow(a, n):
    r = 1
    for _ in range(n):
        r = gmul(r, a)
    return r


def encode_rows(k, m):
    """Parity rows of V * inv(V[0..k)), V[r][c] = r^c (gf_bitslice.h EncodeRows)."""
    w = [[0] * (2 * k) for _ in range(k)]
    for r in range(k):
        for c in range(k):
            w[r][c] = gpow(r, c)
        w[r][k + r] = 1
    for c in range(k):
        p = c
        while w[p][c] == 0:
            p += 1
        w[p], w[c] = w[c], w[p]
        iv = gpow(w[c][c], 254)
        w[c] = [gmul(x, iv) for x in w[c]]
        for r in range(k):
            if r != c and w[r][c]:
                f = w[r][c]
                w[r] = [x ^ gmul(f, y) for x, y in zip(w[r], w[c])]
    return [[_dot(k, r, c, w) for c in range(k)] for r in range(m)]


def _dot(k, r, c, w):
    a = 0
    for i in range(k):
        a ^= gmul(gpow(k + r, i), w[i][k + c])
    return a


def plane_rows(g, cols=range(K), acc=False):
    """Output plane r*8+i = XOR of input planes c*8+j with bit i of g[r][c]*2^j
    over the data shards `cols` (renumbered from 0).  acc: each row also takes
    its own previous value (variable ACC + r*8+i, unique to the row, so never
    shared)."""
    rows = []
    for r in range(len(g)):
        for i in range(8):
            s = {ci * 8 + j for ci, c in enumerate(cols) for j in range(8) if (gmul(g[r][c], 1 << j) >> i) & 1}
            if acc:
                s.add(ACC + r * 8 + i)
            rows.append(s)
    return rows


ACC = 1 << 16  # previous-output variables of an accumulating network


def cost(t):
    return t // 2 if t >= 1 else 0  # ceil((t-1)/2) three-input XORs


def search(rows, seed):
    rng = random.Random(seed)
    rr = [set(s) for s in rows]
    nv, temps = 64, []
    while True:
        best, bg = [], 0
        for width in (3, 2):
            cnt = collections.defaultdict(list)
            for ri, s in enumerate(rr):
                for t in itertools.combinations(sorted(s), width):
                    cnt[t].append(ri)
            for t, rl in cnt.items():
                if len(rl) < 2:
                    continue
                gain = sum(cost(len(rr[ri])) - cost(len(rr[ri]) - width + 1) for ri in rl) - 1
                if gain > bg:
                    bg, best = gain, [t]
                elif gain == bg:
                    best.append(t)
        if bg <= 0:
            break
        t = rng.choice(best)
        temps.append((nv,) + t)
        for s in rr:
            if all(x in s for x in t):
                s.difference_update(t)
                s.add(nv)
        nv += 1
    return len(temps) + sum(cost(len(s)) for s in rr), temps, rr


def name(v):
    return f"O[{v - ACC}]" if v >= ACC else f"P[{v}]" if v < 64 else f"t{v}"


def body(fn, temps, rr, acc=False):
    out = []
    args = "const uint32_t (&P)[64], uint32_t (&O)[32]"
    out.append(f"__device__ __forceinline__ void {fn}({args}) {{")
    for v, *t in temps:
        if len(t) == 3:
            out.append(f"    const uint32_t t{v} = x3({name(t[0])}, {name(t[1])}, {name(t[2])});")
        else:
            out.append(f"    const uint32_t t{v} = {name(t[0])} ^ {name(t[1])};")
    for o, s in enumerate(rr):
        # an accumulating row starts from its own previous value
        terms = [name(v) for v in sorted(s, key=lambda v: (v < ACC, v))]
        if not terms:
            out.append(f"    O[{o}] = 0u;")
            continue
        e = terms[0]
        k = 1
        while k + 1 < len(terms):
            e = f"x3({e}, {terms[k]}, {terms[k + 1]})"
            k += 2
        if k < len(terms):
            e = f"({e} ^ {terms[k]})"
        out.append(f"    O[{o}] = {e};")
    out.append("}")
    return out


def emit(temps, rr, total, seed, g):
    out = []
    out.append("// rs84_xornet.h — GENERATED by tools/gen_xornet.py (do not edit).")
    out.append("// RS(8,4) bit-sliced encode as a straight-line three-input XOR network:")
    out.append(f"// {total} ops ({len(temps)} shared sub-sums + the 32 output planes) against 504")
    out.append("// for folding each output plane separately (1040 ones in the 32 x 64 GF(2)")
    out.append(f"// matrix).  Search seed {seed}.  Parity rows (erasure.rs:448-470 construction):")
    for r in range(M):
        out.append(f"//   row {r}: {g[r]}")
    out.append("// P[c*8+j] = bit plane j of data shard c, O[r*8+i] = bit plane i of parity row r.")
    out.append("// Included by rs_kernels.hip inside namespace rsg, after x3().")
    out.append("#pragma once")
    out.append("")
    out.append("namespace xn {")
    out.append("")
    out += body("rs84_encode_planes", temps, rr)
    out.append("")
    out.append("}  // namespace xn")
    return "\n".join(out) + "\n"


def check(rows, temps, rr):
    rng = random.Random(1)
    for _ in range(8):
        val = {v: rng.getrandbits(32) for s in rows for v in s}
        for v, *t in temps:
            x = 0
            for a in t:
                x ^= val[a]
            val[v] = x
        for o in range(len(rows)):
            want = 0
            for v in rows[o]:
                want ^= val[v]
            got = 0
            for v in rr[o]:
                got ^= val[v]
            assert got == want, o


def best_network(rows, seeds, label):
    best = None
    for seed in range(seeds):
        total, temps, rr = search(rows, seed)
        print(f"{label} seed {seed}: {total} ops", flush=True)
        if best is None or total < best[0]:
            best = (total, temps, rr, seed)
    check(rows, *best[1:3])
    return best


def emit164(lo, hi, g, ones):
    out = []
    out.append("// rs164_xornet.h — GENERATED by tools/gen_xornet.py (do not edit).")
    out.append("// RS(16,4) bit-sliced encode as two straight-line three-input XOR networks:")
    out.append(f"// data shards 0-7 ({lo[0]} ops, search seed {lo[3]}) and 8-15 XOR-accumulated into the")
    out.append(f"// same 32 output planes ({hi[0]} ops, seed {hi[3]}), against {ones // 2} for folding each")
    out.append(f"// output plane separately ({ones} ones in the 32 x 128 GF(2) matrix).  Parity rows")
    out.append("// (erasure.rs:448-470 construction):")
    for r in range(len(g)):
        out.append(f"//   row {r}: {g[r]}")
    out.append("// P[c*8+j] = bit plane j of data shard c (c < 8) or c + 8 (hi), O[r*8+i] = bit")
    out.append("// plane i of parity row r.  Included by rs_kernels.hip inside namespace rsg, after x3().")
    out.append("#pragma once")
    out.append("")
    out.append("namespace xn {")
    out.append("")
    out += body("rs164_planes_lo", lo[1], lo[2])
    out.append("")
    out += body("rs164_planes_hi", hi[1], hi[2])
    out.append("")
    out.append("}  // namespace xn")
    return "\n".join(out) + "\n"


def main():
    seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    here = os.path.join(os.path.dirname(__file__), "..", "rustfs_amd", "csrc")
    g = encode_rows(K, M)
    rows = plane_rows(g)
    assert sum(len(s) for s in rows) == 1040
    total, temps, rr, seed = best_network(rows, seeds, "RS(8,4)")
    path = os.path.join(here, "rs84_xornet.h")
    with open(path, "w") as f:
        f.write(emit(temps, rr, total, seed, g))
    print(f"wrote {os.path.normpath(path)}: {total} ops (seed {seed})")

    g = encode_rows(16, 4)
    lo_rows = plane_rows(g, range(8))
    hi_rows = plane_rows(g, range(8, 16), acc=True)
    ones = sum(len(s) for s in lo_rows) + sum(len(s) - 1 for s in hi_rows)
    lo = best_network(lo_rows, seeds, "RS(16,4) lo")
    hi = best_network(hi_rows, seeds, "RS(16,4) hi")
    path = os.path.join(here, "rs164_xornet.h")
    with open(path, "w") as f:
        f.write(emit164(lo, hi, g, ones))
    print(f"wrote {os.path.normpath(path)}: {lo[0]} + {hi[0]} ops")


if __name__ == "__main__":
    main()
