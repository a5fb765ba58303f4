#!/usr/bin/env python3
"""Generate rustfs_amd/csrc/rs84_decode_nets.h: compile-time XOR networks for
the RS(8,4) one-pass GET / heal kernel (rs_decode_net.hip), one per erasure
pattern of one or two lost shards.

The one-pass GET/heal (k_decode_records_dma) computes R <= 4 rows — rebuilt
data or parity, then surplus parity to compare — as GF(2^8) combinations of
the k = 8 survivors (the first 8 present shards, DecodePlan order), with
run-time v_perm tables: 3 v_perm + 1.5 XOR per word and coefficient, the
v_perm at half the XOR issue rate.  For a FIXED pattern the R x 8 matrix is a
constant, so, as for the encode (gen_xornet.py), the rows become a
straight-line three-input XOR network over the 64 bit planes of the
survivors, about half the issue cycles.  This script enumerates the patterns
the engines see when one or two disks are lost — GET (a data shard among the
lost: rows = missing data ascending, then the present non-survivor parity),
heal (targets = the lost shards ascending, then the present non-survivor
parity) — derives each matrix exactly as rsgpu.cpp does (Codec::plan and
plan_row: survivors' rows of V * inv(V[0..k)) inverted; data row = inv[i],
parity row = G[i] * inv), searches a network (gen_xornet.search, best of a
few seeds), checks it on random planes, and writes the header: the pattern
table (absent mask, mode, present files, R, stored rows, the coefficient
rows) and one `net<PID>` specialisation per pattern.  The launcher matches a
launch's coefficient rows against the table byte for byte, so a pattern not
listed (or any disagreement) keeps the run-time-table kernel.

RS(10,4) (`--k 10`, the default geometry of a 14-drive set) gets four
parts (survivors 0-2 / 3-5 / 6-7 / 8-9) like RS(12,4) (rs104_decode_nets.h,
rs_decode_netq.hip built with RSG_NETQ_K=10).

RS(6,4) (`--k 6`, the default geometry of a 10-drive set) is generated like
RS(8,4), one network over its 6 survivors (rs64_decode_nets.h, run by
rs_decode_net.hip built with RSG_NET_K=6).  `--k 4` (RS(4,4)) still
generates, but the library no longer builds it (round 6: 2-5 % over the
table kernel did not pay for its compile time).

RS(16,4) (`--k 16`) and RS(12,4) (`--k 12`, the default geometry of a
16-drive set, storageclass.rs:24-31): the survivors' 128 / 96 planes do not
fit one wave's registers beside the rows, so each pattern gets one network
per part of the survivors, each producing all R rows, and the kernel XORs the
parts: RS(16,4) two (survivors 0-7 / 8-15, rs_decode_net16.hip,
rs164_decode_nets.h `net_lo` / `net_hi`), RS(12,4) four (0-2 / 3-5 / 6-8 /
9-11, one network wave per SIMD, rs_decode_netq.hip, rs124_decode_nets.h
`net_q<PID, Q>`).  `--quarters` writes RS(8,4) in the same four-part form
(rs84q_decode_nets.h): measured 3-4 % slower than the one-wave RS(8,4)
networks (profiles/r04/l/) and not built.

Usage: python tools/gen_decode_nets.py [seeds] [--k 16|12] [--only heal:1,16 get:0,3 ...]
(writes the header)
"""
import multiprocessing
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_xornet as gx  # noqa: E402

K, M = 8, 4
T = K + M


def set_geometry(k, m):
    global K, M, T
    K, M, T = k, m, k + m


def invert(a):
    n = len(a)
    w = [list(r) + [1 if i == j else 0 for j in range(n)] for i, r in enumerate(a)]
    for c in range(n):
        p = c
        while w[p][c] == 0:
            p += 1
        w[p], w[c] = w[c], w[p]
        iv = gx.gpow(w[c][c], 254)
        w[c] = [gx.gmul(x, iv) for x in w[c]]
        for r in range(n):
            if r != c and w[r][c]:
                f = w[r][c]
                w[r] = [x ^ gx.gmul(f, y) for x, y in zip(w[r], w[c])]
    return [r[n:] for r in w]


def full_matrix():
    g = gx.encode_rows(K, M)
    return [[1 if i == j else 0 for j in range(K)] for i in range(K)] + g


def plan(present):
    """rsgpu.cpp Codec::plan: survivors = first K present; inv of their rows."""
    mat = full_matrix()
    surv = [i for i in range(T) if present[i]][:K]
    inv = invert([mat[s] for s in surv])
    return mat, surv, inv


def plan_row(mat, inv, idx):
    """rsgpu.cpp plan_row: inv[idx] for data, G[idx] * inv for parity."""
    if idx < K:
        return list(inv[idx])
    row = []
    for c in range(K):
        a = 0
        for i in range(K):
            a ^= gx.gmul(mat[idx][i], inv[i][c])
        row.append(a)
    return row


def patterns():
    """(absent mask, heal, nf, R, n_store, coef rows) for 1 and 2 lost shards."""
    out, seen = [], set()
    losses = [(a,) for a in range(T)] + [(a, b) for a in range(T) for b in range(a + 1, T)]
    # RS(12,4): also the heal of all four parity shards — rows = the encode
    # matrix over the data shards, which the fused encode + HH256S kernel
    # (rs_decode_netq.hip, k_encode_hash_net12) runs as its network
    every_parity = [tuple(range(K, T))] if K in (12, 10, 8, 6, 4) else []
    for heal in (0, 1):
        for lost in losses + (every_parity if heal else []):
            present = [0 if i in lost else 1 for i in range(T)]
            files = [i for i in range(T) if present[i]]
            mat, surv, inv = plan(present)
            assert surv == files[:K]
            if heal:
                store = list(lost)  # every lost shard is a target (launch_heal_one_pass)
            else:
                store = [i for i in lost if i < K]  # launch_get_one_pass: missing data
                if not store:
                    continue  # no data lost: the GET needs no rebuild
            rows = [plan_row(mat, inv, i) for i in store] + [plan_row(mat, inv, f) for f in files[K:]]
            assert len(rows) <= 4
            key = (heal, len(files), len(rows), len(store), tuple(map(tuple, rows)))
            if key in seen:
                continue
            seen.add(key)
            mask = sum(1 << i for i in lost)
            out.append((mask, heal, len(files), len(rows), len(store), rows))
    return out


def plane_rows(rows, c0=0, cn=None):
    """Output plane r*8+i over input planes (c-c0)*8+j, survivors c in [c0, c0+cn)."""
    cn = K if cn is None else cn
    return [{(c - c0) * 8 + j for c in range(c0, c0 + cn) for j in range(8) if (gx.gmul(rows[r][c], 1 << j) >> i) & 1}
            for r in range(len(rows)) for i in range(8)]


def best_network(args):
    rows, seeds, c0, cn = args
    pr = plane_rows(rows, c0, cn)
    best = None
    for seed in range(seeds):
        total, temps, rr = gx.search(pr, seed)
        if best is None or total < best[0]:
            best = (total, temps, rr, seed)
    check(pr, best[1], best[2])
    return best


def check(pr, temps, rr):
    rng = random.Random(7)
    for _ in range(8):
        val = {v: rng.getrandbits(32) for v in range(64)}
        for v, *t in temps:
            x = 0
            for a in t:
                x ^= val[a]
            val[v] = x
        for o in range(len(pr)):
            want = got = 0
            for v in pr[o]:
                want ^= val[v]
            for v in rr[o]:
                got ^= val[v]
            assert got == want, o


def emit_net(pid, pat, net, fn="net", what="", targs=None):
    mask, heal, nf, R, nst, rows = pat
    total, temps, rr, seed = net
    name = lambda v: f"P[{v}]" if v < 64 else f"t{v}"
    lost = [i for i in range(T) if mask >> i & 1]
    out = [f"// pattern {pid}: {'heal' if heal else 'GET'}, lost {lost}, {nf} present, R = {R} "
           f"({nst} stored){what}, {total} ops (seed {seed})",
           "template <>",
           f"__device__ __forceinline__ void {fn}<{pid if targs is None else targs}>(const uint32_t (&P)[64], "
           "uint32_t (&O)[32]) {"]
    for v, *t in temps:
        if len(t) == 3:
            out.append(f"    const uint32_t t{v} = x3({name(t[0])}, {name(t[1])}, {name(t[2])});")
        else:
            out.append(f"    const uint32_t t{v} = {name(t[0])} ^ {name(t[1])};")
    for o, s in enumerate(rr):
        terms = [name(v) for v in sorted(s)]
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


def main():
    args = sys.argv[1:]
    k = 8
    if "--k" in args:
        i = args.index("--k")
        k = int(args[i + 1])
        del args[i:i + 2]
    only = None
    if "--only" in args:
        i = args.index("--only")
        only = set(args[i + 1:])
        del args[i:]
    quarters = "--quarters" in args  # RS(8,4) in four parts of 2 survivors (rs_decode_netq.hip)
    if quarters:
        args.remove("--quarters")
    seeds = int(args[0]) if args else 4
    set_geometry(k, 4)
    pats = patterns()
    if only:  # prototype builds: e.g. heal:1,16 get:0,3
        pats = [p for p in pats if f"{'heal' if p[1] else 'get'}:{','.join(str(i) for i in range(T) if p[0] >> i & 1)}" in only]
    # RS(16,4): survivors 0-7 / 8-15 (two network waves, rs_decode_net16.hip);
    # RS(12,4): quarters 0-2 / 3-5 / 6-8 / 9-11 (four network waves, one per
    # SIMD, rs_decode_netq.hip)
    ka = 8
    halves = {4: [(0, 4)], 6: [(0, 6)], 8: [(0, 8)], 16: [(0, 8), (8, 8)], 12: [(0, 3), (3, 3), (6, 3), (9, 3)],
              10: [(0, 3), (3, 3), (6, 2), (8, 2)]}[K]
    if quarters:
        halves = [(c0, K // 4) for c0 in range(0, K, K // 4)]
    tasks = [(p[5], seeds, c0, cn) for c0, cn in halves for p in pats]
    with multiprocessing.Pool(min(8, os.cpu_count() or 1)) as pool:
        res = pool.map(best_network, tasks)
    nets = [res[h * len(pats):(h + 1) * len(pats)] for h in range(len(halves))]
    ops = [sum(n[i][0] for n in nets) for i in range(len(pats))]
    name = ("rs84q_decode_nets.h" if quarters else "rs84_decode_nets.h") if K == 8 else f"rs{K}{M}_decode_nets.h"
    space = f"decnet{'' if K == 8 and not quarters else K}{'q' if quarters else ''}"
    single = K <= 8 and not quarters  # one network over all survivors (rs_decode_net.hip)
    hdr = [
        f"// {name} — GENERATED by tools/gen_decode_nets.py (do not edit).",
        f"// RS({K},{M}) one-pass GET / heal rows as compile-time three-input XOR networks,",
        f"// one per erasure pattern of one or two lost shards: {len(pats)} patterns,",
        f"// {min(ops)}-{max(ops)} ops each (mean {sum(ops) / len(ops):.0f}).  P[c*8+j] = bit plane j of",
        f"// survivor c (the first {K} present shards{'' if single else ', in parts ' + ', '.join(f'{c0}-{c0 + cn - 1}' for c0, cn in halves)}), O[r*8+i] = bit plane i of row r",
        "// (rows [0, n_store) stored, the rest compared with the present",
        f"// non-survivor parity in ascending order).  Included by {'rs_decode_net.hip' if single else 'rs_decode_net16.hip' if K == 16 else 'rs_decode_netq.hip'}",
        "// inside namespace rsg, after x3().",
        "#pragma once",
        "",
        f"namespace {space} {{",
        "",
        "struct Pattern {",
        "    uint16_t absent;  // bit i: shard i lost" if T <= 16 else "    uint32_t absent;  // bit i: shard i lost",
        "    uint8_t heal;     // 1: heal (every lost shard a target), 0: GET",
        "    uint8_t nf;       // present files",
        "    uint8_t R;        // rows",
        "    uint8_t n_store;  // stored rows (the rest compared)",
        f"    uint8_t coef[4][{K}];",
        "};",
        "",
        f"constexpr int kCount = {len(pats)};",
        "constexpr Pattern kPatterns[kCount] = {",
    ]
    for pid, (mask, heal, nf, R, nst, rows) in enumerate(pats):
        rr = rows + [[0] * K] * (4 - R)
        cs = ", ".join("{" + ", ".join(str(x) for x in r) + "}" for r in rr)
        hdr.append(f"    {{0x{mask:03x}, {heal}, {nf}, {R}, {nst}, {{{cs}}}}},  // {pid}")
    hdr += ["};", ""]
    if single:
        hdr += ["template <int PID>", "__device__ void net(const uint32_t (&P)[64], uint32_t (&O)[32]);", ""]
        for pid, pat in enumerate(pats):
            hdr += emit_net(pid, pat, nets[0][pid])
            hdr.append("")
    elif K in (10, 12) or quarters:
        parts = ", ".join(f"{c0}-{c0 + cn - 1}" for c0, cn in halves)
        hdr += [f"// net_q<PID, Q>: all rows over part Q of the survivors ({parts}; its planes first in P)",
                "template <int PID, int Q>", "__device__ void net_q(const uint32_t (&P)[64], uint32_t (&O)[32]);", ""]
        for pid, pat in enumerate(pats):
            for q, (c0, cn) in enumerate(halves):
                hdr += emit_net(pid, pat, nets[q][pid], "net_q", f", survivors {c0}-{c0 + cn - 1}", f"{pid}, {q}")
            hdr.append("")
    else:
        hdr += [f"// net_lo: all rows over survivors 0-{ka - 1} (planes P[0..{8 * ka})); net_hi: over survivors "
                f"{ka}-{K - 1} (planes P[0..{8 * (K - ka)}))",
                "template <int PID>", "__device__ void net_lo(const uint32_t (&P)[64], uint32_t (&O)[32]);",
                "template <int PID>", "__device__ void net_hi(const uint32_t (&P)[64], uint32_t (&O)[32]);", ""]
        for pid, pat in enumerate(pats):
            hdr += emit_net(pid, pat, nets[0][pid], "net_lo", f", survivors 0-{ka - 1}")
            hdr += emit_net(pid, pat, nets[1][pid], "net_hi", f", survivors {ka}-{K - 1}")
            hdr.append("")
    hdr.append(f"}}  // namespace {space}")
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rustfs_amd", "csrc", name)
    with open(path, "w") as f:
        f.write("\n".join(hdr) + "\n")
    print(f"wrote {os.path.normpath(path)}: {len(pats)} patterns, {min(ops)}-{max(ops)} ops")


if __name__ == "__main__":
    main()
