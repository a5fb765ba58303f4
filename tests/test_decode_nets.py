"""The generated RS(8,4) one-pass GET / heal networks
(rustfs_amd/csrc/rs84_decode_nets.h, tools/gen_decode_nets.py; run by
k_decode_records_net) checked on the CPU against the oracle: for every
pattern, a random stripe is encoded by the oracle (the reference's
Vandermonde construction, erasure.rs:448-470), the first 8 present shards
are bit-sliced into the network's 64 input planes, and each output row must
equal the TRUE shard it stands for: the lost data (GET) or every lost shard
(heal), then the present non-survivor parity in ascending order — the rows
launch_get_one_pass / launch_heal_one_pass build (rsgpu.cpp), and the
rows the reference's reconstruct + surplus check produce
(erasure.rs:935-973, heal.rs:179-197).  Also pins the table's coefficient
rows to the oracle's decode matrix.  The GPU tests run every pattern's
kernel (test_gpu_decode_nets.py)."""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "rustfs_amd", "csrc", "rs84_decode_nets.h")
K, M, T = 8, 4, 12


def _table():
    src = open(HEADER).read()
    pats = []
    for m in re.finditer(r"\{0x([0-9a-f]+), (\d), (\d+), (\d), (\d), \{(.*?)\}\},  // (\d+)", src):
        rows = [[int(x) for x in r.split(",")] for r in re.findall(r"\{([0-9, ]+)\}", m.group(6))]
        pats.append(dict(absent=int(m.group(1), 16), heal=int(m.group(2)), nf=int(m.group(3)), R=int(m.group(4)),
                         nst=int(m.group(5)), coef=rows, pid=int(m.group(7))))
    return src, pats


def _program(src, pid, fn="net"):
    a = src.index(f"void {fn}<{pid}>(")
    b = src.index("\n}\n", a)
    return re.findall(r"(?:const uint32_t (t\d+)|O\[(\d+)\]) = (.+?);", src[a:b])


def _run(stmts, P):
    env = {"P": P}
    O = [0] * 32
    x3 = lambda a, b, c: a ^ b ^ c  # noqa: E731
    for t, o, expr in stmts:
        v = eval(expr.replace("0u", "0"), {"x3": x3}, env)
        if t:
            env[t] = v
        else:
            O[int(o)] = v
    return O


def _planes(rows: np.ndarray) -> list:
    """rows (8, 32) bytes -> 64 planes: plane c*8+j bit q = bit j of rows[c][q]."""
    bits = (rows[:, None, :] >> np.arange(8)[None, :, None]) & 1  # (8, 8, 32)
    w = (bits.astype(np.uint64) << np.arange(32, dtype=np.uint64)).sum(axis=2)
    return [int(x) for x in w.reshape(-1)]


def _bytes(O, R) -> np.ndarray:
    out = np.zeros((R, 32), dtype=np.uint8)
    for r in range(R):
        for i in range(8):
            v = O[8 * r + i]
            out[r] |= (((v >> np.arange(32)) & 1) << i).astype(np.uint8)
    return out


def _expected_rows(p, files):
    lost = [i for i in range(T) if p["absent"] >> i & 1]
    store = lost if p["heal"] else [i for i in lost if i < K]
    return store + files[K:]


def test_decode_net_table_shapes():
    src, pats = _table()
    assert len(pats) == int(re.search(r"kCount = (\d+)", src).group(1)) == 147
    keys = set()
    for p in pats:
        lost = [i for i in range(T) if p["absent"] >> i & 1]
        files = [i for i in range(T) if i not in lost]
        # one or two lost shards, or (heal) all four parity shards: the fused encode's rows
        assert (1 <= len(lost) <= 2 or (p["heal"] and lost == list(range(K, T)))) and p["nf"] == len(files)
        assert p["R"] == len(_expected_rows(p, files)) <= 4
        assert p["nst"] == (len(lost) if p["heal"] else len([i for i in lost if i < K])) >= 1
        keys.add((p["heal"], p["absent"]))
    assert len(keys) == len(pats)
    # GET: every pattern with a lost data shard; heal: every 1- and 2-shard loss
    assert sum(1 for p in pats if p["heal"]) == 12 + 66 + 1  # + all four parity shards: the fused encode
    assert sum(1 for p in pats if not p["heal"]) == 8 + 28 + 8 * 4


def test_decode_nets_rebuild_true_shards(oracle):
    src, pats = _table()
    rng = np.random.default_rng(2024)
    gm = oracle.matrix(K, M)
    for p in pats:
        stmts = _program(src, p["pid"])
        n_ops = sum(1 for t, o, e in stmts if t or "x3" in e or "^" in e)
        assert n_ops < 300, (p["pid"], n_ops)
        lost = [i for i in range(T) if p["absent"] >> i & 1]
        files = [i for i in range(T) if i not in lost]
        want_idx = _expected_rows(p, files)
        # the table's coefficient rows are the oracle's decode matrix rows
        inv = oracle.invert(gm[files[:K]])
        for r, idx in enumerate(want_idx):
            row = [0] * K
            for c in range(K):
                a = 0
                for i in range(K):
                    a ^= oracle.gf_mul(int(gm[idx][i]), int(inv[i][c]))
                row[c] = a
            assert row == p["coef"][r], (p["pid"], r)
        for trial in range(2):
            st = np.zeros((T, 32), dtype=np.uint8)
            st[:K] = rng.integers(0, 256, (K, 32), dtype=np.uint8)
            if trial == 1:
                st[:K] = 0xFF
            oracle.encode(K, M, st)
            got = _bytes(_run(stmts, _planes(st[files[:K]])), p["R"])
            assert np.array_equal(got, st[want_idx]), (p["pid"], trial)


# ---------------------------------------------------------------- RS(12,4)
HEADER12 = os.path.join(ROOT, "rustfs_amd", "csrc", "rs124_decode_nets.h")


def test_rs12_decode_nets_rebuild_true_shards(oracle):
    """RS(12,4) (rs124_decode_nets.h, k_decode_records_net12, four network
    waves): per pattern the four part networks over survivors 0-2, 3-5, 6-8
    and 9-11, XOR-combined, must give the true shards; the table is every 1-
    and 2-shard loss (GET: a data shard lost; heal: every loss) plus the heal
    of all four parity shards — the fused encode's rows, which must be the
    oracle's encode matrix — and its rows are the oracle's decode matrix rows."""
    k, t = 12, 16
    src = open(HEADER12).read()
    pats = []
    for m in re.finditer(r"\{0x([0-9a-f]+), (\d), (\d+), (\d), (\d), \{(.*?)\}\},  // (\d+)", src):
        rows = [[int(x) for x in r.split(",")] for r in re.findall(r"\{([0-9, ]+)\}", m.group(6))]
        pats.append(dict(absent=int(m.group(1), 16), heal=int(m.group(2)), nf=int(m.group(3)), R=int(m.group(4)),
                         nst=int(m.group(5)), coef=rows, pid=int(m.group(7))))
    assert len(pats) == int(re.search(r"kCount = (\d+)", src).group(1))
    assert sum(1 for p in pats if p["heal"]) == 16 + 120 + 1
    assert sum(1 for p in pats if not p["heal"]) == 12 + 114
    enc = [p for p in pats if p["heal"] and p["absent"] == 0xF000]
    assert len(enc) == 1
    gm = oracle.matrix(k, 4)
    assert enc[0]["coef"] == [[int(x) for x in gm[k + r]] for r in range(4)]
    rng = np.random.default_rng(124)
    for p in pats:
        lost = [i for i in range(t) if p["absent"] >> i & 1]
        files = [i for i in range(t) if i not in lost]
        store = lost if p["heal"] else [i for i in lost if i < k]
        want_idx = store + files[k:]
        assert p["R"] == len(want_idx) and p["nst"] == len(store) and p["nf"] == len(files)
        inv = oracle.invert(gm[files[:k]])
        for r, idx in enumerate(want_idx):
            row = []
            for c in range(k):
                a = 0
                for i in range(k):
                    a ^= oracle.gf_mul(int(gm[idx][i]), int(inv[i][c]))
                row.append(a)
            assert row == p["coef"][r], (p["pid"], r)
        st = np.zeros((t, 32), dtype=np.uint8)
        st[:k] = rng.integers(0, 256, (k, 32), dtype=np.uint8)
        oracle.encode(k, 4, st)
        acc = [0] * 32
        for q in range(4):
            part = _run(_program(src, f"{p['pid']}, {q}", "net_q"), _planes(st[files[3 * q:3 * q + 3]]))
            acc = [a ^ b for a, b in zip(acc, part)]
        got = _bytes(acc, p["R"])
        assert np.array_equal(got, st[want_idx]), p["pid"]


# ---------------------------------------------------------------- RS(10,4)
HEADER10 = os.path.join(ROOT, "rustfs_amd", "csrc", "rs104_decode_nets.h")


def test_rs10_decode_nets_rebuild_true_shards(oracle):
    """RS(10,4), the default geometry of a 14-drive set (rs104_decode_nets.h,
    k_decode_records_net10: rs_decode_netq.hip's four network waves over
    survivors 0-2, 3-5, 6-7, 8-9): per pattern the four part networks,
    XOR-combined, give the true shards; every 1- and 2-shard loss is listed
    and its rows are the oracle's decode matrix rows."""
    k, t = 10, 14
    parts = [(0, 3), (3, 3), (6, 2), (8, 2)]
    src = open(HEADER10).read()
    pats = []
    for m in re.finditer(r"\{0x([0-9a-f]+), (\d), (\d+), (\d), (\d), \{(.*?)\}\},  // (\d+)", src):
        rows = [[int(x) for x in r.split(",")] for r in re.findall(r"\{([0-9, ]+)\}", m.group(6))]
        pats.append(dict(absent=int(m.group(1), 16), heal=int(m.group(2)), nf=int(m.group(3)), R=int(m.group(4)),
                         nst=int(m.group(5)), coef=rows, pid=int(m.group(7))))
    assert len(pats) == int(re.search(r"kCount = (\d+)", src).group(1))
    assert sum(1 for p in pats if p["heal"]) == 14 + 91 + 1  # + all four parity shards: the fused encode
    assert sum(1 for p in pats if not p["heal"]) == 10 + 45 + 10 * 4
    rng = np.random.default_rng(104)
    gm = oracle.matrix(k, 4)
    for p in pats:
        lost = [i for i in range(t) if p["absent"] >> i & 1]
        files = [i for i in range(t) if i not in lost]
        store = lost if p["heal"] else [i for i in lost if i < k]
        want_idx = store + files[k:]
        assert p["R"] == len(want_idx) and p["nst"] == len(store) and p["nf"] == len(files)
        inv = oracle.invert(gm[files[:k]])
        for r, idx in enumerate(want_idx):
            row = []
            for c in range(k):
                a = 0
                for i in range(k):
                    a ^= oracle.gf_mul(int(gm[idx][i]), int(inv[i][c]))
                row.append(a)
            assert row == p["coef"][r], (p["pid"], r)
        st = np.zeros((t, 32), dtype=np.uint8)
        st[:k] = rng.integers(0, 256, (k, 32), dtype=np.uint8)
        oracle.encode(k, 4, st)
        acc = [0] * 32
        for q, (c0, cn) in enumerate(parts):
            part = _run(_program(src, f"{p['pid']}, {q}", "net_q"), _planes(st[files[c0:c0 + cn]]))
            acc = [a ^ b for a, b in zip(acc, part)]
        assert np.array_equal(_bytes(acc, p["R"]), st[want_idx]), p["pid"]


# ------------------------------------------------------------- RS(6,4)
@pytest.mark.parametrize("k", [6])
def test_rs6_decode_nets_rebuild_true_shards(oracle, k):
    """RS(6,4), the default geometry of a 10-drive set (rs64_decode_nets.h,
    k_decode_records_net6: rs_decode_net.hip over 6 survivors; RS(4,4)'s
    networks were dropped in round 6, its patterns run the table kernel):
    every 1- and 2-shard loss (GET:
    a data shard lost; heal: every loss), one network per pattern giving the
    true shards, its rows the oracle's decode matrix rows."""
    t = k + 4
    src = open(os.path.join(ROOT, "rustfs_amd", "csrc", f"rs{k}4_decode_nets.h")).read()
    pats = []
    for m in re.finditer(r"\{0x([0-9a-f]+), (\d), (\d+), (\d), (\d), \{(.*?)\}\},  // (\d+)", src):
        rows = [[int(x) for x in r.split(",")] for r in re.findall(r"\{([0-9, ]+)\}", m.group(6))]
        pats.append(dict(absent=int(m.group(1), 16), heal=int(m.group(2)), nf=int(m.group(3)), R=int(m.group(4)),
                         nst=int(m.group(5)), coef=rows, pid=int(m.group(7))))
    assert len(pats) == int(re.search(r"kCount = (\d+)", src).group(1))
    assert sum(1 for p in pats if p["heal"]) == t + t * (t - 1) // 2 + 1  # + the fused encode's
    assert sum(1 for p in pats if not p["heal"]) == k + k * (k - 1) // 2 + k * 4
    rng = np.random.default_rng(k * 10 + 4)
    gm = oracle.matrix(k, 4)
    for p in pats:
        lost = [i for i in range(t) if p["absent"] >> i & 1]
        files = [i for i in range(t) if i not in lost]
        store = lost if p["heal"] else [i for i in lost if i < k]
        want_idx = store + files[k:]
        assert p["R"] == len(want_idx) and p["nst"] == len(store) and p["nf"] == len(files)
        inv = oracle.invert(gm[files[:k]])
        for r, idx in enumerate(want_idx):
            row = []
            for c in range(k):
                a = 0
                for i in range(k):
                    a ^= oracle.gf_mul(int(gm[idx][i]), int(inv[i][c]))
                row.append(a)
            assert row == p["coef"][r], (p["pid"], r)
        st = np.zeros((t, 32), dtype=np.uint8)
        st[:k] = rng.integers(0, 256, (k, 32), dtype=np.uint8)
        oracle.encode(k, 4, st)
        got = _bytes(_run(_program(src, p["pid"]), _planes(st[files[:k]])), p["R"])
        assert np.array_equal(got, st[want_idx]), p["pid"]
