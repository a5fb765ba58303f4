"""Pin the CPU oracle to the reference's own known-answer vectors (CPU only).

The oracle (oracle/rs_oracle.c) is the checker for every GPU parity test, so it
must first reproduce every golden vector the reference's tests hold for this
path (tests/golden/reference_vectors.json).
"""
import numpy as np
import pytest

from conftest import compat_data


def test_rs42_compat_shard_digests(oracle, ref_vectors):
    v = ref_vectors["rs42_compat"]
    data = np.frombuffer(compat_data(v["len"]), dtype=np.uint8)
    k, m = v["k"], v["m"]
    S = -(-v["len"] // k)
    buf = np.zeros((k + m, S), dtype=np.uint8)
    buf.reshape(-1)[: data.size] = data
    oracle.encode(k, m, buf)
    got = [oracle.hh256s(buf[i]).hex() for i in range(k + m)]
    assert got == v["shard_hh256s"]


@pytest.mark.parametrize("algo", ["HighwayHash256S", "HighwayHash256SLegacy"])
def test_selftest_chain(oracle, ref_vectors, algo):
    v = ref_vectors["hh_selftest_chain"]
    f = oracle.hh256s if algo == "HighwayHash256S" else oracle.hh256s_legacy
    msg, s = b"", b""
    for _ in range(v["rounds"]):
        s = f(msg)
        msg += s
    assert s.hex() == v[algo]


def test_compat_7557(oracle, ref_vectors):
    assert oracle.hh256s(compat_data(7557)).hex() == ref_vectors["hh_compat_7557"]["HighwayHash256S"]


def test_bitrot_selftest_kats(oracle, ref_vectors):
    v = ref_vectors["bitrot_selftest_kat"]
    p = oracle.xorshift_payload(v["len"])
    assert oracle.hh256s(p).hex() == v["HighwayHash256S"]
    assert oracle.hh256s_legacy(p).hex() == v["HighwayHash256SLegacy"]


def test_matrices_match_derived_fixture(oracle, derived_vectors):
    for key, rows in derived_vectors["parity_rows"].items():
        k, m = map(int, key.split(","))
        got = [bytes(r).hex() for r in oracle.matrix(k, m)[k:]]
        assert got == rows, key


def test_matrix_is_systematic_and_mds(oracle):
    for k, m in [(2, 2), (4, 2), (6, 3), (8, 4), (12, 4), (16, 4), (10, 6)]:
        M = oracle.matrix(k, m)
        assert (M[:k] == np.eye(k, dtype=np.uint8)).all()
        # every k-row subset of a small geometry is invertible (MDS)
        if k + m <= 8:
            import itertools
            for rows in itertools.combinations(range(k + m), k):
                oracle.invert(M[list(rows)])


def test_oracle_roundtrip_all_patterns(oracle):
    import itertools
    rng = np.random.default_rng(7)
    k, m, S = 4, 3, 97
    ref = np.zeros((k + m, S), dtype=np.uint8)
    ref[:k] = rng.integers(0, 256, (k, S), dtype=np.uint8)
    oracle.encode(k, m, ref)
    assert oracle.verify(k, m, ref)
    for e in range(1, m + 1):
        for miss in itertools.combinations(range(k + m), e):
            buf = ref.copy()
            buf[list(miss)] = 0
            present = [i not in miss for i in range(k + m)]
            oracle.reconstruct(k, m, buf, present)
            assert (buf == ref).all(), miss
    bad = ref.copy()
    bad[k, 5] ^= 1
    assert not oracle.verify(k, m, bad)


def test_batch_baseline_matches_scalar(oracle):
    rng = np.random.default_rng(3)
    k, m, S, n = 8, 4, 4096 + 24, 5
    st = np.zeros((n, k + m, S), dtype=np.uint8)
    st[:, :k] = rng.integers(0, 256, (n, k, S), dtype=np.uint8)
    ref = st.copy()
    for s in range(n):
        oracle.encode(k, m, ref[s])
    dig = np.zeros((n, k + m, 32), dtype=np.uint8)
    oracle.encode_batch_mt(k, m, S, st, dig, threads=3)
    assert (st == ref).all()
    assert dig[2, 5].tobytes() == oracle.hh256s(ref[2, 5])
