"""BASELINE configurations at their full sizes, oracle-checked on samples.

Config 2: RS(8,4) encode of 1 MiB stripes at batch 4096 (6 GiB resident).
Config 3: RS(8,4) reconstruct of that batch with 1-4 missing shards.
Config 4: RS(8,4) encode + fused HighwayHash256S over the 64 KiB-16 MiB stripe
sweep at SURVEY §8(d)'s sizing (n = 4 GiB / stripe), which walks every fused
kernel the launcher picks for RS(8,4): the LDS-DMA kernel (n >= 2048), the
wide kernel with split encoders (4 MiB stripes: 4 per workgroup, n = 1024;
8 MiB: 2 per workgroup, n = 512) and ring E = 2 with 1024 chunks per shard
(16 MiB, S = 2 MiB).

The whole batch stays on the device; a sample of stripes (always the first and
the last) is copied back and checked byte for byte — parity and all k+m
digests — against the oracle (the digest is BitrotWriter's record prefix,
bitrot.rs:496-502).  Every other stripe is covered by the device-side
verify/round-trip properties.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GiB = 1 << 30


def _fill(torch, n, k, m, S, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    st = torch.empty((n, k + m, S), dtype=torch.uint8, device="cuda")
    for s0 in range(0, n, 256):
        s1 = min(n, s0 + 256)
        st[s0:s1, :k] = torch.randint(0, 256, (s1 - s0, k, S), dtype=torch.uint8, device="cuda", generator=g)
    st[:, k:] = 0xA5  # parity must be overwritten
    return st


def _sample(n, count=6):
    return sorted({0, n - 1, *np.random.default_rng(n).integers(0, n, count).tolist()})


def _check_stripes(oracle, st, dig, k, m, stripes):
    for s in stripes:
        got = st[s].cpu().numpy()
        ref = got.copy()
        ref[k:] = 0
        oracle.encode(k, m, ref)
        assert np.array_equal(got[k:], ref[k:]), f"parity of stripe {s}"
        if dig is not None:
            d = dig[s].cpu().numpy()
            for i in range(k + m):
                assert d[i].tobytes() == oracle.hh256s(ref[i]), (s, i)


@pytest.mark.parametrize("stripe_bytes", [64 << 10, 128 << 10, 256 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20,
                                          8 << 20, 16 << 20])
def test_config4_fused_sweep_at_survey_sizing(gpu, oracle, stripe_bytes):
    import torch
    from rustfs_amd import Erasure
    k, m = 8, 4
    S = stripe_bytes // k
    n = 4 * GiB // stripe_bytes
    st = _fill(torch, n, k, m, S, seed=stripe_bytes)
    dig = torch.zeros((n, k + m, 32), dtype=torch.uint8, device="cuda")
    e = Erasure(k, m, stripe_bytes)
    e.encode_batch(st, dig)
    torch.cuda.synchronize()
    _check_stripes(oracle, st, dig, k, m, _sample(n, 4 if S >= 1 << 20 else 8))
    # every stripe: parity consistent with its data (device-side verify)
    assert bool(e.verify_batch(st).all())
    # every digest: recompute with the standalone hash kernel and compare
    flat = st.reshape(n * (k + m), S)
    d2 = torch.zeros((n * (k + m), 32), dtype=torch.uint8, device="cuda")
    from rustfs_amd import _lib
    _lib.check(_lib.load().rsg_hash_batch_dev(_lib.context(0).handle, _lib.RSG_HASH_HIGHWAY256S, flat.data_ptr(), S, S,
                                              n * (k + m), d2.data_ptr(), torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert torch.equal(d2.reshape(n, k + m, 32), dig)
    del st, dig, flat, d2
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n,S", [(2049, 512), (2055, 4096), (4093, 4096), (2049, 131072)])
def test_fused_dma_kernel_ragged_batches(gpu, oracle, n, S):
    """RS(8,4) with >= 2048 stripes takes the LDS-DMA bit-sliced fused kernel
    (8 stripes per workgroup): batches that are not a multiple of 8 leave
    dead stripes in the last workgroup, which must neither store nor hash
    anything; one 512-byte step (S = 512) is the shortest walk."""
    import torch
    from rustfs_amd import Erasure, _lib
    k, m = 8, 4
    st = _fill(torch, n, k, m, S, seed=n + S)
    dig = torch.zeros((n + 1, k + m, 32), dtype=torch.uint8, device="cuda")  # one guard stripe of digests
    e = Erasure(k, m, k * S)
    e.encode_batch(st, dig[:n])
    torch.cuda.synchronize()
    _check_stripes(oracle, st, dig, k, m, sorted({0, 1, 7, 8, n - 9, n - 8, n - 2, n - 1}))
    assert bool(e.verify_batch(st).all())
    flat = st.reshape(n * (k + m), S)
    d2 = torch.zeros((n * (k + m), 32), dtype=torch.uint8, device="cuda")
    _lib.check(_lib.load().rsg_hash_batch_dev(_lib.context(0).handle, _lib.RSG_HASH_HIGHWAY256S, flat.data_ptr(), S, S,
                                              n * (k + m), d2.data_ptr(), torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert torch.equal(d2.reshape(n, k + m, 32), dig[:n])
    assert not bool(dig[n].any())  # nothing written past the batch


def test_config2_full_batch(gpu, oracle):
    """RS(8,4), S = 131072, n = 4096: sampled stripes vs the oracle; all stripes
    verified on the device; then config 3's reconstruct patterns on the same
    batch, each checked against the pre-erasure copy and the oracle sample."""
    import torch
    from rustfs_amd import Erasure, RSG_RECONSTRUCT_MISSING
    k, m, S, n = 8, 4, 131072, 4096
    st = _fill(torch, n, k, m, S, seed=2)
    e = Erasure(k, m, 1 << 20)
    e.encode_batch(st)
    torch.cuda.synchronize()
    sample = _sample(n, 10)
    _check_stripes(oracle, st, None, k, m, sample)
    assert bool(e.verify_batch(st).all())
    keep = {s: st[s].clone() for s in sample}
    for miss in ((0,), (0, 3), (0, 3, 5), (0, 3, 5, 7), (2, 9), (8, 9, 10, 11)):
        for i in miss:
            st[:, i] = 0
        e.reconstruct_batch(st, [i not in miss for i in range(k + m)], RSG_RECONSTRUCT_MISSING)
        torch.cuda.synchronize()
        for s in sample:
            assert torch.equal(st[s], keep[s]), (miss, s)
        assert bool(e.verify_batch(st).all()), miss
    del st
    torch.cuda.empty_cache()


def test_config5_geometry_full_batch_per_gpu(gpu, oracle):
    """RS(16,4), 1 MiB stripes: one GPU's share of config 5 (8192 stripes of the
    32768 split over 8), sampled against the oracle and verified whole."""
    import torch
    from rustfs_amd import Erasure
    k, m, S, n = 16, 4, 65536, 8192
    st = _fill(torch, n, k, m, S, seed=5)
    e = Erasure(k, m, 1 << 20)
    e.encode_batch(st)
    torch.cuda.synchronize()
    _check_stripes(oracle, st, None, k, m, _sample(n, 6))
    assert bool(e.verify_batch(st).all())
    del st
    torch.cuda.empty_cache()


@pytest.mark.parametrize("k,m", [(7, 4), (5, 4), (3, 3), (9, 4)])
def test_fused_table_enc_full_batch(gpu, oracle, k, m):
    """Config 4's kernel for geometries without a network (the table kernel's
    ENC mode: RS(7,4) 11 drives, RS(5,4) 9, RS(3,3) 6, RS(9,4) 13) at 1 MiB
    blocks, n = 4096 (ragged S, records at odd offsets): parity and every
    digest of sampled stripes against the oracle, the whole batch verified
    on the device."""
    import torch
    from rustfs_amd import Erasure
    S, n = -(-(1 << 20) // k), 4096
    st = _fill(torch, n, k, m, S, seed=40 + k)
    dig = torch.zeros((n, k + m, 32), dtype=torch.uint8, device="cuda")
    e = Erasure(k, m, 1 << 20)
    e.encode_batch(st, dig)
    torch.cuda.synchronize()
    _check_stripes(oracle, st, dig, k, m, _sample(n, 4))
    assert bool(e.verify_batch(st).all())
    del st, dig
    torch.cuda.empty_cache()


_VARIANT_SNIPPET = r"""
import sys, numpy as np, torch
sys.path.insert(0, {root!r})
from rustfs_amd import Erasure
from oracle import oracle as O
k, m, S, n = 8, 4, 4096, {n}
g = torch.Generator(device="cuda").manual_seed(n)
st = torch.zeros((n, k + m, S), dtype=torch.uint8, device="cuda")
st[:, :k] = torch.randint(0, 256, (n, k, S), dtype=torch.uint8, device="cuda", generator=g)
dig = torch.zeros((n, k + m, 32), dtype=torch.uint8, device="cuda")
Erasure(k, m, k * S).encode_batch(st, dig)
torch.cuda.synchronize()
for s in sorted({{0, 1, 5, n // 2, n - 2, n - 1}}):
    got = st[s].cpu().numpy(); ref = got.copy(); ref[k:] = 0
    O.encode(k, m, ref)
    assert np.array_equal(got[k:], ref[k:]), s
    d = dig[s].cpu().numpy()
    for i in range(k + m):
        assert d[i].tobytes() == O.hh256s(ref[i]), (s, i)
print("ok")
"""


@pytest.mark.parametrize("env", [{"RSG_DMA_SPW": "4"}, {"RSG_DMA_EW": "4"}, {"RSG_DMA_NT": "0"},
                                 {"RSG_ENC_PRIO": "3"}])
def test_dma_kernel_ab_variants(gpu, oracle, env):
    """The fused DMA kernel's A/B knobs, set through rsg_set_tuning for this
    test alone: four stripes per workgroup, the two-wave encoder, cached
    loads/stores, raised priorities — parity and digests vs the oracle on a
    ragged batch (n = 2051) and a 4-aligned one."""
    import os
    from rustfs_amd import _lib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with _lib.tuned(RSG_FUSED_KIND="dma", **env):
        for n in (2051, 2052):
            exec(_VARIANT_SNIPPET.format(root=root, n=n), {})


_WIDE_SNIPPET = r"""
import sys, numpy as np, torch
sys.path.insert(0, {root!r})
from rustfs_amd import Erasure
from oracle import oracle as O
k, m, S, n = 8, 4, {S}, {n}
g = torch.Generator(device="cuda").manual_seed(n + S)
st = torch.zeros((n, k + m, S), dtype=torch.uint8, device="cuda")
st[:, :k] = torch.randint(0, 256, (n, k, S), dtype=torch.uint8, device="cuda", generator=g)
st[:, k:] = 0xA5
dig = torch.zeros((n, k + m, 32), dtype=torch.uint8, device="cuda")
Erasure(k, m, k * S).encode_batch(st, dig)
torch.cuda.synchronize()
for s in sorted({{0, 1, 2, 3, n // 2, n - 3, n - 2, n - 1}} & set(range(n))):
    got = st[s].cpu().numpy(); ref = got.copy(); ref[k:] = 0
    O.encode(k, m, ref)
    assert np.array_equal(got[k:], ref[k:]), s
    d = dig[s].cpu().numpy()
    for i in range(k + m):
        assert d[i].tobytes() == O.hh256s(ref[i]), (s, i)
print("ok")
"""


@pytest.mark.parametrize("kind", ["wide2", "wide4", "split2", "split4"])
def test_wide_kernel_ragged_batches(gpu, oracle, kind):
    """k_encode_hash_wide (RS(8,4), few large stripes: SPW = 2 or 4 stripes
    per workgroup, 1 KiB steps, XOR-network encoder on 16 B per lane of a
    stripe pair): parity and all 12 digests vs the oracle on ragged batches
    (dead stripes in the last workgroup), a single step and many steps.
    Forced with the RSG_FUSED_KIND knob (rsg_set_tuning)."""
    import os
    from rustfs_amd import _lib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with _lib.tuned(RSG_FUSED_KIND=kind):
        for n, S in ((1, 1024), (3, 4096), (5, 2048), (6, 65536), (1027, 8192)):
            exec(_WIDE_SNIPPET.format(root=root, n=n, S=S), {})
