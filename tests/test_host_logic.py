"""Host-side mirror of the reference codec surface (no GPU): geometry, shard
sizing, construction errors and bitrot file-size arithmetic."""
import pytest

from rustfs_amd import Erasure, UnsupportedModernShardCount, ZeroBlockSize, ZeroDataShards, calc_shard_size
from rustfs_amd.bitrot import HashAlgorithm, bitrot_shard_file_size


def test_shard_file_size_reference_cases(rsgpu_lib, ref_vectors):
    for c in ref_vectors["shard_file_size"]["cases"]:
        e = Erasure(c["k"], c["m"], c["block_size"])
        assert e.shard_file_size(c["total"]) == c["want"], c


def test_calc_shard_size():
    # erasure.rs:655 plain ceiling division; docs/architecture/erasure-coding.md:123
    assert calc_shard_size(1 << 20, 6) == 174763
    assert calc_shard_size(1 << 20, 8) == 131072
    assert calc_shard_size(1 << 20, 16) == 65536
    assert calc_shard_size(1 << 20, 2) == 524288
    assert calc_shard_size(0, 4) == 0


def test_construction_errors(rsgpu_lib):
    with pytest.raises(ZeroDataShards):
        Erasure(0, 2, 1024)
    with pytest.raises(ZeroBlockSize):
        Erasure(4, 2, 0)
    with pytest.raises(UnsupportedModernShardCount):
        Erasure(200, 57, 1024)
    Erasure(200, 56, 1024)
    e = Erasure(4, 0, 1024)  # zero parity: no codec (erasure.rs:746-753)
    assert e.encoder is None


def test_shard_file_offset(rsgpu_lib):
    e = Erasure(4, 2, 8)
    assert e.shard_file_offset(0, 8, 16) == 4
    assert e.shard_file_offset(0, 3, 16) == 2
    assert e.shard_file_offset(0, 5, 5) == 2


def test_bitrot_shard_file_size():
    # io_support/bitrot.rs:801-805 / bitrot.rs:593-601
    h = HashAlgorithm.HighwayHash256S
    assert bitrot_shard_file_size(0, 1024, h) == 0
    assert bitrot_shard_file_size(1024, 1024, h) == 1056
    assert bitrot_shard_file_size(1025, 1024, h) == 1025 + 64
    assert bitrot_shard_file_size(524288, 524288, h) == 524288 + 32
    assert bitrot_shard_file_size(1000, 100, HashAlgorithm.NONE) == 1000


def test_bench_geometry_flags(monkeypatch):
    """bench.py takes the geometry as --k/--m or, through torchrun (whose
    parser claims a bare --m), as --data-shards/--parity-shards."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py", "--data-shards", "16", "--parity-shards", "4", "--total-batch", "8"])
    a = bench.parse()
    assert (a.k, a.m, a.total_batch) == (16, 4, 8)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--k", "6", "--m", "3"])
    a = bench.parse()
    assert (a.k, a.m) == (6, 3)
