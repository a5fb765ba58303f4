"""Multi-process (world_size 2, gloo, CPU) coverage of the N>1 path.

Stripes are independent, so the multi-GPU path is a contiguous batch split
with no data-path collective.  These tests check, on CPU, that
ranks' slices partition the batch, that per-rank encoding of the slices equals
encoding the whole batch (the oracle stands in for the per-GPU codec here),
and that bench.py's barrier + max-over-ranks timing protocol runs over gloo.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from rustfs_amd.dispatch import split_batch


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_split_batch_partitions():
    for total in (0, 1, 7, 4096, 32768, 32771):
        for world in (1, 2, 3, 4, 8):
            covered = []
            for r in range(world):
                s0, c = split_batch(total, world, r)
                covered.extend(range(s0, s0 + c))
            assert covered == list(range(total))
    with pytest.raises(ValueError):
        split_batch(10, 2, 2)


def _worker(rank, world, port, k, m, S, total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    from oracle import oracle as O
    rng = np.random.default_rng(123)
    full = np.zeros((total, k + m, S), dtype=np.uint8)
    full[:, :k] = rng.integers(0, 256, (total, k, S), dtype=np.uint8)
    s0, cnt = split_batch(total, world, rank)
    mine = full[s0:s0 + cnt].copy()
    O.encode_batch_mt(k, m, S, mine, None, 1)
    # gather every rank's parity on rank 0 (test-only; the product path has no collective)
    sizes = [split_batch(total, world, r)[1] for r in range(world)]
    t = torch.zeros((max(sizes), m, S), dtype=torch.uint8)  # gloo all_gather needs equal sizes
    t[:cnt] = torch.from_numpy(mine[:, k:].copy())
    gathered = [torch.zeros((max(sizes), m, S), dtype=torch.uint8) for _ in sizes]
    dist.all_gather(gathered, t)
    gathered = [g[:c] for g, c in zip(gathered, sizes)]
    # bench.py's timing protocol: barrier, then max over ranks
    dist.barrier()
    el = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if rank == 0:
        ref = full.copy()
        O.encode_batch_mt(k, m, S, ref, None, 1)
        got = torch.cat(gathered).numpy()
        q.put((bool((got == ref[:, k:]).all()), float(el.item())))
    dist.destroy_process_group()


@pytest.mark.parametrize("k,m,S,total", [(8, 4, 1024, 9), (16, 4, 512, 6)])
def test_two_rank_split_encode_matches_single(oracle, k, m, S, total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, k, m, S, total, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ok, max_el = q.get(timeout=5)
    assert ok
    assert max_el == 2.0
