"""Multi-GPU dispatch of independent stripes.

Stripes never exchange data, so a batch is split contiguously over devices
(or over ranks, one process per GPU) with no collective on the data path.
"""
from __future__ import annotations

import threading
from typing import List, Sequence, Tuple


def split_batch(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous split of `total` stripes: rank r gets [start, start+count);
    the first total % world ranks take one extra stripe."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def encode_host_multi(erasure_by_device: Sequence, stripes, digests=None) -> None:
    """Encode a host batch (n, k+m, S) on several devices at once: one host
    thread per device drives its contiguous slice through
    Erasure.encode_batch_host (the C ABI releases the GIL)."""
    n = stripes.shape[0]
    world = len(erasure_by_device)
    errors: List[BaseException] = []

    def run(r: int) -> None:
        s0, cnt = split_batch(n, world, r)
        if cnt == 0:
            return
        try:
            d = digests[s0:s0 + cnt] if digests is not None else None
            erasure_by_device[r].encode_batch_host(stripes[s0:s0 + cnt], d)
        except BaseException as e:  # pragma: no cover - surfaced below
            errors.append(e)

    threads = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise errors[0]
