"""Multi-GPU dispatch of independent stripes.

Stripes never exchange data, so a batch is split contiguously over devices
(or over ranks, one process per GPU) with no collective on the data path.
"""
from __future__ import annotations

import threading
from typing import Dict, List, Mapping, Optional, Sequence, Tuple


def rank_plan(gpus: int, master_port: int, base_env: Mapping[str, str]) -> List[Dict[str, str]]:
    """Environment of each of `gpus` rank processes started by one launcher on
    one node (bench.py --gpus N without torch.distributed.run): rank r binds
    device r.  The torch.distributed.run variables, rendezvous on 127.0.0.1."""
    if gpus < 1:
        raise ValueError("gpus must be >= 1")
    plans = []
    for r in range(gpus):
        env = dict(base_env)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus), LOCAL_WORLD_SIZE=str(gpus),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(master_port))
        plans.append(env)
    return plans


def check_world(gpus: int, world: int, devices: int, allow_shared: bool) -> Optional[str]:
    """Why a run of `world` ranks asked to measure `gpus` GPUs on a node with
    `devices` visible devices must not start (None: it may).  Ranks share a
    device only when explicitly allowed (a rehearsal on a smaller box): a
    silent share would time N ranks on fewer GPUs and report N."""
    if world != gpus:
        return f"--gpus {gpus} but {world} rank(s) were launched (WORLD_SIZE={world})"
    if devices < 1:
        return "no GPU visible"
    if devices < world and not allow_shared:
        return (f"{world} ranks need {world} GPUs but only {devices} are visible "
                f"(--allow-shared-device runs a rehearsal with ranks sharing devices)")
    return None


def device_for_rank(local_rank: int, devices: int, allow_shared: bool) -> int:
    """Device ordinal of a rank: its local rank, or (rehearsal only) the local
    rank modulo the visible devices."""
    if local_rank < devices:
        return local_rank
    if not allow_shared:
        raise ValueError(f"local rank {local_rank} has no device of its own ({devices} visible)")
    return local_rank % devices


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
