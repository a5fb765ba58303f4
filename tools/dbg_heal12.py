"""Debug: RS(12,4) heal of shards (0, 1) through the one-pass network kernel
on oracle-built records; prints which target headers / bodies match."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from oracle import oracle as O
    from rustfs_amd import Erasure, _lib
    k, m = 12, 4
    t = k + m
    for S, n in ((1000, 11), (1024, 8), (4096, 5)):
        rec = 32 + S
        rng = np.random.default_rng(S)
        shards = np.zeros((n, t, S), dtype=np.uint8)
        recs = np.zeros((t, n, rec), dtype=np.uint8)
        for s in range(n):
            shards[s, :k] = rng.integers(0, 256, (k, S), dtype=np.uint8)
            O.encode(k, m, shards[s])
            for i in range(t):
                recs[i, s, :32] = np.frombuffer(O.hh256s(shards[s, i].tobytes()), dtype=np.uint8)
                recs[i, s, 32:] = shards[s, i]
        files = [torch.from_numpy(recs[i].reshape(-1).copy()).cuda() for i in range(t)]
        e = Erasure(k, m, k * S)
        L = _lib.load()
        for eng in (_lib.RSG_RECORD_ENGINE_ONE_PASS, _lib.RSG_RECORD_ENGINE_TWO_PASS):
            _lib.check(L.rsg_set_record_engine(_lib.context(0).handle, eng))
            for lost in ((0, 1), (0, 12), (1,), (0, 1, 2)):
                tg = [torch.zeros(n * rec, dtype=torch.uint8, device="cuda") if i in lost else None for i in range(t)]
                st = e.heal_records_batch([None if i in lost else files[i] for i in range(t)], tg, S, n)
                res = []
                for i in lost:
                    got = tg[i].cpu().numpy().reshape(n, rec)
                    res.append((i, bool((got[:, :32] == recs[i][:, :32]).all()), bool((got[:, 32:] == recs[i][:, 32:]).all()),
                                int((got[:, :32] == 0).all(axis=1).sum())))
                print(f"S={S} n={n} engine={eng} lost={lost} status={set(st)} (shard, hdr ok, body ok, zero hdrs)={res}",
                      flush=True)
        _lib.check(L.rsg_set_record_engine(_lib.context(0).handle, _lib.RSG_RECORD_ENGINE_AUTO))


if __name__ == "__main__":
    main()
