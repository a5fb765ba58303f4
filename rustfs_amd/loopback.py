"""Single-node loopback erasure set: BASELINE config 1 plumbing.

A minimal mirror of the reference's set-level PUT/GET for one erasure set of
local directories (`SetDisks::put_object`, crates/ecstore/src/set_disk/ops/object.rs:1852;
`get_object_with_fileinfo`, crates/ecstore/src/set_disk/read.rs:683), kept to
what exercises the codec path:

* PUT: split the object into `block_size` blocks, encode every block
  (Erasure::encode_data), write each shard as interleaved `[HH256S][block]`
  records (BitrotWriter::write, bitrot.rs:464-510) to `<dir_i>/<object>/part.1`.
  Full blocks go through one batched call (rsg_encode_batch_host) that returns
  parity and all bitrot digests in the same pass (the encode_batched dispatch
  point, encode.rs:795-919); the short tail block through encode_data.
* GET: read every available shard file, verify each record before use
  (split_and_verify, bitrot.rs:227-247; a mismatching record marks that shard
  missing for the block), reconstruct missing data shards
  (decode_data_with_reconstruction_verification, erasure.rs:935-973), and
  return the first `size` bytes.

Shard placement is identity (shard i on disk i); the reference's key-hash
distribution, xl.meta, quorum and locking are out of scope.
"""
from __future__ import annotations

import json
import os
from typing import List, Optional

import numpy as np

from . import _lib
from .bitrot import HashAlgorithm, bitrot_shard_file_size
from .erasure import Erasure, calc_shard_size


class LocalErasureSet:
    def __init__(self, dirs: List[str], data_shards: int, parity_shards: int, block_size: int = 1 << 20,
                 algo: HashAlgorithm = HashAlgorithm.HighwayHash256S, device: Optional[int] = None):
        if len(dirs) != data_shards + parity_shards:
            raise ValueError("one directory per shard")
        self.dirs = dirs
        self.erasure = Erasure(data_shards, parity_shards, block_size, device=device)
        self.algo = algo

    @property
    def k(self) -> int:
        return self.erasure.data_shards

    @property
    def m(self) -> int:
        return self.erasure.parity_shards

    def _path(self, i: int, name: str) -> str:
        return os.path.join(self.dirs[i], name, "part.1")

    # ------------------------------------------------------------------ PUT
    def put_object(self, name: str, data) -> dict:
        data = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        e, k, t = self.erasure, self.k, self.k + self.m
        bs = e.block_size
        S = e.shard_size()
        nfull = data.size // bs
        tail = data.size - nfull * bs
        records: List[List[bytes]] = [[] for _ in range(t)]
        if nfull:
            st = np.zeros((nfull, t, S), dtype=np.uint8)
            flat = st.reshape(nfull, t * S)
            flat[:, :bs] = data[: nfull * bs].reshape(nfull, bs)  # zero-pad to k*S (erasure.rs:863)
            dig = np.zeros((nfull, t, 32), dtype=np.uint8)
            e.encode_batch_host(st, dig, algo=self.algo.value)
            for b in range(nfull):
                for i in range(t):
                    records[i].append(dig[b, i].tobytes() + st[b, i].tobytes())
        if tail:
            shards = e.encode_data(data[nfull * bs:])
            for i in range(t):
                records[i].append(self.algo.hash_encode(shards[i]) + shards[i])
        for i in range(t):
            os.makedirs(os.path.dirname(self._path(i, name)), exist_ok=True)
            with open(self._path(i, name), "wb") as f:
                for r in records[i]:
                    f.write(r)
        meta = {"size": int(data.size), "data_blocks": k, "parity_blocks": self.m, "block_size": bs,
                "shard_size": S, "algorithm": self.algo.name}
        for i in range(t):
            with open(os.path.join(self.dirs[i], name, "meta.json"), "w") as f:
                json.dump(meta, f)
        return meta

    # ------------------------------------------------------------------ GET
    def get_object(self, name: str) -> bytes:
        meta = None
        for i in range(self.k + self.m):
            try:
                with open(os.path.join(self.dirs[i], name, "meta.json")) as f:
                    meta = json.load(f)
                break
            except OSError:
                continue
        if meta is None:
            raise FileNotFoundError(name)
        e, k, t = self.erasure, self.k, self.k + self.m
        size, bs = meta["size"], meta["block_size"]
        S = e.shard_size()
        hs = self.algo.size()
        want = e.shard_file_size(size)
        files = []
        for i in range(t):
            try:
                f = open(self._path(i, name), "rb")
                if os.fstat(f.fileno()).st_size != bitrot_shard_file_size(want, S, self.algo):
                    f.close()
                    f = None
            except OSError:
                f = None
            files.append(f)
        out = bytearray()
        left = size
        nfull = size // bs
        try:
            if nfull:  # full blocks: one batched verify + rebuild on the GPU
                out += self._get_full_blocks(files, nfull, S)
                left -= nfull * bs
            while left > 0:
                blk = min(bs, left)
                s_blk = calc_shard_size(blk, k)
                shards: List[Optional[bytes]] = [None] * t
                for i, f in enumerate(files):
                    if f is None:
                        continue
                    rec = f.read(hs + s_blk)
                    if len(rec) < hs + s_blk:
                        files[i] = None
                        continue
                    h, body = rec[:hs], rec[hs:]
                    if self.algo.hash_encode(body) != h:  # bitrot: drop this shard for the block
                        continue
                    shards[i] = body
                if sum(s is not None for s in shards) < k:
                    raise _lib.RsgError(_lib.RSG_ERR_TOO_FEW_SHARDS, f"read quorum lost for {name}")
                e.decode_data_with_reconstruction_verification(shards)
                block = b"".join(bytes(shards[i]) for i in range(k))
                out += block[:blk]
                left -= blk
        finally:
            for f in files:
                if f is not None:
                    f.close()
        return bytes(out)

    def _get_full_blocks(self, files, nfull: int, S: int) -> bytes:
        """Read the nfull full-block records of every available shard file,
        move them to the GPU and run the GET engine (rsg_decode_records_dev):
        verify every record, rebuild missing data shards, check surplus parity."""
        import torch
        k, bs = self.k, self.erasure.block_size
        rec = 32 + S
        dev_files = []
        for f in files:
            if f is None:
                dev_files.append(None)
                continue
            raw = f.read(nfull * rec)
            if len(raw) < nfull * rec:
                dev_files.append(None)
                continue
            # pageable H2D: pinning per object (hipHostMalloc) costs more than it saves at MiB sizes
            dev_files.append(torch.frombuffer(bytearray(raw), dtype=torch.uint8).to("cuda"))
        if sum(d is not None for d in dev_files) < k:
            raise _lib.RsgError(_lib.RSG_ERR_TOO_FEW_SHARDS, "read quorum lost")
        data, status = self.erasure.decode_records_batch(dev_files, S, nfull)
        bad = [s for s in status if s != _lib.RSG_OK]
        if bad:
            _lib.check(bad[0], "erasure decode")
        return data[:, :bs].contiguous().cpu().numpy().tobytes()
