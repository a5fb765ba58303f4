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
  return the first `size` bytes.  Full blocks go through the GPU GET engine
  (rsg_decode_records_dev).
* HEAL: rebuild the shard files of replaced disks (Erasure::heal,
  heal.rs:112-206) — full blocks in one rsg_heal_records_dev call, the tail
  block through decode_data_and_parity — byte-identical to what PUT wrote.
* VERIFY: deep-scan every shard file (bitrot_verify, bitrot.rs:616-655) with
  one rsg_bitrot_verify_dev call.

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
    def _meta(self, name: str) -> dict:
        for i in range(self.k + self.m):
            try:
                with open(os.path.join(self.dirs[i], name, "meta.json")) as f:
                    return json.load(f)
            except OSError:
                continue
        raise FileNotFoundError(name)

    def get_object(self, name: str) -> bytes:
        meta = self._meta(name)
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

    # ----------------------------------------------------------------- HEAL
    def heal_object(self, name: str, targets: List[int]) -> None:
        """Rewrite the part files of the disks in `targets` from the others."""
        import torch
        meta = self._meta(name)
        e, k, t = self.erasure, self.k, self.k + self.m
        size, bs = meta["size"], meta["block_size"]
        S = e.shard_size()
        want = bitrot_shard_file_size(e.shard_file_size(size), S, self.algo)
        raws: List[Optional[bytes]] = []
        for i in range(t):
            raw = None
            if i not in targets:
                try:
                    with open(self._path(i, name), "rb") as f:
                        raw = f.read()
                except OSError:
                    raw = None
                if raw is not None and len(raw) != want:
                    raw = None
            raws.append(raw)
        nfull = size // bs
        rec = 32 + S
        out = {i: bytearray() for i in targets}
        if nfull:
            src = [torch.frombuffer(bytearray(r[: nfull * rec]), dtype=torch.uint8).to("cuda") if r else None
                   for r in raws]
            dst = [torch.empty(nfull * rec, dtype=torch.uint8, device="cuda") if i in targets else None
                   for i in range(t)]
            status = e.heal_records_batch(src, dst, S, nfull, algo=self.algo.value)
            bad = [x for x in status if x != _lib.RSG_OK]
            if bad:
                _lib.check(bad[0], f"heal {name}")
            for i in targets:
                out[i] += dst[i].cpu().numpy().tobytes()
        tail = size - nfull * bs
        if tail:  # the short last block: host path, verify-before-use per record
            s_blk = calc_shard_size(tail, k)
            hs = self.algo.size()
            shards: List[Optional[bytes]] = [None] * t
            for i, r in enumerate(raws):
                if r is None:
                    continue
                h, body = r[nfull * rec: nfull * rec + hs], r[nfull * rec + hs: nfull * rec + hs + s_blk]
                if len(body) == s_blk and self.algo.hash_encode(body) == h:
                    shards[i] = body
            if sum(x is not None for x in shards) < k:
                raise _lib.RsgError(_lib.RSG_ERR_TOO_FEW_SHARDS, f"heal {name}: read quorum")
            source_parity = {i: shards[i] for i in range(k, t) if shards[i] is not None}
            e.decode_data_and_parity(shards)
            for i, src_p in source_parity.items():
                if bytes(shards[i]) != bytes(src_p):
                    raise _lib.InvalidDataError(_lib.RSG_ERR_INCONSISTENT_SOURCES, f"heal {name}")
            for i in targets:
                out[i] += self.algo.hash_encode(bytes(shards[i])) + bytes(shards[i])
        for i in targets:
            os.makedirs(os.path.dirname(self._path(i, name)), exist_ok=True)
            with open(self._path(i, name), "wb") as f:
                f.write(bytes(out[i]))
            with open(os.path.join(self.dirs[i], name, "meta.json"), "w") as f:
                json.dump(meta, f)

    # --------------------------------------------------------------- VERIFY
    def verify_object(self, name: str) -> List[int]:
        """Deep scan: rsg_status of every shard file (RSG_OK = healthy)."""
        import torch
        from .bitrot import bitrot_verify_batch
        meta = self._meta(name)
        e, t = self.erasure, self.k + self.m
        S = e.shard_size()
        part = e.shard_file_size(meta["size"])
        want = bitrot_shard_file_size(part, S, self.algo)
        files = []
        for i in range(t):
            try:
                with open(self._path(i, name), "rb") as f:
                    raw = f.read()
                files.append(torch.frombuffer(bytearray(raw), dtype=torch.uint8).to("cuda") if raw
                             else torch.empty(0, dtype=torch.uint8, device="cuda"))
            except OSError:
                files.append(None)
        present = [f for f in files if f is not None]
        status = bitrot_verify_batch(present, want, part, self.algo, S) if present else []
        it = iter(status)
        return [_lib.RSG_ERR_UNEXPECTED_EOF if f is None else next(it) for f in files]
