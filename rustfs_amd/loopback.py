"""Single-node loopback erasure set: BASELINE config 1 plumbing.

A minimal mirror of the reference's set-level PUT/GET for one erasure set of
local directories (`SetDisks::put_object`, crates/ecstore/src/set_disk/ops/object.rs:1852;
`get_object_with_fileinfo`, crates/ecstore/src/set_disk/read.rs:683), kept to
what exercises the codec path:

* PUT: split the object into `block_size` blocks, encode every block
  (Erasure::encode_data), write each shard as interleaved `[HH256S][block]`
  records (BitrotWriter::write, bitrot.rs:464-510) to
  `<dir_i>/<object>/<version>/part.1`.
  Full blocks go through one batched call (rsg_encode_batch_host) that returns
  parity and all bitrot digests in the same pass (the encode_batched dispatch
  point, encode.rs:795-919); the short tail block through encode_data.
* GET: read every available shard file, verify each record before use
  (split_and_verify, bitrot.rs:227-247; a mismatching record marks that shard
  missing for the block), reconstruct missing data shards
  (decode_data_with_reconstruction_verification, erasure.rs:935-973), and
  return the first `size` bytes.  Full blocks go through the GPU GET engine
  (rsg_decode_records_into_dev, in place: only the rebuilt shards are written).
* HEAL: rebuild the shard files of replaced disks (Erasure::heal,
  heal.rs:112-206) — full blocks in one rsg_heal_records_dev call, the tail
  block through decode_data_and_parity — byte-identical to what PUT wrote.
* VERIFY: deep-scan every shard file (bitrot_verify, bitrot.rs:616-655) with
  one rsg_bitrot_verify_dev call.

Commit: a PUT writes every shard file into a directory of its own version id
(the reference's per-version data_dir, which xl.meta points to), and only once
the write quorum holds replaces each disk's meta.json (naming that version and
its modification time) — one atomic rename switches a disk's part and
metadata together — then removes the version directory that meta.json named
before (a concurrent PUT's uncommitted directory is left to that PUT).  A
crash or an interleaved PUT can leave a disk on either version, never with one
version's part under another's metadata.  A disk whose writer was dropped
loses its previous version (heal rebuilds it), and a PUT that fails leaves the
previous version untouched (rename_data).  GET and heal pick the metadata
version held by at least k disks (read quorum; the most disks, then the newest
modification time) and read only the shard files of disks holding it (the
reference's quorum choice of FileInfo); no version with k disks is a read-quorum
error.

Shard placement is identity (shard i on disk i); the reference's key-hash
distribution, xl.meta, quorum and locking are out of scope.
"""
from __future__ import annotations

import json
import os
import shutil
import threading
import time
import uuid
from typing import Iterator, List, Optional

import numpy as np

from . import _lib
from .bitrot import HashAlgorithm, bitrot_shard_file_size
from .erasure import Erasure, calc_shard_size
from .pipeline import DEFAULT_BATCH_BLOCKS, DEFAULT_INFLIGHT_BATCHES, GetStage, PutStage, get_stream, put_stream


class LocalErasureSet:
    def __init__(self, dirs: List[str], data_shards: int, parity_shards: int, block_size: int = 1 << 20,
                 algo: HashAlgorithm = HashAlgorithm.HighwayHash256S, device: Optional[int] = None):
        if len(dirs) != data_shards + parity_shards:
            raise ValueError("one directory per shard")
        self.dirs = dirs
        self.erasure = Erasure(data_shards, parity_shards, block_size, device=device)
        self.algo = algo
        self._put_stage = None  # page-locked PUT staging, reused across objects
        self._stage_lock = threading.Lock()  # put_object's use of _put_stage
        self._get_stage = GetStage()  # page-locked GET staging + device buffers, reused across objects
        self.last_put: dict = {}  # put_stream's counts and producer/consumer clocks

    def close(self) -> None:
        """Release the reusable GET stage's read pool (a later streamed GET
        starts a new one)."""
        self._get_stage.close()

    @property
    def k(self) -> int:
        return self.erasure.data_shards

    @property
    def m(self) -> int:
        return self.erasure.parity_shards

    def _path(self, i: int, name: str, version: str) -> str:
        """Disk i's part file of `version` (the version's own data dir)."""
        return os.path.join(self.dirs[i], name, version, "part.1")

    def part_file(self, i: int, name: str) -> Optional[str]:
        """Disk i's part file of the version its meta.json names (None: the
        disk holds no committed version of `name`)."""
        try:
            with open(os.path.join(self.dirs[i], name, "meta.json")) as f:
                return self._path(i, name, json.load(f)["version"])
        except (OSError, ValueError, KeyError):
            return None

    # ------------------------------------------------------------------ PUT
    def put_object(self, name: str, data) -> dict:
        data = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        e, k, t = self.erasure, self.k, self.k + self.m
        bs = e.block_size
        S = e.shard_size()
        nfull = data.size // bs
        tail = data.size - nfull * bs
        records: List[list] = [[] for _ in range(t)]  # buffers written with one writev per shard file
        staged = bool(nfull) and self._stage_lock.acquire(blocking=False)
        try:
            if nfull:
                if staged:
                    # page-locked (n, k+m, S) stripes + digests reused across
                    # objects (PutStage: the pad between a block's end and k*S
                    # is never written, so it stays zero, erasure.rs:858-866)
                    if self._put_stage is None or not self._put_stage.fits(1, nfull, t, S):
                        self._put_stage = PutStage(1, nfull, t, S)
                    st = self._put_stage.stripes[0][:nfull]
                    dig = self._put_stage.digests[0][:nfull]
                else:  # another thread's PUT holds the stage
                    st = np.zeros((nfull, t, S), dtype=np.uint8)
                    dig = np.zeros((nfull, t, 32), dtype=np.uint8)
                st.reshape(nfull, t * S)[:, :bs] = data[: nfull * bs].reshape(nfull, bs)
                e.encode_batch_host(st, dig, algo=self.algo.value)
                for b in range(nfull):
                    for i in range(t):
                        records[i] += [dig[b, i], st[b, i]]
            version = uuid.uuid4().hex
            try:
                self._write_records(name, records, data[nfull * bs:] if tail else None, version)
            except BaseException:
                self._discard(name, version)
                raise
        finally:
            if staged:
                self._stage_lock.release()
        return self._commit(name, int(data.size), version)

    def _write_records(self, name: str, records: List[list], tail, version: str) -> None:
        e, t = self.erasure, self.k + self.m
        if tail is not None:
            shards = e.encode_data(tail)
            for i in range(t):
                records[i] += [self.algo.hash_encode(shards[i]), shards[i]]
        for i in range(t):
            os.makedirs(os.path.dirname(self._path(i, name, version)), exist_ok=True)
            fd = os.open(self._path(i, name, version), os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
            try:
                for c0 in range(0, len(records[i]), 512):  # IOV_MAX is 1024 on Linux
                    chunk = records[i][c0:c0 + 512]
                    done = os.writev(fd, chunk)
                    if done != sum(memoryview(r).nbytes for r in chunk):  # short write: finish plainly
                        rest = b"".join(bytes(r) for r in chunk)[done:]
                        while rest:
                            rest = rest[os.write(fd, rest):]
            finally:
                os.close(fd)

    def put_object_stream(self, name: str, reader, size: int, batch_blocks: int = DEFAULT_BATCH_BLOCKS,
                          inflight_batches: int = DEFAULT_INFLIGHT_BATCHES, read_threads: int = 4,
                          write_quorum: Optional[int] = None) -> dict:
        """PUT of a `size`-byte body read from `reader` (``readinto``) without
        holding it in memory: encode_batched's pipeline (encode.rs:795-919) —
        B-block batches through page-locked staging, GPU encode + HH256S of
        batch i overlapping the read of batch i+1 and the shard-file writes of
        batch i-1.  Produces the same files as put_object.  A shard file
        whose write fails is dropped and the PUT completes while the write
        quorum holds (MultiWriter::write_shards, encode.rs:374-430); the
        dropped shards are not committed and heal rebuilds them."""
        e, t = self.erasure, self.k + self.m
        fds: List[Optional[int]] = []
        version = uuid.uuid4().hex
        staged = self._stage_lock.acquire(blocking=False)  # else another PUT holds the stage
        try:
            for i in range(t):
                try:  # a disk that cannot take the part has no writer (DiskNotFound)
                    os.makedirs(os.path.dirname(self._path(i, name, version)), exist_ok=True)
                    fds.append(os.open(self._path(i, name, version), os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644))
                except OSError:
                    fds.append(None)
            info = put_stream(e, reader, size, fds, self.algo, batch_blocks, inflight_batches,
                              self._put_stage if staged else None, read_threads, write_quorum)
            stage = info.pop("stage")
            if staged:
                self._put_stage = stage
            self.last_put = info
        except BaseException:
            self._discard(name, version)  # below quorum (or any failure): the previous version stays
            raise
        finally:
            if staged:
                self._stage_lock.release()
            for fd in fds:
                if fd is not None:
                    try:
                        os.close(fd)
                    except OSError:
                        pass
        # the dropped writers' disks are left out of the commit, as the
        # reference drops them before renaming the object into place
        return self._commit(name, size, version, skip=set(info["failed_shards"]))

    def _discard(self, name: str, version: str) -> None:
        for i in range(self.k + self.m):
            shutil.rmtree(os.path.join(self.dirs[i], name, version), ignore_errors=True)

    def _disk_version(self, i: int, name: str) -> Optional[str]:
        """The version disk i's meta.json names (None: none committed)."""
        try:
            with open(os.path.join(self.dirs[i], name, "meta.json")) as f:
                return json.load(f).get("version")
        except (OSError, ValueError):
            return None

    def _drop_version(self, i: int, name: str, version: Optional[str]) -> None:
        """Remove one version's directory on disk i — the one its meta.json
        named before a switch (nothing reads it any more).  Only that one: a
        concurrent PUT's uncommitted directory stays (that PUT commits or
        discards it)."""
        if version:
            shutil.rmtree(os.path.join(self.dirs[i], name, version), ignore_errors=True)

    def _commit(self, name: str, size: int, version: str, skip=()) -> dict:
        """Switch each disk to the new version: its meta.json is replaced in
        one rename (the part file already sits in the version's directory),
        then the disk's other versions are removed.  A skipped (dropped) disk
        keeps nothing of the previous version, so no GET or heal reads a stale
        part or size from it."""
        e = self.erasure
        meta = {"size": int(size), "data_blocks": self.k, "parity_blocks": self.m, "block_size": e.block_size,
                "shard_size": e.shard_size(), "algorithm": self.algo.name, "version": version,
                "mod_time": time.time_ns()}
        for i in range(self.k + self.m):
            old = self._disk_version(i, name)
            if i in skip:
                try:
                    os.unlink(os.path.join(self.dirs[i], name, "meta.json"))
                except OSError:
                    pass
                self._drop_version(i, name, old)
                self._drop_version(i, name, version)  # the dropped writer's partial part
                continue
            self._write_meta_file(i, name, meta)
            if old != version:
                self._drop_version(i, name, old)
        return meta

    def _write_meta_file(self, i: int, name: str, meta: dict) -> None:
        path = os.path.join(self.dirs[i], name, "meta.json")
        with open(path + ".tmp", "w") as f:
            json.dump(meta, f)
        os.replace(path + ".tmp", path)

    # ------------------------------------------------------------------ GET
    def _meta(self, name: str) -> dict:
        """The metadata version the set serves, with "disks": the disks that
        hold it.  Only a version on at least k disks can be read (read quorum,
        the reference's quorum choice of FileInfo); among those, the one held
        by the most disks, then the newest modification time.  No version
        with k disks: a read-quorum error."""
        votes: dict = {}
        for i in range(self.k + self.m):
            try:
                with open(os.path.join(self.dirs[i], name, "meta.json")) as f:
                    meta = json.load(f)
            except (OSError, ValueError):
                continue
            key = json.dumps(meta, sort_keys=True)
            votes.setdefault(key, (meta, []))[1].append(i)
        if not votes:
            raise FileNotFoundError(name)
        quorum = [v for v in votes.values() if len(v[1]) >= self.k]
        if not quorum:
            raise _lib.RsgError(_lib.RSG_ERR_TOO_FEW_SHARDS, f"{name}: no metadata version reaches read quorum")
        meta, disks = max(quorum, key=lambda v: (len(v[1]), v[0].get("mod_time", 0), -v[1][0]))
        return dict(meta, disks=disks)

    def _open_shards(self, name: str, size: int, version: str, disks=None) -> List[Optional[int]]:
        """Shard file descriptors; a missing or wrong-length file, or a disk
        not holding the chosen metadata version, is None (the reader for that
        disk is unavailable)."""
        e = self.erasure
        want = bitrot_shard_file_size(e.shard_file_size(size), e.shard_size(), self.algo)
        fds: List[Optional[int]] = []
        for i in range(self.k + self.m):
            if disks is not None and i not in disks:
                fds.append(None)
                continue
            try:
                fd = os.open(self._path(i, name, version), os.O_RDONLY)
            except OSError:
                fds.append(None)
                continue
            if os.fstat(fd).st_size != want:
                os.close(fd)
                fd = None
            fds.append(fd)
        return fds

    def get_object_stream(self, name: str, offset: int = 0, length: Optional[int] = None,
                          batch_blocks: int = DEFAULT_BATCH_BLOCKS, data_shards_only: bool = False) -> Iterator[bytes]:
        """Stream bytes [offset, offset + length) (default: to the end) of
        `name`: decode_inner's range read (decode.rs:1702-1968) with full
        blocks verified and rebuilt on the GPU B blocks at a time, the next
        batch read from the shard files while this one decodes.  The set's
        reusable GET stage stays locked while the stream is open: close() an
        abandoned stream (or consume it) so other GETs can reuse the stage;
        get_object_range does.  data_shards_only: the reference's optional
        data-shards-only read (RUSTFS_GET_LOCKSTEP_DATA_SHARDS_ONLY_ENABLE,
        pipeline.get_stream)."""
        meta = self._meta(name)
        size = meta["size"]
        fds = self._open_shards(name, size, meta["version"], meta["disks"])
        try:
            yield from get_stream(self.erasure, fds, size, offset, length, self.algo, batch_blocks, self._get_stage,
                                  data_shards_only=data_shards_only)
        finally:
            for fd in fds:
                if fd is not None:
                    os.close(fd)

    def get_object_range(self, name: str, offset: int = 0, length: Optional[int] = None) -> bytes:
        return b"".join(self.get_object_stream(name, offset, length))

    def get_object(self, name: str) -> bytes:
        return self.get_object_range(name)

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
            if i not in targets and i in meta["disks"]:
                try:
                    with open(self._path(i, name, meta["version"]), "rb") as f:
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
        meta = {key: v for key, v in meta.items() if key != "disks"}
        for i in targets:  # the healed part in the version's directory, then the disk's meta switches to it
            path = self._path(i, name, meta["version"])
            os.makedirs(os.path.dirname(path), exist_ok=True)
            tmp = path + ".heal-tmp"
            with open(tmp, "wb") as f:
                f.write(bytes(out[i]))
            os.replace(tmp, path)
            old = self._disk_version(i, name)
            self._write_meta_file(i, name, meta)
            if old != meta["version"]:
                self._drop_version(i, name, old)

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
                with open(self._path(i, name, meta["version"]), "rb") as f:
                    raw = f.read()
                files.append(torch.frombuffer(bytearray(raw), dtype=torch.uint8).to("cuda") if raw
                             else torch.empty(0, dtype=torch.uint8, device="cuda"))
            except OSError:
                files.append(None)
        present = [f for f in files if f is not None]
        status = bitrot_verify_batch(present, want, part, self.algo, S) if present else []
        it = iter(status)
        return [_lib.RSG_ERR_UNEXPECTED_EOF if f is None else next(it) for f in files]
