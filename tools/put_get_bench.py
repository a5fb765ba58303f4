"""End-to-end streamed PUT / GET rate of the loopback erasure set for a
multi-GiB object: put_object_stream (encode_batched's
pipeline on the GPU, encode.rs:795-919) and get_object_stream (decode_inner,
decode.rs:1702-1968), with the pieces timed alone for the breakdown:

  read      source file -> page-locked staging (the producer's memcpy)
  encode    rsg_encode_batch_host_submit pipeline alone (H2D + encode+HH256S + D2H)
  put       the whole PUT: read + encode + k+m shard-file writes
  get       the whole GET: shard-file reads + H2D + verify/decode + D2H
  get_lost  GET with two data disks lost (rebuild on the GPU)

Files live in tmpfs (/dev/shm) when it has room, so the figures are the
host pipeline's, not a disk's.  Measurement code.
Usage: python tools/put_get_bench.py [--gib 4] [--k 8 --m 4] [--batch 64]
"""
import argparse
import json
import os
import shutil
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--block", type=int, default=1 << 20)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--inflight", type=int, default=2)
    ap.add_argument("--read-threads", type=int, default=4)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    from rustfs_amd.erasure import Erasure
    from rustfs_amd.loopback import LocalErasureSet
    from rustfs_amd.pipeline import _pinned

    size = int(a.gib * (1 << 30)) // a.block * a.block
    t = a.k + a.m
    need = size * (1 + t / a.k) * 1.1
    root = a.dir
    if root is None:
        st = os.statvfs("/dev/shm")
        root = "/dev/shm" if st.f_bavail * st.f_frsize > need else os.environ.get("TMPDIR", "/tmp")
    root = os.path.join(root, f"rsg_pgb_{os.getpid()}")
    os.makedirs(root)
    res = {"object_bytes": size, "k": a.k, "m": a.m, "block": a.block, "batch_blocks": a.batch,
           "inflight_batches": a.inflight, "dir": os.path.dirname(root)}
    try:
        src = os.path.join(root, "src")
        pat = np.random.default_rng(1).integers(0, 256, 64 << 20, dtype=np.uint8)
        with open(src, "wb") as f:
            left = size
            i = 0
            while left:
                n = min(left, pat.size)
                pat[:8] = np.frombuffer(np.uint64(i).tobytes(), np.uint8)  # every chunk distinct
                f.write(pat[:n].tobytes())
                left -= n
                i += 1
        torch.cuda.init()
        es = LocalErasureSet([os.path.join(root, f"d{i}") for i in range(t)], a.k, a.m, block_size=a.block)
        e: Erasure = es.erasure
        S = e.shard_size()

        # read alone: source -> page-locked (B, t, S) staging
        buf = _pinned((a.batch, t, S))
        t0 = time.perf_counter()
        with open(src, "rb", buffering=0) as f:
            for b0 in range(0, size // a.block, a.batch):
                for b in range(min(a.batch, size // a.block - b0)):
                    f.readinto(memoryview(buf[b]).cast("B")[: a.block])
        res["read_GBps"] = size / (time.perf_counter() - t0) / 1e9

        # encode pipeline alone: same batches, no file I/O (data resident in two pinned buffers)
        bufs = [buf, _pinned((a.batch, t, S)), _pinned((a.batch, t, S))]
        digs = [_pinned((a.batch, t, 32)) for _ in bufs]
        nb = size // a.block
        for rep in range(2):  # the first pass allocates the device staging
            t0 = time.perf_counter()
            tickets = []
            for j, b0 in enumerate(range(0, nb, a.batch)):
                if len(tickets) >= len(bufs):
                    tickets.pop(0).wait()
                c = min(a.batch, nb - b0)
                tickets.append(e.encode_batch_host_submit(bufs[j % 3][:c], digs[j % 3][:c]))
            for tk in tickets:
                tk.wait()
        res["encode_pipeline_GBps"] = size / (time.perf_counter() - t0) / 1e9
        del bufs, buf

        # shard-file writes alone: t files of size/k bytes each, the PUT's thread pool shape
        from concurrent.futures import ThreadPoolExecutor
        wbuf = _pinned((a.batch, t, S))
        per_file = size // a.k
        t0 = time.perf_counter()
        with ThreadPoolExecutor(min(t, 8)) as pool:
            def wr(i):
                fd = os.open(os.path.join(root, f"w{i}"), os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
                left = per_file
                while left > 0:
                    left -= os.write(fd, memoryview(wbuf).cast("B")[: min(left, wbuf.nbytes)])
                os.close(fd)
            list(pool.map(wr, range(t)))
        res["write_GBps_object"] = size / (time.perf_counter() - t0) / 1e9
        for i in range(t):
            os.remove(os.path.join(root, f"w{i}"))
        del wbuf

        # the whole PUT (first one warms the stage allocation; time the second),
        # sequential readinto producer and parallel pread producer
        for tag, rt in (("put_seqread", 1), ("put", a.read_threads)):
            for rep in range(2):
                for i in range(t):  # a new object: no truncation of the old part files in the timed region
                    shutil.rmtree(os.path.join(root, f"d{i}", "b"), ignore_errors=True)
                t0 = time.perf_counter()
                with open(src, "rb", buffering=0) as f:
                    es.put_object_stream("b/o", f, size, batch_blocks=a.batch, inflight_batches=a.inflight,
                                         read_threads=rt)
                dt = time.perf_counter() - t0
            res[f"{tag}_GBps"] = size / dt / 1e9
            res[f"{tag}_clock"] = {x: round(es.last_put[x], 4) for x in ("read_s", "submit_s", "wait_s", "write_s")}

        def get_rate(tag):
            n = 0
            h = 0
            t0 = time.perf_counter()
            with open(src, "rb", buffering=0) as f:
                for chunk in es.get_object_stream("b/o", batch_blocks=a.batch):
                    if n % (256 << 20) < len(chunk):  # spot-check one block per 256 MiB
                        f.seek(n)
                        if f.read(len(chunk)) != chunk:
                            raise SystemExit(f"{tag}: GET mismatch at {n}")
                    n += len(chunk)
                    h += 1
            dt = time.perf_counter() - t0
            if n != size:
                raise SystemExit(f"{tag}: GET returned {n} of {size} bytes")
            res[f"{tag}_GBps"] = size / dt / 1e9

        get_rate("get")  # warm (stage allocation, page cache of the shard files)
        get_rate("get")
        for i in (0, 1):
            os.remove(es.part_file(i, "b/o"))
        get_rate("get_2_data_lost")
        res["pcie_h2d_d2h_ceiling_GBps"] = 57.0
        res["note"] = ("put/get: whole-object wall-clock rate in object bytes/s; the PUT moves "
                       f"{t / a.k:.2f}x the object bytes to the shard files and the GPU")
    finally:
        shutil.rmtree(root, ignore_errors=True)
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
