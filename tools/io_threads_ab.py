"""Host pipeline thread counts: streamed GET / PUT of a 1 GiB RS(8,4) object in
tmpfs with IO_THREADS and put read_threads varied (best of 4)."""
import json, os, shutil, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from rustfs_amd import Erasure, pipeline
from rustfs_amd.pipeline import _pinned
k, m, bs, n = 8, 4, 1 << 20, 1024
S, t, rec = bs // k, 12, 32 + bs // k
e = Erasure(k, m, bs)
st = _pinned((n, t, S))
st[:, :k] = np.random.default_rng(1).integers(0, 256, (n, k, S), dtype=np.uint8)
dg = _pinned((n, t, 32))
e.encode_batch_host(st, dg)
root = f"/dev/shm/ioab_{os.getpid()}"
os.makedirs(root)
try:
    paths = [f"{root}/p{i}" for i in range(t)]
    for i in range(t):
        r = np.empty((n, rec), np.uint8); r[:, :32] = dg[:, i]; r[:, 32:] = st[:, i]
        open(paths[i], "wb").write(r.data)
    body = f"{root}/body"
    open(body, "wb").write(np.ascontiguousarray(st[:, :k]).data)
    def best(fn, reps=4):
        fn(); b = 1e9
        for _ in range(reps):
            t0 = time.perf_counter(); fn(); b = min(b, time.perf_counter() - t0)
        return round(b * 1e3, 2)
    for io in (8, 12):
        pipeline.IO_THREADS = io
        stage = pipeline.GetStage()
        def get(data_only=False):
            fds = [os.open(p, os.O_RDONLY) for p in paths]
            try:
                for c in pipeline.get_stream(e, fds, n * bs, stage=stage, views=True, data_shards_only=data_only):
                    pass
            finally:
                for fd in fds: os.close(fd)
        g = best(get); gd = best(lambda: get(True))
        stage.close()
        for rt in (4, 8):
            ps = {}
            def put():
                wp = [f"{root}/w{i}" for i in range(t)]
                for p in wp:
                    if os.path.exists(p): os.remove(p)
                fds = [os.open(p, os.O_WRONLY | os.O_CREAT, 0o644) for p in wp]
                try:
                    with open(body, "rb", buffering=0) as f:
                        r = pipeline.put_stream(e, f, n * bs, fds, stage=ps.get("s"), read_threads=rt)
                    ps["s"] = r["stage"]
                finally:
                    for fd in fds: os.close(fd)
            print(json.dumps({"io_threads": io, "read_threads": rt, "get_ms": g, "get_data_only_ms": gd, "put_ms": best(put)}), flush=True)
finally:
    shutil.rmtree(root, ignore_errors=True)
