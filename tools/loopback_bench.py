"""BASELINE config 1 timing: single-node 4-drive loopback RS(2,2), PUT+GET of
1 MiB objects through rustfs_amd.loopback (GPU codec + GPU HH256S), beside the
same plumbing on the CPU oracle (restated reference algorithm).  Files go to a
tmpfs-backed temp dir when available so the disk does not dominate."""
import json
import os
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402


def cpu_put_get(dirs, data, k=2, m=2, block=1 << 20):
    from oracle import oracle as O
    S = -(-len(data) // k)
    st = np.zeros((k + m, S), dtype=np.uint8)
    st.reshape(-1)[: len(data)] = np.frombuffer(data, dtype=np.uint8)
    O.encode(k, m, st)
    for i in range(k + m):
        os.makedirs(os.path.join(dirs[i], "o"), exist_ok=True)
        with open(os.path.join(dirs[i], "o", "part.1"), "wb") as f:
            f.write(O.hh256s(st[i]) + st[i].tobytes())
    out = b""
    for i in range(k):
        raw = open(os.path.join(dirs[i], "o", "part.1"), "rb").read()
        assert O.hh256s(raw[32:]) == raw[:32]
        out += raw[32:]
    return out[: len(data)]


def main():
    import torch  # noqa: F401
    from rustfs_amd.loopback import LocalErasureSet
    n = int(os.environ.get("LOOPBACK_OBJECTS", "64"))
    base = "/dev/shm" if os.path.isdir("/dev/shm") else None
    root = tempfile.mkdtemp(dir=base)
    try:
        dirs = [os.path.join(root, f"disk{i}") for i in range(4)]
        es = LocalErasureSet(dirs, 2, 2)
        objs = [np.random.default_rng(i).integers(0, 256, 1 << 20, dtype=np.uint8).tobytes() for i in range(n)]
        es.put_object("warm", objs[0])
        es.get_object("warm")
        t0 = time.perf_counter()
        for i, d in enumerate(objs):
            es.put_object(f"o{i}", d)
        t_put = time.perf_counter() - t0
        t0 = time.perf_counter()
        for i, d in enumerate(objs):
            assert es.get_object(f"o{i}") == d
        t_get = time.perf_counter() - t0
        shutil.rmtree(os.path.join(dirs[0]))  # degraded GET (one drive lost)
        t0 = time.perf_counter()
        for i, d in enumerate(objs):
            assert es.get_object(f"o{i}") == d
        t_get_deg = time.perf_counter() - t0
        cdirs = [os.path.join(root, f"cpu{i}") for i in range(4)]
        t0 = time.perf_counter()
        for d in objs:
            assert cpu_put_get(cdirs, d) == d
        t_cpu = time.perf_counter() - t0
        mib = n
        print(json.dumps({
            "config": "RS(2,2) 4 local dirs (tmpfs), 1 MiB objects, files [HH256S][512 KiB]",
            "objects": n,
            "gpu_put_MiB_s": round(mib / t_put, 1), "gpu_put_ms_per_object": round(t_put / n * 1e3, 3),
            "gpu_get_MiB_s": round(mib / t_get, 1), "gpu_get_ms_per_object": round(t_get / n * 1e3, 3),
            "gpu_get_degraded_MiB_s": round(mib / t_get_deg, 1),
            "cpu_oracle_put_get_MiB_s": round(mib / t_cpu, 1),
            "note": "host-buffer path per object (PCIe + launch latency bound at 1 MiB); scalar CPU oracle"}))
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
