"""Host-memory (PCIe-inclusive) rates for DESIGN.md: pinned H2D/D2H copy
bandwidth and rsg_encode_batch_host (H2D data -> encode [+HH256S] -> D2H parity
[+digests], pipelined over two streams) on RS(8,4) 1 MiB stripes."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rustfs_amd import Erasure  # noqa: E402

GiB = float(1 << 30)


def copy_rate(nbytes, h2d=True, reps=5):
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    for _ in range(2):
        (d.copy_(h, non_blocking=True) if h2d else h.copy_(d, non_blocking=True))
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        (d.copy_(h, non_blocking=True) if h2d else h.copy_(d, non_blocking=True))
    torch.cuda.synchronize()
    return reps * nbytes / (time.perf_counter() - t) / 1e9


def main():
    k, m, S, n = 8, 4, 131072, int(os.environ.get("PCIE_STRIPES", "1024"))
    out = {"h2d_GB_s": round(copy_rate(1 << 30, True), 2), "d2h_GB_s": round(copy_rate(1 << 30, False), 2)}
    e = Erasure(k, m, k * S)
    st = torch.zeros((n, k + m, S), dtype=torch.uint8).pin_memory().numpy()
    st[:, :k] = np.random.default_rng(0).integers(0, 256, (n, k, S), dtype=np.uint8)
    dig = torch.zeros((n, k + m, 32), dtype=torch.uint8).pin_memory().numpy()
    for hashed in (False, True):
        e.encode_batch_host(st, dig if hashed else None)
        reps = 5
        t = time.perf_counter()
        for _ in range(reps):
            e.encode_batch_host(st, dig if hashed else None)
        el = (time.perf_counter() - t) / reps
        out["encode_host%s" % ("_hh256s" if hashed else "")] = {
            "GiB_s_payload": round(n * k * S / el / GiB, 2), "ms_per_batch": round(el * 1e3, 2),
            "pcie_bytes_GB_s": round(n * (k + m) * S / el / 1e9 if True else 0, 2)}
    out["config"] = f"RS({k},{m}) S={S} n={n} pinned host buffers"
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
