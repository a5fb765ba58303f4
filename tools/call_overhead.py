"""Fixed host cost of one synchronous engine call (rsg_decode_records_dev via
Erasure.decode_records_batch) at a tiny batch, and the same call made
directly through ctypes with prebuilt arguments.  Measurement code."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from rustfs_amd import Erasure, _lib
    k, m, S = 8, 4, 131072
    t, rec = k + m, 32 + S
    for n in (8, 4096):
        e = Erasure(k, m, k * S)
        st = torch.zeros((n, t, S), dtype=torch.uint8, device="cuda")
        st[:, :k] = torch.randint(0, 256, (n, k, S), dtype=torch.uint8, device="cuda")
        dig = torch.zeros((n, t, 32), dtype=torch.uint8, device="cuda")
        e.encode_batch(st, dig)
        files = [torch.cat([dig[:, i], st[:, i]], dim=1).contiguous().reshape(-1) for i in range(t)]
        del st, dig
        out = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
        lost = [None if i in (0, 3) else files[i] for i in range(t)]
        for _ in range(3):
            e.decode_records_batch(lost, S, n, out=out)
        torch.cuda.synchronize()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            e.decode_records_batch(lost, S, n, out=out)
        py = (time.perf_counter() - t0) / reps
        ptrs = (ctypes.c_void_p * t)(*[f.data_ptr() if f is not None else None for f in lost])
        status = (ctypes.c_int * n)()
        h = _lib.context(0).handle
        lib = _lib.load()
        s = torch.cuda.current_stream().cuda_stream
        t0 = time.perf_counter()
        for _ in range(reps):
            lib.rsg_decode_records_dev(h, k, m, S, n, ptrs, _lib.RSG_HASH_HIGHWAY256S, 1, out.data_ptr(), status, s)
        raw = (time.perf_counter() - t0) / reps
        print(f"n={n}: decode_records_batch {py * 1e3:.3f} ms/call, raw ctypes call {raw * 1e3:.3f} ms/call", flush=True)
        del files, lost, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
