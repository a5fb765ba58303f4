"""Cross-check of the record engines' kernel-timing hook (rsg_set_kernel_timing
/ rsg_last_kernel_ms) against the call time and, when run under
`rocprofv3 --kernel-trace --stats`, against rocprof's kernel durations.
RS(8,4) 1 MiB stripes, n = 4096: in-place GET with 2 data disks lost, all
present, heal.  Usage: python tools/hook_check.py [reps]"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from rustfs_amd import Erasure, _lib
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    k, m, n, S = 8, 4, 4096, 131072
    t, rec = k + m, 32 + S
    e = Erasure(k, m, 1 << 20)
    st = torch.zeros((n, t, S), dtype=torch.uint8, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(5)
    for s0 in range(0, n, 256):
        st[s0:s0 + 256, :k] = torch.randint(0, 256, (256, k, S), dtype=torch.uint8, device="cuda", generator=g)
    dig = torch.empty((n, t, 32), dtype=torch.uint8, device="cuda")
    e.encode_batch(st, dig)
    files = [torch.empty(n * rec, dtype=torch.uint8, device="cuda") for _ in range(t)]
    for i in range(t):
        f = files[i].view(n, rec)
        f[:, :32] = dig[:, i]
        f[:, 32:] = st[:, i]
    del st, dig
    slots = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
    lost = [None if i in (0, 3) else files[i] for i in range(t)]
    tg = [torch.empty(n * rec, dtype=torch.uint8, device="cuda") if i in (1, k) else None for i in range(t)]
    src = [None if i in (1, k) else files[i] for i in range(t)]
    L, ctx = _lib.load(), _lib.context(0).handle
    stream = torch.cuda.current_stream()
    calls = {"into2": lambda: e.decode_records_into_batch(lost, S, n, targets=slots, stream=stream),
             "into0": lambda: e.decode_records_into_batch(files, S, n, targets=slots, stream=stream),
             "heal": lambda: e.heal_records_batch(src, tg, S, n, stream=stream)}
    out = {}
    for name, fn in calls.items():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(stream)
        for _ in range(reps):
            fn()
        ev[1].record(stream)
        torch.cuda.synchronize()
        call = ev[0].elapsed_time(ev[1]) / reps
        _lib.check(L.rsg_set_kernel_timing(ctx, 1))
        hook = []
        for _ in range(reps):
            fn()
            v = ctypes.c_float(-1)
            _lib.check(L.rsg_last_kernel_ms(ctx, ctypes.byref(v)))
            hook.append(round(v.value, 4))
        _lib.check(L.rsg_set_kernel_timing(ctx, 0))
        out[name] = {"call_ms": round(call, 4), "hook_ms": hook}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
