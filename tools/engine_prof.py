"""One engine call repeated (for rocprofv3 --kernel-trace --stats): GET with
two data disks lost, or heal, RS(8,4) 1 MiB stripes, n = 4096 records.
get* = the gather form (rsg_decode_records_dev), into* = the in-place form
(rsg_decode_records_into_dev).
Usage: python tools/engine_prof.py get2|get2_01|get1|get0|into2|into1|into0|heal [reps]
EP_LOOPS=L EP_SLEEP=s: L loops of `reps` calls, each after s seconds idle (the
bench's engine protocol of round 4, for the per-dispatch clock table)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from rustfs_amd import Erasure
    what = sys.argv[1] if len(sys.argv) > 1 else "get2"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    k = int(os.environ.get("EP_K", "8"))  # EP_K=12: RS(12,4), the 16-drive default (ragged walks)
    m, n = 4, 4096
    S, t = -(-(1 << 20) // k), k + 4
    rec = 32 + S
    e = Erasure(k, m, 1 << 20)
    early = os.environ.get("EP_FILES_FIRST") == "1"  # allocate the record files and output before the staging
    if early:
        files = [torch.empty(n * rec, dtype=torch.uint8, device="cuda") for _ in range(t)]
        out = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
    st = torch.zeros((n, t, S), dtype=torch.uint8, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(5)
    for s0 in range(0, n, 256):
        st[s0:s0 + 256, :k] = torch.randint(0, 256, (min(256, n - s0), k, S), dtype=torch.uint8, device="cuda",
                                            generator=g)
    dig = torch.empty((n, t, 32), dtype=torch.uint8, device="cuda")
    e.encode_batch(st, dig)
    if not early:
        files = [torch.empty(n * rec, dtype=torch.uint8, device="cuda") for _ in range(t)]
    for i in range(t):
        f = files[i].view(n, rec)
        f[:, :32] = dig[:, i]
        f[:, 32:] = st[:, i]
    del st, dig
    if os.environ.get("EP_BAD_PARITY") == "1":  # surplus parity 10 inconsistent in every stripe (compare mismatch)
        files[10].view(n, rec)[:, 32:] ^= 0x5A
    if not early:
        out = torch.empty((n, k * S), dtype=torch.uint8, device="cuda")
    loops = int(os.environ.get("EP_LOOPS", "1"))
    idle = float(os.environ.get("EP_SLEEP", "0"))
    for _ in range(loops * reps):
        if idle and _ % reps == 0:
            torch.cuda.synchronize()
            time.sleep(idle)
        if what == "heal":
            tg = [torch.empty(n * rec, dtype=torch.uint8, device="cuda") if i in (1, k) else None for i in range(t)]
            e.heal_records_batch([None if i in (1, k) else files[i] for i in range(t)], tg, S, n)
        elif what.startswith("into"):
            lost = {"into2": (0, 3), "into1": (0,)}.get(what, ())
            e.decode_records_into_batch([None if i in lost else files[i] for i in range(t)], S, n, targets=out)
        else:
            lost = {"get2": (0, 3), "get2_01": (0, 1), "get1": (0,)}.get(what, ())
            e.decode_records_batch([None if i in lost else files[i] for i in range(t)], S, n, out=out)
    torch.cuda.synchronize()
    print("done", what, reps)


if __name__ == "__main__":
    main()
