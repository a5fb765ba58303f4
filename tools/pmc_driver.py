"""One configuration of bench.py's line, called a few times, for a rocprofv3
--pmc FETCH_SIZE / WRITE_SIZE pass (tools/pmc_table.sh): the same geometry,
batch and call as the line's entry whose `traffic` it measures, so the
committed counters (profiles/r05/pmc/<key>/) are the shipped library's on that
exact launch.  Writes <outdir>/meta.json: the key, the kernel-name substring
that identifies the measured dispatches, and the calls made.

Usage: python tools/pmc_driver.py KEY OUTDIR [calls]
Keys (bench.py's pmc_lookup keys): rs84_S131072_n4096, rs84_S131072_n4096_hash,
rs164_S65536_n4096, rs124_S87382_n4096, rs124_S87382_n4096_hash,
reconstruct_e{1,2,3,4}_rs84_S131072_n4096, {get_into0,get_into2,heal_1d1p,
verify_all}_rs{84_S131072,124_S87382}_n4096."""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse(key):
    m = re.fullmatch(r"rs(\d+)4_S(\d+)_n(\d+)(_hash)?", key)
    if m:
        return "encode", int(m.group(1)), 4, int(m.group(2)), int(m.group(3)), bool(m.group(4)), None
    m = re.fullmatch(r"reconstruct_e(\d)_rs(\d+)4_S(\d+)_n(\d+)", key)
    if m:
        return "reconstruct", int(m.group(2)), 4, int(m.group(3)), int(m.group(4)), False, int(m.group(1))
    m = re.fullmatch(r"(get_into0|get_into2|heal_1d1p|verify_all)_rs(\d+)4_S(\d+)_n(\d+)", key)
    if m:
        return m.group(1), int(m.group(2)), 4, int(m.group(3)), int(m.group(4)), False, None
    raise SystemExit(f"unknown key {key}")


def main():
    key, outdir = sys.argv[1], sys.argv[2]
    calls = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    import torch
    import bench
    from rustfs_amd import Erasure, RSG_RECONSTRUCT_MISSING
    from rustfs_amd.bitrot import HashAlgorithm, bitrot_verify_batch
    what, k, m, S, n, digests, e_lost = parse(key)
    t, rec = k + m, 32 + S
    dev = torch.device("cuda", 0)
    e = Erasure(k, m, 1 << 20)
    assert e.shard_size() == S, (key, e.shard_size())
    st = bench.random_stripes(dev, k, m, S, n, 11)
    if what == "encode":
        dig = torch.empty((n, t, 32), dtype=torch.uint8, device=dev) if digests else None
        fn = lambda: e.encode_batch(st, dig)  # noqa: E731
        filt = {(8, True): "k_encode_hash", (12, True): "k_decode_records_net12<", (8, False): "k_gf_apply_vec<8, 4",
                (16, False): "k_gf_apply_loop<", (12, False): "k_gf_apply_loop<"}[(k, digests)]
    elif what == "reconstruct":
        e.encode_batch(st)
        miss = (0, 3, 5, 7)[:e_lost]
        present = [i not in miss for i in range(t)]
        fn = lambda: e.reconstruct_batch(st, present, RSG_RECONSTRUCT_MISSING)  # noqa: E731
        filt = f"k_gf_apply_vec<8, {e_lost},"
    else:
        dig = torch.empty((n, t, 32), dtype=torch.uint8, device=dev)
        e.encode_batch(st, dig)
        files = []
        for i in range(t):
            f = torch.empty((n, rec), dtype=torch.uint8, device=dev)
            f[:, :32] = dig[:, i]
            f[:, 32:] = st[:, i]
            files.append(f.reshape(-1))
        del dig, st
        torch.cuda.synchronize()
        slots = torch.empty((n, k * S), dtype=torch.uint8, device=dev)
        if what == "get_into0":
            fn = lambda: e.decode_records_into_batch(files, S, n, targets=slots)  # noqa: E731
            # records off 16-byte alignment: the LDS-DMA ring verify (rs_verify.hip)
            filt = "k_hh256_quad" if rec % 16 == 0 else "k_verify_records_dma"
        elif what == "get_into2":
            lost = [None if i in (0, 3) else files[i] for i in range(t)]
            fn = lambda: e.decode_records_into_batch(lost, S, n, targets=slots)  # noqa: E731
            filt = "k_decode_records_net"
        elif what == "heal_1d1p":
            tg = [torch.empty(n * rec, dtype=torch.uint8, device=dev) if i in (1, k) else None for i in range(t)]
            src = [None if i in (1, k) else files[i] for i in range(t)]
            fn = lambda: e.heal_records_batch(src, tg, S, n)  # noqa: E731
            filt = "k_decode_records_net"
        else:  # verify_all: every shard file of the part, one rsg_bitrot_verify_dev
            fn = lambda: bitrot_verify_batch(files, n * rec, n * S, HashAlgorithm.HighwayHash256S, S)  # noqa: E731
            filt = "k_hh256_quad"
    torch.cuda.synchronize()
    for _ in range(calls):
        fn()
    torch.cuda.synchronize()
    os.makedirs(outdir, exist_ok=True)
    json.dump({"key": key, "kernel": filt, "calls": calls}, open(os.path.join(outdir, "meta.json"), "w"))
    print("done", key, filt, calls, flush=True)


if __name__ == "__main__":
    main()
