"""Host-batch PUT pipeline alone (rsg_encode_batch_host[_submit]) on page-
locked buffers: where does the time go?  Measurement code.
Usage: python tools/pipe_probe.py [gib] [batch]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from rustfs_amd.erasure import Erasure
    from rustfs_amd.pipeline import _pinned
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    k, m = 8, 4
    e = Erasure(k, m, 1 << 20)
    S = e.shard_size()
    nb = int(gib * 1024)
    torch.cuda.init()
    # (1) one big synchronous host batch: the C++ pipeline chunks it itself
    big = _pinned((nb, k + m, S))
    dig = _pinned((nb, k + m, 32))
    for rep in range(3):
        t0 = time.perf_counter()
        e.encode_batch_host(big, dig)
        dt = time.perf_counter() - t0
    print(f"encode_batch_host one call {nb} blocks: {dt * 1e3:.1f} ms -> {nb * (1 << 20) / dt / 1e9:.1f} GB/s", flush=True)
    e.encode_batch_host(big, None, algo=0)
    t0 = time.perf_counter()
    e.encode_batch_host(big, None, algo=0)
    dt = time.perf_counter() - t0
    print(f"  same, no digests: {dt * 1e3:.1f} ms -> {nb * (1 << 20) / dt / 1e9:.1f} GB/s", flush=True)
    # (2) B-block jobs over 3 rotating buffers, waiting when 3 are out
    for nbuf in (3, 6):
        bufs = [big[i * B:(i + 1) * B] for i in range(nbuf)]
        digs = [dig[i * B:(i + 1) * B] for i in range(nbuf)]
        for rep in range(2):
            t0 = time.perf_counter()
            tickets = []
            sub = 0.0
            wt = 0.0
            for j in range(nb // B):
                if len(tickets) >= nbuf:
                    w0 = time.perf_counter()
                    tickets.pop(0).wait()
                    wt += time.perf_counter() - w0
                s0 = time.perf_counter()
                tickets.append(e.encode_batch_host_submit(bufs[j % nbuf], digs[j % nbuf]))
                sub += time.perf_counter() - s0
            for tk in tickets:
                tk.wait()
            dt = time.perf_counter() - t0
        print(f"submit/wait B={B} bufs={nbuf}: {dt * 1e3:.1f} ms -> {nb * (1 << 20) / dt / 1e9:.1f} GB/s "
              f"(submit {sub * 1e3:.1f} ms, wait {wt * 1e3:.1f} ms)", flush=True)


if __name__ == "__main__":
    main()
