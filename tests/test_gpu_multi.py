"""Multi-GPU readiness on one device: what the driver's 8-GPU run relies on.

Stripes are independent, so each rank owns a context and a
stream and encodes its contiguous slice with no collective.  These tests run
two contexts with their own streams concurrently on device 0 through the
device-batch ABI, and the host-side multi-device splitter
(dispatch.encode_host_multi) — every result checked against the oracle.
"""
import ctypes
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_two_contexts_two_streams_concurrently(gpu, oracle):
    import torch
    from rustfs_amd import _lib
    from rustfs_amd.dispatch import split_batch
    k, m, S, total = 8, 4, 131072, 96
    g = torch.Generator(device="cuda").manual_seed(3)
    st = torch.zeros((total, k + m, S), dtype=torch.uint8, device="cuda")
    st[:, :k] = torch.randint(0, 256, (total, k, S), dtype=torch.uint8, device="cuda", generator=g)
    dig = torch.zeros((total, k + m, 32), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ctxs = [_lib.Context(0), _lib.Context(0)]  # one per "rank"
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    errs = []

    def rank(r):
        try:
            s0, cnt = split_batch(total, 2, r)
            for _ in range(3):  # repeated launches interleave with the other rank's
                rc = _lib.load().rsg_encode_batch_dev(
                    ctxs[r].handle, k, m, S, cnt, st[s0].data_ptr(), S, (k + m) * S, dig[s0].data_ptr(),
                    _lib.RSG_HASH_HIGHWAY256S, streams[r].cuda_stream)
                _lib.check(rc)
            _lib.check(_lib.load().rsg_sync(ctxs[r].handle, streams[r].cuda_stream))
        except Exception as exc:  # surfaced below
            errs.append(repr(exc))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    host, hd = st.cpu().numpy(), dig.cpu().numpy()
    for s in (0, 47, 48, 95):  # both sides of the split
        ref = host[s].copy()
        ref[k:] = 0
        oracle.encode(k, m, ref)
        assert np.array_equal(ref, host[s]), s
        for i in range(k + m):
            assert hd[s, i].tobytes() == oracle.hh256s(ref[i]), (s, i)
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("world", [2, 3])
def test_encode_host_multi(gpu, oracle, world):
    """dispatch.encode_host_multi: one host thread per (device) slice; on a
    one-GPU box every slice lands on device 0, as the 2-rank rehearsal does."""
    import torch
    from rustfs_amd import Erasure
    from rustfs_amd.dispatch import encode_host_multi
    k, m, S, n = 8, 4, 65536, 31
    st = torch.zeros((n, k + m, S), dtype=torch.uint8).pin_memory().numpy()
    st[:, :k] = np.random.default_rng(world).integers(0, 256, (n, k, S), dtype=np.uint8)
    dig = np.zeros((n, k + m, 32), dtype=np.uint8)
    encode_host_multi([Erasure(k, m, k * S, device=0) for _ in range(world)], st, dig)
    for s in range(n):
        ref = st[s].copy()
        ref[k:] = 0
        oracle.encode(k, m, ref)
        assert np.array_equal(ref, st[s]), s
        assert dig[s, k + m - 1].tobytes() == oracle.hh256s(ref[k + m - 1]), s
        assert dig[s, 0].tobytes() == oracle.hh256s(ref[0]), s


def test_device_count_and_context_per_device(gpu):
    from rustfs_amd import _lib
    n = _lib.device_count()
    assert n >= 1
    h = ctypes.c_void_p()
    assert _lib.load().rsg_create(n, ctypes.byref(h)) == _lib.RSG_ERR_NO_DEVICE  # ordinal past the last device


def test_bench_self_launch_two_ranks_rehearsal(gpu):
    """`bench.py --gpus 2` starts its two ranks itself (no torch.distributed.run)
    and reports n_gpus 2 with each rank's device; on a one-GPU box only as an
    explicit --allow-shared-device rehearsal, which the line says it was."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--allow-shared-device", "--batch", "256",
           "--steps", "2", "--warmup", "1", "--warm-seconds", "0", "--no-cpu-baseline", "--no-engines",
           "--config4-batch", "256", "--config5-total", "1001"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=150)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["total_stripes"] == 512
    import torch
    ndev = torch.cuda.device_count()
    assert line["roofline"]["per_rank_device"] == [0, 1 % ndev]
    assert line["roofline"]["shared_device"] == (ndev < 2)
    assert len(line["roofline"]["per_rank_kernel_ms"]) == 2
    # config 5 (RS(16,4), the batch split over the ranks) and config 4 (fused
    # digests, per rank) ride on the N-GPU line
    c5 = line["extras"]["encode_rs16_4"]
    assert c5["n_gpus"] == 2 and c5["total_stripes"] == 1001 and c5["per_rank_stripes"] == [501, 500]
    assert len(c5["per_rank_kernel_ms"]) == 2 and all(f > 0 for f in c5["per_rank_frac"])
    assert c5["per_rank_device"] == [0, 1 % ndev] and c5["GiB_s_payload_all_ranks"] > 0
    c4 = line["extras"]["encode_fused_hh256s"]
    assert c4["n_gpus"] == 2 and c4["per_rank_stripes"] == [256, 256] and len(c4["per_rank_frac"]) == 2
    assert line["extras"]["verify_all_ok_after_reconstruct"]
