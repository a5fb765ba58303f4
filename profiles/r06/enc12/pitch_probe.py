"""RS(12,4) encode at S = 87382 with the shard rows at padded pitches (row
starts 2, 4, 16, 128-byte aligned): is the ragged layout's cost the row
alignment?"""
import ctypes, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from rustfs_amd import _lib
L = _lib.load()
ctx = _lib.context(0).handle
k, m, S, n = 12, 4, 87382, 4096
t = k + m
stream = torch.cuda.current_stream()
for pitch in (87382, 87384, 87392, 87424, 87552):
    stride = t * pitch
    buf = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device="cuda")
    def go():
        _lib.check(L.rsg_encode_batch_dev(ctx, k, m, S, n, buf.data_ptr(), pitch, stride, None, 0, stream.cuda_stream))
    for _ in range(3): go()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        for _ in range(4): go()
        torch.cuda.synchronize()
    res = []
    for r in range(3):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for a, b in ev:
            a.record(stream); go(); b.record(stream)
        torch.cuda.synchronize()
        res.append(sum(a.elapsed_time(b) for a, b in ev) / len(ev))
    ms = sorted(res)[1]
    alg = n * t * S
    print(json.dumps({"pitch": pitch, "ms": round(ms, 4), "frac": round(alg / (ms * 1e-3) / 8e12, 4)}), flush=True)
    del buf
    torch.cuda.empty_cache()
