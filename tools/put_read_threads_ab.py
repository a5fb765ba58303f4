"""PUT body read threads (put_stream read_threads 4 / 8 / 16) through bench.py's own
host-path measurement (1 GiB, tmpfs), two interleaved rounds."""
import functools, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
import torch
import bench
from rustfs_amd import pipeline
orig = pipeline.put_stream
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev)
for rnd in range(2):
    for rt in (4, 8, 16):
        pipeline.put_stream = functools.partial(orig, read_threads=rt)
        out = bench.host_path_extras(dev, stream, n=1024, reps=4)
        p = out["put_stream_hh256s"]
        g = out["get_stream_all_present"]
        print(json.dumps({"read_threads": rt, "put_ms": p["ms"], "clock": p["clock_ms"], "get_ms": g["ms"]}), flush=True)
