"""CPU tests of bench.py's multi-GPU launch: `bench.py --gpus
N` starts N rank processes itself, each bound to its own device, and refuses
(non-zero, with a message) any run that would time fewer GPUs than it reports.
"""
import json
import os
import subprocess
import sys

import pytest

import bench
from rustfs_amd.dispatch import check_world, device_for_rank, rank_plan

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rank_plan_env():
    plans = rank_plan(4, 29555, {"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    assert len(plans) == 4
    for r, env in enumerate(plans):
        assert env["RANK"] == env["LOCAL_RANK"] == str(r)
        assert env["WORLD_SIZE"] == env["LOCAL_WORLD_SIZE"] == "4"
        assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29555"
        assert env["PATH"] == "/bin" and env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    with pytest.raises(ValueError):
        rank_plan(0, 1, {})


def test_check_world_refusals():
    assert check_world(8, 8, 8, False) is None
    assert check_world(1, 1, 1, False) is None
    assert "launched" in check_world(8, 1, 8, False)        # --gpus 8, one rank
    assert "launched" in check_world(1, 2, 8, False)        # torchrun 2 ranks, --gpus 1
    assert "only 1 are visible" in check_world(2, 2, 1, False)
    assert check_world(2, 2, 1, True) is None               # explicit rehearsal
    assert "no GPU" in check_world(1, 1, 0, True)


def test_device_for_rank():
    assert [device_for_rank(r, 8, False) for r in range(8)] == list(range(8))
    assert [device_for_rank(r, 1, True) for r in range(3)] == [0, 0, 0]
    with pytest.raises(ValueError):
        device_for_rank(1, 1, False)


STAND_IN = r'''
import json, os, sys
r = int(os.environ["RANK"])
if "--fail-rank" in sys.argv and str(r) == sys.argv[sys.argv.index("--fail-rank") + 1]:
    sys.exit(3)
if r == 0:
    print(json.dumps({"rank": r, "world": os.environ["WORLD_SIZE"], "local": os.environ["LOCAL_RANK"],
                      "master": os.environ["MASTER_ADDR"], "argv": sys.argv[1:]}), flush=True)
'''


def test_launcher_relays_rank0_line(tmp_path, capfd):
    script = tmp_path / "rank.py"
    script.write_text(STAND_IN)
    argv = ["--gpus", "3", "--steps", "2"]
    a = bench.parse(argv)
    assert bench.launch_ranks(a, argv, script=str(script), devices=3) == 0
    out = capfd.readouterr().out.strip().splitlines()
    assert len(out) == 1
    line = json.loads(out[0])
    assert line == {"rank": 0, "world": "3", "local": "0", "master": "127.0.0.1", "argv": argv}


def test_launcher_propagates_rank_failure(tmp_path, capfd):
    script = tmp_path / "rank.py"
    script.write_text(STAND_IN)
    argv = ["--gpus", "2"]
    a = bench.parse(argv)
    assert bench.launch_ranks(a, argv + ["--fail-rank", "1"], script=str(script), devices=2) == 3
    assert "rank 1 exited with 3" in capfd.readouterr().err


def test_launcher_refuses_too_few_devices(tmp_path, capfd):
    script = tmp_path / "rank.py"
    script.write_text(STAND_IN)
    a = bench.parse(["--gpus", "8"])
    assert bench.launch_ranks(a, ["--gpus", "8"], script=str(script), devices=1) == 2
    assert "only 1 are visible" in capfd.readouterr().err


def test_bench_refuses_without_gpu_or_matching_world():
    """The real script, no GPU in this container: --gpus 2 must fail loudly
    (not time one rank), and so must a torchrun-style world that differs
    from --gpus.  Neither touches a device."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2 and "no GPU visible" in p.stderr and p.stdout == ""
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2 and "2 rank(s) were launched" in p.stderr and p.stdout == ""


SLEEPER = r'''
import os, sys, time
open(os.path.join(sys.argv[-1], "rank%s.pid" % os.environ["RANK"]), "w").write(str(os.getpid()))
time.sleep(300)
'''


def test_launcher_terminated_takes_ranks_along(tmp_path):
    """SIGTERM to `bench.py --gpus N` (a driver's time limit) ends its rank
    processes too: none is left holding a GPU."""
    import signal
    import time
    script = tmp_path / "rank.py"
    script.write_text(SLEEPER)
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "a = bench.parse(['--gpus', '2']); "
            "sys.exit(bench.launch_ranks(a, ['--gpus', '2', %r], script=%r, devices=2))"
            % (ROOT, str(tmp_path), str(script)))
    p = subprocess.Popen([sys.executable, "-c", code])
    pids = []
    for _ in range(200):
        pids = [tmp_path / f"rank{r}.pid" for r in range(2)]
        if all(f.exists() and f.read_text() for f in pids):
            break
        time.sleep(0.05)
    pids = [int(f.read_text()) for f in pids]
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=30) != 0
    for pid in pids:
        for _ in range(100):
            try:
                os.kill(pid, 0)
            except ProcessLookupError:
                break
            time.sleep(0.05)
        else:
            os.kill(pid, signal.SIGKILL)
            raise AssertionError(f"rank process {pid} outlived the launcher")


@pytest.mark.parametrize("world", [1, 2, 8])
def test_config5_plan(world):
    """Config 5 extra (RS(16,4), the batch split over the node's GPUs): every
    stripe of the 32768-stripe batch is encoded by exactly one rank; one GPU
    alone runs its 1/8 share."""
    import bench
    total = 32768
    plans = [bench.config5_plan(world, r, total) for r in range(world)]
    if world == 1:
        assert plans == [(0, total // 8, total // 8)]
        return
    assert all(p[2] == total for p in plans)
    covered = []
    for s0, cnt, _ in plans:
        covered += list(range(s0, s0 + cnt))
    assert covered == list(range(total))
    assert max(p[1] for p in plans) - min(p[1] for p in plans) <= 1


def test_pmc_traffic_covers_the_default_line():
    """Every traffic entry the default bench line looks up (headline, configs
    3/4/5, the RS(8,4) engines and the RS(12,4) extras) is in
    tools/pmc_traffic.json (shipped with the tree), and each is within 1.5 % of
    the algorithmic bytes of its launch at RS(8,4) / RS(16,4) (no wasted
    re-reads; the whole-file verify reads each 32-byte digest header as a
    sector of its own: 1.011) and 5 % at RS(12,4): its unaligned 87382-byte rows are written a
    512-byte step at a time, and a step's first and last sectors, shared with
    the neighbouring step, leave the L2 twice (writes 1-15 % over the payload,
    1.00-1.041 overall)."""
    import bench
    want = {}
    for k, S in ((8, 131072), (12, 87382)):
        n = 4096
        t, rec = k + 4, 32 + S
        want[f"rs{k}4_S{S}_n{n}"] = n * t * S
        want[f"rs{k}4_S{S}_n{n}_hash"] = n * t * S
        for name, alg, key in bench.engine_plan(k, 4, S, n, full=False):
            want[key] = alg
    want["rs164_S65536_n4096"] = 4096 * 20 * 65536
    for r in (1, 2, 3, 4):
        want[f"reconstruct_e{r}_rs84_S131072_n4096"] = 4096 * (8 + r) * 131072
    for key, alg in want.items():
        got = bench.pmc_lookup(key)
        assert got is not None, key
        assert abs(got / alg - 1) < (0.05 if "rs124" in key else 0.015), (key, got, alg)


def test_pmc_traffic_sources_are_committed_counters():
    """Every entry of tools/pmc_traffic.json names a committed directory of raw
    rocprofv3 counters (profiles/r05/pmc/<key>/, tools/pmc_table.sh on the
    shipped library), and its bytes_per_launch is FETCH_SIZE x 2 + WRITE_SIZE
    (KiB, the microarch guide's gfx950 correction) recomputed from those
    CSVs."""
    import json
    import subprocess
    import tools.pmc_traffic as P
    data = json.load(open(os.path.join(ROOT, "tools", "pmc_traffic.json")))
    tracked = set(subprocess.run(["git", "ls-files"], cwd=ROOT, capture_output=True, text=True,
                                 check=True).stdout.split())
    assert data
    for key, v in data.items():
        src = v["source"]
        for f in ("meta.json", "FETCH_SIZE/run_counter_collection.csv", "WRITE_SIZE/run_counter_collection.csv"):
            assert f"{src}/{f}" in tracked, (key, f)
        k2, again = P.entry(os.path.join(ROOT, src))
        assert k2 == key and again["bytes_per_launch"] == v["bytes_per_launch"], key


def test_engine_plan_rs12_4():
    """The RS(12,4) extras of the driver's line (the 16-drive default set,
    storageclass.rs:24-31): in-place GET with 0 and 2 data lost, heal of one
    data + one parity disk and the whole-file bitrot_verify, priced on the
    contract's minimum bytes at S = ceil(1 MiB / 12) = 87382, n = 4096; the
    RS(8,4) line adds the asynchronous GETs (all present, two lost) and heal."""
    import bench
    k, m, n = 12, 4, 4096
    S = -(-(1 << 20) // k)
    assert S == 87382
    t, rec = k + m, 32 + S
    plan = {name: (alg, key) for name, alg, key in bench.engine_plan(k, m, S, n, full=False)}
    assert plan == {
        "get_all_present": (n * k * rec, "get_into0_rs124_S87382_n4096"),
        "get_2_data_lost": (n * (14 * rec + 2 * S), "get_into2_rs124_S87382_n4096"),
        "heal_1data_1parity": (n * t * rec, "heal_1d1p_rs124_S87382_n4096"),
        "bitrot_verify_all_files": (t * n * rec, "verify_all_rs124_S87382_n4096"),
    }
    full = [name for name, _, _ in bench.engine_plan(8, 4, 131072, 4096)]
    assert full[-3:] == ["get_all_present_async", "get_2_data_lost_async", "heal_1data_1parity_async"]
    # the engine loops time at least 20 calls after a >= 0.5 s busy warm-up
    assert bench.ENGINE_REPS >= 20 and bench.ENGINE_WARM_S >= 0.5
    a = bench.parse([])
    assert a.rs12_batch == 4096 and not a.no_rs12


def test_host_path_plan():
    """extras.host_path (north_star: the rate including pinned hipMemcpyAsync
    to and from the GPU): RS(8,4), 1 MiB blocks, 1024 blocks per call on the
    default line; the bytes each entry moves over the link and its link bound
    at the measured copy rates (both directions overlapped)."""
    k, m, S, n = 8, 4, 131072, 1024
    t, rec = k + m, 32 + S
    plan = {name: (bi, bo, pay) for name, bi, bo, pay in bench.host_path_plan(k, m, S, n)}
    pay = n * k * S
    assert pay == 1 << 30
    assert plan == {
        "encode_batch_host": (pay, n * m * S, pay),
        "encode_batch_host_hh256s": (pay, n * m * S + n * t * 32, pay),
        # every present record in, only the rebuilt data shards out
        "get_stream_all_present": (n * t * rec, 0, pay),
        "get_stream_2_data_lost": (n * (t - 2) * rec, 2 * n * S, pay),
        "get_stream_bytes_all_present": (n * t * rec, 0, pay),
        "get_stream_data_shards_only_all_present": (n * k * rec, 0, pay),
        "put_stream_hh256s": (pay, n * m * S + n * t * 32, pay),
    }
    # the larger direction bounds a full-duplex transfer
    assert bench.link_bound_ms(50e9, 10e9, 50.0, 50.0) == pytest.approx(1000.0)
    assert bench.link_bound_ms(10e9, 50e9, 50.0, 25.0) == pytest.approx(2000.0)
    a = bench.parse([])
    assert a.host_path_blocks == 1024 and not a.no_host_path
