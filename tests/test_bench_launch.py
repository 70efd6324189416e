"""CPU: bench.py's multi-GPU launch contract without a GPU.  `python bench.py --gpus N`
started without torchrun launches N rank processes itself (before anything touches a
GPU); --dry-run stops each rank right after torch.distributed is up."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
sys.path.insert(0, ROOT)


def clean_env():
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    return env


def test_bench_launches_one_process_per_gpu():
    for n in (2, 4):
        r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--dry-run"], capture_output=True, text=True,
                           timeout=180, env=clean_env())
        assert r.returncode == 0, r.stderr[-3000:]
        out = json.loads(r.stdout.strip().splitlines()[-1])
        assert out["dry_run"] and out["n_gpus"] == n
        ranks = sorted(out["ranks"], key=lambda i: i["rank"])
        assert [i["rank"] for i in ranks] == list(range(n))
        assert [i["local_rank"] for i in ranks] == list(range(n))      # rank r drives GPU r
        assert all(i["world"] == n for i in ranks)
        assert len(set(i["pid"] for i in ranks)) == n                   # one process per GPU
        assert len(set(i["master"] for i in ranks)) == 1 and ranks[0]["master"].startswith("127.0.0.1:")
        assert all(i["events_per_gpu"] == 100_000_000 for i in ranks)


def test_bench_eight_gpus_is_one_billion_events():
    import bench
    assert bench.parse_args(["--gpus", "8"]).events == 125_000_000          # configs[3]: 1B events
    assert bench.parse_args(["--gpus", "1"]).events == 100_000_000          # configs[1]
    assert bench.parse_args(["--gpus", "2"]).events == 100_000_000
    assert bench.parse_args(["--gpus", "8", "--events", "7"]).events == 7


def test_bench_launcher_stops_the_ranks_when_one_fails():
    env = clean_env()
    env["YSB_BENCH_FAIL_RANK"] = "1"
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--dry-run"], capture_output=True, text=True,
                       timeout=180, env=env)
    assert r.returncode == 3 and "stopping the others" in r.stderr


def test_rank_device_mapping():
    """LOCAL_RANK -> device (bench.Dist.resolve_device over the library's hipGetDeviceCount):
    the local rank on a node that shows every GPU, modulo the visible ones when the launcher
    shows each process fewer, and the local rank itself when none is visible (the context's
    open then fails loudly instead of every rank sharing device 0)."""
    from ysb_amd import rank_device
    assert [rank_device(r, 8) for r in range(8)] == list(range(8))
    assert [rank_device(r, 1) for r in range(4)] == [0, 0, 0, 0]
    assert [rank_device(r, 2) for r in range(4)] == [0, 1, 0, 1]
    assert rank_device(5, 0) == 5


def test_device_count_without_a_gpu_is_zero():
    """ysb_device_count on this CPU-only container: 0, no exception, no framework needed."""
    from ysb_amd import device_count
    assert device_count() == 0
