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


def test_live_traffic_reads_the_two_pmc_passes(monkeypatch, tmp_path):
    """bench.live_traffic (roofline.traffic measured in the run): two child passes of bench.py
    under rocprofv3, one counter each, launched with the program after `--`; per-dispatch
    averages of the named kernel only, FETCH_SIZE x 2 (gfx950) and KiB -> bytes.  The
    profiler is stubbed: this checks the commands and the arithmetic, not the counters."""
    import shutil
    import bench
    calls = []

    def fake_run(cmd, cwd=None, env=None, capture_output=None, text=None, timeout=None):
        calls.append(cmd)
        counter = cmd[cmd.index("--pmc") + 1]
        out = cmd[cmd.index("-d") + 1]
        os.makedirs(out, exist_ok=True)
        kern = "void ysb::scan_kernel<false, false, false, 0>(ysb::ScanParams)"
        rows = [("__amd_rocclr_fillBufferAligned", 5.0), (kern, 100.0), (kern, 300.0)]
        with open(os.path.join(out, "run_counter_collection.csv"), "w") as f:
            f.write('"Kernel_Name","Counter_Name","Counter_Value"\n')
            for k, v in rows:
                f.write('"%s","%s",%f\n' % (k, counter, v * (1 if counter == "FETCH_SIZE" else 0.5)))
        return subprocess.CompletedProcess(cmd, 0, "", "")

    monkeypatch.setattr(shutil, "which", lambda name: "/opt/rocm/bin/rocprofv3" if name == "rocprofv3" else None)
    monkeypatch.setattr(subprocess, "run", fake_run)
    args = bench.parse_args([])
    r = bench.live_traffic(args, "void ysb::scan_kernel<false, false, false, 0>")
    assert len(calls) == 2
    for cmd, counter in zip(calls, ("FETCH_SIZE", "WRITE_SIZE")):
        assert cmd[cmd.index("--pmc") + 1] == counter
        assert cmd[cmd.index("--") + 1] == sys.executable and "--no-live-traffic" in cmd   # no nested profiler
    assert r["hbm_read_bytes_per_launch"] == int(2 * 200.0 * 1024)     # mean of the kernel's dispatches
    assert r["hbm_write_bytes_per_launch"] == int(100.0 * 1024)
    assert r["hbm_bytes_per_launch"] == r["hbm_read_bytes_per_launch"] + r["hbm_write_bytes_per_launch"]
    # without rocprofv3 there is no live figure (the line falls back to pmc_traffic.json)
    monkeypatch.setattr(shutil, "which", lambda name: None)
    assert bench.live_traffic(args, "x") is None


REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "check")


def _r05_line():
    """profiles/r05_bench.json: the round-5 line with its 19 extras legs in full (the line the
    driver could not parse: 21.8 KB)."""
    with open(os.path.join(ROOT, "profiles", "r05_bench.json")) as f:
        d = json.load(f)
    extra = d.pop("extras")
    return d, extra


def test_bench_line_is_compact_and_parseable(tmp_path, capsys):
    """The printed line (bench.emit): the contract keys + one summary per extra leg, <= 6 KB,
    the last stdout line, json.loads-able; the extras in full go to the file and to stderr."""
    import bench
    out, extra = _r05_line()
    assert len(json.dumps(dict(out, extras=extra))) > 20000          # the round-5 failure
    path = str(tmp_path / "extras.json")
    bench.emit(out, extra, path)
    cap = capsys.readouterr()
    last = cap.out.strip().splitlines()[-1]
    assert len(last) <= bench.LINE_MAX_BYTES
    line = json.loads(last)
    for k in REQUIRED:
        assert k in line, k
    assert line["roofline"]["frac"] == out["roofline"]["frac"] and line["roofline"]["traffic"]
    assert line["cpu_baseline"]["cores"] >= 1
    summ = line["extras_summary"]
    assert set(summ) == set(extra) and not line.get("extras_truncated")
    assert summ["config3"]["exact"] is True and summ["config3"]["hbm_frac"] > 0.5
    assert summ["stream_native"]["exact"] is True and summ["stream_native"]["events_per_s"] > 1e8
    assert set(summ["host_staged"]) == {"offsets", "raw", "offsets_dma_engine"}
    assert summ["native_runner"]["gpu_split"]["events_per_s"] > 1e8
    with open(path) as f:
        assert json.load(f) == extra                                   # the file holds them in full
    assert "bench extras: " in cap.err


def test_bench_line_n_gpus_and_watchdog(capsys):
    """The N > 1 line (exchange block, the configs[2]-table leg with its checksum check) and the
    watchdog's line (a timed-out leg) follow the same format and size bound."""
    import bench
    out, _ = _r05_line()
    out = dict(out, n_gpus=8, scaling="weak",
               exchange={"ms_per_step": 0.31, "critical_ms_per_step": 0.12, "rs_ms_per_step": 0.2,
                         "exposed_ms_per_step": 0.01, "hidden_ms_per_step": 0.19, "bytes_per_step_per_gpu": 12800,
                         "buckets": 16, "cell_bytes": 1, "whole_ring_u64_bytes": 819200})
    c3 = {"workload": "x" * 300, "events_per_s": 1.5e11, "hbm_frac": 0.6,
          "check": {"checksum_blocks_mismatched": 0, "truth_mismatched_cells": 0, "truth_views": 5, "counted_views": 5}}
    bad = dict(c3, check=dict(c3["check"], checksum_blocks_mismatched=1))
    for extra, exact in (({"config3": c3}, True), ({"config3": bad}, False)):
        bench.emit(out, extra, None)
        line = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
        assert line["n_gpus"] == 8 and line["exchange"]["buckets"] == 16
        assert line["extras_summary"]["config3"]["exact"] is exact
    bench.emit(out, {"config3": c3, "timed_out": {"error": "the N > 1 extras timed out after 600 s"}}, None)
    last = capsys.readouterr().out.strip().splitlines()[-1]
    assert len(last) <= bench.LINE_MAX_BYTES
    assert "timed out" in json.loads(last)["extras_summary"]["timed_out"]["error"]


def test_bench_line_drops_legs_rather_than_overflow():
    import bench
    out, extra = _r05_line()
    many = {("leg%03d" % i): v for i, v in enumerate(list(extra.values()) * 10)}
    txt = bench.bench_line(out, many)
    assert len(txt) <= bench.LINE_MAX_BYTES
    line = json.loads(txt)
    assert line["extras_truncated"] and 0 < len(line["extras_summary"]) < len(many)
    for k in REQUIRED:
        assert k in line


def test_bench_never_initialises_torch_cuda():
    """The two-runtime hazard (torch bundles its own HIP runtime): bench.py's device waits go
    through the library (ysb_device_sync), never torch.cuda."""
    import ast
    with open(BENCH) as f:
        tree = ast.parse(f.read())
    uses = [n for n in ast.walk(tree) if isinstance(n, ast.Attribute) and n.attr == "cuda"
            and isinstance(n.value, ast.Name) and n.value.id == "torch"]
    assert not uses
