"""CPU: the native drop-in runner (streaming-benchmarks_amd/bin/ysb_topology, C++ above
the C ABI) -- config loading (Utils.findAndReadConfigFile), both ad-map formats
(getAdCampaignMap, core.clj:58), the events source (FileBasedDataSource) and the C++
Redis writer, all without a GPU (--dry-run / --replay-rows).  The GPU runs are in
tests/test_gpu_topology.py."""
import json
import os
import subprocess

import pytest

import golden_data as gd
from oracle import dostats
from fake_redis import FakeRedis
from test_redis_sink import canonical, dostats_shape, golden_rows
from ysb_amd.redis_sink import RespClient, RedisWindowWriter, check_correct

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "streaming-benchmarks_amd", "bin", "ysb_topology")


def write_conf(tmp_path, events, admap, extra=""):
    p = tmp_path / "benchmarkConf.yaml"
    p.write_text("""# a config with the reference's keys (conf/benchmarkConf.yaml)
ad_to_campaign_path: "%s"

events_path: '%s'
kafka.brokers:
    - "localhost"
    - other   # a comment
zookeeper.servers:
    - "localhost"
kafka.port: 9092
redis.host: "localhost"
redis.hashtable: "t1"
window.size: 5000
map.partitions: 3
reduce.partitions: 1
%s""" % (admap, events, extra))
    return str(p)


def run(*args, ok=True):
    r = subprocess.run([EXE] + list(args), capture_output=True, text=True, timeout=120)
    if ok:
        assert r.returncode == 0, r.stderr
    return r


def last_json(r):
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("events,admap,n,fmt", [
    ("gen_s7.jsonl", "gen_s7.ad_to_campaign.txt", 1500, "json"),
    ("gen_s7.jsonl", "gen_s7.ad_to_campaign.csv", 1500, "json"),
    ("gen_s7.tbl", "gen_s7.ad_to_campaign.csv", 1500, "tbl"),
    ("edge_tbl.tbl", "gen_s7.ad_to_campaign.txt", 21, "tbl"),
])
def test_dry_run_reads_map_and_events(tmp_path, events, admap, n, fmt):
    conf = write_conf(tmp_path, gd.path(events), gd.path(admap))
    out = last_json(run("--confPath", conf, "--dry-run"))
    assert out["events"] == n and out["format"] == fmt
    assert out["ads"] == len(gd.ad_map()) and out["campaigns"] == len(gd.campaigns())


def test_source_batches_carry_partial_lines(tmp_path):
    conf = write_conf(tmp_path, gd.path("gen_s7.jsonl"), gd.path("gen_s7.ad_to_campaign.txt"))
    size = os.path.getsize(gd.path("gen_s7.jsonl"))
    for extra in (["--batch-bytes", "1000"], ["--batch-events", "7"], ["--batch-bytes", "4096", "--batch-events", "3"]):
        out = last_json(run("--confPath", conf, "--dry-run", *extra))
        assert out["events"] == 1500 and out["bytes"] == size and out["batches"] > 1


def test_readline_terminators(tmp_path):
    raw, offs = gd.events("gen_s7")
    lines = raw.split(b"\n")[:-1]
    ev = tmp_path / "crlf.jsonl"
    ev.write_bytes(b"\r\n".join(lines[:100]))          # CRLF, no final terminator
    conf = write_conf(tmp_path, str(ev), gd.path("gen_s7.ad_to_campaign.txt"))
    assert last_json(run("--confPath", conf, "--dry-run"))["events"] == 100


@pytest.mark.parametrize("batch", [[], ["--batch-bytes", "600"], ["--batch-bytes", "300"], ["--batch-bytes", "523"], ["--batch-bytes", "777"]])
def test_readline_lone_cr_and_mixed_terminators(tmp_path, batch):
    """BufferedReader.readLine ends a line at "\\n", "\\r\\n" or a lone "\\r": the source
    yields the records oracle/dostats.split_lines does, also when a batch ends between
    '\\r' and '\\n'."""
    raw, _ = gd.events("gen_s7")
    lines = raw.split(b"\n")[:-1][:60]
    seps = [b"\n", b"\r\n", b"\r", b"\r\r", b"\n\n", b"\r\n\r"]
    data = b"".join(ln + seps[i % len(seps)] for i, ln in enumerate(lines)) + b"x\ry"
    ev = tmp_path / "mixed.jsonl"
    ev.write_bytes(data)
    conf = write_conf(tmp_path, str(ev), gd.path("gen_s7.ad_to_campaign.txt"))
    want = len(dostats.split_lines(data)[0])
    out = last_json(run("--confPath", conf, "--dry-run", *batch))
    assert out["events"] == want and out["bytes"] == len(data)


@pytest.mark.parametrize("batch", ["300", "523", "777", "4096", "268435456"])
def test_mapped_source_ranges_are_whole_lines(tmp_path, batch):
    """--io mapped hands the GPU ranges of the file mapping itself (nextMapped): back to back,
    every byte once, each ending at a readLine terminator -- never between '\r' and '\n' --
    except the file's unterminated last line."""
    raw, _ = gd.events("gen_s7")
    lines = raw.split(b"\n")[:-1][:60]
    seps = [b"\n", b"\r\n", b"\r", b"\r\r", b"\n\n", b"\r\n\r"]
    data = b"".join(ln + seps[i % len(seps)] for i, ln in enumerate(lines)) + b"x\ry"
    ev = tmp_path / "mixed.jsonl"
    ev.write_bytes(data)
    conf = write_conf(tmp_path, str(ev), gd.path("gen_s7.ad_to_campaign.txt"))
    out = last_json(run("--confPath", conf, "--dry-run", "--io", "mapped", "--batch-bytes", batch))
    assert out["io"] == "mapped" and out["bytes"] == len(data) and out["unterminated"] == 1
    assert out["batches"] == (1 if int(batch) > len(data) else out["batches"]) and out["batches"] >= 1
    if int(batch) < len(data):
        assert out["batches"] >= len(data) // int(batch)
    r = run("--confPath", conf, "--io", "mapped", "--host-split", ok=False)
    assert r.returncode == 2 and "--host-split" in r.stderr


@pytest.mark.parametrize("shards,seed", [(1, 1), (2, 2), (3, 3), (8, 4)])
def test_stream_shards_flush_merge(shards, seed):
    """--stream-merge-check (CPU, no GPU): the per-shard feeders' flushes, delivered by one
    thread per shard at random moments with jittered watermarks, go through the runner's own
    merger and sink thread: every index once and in order, every shard's rows, the minimum
    watermark (Flink's at a keyed operator), and exactly the windows those watermarks pass
    closed (host/ysb_stream.cpp FlushMerger, SinkThread; CampaignProcessorCommon.java:35-55)."""
    r = run("--stream-merge-check", "--shards", str(shards), "--merge-flushes", "250", "--seed", str(seed))
    out = last_json(r)
    assert out["ok"] and out["in_order"] and out["watermark_min"] and out["rows"]
    assert out["delivered"] == 250 and out["closed"] == out["closed_expected"] > 50


def test_print_config(tmp_path):
    conf = write_conf(tmp_path, "/x/events.tbl", gd.path("gen_s7.ad_to_campaign.csv"))
    r = run("--confPath", conf, "--print-config", "--dry-run", ok=False)
    cfg = json.loads(r.stdout.splitlines()[0])
    assert cfg["kafka.brokers"] == ["localhost", "other"]
    assert cfg["events_path"] == "/x/events.tbl" and cfg["window.size"] == "5000"
    assert cfg["redis.host"] == "localhost" and cfg["ad_to_campaign_path"].endswith(".csv")


def test_reference_errors(tmp_path):
    r = run("--confPath", str(tmp_path / "nope.yaml"), ok=False)
    assert r.returncode == 1 and "Could not find config file" in r.stderr
    bad = tmp_path / "bad.csv"
    bad.write_text("a1,c1\na2\n")                       # split(",") -> 1 item: kv[1] throws
    conf = write_conf(tmp_path, gd.path("gen_s7.jsonl"), str(bad))
    r = run("--confPath", conf, "--dry-run", ok=False)
    assert r.returncode == 1 and "ArrayIndexOutOfBounds" in r.stderr
    conf = write_conf(tmp_path, str(tmp_path / "missing.jsonl"), gd.path("gen_s7.ad_to_campaign.csv"))
    r = run("--confPath", conf, "--dry-run", ok=False)
    assert r.returncode == 1 and "FileNotFoundException" in r.stderr
    r = subprocess.run([EXE], capture_output=True, text=True)
    assert r.returncode == 2 and "confPath" in r.stderr


def test_csv_map_later_duplicate_wins(tmp_path):
    m = tmp_path / "m.csv"
    m.write_text("a1,c1\na2,c2\na1,c2\n")
    conf = write_conf(tmp_path, gd.path("gen_s7.jsonl"), str(m))
    out = last_json(run("--confPath", conf, "--dry-run"))
    assert out["ads"] == 2 and out["campaigns"] == 2


def test_cpp_redis_writer_matches_python_writer(tmp_path):
    rows = golden_rows()
    camps = gd.campaigns()
    csv = tmp_path / "rows.csv"
    csv.write_text("campaign_id,window_ms,count\n" + "".join("%s,%d,%d\n" % (camps[c], w, n) for c, w, n in rows))
    conf = write_conf(tmp_path, gd.path("gen_s7.jsonl"), gd.path("gen_s7.ad_to_campaign.txt"))
    a, b = FakeRedis(), FakeRedis()
    try:
        out = last_json(run("--confPath", conf, "--sink", "redis:127.0.0.1:%d" % a.port, "--replay-rows", str(csv)))
        assert out["rows"] == len(rows) and out["round_trips"] == 2
        cli = RespClient("127.0.0.1", a.port)
        assert all(s == "CORRECT" for _, _, s, _ in check_correct(cli, dostats_shape()))
        cli.close()
        cb = RespClient("127.0.0.1", b.port)
        RedisWindowWriter(cb, camps, clock_ms=lambda: 0).write(rows)
        cb.close()
        ca, cbb = canonical(a.kv), canonical(b.kv)
        # time_updated values differ (wall clocks); everything else is identical
        for kv in (ca, cbb):
            kv.pop("time_updated")
            for k, v in kv.items():
                if isinstance(v, dict):
                    v.pop("time_updated", None)
        assert ca == cbb
    finally:
        a.close()
        b.close()


def test_cpp_redis_writer_many_rows(tmp_path):
    """A config-3-sized flush (30k distinct (campaign, window) rows) is written in two
    round trips and in linear time (the writer dedups its pending keys with sets)."""
    camps = ["c%05d" % i for i in range(300)]
    rows = [(c, 1700000000000 + 10000 * w, 1 + (c + w) % 5) for c in range(300) for w in range(100)]
    csv = tmp_path / "rows.csv"
    csv.write_text("campaign_id,window_ms,count\n" + "".join("%s,%d,%d\n" % (camps[c], w, n) for c, w, n in rows))
    conf = write_conf(tmp_path, gd.path("gen_s7.jsonl"), gd.path("gen_s7.ad_to_campaign.txt"))
    a = FakeRedis()
    try:
        out = last_json(run("--confPath", conf, "--sink", "redis:127.0.0.1:%d" % a.port, "--replay-rows", str(csv)))
        assert out["rows"] == len(rows) and out["round_trips"] == 2
        cli = RespClient("127.0.0.1", a.port)
        for c, w, n in rows[::997]:
            wid = cli.execute("HGET", camps[c], str(w))
            assert int(cli.execute("HGET", wid, "seen_count")) == n
        cli.close()
    finally:
        a.close()


def test_parallel_source_on_a_large_file(tmp_path):
    """Blocks of >= 8 MiB take the multi-threaded pread + split path."""
    d = tmp_path / "gen"
    d.mkdir()
    gen = os.path.join(ROOT, "streaming-benchmarks_amd", "bin", "ysb_gen")
    subprocess.run([gen, "-d", str(d), "-n", "250000", "--seed", "9"], check=True)
    ev = d / "kafka-json.txt"
    conf = write_conf(tmp_path, str(ev), str(d / "ad-to-campaign.csv"))
    for extra in (["--batch-mb", "16"], ["--batch-mb", "9", "--batch-events", "40000"], ["--batch-mb", "256"]):
        out = last_json(run("--confPath", conf, "--dry-run", *extra))
        assert out["events"] == 250000 and out["bytes"] == os.path.getsize(ev), extra


@pytest.mark.parametrize("rate,skew,batch_ms", [(20_000, 1, 100), (3_000, 2, 7), (50_000, 0, 100)])
def test_stream_replay_rebasing_equals_the_generator(rate, skew, batch_ms):
    """The streaming mode's replay (host/ysb_stream.cpp): one generated cycle of 10 s of event
    time, cycled with every event_time moved by the cycle length by patching the nine leading
    time digits while a batch is copied.  For cycles 0, 1, 2, 7 and 1000 every batch equals,
    byte for byte, the generator's own lines of that cycle (t0 moved by cycle x 10 s) -- with the
    reference's skew and late events (skew 1: late times several windows back), skew only, and
    none; so the truth of a streaming run is the generator truth of each played cycle."""
    exe = os.path.join(ROOT, "streaming-benchmarks_amd", "bin", "ysb_topology")
    r = subprocess.run([exe, "--stream-self-check", "--event-rate", str(rate), "--skew", str(skew),
                        "--batch-ms", str(batch_ms), "--batch-mb", "1"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    s = json.loads(r.stdout.strip().splitlines()[-1])
    assert s["lines_per_cycle"] == rate * 10 and s["lines"] == 5 * s["lines_per_cycle"]
    assert s["mismatched_batches"] == 0
    assert s["misaligned_batches"] == 0      # every batch 64-byte aligned (ysb_submit_raw_mapped)
    assert s["upper_values"] >= {0: 1, 1: 7, 2: 2}[skew]


def test_stream_feed_check_runs_one_feeder_per_shard():
    """--stream-feed-check (CPU, no GPU): each shard's feeder on a thread of its own, filling its
    slot (round 5's copy path: memcpy + time-digit patch) -- the aggregate rate is reported per
    shard count; the numbers for DESIGN.md come from a quiet machine, here only the contract."""
    exe = os.path.join(ROOT, "streaming-benchmarks_amd", "bin", "ysb_topology")
    for shards in (1, 2):
        r = subprocess.run([exe, "--stream-feed-check", "--shards", str(shards), "--event-rate", "20000",
                            "--feed-seconds", "0.3", "--batch-mb", "4"], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        s = json.loads(r.stdout.strip().splitlines()[-1])
        assert s["shards"] == shards and s["lines_per_cycle"] == 200_000 and s["copy_events_per_s"] > 0
