"""GPU: the native runner (bin/ysb_topology) end to end -- config, map, events file,
pinned double-buffered slots, the fused kernel, flushes -- against the golden
expectations, through the CSV sink and the Redis sink (check-correct reads CORRECT)."""
import csv
import json
import os
import subprocess

import pytest

import golden_data as gd
from fake_redis import FakeRedis
from test_redis_sink import dostats_shape
from test_topology import EXE, last_json, write_conf
from ysb_amd.redis_sink import RespClient, check_correct

pytestmark = pytest.mark.gpu


def read_csv(path):
    idx = gd.campaign_index()
    with open(path) as f:
        return {(idx[r["campaign_id"]], int(r["window_ms"]) // 10000): int(r["count"]) for r in csv.DictReader(f)}


@pytest.mark.parametrize("events,admap,stem,extra", [
    ("gen_s7.jsonl", "gen_s7.ad_to_campaign.txt", "gen_s7", []),
    ("gen_s7.jsonl", "gen_s7.ad_to_campaign.csv", "gen_s7", ["--batch-bytes", "20000", "--batch-events", "50"]),
    ("edge.jsonl", "gen_s7.ad_to_campaign.txt", "edge", []),
    ("edge_long.jsonl", "gen_s7.ad_to_campaign.txt", "edge_long", []),
    ("gen_s7.tbl", "gen_s7.ad_to_campaign.csv", "gen_s7_tbl", ["--batch-bytes", "8192"]),
    ("edge_tbl.tbl", "gen_s7.ad_to_campaign.txt", "edge_tbl", []),
])
@pytest.mark.parametrize("io", ["mmap", "mapped"])
def test_runner_csv_sink_matches_golden(tmp_path, events, admap, stem, extra, io):
    """io = mapped: the file's mapping registered, every batch read in place at whatever byte
    alignment its first line has (ysb_submit_raw_mapped, launch_h2d_copy_unaligned)."""
    conf = write_conf(tmp_path, gd.path(events), gd.path(admap))
    out_csv = tmp_path / "windows.csv"
    r = subprocess.run([EXE, "--confPath", conf, "--sink", "csv:%s" % out_csv, "--flush-ms", "0", "--io", io] + extra,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = last_json(r)
    assert out["h2d"] == ("mapped" if io == "mapped" else "kernel")
    exp_rows, exp_st = gd.expected(stem)
    assert read_csv(out_csv) == exp_rows
    for k, v in exp_st.items():
        assert out[k] == v, k


@pytest.mark.parametrize("batch", ["300", "523", "4096", "268435456"])
def test_runner_mapped_io_readline_terminators(tmp_path, batch):
    """--io mapped over a file whose lines end in "\\n", "\\r\\n", a lone "\\r", blank lines
    and an unterminated last line, cut into tiny batches at every byte alignment: the windows
    and stats equal the oracle's over readLine's records (oracle/dostats.split_lines, run) and
    the slot-copy path's."""
    from oracle import dostats
    raw, _ = gd.events("gen_s7")
    lines = raw.split(b"\n")[:-1][:600]
    seps = [b"\n", b"\r\n", b"\r", b"\r\r", b"\n\n", b"\r\n\r", b"\n"]
    data = b"".join(ln + seps[i % len(seps)] for i, ln in enumerate(lines)) + lines[0][:-3]
    ev = tmp_path / "mixed.jsonl"
    ev.write_bytes(data)
    admap = gd.path("gen_s7.ad_to_campaign.txt")
    conf = write_conf(tmp_path, str(ev), admap)
    with open(admap, "rb") as f:
        want = dostats.run(dostats.split_lines(data)[0], dostats.load_ad_map_json_lines(f.read()))
    idx = gd.campaign_index()
    want_rows = {(idx[c], b): n for (c, b), n in want.counts.items()}
    outs = {}
    for io in ("mapped", "mmap"):
        out_csv = tmp_path / ("w_%s.csv" % io)
        r = subprocess.run([EXE, "--confPath", conf, "--sink", "csv:%s" % out_csv, "--flush-ms", "0", "--io", io,
                            "--batch-bytes", batch], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        outs[io] = last_json(r)
        assert read_csv(out_csv) == want_rows, io
        assert outs[io]["events"] == want.events and outs[io]["parse_errors"] == want.parse_errors, io
    assert outs["mapped"]["h2d"] == "mapped" and outs["mmap"]["h2d"] == "kernel"


def test_runner_redis_sink_check_correct(tmp_path):
    conf = write_conf(tmp_path, gd.path("gen_s7.jsonl"), gd.path("gen_s7.ad_to_campaign.txt"))
    srv = FakeRedis()
    try:
        r = subprocess.run([EXE, "--confPath", conf, "--sink", "redis:127.0.0.1:%d" % srv.port,
                            "--batch-events", "100", "--flush-ms", "0"], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        cli = RespClient("127.0.0.1", srv.port)
        res = check_correct(cli, dostats_shape())
        cli.close()
        assert res and all(s == "CORRECT" for _, _, s, _ in res)
    finally:
        srv.close()


@pytest.mark.parametrize("shards,skew", [(1, 2), (2, 1)])
def test_native_stream_mode_exact(shards, skew):
    """bin/ysb_topology --stream (host/ysb_stream.hpp): a short replay through the pinned
    slots with asynchronous flushes to the Redis writer; every (campaign, window) read back
    through Redis equals the generator truth of what the runner played (check-correct), the
    runner's own totals agree, and the windows the final watermark passed were closed with a
    get-stats sample per (campaign, window).  Two shards share the one GPU (each its own
    context and slots, one watermark = the minimum); skew 1 adds the reference's late events."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import bench_stream
    r = bench_stream.stream_native(device=0, seconds=1.5, event_rate=1_000_000, speedup=20.0, shards=shards,
                                   slot_mb=64, skew=skew, threads=8)
    c = r["check"]
    assert r["exact_vs_generator_truth"], c
    assert c["truth_mismatched_cells"] == 0 and c["counted_views"] == c["truth_views"] > 0
    assert c["parse_errors"] == 0 and c["join_misses"] == 0 and c["overflow_dropped"] == 0
    assert r["flushes"] >= 20 and r["windows_closed"] >= 1
    # a get-stats sample per (campaign, window) of every closed window: 100 per on-time window;
    # with skew 1 a late event (1e-5 of them, < 60 s late) can make an old window of one campaign
    assert 100 <= r["get_stats"]["samples_closed_windows"] <= 100 * r["windows_closed"]
    assert r["runner"]["cycles"] and len(r["runner"]["cycles"]) == shards


def test_native_stream_mode_ring_follows_the_watermark():
    """A 16-bucket ring under 150 s of event time: the runner moves the ring forward as the
    watermark advances (ysb_ring_advance after taking the outstanding flushes), and every
    count -- the buckets the ring left included -- still reaches Redis exactly."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import bench_stream
    r = bench_stream.stream_native(device=0, seconds=2.5, event_rate=500_000, speedup=60.0, slot_mb=32, threads=8,
                                   window_ring=16)
    c = r["check"]
    assert r["ring_advances"] >= 1, r["ring_advances"]
    assert r["exact_vs_generator_truth"], c
    assert c["truth_mismatched_cells"] == 0 and c["counted_views"] == c["truth_views"] > 0
    assert c["overflow_dropped"] == 0 and c["parse_errors"] == 0 and c["join_misses"] == 0
