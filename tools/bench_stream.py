"""configs[4] natively: bin/ysb_topology --stream (host/ysb_stream.hpp) fed from pre-generated
replay bytes through the pinned double-buffered slots, its flushes written through the C++
Redis writer to an in-process RESP server (tests/fake_redis.py), then read back the way the
reference's tooling reads them:

  * get-stats (data/src/setup/core.clj:130-149): per (campaign, window), time_updated -
    window_ms -- the reference's latency metric -- over the windows the watermark closed;
  * check-correct (core.clj:215-237): every (campaign, window)'s seen_count against the
    generator truth (ysb_truth_accumulate over every replay cycle the runner played, each
    cycle's event times moved by the cycle length), plus the runner's own totals CSV.

The replay clock runs `speedup` times faster than the wall clock (a recorded stream played
fast, ysb_stream.hpp): latencies are reported in event-time ms (what get-stats computes with a
writer whose clock is the replay's) and, divided by the speedup, in wall ms.

    python tools/bench_stream.py [--seconds S] [--event-rate E] [--speedup F] ...
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "streaming-benchmarks_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

RUNNER = os.path.join(ROOT, "streaming-benchmarks_amd", "bin", "ysb_topology")


def pct(v, q):
    return float(np.percentile(np.asarray(v, dtype=np.float64), q)) if len(v) else None


def truth_table(device, summary):
    """{(campaign uuid, window_ms): count} of everything the runner played: per shard, its
    generator stream (event_stream 1 + shard over its ad shard) for every whole cycle and the
    lines of the partial one, each cycle's times moved by cycle_ms."""
    from ysb_amd import GenParams, YsbContext, shard_ads
    from ysb_amd.group import table_rows
    s = summary
    base = GenParams(seed=s["seed"], n_campaigns=s["campaigns"], ads_per_campaign=s["ads_per_campaign"])
    cids, aids = base.ids()
    nsh = s["shards"]
    subsets = shard_ads(aids, nsh) if nsh > 1 else [None]
    out = {}
    with YsbContext(device=device, n_campaigns=s["campaigns"], window_ring=1024,
                    ring_base_bucket=s["t0_ms"] // 10000 - 16) as ctx:
        for r in range(nsh):
            for c in range(s["cycles"][r] + 1):
                n = s["lines_per_cycle"] if c < s["cycles"][r] else s["partial_lines"][r]
                if not n:
                    continue
                g = GenParams(seed=s["seed"], n_campaigns=s["campaigns"], ads_per_campaign=s["ads_per_campaign"],
                              t0_ms=s["t0_ms"] + c * s["cycle_ms"], events_per_sec=int(s["event_rate"]),
                              with_skew=s["skew"], event_stream=1 + r,
                              ad_subset=None if subsets[0] is None else subsets[r])
                ctx.truth_accumulate(g, 0, n)
        t, lo = ctx.truth_read()
        _, total, _ = ctx.truth_compare()
        outside = total - int(t.sum())
    for (c, b), v in table_rows(t, lo).items():
        out[(cids[c], b * 10000)] = v
    return out, outside, cids


def stream_native(device=0, seconds=12.0, event_rate=5_000_000, speedup=32.0, shards=1, slot_mb=256,
                  flush_ms=1000, batch_ms=100, ooo_ms=100, skew=2, threads=0, workdir=None, window_ring=64,
                  replay="mapped"):
    from fake_redis import FakeRedis
    from ysb_amd import GenParams
    from ysb_amd.redis_sink import RespClient, check_correct, get_stats, new_setup
    cids, _ = GenParams(seed=42).ids()
    srv = FakeRedis()
    tmp = workdir or tempfile.mkdtemp(prefix="ysb_stream_", dir=os.environ.get("TMPDIR") or "/tmp")
    totals_csv = os.path.join(tmp, "totals.csv")
    try:
        cl = RespClient("127.0.0.1", srv.port)
        new_setup(cl, cids)   # do-new-setup (core.clj:209-214): FLUSHALL, SADD campaigns
        cmd = [RUNNER, "--stream", "--device", str(device), "--sink", "redis:127.0.0.1:%d" % srv.port,
               "--totals", totals_csv, "--seconds", str(seconds), "--event-rate", str(event_rate),
               "--speedup", str(speedup), "--shards", str(shards), "--batch-mb", str(slot_mb),
               "--flush-ms", str(flush_ms), "--batch-ms", str(batch_ms), "--ooo-ms", str(ooo_ms),
               "--skew", str(skew), "--io-threads", str(threads), "--window-ring", str(window_ring),
               "--replay", replay]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            raise RuntimeError("ysb_topology --stream exited %d: %s" % (r.returncode, r.stderr[-2000:]))
        s = json.loads(r.stdout.strip().splitlines()[-1])
        commands = srv.server.state.commands
        # get-stats, exactly as core.clj:130-149 reads it: every campaign window's
        # (seen_count, time_updated - window_ms)
        stats = []
        for campaign in sorted(cl.execute("SMEMBERS", "campaigns")):
            wkey = cl.execute("HGET", campaign, "windows")
            if wkey is None:
                continue
            for wt in cl.execute("LRANGE", wkey, 0, cl.execute("LLEN", wkey)):
                wk = cl.execute("HGET", campaign, wt)
                stats.append((int(wt), int(cl.execute("HGET", wk, "seen_count")),
                              int(cl.execute("HGET", wk, "time_updated")) - int(wt)))
        assert len(stats) == len(get_stats(cl))
        truth, outside, cids = truth_table(device, s)
        # windows the final watermark closed (the runner's last flush): the latency samples
        samples = [lat for w, _, lat in stats if w + 10000 <= s["final_watermark_ms"]]
        closed_set = {w for w, _, _ in stats if w + 10000 <= s["final_watermark_ms"]}
        # check-correct (core.clj:215-237) against the truth, through Redis
        expected = {}
        for (c, w), v in truth.items():
            expected.setdefault(c, {})[w // 10000] = v
        cc = check_correct(cl, expected)
        status = {}
        for _, _, st, _ in cc:
            status[st] = status.get(st, 0) + 1
        # the runner's own totals
        got = {}
        with open(totals_csv) as f:
            next(f)
            for ln in f:
                c, w, n = ln.rstrip("\n").split(",")
                got[(c, int(w))] = int(n)
        mism = sum(1 for k in set(got) | set(truth) if got.get(k, 0) != truth.get(k, 0))
        cl.close()
    finally:
        srv.close()
    f = 1.0 / s["speedup"]
    out = {
        "config": "configs[4] natively (bin/ysb_topology --stream, host/ysb_stream.hpp): %d shard(s), one feeder "
                  "thread per shard on its GPU's NUMA node, the data/ generator's lines replayed from host memory %s, "
                  "event time %.0fx the wall clock (%.2fM events per event-second per shard), skew %s, watermark = "
                  "max event_time - %d ms, asynchronous flush every %d event-ms (ysb_flush_begin/end) through the "
                  "C++ Redis writer to an in-process RESP server"
                  % (s["shards"], {"mapped": "in place (ysb_submit_mapped: the registered cycle read by the copy kernel, "
                                           "its line offsets kept in HBM, the time digits rebased on the GPU)",
                                 "mapped-raw": "in place with the line split on the GPU (ysb_submit_raw_mapped, the time "
                                               "digits rebased on the GPU)"}.get(
                         s.get("replay"), "through the pinned double-buffered slots (host copy + time patch, ysb_submit_raw)"),
                     s["speedup"], s["event_rate"] / 1e6,
                     "+-50 ms, no late events" if s["skew"] == 2 else ("+-50 ms and 1e-5 late < 60 s" if s["skew"] else "off"),
                     s["ooo_ms"], s["flush_ms"]),
        "replay": s.get("replay"),
        "events": s["events"], "events_per_s": s["events_per_s"], "target_events_per_s": s["target_events_per_s"],
        "submit_events_per_s": s.get("submit_events_per_s"),
        "per_gpu_events_per_s": round(s["events_per_s"] / s["shards"], 1),
        "per_shard": s.get("per_shard"),
        "wall_s": s["wall_s"], "batches": s["batches"], "copy_GBs": s["copy_GBs"],
        "copy_busy_frac": s["copy_busy_frac"], "slot_waits": s["slot_waits"], "slot_wait_ms": s["slot_wait_ms"],
        "slot_wait_max_ms": s["slot_wait_max_ms"], "max_behind_ms": s["max_behind_ms"],
        "flushes": s["flushes"], "rows_written": s["rows_written"], "redis_commands": commands,
        "ring_advances": s["ring_advances"], "window_ring": window_ring,
        "windows_closed": s["window_close_ms"]["n"],
        "window_close_latency_event_ms": s["window_close_ms"],
        "window_close_latency_wall_ms": s["window_close_wall_ms"],
        "get_stats": {"campaign_windows": len(stats), "closed_windows": len(closed_set),
                      "samples_closed_windows": len(samples),
                      "p50_ms": pct(samples, 50), "p99_ms": pct(samples, 99), "max_ms": max(samples) if samples else None,
                      "p50_wall_ms_after_window_end": None if not samples else round((pct(samples, 50) - 10000) * f, 2),
                      "p99_wall_ms_after_window_end": None if not samples else round((pct(samples, 99) - 10000) * f, 2),
                      "note": "time_updated - window_ms per (campaign, window) read back from Redis as core.clj "
                              "get-stats does (event-time ms, the writer's clock being the replay's); wall = "
                              "(value - 10 000) / speedup"},
        "runner_get_stats_at_close": s["get_stats_ms"],
        "check": {"truth_mismatched_cells": mism, "cells": len(truth), "truth_outside_ring": outside,
                  "check_correct": status, "counted_views": sum(got.values()), "truth_views": sum(truth.values()),
                  "overflow_dropped": s["overflow_dropped"], "parse_errors": s["parse_errors"],
                  "join_misses": s["join_misses"]},
        "exact_vs_generator_truth": mism == 0 and status.get("CORRECT", 0) == len(cc),
        "runner": {k: s[k] for k in ("speedup", "event_rate", "cycle_ms", "flush_ms", "batch_ms", "ooo_ms", "skew",
                                     "lines_per_cycle", "cycles", "partial_lines", "prepare_s", "open_at_end",
                                     "final_watermark_ms")},
    }
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--seconds", type=float, default=12.0)
    ap.add_argument("--event-rate", type=int, default=5_000_000)
    ap.add_argument("--speedup", type=float, default=32.0)
    ap.add_argument("--shards", type=int, default=1)
    ap.add_argument("--slot-mb", type=int, default=256)
    ap.add_argument("--flush-ms", type=int, default=1000)
    ap.add_argument("--batch-ms", type=int, default=100)
    ap.add_argument("--skew", type=int, default=2)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--replay", choices=("mapped", "mapped-raw", "copy"), default="mapped")
    a = ap.parse_args()
    print(json.dumps(stream_native(a.device, a.seconds, a.event_rate, a.speedup, a.shards, a.slot_mb, a.flush_ms,
                                   a.batch_ms, skew=a.skew, threads=a.threads, replay=a.replay)), flush=True)


if __name__ == "__main__":
    main()
