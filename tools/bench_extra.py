"""Measurements of the BASELINE configs that are not bench.py's headline line.

    python tools/bench_extra.py config3 [--events N] [--steps K]
        configs[2]: 1M campaigns / 10M ads (join table and count table in HBM);
        events/s and the scan kernel's algorithmic GB/s, generator-truth check.
    python tools/bench_extra.py tbl [--events N] [--steps K]
        configs[1]'s events as the fork's live .tbl rows (MockWindowedFlatMap,
        AdvertisingTopologyNative.java:197-226), generated in HBM: tbl_scan_kernel's
        events/s and algorithmic GB/s, generator-truth check.
    python tools/bench_extra.py general [--events N] [--steps K]
        the same events re-laid-out so no line is in the generator's layout (no space
        after ':'): every line through the deferred org.json parser (defer_kernel);
        events/s, exact vs the C oracle on the same bytes.
    python tools/bench_extra.py pcie [--batch-mb M] [--seconds S]
        host-staged throughput: pre-staged pinned double-buffered slots -> H2D copy
        stream -> scan kernel (PCIe-inclusive rate; never bench.py's value).
    python tools/bench_extra.py stream_sharded --shards N [--rate R] [--seconds S]
        configs[4] across N contexts (one per GPU; N contexts on one GPU when only one is
        visible): per-shard real-time producers, one global watermark; p99 close latency.
    python tools/bench_extra.py stream [--rate R] [--seconds S]
        configs[4] on one GPU: a real-time producer (generator with skew and late
        events, core.clj:166-204) feeding the streaming operator; p50/p99 window-close
        latency; counts checked exactly against the batch path over the same events.

Each prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "streaming-benchmarks_amd"))

import numpy as np  # noqa: E402

from ysb_amd import GenParams, YsbContext  # noqa: E402

HBM_PEAK_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def submit_segments(ctx, segs, per_batch):
    """The resident batches: one launch over all (default) or one launch per batch."""
    if per_batch:
        for (_, n, d_b, nb, d_o) in segs:
            ctx.submit_device(d_b, nb, d_o, n)
    else:
        ctx.submit_device_segments([(d_b, nb, d_o, n) for (_, n, d_b, nb, d_o) in segs])


def config3(args):
    g = GenParams(seed=42, n_campaigns=args.campaigns, ads_per_campaign=10_000_000 // args.campaigns,
                  events_per_sec=args.c3_rate)
    t = time.perf_counter()
    _, ab = g.ids_packed()
    # 100M events at 100k/s span 1000 s = 100 buckets: a 128-bucket ring holds them all
    ctx = YsbContext(n_campaigns=args.campaigns, window_ring=args.ring, timing=True, max_batch_bytes=1 << 20,
                     max_batch_events=1 << 12)
    ctx.load_ad_map_packed(ab, g.ad_campaign_index_array())
    t_load = time.perf_counter() - t
    segs, first = [], 0
    while first < args.events:
        n = min(args.segment, args.events - first)
        cap = n * g.max_line_bytes()
        d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n + 64)
        nb = ctx.gen_events_device(g, first, n, d_b, cap, d_o)
        segs.append((first, n, d_b, nb, d_o))
        first += n
    total_bytes = sum(s[3] for s in segs)

    def step():
        submit_segments(ctx, segs, args.per_batch)
    for _ in range(args.warmup):   # steady clocks before timing (bench.py)
        step()
    ctx.sync()
    ctx.kernel_time()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.sync()
    el = time.perf_counter() - t0
    kms, launches = ctx.kernel_time()
    pms, _, _ = ctx.path_time()
    ctx.reset()
    submit_segments(ctx, segs, args.per_batch)
    for (f, n, d_b, nb, d_o) in segs:
        ctx.truth_accumulate(g, f, n)
    mism, truth, ring = ctx.truth_compare()
    st = ctx.stats()
    alg = (total_bytes + 4 * args.events) / (len(segs) if args.per_batch else 1)
    ach = alg / (kms / launches * 1e-3) / 1e9
    return {"config": "configs[2]: %d campaigns / 10M ads, %d events, W=%d, %d events/s of event time" % (
                args.campaigns, args.events, args.ring, args.c3_rate),
            "events_per_s": round(args.events * args.steps / el, 1), "ms_per_step": round(el / args.steps * 1e3, 3),
            "batches_per_step": len(segs), "launches_per_step": len(segs) if args.per_batch else 1,
            "scan_avg_launch_ms": round(kms / launches, 4), "path_avg_ms": round(pms / launches, 4),
            "scan_alg_GBs": round(ach, 1),
            "hbm_frac": round(ach / HBM_PEAK_GBS, 4), "ad_map_load_s": round(t_load, 2),
            "check": {"truth_mismatched_cells": mism, "truth_views": truth, "counted_views": ring,
                      "join_misses": st["join_misses"], "parse_errors": st["parse_errors"],
                      "deferred": st["deferred"], "out_of_ring": st["out_of_ring"],
                      "overflow_dropped": st["overflow_dropped"]}}


def tbl(args):
    g = GenParams(seed=42, n_campaigns=100, ads_per_campaign=10, events_per_sec=100_000, fmt="tbl")
    _, aids = g.ids()
    ctx = YsbContext(n_campaigns=100, window_ring=1024, timing=True, input_format="tbl",
                     max_batch_bytes=16 << 20, max_batch_events=1 << 16)
    ctx.load_ad_map(aids, g.ad_campaign_index())
    segs, first = [], 0
    while first < args.events:
        n = min(args.segment, args.events - first)
        cap = n * g.max_line_bytes()
        d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n + 64)
        nb = ctx.gen_events_device(g, first, n, d_b, cap, d_o)
        segs.append((first, n, d_b, nb, d_o))
        first += n
    total_bytes = sum(s[3] for s in segs)

    def step():
        submit_segments(ctx, segs, args.per_batch)
    for _ in range(args.warmup):   # steady clocks before timing (bench.py)
        step()
    ctx.sync()
    ctx.kernel_time()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.sync()
    el = time.perf_counter() - t0
    kms, launches = ctx.kernel_time()
    pms, _, _ = ctx.path_time()
    ctx.reset()
    submit_segments(ctx, segs, args.per_batch)
    for (f, n, d_b, nb, d_o) in segs:
        ctx.truth_accumulate(g, f, n)
    mism, truth, ring = ctx.truth_compare()
    st = ctx.stats()
    alg = (total_bytes + 4 * args.events) / (len(segs) if args.per_batch else 1)
    ach = alg / (kms / launches * 1e-3) / 1e9
    return {"config": "configs[1] events as .tbl rows: %d events, 100 campaigns x 10 ads" % args.events,
            "tbl_bytes_per_event": round(total_bytes / args.events, 3),
            "events_per_s": round(args.events * args.steps / el, 1), "ms_per_step": round(el / args.steps * 1e3, 3),
            "batches_per_step": len(segs), "launches_per_step": len(segs) if args.per_batch else 1,
            "scan_avg_launch_ms": round(kms / launches, 4), "path_avg_ms": round(pms / launches, 4),
            "scan_alg_GBs": round(ach, 1),
            "hbm_frac": round(ach / HBM_PEAK_GBS, 4),
            "check": {"truth_mismatched_cells": mism, "truth_views": truth, "counted_views": ring,
                      "join_misses": st["join_misses"], "parse_errors": st["parse_errors"],
                      "time_errors": st["time_errors"], "out_of_ring": st["out_of_ring"]}}


def general_host(args, ctx, g, aids, data, offs2, n):
    """The general-path workload as host batches of <= --batch-mb through the pinned slots
    (ysb_submit), so YSB_F_LAYOUT_AUTO can read each batch's first line; the rate is the
    device path's (kernel time), the PCIe copies aside."""
    from oracle import oracle as orc
    ctx.load_ad_map(aids, g.ad_campaign_index())
    cap = args.batch_mb << 20
    batches, i = [], 0
    ends = np.append(offs2[1:].astype(np.int64), len(data))
    while i < n:
        j = int(np.searchsorted(ends, int(offs2[i]) + cap, side="right"))
        j = max(j, i + 1)
        j = min(j, i + ((args.batch_mb << 20) // 200))
        base = int(offs2[i])
        batches.append((data[base:int(ends[j - 1])], (offs2[i:j] - base).astype(np.uint32)))
        i = j

    def step():
        for k, (b, o) in enumerate(batches):
            ctx.submit(b, o, slot=k & 1)
    step()
    ctx.sync()
    ctx.reset()
    ctx.kernel_time()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.sync()
    el = time.perf_counter() - t0
    ctx.kernel_time()
    dev_ms, launches, _ = ctx.path_time()
    ctx.reset()
    step()
    got = ctx.drain_buckets()
    st = ctx.stats()
    rows, ost = orc.run(orc.AdMap(aids, g.ad_campaign_index()), data, offs2.tolist(), threads=8)
    return {"config": "%d generator events, shape %s, layout hint auto, %d host batches" % (n, args.shape, len(batches)),
            "events_per_s_device": round(n * args.steps / (dev_ms * 1e-3), 1),
            "events_per_s_pcie_inclusive": round(n * args.steps / el, 1),
            "device_ms_per_step": round(dev_ms / max(1, args.steps), 3), "launches": launches,
            "deferred": st["deferred"], "exact_vs_oracle": got == rows and all(st[k] == v for k, v in ost.items())}


def general(args):
    from oracle import oracle as orc   # the checker (test infrastructure), not the measured path
    g = GenParams(seed=42, n_campaigns=100, ads_per_campaign=10, events_per_sec=100_000)
    _, aids = g.ids()
    n = min(args.events, 4_000_000)
    raw, offs = g.events_host(0, n)
    data = raw.tobytes()
    if args.shape == "compact":      # '":"': the scan's compact tier takes these
        data = data.replace(b'": "', b'":"')
    elif args.shape == "reorder":    # page_id before user_id: no scan tier, the general path's flat tier
        data = data.replace(b'{"user_id": ', b'{"XXXX_id": ').replace(b', "page_id": ', b', "user_id": ')
        data = data.replace(b'{"XXXX_id": ', b'{"page_id": ')
    elif args.shape == "spaced":     # '" : "': the flat tier too
        data = data.replace(b'": "', b'" : "')
    elif args.shape == "extra":      # a producer's extra field first: the flat tier (one extra key allowed)
        data = data.replace(b'{"user_id": ', b'{"source": "web", "user_id": ')
    elif args.shape == "escaped":    # a \u escape in every key: org.json's full machine
        data = data.replace(b'"ad_id"', b'"ad_\\u0069d"')
    offs2 = np.zeros(n, dtype=np.uint32)
    nl = np.flatnonzero(np.frombuffer(data, dtype=np.uint8) == 0x0A)
    offs2[1:] = (nl[:-1] + 1).astype(np.uint32)
    ctx = YsbContext(n_campaigns=100, window_ring=1024, timing=True, max_batch_bytes=args.batch_mb << 20,
                     max_batch_events=(args.batch_mb << 20) // 200, compact_first=args.hint == "compact",
                     flat_first=args.hint == "flat", layout_auto=args.hint == "auto")
    if args.hint == "auto":   # YSB_F_LAYOUT_AUTO acts on host batches: the pinned slots
        return general_host(args, ctx, g, aids, data, offs2, n)
    ctx.load_ad_map(aids, g.ad_campaign_index())
    d_b, d_o = ctx.device_alloc(len(data) + 64), ctx.device_alloc(4 * n + 64)
    ctx.h2d(d_b, np.frombuffer(data, dtype=np.uint8))
    ctx.h2d(d_o, offs2)
    ctx.submit_device(d_b, len(data), d_o, n)
    ctx.sync()
    ctx.reset()
    ctx.kernel_time()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.submit_device(d_b, len(data), d_o, n)
    ctx.sync()
    el = time.perf_counter() - t0
    ctx.kernel_time()
    dev_ms, launches, _ = ctx.path_time()
    ctx.reset()
    ctx.submit_device(d_b, len(data), d_o, n)
    got = ctx.drain_buckets()
    st = ctx.stats()
    rows, ost = orc.run(orc.AdMap(aids, g.ad_campaign_index()), data, offs2.tolist(), threads=8)
    return {"config": "%d generator events, shape %s, layout hint %s" % (n, args.shape, args.hint),
            "events_per_s": round(n * args.steps / el, 1), "ms_per_step": round(el / args.steps * 1e3, 3),
            "device_ms_per_step": round(dev_ms / max(1, args.steps), 3), "launches": launches,
            "deferred": st["deferred"], "exact_vs_oracle": got == rows and all(st[k] == v for k, v in ost.items())}


def pcie(args):
    g = GenParams(seed=42, events_per_sec=100_000)
    _, aids = g.ids()
    per = int(args.batch_mb * (1 << 20) / g.max_line_bytes())
    ctx = YsbContext(n_campaigns=100, window_ring=1024, max_batch_bytes=args.batch_mb << 20, max_batch_events=per,
                     timing=True)
    ctx.load_ad_map(aids, g.ad_campaign_index())
    from ysb_amd.stream import SlotContext
    sc = SlotContext(ctx)
    sizes = []
    for s in (0, 1):     # stage two distinct batches in the pinned slots once (a replay source)
        raw, offs = g.events_host(s * per, per)
        _, _, bv, ov = sc.slot_views(s)
        bv[:raw.size] = raw
        ov[:per] = offs
        sizes.append(raw.size)
    for s in (0, 1):
        sc.submit_slot(s, sizes[s], per)
    ctx.sync()
    ctx.kernel_time()
    n_sub, t0 = 0, time.perf_counter()
    slot = 0
    while time.perf_counter() - t0 < args.seconds:
        sc.submit_slot(slot, sizes[slot], per)   # waits for the slot's previous H2D inside
        slot ^= 1
        n_sub += 1
    ctx.sync()
    el = time.perf_counter() - t0
    kms, launches = ctx.kernel_time()
    nbytes = sum(sizes[i % 2] for i in range(n_sub))
    return {"config": "host-staged replay: pinned double-buffered slots of %d MB (%d events), H2D + scan" %
            (args.batch_mb, per), "events_per_s": round(n_sub * per / el, 1),
            "h2d_GBs": round((nbytes + 4 * per * n_sub) / el / 1e9, 2), "batches": n_sub,
            "scan_ms_per_batch": round(kms / max(launches, 1), 4),
            "note": "PCIe-inclusive; bench.py's value is the HBM-resident rate"}


def stream(args):
    from ysb_amd.stream import SlotContext, StreamingOperator
    rate = args.rate
    t0_ms = (int(time.time() * 1000) // 10000 + 1) * 10000 - 2000     # 2 s before a window edge
    g = GenParams(seed=7, n_campaigns=100, ads_per_campaign=10, events_per_sec=rate, with_skew=True, n_users=100,
                  t0_ms=t0_ms)
    _, aids = g.ids()
    per_batch = max(1, rate * args.batch_ms // 1000)
    cap_b = per_batch * g.max_line_bytes() * 2
    ctx = YsbContext(n_campaigns=100, window_ring=16, max_batch_bytes=cap_b, max_batch_events=per_batch * 2)
    ctx.load_ad_map(aids, g.ad_campaign_index())
    op = StreamingOperator(SlotContext(ctx), batch_interval_ms=args.batch_ms, flush_interval_ms=1000,
                           max_out_of_orderness_ms=args.ooo_ms)
    n_total = rate * args.seconds
    produced = 0
    behind_max = 0.0
    lat_gen = []
    wall0 = time.time() * 1000.0
    # wall clock starts at the generator's t0 (the real-time emitter's start-time, core.clj:189)
    clock_off = t0_ms - wall0
    op.clock = lambda: time.time() * 1000.0 + clock_off

    def produce(bv, ov, cap_bb, cap_e):
        nonlocal produced
        now_ev = op.clock()
        due = int((now_ev - t0_ms) * rate / 1000)      # events whose emission time has come
        m = min(cap_e, cap_bb // g.max_line_bytes(), max(0, min(due, n_total) - produced))
        if m <= 0:
            return 0, 0
        t = time.perf_counter()
        raw, offs = g.events_host(produced, m)
        lat_gen.append(time.perf_counter() - t)
        bv[:raw.size] = raw
        ov[:m] = offs
        produced += m
        return raw.size, m

    last_log = time.time()
    while produced < n_total:
        if time.time() - last_log > 20:                   # progress (long runs)
            log("stream: %d / %d events, %d batches, %d windows closed" % (produced, n_total, op.batches,
                                                                            op.latency_summary().get("windows", 0)))
            last_log = time.time()
        op.fill_with(produce)
        behind = op.clock() - (t0_ms + produced * 1000.0 / rate)
        behind_max = max(behind_max, behind)
        if op.due() or op.fill_events >= per_batch:
            op.submit()
        else:
            time.sleep(0.002)
    op.close()
    # exactness: the same events through the batch path (device generator, big ring)
    with YsbContext(n_campaigns=100, window_ring=64) as c2:
        c2.load_ad_map(aids, g.ad_campaign_index())
        seg = 10_000_000
        cap = seg * g.max_line_bytes()
        d_b, d_o = c2.device_alloc(cap), c2.device_alloc(4 * seg + 64)
        for f in range(0, n_total, seg):
            m = min(seg, n_total - f)
            nb = c2.gen_events_device(g, f, m, d_b, cap, d_o)
            c2.submit_device(d_b, nb, d_o, m)
            c2.sync()
        ref = c2.drain_buckets()
    lat = op.latency_summary()
    return {"config": "configs[4] on 1 GPU: real-time producer %d events/s for %d s, skew +-50 ms, late p=1e-5 "
                      "(core.clj:166-174); %d ms batches, watermark close" % (rate, args.seconds, args.batch_ms),
            "events": op.events, "batches": op.batches, "flushes": op.flushes, "window_close_latency": lat,
            "batch_interval_ms": args.batch_ms, "max_out_of_orderness_ms": args.ooo_ms,
            "late_rows": op.late_rows, "open_at_end": op.open_at_end,
            "producer_max_behind_ms": round(behind_max, 1),
            "exact_vs_batch_path": op.totals == ref, "rows": len(ref)}


def stream_sharded(args):
    """configs[4] with N shards: N contexts (one per GPU, round robin over the visible
    devices; on a one-GPU box N contexts share it), each fed in real time by its ad_id
    shard's producer (rate / N events per second each), one global watermark.  Producers
    write straight into the pinned slots with --threads host threads each
    (ysb_gen_events_host_mt); a slot that fills before its tick is submitted at once
    (full_submits, back-pressure), and the time spent waiting for a slot's H2D is reported."""
    from ysb_amd import shard_ads
    from ysb_amd.stream import ShardedStreamingOperator, SlotContext
    n = args.shards
    from ysb_amd import device_count
    ndev = max(1, device_count())   # hipGetDeviceCount (torch's count may be 0 where HIP sees GPUs)
    rate = args.rate
    t0_ms = (int(time.time() * 1000) // 10000 + 1) * 10000 - 2000
    base = GenParams(seed=7, n_campaigns=100, ads_per_campaign=10, events_per_sec=rate)
    _, aids = base.ids()
    subsets = shard_ads(aids, n)
    gens = [GenParams(seed=7, event_stream=1 + r, n_campaigns=100, ads_per_campaign=10, events_per_sec=rate // n,
                      ad_subset=subsets[r], with_skew=True, n_users=100, t0_ms=t0_ms) for r in range(n)]
    line = gens[0].max_line_bytes()
    per_batch = max(1, rate // n * args.batch_ms // 1000)
    cap_b = per_batch * line * 2
    ctxs = [YsbContext(device=r % ndev, n_campaigns=100, window_ring=16, max_batch_bytes=cap_b,
                       max_batch_events=per_batch * 2) for r in range(n)]
    for c in ctxs:
        c.load_ad_map(aids, base.ad_campaign_index())
    wall0 = time.time() * 1000.0
    clock_off = t0_ms - wall0
    clock = lambda: time.time() * 1000.0 + clock_off   # noqa: E731
    op = ShardedStreamingOperator([SlotContext(c) for c in ctxs], clock_ms=clock,
                                  flush_every=max(1, 1000 // args.batch_ms), max_out_of_orderness_ms=args.ooo_ms)
    n_total = rate // n * args.seconds
    produced = [0] * n
    threads = max(1, args.threads)
    behind_max = 0.0

    def producer(r):
        def fill(bv, ov, cap_bb, cap_e):
            due = int((clock() - t0_ms) * (rate // n) / 1000)
            m = min(cap_e, cap_bb // line, max(0, min(due, n_total) - produced[r]))
            if m <= 0:
                return 0, 0
            nb = gens[r].write_host(produced[r], m, bv[:cap_bb], ov[:m], threads)
            produced[r] += m
            return nb, m
        return fill
    last_tick = clock()
    last_log = time.time()
    t_start = time.perf_counter()
    while min(produced) < n_total:
        for r in range(n):
            op.fill_with(r, producer(r))
            if op.shards[r].full(line):
                op.shards[r].submit_full()
        behind_max = max(behind_max, clock() - (t0_ms + min(produced) * 1000.0 / (rate // n)))
        if clock() - last_tick >= args.batch_ms:
            op.tick()
            last_tick = clock()
        elif rate < 5_000_000:
            time.sleep(0.001)
        if time.time() - last_log >= 30:   # progress (a long run stays visibly alive)
            last_log = time.time()
            log("stream_sharded: %.0f s, %d events, %d flushes" % (last_log - wall0 / 1000.0, sum(produced),
                                                                    op.flushes))
    op.close()
    el = time.perf_counter() - t_start
    # the reference counts: the generator truth of every event each producer made, straight
    # from the RNG (ysb_truth_accumulate: no bytes, no parsing -- independent of the path
    # under test), in a ring wide enough for the late events (<= 60 s, core.clj:166-174)
    from ysb_amd import table_rows
    ref, outside = {}, 0
    for r in range(n):
        with YsbContext(n_campaigns=100, window_ring=64, ring_base_bucket=t0_ms // 10000 - 8) as c2:
            for f in range(0, produced[r], 100_000_000):
                c2.truth_accumulate(gens[r], f, min(100_000_000, produced[r] - f))
            truth, lo = c2.truth_read()
            _, ttotal, _ = c2.truth_compare()
            outside += ttotal - int(truth.sum())
            for k, v in table_rows(truth, lo).items():
                ref[k] = ref.get(k, 0) + v
    for c in ctxs:
        c.close()
    lat = op.latency_summary()
    return {"config": "configs[4] with %d shards (%d GPU(s) visible): real-time producers, %d events/s in all, "
                      "skew +-50 ms, late p=1e-5 (core.clj:166-174); %d ms ticks, one global watermark; %d s; "
                      "producers: ysb_gen_events_host_mt with %d threads each, straight into the pinned slots"
                      % (n, ndev, rate, args.batch_ms, args.seconds, threads),
            "shards": n, "devices": ndev, "target_events_per_s": rate,
            "sustained_events_per_s": round(op.events / el, 1), "events": op.events, "batches": op.batches,
            "flushes": op.flushes, "window_close_latency": lat, "open_at_end": op.open_at_end,
            "producer_max_behind_ms": round(behind_max, 1), "slot_full_submits": op.full_submits,
            "slot_wait_ms_total": round(op.wait_ms, 1), "slot_wait_max_ms": round(op.wait_max_ms, 2),
            "exact_vs_generator_truth": op.totals == ref and outside == 0, "rows": len(ref),
            "truth_outside_ring": outside}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["config3", "tbl", "general", "pcie", "stream", "stream_sharded"])
    ap.add_argument("--events", type=int, default=100_000_000)
    ap.add_argument("--segment", type=int, default=12_500_000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--per-batch", action="store_true", help="one scan launch per batch (config3 / tbl)")
    ap.add_argument("--batch-mb", type=int, default=64)
    ap.add_argument("--seconds", type=int, default=10)
    ap.add_argument("--rate", type=int, default=1_000_000)
    ap.add_argument("--ring", type=int, default=128)
    ap.add_argument("--campaigns", type=int, default=1_000_000, help="config3: campaigns (10M ads in all)")
    ap.add_argument("--c3-rate", type=int, default=100_000, help="config3: events per second of event time")
    ap.add_argument("--batch-ms", type=int, default=100)
    ap.add_argument("--ooo-ms", type=int, default=100)
    ap.add_argument("--shape", default="reorder", choices=["generator", "compact", "reorder", "spaced", "extra", "escaped"],
                    help="general: how the generator's lines are re-laid")
    ap.add_argument("--shards", type=int, default=2, help="stream_sharded: contexts (one per GPU)")
    ap.add_argument("--threads", type=int, default=16, help="stream_sharded: host threads per producer call")
    ap.add_argument("--hint", default="none", choices=["none", "compact", "flat", "auto"],
                    help="general: layout hint (YSB_F_COMPACT_FIRST / YSB_F_FLAT_FIRST / YSB_F_LAYOUT_AUTO, host batches)")
    args = ap.parse_args()
    out = {"config3": config3, "tbl": tbl, "general": general, "pcie": pcie, "stream": stream,
           "stream_sharded": stream_sharded}[args.mode](args)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
