"""The drop-in path, timed: host batches through the pinned double-buffered slots
(AdvertisingTopologyNative.java:111-119, FileBasedDataSource.run :144-165), each with a
generator-truth check.  bench.py puts both results in its line (extras.host_staged,
extras.native_runner); `python tools/bench_dropin.py staged|runner` runs one alone.

host_staged: two distinct ~256 MB batches of configs[1]'s events staged once in the
library's pinned slots and resubmitted alternately (a replay source with no host
production cost) until --events events went through H2D + scan: once with host-built
line offsets (ysb_submit) and once as raw lines with the line split on the GPU
(ysb_submit_raw).  Reports events/s, the H2D rate (bytes / copy-engine time, HIP events
on the copy stream) against PCIe Gen5 x16, and how much of the scan time hid under the
copies.

native_runner: bin/ysb_topology (the C++ drop-in for `flink run ... --confPath`) over a
replay file of configs[1]'s events in the box's page cache, read --repeat times, raw lines
(GPU split) and, for comparison, host-split offsets; its CSV sink is compared with the
generator truth times the repeats.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "streaming-benchmarks_amd"))

import numpy as np  # noqa: E402

PCIE_GEN5_X16_GBS = 63.0   # 32 GT/s x 16 lanes x 128/130 / 8, one direction
RUNNER = os.path.join(ROOT, "streaming-benchmarks_amd", "bin", "ysb_topology")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_staged(device=0, events=100_000_000, slot_mb=256, raw=False, rate=100_000, h2d_sdma=False):
    from ysb_amd import GenParams, YsbContext
    from ysb_amd.stream import SlotContext
    g = GenParams(seed=42, events_per_sec=rate)
    _, aids = g.ids()
    per = int((slot_mb << 20) // g.max_line_bytes())
    with YsbContext(device=device, n_campaigns=100, window_ring=1024, timing=True, max_batch_bytes=slot_mb << 20,
                    max_batch_events=per, ring_base_bucket=g.c.t0_ms // 10000 - 8, h2d_sdma=h2d_sdma) as ctx:
        ctx.load_ad_map(aids, g.ad_campaign_index())
        sc = SlotContext(ctx)
        sizes = []
        for s in (0, 1):   # two distinct batches, generated on the device, staged once
            d_b, d_o = ctx.device_alloc(per * g.max_line_bytes()), ctx.device_alloc(4 * per + 64)
            nb = ctx.gen_events_device(g, s * per, per, d_b, per * g.max_line_bytes(), d_o)
            _, _, bv, ov = sc.slot_views(s)
            ctx.d2h(bv[:nb], d_b)
            ctx.d2h(ov[:per], d_o)
            ctx.device_free(d_b)
            ctx.device_free(d_o)
            sizes.append(nb)
        addr = [sc.slot_views(s)[0] for s in (0, 1)]
        import numa_info
        where = {"gpu": numa_info.gpu_node(device), "slot0": numa_info.placement(addr[0], sizes[0]),
                 "slot1_pages_by_node": numa_info.page_nodes(addr[1], sizes[1])}

        def submit(s):
            if raw:
                import ctypes as C
                from ysb_amd._lib import check, lib
                check(lib().ysb_submit_raw(ctx._h, s, C.c_void_p(addr[s]), sizes[s]), ctx._h)
            else:
                sc.submit_slot(s, sizes[s], per)
        for s in (0, 1, 0, 1):   # warmup
            submit(s)
        ctx.sync()
        ctx.kernel_time()
        ctx.copy_time()
        ctx.reset()
        nsub = max(2, -(-events // per))
        t0 = time.perf_counter()
        for i in range(nsub):
            submit(i & 1)   # waits for the slot's previous H2D inside
        ctx.sync()
        el = time.perf_counter() - t0
        kms, launches = ctx.kernel_time()
        cms, copies, cbytes = ctx.copy_time()
        st = ctx.stats()
        for i in range(nsub):
            ctx.truth_accumulate(g, (i & 1) * per, per)
        mism, truth, counted = ctx.truth_compare()
    n = nsub * per
    nbytes = sum(sizes[i & 1] for i in range(nsub))
    h2d = cbytes / (cms * 1e-3) / 1e9 if cms else 0.0
    return {"path": "ysb_submit_raw (line starts found on the GPU)" if raw else
            "ysb_submit (host line offsets)",
            "events": n, "batches": nsub, "events_per_batch": per, "slot_MB": slot_mb,
            "events_per_s": round(n / el, 1), "wall_GBs": round(cbytes / el / 1e9, 2),
            "h2d_GBs": round(h2d, 2), "pcie_peak_GBs": PCIE_GEN5_X16_GBS,
            "h2d_frac_of_pcie": round(h2d / PCIE_GEN5_X16_GBS, 4),
            "h2d_ms_per_batch": round(cms / max(copies, 1), 4),
            "scan_ms_per_batch": round(kms / max(launches, 1), 4),
            "copy_busy_frac": round(cms * 1e-3 / el, 4),
            "scan_hidden_frac": round(1.0 - max(0.0, el * 1e3 - cms) / max(kms, 1e-9), 4),
            "json_bytes_per_event": round(nbytes / n, 3), "placement": where,
            "check": {"truth_mismatched_cells": mism, "truth_views": truth, "counted_views": counted,
                      "events": st["events"], "parse_errors": st["parse_errors"], "join_misses": st["join_misses"],
                      "deferred": st["deferred"]},
            "note": "PCIe-inclusive; the bench line's value is the HBM-resident rate. h2d_GBs = copy bytes / "
                    "copy-engine time (HIP events on the copy stream); copy_busy_frac = copy time / wall; "
                    "scan_hidden_frac = share of the scan time that ran under the copies"}


def write_replay(device, path, n, seg=10_000_000, rate=100_000):
    """configs[1]'s first n events as a replay file (the data/ generator's kafka-json.txt
    format), generated on the GPU and written in segments; the map as ad-to-campaign.csv."""
    from ysb_amd import GenParams, YsbContext
    g = GenParams(seed=42, events_per_sec=rate)
    cids, aids = g.ids()
    camp = g.ad_campaign_index()
    with open(os.path.join(path, "ad-to-campaign.csv"), "w") as f:
        for a, c in zip(aids, camp):
            f.write("%s,%s\n" % (a, cids[c]))
    total = 0
    with YsbContext(device=device) as ctx, open(os.path.join(path, "kafka-json.txt"), "wb") as f:
        cap = seg * g.max_line_bytes()
        d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * seg + 64)
        host = np.empty(cap, dtype=np.uint8)
        for first in range(0, n, seg):
            m = min(seg, n - first)
            nb = ctx.gen_events_device(g, first, m, d_b, cap, d_o)
            ctx.d2h(host[:nb], d_b)
            f.write(host[:nb].data)
            total += nb
        ctx.device_free(d_b)
        ctx.device_free(d_o)
    with open(os.path.join(path, "conf.yaml"), "w") as f:
        f.write("ad_to_campaign_path: %s\nevents_path: %s\n" % (os.path.join(path, "ad-to-campaign.csv"),
                                                                os.path.join(path, "kafka-json.txt")))
    return g, cids, total


def truth_rows(device, g, n, cids, repeat):
    """{(campaign uuid, window_ms): count} of the generator truth of events [0, n), x repeat."""
    from ysb_amd import YsbContext
    from ysb_amd.group import table_rows
    with YsbContext(device=device, n_campaigns=100, window_ring=64,
                    ring_base_bucket=g.c.t0_ms // 10000 - 8) as ctx:
        for first in range(0, n, 50_000_000):
            ctx.truth_accumulate(g, first, min(50_000_000, n - first))
        t, lo = ctx.truth_read()
        _, ttotal, _ = ctx.truth_compare()
        outside = ttotal - int(t.sum())
    return {(cids[c], b * 10000): v * repeat for (c, b), v in table_rows(t, lo).items()}, outside


def native_runner(device=0, file_events=20_000_000, repeat=5, slot_mb=256, host_split=False, workdir=None,
                  keep=None, io="mmap", h2d_sdma=False):
    made = workdir is None
    path = workdir or tempfile.mkdtemp(prefix="ysb_replay_", dir=os.environ.get("TMPDIR") or "/tmp")
    try:
        if not os.path.exists(os.path.join(path, "conf.yaml")):
            t = time.perf_counter()
            write_replay(device, path, file_events)
            log("native_runner: replay file of %d events written in %.1f s" % (file_events,
                                                                               time.perf_counter() - t))
        from ysb_amd import GenParams
        g = GenParams(seed=42, events_per_sec=100_000)
        cids, _ = g.ids()
        out_csv = os.path.join(path, "out.csv")
        cmd = [RUNNER, "--confPath", os.path.join(path, "conf.yaml"), "--device", str(device), "--sink",
               "csv:" + out_csv, "--batch-mb", str(slot_mb), "--repeat", str(repeat), "--io", io]
        if host_split:
            cmd += ["--host-split", "--batch-events", str((slot_mb << 20) // 200)]
        if h2d_sdma:
            cmd += ["--h2d-sdma"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            raise RuntimeError("ysb_topology exited %d: %s" % (r.returncode, r.stderr[-2000:]))
        summary = json.loads(r.stdout.strip().splitlines()[-1])
        got = {}
        with open(out_csv) as f:
            next(f)
            for ln in f:
                c, w, n = ln.rstrip("\n").split(",")
                got[(c, int(w))] = int(n)
        want, outside = truth_rows(device, g, file_events, cids, repeat)
        mism = sum(1 for k in set(got) | set(want) if got.get(k, 0) != want.get(k, 0))
        summary.update({"io": io, "file_events": file_events, "file_GB": round(os.path.getsize(
            os.path.join(path, "kafka-json.txt")) / 1e9, 3),
            "check": {"truth_mismatched_cells": mism, "cells": len(want), "truth_outside_ring": outside,
                      "counted_views": sum(got.values()), "truth_views": sum(want.values())}})
        return summary
    finally:
        if made and not keep:
            shutil.rmtree(path, ignore_errors=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["staged", "runner"])
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--events", type=int, default=100_000_000)
    ap.add_argument("--slot-mb", type=int, default=256)
    ap.add_argument("--raw", action="store_true")
    ap.add_argument("--file-events", type=int, default=20_000_000)
    ap.add_argument("--repeat", type=int, default=5)
    ap.add_argument("--host-split", action="store_true")
    ap.add_argument("--io", default="mmap", choices=["auto", "mapped", "mmap", "pread"])
    ap.add_argument("--h2d-sdma", action="store_true", help="the slots' H2D by the DMA engine (default: a copy kernel)")
    ap.add_argument("--workdir", default=None, help="runner: keep / reuse the replay file here")
    a = ap.parse_args()
    if a.mode == "staged":
        out = host_staged(a.device, a.events, a.slot_mb, a.raw, h2d_sdma=a.h2d_sdma)
    else:
        if a.workdir:
            os.makedirs(a.workdir, exist_ok=True)
        out = native_runner(a.device, a.file_events, a.repeat, a.slot_mb, a.host_split, workdir=a.workdir, io=a.io,
                            h2d_sdma=a.h2d_sdma)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
