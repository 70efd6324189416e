"""Probe (GPU box): the copy kernel's PCIe read rate from registered host memory, by kind of
memory and source alignment -- anonymous memory vs a file's page-cache mapping (the native
runner's --io mapped), 16-byte aligned vs shifted batches (launch_h2d_copy vs
launch_h2d_copy_unaligned).  Each batch is one 256 MB ysb_submit_raw_mapped (the GPU splits
its lines; a batch cut mid-line only costs a parse error at each end); the rate is
ysb_copy_time's (copy events on the copy stream).

usage: python tools/probe_mapped_copy.py [--gb 2] [--rounds 3]"""
import argparse
import json
import mmap
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "streaming-benchmarks_amd")]
from ysb_amd import GenParams, YsbContext  # noqa: E402

BATCH = 256 << 20
T0 = time.time()


def log(msg):
    print("[%6.1f s] %s" % (time.time() - T0, msg), file=sys.stderr, flush=True)


def rate(ctx, arr, shift, n_batches):
    ctx.copy_time()
    for i in range(n_batches):
        ctx.submit_raw_mapped(arr, i * BATCH + shift, BATCH - 64, slot=i % 2)
    ctx.sync()
    ms, copies, nbytes = ctx.copy_time()
    return round(nbytes / (ms * 1e-3) / 1e9, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=1.0)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    n_batches = max(2, int(a.gb * 1e9) // BATCH)
    size = n_batches * BATCH
    log("start")
    g = GenParams(events_per_sec=100_000)
    data, _ = g.events_host(0, 1_000_000)
    log("events generated")
    _, aids = g.ids()
    anon = np.empty(size, dtype=np.uint8)
    for p in range(0, size, data.size):
        k = min(data.size, size - p)
        anon[p:p + k] = data[:k]
    d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR") or "/tmp")
    path = os.path.join(d, "events.txt")
    anon.tofile(path)
    with open(path, "rb") as f:
        mm = mmap.mmap(f.fileno(), 0, flags=mmap.MAP_SHARED, prot=mmap.PROT_READ)
    filemap = np.frombuffer(mm, dtype=np.uint8)
    _ = int(filemap[::4096].sum())   # fault the pages in (page cache already holds them)
    log("file written and mapped")
    out = {"batch_bytes": BATCH, "batches": n_batches}
    with YsbContext(n_campaigns=100, window_ring=1024, ring_base_bucket=g.c.t0_ms // 10000 - 8,
                    timing=True) as ctx:
        ctx.load_ad_map(aids, g.ad_campaign_index())
        log("context open")
        for name, arr in (("anonymous", anon), ("file_mapping", filemap)):
            ctx.host_register(arr)
            log("%s registered" % name)
            for shift in (0, 5, 8):
                k = "%s_shift%d_GBs" % (name, shift)
                out[k] = max(rate(ctx, arr, shift, n_batches - 1) for _ in range(a.rounds))
                log("%s %s" % (k, out[k]))
            ctx.host_unregister(arr)
    print(json.dumps(out), flush=True)
    del arr, filemap
    mm.close()
    os.unlink(path)


if __name__ == "__main__":
    main()
