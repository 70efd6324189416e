"""Probe (GPU box): can a read-only mapping of a file (the native runner's replay file) be
registered for zero-copy raw batches (ysb_host_register on page-cache pages)?"""
import mmap
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "streaming-benchmarks_amd")]
from ysb_amd import GenParams, YsbContext, YsbError  # noqa: E402

g = GenParams(events_per_sec=100_000)
data, off = g.events_host(0, 200_000)
_, aids = g.ids()
d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR") or "/tmp")
path = os.path.join(d, "events.txt")
with open(path, "wb") as f:
    f.write(bytes(data))
for prot, label in ((mmap.PROT_READ, "read-only shared"), (mmap.PROT_READ | mmap.PROT_WRITE, "private rw")):
    with open(path, "rb") as f:
        flags = mmap.MAP_SHARED if prot == mmap.PROT_READ else mmap.MAP_PRIVATE
        mm = mmap.mmap(f.fileno(), 0, flags=flags, prot=prot)
    arr = np.frombuffer(mm, dtype=np.uint8)
    with YsbContext(n_campaigns=100, window_ring=1024, ring_base_bucket=g.c.t0_ms // 10000 - 8) as ctx:
        ctx.load_ad_map(aids, g.ad_campaign_index())
        try:
            ctx.host_register(arr[: (arr.size // 4096) * 4096])
            ctx.submit_raw_mapped(arr, 0, (arr.size // 4096) * 4096 - 64)
            ctx.sync()
            print(label, "registered, events", ctx.stats()["events"], flush=True)
        except YsbError as e:
            print(label, "FAILED:", e, flush=True)
