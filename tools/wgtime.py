"""Diagnostic: per-workgroup start / end times of one scan launch (YSB_WGTIME build),
to see how much of a launch is its tail.  Never used for results.

    YSB_LIB_VARIANT=wgtime python tools/wgtime.py [events] [segments]   (on the GPU box)

segments > 1: that many batches of `events` each, in one ysb_submit_device_segments launch.
"""
import ctypes as C
import os
import sys

os.environ.setdefault("YSB_LIB_VARIANT", "wgtime")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "streaming-benchmarks_amd"))

import numpy as np  # noqa: E402

from ysb_amd import GenParams, YsbContext  # noqa: E402
from ysb_amd._lib import lib  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16_666_667
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    g = GenParams(seed=42, events_per_sec=100_000)
    _, aids = g.ids()
    ctx = YsbContext(n_campaigns=100)
    ctx.load_ad_map(aids, g.ad_campaign_index())
    cap = n * g.max_line_bytes()
    segs = []
    for i in range(k):
        d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n)
        nb = ctx.gen_events_device(g, i * n, n, d_b, cap, d_o)
        segs.append((d_b, nb, d_o, n))
    L = lib()
    L.ysb_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
    for rep in range(4):
        ctx.submit_device_segments(segs)
        ctx.sync()
        cnt = C.c_uint64()
        L.ysb_debug_stamps(ctx._h, None, 0, C.byref(cnt))
        buf = np.zeros(cnt.value, dtype=np.uint64)
        L.ysb_debug_stamps(ctx._h, C.c_void_p(buf.ctypes.data), cnt.value, C.byref(cnt))
        if rep == 0:
            continue
        w = buf.reshape(-1, 8)
        w = w[w[:, 1] > 0]
        t0, t1, tiles = w[:, 0].astype(np.int64), w[:, 1].astype(np.int64), w[:, 2]
        base = t0.min()
        s, e = (t0 - base) / 100.0, (t1 - base) / 100.0          # microseconds (100 MHz clock)
        d = e - s
        xcd = np.arange(len(w)) % 8
        print("rep %d: %d workgroups, tiles/wg %d..%d" % (rep, len(w), tiles.min(), tiles.max()))
        print("  start: max %.1f us; end: min %.1f mean %.1f p99 %.1f max %.1f us" %
              (s.max(), e.min(), e.mean(), np.percentile(e, 99), e.max()))
        print("  duration: mean %.1f sd %.1f min %.1f max %.1f us" % (d.mean(), d.std(), d.min(), d.max()))
        print("  mean end by blockIdx %% 8: " + " ".join("%.1f" % e[xcd == k].mean() for k in range(8)))
        odd = (np.arange(len(w)) & 1) == 1
        print("  end: odd workgroups (s_setprio 1) mean %.1f max %.1f; even mean %.1f max %.1f us" %
              (e[odd].mean(), e[odd].max(), e[~odd].mean(), e[~odd].max()))
        print("  tail (max end - mean end): %.1f us = %.1f %% of the launch" %
              (e.max() - e.mean(), 100.0 * (e.max() - e.mean()) / e.max()))


if __name__ == "__main__":
    main()
