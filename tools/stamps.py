"""Diagnostic: per-phase cycle shares of the scan kernel from the YSB_STAMPS build.

    YSB_LIB_VARIANT=stamps python tools/stamps.py      (on the GPU box)

Never used for results: the stamp build's fences change overlap, so only the
SHARES are meaningful (cdna_hip_programming.md section 7, "In-kernel stamps").
"""
import ctypes as C
import os
import sys

os.environ.setdefault("YSB_LIB_VARIANT", "stamps")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "streaming-benchmarks_amd"))

import numpy as np  # noqa: E402

from ysb_amd import GenParams, YsbContext  # noqa: E402
from ysb_amd._lib import lib  # noqa: E402

PHASES = ["A: regs->LDS + classify", "barrier after A", "B1: canonical parse, probe issue, defer",
          "prefetch issue + B2 (probe wait)", "count", "end barrier", "wait for the prefetched tile"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_000
    g = GenParams(seed=42, events_per_sec=100_000)
    cids, aids = g.ids()
    ctx = YsbContext(n_campaigns=100)
    ctx.load_ad_map(aids, g.ad_campaign_index())
    cap = n * g.max_line_bytes()
    d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n)
    nb = ctx.gen_events_device(g, 0, n, d_b, cap, d_o)
    L = lib()
    L.ysb_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
    for rep in range(3):
        ctx.submit_device(d_b, nb, d_o, n)
        ctx.sync()
        cnt = C.c_uint64()
        L.ysb_debug_stamps(ctx._h, None, 0, C.byref(cnt))
        buf = np.zeros(cnt.value, dtype=np.uint64)
        L.ysb_debug_stamps(ctx._h, buf.ctypes.data, buf.size, C.byref(cnt))
        w = buf.reshape(-1, 8)
        w = w[w[:, 7] > 0]
        tot = w[:, :7].sum(axis=0).astype(float)
        tiles = w[:, 7].sum()
        print("rep %d: %d waves, %.0f tiles/wave; cycles per tile per wave:" % (rep, len(w), tiles / len(w)))
        for i, name in enumerate(PHASES):
            print("   %-48s %8.0f  %5.1f%%" % (name, tot[i] / tiles, 100 * tot[i] / tot.sum()))
    print(ctx.stats())


if __name__ == "__main__":
    main()
