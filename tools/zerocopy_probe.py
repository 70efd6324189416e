"""Experiment (not a result): the scan reading the pinned slots in place -- device batches
whose pointers are the pinned host buffers (ysb_submit_device on hipHostMalloc memory), so
no SDMA copy runs at all; vs the staged path (ysb_submit).  Prints one JSON line."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "streaming-benchmarks_amd")]
import bench_dropin  # noqa: E402


def zero_copy(events=60_000_000, slot_mb=256):
    from ysb_amd import GenParams, YsbContext
    from ysb_amd.stream import SlotContext
    hip = C.CDLL("/opt/rocm/lib/libamdhip64.so")
    hip.hipHostGetDevicePointer.argtypes = [C.c_void_p, C.c_void_p, C.c_uint]
    g = GenParams(seed=42, events_per_sec=100_000)
    _, aids = g.ids()
    per = int((slot_mb << 20) // g.max_line_bytes())
    with YsbContext(device=0, n_campaigns=100, window_ring=1024, timing=True, max_batch_bytes=slot_mb << 20,
                    max_batch_events=per, ring_base_bucket=g.c.t0_ms // 10000 - 8) as ctx:
        ctx.load_ad_map(aids, g.ad_campaign_index())
        sc = SlotContext(ctx)
        sizes, dptr = [], []
        for s in (0, 1):
            d_b, d_o = ctx.device_alloc(per * g.max_line_bytes()), ctx.device_alloc(4 * per + 64)
            nb = ctx.gen_events_device(g, s * per, per, d_b, per * g.max_line_bytes(), d_o)
            b, o, bv, ov = sc.slot_views(s)
            ctx.d2h(bv[:nb], d_b)
            ctx.d2h(ov[:per], d_o)
            ctx.device_free(d_b)
            ctx.device_free(d_o)
            sizes.append(nb)
            db, do = C.c_void_p(), C.c_void_p()
            assert hip.hipHostGetDevicePointer(C.byref(db), C.c_void_p(b), 0) == 0
            assert hip.hipHostGetDevicePointer(C.byref(do), C.c_void_p(o), 0) == 0
            dptr.append((db.value, do.value))
        for s in (0, 1, 0, 1):
            ctx.submit_device(dptr[s][0], sizes[s], dptr[s][1], per)
        ctx.sync()
        ctx.kernel_time()
        ctx.reset()
        nsub = max(2, -(-events // per))
        t0 = time.perf_counter()
        for i in range(nsub):
            ctx.submit_device(dptr[i & 1][0], sizes[i & 1], dptr[i & 1][1], per)
        ctx.sync()
        el = time.perf_counter() - t0
        kms, launches = ctx.kernel_time()
        for i in range(nsub):
            ctx.truth_accumulate(g, (i & 1) * per, per)
        mism, truth, counted = ctx.truth_compare()
    n = nsub * per
    nbytes = sum(sizes[i & 1] for i in range(nsub))
    return {"events_per_s": round(n / el, 1), "GBs": round((nbytes + 4 * n) / el / 1e9, 2),
            "scan_ms_per_batch": round(kms / max(launches, 1), 3), "exact": mism == 0 and truth == counted}


if __name__ == "__main__":
    out = {}
    for k in range(3):
        out["zero_copy_%d" % k] = zero_copy()
        out["staged_%d" % k] = {x: v for x, v in bench_dropin.host_staged(0, 60_000_000).items()
                                if x in ("events_per_s", "h2d_GBs", "scan_ms_per_batch")}
    print(json.dumps(out), flush=True)
