"""Diagnostic (not a result): the host-staged leg alone, then after what bench.py does before
it in the same process (torch's context, the headline's 25 GB of HBM segments and launches,
the CPU baseline's 16 oracle threads and its 1 GB device-to-host copy), then once more --
each with the slots' page placement and the submitting thread's node.  Prints one JSON line."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "streaming-benchmarks_amd")]

import bench  # noqa: E402
import bench_dropin  # noqa: E402
import numa_info  # noqa: E402


def brief(r):
    return {k: r[k] for k in ("events_per_s", "h2d_GBs", "copy_busy_frac", "placement")} | {
        "exact": r["check"]["truth_mismatched_cells"] == 0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=30_000_000)
    ap.add_argument("--skip-headline", action="store_true")
    ap.add_argument("--sdma", action="store_true", help="after the headline: DMA-engine / copy-kernel legs interleaved")
    ap.add_argument("--zc", action="store_true", help="after the headline: staged / zero-copy legs interleaved")
    ap.add_argument("--pre", default=None,
                    help="one precondition only, then the offsets leg: torch | segments | pageable | oracle | none")
    a = ap.parse_args()
    if a.pre:
        return pre_only(a)
    out = {"nodes_before": numa_info.node_meminfo()}
    out["fresh"] = brief(bench_dropin.host_staged(0, a.events))
    if not a.skip_headline:
        from ysb_amd import GenParams, YsbContext
        t = time.perf_counter()
        bench.torch_sync(0)
        g = GenParams(seed=42, n_campaigns=100, ads_per_campaign=10, events_per_sec=100_000)
        cids, aids = g.ids()
        camp = g.ad_campaign_index()
        ctx = YsbContext(device=0, n_campaigns=100, window_ring=1024, timing=True, max_batch_bytes=16 << 20,
                         max_batch_events=1 << 16)
        ctx.load_ad_map(aids, camp)
        segs = bench.gen_segments(ctx, g, 100_000_000, 16_666_667)
        sub = [(d_b, nb, d_o, n) for (_, n, d_b, nb, d_o) in segs]
        for _ in range(20):
            ctx.submit_device_segments(sub)
        ctx.sync()
        s0 = segs[0]
        cpu = bench.cpu_baseline(ctx, s0[2], s0[4], s0[3], s0[1], aids, camp, 4_000_000, 10.0)
        bench.free_segments(ctx, segs)
        ctx.close()
        out["headline_like_s"] = round(time.perf_counter() - t, 1)
        out["cpu_baseline_value"] = cpu["value"]
        out["nodes_after_headline"] = numa_info.node_meminfo()
        out["after_headline"] = brief(bench_dropin.host_staged(0, a.events))
    if a.zc:   # staged and zero-copy legs interleaved in the same (slow-prone) period
        import zerocopy_probe
        for k in range(3):
            out["zc_staged_%d" % k] = brief(bench_dropin.host_staged(0, a.events))
            out["zc_zero_copy_%d" % k] = zerocopy_probe.zero_copy(a.events)
    if a.sdma:   # the DMA engine and the copy kernel interleaved in the same period
        for k in range(3):
            out["sdma_%d" % k] = brief(bench_dropin.host_staged(0, a.events, h2d_sdma=True))
            out["kernel_%d" % k] = brief(bench_dropin.host_staged(0, a.events))
    out["again"] = brief(bench_dropin.host_staged(0, a.events))
    out["raw_again"] = brief(bench_dropin.host_staged(0, a.events, raw=True))
    print(json.dumps(out), flush=True)


def pre_only(a):
    """One of the headline phase's parts in a fresh process, then the offsets leg (and the raw
    leg): which part leaves the offsets path's copies slow."""
    import numpy as np
    from ysb_amd import GenParams, YsbContext
    out = {"pre": a.pre}
    g = GenParams(seed=42, n_campaigns=100, ads_per_campaign=10, events_per_sec=100_000)
    cids, aids = g.ids()
    camp = g.ad_campaign_index()
    t = time.perf_counter()
    if a.pre == "torch":
        bench.torch_sync(0)
    elif a.pre in ("segments", "pageable"):
        with YsbContext(device=0, n_campaigns=100, window_ring=1024, timing=True, max_batch_bytes=16 << 20,
                        max_batch_events=1 << 16) as ctx:
            ctx.load_ad_map(aids, camp)
            n = 16_666_667 if a.pre == "segments" else 4_000_000
            segs = bench.gen_segments(ctx, g, 100_000_000 if a.pre == "segments" else n, n)
            if a.pre == "segments":
                sub = [(d_b, nb, d_o, m) for (_, m, d_b, nb, d_o) in segs]
                for _ in range(20):
                    ctx.submit_device_segments(sub)
                ctx.sync()
            else:   # cpu_baseline's reads: offsets and ~1 GB of bytes into pageable numpy arrays
                s0 = segs[0]
                off = ctx.d2h(np.empty(s0[1], dtype=np.uint32), s0[4])
                data = ctx.d2h(np.empty(s0[3], dtype=np.uint8), s0[2])
                out["pageable_bytes"] = int(data.size + 4 * off.size)
                del data, off
            bench.free_segments(ctx, segs)
    elif a.pre == "oracle":
        from oracle import oracle
        raw, offs = g.events_host(0, 2_000_000)
        am = oracle.AdMap(aids, camp)
        t1 = time.perf_counter()
        while time.perf_counter() - t1 < 8:
            oracle.run(am, raw.tobytes(), offs, threads=16)
    out["pre_s"] = round(time.perf_counter() - t, 1)
    out["offsets"] = brief(bench_dropin.host_staged(0, a.events))
    out["raw"] = brief(bench_dropin.host_staged(0, a.events, raw=True))
    out["offsets_again"] = brief(bench_dropin.host_staged(0, a.events))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
