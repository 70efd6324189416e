"""Runs one of bench.py's extra legs by itself (profiling passes, A/B runs):
    python tools/extra_one.py config3|config3_compact|config3_reorder|tbl|stream|host_staged|native_runner|
                              generator|reorder|reorder_fixed|reorder_flat|reorder_flat_fixed|compact|mixed|mixed_flat_fixed|
                              mixed_blocks|mixed_blocks_flat_fixed|alternating|stream_native
                              [bench.py options]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def layout(args, variant, **kw):
    from ysb_amd import GenParams, YsbContext
    g = GenParams(seed=42, n_campaigns=100, ads_per_campaign=10, events_per_sec=args.rate, variant=variant)
    _, aids = g.ids()
    with YsbContext(device=0, n_campaigns=100, window_ring=1024, timing=True, max_batch_bytes=16 << 20,
                    max_batch_events=1 << 16, **kw) as ctx:
        ctx.load_ad_map(aids, g.ad_campaign_index())
        segs = bench.gen_segments(ctx, g, args.events, 14_285_715)
        r = bench.timed_extra("layout variant %d %s" % (variant, kw), ctx, g, segs, args.extra_steps, args.warmup, None)
        r["kernel"] = "ysb::scan_kernel<false, false, false, %d>" % ctx.launch_info()["layout"]
        bench.free_segments(ctx, segs)
    return r


if __name__ == "__main__":
    leg = sys.argv[1]
    args = bench.parse_args(sys.argv[2:])
    from ysb_amd import GEN_COMPACT, GEN_MIXED, GEN_MIXED_BLOCKS, GEN_REORDER
    fn = {"config3": lambda: bench.extra_config3(args, 0), "tbl": lambda: bench.extra_tbl(args, 0),
          "config3_compact": lambda: bench.extra_config3(args, 0, GEN_COMPACT, "compact"),
          "config3_reorder": lambda: bench.extra_config3(args, 0, GEN_REORDER, "reordered keys"),
          "host_staged": lambda: bench.extra_host_staged(args, 0),
          "native_runner": lambda: bench.extra_native_runner(args, 0, None),
          "generator": lambda: layout(args, 0),
          "mixed": lambda: layout(args, GEN_MIXED),
          "mixed_blocks": lambda: layout(args, GEN_MIXED_BLOCKS),
          "mixed_blocks_flat_fixed": lambda: layout(args, GEN_MIXED_BLOCKS, flat_first=True, layout_auto=False),
          "mixed_flat_fixed": lambda: layout(args, GEN_MIXED, flat_first=True, layout_auto=False),
          "stream": lambda: bench.extra_stream(args),
          "reorder": lambda: layout(args, GEN_REORDER),
          "reorder_fixed": lambda: layout(args, GEN_REORDER, layout_auto=False),
          "reorder_flat": lambda: layout(args, GEN_REORDER, flat_first=True),
          "reorder_flat_fixed": lambda: layout(args, GEN_REORDER, flat_first=True, layout_auto=False),
          "compact": lambda: layout(args, GEN_COMPACT),
          "alternating": lambda: bench.extra_alternating(args, 0),
          "stream_native": lambda: bench.extra_stream_native(args, 0)}[leg]
    print(json.dumps(fn()), flush=True)
