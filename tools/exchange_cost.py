"""What the range-limited exchange costs per step, measured on one GPU with a real one-rank
RCCL group (the N-rank collective itself needs a multi-GPU node): the headline workload and
configs[2]'s tables, each stepped without an exchange, with the complete
ysb_group_reduce_scatter every step, and with ysb_group_exchange_pipelined (bench.py's
timed loop: pipelined, the last step complete).

    python tools/exchange_cost.py [--steps 20] [--warmup 5]

Prints one JSON object: per workload the step time without / with the exchange, the
exchange's device time (HIP events around plan, all-reduce(max), read-back, pack,
reduce-scatter, unpack) and bytes per step.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "streaming-benchmarks_amd"))

import bench  # noqa: E402
from ysb_amd import GenParams, YsbContext  # noqa: E402


def measure(ctx, sub, steps, warmup, exchange):
    """exchange: None, "complete" (every step), "pipelined" (as bench.py: pipelined, the
    last step complete)."""
    def step(last=False):
        ctx.submit_device_segments(sub)
        if exchange == "complete" or (exchange == "pipelined" and last):
            ctx.group_reduce_scatter()
        elif exchange == "pipelined":
            ctx.group_exchange_pipelined()
    for _ in range(warmup):
        step()
    ctx.sync()
    ctx.exchange_info(reset=True)
    t0 = time.perf_counter()
    for i in range(steps):
        step(i == steps - 1)
    ctx.sync()
    el = time.perf_counter() - t0
    x = ctx.exchange_info(reset=True)
    return el / steps * 1e3, x


def workload(name, g, n_campaigns, W, events, seg, table, args):
    with YsbContext(n_campaigns=n_campaigns, window_ring=W, timing=True, ring_base_bucket=g.c.t0_ms // 10000 - W // 8,
                    max_batch_bytes=1 << 20, max_batch_events=1 << 12) as ctx:
        table(ctx)
        ctx.group_init(0, 1, YsbContext.group_unique_id())
        segs = bench.gen_segments(ctx, g, events, seg)
        sub = [(d_b, nb, d_o, n) for (_, n, d_b, nb, d_o) in segs]
        plain, _ = measure(ctx, sub, args.steps, args.warmup, None)
        ctx.group_reduce_scatter()
        with_x, x = measure(ctx, sub, args.steps, args.warmup, "complete")
        piped, xp = measure(ctx, sub, args.steps, args.warmup, "pipelined")
        bench.free_segments(ctx, segs)
    return {"workload": name, "ms_per_step_no_exchange": round(plain, 4), "ms_per_step_with_exchange": round(with_x, 4),
            "ms_per_step_with_pipelined_exchange": round(piped, 4),
            "exchange_device_ms_per_step": round(x["ms"] / max(x["exchanges"], 1), 4),
            "pipelined_exchange_device_ms_per_step": round(xp["ms"] / max(xp["exchanges"], 1), 4),
            "exchange_critical_ms_per_step": round(x["critical_ms"] / max(x["exchanges"], 1), 4),
            "pipelined_exchange_critical_ms_per_step": round(xp["critical_ms"] / max(xp["exchanges"], 1), 4),
            "exchange_bytes_per_step": x["bytes"] // max(x["exchanges"], 1), "buckets": x["last_buckets"],
            "cell_bytes": x["last_width"], "whole_ring_u64_bytes": x["full_ring_bytes"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    args = ap.parse_args()
    out = []
    g = GenParams(seed=42, n_campaigns=100, ads_per_campaign=10, events_per_sec=100_000)
    _, aids = g.ids()
    out.append(workload("configs[1]: 100M events, 100 campaigns, W 1024", g, 100, 1024, 100_000_000, 16_666_667,
                        lambda ctx: ctx.load_ad_map(aids, g.ad_campaign_index()), args))
    g3 = GenParams(seed=42, n_campaigns=1_000_000, ads_per_campaign=10, events_per_sec=100_000)
    _, ab = g3.ids_packed()
    out.append(workload("configs[2] tables: 100M events, 1M campaigns x 10 ads, W 128", g3, 1_000_000, 128,
                        100_000_000, 16_666_667, lambda ctx: ctx.load_ad_map_packed(ab, g3.ad_campaign_index_array()),
                        args))
    print(json.dumps({"exchange_cost_one_rank_rccl": out}), flush=True)


if __name__ == "__main__":
    main()
