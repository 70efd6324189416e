"""One rank of the N-rank GPU rehearsal on one MI355X (tests/test_gpu_group_host.py).

RCCL refuses two ranks on one device, so the ranks here run the library's whole group
path -- ring agreement, the range-limited exchange (xplan / all-reduce(max) / plan / xpack /
reduce-scatter / xunpack), owner blocks, checksums -- over ysb_group_init_host with
torch.distributed (gloo) as the transport, each rank a process with its own context on
cuda:0.  Only the transport differs from bench.py --gpus N.

    RANK=r WORLD_SIZE=n MASTER_ADDR=127.0.0.1 MASTER_PORT=p python group_worker.py SCENARIO OUT.json
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "streaming-benchmarks_amd"), HERE):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

from ysb_amd import GenParams, YsbContext, shard_packed  # noqa: E402

M64 = (1 << 64) - 1


def config3(rank, world, res):
    """configs[2]-like tables (200k campaigns x 10 ads, each rank 1/N of the table), record
    mode, three steps with an exchange each, then bench.py's checksum check."""
    C = 200_000
    base = GenParams(seed=42, n_campaigns=C, ads_per_campaign=10, events_per_sec=100_000)
    _, ab = base.ids_packed()
    subset = np.nonzero(shard_packed(ab, world) == rank)[0].astype(np.uint32)
    g = GenParams(seed=42, event_stream=1 + rank, n_campaigns=C, ads_per_campaign=10, events_per_sec=100_000,
                  ad_subset=subset)
    W = 128
    n = 2_000_000
    with YsbContext(device=0, n_campaigns=C, window_ring=W, ring_base_bucket=g.c.t0_ms // 10000 - W // 8,
                    max_batch_bytes=1 << 20, max_batch_events=1 << 12, record_count=True, strict=True) as ctx:
        ctx.load_ad_map_packed(ab, base.ad_campaign_index_array(), shard=(rank, world))
        ctx.group_init_host(rank, world, dist)
        cap = n * g.max_line_bytes()
        d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n + 64)
        nb = ctx.gen_events_device(g, 0, n, d_b, cap, d_o)
        for _ in range(3):
            ctx.submit_device_segments([(d_b, nb, d_o, n)])
            ctx.group_reduce_scatter()
        x = ctx.exchange_info(reset=True)
        res["steps"] = {"exchanges": x["exchanges"], "bytes": x["bytes"], "width": x["last_width"],
                        "buckets": x["last_buckets"], "record_launches": ctx.path_time()[2]}
        # the check (bench.py config3_ranks): one pass, its truth, one exchange, checksums
        ctx.reset()
        ctx.submit_device_segments([(d_b, nb, d_o, n)])
        ctx.truth_accumulate(g, 0, n)
        mism, truth, ring = ctx.truth_compare()
        tsum = ctx.checksum("truth", world)
        ctx.group_reduce_scatter()
        own = ctx.checksum("owned")[0]
        pend = ctx.checksum("pending", world)
        st = ctx.stats()
        owned_total = sum(ctx.drain_buckets().values())
        per = [None] * world
        dist.all_gather_object(per, {"tsum": tsum, "own": own, "pend": pend, "mism": mism, "truth": truth,
                                     "ring": ring, "owned_total": owned_total, "foreign": st["foreign_shard"],
                                     "misses": st["join_misses"], "ranks": ctx.group_info()})
    if rank == 0:
        res["blocks_mismatched"] = sum(
            (sum(p["tsum"][r] for p in per) & M64) != ((per[r]["own"] + sum(p["pend"][r] for p in per)) & M64)
            for r in range(world))
        res["per_rank"] = per


def pipelined(rank, world, res):
    """ysb_group_exchange_pipelined: a step whose counts outgrow the previous plan's width
    (held back by the cap) and fill buckets outside it (held back by the plan), then steps
    that catch up, then a complete exchange.  After every exchange: owned + pending = truth,
    summed over the ranks, per owner block."""
    C = 1000
    base = GenParams(seed=7, n_campaigns=C, ads_per_campaign=10, events_per_sec=100_000)
    _, ab = base.ids_packed()
    subset = np.nonzero(shard_packed(ab, world) == rank)[0].astype(np.uint32)
    g = GenParams(seed=7, event_stream=1 + rank, n_campaigns=C, ads_per_campaign=10, events_per_sec=100_000,
                  ad_subset=subset)
    W = 128
    n = 2_000_000
    # step ranges: 1 s of events (small cells: a 1-byte plan), the next 19 s (cells past
    # the 1-byte cap, a second bucket), nothing new (catch up), the complete exchange
    ranges = [(0, 100_000), (100_000, n), None, None]
    kinds = ["pipelined", "pipelined", "pipelined", "complete"]
    res["log"] = []
    with YsbContext(device=0, n_campaigns=C, window_ring=W, ring_base_bucket=g.c.t0_ms // 10000 - W // 8,
                    max_batch_bytes=1 << 20, max_batch_events=1 << 12, record_count=True, strict=True) as ctx:
        ctx.load_ad_map_packed(ab, base.ad_campaign_index_array(), shard=(rank, world))
        ctx.group_init_host(rank, world, dist)
        segs = {}
        for rg in ranges:
            if rg is not None:
                f, t = rg
                cap = (t - f) * g.max_line_bytes()
                d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * (t - f) + 64)
                segs[rg] = (d_b, ctx.gen_events_device(g, f, t - f, d_b, cap, d_o), d_o, t - f)
        ctx.group_reduce_scatter()   # the first exchange is complete anyway: agree the ring
        for rg, kind in zip(ranges, kinds):
            if rg is not None:
                ctx.submit_device_segments([segs[rg]])
                ctx.truth_accumulate(g, rg[0], rg[1] - rg[0])
            (ctx.group_exchange_pipelined if kind == "pipelined" else ctx.group_reduce_scatter)()
            x = ctx.exchange_info(reset=True)
            tsum = ctx.checksum("truth", world)
            own = ctx.checksum("owned")[0]
            pend = ctx.checksum("pending", world)
            per = [None] * world
            dist.all_gather_object(per, {"tsum": tsum, "own": own, "pend": pend})
            bad = sum((sum(p["tsum"][r] for p in per) & M64) != ((per[r]["own"] + sum(p["pend"][r] for p in per)) & M64)
                      for r in range(world))
            res["log"].append({"kind": kind, "bad_blocks": bad, "pending_nonzero": any(any(p["pend"]) for p in per),
                               "width": x["last_width"], "buckets": x["last_buckets"]})
        # (the local ring is empty now: everything went to the owners)
        _, truth, ring = ctx.truth_compare()
        res["views"] = {"truth": truth, "ring": ring, "owned": sum(ctx.drain_buckets().values())}


def config2(rank, world, res):
    """bench.py's own N > 1 config-2 workload (100 campaigns, LDS window counters, the u64
    ring), run through bench.exchange_check -- owners' rows against the truth summed over
    the ranks."""
    import bench
    base = GenParams(seed=42, n_campaigns=100, ads_per_campaign=10, events_per_sec=100_000)
    _, aids = base.ids()
    from ysb_amd import shard_ads
    g = GenParams(seed=42, event_stream=1 + rank, n_campaigns=100, ads_per_campaign=10, events_per_sec=100_000,
                  ad_subset=shard_ads(aids, world)[rank])
    n = 3_000_000
    with YsbContext(device=0, n_campaigns=100, window_ring=1024, ring_base_bucket=g.c.t0_ms // 10000 - 128,
                    max_batch_bytes=16 << 20, max_batch_events=1 << 16) as ctx:
        ctx.load_ad_map(aids, base.ad_campaign_index(), shard=(rank, world))
        ctx.group_init_host(rank, world, dist)
        cap = n * g.max_line_bytes()
        d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n + 64)
        nb = ctx.gen_events_device(g, 0, n, d_b, cap, d_o)

        def submit_all():
            ctx.submit_device_segments([(d_b, nb, d_o, n)])
        for _ in range(2):
            submit_all()
            ctx.group_reduce_scatter()
        x = ctx.exchange_info(reset=True)
        res["steps"] = {"exchanges": x["exchanges"], "width": x["last_width"], "buckets": x["last_buckets"]}
        os.environ["WORLD_SIZE"] = str(world)
        d = bench.Dist.__new__(bench.Dist)
        d.world, d.rank, d.local, d.device, d.dist = world, rank, rank, 0, dist
        chk = bench.exchange_check(d, ctx, g, [(0, n, d_b, nb, d_o)], submit_all)
    if rank == 0:
        res["check"] = chk


def main():
    scenario, out_path = sys.argv[1], sys.argv[2]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {"rank": rank}
    {"config3": config3, "config2": config2, "pipelined": pipelined}[scenario](rank, world, res)
    dist.barrier()
    dist.destroy_process_group()
    with open(out_path, "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
