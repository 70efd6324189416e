"""One rank of the CPU rehearsal of the multi-GPU path (run by tests/test_multirank.py).

The GPU path (bench.py --gpus N, libysb_hip.so) is: events sharded by ad_id hash ->
each rank counts its shard into a campaign-major [C_pad][W] (campaign, bucket mod W)
table -> one reduce-scatter (sum) -> rank r owns campaigns owned_block(C, r, N) ->
each owner drains its rows.  Here the per-rank count comes from the CPU oracle (test
infrastructure) and the collective is torch.distributed's gloo reduce_scatter_tensor,
which has ncclReduceScatter's semantics; routing, ownership and the table layout are
the library's own host functions.

    RANK=r WORLD_SIZE=n MASTER_ADDR=127.0.0.1 MASTER_PORT=p python multirank_worker.py SCENARIO OUT.json
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "streaming-benchmarks_amd"), HERE):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import golden_data as gd  # noqa: E402
from oracle import oracle  # noqa: E402
from ysb_amd import (GenParams, exchange_mismatches, owned_block, ring_agreement, route_lines,  # noqa: E402
                     shard_ads, split_batch, table_rows)

W = 64   # ring width (power of two), like ysb_config.window_ring


def table_of(rows, c_pad, ring_lo):
    """Dense campaign-major table, cell (c, b & (W-1)), as the device ring lays it out."""
    t = torch.zeros(c_pad * W, dtype=torch.int64)
    for (c, b), n in rows.items():
        assert ring_lo <= b < ring_lo + W, "bucket outside the ring"
        t[c * W + (b & (W - 1))] += n
    return t


def rows_of_block(block, lo, ring_lo):
    """The owner's drain of its block (the library's table layout: ysb_amd.table_rows)."""
    return table_rows(block.numpy().reshape(-1, W), ring_lo, c_off=lo)


def main():
    scenario, out_path = sys.argv[1], sys.argv[2]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {"rank": rank}

    if scenario == "route":
        # a fixture batch routed by the host router (batches that are not pre-sharded)
        ads, camp = gd.ad_arrays()
        n_campaigns = len(gd.campaigns())
        raw, offs = gd.events("gen_s7")
        shard, counts = route_lines(np.frombuffer(raw, dtype=np.uint8), offs, world)
        mine_raw, mine_off = split_batch(np.frombuffer(raw, dtype=np.uint8), offs, shard, rank)
        rows, st = oracle.run(oracle.AdMap(ads, camp), mine_raw.tobytes(), mine_off)
        res["lines"] = int(mine_off.size)
        res["shard_counts"] = [int(x) for x in counts]
    elif scenario == "gen":
        # per-rank generation from the rank's ad shard (bench.py's N > 1 workload)
        base = GenParams(seed=42, n_campaigns=20, ads_per_campaign=10, events_per_sec=1000)
        _, aids = base.ids()
        n_campaigns = 20
        subset = shard_ads(aids, world)[rank]
        g = GenParams(seed=42, event_stream=1 + rank, n_campaigns=20, ads_per_campaign=10, events_per_sec=1000,
                      ad_subset=subset)
        raw, offs = g.events_host(0, 20_000)
        shard, _ = route_lines(raw, offs, world)
        res["all_routed_here"] = bool((shard == rank).all())
        rows, st = oracle.run(oracle.AdMap(aids, base.ad_campaign_index()), raw, offs)
        res["lines"] = int(offs.size)
    elif scenario == "skew":
        # per-rank real-time streams with skew and late events (core.clj:166-174) that start
        # 10 minutes apart: every rank auto-bases its ring differently (first bucket - W/8,
        # ring_autobase_kernel) and rank 1's later buckets fall past the common ring
        base = GenParams(seed=42, n_campaigns=20, ads_per_campaign=10, events_per_sec=1000)
        _, aids = base.ids()
        n_campaigns = 20
        subset = shard_ads(aids, world)[rank]
        g = GenParams(seed=42, event_stream=1 + rank, n_campaigns=20, ads_per_campaign=10, events_per_sec=1000,
                      ad_subset=subset, with_skew=True, n_users=100, t0_ms=1_700_000_000_000 + rank * 600_000)
        raw, offs = g.events_host(0, 20_000)
        rows, st = oracle.run(oracle.AdMap(aids, base.ad_campaign_index()), raw, offs)
        res["lines"] = int(offs.size)
    else:
        raise SystemExit("unknown scenario " + scenario)

    # ring-base agreement (ysb_group_init / the first exchange, ysb_capi.cpp agree_ring):
    # each rank's auto-base is its first bucket - W/8; the common base is the smallest;
    # a rank's rows the common ring cannot hold go to its exact side list (additive deltas)
    my_base = min((b for (_, b) in rows), default=None)
    my_base = None if my_base is None else my_base - W // 8
    bases = [None] * world
    dist.all_gather_object(bases, my_base)
    ring_lo = ring_agreement(bases)
    side = {k: v for k, v in rows.items() if not ring_lo <= k[1] < ring_lo + W}
    in_ring = {k: v for k, v in rows.items() if k not in side}
    c_pad = (n_campaigns + world - 1) // world * world
    table = table_of(in_ring, c_pad, ring_lo)
    block = torch.zeros(c_pad // world * W, dtype=torch.int64)
    dist.reduce_scatter_tensor(block, table)
    lo, hi = owned_block(n_campaigns, rank, world)
    owned = rows_of_block(block, lo, ring_lo)
    assert all(lo <= c < hi for (c, _) in owned)

    # every rank's local rows and owned rows, for rank 0 to check
    gathered = [None] * world
    dist.all_gather_object(gathered, {"local": [[c, b, n] for (c, b), n in rows.items()],
                                      "owned": [[c, b, n] for (c, b), n in owned.items()],
                                      "side": [[c, b, n] for (c, b), n in side.items()],
                                      "block": [lo, hi], "stats": st, "base": my_base})
    if rank == 0:
        res["ranks"] = gathered
        res["ring_lo"] = ring_lo
        # bench.py's post-exchange check: the owners' rows (+ every rank's side deltas, any
        # campaign) against the truth summed over ranks
        expected = {}
        for gi in gathered:
            for c, b, n in gi["local"]:
                expected[(c, b)] = expected.get((c, b), 0) + n
        per = [(gi["block"][0], gi["block"][1], {(c, b): n for c, b, n in gi["owned"]}) for gi in gathered]
        per += [(0, n_campaigns, {(c, b): n for c, b, n in gi["side"]}) for gi in gathered]
        res["exchange"] = list(exchange_mismatches(expected, per))
    dist.barrier()
    dist.destroy_process_group()
    with open(out_path, "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
