"""One rank of the multi-process rehearsal of configs[4] (run by tests/test_multirank.py):
each rank streams its ad_id shard (its own generator event stream with skew and late
events, core.clj:166-174) through a ShardedStreamingOperator whose watermark is reduced
across ranks with torch.distributed (gloo); the device is the CPU-oracle stand-in of
tests/test_stream.py.  Every rank ticks in lockstep (one tick = 100 ms of event time).

    RANK=r WORLD_SIZE=n MASTER_ADDR=127.0.0.1 MASTER_PORT=p python stream_worker.py OUT.json
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

from oracle import oracle  # noqa: E402
from test_stream import Clock, OracleSlots  # noqa: E402
from ysb_amd import GenParams, shard_ads  # noqa: E402
from ysb_amd.stream import ShardedStreamingOperator  # noqa: E402

NONE = -(1 << 62)


def wm_reduce(wm):
    t = torch.tensor([NONE if wm is None else wm], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    v = int(t.item())
    return None if v == NONE else v


def main():
    out_path = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    base = GenParams(seed=42, n_campaigns=20, ads_per_campaign=10, events_per_sec=1000)
    _, aids = base.ids()
    subset = shard_ads(aids, world)[rank]
    g = GenParams(seed=42, event_stream=1 + rank, n_campaigns=20, ads_per_campaign=10, events_per_sec=1000,
                  ad_subset=subset, with_skew=True, n_users=100, t0_ms=1_700_000_000_000)
    raw, offs = g.events_host(0, 40_000)          # 40 s of event time per rank
    am = oracle.AdMap(aids, base.ad_campaign_index())
    clk = Clock(1_700_000_000_000.0)
    op = ShardedStreamingOperator([OracleSlots(am, cap_bytes=1 << 18, cap_events=400)], clock_ms=clk,
                                  flush_every=10, watermark_reduce=wm_reduce)
    per = 100
    for i in range(0, offs.size, per):
        j = min(offs.size, i + per)
        clk.t = 1_700_000_000_000 + j + 5
        e = offs[j] if j < offs.size else raw.size
        op.append(raw[offs[i]:e], (offs[i:j] - offs[i]).astype(np.uint32))
        op.tick()
    op.close()
    ref, _ = oracle.run(am, raw, offs)
    res = {"rank": rank, "exact": op.totals == ref, "flushes": op.flushes,
           "closed": sorted(b for b, v in op.book.closed.items() if v is not None),
           "latency": op.latency_summary(), "watermark": op.watermark}
    gathered = [None] * world
    dist.all_gather_object(gathered, res)
    dist.destroy_process_group()
    with open(out_path, "w") as f:
        json.dump(gathered if rank == 0 else res, f)


if __name__ == "__main__":
    main()
