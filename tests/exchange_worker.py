"""One rank of the CPU rehearsal of the range-limited exchange (run by
tests/test_multirank.py::test_range_limited_exchange_*).

ysb_group_reduce_scatter (streaming-benchmarks_amd/csrc/ysb_capi.cpp) step by step, with
the per-rank counting done by the CPU oracle (test infrastructure) and gloo standing in for
RCCL:

  pending [C_pad][W] u64 (counts since the last exchange, campaign-major ring cells)
  -> slot_max[s] = max over campaigns          (xplan_kernel)
  -> all_reduce(MAX) over the ranks            (ncclAllReduce)
  -> exchange_plan(slot_max, N)                (ysb_exchange_plan: the library's own code)
  -> send = pending[:, slots] as width-byte cells, pending[:, slots] = 0   (xpack_kernel)
  -> reduce_scatter_tensor(block, send)        (ncclReduceScatter, uint8 / uint32 / uint64)
  -> owned[:, slots] += block                  (xunpack_kernel)

Events: configs[2]-like tables (250k campaigns x 2 ads), rank r draws from its ad_id-hash
shard (shard_packed) in its own event stream, two rounds with an exchange after each.

    RANK=r WORLD_SIZE=n MASTER_ADDR=127.0.0.1 MASTER_PORT=p python exchange_worker.py OUT.json [campaigns] [mult]
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
from ysb_amd import GenParams, exchange_mismatches, exchange_plan, owned_block, shard_packed, table_rows  # noqa: E402

W = 64
TORCH_CELL = {1: torch.uint8, 4: torch.int32, 8: torch.int64}   # same bits as uint8 / uint32 / uint64 sums
NP_CELL = {1: np.uint8, 4: np.uint32, 8: np.uint64}


def main():
    out_path = sys.argv[1]
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 250_000
    mult = int(sys.argv[3]) if len(sys.argv) > 3 else 1     # > 1: heavy cells (wider exchange widths)
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    base = GenParams(seed=42, n_campaigns=C, ads_per_campaign=2, events_per_sec=2000)
    _, ab = base.ids_packed()
    aids = [bytes(ab[36 * i:36 * i + 36]).decode() for i in range(base.n_ads)]
    camp = base.ad_campaign_index_array()
    if mult > 1:
        camp = camp % 7     # every view in 7 campaigns: hundreds per cell
    subset = np.nonzero(shard_packed(ab, world) == rank)[0].astype(np.uint32)
    g = GenParams(seed=42, event_stream=1 + rank, n_campaigns=C, ads_per_campaign=2, events_per_sec=2000,
                  ad_subset=subset)
    am = oracle.AdMap(aids, [int(x) for x in camp])
    ring_lo = g.c.t0_ms // 10000 - W // 8
    c_pad = (C + world - 1) // world * world
    per = c_pad // world
    pending = np.zeros((c_pad, W), dtype=np.uint64)
    owned = np.zeros((per, W), dtype=np.uint64)
    local = {}
    rounds = []
    n = 40_000
    for rnd in range(2):
        raw, offs = g.events_host(rnd * n, n)
        rows, st = oracle.run(am, raw, offs)
        for (c, b), v in rows.items():
            assert ring_lo <= b < ring_lo + W
            pending[c, b & (W - 1)] += np.uint64(v)
            local[(c, b)] = local.get((c, b), 0) + v
        # plan: per-slot maxima, all-reduced
        smax = torch.from_numpy(pending.max(axis=0).astype(np.int64))
        dist.all_reduce(smax, op=dist.ReduceOp.MAX)
        slots, width = exchange_plan(smax.numpy().astype(np.uint64), world)
        R = int(slots.size)
        # pack (and zero the pending cells), reduce-scatter, unpack
        send = np.ascontiguousarray(pending[:, slots].astype(NP_CELL[width]))
        pending[:, slots] = 0
        block = torch.zeros(per * R, dtype=TORCH_CELL[width])
        bits = {1: np.uint8, 4: np.int32, 8: np.int64}[width]   # the same bits, a gloo-summable type
        dist.reduce_scatter_tensor(block, torch.from_numpy(send.reshape(-1).view(bits)))
        got = block.numpy().view(NP_CELL[width]).reshape(per, R).astype(np.uint64)
        owned[:, slots] += got
        rounds.append({"buckets": R, "width": width, "bytes": int(c_pad * R * width),
                       "views": int(st["joined"]), "pending_left": int(pending.sum())})
    lo, hi = owned_block(C, rank, world)
    owned_rows = table_rows(owned, ring_lo, c_off=rank * per)
    gathered = [None] * world
    dist.all_gather_object(gathered, {"local": [[c, b, v] for (c, b), v in local.items()],
                                      "owned": [[c, b, v] for (c, b), v in owned_rows.items()],
                                      "block": [lo, hi], "rounds": rounds})
    res = {"rank": rank, "rounds": rounds}
    if rank == 0:
        expected = {}
        for gi in gathered:
            for c, b, v in gi["local"]:
                expected[(c, b)] = expected.get((c, b), 0) + v
        per_rank = [(gi["block"][0], gi["block"][1], {(c, b): v for c, b, v in gi["owned"]}) for gi in gathered]
        res["exchange"] = list(exchange_mismatches(expected, per_rank))
        res["ranks_rounds"] = [gi["rounds"] for gi in gathered]
        res["full_ring_bytes"] = int(c_pad * W * 8)
    dist.barrier()
    dist.destroy_process_group()
    with open(out_path, "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
