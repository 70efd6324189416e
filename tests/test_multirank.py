"""CPU (gloo, world_size 2 and 3) rehearsal of the multi-GPU path: ad_id-hash routing,
the campaign-major (campaign, window) tables, one reduce-scatter, owner blocks.
The per-rank counting is the CPU oracle; what is under test is the partitioning and
exchange logic the GPU path shares (libysb_hip.so host functions + the collective's
semantics).  See tests/multirank_worker.py."""
import json
import os
import socket
import subprocess
import sys
from collections import Counter

import pytest

import golden_data as gd
from oracle import oracle
from ysb_amd import GenParams, owned_block, route_lines, split_batch

HERE = os.path.dirname(os.path.abspath(__file__))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_ranks(scenario, world, tmp_path, worker="multirank_worker.py"):
    port = free_port()
    procs, outs = [], []
    for r in range(world):
        out = tmp_path / ("rank%d.json" % r)
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1")
        args = [scenario, str(out)] if scenario else [str(out)]
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, worker)] + args,
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
        outs.append(out)
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=240)[0].decode(errors="replace"))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    for p, lg in zip(procs, logs):
        assert p.returncode == 0, lg[-3000:]
    return [json.load(open(o)) for o in outs]


def merged(rank_infos, key):
    tot = Counter()
    for info in rank_infos:
        for c, b, n in info[key]:
            tot[(c, b)] += n
    return dict(tot)


@pytest.mark.parametrize("world", [2, 3])
def test_routed_fixture_reduce_scatter_equals_oracle(world, tmp_path):
    res = run_ranks("route", world, tmp_path)
    infos = res[0]["ranks"]
    exp_rows, exp_st = gd.expected("gen_s7")
    # every line went to exactly one rank
    raw, offs = gd.events("gen_s7")
    assert sum(r["lines"] for r in res) == len(offs)
    assert sum(res[0]["shard_counts"]) == len(offs)
    # the owners' rows after the exchange are exactly the single-process oracle's
    assert merged(infos, "owned") == exp_rows
    # and so is the plain sum of the per-rank tables (the exchange loses nothing)
    assert merged(infos, "local") == exp_rows
    for k in ("events", "views", "joined", "join_misses", "parse_errors"):
        assert sum(i["stats"][k] for i in infos) == exp_st[k], k
    # owner blocks tile [0, C)
    blocks = sorted(tuple(i["block"]) for i in infos)
    assert blocks[0][0] == 0 and blocks[-1][1] == len(gd.campaigns())
    assert all(a[1] == b[0] for a, b in zip(blocks, blocks[1:]))


def test_per_rank_generation_reduce_scatter(tmp_path):
    res = run_ranks("gen", 2, tmp_path)
    assert all(r["all_routed_here"] for r in res)   # generator shards == router shards
    infos = res[0]["ranks"]
    # every rank's event stream draws the shared ad ids: no join misses anywhere
    assert all(i["stats"]["join_misses"] == 0 and i["stats"]["joined"] > 0 for i in infos)
    assert merged(infos, "owned") == merged(infos, "local")
    assert sum(sum(n for _, _, n in i["owned"]) for i in infos) == sum(i["stats"]["joined"] for i in infos)


@pytest.mark.parametrize("scenario,world", [("route", 2), ("gen", 3), ("skew", 2), ("skew", 3)])
def test_post_exchange_check(scenario, world, tmp_path):
    """bench.py's N > 1 check (ysb_amd.exchange_mismatches): the owners' rows after the
    reduce-scatter equal the truth summed over ranks, none outside its block."""
    res = run_ranks(scenario, world, tmp_path)
    mism, outside, cells = res[0]["exchange"]
    assert mism == 0 and outside == 0 and cells > 0


def test_skewed_ranks_agree_on_a_ring_base(tmp_path):
    """Per-rank skewed streams auto-base differently; the agreement takes the smallest base
    and the rows past the common ring travel as side deltas -- nothing is lost."""
    res = run_ranks("skew", 2, tmp_path)
    infos = res[0]["ranks"]
    assert len(set(i["base"] for i in infos)) == 2           # the ranks disagreed ...
    assert res[0]["ring_lo"] == min(i["base"] for i in infos)
    assert sum(len(i["side"]) for i in infos) > 0            # ... and rank 1's late buckets moved out
    tot = Counter()
    for i in infos:
        for c, b, n in i["owned"] + i["side"]:
            tot[(c, b)] += n
    assert dict(tot) == merged(infos, "local")


def test_exchange_mismatches_detects_errors():
    from ysb_amd import exchange_mismatches
    exp = {(0, 5): 3, (1, 5): 2, (3, 6): 1}
    ok = [(0, 2, {(0, 5): 3, (1, 5): 2}), (2, 4, {(3, 6): 1})]
    assert exchange_mismatches(exp, ok) == (0, 0, 3)
    bad = [(0, 2, {(0, 5): 3, (1, 5): 1}), (2, 4, {(3, 6): 1, (1, 5): 1})]
    assert exchange_mismatches(exp, bad) == (0, 1, 3)        # the sum holds, one row in the wrong block
    assert exchange_mismatches(exp, [(0, 4, {(0, 5): 3})])[0] == 2


def test_owned_block_matches_padding_rule():
    for C in (1, 7, 100, 1_000_000):
        for N in (1, 2, 3, 8):
            cp = (C + N - 1) // N * N
            prev = 0
            for r in range(N):
                lo, hi = owned_block(C, r, N)
                assert lo == min(C, r * (cp // N)) and hi == min(C, lo + cp // N)
                assert lo == prev
                prev = hi
            assert prev == C


def test_router_is_deterministic_and_consistent_with_ad_shard():
    from ysb_amd import ad_shard
    raw, offs = gd.events("gen_s7")
    import numpy as np
    a = np.frombuffer(raw, dtype=np.uint8)
    s1, c1 = route_lines(a, offs, 4)
    s2, _ = route_lines(a, offs, 4)
    assert (s1 == s2).all() and int(c1.sum()) == len(offs)
    ends = list(offs[1:]) + [len(raw)]
    for i in range(0, len(offs), 97):
        ev = json.loads(raw[offs[i]:ends[i]])
        assert s1[i] == ad_shard(ev["ad_id"], 4)
    # a non-canonical layout routes by the same key
    line = b'{ "ad_id" : "%s", "event_type": "view", "user_id": "u", "page_id": "p", "ad_type": "x", ' \
           b'"event_time": "1"}\n' % json.loads(raw[offs[0]:ends[0]])["ad_id"].encode()
    s3, _ = route_lines(np.frombuffer(line, dtype=np.uint8), np.zeros(1, dtype=np.uint32), 4)
    assert s3[0] == s1[0]
    # split + oracle over all shards == oracle over the batch
    ads, camp = gd.ad_arrays()
    am = oracle.AdMap(ads, camp)
    tot = Counter()
    for r in range(4):
        br, bo = split_batch(a, offs, s1, r)
        rows, _ = oracle.run(am, br.tobytes(), bo)
        tot.update(rows)
    assert dict(tot) == gd.expected("gen_s7")[0]


def test_dump_shards(tmp_path):
    g = GenParams(seed=3, n_campaigns=5, ads_per_campaign=4, events_per_sec=100)
    g.dump(300, tmp_path)
    whole = (tmp_path / "kafka-json.txt").read_bytes().splitlines()
    g.dump_shards(300, tmp_path, 3)
    parts = [(tmp_path / ("kafka-json.%d.txt" % r)).read_bytes().splitlines() for r in range(3)]
    assert sorted(whole) == sorted(sum(parts, []))
    from ysb_amd import ad_shard
    for r, lines in enumerate(parts):
        assert all(ad_shard(json.loads(ln)["ad_id"], 3) == r for ln in lines)


@pytest.mark.parametrize("world", [2, 3])
def test_streaming_ranks_share_one_watermark(world, tmp_path):
    """configs[4] across processes: each rank streams its shard; the watermark is the
    minimum over ranks (gloo all-reduce), so every rank closes the same windows at the
    same tick, and each rank's deltas are exact for its shard."""
    res = run_ranks(None, world, tmp_path, worker="stream_worker.py")[0]
    assert len(res) == world and all(r["exact"] for r in res)
    assert len(set(tuple(r["closed"]) for r in res)) == 1 and len(res[0]["closed"]) >= 2
    assert len(set(r["watermark"] for r in res)) == 1
    assert len(set(r["flushes"] for r in res)) == 1


def _range_ranks(world, tmp_path, *extra):
    port = free_port()
    procs, outs = [], []
    for r in range(world):
        out = tmp_path / ("x%d.json" % r)
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "exchange_worker.py"), str(out)] +
                                      list(extra), env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
        outs.append(out)
    logs = [p.communicate(timeout=300)[0].decode(errors="replace") for p in procs]
    for p, lg in zip(procs, logs):
        assert p.returncode == 0, lg[-3000:]
    return [json.load(open(o)) for o in outs]


@pytest.mark.parametrize("world", [2, 3])
def test_range_limited_exchange_250k_campaigns(world, tmp_path):
    """ysb_group_reduce_scatter's protocol (per-bucket maxima -> all-reduce(max) ->
    ysb_exchange_plan -> pack only the touched buckets in the narrowest width ->
    reduce-scatter -> unpack), gloo standing in for RCCL, at configs[2]-like size (250k
    campaigns, 500k ads sharded by ad_id hash), two exchanges: the owners' rows equal the
    truth summed over ranks, nothing stays pending, and each exchange moved 1-byte cells of
    the touched buckets only -- a small fraction of the whole u64 ring."""
    res = _range_ranks(world, tmp_path)
    mism, outside, cells = res[0]["exchange"]
    assert mism == 0 and outside == 0 and cells > 0
    for rr in res[0]["ranks_rounds"]:
        for rnd in rr:
            assert rnd["pending_left"] == 0 and rnd["width"] == 1
            assert 0 < rnd["buckets"] < 64 and rnd["bytes"] * 16 < res[0]["full_ring_bytes"]
    # every rank made the same plan (the all-reduced maxima)
    assert len({json.dumps([(r["buckets"], r["width"]) for r in rr]) for rr in res[0]["ranks_rounds"]}) == 1


def test_range_limited_exchange_wide_cells(tmp_path):
    """Heavy cells (every view in 7 campaigns, hundreds per cell): the plan widens the cells
    to 4 bytes so the sum over the ranks cannot wrap; still exact."""
    res = _range_ranks(2, tmp_path, "20000", "2")
    mism, outside, cells = res[0]["exchange"]
    assert mism == 0 and outside == 0 and cells > 0
    assert {rnd["width"] for rr in res[0]["ranks_rounds"] for rnd in rr} == {4}
