"""GPU: the library's N-rank group path on ONE MI355X -- N processes, each with its own
context on cuda:0, the exchange over ysb_group_init_host with gloo as the transport (RCCL
refuses two ranks per device; everything else is what bench.py --gpus N runs): ring
agreement, the range-limited exchange at configs[2]-like table sizes with a sharded join
table, the owners' tables against the generator truth summed over the ranks."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def run(scenario, world, tmp_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs, outs = [], []
    for r in range(world):
        out = tmp_path / ("g%d.json" % r)
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OMP_NUM_THREADS="2")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "group_worker.py"), scenario, str(out)],
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


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_n_ranks_range_exchange_config3_tables(world, tmp_path):
    res = run("config3", world, tmp_path)
    r0 = res[0]
    per = r0["per_rank"]
    assert r0["blocks_mismatched"] == 0
    assert all(p["mism"] == 0 and p["truth"] == p["ring"] > 0 for p in per)      # each rank vs its own truth
    assert sum(p["owned_total"] for p in per) == sum(p["truth"] for p in per)    # nothing lost in the exchange
    assert all(p["foreign"] == 0 and p["misses"] == 0 for p in per)              # routing matches the sharded table
    assert all(p["ranks"] == [i, world] for i, p in enumerate(per))
    for r in res:
        st = r["steps"]
        assert st["exchanges"] == 3 and st["record_launches"] == 3
        assert st["width"] == 1 and 0 < st["buckets"] <= 128                    # 1-byte cells, touched buckets only
        rows = 3 * ((200_000 + world - 1) // world * world)
        row = st["bytes"] // rows                          # whole aligned 4-slot groups per row
        assert st["bytes"] % rows == 0 and row % 4 == 0 and st["buckets"] <= row <= st["buckets"] + 6


@pytest.mark.timeout(300)
def test_n_ranks_bench_exchange_check_config2(tmp_path):
    res = run("config2", 2, tmp_path)
    chk = res[0]["check"]
    ex = chk["exchange"]
    assert chk["truth_mismatched_cells"] == 0 and chk["truth_views"] == chk["counted_views"] > 0
    assert ex["post_exchange_mismatched_cells"] == 0 and ex["owner_rows_outside_block"] == 0
    assert ex["owned_views"] == ex["truth_views_summed"] == chk["truth_views"]
    assert ex["ring_bases_equal"] and ex["rccl_ranks"] == [2]
    for r in res:
        assert r["steps"]["exchanges"] == 2 and r["steps"]["width"] == 4   # config-2 cells: thousands of views


@pytest.mark.timeout(300)
def test_n_ranks_pipelined_exchange_holds_back_then_settles(tmp_path):
    res = run("pipelined", 2, tmp_path)
    for r in res:
        log = r["log"]
        assert [e["bad_blocks"] for e in log] == [0, 0, 0, 0]     # owned + pending = truth after every call
        assert log[0]["buckets"] == 0 and log[0]["pending_nonzero"]   # packs the agreeing call's empty plan
        assert log[1]["pending_nonzero"]        # outgrew step 0's 1-byte plan / new buckets: held back
        assert log[2]["width"] == 4 and log[2]["buckets"] >= 2 and not log[2]["pending_nonzero"]   # caught up
        assert log[3]["buckets"] == 0 and not log[3]["pending_nonzero"]
        assert r["views"]["ring"] == 0
    assert sum(r["views"]["owned"] for r in res) == sum(r["views"]["truth"] for r in res) > 0
