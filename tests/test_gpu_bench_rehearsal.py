"""GPU: bench.py's N-rank flow end to end on one GPU (the driver's 8-GPU run has never been
possible here: RCCL refuses two ranks on one device).  `--rehearse-host-collectives` runs the
same launcher, sharded generation, per-step exchange, post-exchange check, configs[2]-table leg
(checksums) and N-shard native stream as `bench.py --gpus N`, with the keyBy exchange over the
ranks' gloo collectives (ysb_group_init_host) instead of RCCL.  The printed line must be the
contract line with every check exact."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_rehearsal(tmp_path):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    extras = str(tmp_path / "extras.json")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rehearse-host-collectives",
                        "--events", "4000000", "--steps", "2", "--warmup", "1", "--c3-events", "2000000",
                        "--extra-steps", "1", "--stream-seconds", "2", "--stream-target", "40e6",
                        "--stream-host-gb", "4", "--extras-out", extras],
                       capture_output=True, text=True, timeout=400, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    last = r.stdout.strip().splitlines()[-1]
    assert len(last) <= 6000
    line = json.loads(last)
    assert line["n_gpus"] == 2 and line["value"] > 0 and "REHEARSAL" in line["config"]["parallelism"]
    c = line["check"]
    assert c["truth_mismatched_cells"] == 0 and c["truth_views"] == c["counted_views"] > 0
    x = c["exchange"]
    assert x["post_exchange_mismatched_cells"] == 0 and x["owned_views"] == x["truth_views_summed"]
    assert x["owned_blocks"] == [[0, 50], [50, 100]]
    s = line["extras_summary"]
    assert s["config3"]["exact"] is True, s
    assert s["stream_native"]["exact"] is True, s
    with open(extras) as f:
        full = json.load(f)
    assert full["config3"]["check"]["checksum_blocks_mismatched"] == 0
    assert full["stream_native"]["runner"]["cycles"] and len(full["stream_native"]["runner"]["cycles"]) == 2
