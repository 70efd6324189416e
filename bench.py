"""Benchmark of the MI355X YSB advertising hot path (BASELINE.json configs[1] / configs[3]).

One step = one pass of parse + view filter + ad->campaign join + 10 s window count
over the rank's whole resident batch: generator-format JSON events (100 campaigns x 10
ads, 10 s windows), HBM-resident before timing starts, as batches of 16.67M events (u32
line offsets cap a batch at 4 GiB) scanned by ONE kernel launch
(ysb_submit_device_segments; --per-batch: one launch per batch).

    python bench.py [--gpus N] [--steps K] [--warmup W]

--gpus 1 (default): configs[1], 100M events.  Then, after the headline line's numbers
are taken, the same process times configs[2] (1M campaigns / 10M ads) and the fork's
.tbl rows as extra keys (--no-extras skips them).

--gpus N > 1: one process per GPU.  Started without torchrun (WORLD_SIZE unset), this
process is only a launcher: it starts N rank processes (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_* set, 127.0.0.1) before anything touches a GPU and exits with their status;
under torchrun each rank runs directly.  Events are sharded by ad_id hash (rank r draws
from its own ad shard; per-GPU work fixed: weak scaling; 1B / N events per GPU at N >= 8,
so N = 8 is configs[3]'s 1B events), every step ends with the RCCL reduce-scatter of the
(campaign, window) tables over xGMI, and after timing the owners' rows are checked
against the generator truth summed over ranks (check.exchange).

Rank 0 prints one JSON line (metric/value/unit/... + roofline + cpu_baseline).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "streaming-benchmarks_amd"))

import numpy as np  # noqa: E402

METRIC = "events/sec (parse+filter+join+window count) at 1/8 GPUs; % HBM roofline"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
TOTAL_EVENTS_8 = 1_000_000_000   # configs[3]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10,
                    help="untimed steps (~40 ms; the clocks reach their steady state after ~8)")
    ap.add_argument("--events", type=int, default=None,
                    help="events per GPU (default 100M; 1B / N at N >= 8: configs[3]'s 1B events at N = 8)")
    ap.add_argument("--segment", type=int, default=16_666_667,
                    help="events per batch (6 per 100M: the largest that keep a batch's bytes under the "
                         "4 GiB of u32 line offsets)")
    ap.add_argument("--per-batch", action="store_true",
                    help="one launch per batch (ysb_submit_device) instead of one launch over all batches")
    ap.add_argument("--rate", type=int, default=100_000, help="events per second of event time")
    ap.add_argument("--cpu-sample", type=int, default=4_000_000, help="events in the CPU baseline sample")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-check", action="store_true", help="skip the generator-truth check")
    ap.add_argument("--no-extras", action="store_true", help="skip the configs[2] / .tbl extra measurements")
    ap.add_argument("--extra-steps", type=int, default=20)
    ap.add_argument("--stream-seconds", type=float, default=12.0,
                    help="extras: wall seconds of the native streaming leg (configs[4]; at the default speedup "
                         "12 s of input is 420 s of event time: >= 30 windows close); 0 skips it")
    ap.add_argument("--stream-target", type=float, default=210e6,
                    help="extras: events/s per shard (GPU) the streaming replay releases (the zero-copy feed's "
                         "ceiling is the slot copy over PCIe, ~215M/s at 254 B per event)")
    ap.add_argument("--stream-host-gb", type=float, default=64.0,
                    help="extras: host memory for all shards' replay cycles (each cycle is 10 s of event time, "
                         "at most 16 GB per shard): sets the event rate per shard, and the speedup follows "
                         "from --stream-target")
    ap.add_argument("--stream-replay", choices=("mapped", "mapped-raw", "copy"), default="mapped",
                    help="extras: the streaming feed: in place from the registered cycle, or round 5's host copy")
    ap.add_argument("--stream-rate", type=int, default=20_000_000,
                    help="tools/bench_extra.py stream_sharded: aggregate events/s of the Python producers")
    ap.add_argument("--dropin-events", type=int, default=100_000_000,
                    help="extras: events through the host-staged (pinned slots, H2D) path")
    ap.add_argument("--runner-file-events", type=int, default=20_000_000,
                    help="extras: events in the native runner's replay file")
    ap.add_argument("--runner-repeat", type=int, default=5, help="extras: times the runner reads its replay file")
    ap.add_argument("--extras-timeout", type=int, default=600,
                    help="N > 1: seconds the extras (configs[2]-table leg, then rank 0's N-GPU native stream) may "
                         "take before rank 0 prints the headline without them")
    ap.add_argument("--c3-events", type=int, default=100_000_000,
                    help="extras at N > 1: events per GPU of the configs[2]-table leg (1M campaigns / 10M ads)")
    ap.add_argument("--layout-fixed", action="store_true",
                    help="A/B: no first-line layout sampling of the device batches (YSB_F_LAYOUT_FIXED)")
    ap.add_argument("--rehearse-host-collectives", action="store_true",
                    help="N > 1 on a box with fewer GPUs: the ranks share the visible GPUs and exchange over gloo "
                         "on host memory (ysb_group_init_host) instead of RCCL -- a rehearsal of the N-rank flow, "
                         "not a measurement")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch the ranks and set up torch.distributed, then stop before any GPU call")
    ap.add_argument("--extras-out", default=os.path.join(ROOT, "gpurun_out", "bench_extras.json"),
                    help="where the extras go in full (the printed line holds a summary per leg)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--no-live-traffic", action="store_true",
                    help="N = 1: take roofline.traffic from --traffic instead of two rocprofv3 --pmc child passes")
    a = ap.parse_args(argv)
    if a.events is None:
        a.events = TOTAL_EVENTS_8 // a.gpus if a.gpus >= 8 else 100_000_000
    return a


# ---- launcher ----------------------------------------------------------------------------

def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n, argv):
    """Starts n rank processes of this script (one per GPU) and waits for them.  Called
    before anything in this process touches a GPU (no HIP call, no torch.cuda): the
    children are fresh processes, and this one only waits.  If a rank fails, the others
    are stopped (they would wait forever in a collective)."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    failed = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad and not failed:
            failed = bad[0]
            log("bench: a rank exited with %d; stopping the others" % failed)
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            deadline = time.time() + 20
            while time.time() < deadline and any(p.poll() is None for p in procs):
                time.sleep(0.2)
            for p in procs:
                if p.poll() is None:
                    p.kill()
        if all(c is not None for c in (p.poll() for p in procs)):
            break
        time.sleep(0.2)
    return failed or max(abs(p.returncode) for p in procs)


# ---- ranks --------------------------------------------------------------------------------

class Dist:
    def __init__(self, n):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        # this rank's GPU: LOCAL_RANK until resolve_device() (not in a dry run: nothing here
        # touches a GPU)
        self.device = self.local
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist
        if n != self.world:
            log("note: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (n, self.world))

    def resolve_device(self):
        """LOCAL_RANK, unless the launcher left each process fewer visible devices (e.g. one per
        rank through HIP_VISIBLE_DEVICES): then the k-th visible one -- counted by the library
        (hipGetDeviceCount), not by torch, whose ROCm build may not see a GPU HIP sees."""
        from ysb_amd import device_count, rank_device
        self.n_visible = device_count()
        self.device = rank_device(self.local, self.n_visible)
        return self.device

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, v):
        if not self.dist:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, v):
        if not self.dist:
            return v
        import torch
        t = torch.tensor([int(v)], dtype=torch.int64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return int(t.item())

    def sum_array(self, a):
        """Elementwise sum over ranks of a uint64 array (counts < 2^63)."""
        if not self.dist:
            return a
        import torch
        t = torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).clone()
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return t.numpy().view(np.uint64).reshape(a.shape)

    def gather(self, obj):
        if not self.dist:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def bcast_bytes(self, b):
        if not self.dist:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]


def dry_run(d, args):
    """Launch rehearsal: every rank reports its environment; nothing touches a GPU.
    YSB_BENCH_FAIL_RANK=r makes rank r exit with status 3 first (tests the launcher's
    stop-the-others path: the remaining ranks would wait in the gather forever)."""
    if os.environ.get("YSB_BENCH_FAIL_RANK") == str(d.rank):
        sys.exit(3)
    info = {"rank": d.rank, "local_rank": d.local, "device": d.device, "world": d.world, "pid": os.getpid(),
            "master": "%s:%s" % (os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT")),
            "events_per_gpu": args.events}
    allinfo = d.gather(info)
    if d.rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": d.world, "ranks": allinfo}), flush=True)
    if d.dist:
        d.dist.destroy_process_group()


def device_sync(device=0):
    """The contract's device-wide synchronize on this rank's own GPU, through the library's own
    HIP runtime (ysb_device_sync = hipDeviceSynchronize; the library's streams are synchronised
    by ctx.sync() before it).  Not torch.cuda.synchronize: torch 2.10 bundles its own HIP/HSA
    runtime, and whichever runtime opens the GPU first in a process is the one that sees it
     -- bench.py never initialises torch's."""
    from ysb_amd import device_sync as _sync
    _sync(device)


# ---- the printed line ---------------------------------------------------------------------
# The driver reads the LAST stdout line and keeps a bounded tail of stdout: the line holds the
# contract keys and one short summary per extra leg; the extras in full go to a file
# (--extras-out) and to one stderr line before it.
LINE_MAX_BYTES = 6000


def _exact(r):
    """True / False when the leg carries a check, else None."""
    if "exact_vs_generator_truth" in r:
        return bool(r["exact_vs_generator_truth"])
    ch = r.get("check")
    if not isinstance(ch, dict):
        return None
    bad = 0
    for k in ("truth_mismatched_cells", "checksum_blocks_mismatched", "overflow_dropped", "parse_errors",
              "join_misses", "deferred", "deferred_to_general_path"):
        v = ch.get(k)
        if isinstance(v, (int, float)):
            bad += v
    x = ch.get("exchange")
    if isinstance(x, dict):
        bad += x.get("post_exchange_mismatched_cells", 0)
    if "truth_views" in ch and "counted_views" in ch:
        bad += ch["truth_views"] != ch["counted_views"]
    return bad == 0


def leg_summary(r):
    """One extra leg in a few keys: events_per_s, hbm_frac, exact (or its error)."""
    if not isinstance(r, dict):
        return None
    if "error" in r:
        return {"error": str(r["error"])[:160]}
    s = {}
    eps = r.get("stream_events_per_s", r.get("events_per_s"))
    if eps is not None:
        s["events_per_s"] = eps
    if r.get("hbm_frac") is not None:
        s["hbm_frac"] = r["hbm_frac"]
    if r.get("vs_host_staged") is not None and eps is not None:
        s["vs_host_staged"] = r["vs_host_staged"]
    ex = _exact(r)
    if ex is not None:
        s["exact"] = ex
    if not s:   # a leg of sub-legs (host_staged, native_runner)
        for k, v in r.items():
            if isinstance(v, dict) and (v.get("events_per_s") is not None or v.get("stream_events_per_s") is not None):
                s[k] = leg_summary(v)
    return s


def extras_summary(extra):
    return {k: leg_summary(v) for k, v in (extra or {}).items()}


def bench_line(out, extra, extras_path=None):
    """The one JSON line rank 0 prints last: `out` (the contract keys) plus the extras'
    summary, at most LINE_MAX_BYTES (the summary is dropped leg by leg if it would not fit)."""
    line = dict(out)
    if extra is not None:
        line["extras_summary"] = extras_summary(extra)
        if extras_path:
            line["extras_file"] = os.path.relpath(extras_path, ROOT) if extras_path.startswith(ROOT) else extras_path
    txt = json.dumps(line, separators=(",", ":"))
    while len(txt) > LINE_MAX_BYTES and line.get("extras_summary"):
        line["extras_summary"].popitem()
        line["extras_truncated"] = True
        txt = json.dumps(line, separators=(",", ":"))
    return txt


def emit(out, extra, extras_out):
    """Full extras to extras_out and to stderr, then the compact line on stdout (last)."""
    path = None
    if extra is not None:
        full = json.dumps(extra)
        log("bench extras: " + full)
        if extras_out:
            try:
                os.makedirs(os.path.dirname(os.path.abspath(extras_out)), exist_ok=True)
                with open(extras_out, "w") as f:
                    f.write(full + "\n")
                path = os.path.abspath(extras_out)
            except OSError as e:
                log("bench: could not write %s: %s" % (extras_out, e))
    print(bench_line(out, extra, path), flush=True)


def cpu_baseline(ctx, d_b, d_o, nb_seg, n_seg, ads, camp, sample, seconds):
    """The C oracle (oracle/ysb_oracle.c, a port) on the host cores, on a bounded
    sample: the first `sample` events of segment 0, re-run until `seconds` elapse."""
    from oracle import oracle
    n = min(sample, n_seg)
    off = ctx.d2h(np.empty(n_seg, dtype=np.uint32), d_o)
    end = int(off[n]) if n < n_seg else nb_seg
    data = ctx.d2h(np.empty(end, dtype=np.uint8), d_b)
    off = np.ascontiguousarray(off[:n])
    am = oracle.AdMap(ads, camp)
    threads = min(16, os.cpu_count() or 1)
    res = {}
    for th in (threads, 1):
        done, t0 = 0, time.perf_counter()
        while True:
            rows, st = oracle.run(am, data, off, threads=th)
            done += n
            el = time.perf_counter() - t0
            if el >= (seconds if th == threads else seconds / 4):
                break
        res[th] = (done / el, rows, st, el)
    # the same sample through the GPU path: identical counts
    from ysb_amd import YsbContext
    with YsbContext(device=ctx.device, n_campaigns=100) as c2:
        c2.load_ad_map(ads, camp)
        c2.submit_device(d_b, end, d_o, n)
        same = c2.drain_buckets() == res[threads][1] and all(
            c2.stats()[k] == v for k, v in res[threads][2].items())
    v, _, _, el = res[threads]
    return {"value": round(v, 1), "unit": "events/s", "cores": threads, "kind": "port",
            "sample": "first %d events (%.2f GB) of the GPU workload, oracle/ysb_oracle.c with %d threads, "
                      "%.1f s of repeats; 1 thread: %.0f events/s; counts identical to the GPU path on "
                      "that sample: %s" % (n, end / 1e9, threads, el, res[1][0], same)}


def gen_segments(ctx, g, events, segment):
    segs, first = [], 0
    while first < events:
        n = min(segment, events - first)
        cap = n * g.max_line_bytes()
        d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n + 64)
        nb = ctx.gen_events_device(g, first, n, d_b, cap, d_o)
        segs.append((first, n, d_b, nb, d_o))
        first += n
    return segs


def free_segments(ctx, segs):
    for (_, _, d_b, _, d_o) in segs:
        ctx.device_free(d_b)
        ctx.device_free(d_o)


def timed_extra(name, ctx, g, segs, steps, warmup, kernel):
    """One extra configuration: warmup, `steps` timed single-launch steps, then the
    generator-truth check of one more pass."""
    sub = [(d_b, nb, d_o, n) for (_, n, d_b, nb, d_o) in segs]
    for _ in range(warmup):
        ctx.submit_device_segments(sub)
    ctx.sync()
    ctx.kernel_time()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.submit_device_segments(sub)
    ctx.sync()
    el = time.perf_counter() - t0
    kms, launches = ctx.kernel_time()
    pms, _, nrec = ctx.path_time()
    ctx.reset()
    ctx.submit_device_segments(sub)
    for (f, n, _, _, _) in segs:
        ctx.truth_accumulate(g, f, n)
    mism, truth, ring = ctx.truth_compare()
    st = ctx.stats()
    events = sum(s[1] for s in segs)
    nbytes = sum(s[3] for s in segs)
    alg = nbytes + 4 * events
    avg = kms / max(launches, 1)
    path = pms / max(launches, 1)
    ach = alg / (path * 1e-3) / 1e9
    return {"workload": name, "events": events, "bytes_per_event": round(nbytes / events, 3),
            "events_per_s": round(events * steps / el, 1), "ms_per_step": round(el / steps * 1e3, 4),
            "kernel": kernel, "avg_launch_ms": round(avg, 4),
            "avg_path_ms": round(path, 4), "record_mode": nrec > 0,
            "alg_GBs": round(ach, 1), "hbm_frac": round(ach / HBM_PEAK_GBS, 4),
            "note": "alg_GBs / hbm_frac over the launch's whole device sequence (scan, general path and, "
                    "in record mode, the partition + count kernels: avg_path_ms)",
            "check": {"truth_mismatched_cells": mism, "truth_views": truth, "counted_views": ring,
                      "join_misses": st["join_misses"], "parse_errors": st["parse_errors"],
                      "deferred": st["deferred"], "out_of_ring": st["out_of_ring"],
                      "overflow_dropped": st["overflow_dropped"]}}


def guarded(out, key, fn):
    """One extra measurement: its result, or {"error": ...} -- a failing extra never costs the
    headline line."""
    try:
        out[key] = fn()
    except Exception as e:   # noqa: BLE001 (recorded in the line, the headline still prints)
        import traceback
        log("extras: %s failed: %s" % (key, traceback.format_exc()))
        out[key] = {"error": "%s: %s" % (type(e).__name__, e)}


def extras(args, device):
    """configs[2] (1M campaigns / 10M ads: join and count tables in HBM), configs[1]'s
    events as the fork's .tbl rows and in other producers' layouts, each timed like the
    headline (one launch per step), and configs[4]'s sharded streaming.  Each leg is
    guarded: a failure is recorded as {"error": ...} under its key."""
    out = {}
    guarded(out, "host_staged", lambda: extra_host_staged(args, device))
    guarded(out, "native_runner", lambda: extra_native_runner(args, device, out.get("host_staged")))
    guarded(out, "config3", lambda: extra_config3(args, device))
    from ysb_amd import GEN_COMPACT, GEN_REORDER
    guarded(out, "config3_compact", lambda: extra_config3(
        args, device, GEN_COMPACT, "compact JSON (no space after ':' and ','), no hint: the layout read from "
        "each batch's first line"))
    guarded(out, "config3_reordered_no_hint", lambda: extra_config3(
        args, device, GEN_REORDER, "the keys in another order (ad_type, event_time, ad_id, ip_address, user_id, "
        "event_type, page_id), no hint: the learned-order instantiation from each batch's first line"))
    guarded(out, "tbl", lambda: extra_tbl(args, device))
    extra_layouts(args, device, out)
    guarded(out, "alternating_producers", lambda: extra_alternating(args, device))
    if args.stream_seconds > 0:
        guarded(out, "stream_native", lambda: extra_stream_native(args, device))
        sn, hs = out.get("stream_native", {}), out.get("host_staged", {})
        if "events_per_s" in sn and isinstance(hs.get("raw"), dict) and hs["raw"].get("events_per_s"):
            # the sustained stream against the drop-in path's PCIe-bound rate in the same run
            sn["vs_host_staged"] = round(sn["events_per_s"] / hs["raw"]["events_per_s"], 4)
    return out


def extra_host_staged(args, device):
    """The drop-in's host-staged path (AdvertisingTopologyNative.java:111-119): configs[1]'s
    events through the pinned double-buffered slots, H2D + scan, with host line offsets
    (ysb_submit) and as raw lines split on the GPU (ysb_submit_raw) -- tools/bench_dropin.py."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_dropin
    r = {"offsets": bench_dropin.host_staged(device, args.dropin_events, raw=False),
         "raw": bench_dropin.host_staged(device, args.dropin_events, raw=True),
         # the same offsets leg with the DMA engine doing the H2D (YSB_F_H2D_SDMA): the path
         # round 4 shipped, in the same process and period ("H2D")
         "offsets_dma_engine": bench_dropin.host_staged(device, args.dropin_events, raw=False, h2d_sdma=True)}
    log("extras: host_staged %.3f / raw %.3f / DMA-engine offsets %.3f G events/s"
        % (r["offsets"]["events_per_s"] / 1e9, r["raw"]["events_per_s"] / 1e9,
           r["offsets_dma_engine"]["events_per_s"] / 1e9))
    return r


def extra_native_runner(args, device, staged):
    """bin/ysb_topology (the native drop-in for `flink run ... --confPath`) over a replay file
    in the page cache, read --runner-repeat times, against the generator truth: gpu_split is
    the runner's default (--io auto: the file's mapping registered, every batch read in place
    by the copy kernel, the lines split on the GPU); gpu_split_slot_copies the same through the
    pinned slots (parallel copies out of the mapping); host_split the host's line split;
    gpu_split_dma_engine the slots' H2D by the DMA engine.  vs_host_staged = the default's
    stream rate / the host-staged raw path's (the H2D-bound rate)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_dropin
    import tempfile
    path = tempfile.mkdtemp(prefix="ysb_replay_", dir=os.environ.get("TMPDIR") or "/tmp")
    n, k = args.runner_file_events, args.runner_repeat
    try:
        r = {"gpu_split": bench_dropin.native_runner(device, n, k, workdir=path, io="auto"),
             "gpu_split_slot_copies": bench_dropin.native_runner(device, n, k, workdir=path, io="mmap"),
             "host_split": bench_dropin.native_runner(device, n, k, host_split=True, workdir=path),
             "gpu_split_dma_engine": bench_dropin.native_runner(device, n, k, workdir=path, h2d_sdma=True)}
    finally:
        import shutil
        shutil.rmtree(path, ignore_errors=True)
    if staged and "raw" in staged:
        r["vs_host_staged"] = round(r["gpu_split"]["stream_events_per_s"] / staged["raw"]["events_per_s"], 4)
    log("extras: native_runner %.3f G events/s (%s; slot copies %.3f, host split %.3f, DMA engine %.3f)"
        % (r["gpu_split"]["stream_events_per_s"] / 1e9, r["gpu_split"].get("h2d"),
           r["gpu_split_slot_copies"]["stream_events_per_s"] / 1e9, r["host_split"]["stream_events_per_s"] / 1e9,
           r["gpu_split_dma_engine"]["stream_events_per_s"] / 1e9))
    return r


def extra_config3(args, device, variant=0, what=None):
    """configs[2] (1M campaigns / 10M ads: the HBM-resident bucket join table, record-mode
    counting); variant: the same events as another producer writes them (compact JSON,
    another key order), the layout read from each batch's first line."""
    from ysb_amd import GenParams, YsbContext
    t = time.perf_counter()
    g = GenParams(seed=42, n_campaigns=1_000_000, ads_per_campaign=10, events_per_sec=args.rate, variant=variant)
    _, ab = g.ids_packed()
    with YsbContext(device=device, n_campaigns=1_000_000, window_ring=128, timing=True,
                    max_batch_bytes=1 << 20, max_batch_events=1 << 12) as ctx:
        ctx.load_ad_map_packed(ab, g.ad_campaign_index_array())
        load_s = time.perf_counter() - t
        # 6 batches, as the headline (other producers' lines up to ~280 B: 7)
        segs = gen_segments(ctx, g, 100_000_000, 14_285_715 if variant else 16_666_667)
        r = timed_extra("configs[2]: 100M JSON events, 1M campaigns x 10 ads (10M-ad join table and "
                        "1M x 128-bucket count ring in HBM)" + (", " + what if what else ""), ctx, g, segs,
                        args.extra_steps, args.warmup, None)
        lay = ctx.launch_info()["layout"]
        r["kernel"] = "ysb::scan_kernel<true, false, true, %d>" % lay
        r["ad_map_load_s"] = round(load_s, 2)
        free_segments(ctx, segs)
    log("extras: config3%s %.2f G events/s" % (" variant %d" % variant if variant else "", r["events_per_s"] / 1e9))
    return r


def extra_tbl(args, device):
    from ysb_amd import GenParams, YsbContext
    g = GenParams(seed=42, n_campaigns=100, ads_per_campaign=10, events_per_sec=args.rate, fmt="tbl")
    _, aids = g.ids()
    with YsbContext(device=device, n_campaigns=100, window_ring=1024, timing=True, input_format="tbl",
                    max_batch_bytes=16 << 20, max_batch_events=1 << 16) as ctx:
        ctx.load_ad_map(aids, g.ad_campaign_index())
        segs = gen_segments(ctx, g, 100_000_000, 25_000_000)   # 4 batches of ~3.5 GB (rows ~140 B)
        r = timed_extra("configs[1]'s 100M events as the fork's .tbl rows (MockWindowedFlatMap, "
                        "AdvertisingTopologyNative.java:197-226)", ctx, g, segs, args.extra_steps,
                        args.warmup, "ysb::scan_kernel<false, true, false, 0>")
        free_segments(ctx, segs)
    log("extras: tbl %.2f G events/s" % (r["events_per_s"] / 1e9))
    return r


def extra_layouts(args, device, out):
    """The same events as other producers would write them: other ip / ad_type values (the
    vocabulary path's generic-value branches), compact JSON and another key order -- with
    the layout read from each batch's first line (the default), with an explicit hint, and
    (_fixed) with neither."""
    from ysb_amd import (GEN_COMPACT, GEN_MIXED, GEN_MIXED_BLOCKS, GEN_MORE_AD_TYPES, GEN_RANDOM_IP, GEN_REORDER,
                         GenParams, YsbContext)
    for key, variant, cf, what in (("mixed_layouts", GEN_MIXED, False,
                                    "four producers interleaved line by line (the generator's layout, compact JSON, "
                                    "reordered keys, random ip with 8 ad_types; a quarter each), no hint: the "
                                    "flat tier (the sample's adjacent lines differ)"),
                                   ("mixed_blocks", GEN_MIXED_BLOCKS, False,
                                    "the same four producers in runs of 256 events (a consumer's batches from "
                                    "several partitions), no hint: the per-tile dispatch, a tile of one producer "
                                    "takes that producer's path"),
                                   ("mixed_layouts_flat_tier", GEN_MIXED, "flat_fixed",
                                    "four producers interleaved line by line, YSB_F_FLAT_FIRST with YSB_F_LAYOUT_FIXED: "
                                    "the flat-object tier parses every line"),("random_ip", GEN_RANDOM_IP, False, "random dotted-quad ip_address"),
                                   ("random_ip_8_ad_types", GEN_RANDOM_IP | GEN_MORE_AD_TYPES, False,
                                    "random dotted-quad ip_address and 8 ad_types"),
                                   ("compact_json", GEN_COMPACT, True,
                                    "compact JSON, no space after ':' and ',' (layout hint YSB_F_COMPACT_FIRST: "
                                    "the compact layout's vocabulary path first)"),
                                   ("compact_json_no_hint", GEN_COMPACT, False,
                                    "compact JSON without a hint (the layout read from each batch's first line)"),
                                   ("reordered_keys", GEN_REORDER, "flat",
                                    "the keys in another order (ad_type, event_time, ad_id, ip_address, user_id, "
                                    "event_type, page_id), layout hint YSB_F_FLAT_FIRST (the first line names one key "
                                    "order: the learned-order instantiation, off-order lines to the flat tier)"),
                                   ("reordered_keys_flat_tier", GEN_REORDER, "flat_fixed",
                                    "the keys in another order, YSB_F_FLAT_FIRST with YSB_F_LAYOUT_FIXED: the "
                                    "flat-object tier (any key order or spacing) parses every line"),
                                   ("reordered_keys_no_hint", GEN_REORDER, False,
                                    "the keys in another order without a hint (the layout read from each batch's "
                                    "first line)"),
                                   ("reordered_keys_fixed", GEN_REORDER, "fixed",
                                    "the keys in another order with the layout fixed to the generator's "
                                    "(YSB_F_LAYOUT_FIXED: the scan's fourth tier, after the vocabulary path fails)")):
        def one(key=key, variant=variant, cf=cf, what=what):
            g = GenParams(seed=42, n_campaigns=100, ads_per_campaign=10, events_per_sec=args.rate, variant=variant)
            _, aids = g.ids()
            with YsbContext(device=device, n_campaigns=100, window_ring=1024, timing=True,
                            max_batch_bytes=16 << 20, max_batch_events=1 << 16, compact_first=cf is True,
                            flat_first=cf in ("flat", "flat_fixed"), layout_auto=cf not in ("fixed", "flat_fixed")) as ctx:
                ctx.load_ad_map(aids, g.ad_campaign_index())
                # lines up to ~280 B: 7 batches keep each under the 4 GiB of u32 offsets
                segs = gen_segments(ctx, g, 100_000_000, 14_285_715)
                r = timed_extra("configs[1]'s 100M events, " + what, ctx, g, segs, args.extra_steps,
                                args.warmup, None)
                lay = ctx.launch_info()["layout"]
                r["kernel"] = "ysb::scan_kernel<false, false, false, %d>" % lay
                free_segments(ctx, segs)
            log("extras: %s %.2f G events/s" % (key, r["events_per_s"] / 1e9))
            return r
        guarded(out, key, one)


def extra_alternating(args, device):
    """Device batches whose producers alternate per launch (the generator's layout, reordered
    keys, compact JSON -- one producer's 33.3M events per launch, in turn) on a busy compute
    stream: each launch is decided on the previous launch's sample, the two last samples
    disagree, so the per-tile dispatch runs (ABI 4; round 4 ran the previous producer's
    instantiation, reordered lines through layout 0's fourth tier).  Exact vs the truth of
    every submission."""
    from ysb_amd import GEN_COMPACT, GEN_REORDER, GenParams, YsbContext
    per = 33_333_334
    gens = [GenParams(seed=42, n_campaigns=100, ads_per_campaign=10, events_per_sec=args.rate, variant=v)
            for v in (0, GEN_REORDER, GEN_COMPACT)]
    _, aids = gens[0].ids()
    with YsbContext(device=device, n_campaigns=100, window_ring=1024, timing=True, max_batch_bytes=16 << 20,
                    max_batch_events=1 << 16) as ctx:
        ctx.load_ad_map(aids, gens[0].ad_campaign_index())
        sets = [gen_segments(ctx, g, per, 14_285_715) for g in gens]
        subs = [[(d_b, nb, d_o, n) for (_, n, d_b, nb, d_o) in segs] for segs in sets]
        steps = 3 * max(1, args.extra_steps // 3)
        for k in range(3 * max(1, args.warmup // 3)):
            ctx.submit_device_segments(subs[k % 3])
        ctx.sync()
        ctx.kernel_time()
        t0 = time.perf_counter()
        layouts = []
        for k in range(steps):
            ctx.submit_device_segments(subs[k % 3])
            layouts.append(ctx.launch_info()["layout"])
        ctx.sync()
        el = time.perf_counter() - t0
        kms, launches = ctx.kernel_time()
        pms, _, _ = ctx.path_time()
        ctx.reset()
        for k in range(3):
            ctx.submit_device_segments(subs[k])
            for (f, n, _, _, _) in sets[k]:
                ctx.truth_accumulate(gens[k], f, n)
        mism, truth, ring = ctx.truth_compare()
        st = ctx.stats()
        nbytes = sum(s[3] for segs in sets for s in segs)
        for segs in sets:
            free_segments(ctx, segs)
    events = 3 * per
    alg = (nbytes + 4 * events) / 3   # per launch
    path = pms / max(launches, 1)
    ach = alg / (path * 1e-3) / 1e9
    r = {"workload": "configs[1]'s events as three producers write them (the generator's layout, reordered keys, "
                     "compact JSON), %dM events per launch, the producer changing every launch, on a busy compute "
                     "stream (ABI 4: the per-tile dispatch once two samples disagree)" % (per // 1_000_000),
         "events_per_s": round(per * steps / el, 1), "ms_per_step": round(el / steps * 1e3, 4),
         "avg_path_ms": round(path, 4), "alg_GBs": round(ach, 1), "hbm_frac": round(ach / HBM_PEAK_GBS, 4),
         "layouts_timed": {str(x): layouts.count(x) for x in sorted(set(layouts))},
         "check": {"truth_mismatched_cells": mism, "truth_views": truth, "counted_views": ring,
                   "deferred": st["deferred"], "parse_errors": st["parse_errors"], "join_misses": st["join_misses"]}}
    log("extras: alternating_producers %.2f G events/s, %.3f of HBM" % (r["events_per_s"] / 1e9, r["hbm_frac"]))
    return r


STREAM_LINE_BYTES = 260   # a replay line (254 B) plus its share of the batches' alignment


def stream_rates(args, shards):
    """(event rate per shard, speedup) of the streaming replay: each shard's cycle (10 s of
    event time) within its share of --stream-host-gb (16 GB at most), released at
    --stream-target events/s per shard."""
    per_gb = min(16.0, args.stream_host_gb / shards)
    rate = int(min(args.stream_target / 35.0, per_gb * 1e9 / (10 * STREAM_LINE_BYTES)))
    return rate, args.stream_target / rate


def extra_stream_native(args, device, shards=1):
    """configs[4] natively: bin/ysb_topology --stream (tools/bench_stream.py): every shard's
    replay cycle registered with its context and fed in place by a feeder thread of its own on
    its GPU's NUMA node (the copy kernel reads the batch over PCIe, the GPU rebases the event
    times), asynchronous flushes through the C++ Redis writer, get-stats' per-(campaign,
    window) latency read back, exact vs the generator truth (check-correct).  shards > 1
    (bench.py --gpus N, rank 0 after the other legs): one shard per GPU of the node (shard s on
    device s), each at --stream-target events/s, one watermark = the minimum over them."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_stream
    rate, speedup = stream_rates(args, shards)
    r = bench_stream.stream_native(device, seconds=args.stream_seconds, event_rate=rate, speedup=speedup,
                                   shards=shards, replay=args.stream_replay)
    log("extras: stream_native %.3f G events/s, get-stats p50 / p99 %s / %s ms (closed windows %d), exact %s"
        % (r["events_per_s"] / 1e9, r["get_stats"]["p50_ms"], r["get_stats"]["p99_ms"],
           r["get_stats"]["closed_windows"], r["exact_vs_generator_truth"]))
    return r


def extra_stream(args):
    # configs[4] under load: real-time producers (16 host threads each call) writing
    # args.stream_rate events/s in all into double-buffered pinned slots, one context per
    # visible GPU (2..8 shards: configs[4]'s 8 GPUs on an 8-GPU node; on a one-GPU box two
    # contexts share it), one global watermark: sustained rate, back-pressure, p50 / p99 close
    # latency, exact vs the generator truth
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_extra
    from ysb_amd import device_count
    visible = device_count()
    ns = argparse.Namespace(shards=min(8, max(2, visible)), rate=args.stream_rate, seconds=args.stream_seconds,
                            batch_ms=20, ooo_ms=100, threads=16)
    r = bench_extra.stream_sharded(ns)
    log("extras: stream %s" % json.dumps(r["window_close_latency"]))
    return r


def config3_ranks(args, d):
    """configs[2]'s tables at N > 1 (configs[3]'s layout with 1M campaigns / 10M ads): each
    rank loads its 1/N ad_id-hash shard of the 10M-ad table (ysb_load_ad_map_packed_shard),
    scans args.c3_events of its own shard's events per step in record mode (W = 128), and
    every step ends with the range-limited exchange (only the buckets holding counts, in the
    narrowest cell width).  After timing: one more pass with the generator truth, one
    exchange, and the linear checksums (ysb_group_checksum): for every owner block r,
    owned(r) + SUM over ranks pending(r) == SUM over ranks truth(r) (mod 2^64) -- moving no
    table between ranks."""
    from ysb_amd import GenParams, YsbContext, shard_packed
    t = time.perf_counter()
    C3 = 1_000_000
    base = GenParams(seed=42, n_campaigns=C3, ads_per_campaign=10, events_per_sec=args.rate)
    _, ab = base.ids_packed()
    subset = np.nonzero(shard_packed(ab, d.world) == d.rank)[0].astype(np.uint32)
    g = GenParams(seed=42, event_stream=1 + d.rank, n_campaigns=C3, ads_per_campaign=10, events_per_sec=args.rate,
                  ad_subset=subset)
    W = 128
    # phase 1 is rank-local (no collective): a failure anywhere is agreed on before any rank
    # enters a collective, so every rank skips the leg together instead of waiting forever
    ctx, segs, err = None, [], None
    try:
        ctx = YsbContext(device=d.device, n_campaigns=C3, window_ring=W, timing=True,
                         ring_base_bucket=g.c.t0_ms // 10000 - W // 8, max_batch_bytes=1 << 20,
                         max_batch_events=1 << 12, layout_auto=not args.layout_fixed)
        ctx.load_ad_map_packed(ab, base.ad_campaign_index_array(), shard=(d.rank, d.world))
        del ab
        segs = gen_segments(ctx, g, args.c3_events, 16_666_667)
    except Exception as e:   # noqa: BLE001
        err = "rank %d: %s: %s" % (d.rank, type(e).__name__, e)
    errs = [x for x in d.gather(err) if x]
    if errs:
        if ctx is not None:
            free_segments(ctx, segs)
            ctx.close()
        raise RuntimeError("; ".join(errs))
    try:
        group_init(ctx, d, args)
        load_s = time.perf_counter() - t
        sub = [(d_b, nb, d_o, n) for (_, n, d_b, nb, d_o) in segs]

        def step(last=False):
            ctx.submit_device_segments(sub)
            exchange(ctx, last)
        for _ in range(args.warmup):
            step()
        ctx.sync()
        ctx.kernel_time()
        ctx.exchange_info(reset=True)
        device_sync(d.device)
        d.barrier()
        t0 = time.perf_counter()
        for i in range(args.extra_steps):
            step(i == args.extra_steps - 1)
        ctx.sync()
        device_sync(d.device)
        d.barrier()
        el = d.max(time.perf_counter() - t0)
        kms, launches = ctx.kernel_time()
        pms, _, nrec = ctx.path_time()
        x = ctx.exchange_info(reset=True)
        # the check: one more pass, its truth, one exchange, the checksums
        ctx.reset()
        ctx.submit_device_segments(sub)
        for (f, n, _, _, _) in segs:
            ctx.truth_accumulate(g, f, n)
        ctx.sync()
        mism, truth, ring = ctx.truth_compare()
        tsum = ctx.checksum("truth", d.world)
        st = ctx.stats()
        ctx.group_reduce_scatter()
        own = ctx.checksum("owned")[0]
        pend = ctx.checksum("pending", d.world)
        xi = ctx.exchange_info(reset=True)
        events = sum(s[1] for s in segs)
        nbytes = sum(s[3] for s in segs)
        per = d.gather({"tsum": tsum, "own": own, "pend": pend, "mism": mism, "truth": truth, "ring": ring,
                        "misses": st["join_misses"], "foreign": st["foreign_shard"], "perr": st["parse_errors"],
                        "oor": st["out_of_ring"], "chk_width": xi["last_width"], "chk_buckets": xi["last_buckets"]})
        free_segments(ctx, segs)
    finally:
        ctx.close()
    if d.rank != 0:
        return None
    M = (1 << 64) - 1
    bad_blocks = 0
    for r in range(d.world):
        want = sum(p["tsum"][r] for p in per) & M
        got = (per[r]["own"] + sum(p["pend"][r] for p in per)) & M
        bad_blocks += want != got
    alg = (nbytes + 4 * events)
    path = pms / max(launches, 1)
    ach = alg / (path * 1e-3) / 1e9
    steps = args.extra_steps
    return {"workload": "configs[2]'s tables at N = %d: %dM JSON events per GPU, 1M campaigns x 10 ads (each rank "
                        "1/%d of the 10M-ad join table), W = 128, range-limited RCCL exchange every step"
                        % (d.world, events // 1_000_000, d.world),
            "n_gpus": d.world, "events_per_gpu": events, "bytes_per_event": round(nbytes / events, 3),
            "events_per_s": round(events * d.world * steps / el, 1), "ms_per_step": round(el / steps * 1e3, 4),
            "avg_launch_ms": round(kms / max(launches, 1), 4), "avg_path_ms": round(path, 4),
            "record_mode": nrec > 0, "alg_GBs_per_gpu": round(ach, 1), "hbm_frac": round(ach / HBM_PEAK_GBS, 4),
            "ad_map_load_s": round(load_s, 2),
            "exchange": {"ms_per_step": round(x["ms"] / max(x["exchanges"], 1), 4),
                         "critical_ms_per_step": round(x["critical_ms"] / max(x["exchanges"], 1), 4),
                         **exchange_overlap(x),
                         "bytes_per_step_per_gpu": x["bytes"] // max(x["exchanges"], 1),
                         "buckets": x["last_buckets"], "cell_bytes": x["last_width"],
                         "whole_ring_u64_bytes": x["full_ring_bytes"],
                         "note": "ms: HIP events from the plan (compute stream) to the end of the unpack (exchange "
                                 "stream): plan, all-reduce(max), read-back, pack, reduce-scatter, unpack, per step; "
                                 "critical_ms: plan to pack on the compute stream (the reduce-scatter and unpack run "
                                 "beside the next launch); rs: pack done to reduce-scatter done on the exchange stream "
                                 "(peers' arrival included), exposed: the compute stream's wait for it at the unpack, "
                                 "hidden = rs - exposed"},
            "check": {"checksum_blocks_mismatched": bad_blocks, "blocks": d.world,
                      "truth_mismatched_cells": sum(p["mism"] for p in per),
                      "truth_views": sum(p["truth"] for p in per), "counted_views": sum(p["ring"] for p in per),
                      "join_misses": sum(p["misses"] for p in per), "foreign_shard": sum(p["foreign"] for p in per),
                      "parse_errors": sum(p["perr"] for p in per), "out_of_ring": sum(p["oor"] for p in per),
                      "check_exchange_cell_bytes": per[0]["chk_width"]}}


def live_traffic(args, kernel):
    """HBM bytes per launch of the headline kernel, measured for this run's configuration by two
    child passes of this script under `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` (one
    counter each: the passes stay within the hardware's per-block limits), after this process's
    timed region: per-dispatch averages of `kernel`, FETCH_SIZE x 2 (the gfx950 correction of
    MI355X_MICROARCH.md's HBM section), KiB -> bytes.  None when rocprofv3 is absent or a pass
    fails (the line then falls back to profiles/pmc_traffic.json)."""
    import csv
    import shutil
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return None
    tmp = tempfile.mkdtemp(prefix="ysb_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    got = {}
    try:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            out = os.path.join(tmp, counter)
            cmd = ["timeout", "-s", "KILL", "150", prof, "--pmc", counter, "--output-format", "csv", "-d", out,
                   "-o", "run", "--", sys.executable, os.path.abspath(__file__), "--steps", "3", "--warmup", "1",
                   "--no-cpu", "--no-check", "--no-extras", "--no-live-traffic", "--events", str(args.events),
                   "--segment", str(args.segment), "--rate", str(args.rate)]
            if args.per_batch:
                cmd.append("--per-batch")
            r = subprocess.run(cmd, cwd=tmp, env=env, capture_output=True, text=True, timeout=200)
            if r.returncode != 0:
                log("live traffic: the %s pass exited %d" % (counter, r.returncode))
                return None
            vals = []
            for fn in os.listdir(out):
                if fn.endswith("counter_collection.csv"):
                    for row in csv.DictReader(open(os.path.join(out, fn))):
                        if row["Kernel_Name"].startswith(kernel) and row["Counter_Name"] == counter:
                            vals.append(float(row["Counter_Value"]))
            if not vals:
                return None
            got[counter] = sum(vals) / len(vals)
    except Exception as e:   # noqa: BLE001 (the constant file is the fallback)
        log("live traffic: %s" % e)
        return None
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    rd, wr = 2 * got["FETCH_SIZE"] * 1024, got["WRITE_SIZE"] * 1024
    return {"hbm_read_bytes_per_launch": int(rd), "hbm_write_bytes_per_launch": int(wr),
            "hbm_bytes_per_launch": int(rd + wr)}


def group_init(ctx, d, args):
    """The keyBy exchange's group: RCCL over the node's GPUs (ysb_group_init), or -- the
    --rehearse-host-collectives rehearsal of the N-rank flow on a box with fewer GPUs, where
    RCCL refuses two ranks on one device -- the same exchange over the ranks' gloo
    collectives on host memory (ysb_group_init_host)."""
    if args.rehearse_host_collectives:
        ctx.group_init_host(d.rank, d.world, d.dist)
        return
    from ysb_amd import YsbContext
    uid = d.bcast_bytes(YsbContext.group_unique_id() if d.rank == 0 else None)
    ctx.group_init(d.rank, d.world, uid)


def exchange_overlap(x):
    """Per step: the reduce-scatter's own time (rs), the part of it the compute stream waited
    for at the unpack (exposed) and the rest, which ran beside the queued launches (hidden)."""
    n = max(x["exchanges"], 1)
    rs, exp = x["rs_ms"] / n, x["exposed_ms"] / n
    return {"rs_ms_per_step": round(rs, 4), "exposed_ms_per_step": round(exp, 4),
            "hidden_ms_per_step": round(max(rs - exp, 0.0), 4)}


def exchange(ctx, last):
    """One step's keyBy exchange: pipelined (no host wait, ysb_group_exchange_pipelined)
    inside the stream, complete on the timed region's last step so every count the timed
    steps made has reached its owner when the clock stops."""
    if last:
        ctx.group_reduce_scatter()
    else:
        ctx.group_exchange_pipelined()


def exchange_check(d, ctx, g, segs, submit_all):
    """After the timed loop (N > 1): one more pass with the generator truth, one
    reduce-scatter, every owner drains its block; rank 0 compares the owners' rows with
    the truth summed over ranks (host gloo, independent of RCCL)."""
    from ysb_amd import exchange_mismatches, table_rows
    ctx.reset()
    submit_all()
    for (f, n, _, _, _) in segs:
        ctx.truth_accumulate(g, f, n)
    ctx.sync()
    mism_local, truth_local, ring_local = ctx.truth_compare()
    truth, ring_lo = ctx.truth_read()
    st = ctx.stats()
    ctx.group_reduce_scatter()
    rows = ctx.drain_buckets()
    lo, hi = ctx.group_owned()
    rrank, rn = ctx.group_info()
    truth_sum = d.sum_array(truth)
    los = d.gather(ring_lo)
    per = d.gather((lo, hi, rows, rrank, rn, int(st["out_of_ring"])))
    sums = [int(d.sum(v)) for v in (mism_local, truth_local, ring_local, st["parse_errors"], st["deferred"],
                                    st["join_misses"], st["out_of_ring"])]
    if d.rank != 0:
        return None
    expected = table_rows(truth_sum, ring_lo)
    mism, outside, cells = exchange_mismatches(expected, [(p[0], p[1], p[2]) for p in per])
    return {"truth_mismatched_cells": sums[0], "truth_views": sums[1], "counted_views": sums[2],
            "parse_errors": sums[3], "deferred_to_general_path": sums[4], "join_misses": sums[5],
            "out_of_ring": sums[6],
            "note": "truth_* / counted_views: sum over ranks of each rank's table vs its own truth, before the "
                    "exchange; exchange: the owners' rows after the RCCL reduce-scatter vs the truth summed "
                    "over ranks",
            "exchange": {"post_exchange_mismatched_cells": mism, "cells_compared": cells,
                         "owner_rows_outside_block": outside,
                         "owned_views": int(sum(sum(p[2].values()) for p in per)),
                         "truth_views_summed": int(truth_sum.sum()),
                         "ring_bases_equal": len(set(los)) == 1,
                         "rccl_ranks": sorted(set(p[4] for p in per)), "rccl_user_ranks": [p[3] for p in per],
                         "owned_blocks": [[p[0], p[1]] for p in per]}}


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # launcher: nothing here touches a GPU before the ranks are started
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    d = Dist(args.gpus)
    if args.dry_run:
        dry_run(d, args)
        return
    d.resolve_device()
    from ysb_amd import GenParams, YsbContext, shard_ads

    base = GenParams(seed=42, n_campaigns=100, ads_per_campaign=10, events_per_sec=args.rate)
    cids, aids = base.ids()
    camp = base.ad_campaign_index()
    W = 1024
    ring_base = None
    if d.world > 1:
        subset = shard_ads(aids, d.world)[d.rank]
        g = GenParams(seed=42, event_stream=1 + d.rank, n_campaigns=100, ads_per_campaign=10,
                      events_per_sec=args.rate, ad_subset=subset)
        # every rank derives the same ring base from the shared t0 (the library would also
        # agree on one at ysb_group_init / the first exchange)
        ring_base = g.c.t0_ms // 10000 - W // 8
    else:
        g = base

    ctx = YsbContext(device=d.device, n_campaigns=100, window_ring=W, timing=True, ring_base_bucket=ring_base,
                     max_batch_bytes=16 << 20, max_batch_events=1 << 16, layout_auto=not args.layout_fixed)
    # N > 1: the input is sharded by ad_id hash, so each rank holds only its shard of the
    # join table; the post-exchange check proves nothing is missed
    ctx.load_ad_map(aids, camp, shard=(d.rank, d.world) if d.world > 1 else None)
    if d.world > 1:
        group_init(ctx, d, args)

    # ---- resident input: generated straight into HBM ----------------------------------
    t_gen = time.perf_counter()
    segs = gen_segments(ctx, g, args.events, args.segment)
    total_bytes = sum(s[3] for s in segs)
    log("rank %d: generated %d events, %.2f GB in %.1f s" % (d.rank, args.events, total_bytes / 1e9,
                                                            time.perf_counter() - t_gen))

    def submit_all():
        if args.per_batch:
            for (_, n, d_b, nb, d_o) in segs:
                ctx.submit_device(d_b, nb, d_o, n)
        else:
            ctx.submit_device_segments([(d_b, nb, d_o, n) for (_, n, d_b, nb, d_o) in segs])
    launches_per_step = len(segs) if args.per_batch else 1

    def step(last=False):
        submit_all()
        if d.world > 1:
            exchange(ctx, last)

    device_sync(d.device)
    for _ in range(args.warmup):
        step()
    ctx.sync()
    ctx.kernel_time()   # discard warmup launches
    if d.world > 1:
        ctx.exchange_info(reset=True)
    device_sync(d.device)
    d.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i == args.steps - 1)
    ctx.sync()
    device_sync(d.device)
    d.barrier()
    el = d.max(time.perf_counter() - t0)
    kms, launches = ctx.kernel_time()
    xinfo = ctx.exchange_info(reset=True) if d.world > 1 else None
    layout_run = ctx.launch_info()["layout"]

    events_all = args.events * d.world * args.steps
    value = events_all / el
    alg_bytes_launch = (total_bytes + 4 * args.events) / launches_per_step   # B = L_json + 4 per event
    avg_launch_ms = kms / max(launches, 1)
    achieved = alg_bytes_launch / (avg_launch_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic):
        try:
            tj = json.load(open(args.traffic))
            if (tj.get("segment_events") == args.segment and tj.get("events_per_sec") == args.rate
                    and tj.get("events_per_gpu", 100_000_000) == args.events
                    and tj.get("launches_per_step", 6) == launches_per_step):
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    check = None
    if not args.no_check:
        if d.world > 1:
            check = exchange_check(d, ctx, g, segs, submit_all)
        else:
            ctx.reset()
            submit_all()
            for (f, n, d_b, nb, d_o) in segs:
                ctx.truth_accumulate(g, f, n)
            ctx.sync()
            mism, truth, ring = ctx.truth_compare()
            st = ctx.stats()
            check = {"truth_mismatched_cells": mism, "truth_views": truth, "counted_views": ring,
                     "parse_errors": st["parse_errors"], "out_of_ring": st["out_of_ring"],
                     "deferred_to_general_path": st["deferred"], "join_misses": st["join_misses"]}

    cpu = None
    if d.rank == 0 and d.world == 1 and not args.no_cpu:
        s0 = segs[0]
        cpu = cpu_baseline(ctx, s0[2], s0[4], s0[3], s0[1], aids, camp, args.cpu_sample, args.cpu_seconds)

    traffic_source = "profiles/pmc_traffic.json (PMC passes of this configuration, tools/final_profile.sh)"
    # (not when this process runs under rocprofv3 itself: a profiler started from a profiled
    # process would exec its program from a process whose GPU is already initialised)
    profiled = any(k.startswith("ROCPROF_") for k in os.environ)
    if d.world == 1 and not args.no_live_traffic and not profiled:
        lt = live_traffic(args, "void ysb::scan_kernel<false, false, false, %d>" % layout_run)
        if lt:
            traffic = lt["hbm_bytes_per_launch"]
            traffic_source = ("measured in this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE child passes of this "
                              "configuration, per-dispatch averages, FETCH_SIZE x 2 (gfx950); read %d B, write %d B"
                              % (lt["hbm_read_bytes_per_launch"], lt["hbm_write_bytes_per_launch"]))
    if traffic is None:
        traffic_source = None

    out = None
    if d.rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "events/s", "n_gpus": d.world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: seeded generator, data/ core.clj:90-97 line format, generated in HBM",
            "config": {"workload": ("configs[1]: %dM JSON events per GPU, 100 campaigns x 10 ads, 10 s windows"
                                    % (args.events // 1_000_000)) if d.world == 1 else
                                   ("configs[3] layout at weak scaling: %dM JSON events per GPU (%dM total), "
                                    "events sharded by ad_id hash, RCCL reduce-scatter of (campaign, window) counts"
                                    % (args.events // 1_000_000, args.events * d.world // 1_000_000)),
                       "events_per_gpu": args.events, "campaigns": 100, "ads": 1000,
                       "event_time_rate_per_s": args.rate, "batches_per_step": len(segs),
                       "launches_per_step": launches_per_step,
                       "json_bytes_per_event": round(total_bytes / args.events, 3),
                       "parallelism": ("ad_id-hash shards x%d, %s" % (d.world, "REHEARSAL: gloo host collectives, ranks "
                                                                     "sharing the box's GPUs (not a measurement)"
                                                                     if args.rehearse_host_collectives else
                                                                     "RCCL reduce-scatter")) if d.world > 1
                       else "1 GPU"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_source,
                         "kernel": "ysb::scan_kernel<false, false, false, %d>" % layout_run,
                         "avg_launch_ms": round(avg_launch_ms, 4),
                         "alg_bytes_per_launch": int(alg_bytes_launch)},
            "cpu_baseline": cpu,
            "check": check,
        }
        if xinfo is not None:
            out["exchange"] = {"ms_per_step": round(xinfo["ms"] / max(xinfo["exchanges"], 1), 4),
                               "critical_ms_per_step": round(xinfo["critical_ms"] / max(xinfo["exchanges"], 1), 4),
                               **exchange_overlap(xinfo),
                               "bytes_per_step_per_gpu": xinfo["bytes"] // max(xinfo["exchanges"], 1),
                               "buckets": xinfo["last_buckets"], "cell_bytes": xinfo["last_width"],
                               "whole_ring_u64_bytes": xinfo["full_ring_bytes"]}
    extra = None if args.no_extras else {}
    import threading
    printed_lock, printed = threading.Lock(), []
    if not args.no_extras:
        free_segments(ctx, segs)
        ctx.close()
        if d.world == 1:
            extra.update(extras(args, d.device))
        else:
            # a rank that stopped inside a collective of the leg would hold every rank (and
            # the headline line) forever: after --extras-timeout seconds rank 0 prints the
            # headline with the leg marked timed out and every rank exits
            def give_up():
                with printed_lock:
                    if d.rank == 0 and not printed:
                        extra["timed_out"] = {"error": "the N > 1 extras timed out after %d s"
                                                                 % args.extras_timeout}
                        emit(out, extra, args.extras_out)
                        printed.append(True)
                # every rank's watchdog fires at the same deadline, so every rank leaves (one
                # stuck in a collective too); 0: the headline line is valid, the leg's timeout is
                # recorded in it
                os._exit(0)
            dog = threading.Timer(args.extras_timeout, give_up)
            dog.daemon = True
            dog.start()
            guarded(extra, "config3", lambda: config3_ranks(args, d))
            # configs[4] across the node's GPUs: rank 0 runs the native streaming mode with one
            # shard per rank's GPU (a process of its own; the other ranks are done with theirs)
            if d.rank == 0 and args.stream_seconds > 0:
                guarded(extra, "stream_native", lambda: extra_stream_native(args, 0, shards=d.world))
            dog.cancel()

    with printed_lock:   # (the watchdog may print the line instead, never both)
        if d.rank == 0 and not printed:
            emit(out, extra, args.extras_out)
            printed.append(True)
    if d.dist:
        d.dist.destroy_process_group()


if __name__ == "__main__":
    main()
