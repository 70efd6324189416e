"""GPU: ABI 5 -- zero-copy raw batches read in place from registered host memory
(ysb_host_register / ysb_submit_raw_mapped: FileBasedDataSource.run's batches,
AdvertisingTopologyNative.java:144-165, with the source's own buffer pinned), the replay's
event-time rebasing on the device (ysb_rebase_table: the data/ generator's lines played past
their first cycle, core.clj:166-174), the timing records' folding, and the library's behaviour
when another HIP runtime (torch's) opened the GPU first."""
import os
import subprocess
import sys

import numpy as np
import pytest

from ysb_amd import GenParams, YsbContext, YsbError

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
T0 = 1_700_000_000_000
ET_KEY = b'"event_time": "'


def aligned(nbytes):
    """A 64-byte aligned uint8 array of nbytes (+ 64 B slack)."""
    buf = np.zeros(nbytes + 192, dtype=np.uint8)
    a = (-buf.ctypes.data) % 64
    return buf[a:a + nbytes + 64]


def layout_batches(data, off, n_batches):
    """The lines cut into n_batches batches at line boundaries, each placed 16-byte aligned in
    one array: (array, [(byte offset, nbytes, first line, lines)])."""
    n = off.size
    cuts = [n * i // n_batches for i in range(n_batches + 1)]
    ends = np.append(off[1:], len(data)).astype(np.int64)
    parts, pos = [], 0
    for i in range(n_batches):
        a, b = cuts[i], cuts[i + 1]
        nb = int(ends[b - 1] - off[a])
        parts.append((pos, nb, a, b - a))
        pos += (nb + 15) // 16 * 16 + 16
    buf = aligned(pos)
    for (p, nb, a, _) in parts:
        buf[p:p + nb] = data[off[a]:off[a] + nb]
    return buf, parts


def time_table(data, off):
    """Per line: offset of its 13 event_time digits | (bucket index << 16), and the base
    bucket (the replay runner's table, host/ysb_stream.cpp build_cycle)."""
    raw = bytes(data)
    ends = list(off[1:]) + [len(raw)]
    pos, lead = [], []
    for s, e in zip(off, ends):
        k = raw.index(ET_KEY, s, e) + len(ET_KEY)
        pos.append(k - s)
        lead.append(int(raw[k:k + 9]))
    lead = np.asarray(lead, dtype=np.int64)
    base = int(lead.min())
    return (np.asarray(pos, dtype=np.uint32) | ((lead - base).astype(np.uint32) << 16)), base


def ctx_for(g, **kw):
    c = YsbContext(n_campaigns=100, window_ring=1024, ring_base_bucket=T0 // 10000 - 8, timing=True, **kw)
    _, aids = g.ids()
    c.load_ad_map(aids, g.ad_campaign_index())
    return c


def submit_mapped(ctx, buf, parts, rebase_shift=None):
    for i, (p, nb, a, _) in enumerate(parts):
        ctx.submit_raw_mapped(buf, p, nb, slot=i % 2,
                              rebase=None if rebase_shift is None else (a, rebase_shift))
    ctx.sync()


def test_mapped_batches_count_like_copied_ones():
    g = GenParams(events_per_sec=100_000, with_skew=2)
    data, off = g.events_host(0, 120_000)
    buf, parts = layout_batches(data, off, 5)
    with ctx_for(g) as a, ctx_for(g) as b:
        a.host_register(buf)
        submit_mapped(a, buf, parts)
        for i, (p, nb, _, _) in enumerate(parts):
            b.submit_raw(buf[p:p + nb], slot=i % 2)
        b.sync()
        got = a.drain()
        assert got == b.drain() and sum(got.values()) > 0
        assert a.stats()["events"] == off.size and a.stats()["parse_errors"] == 0
        a.truth_accumulate(g, 0, off.size)
        mism, truth, ring = a.truth_compare()
        assert mism == 0 and truth == ring
        a.host_unregister(buf)


@pytest.mark.parametrize("shift", [0, 1, 37])
def test_rebase_moves_every_event_by_whole_buckets(shift):
    """Every line's leading nine event_time digits rewritten on the device: the counts equal
    the generator truth of the same events with t0 moved by shift x 10 s, and no line broke."""
    g = GenParams(events_per_sec=100_000, with_skew=2)
    data, off = g.events_host(0, 100_000)
    tab, base = time_table(data, off)
    buf, parts = layout_batches(data, off, 4)
    with ctx_for(g) as ctx:
        ctx.host_register(buf)
        ctx.rebase_table(tab, base)
        submit_mapped(ctx, buf, parts, rebase_shift=shift)
        st = ctx.stats()
        assert st["parse_errors"] == 0 and st["deferred"] == 0 and st["events"] == off.size
        gs = GenParams(events_per_sec=100_000, with_skew=2, t0_ms=T0 + shift * 10_000)
        ctx.truth_accumulate(gs, 0, off.size)
        mism, truth, ring = ctx.truth_compare()
        assert mism == 0 and truth == ring and truth > 0
    # the source bytes themselves are never written (the rebase runs on the device copy)
    assert bytes(buf[parts[0][0]:parts[0][0] + parts[0][1]]) == bytes(data[:parts[0][1]])


@pytest.mark.parametrize("shift", [None, 5])
def test_mapped_batches_with_device_offsets(shift):
    """ysb_submit_mapped: the same batches with their line offsets already in HBM (no split):
    counts equal the raw-mapped path's and the generator truth, rebased or not."""
    g = GenParams(events_per_sec=100_000, with_skew=2)
    data, off = g.events_host(0, 150_000)
    tab, base = time_table(data, off)
    buf, parts = layout_batches(data, off, 6)
    # every line's offset within its batch (what the replay runner keeps in HBM per cycle)
    lo = np.empty(off.size, dtype=np.uint32)
    for (p, nb, a, n) in parts:
        lo[a:a + n] = off[a:a + n] - off[a]
    with ctx_for(g) as ctx:
        ctx.host_register(buf)
        ctx.rebase_table(tab, base)
        d_lo = ctx.device_alloc(lo.nbytes + 64)
        ctx.h2d(d_lo, lo)
        for i, (p, nb, a, n) in enumerate(parts):
            ctx.submit_mapped(buf, p, nb, d_lo + 4 * a, n, slot=i % 2,
                              rebase=None if shift is None else (a, shift))
        ctx.sync()
        st = ctx.stats()
        assert st["events"] == off.size and st["parse_errors"] == 0 and st["deferred"] == 0
        gs = GenParams(events_per_sec=100_000, with_skew=2, t0_ms=T0 + (shift or 0) * 10_000)
        ctx.truth_accumulate(gs, 0, off.size)
        mism, truth, ring = ctx.truth_compare()
        assert mism == 0 and truth == ring and truth > 0
        with pytest.raises(YsbError, match="YSB_ERR_ARG"):   # lines past the rebase table
            ctx.submit_mapped(buf, parts[-1][0], parts[-1][1], d_lo, off.size, rebase=(1, 0))
        ctx.device_free(d_lo)


def test_mapped_argument_errors():
    g = GenParams(events_per_sec=100_000)
    data, off = g.events_host(0, 2000)
    buf, parts = layout_batches(data, off, 1)
    other = aligned(1 << 16)
    with ctx_for(g) as ctx:
        with pytest.raises(YsbError, match="YSB_ERR_ARG"):
            ctx.submit_raw_mapped(buf, 0, parts[0][1])          # not registered
        ctx.host_register(buf)
        with pytest.raises(YsbError, match="YSB_ERR_ARG"):
            ctx.host_register(buf[16:])                          # overlaps
        with pytest.raises(YsbError, match="YSB_ERR_ARG"):
            ctx.submit_raw_mapped(buf, buf.size - 8, 16)         # past the range's end
        with pytest.raises(YsbError, match="YSB_ERR_ARG"):
            ctx.submit_raw_mapped(buf, 0, buf.size + 64)         # past the registered range
        with pytest.raises(YsbError, match="YSB_ERR_STATE"):
            ctx.submit_raw_mapped(buf, 0, parts[0][1], rebase=(0, 1))   # no rebase table
        ctx.host_register(other)
        ctx.host_unregister(other)
        tab, base = time_table(data, off)
        ctx.rebase_table(tab[:100], base)                         # fewer lines than the batch holds
        ctx.submit_raw_mapped(buf, 0, parts[0][1], rebase=(0, 1))
        with pytest.raises(YsbError, match="rebase table"):
            ctx.sync()                                           # the launch fails, sticky until reset


def test_unaligned_batches_back_to_back():
    """A file mapping's batches (the native runner's mapped FileBasedDataSource): cut at line
    boundaries and submitted where they lie, back to back at every byte alignment -- the copy
    kernel's shifted path (launch_h2d_copy_unaligned).  Counts equal the copied batches' and
    the generator truth; no line broke."""
    g = GenParams(events_per_sec=100_000, with_skew=2)
    data, off = g.events_host(0, 60_000)
    ends = np.append(off[1:], len(data)).astype(np.int64)
    rng = np.random.default_rng(7)
    cuts = np.unique(np.concatenate([[0, off.size], rng.integers(1, off.size, 40), np.arange(1, 40)]))
    for lead in (0, 3, 8, 15):   # the whole file's start alignment
        buf = aligned(len(data) + 32)
        buf[lead:lead + len(data)] = data
        with ctx_for(g) as a, ctx_for(g) as b:
            a.host_register(buf)
            shifts = set()
            for i, (x, y) in enumerate(zip(cuts[:-1], cuts[1:])):
                p, nb = lead + int(off[x]), int(ends[y - 1] - off[x])
                shifts.add(p % 16)
                a.submit_raw_mapped(buf, p, nb, slot=i % 2)
                b.submit_raw(buf[p:p + nb], slot=i % 2)
            a.sync()
            b.sync()
            assert len(shifts) == 16
            got = a.drain()
            assert got == b.drain() and sum(got.values()) > 0
            st = a.stats()
            assert st["events"] == off.size and st["parse_errors"] == 0 and st["deferred"] == 0
            a.truth_accumulate(g, 0, off.size)
            mism, truth, ring = a.truth_compare()
            assert mism == 0 and truth == ring
            a.host_unregister(buf)


def test_unaligned_mapped_with_device_offsets_and_rebase():
    """ysb_submit_mapped of unaligned batches, rebased: the shifted copy feeds the rebase and
    the scan the same bytes as an aligned one."""
    g = GenParams(events_per_sec=100_000, with_skew=2)
    data, off = g.events_host(0, 50_000)
    tab, base = time_table(data, off)
    ends = np.append(off[1:], len(data)).astype(np.int64)
    cuts = [0, 1, 2, 3, 777, 5000, 12345, 30001, 49999, off.size]
    lo = np.empty(off.size, dtype=np.uint32)
    for x, y in zip(cuts[:-1], cuts[1:]):
        lo[x:y] = off[x:y] - off[x]
    buf = aligned(len(data) + 32)
    buf[5:5 + len(data)] = data
    with ctx_for(g) as ctx:
        ctx.host_register(buf)
        ctx.rebase_table(tab, base)
        d_lo = ctx.device_alloc(lo.nbytes + 64)
        ctx.h2d(d_lo, lo)
        for i, (x, y) in enumerate(zip(cuts[:-1], cuts[1:])):
            ctx.submit_mapped(buf, 5 + int(off[x]), int(ends[y - 1] - off[x]), d_lo + 4 * x, y - x,
                              slot=i % 2, rebase=(x, 3))
        ctx.sync()
        st = ctx.stats()
        assert st["events"] == off.size and st["parse_errors"] == 0 and st["deferred"] == 0
        gs = GenParams(events_per_sec=100_000, with_skew=2, t0_ms=T0 + 30_000)
        ctx.truth_accumulate(gs, 0, off.size)
        mism, truth, ring = ctx.truth_compare()
        assert mism == 0 and truth == ring and truth > 0
        ctx.device_free(d_lo)


def test_mapped_range_is_checked_at_16_byte_boundaries():
    """The copy reads whole 16-byte vectors: a batch whose widened span leaves the registered
    range is refused even when its own bytes are inside."""
    g = GenParams(events_per_sec=100_000)
    data, off = g.events_host(0, 100)
    buf = aligned(len(data) + 64)
    buf[8:8 + len(data)] = data
    view = buf[8:8 + len(data)]                                    # starts 8 bytes past a boundary
    with ctx_for(g) as ctx:
        ctx.host_register(view)
        with pytest.raises(YsbError, match="registered range"):
            ctx.submit_raw_mapped(view, 0, len(data))
        ctx.host_unregister(view)
        ctx.host_register(buf)
        ctx.submit_raw_mapped(buf, 8, len(data))
        ctx.sync()
        assert ctx.stats()["events"] == off.size and ctx.stats()["parse_errors"] == 0


@pytest.mark.parametrize("cap", [777, 64 << 10, 256 << 20])
def test_file_source_in_place_equals_oracle(tmp_path, cap):
    """ysb_amd.FileBasedDataSource.run: a file with every readLine terminator, its mapping
    registered and every batch submitted in place (any byte alignment): the counts and stats
    equal the oracle's over readLine's records (oracle/dostats), and the generator's own file
    equals its truth."""
    import golden_data as gd
    from oracle import dostats
    from ysb_amd import FileBasedDataSource
    raw, _ = gd.events("gen_s7")
    lines = raw.split(b"\n")[:-1]
    seps = [b"\n", b"\r\n", b"\r", b"\r\r", b"\n\n", b"\r\n\r", b"\n"]
    data = b"".join(ln + seps[i % len(seps)] for i, ln in enumerate(lines)) + lines[1][:-2]
    ev = tmp_path / "mixed.jsonl"
    ev.write_bytes(data)
    want = dostats.run(dostats.split_lines(data)[0], gd.ad_map())
    cidx = gd.campaign_index()
    with YsbContext(n_campaigns=len(cidx), max_batch_bytes=max(cap, 4096)) as ctx:
        ctx.load_ad_map(*gd.ad_arrays())
        with FileBasedDataSource(str(ev)) as src:
            assert src.run(ctx, cap) == len(data) and src.batches >= 1
        st = ctx.stats()
        assert st["events"] == want.events and st["parse_errors"] == want.parse_errors
        got = {(c, w // 10000): n for (c, w), n in ctx.drain().items()}
        assert got == {(cidx[c], b): n for (c, b), n in want.counts.items()}


def test_timing_records_are_folded():
    """YSB_F_TIMING with many launches and no kernel_time call in between (a streaming job):
    the records are folded into totals (TIMING_KEEP = 256 pending at most), every launch and
    copy still counted once."""
    g = GenParams(events_per_sec=100_000)
    data, off = g.events_host(0, 3000)
    buf, parts = layout_batches(data, off, 1)
    n = 700
    with ctx_for(g) as ctx:
        ctx.host_register(buf)
        for i in range(n):
            ctx.submit_raw_mapped(buf, 0, parts[0][1], slot=i % 2)
        ctx.sync()
        ms, launches = ctx.kernel_time()
        cms, copies, cbytes = ctx.copy_time()
        assert launches == n and ms > 0
        assert copies == n and cbytes == n * parts[0][1] and cms > 0
        assert ctx.stats()["events"] == n * off.size


def test_library_after_torch_opened_the_gpu():
    """Weak 6 of the round-5 review: torch bundles another HIP runtime.  With torch's opened
    first, the library either opens a context (the runtimes coexist on this box) or fails with
    the error that names the cause -- never a bare 'no HIP device'."""
    script = (
        "import sys; sys.path[:0] = [%r, %r]\n"
        "import torch\n"
        "ok = torch.cuda.is_available()\n"
        "if ok:\n"
        "    torch.zeros(1, device='cuda'); torch.cuda.synchronize()\n"
        "print('TORCH', ok, flush=True)\n"
        "from ysb_amd import YsbContext, YsbError, device_sync\n"
        "try:\n"
        "    with YsbContext() as c:\n"
        "        device_sync(0)\n"
        "    print('OPEN', flush=True)\n"
        "except YsbError as e:\n"
        "    print('ERR', e, flush=True)\n" % (ROOT, os.path.join(ROOT, "streaming-benchmarks_amd")))
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.strip().splitlines()
    assert lines[0].startswith("TORCH")
    last = lines[-1]
    assert last == "OPEN" or ("another HIP/HSA runtime" in last and "INTEGRATION.md" in last), last
    print(lines)
