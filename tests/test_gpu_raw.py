"""GPU: raw batches (ABI 3) -- the line split on the GPU (ysb_split_lines_device,
ysb_submit_raw; FileBasedDataSource.run's BufferedReader.readLine,
AdvertisingTopologyNative.java:144-165) against readLine's split restated in
oracle/dostats.split_lines, and the chain's counts through raw submits equal to the golden
fixtures and the C oracle; plus the device batches' layout sample taken in stream order
after a producer on another stream."""
import numpy as np
import pytest

import golden_data as gd
from oracle import dostats, oracle
from ysb_amd import GEN_COMPACT, GEN_REORDER, GenParams, YsbContext
from test_gpu_parity import check_against, make_ctx

pytestmark = pytest.mark.gpu

CHUNK = 65536   # ysb_split.hip SPLIT_CHUNK


def gpu_split(ctx, data):
    """Line starts of `data` by ysb_split_lines_device."""
    d_b = ctx.device_alloc(len(data) + 64)
    cap = len(data) + 1
    d_o = ctx.device_alloc(4 * cap + 64)
    try:
        if data:
            ctx.h2d(d_b, np.frombuffer(data, dtype=np.uint8))
        n = ctx.split_lines_device(d_b, len(data), d_o, cap)
        out = ctx.d2h(np.empty(n, dtype=np.uint32), d_o) if n else np.empty(0, dtype=np.uint32)
        return out.tolist()
    finally:
        ctx.device_free(d_b)
        ctx.device_free(d_o)


def random_text(rng, n, p_term):
    """n bytes of printable text with '\\n', '\\r' and "\\r\\n" terminators at rate p_term."""
    b = rng.integers(0x20, 0x7F, size=n, dtype=np.uint8)
    t = rng.random(n) < p_term
    b[t] = rng.choice(np.frombuffer(b"\n\r\n\r", dtype=np.uint8), size=int(t.sum()))
    return b.tobytes()


SMALL = [b"", b"\n", b"a", b"a\n", b"\r", b"\r\n", b"\n\r", b"a\rb", b"a\r\nb\r", b"\n\n\r\r\n", b"\r\r\r",
         b"x" * 15 + b"\r" + b"\n" + b"y", b"x" * 16 + b"\r\n", b"x" * 31 + b"\n", b"{}\r\n{}\n{}"]


def test_split_small_cases_match_readline():
    with YsbContext() as ctx:
        for data in SMALL:
            assert gpu_split(ctx, data) == dostats.split_lines(data)[1], data


@pytest.mark.parametrize("seed,n,p", [(1, 1000, 0.05), (2, 3 * CHUNK + 17, 0.004), (3, 2 * CHUNK, 0.3),
                                      (4, 5 * CHUNK + 1, 0.0), (5, 700_001, 0.01)])
def test_split_random_text_matches_readline(seed, n, p):
    rng = np.random.default_rng(seed)
    data = random_text(rng, n, p)
    with YsbContext() as ctx:
        assert gpu_split(ctx, data) == dostats.split_lines(data)[1]


def test_split_terminators_on_vector_and_chunk_edges():
    """'\\r' / "\\r\\n" / '\\n' on either side of every 16-byte vector and 64-KiB chunk edge
    (the '\\r' test reads the next vector's first byte)."""
    data = bytearray(b"z" * (3 * CHUNK + 64))
    for edge in (16, 32, 48, CHUNK, 2 * CHUNK, 3 * CHUNK):
        data[edge - 1:edge + 1] = b"\r\n"
    for edge in (64, CHUNK + 16):
        data[edge - 1] = ord("\r")
    for edge in (80, 2 * CHUNK + 16):
        data[edge] = ord("\r")
    data[CHUNK + 33] = ord("\n")
    data[-1] = ord("\r")   # a terminator that ends the batch starts no line
    data = bytes(data)
    with YsbContext() as ctx:
        assert gpu_split(ctx, data) == dostats.split_lines(data)[1]


def test_split_capacity_is_reported():
    with YsbContext() as ctx:
        data = b"a\nb\nc\nd\n"
        d_b, d_o = ctx.device_alloc(64), ctx.device_alloc(64)
        ctx.h2d(d_b, np.frombuffer(data, dtype=np.uint8))
        from ysb_amd import YsbError
        with pytest.raises(YsbError):
            ctx.split_lines_device(d_b, len(data), d_o, 2)
        assert ctx.split_lines_device(d_b, len(data), d_o, 4) == 4
        ctx.device_free(d_b)
        ctx.device_free(d_o)


def test_split_generator_batch_equals_generator_offsets():
    g = GenParams(seed=11, events_per_sec=100_000)
    n = 1_000_000
    with YsbContext() as ctx:
        cap = n * g.max_line_bytes()
        d_b, d_o, d_s = ctx.device_alloc(cap), ctx.device_alloc(4 * n + 64), ctx.device_alloc(4 * n + 64)
        nb = ctx.gen_events_device(g, 0, n, d_b, cap, d_o)
        assert ctx.split_lines_device(d_b, nb, d_s, n) == n
        want = ctx.d2h(np.empty(n, dtype=np.uint32), d_o)
        got = ctx.d2h(np.empty(n, dtype=np.uint32), d_s)
        assert np.array_equal(want, got)
        for d in (d_b, d_o, d_s):
            ctx.device_free(d)


@pytest.mark.parametrize("stem,require_ip", gd.FIXTURES)
def test_raw_submit_fixture(stem, require_ip):
    raw, _ = gd.events(stem)
    with make_ctx(require_ip=require_ip) as ctx:
        ctx.submit_raw(raw, slot=0)
        check_against(ctx, *gd.expected(stem, require_ip))


@pytest.mark.parametrize("stem", sorted(gd.TBL_FILES))
def test_raw_submit_tbl_fixture(stem):
    raw, _ = gd.tbl_events(stem)
    with make_ctx(input_format="tbl") as ctx:
        ctx.submit_raw(raw, slot=1)
        check_against(ctx, *gd.expected(stem))


def test_raw_batches_alternate_slots_and_mix_with_other_submits():
    """The gen_s7 fixture cut at line boundaries into raw batches over both slots, with an
    offsets batch (ysb_submit) and a device batch in between: the batches launch in order and
    the counts equal the fixture's."""
    raw, offs = gd.events("gen_s7")
    cuts = [0, 1, 2, 300, 301, 900, 1200, len(offs)]
    ends = list(offs) + [len(raw)]
    with make_ctx(max_batch_bytes=1 << 20) as ctx:
        for k in range(len(cuts) - 1):
            a, b = ends[cuts[k]], ends[cuts[k + 1]]
            piece = raw[a:b]
            if k == 3:   # offsets batch
                ctx.submit(piece, [o - a for o in offs[cuts[k]:cuts[k + 1]]], slot=k & 1)
            elif k == 5:   # device batch
                d_b = ctx.device_alloc(len(piece) + 64)
                d_o = ctx.device_alloc(4 * (cuts[k + 1] - cuts[k]) + 64)
                ctx.h2d(d_b, np.frombuffer(piece, dtype=np.uint8))
                ctx.h2d(d_o, np.asarray([o - a for o in offs[cuts[k]:cuts[k + 1]]], dtype=np.uint32))
                ctx.submit_device(d_b, len(piece), d_o, cuts[k + 1] - cuts[k])
                ctx.sync()
                ctx.device_free(d_b)
                ctx.device_free(d_o)
            else:
                ctx.submit_raw(piece, slot=k & 1)
        ctx.submit_raw(b"", slot=0)   # an empty raw batch: no lines
        check_against(ctx, *gd.expected("gen_s7"))
        assert ctx.stats()["events"] == len(offs)


def test_raw_crlf_and_lone_cr_lines_match_oracle():
    """Generator lines re-terminated with "\\r\\n" and lone '\\r' (readLine takes both), some
    blank lines (parse errors), through raw batches of 20k lines: counts and counters equal
    the C oracle on the same records."""
    g = GenParams(seed=5, events_per_sec=1000)
    _, aids = g.ids()
    camp = g.ad_campaign_index()
    raw, offs = g.events_host(0, 60_000)
    lines = [raw[a:b] for a, b in zip(offs, list(offs[1:]) + [len(raw)])]
    rng = np.random.default_rng(9)
    out = []
    for i, ln in enumerate(lines):
        body = bytes(ln[:-1])
        r = rng.random()
        out.append(body + (b"\r\n" if r < 0.3 else b"\r" if r < 0.5 else b"\n"))
        if i % 997 == 0:
            out.append(b"\n")
    data = b"".join(out)
    _, ref_offs = dostats.split_lines(data)
    rows, ost = oracle.run(oracle.AdMap(aids, camp), data, ref_offs)
    with make_ctx(n_campaigns=100, ads=(aids, camp), max_batch_bytes=8 << 20) as ctx:
        ends = ref_offs + [len(data)]
        for k, a in enumerate(range(0, len(ref_offs), 20_000)):
            b = min(a + 20_000, len(ref_offs))
            ctx.submit_raw(data[ends[a]:ends[b]], slot=k & 1)
        st = ctx.stats()
        for k, v in ost.items():
            assert st[k] == v, (k, st[k], v)
        assert st["events"] == len(ref_offs)
        assert ctx.drain_buckets() == rows


def _hip():
    """The HIP runtime libysb_hip.so itself loaded (same instance: its streams and events are
    the library's)."""
    import ctypes as C
    from ysb_amd import lib
    lib()
    h = C.CDLL("/opt/rocm/lib/libamdhip64.so.7")
    for f, args in (("hipStreamCreate", [C.c_void_p]), ("hipStreamDestroy", [C.c_void_p]),
                    ("hipEventCreate", [C.c_void_p]), ("hipEventDestroy", [C.c_void_p]),
                    ("hipEventRecord", [C.c_void_p, C.c_void_p]),
                    ("hipStreamWaitEvent", [C.c_void_p, C.c_void_p, C.c_uint]),
                    ("hipMemsetAsync", [C.c_void_p, C.c_int, C.c_size_t, C.c_void_p]),
                    ("hipMemcpyAsync", [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]),
                    ("hipStreamSynchronize", [C.c_void_p]), ("hipDeviceSynchronize", [])):
        getattr(h, f).argtypes = args
        getattr(h, f).restype = C.c_int
    return h


def test_device_sample_follows_a_producer_on_another_stream():
    """A compact-JSON batch written into its device buffer by a copy queued on another stream
    behind ~6 GB of memsets (the producer is still running when the batch is submitted); the
    compute stream waits for the producer's event (hipStreamWaitEvent(ysb_stream(ctx), ...),
    the documented contract) and the batch is submitted at once.  The layout sample runs in
    stream order, so it sees the compact lines (layout 1), not the reordered-key lines the
    buffer held before, and the counts equal the C oracle's.  Since
    ABI 4 the first launch on a busy stream takes the per-tile dispatch instead of waiting for
    its own sample; an idle stream's launch then reads its own sample (compact: layout 1)."""
    import ctypes as C
    hip = _hip()
    D2D = 3
    gc = GenParams(seed=21, events_per_sec=1000, variant=GEN_COMPACT)
    gr = GenParams(seed=21, events_per_sec=1000, variant=GEN_REORDER)
    _, aids = gc.ids()
    camp = gc.ad_campaign_index()
    n = 20_000
    raw_c, off_c = gc.events_host(0, n)
    raw_r, off_r = gr.events_host(0, n)
    rows, ost = oracle.run(oracle.AdMap(aids, camp), raw_c.tobytes(), off_c.tolist())
    with make_ctx(n_campaigns=100, ads=(aids, camp)) as ctx:
        size = max(raw_c.size, raw_r.size) + 64
        d_b, d_o = ctx.device_alloc(size), ctx.device_alloc(4 * n + 64)
        s_b, s_o = ctx.device_alloc(size), ctx.device_alloc(4 * n + 64)
        junk_n = 6 << 30
        junk = ctx.device_alloc(junk_n)
        ctx.h2d(d_b, raw_r)                      # stale content: another layout
        ctx.h2d(d_o, off_r)
        ctx.h2d(s_b, raw_c)                      # what the producer will copy in
        ctx.h2d(s_o, off_c)
        side, ev = C.c_void_p(), C.c_void_p()
        assert hip.hipStreamCreate(C.byref(side)) == 0 and hip.hipEventCreate(C.byref(ev)) == 0
        for _ in range(4):                       # the producer is still queued ...
            assert hip.hipMemsetAsync(C.c_void_p(junk), 0, junk_n, side) == 0
        assert hip.hipMemcpyAsync(C.c_void_p(d_b), C.c_void_p(s_b), int(raw_c.size), D2D, side) == 0
        assert hip.hipMemcpyAsync(C.c_void_p(d_o), C.c_void_p(s_o), 4 * n, D2D, side) == 0
        assert hip.hipEventRecord(ev, side) == 0
        assert hip.hipStreamWaitEvent(C.c_void_p(ctx.stream()), ev, 0) == 0
        ctx.submit_device(d_b, int(raw_c.size), d_o, n)   # ... when the batch is submitted
        # the stream is busy and no earlier sample exists: the per-tile dispatch, no host wait
        # (ABI 4; it takes the compact lines' tiles by their own path)
        assert ctx.launch_info()["layout"] == 4
        st = ctx.stats()
        for k, v in ost.items():
            assert st[k] == v, (k, st[k], v)
        assert ctx.drain_buckets() == rows
        assert hip.hipStreamSynchronize(side) == 0
        ctx.reset()
        ctx.submit_device(d_b, int(raw_c.size), d_o, n)   # idle stream: its own sample
        assert ctx.launch_info()["layout"] == 1
        assert ctx.drain_buckets() == rows
        hip.hipEventDestroy(ev)
        hip.hipStreamDestroy(side)
        for d in (d_b, d_o, s_b, s_o, junk):
            ctx.device_free(d)


def _producer_batches(n):
    """The same events as three producers write them (the generator's layout, reordered keys,
    compact JSON), each a device batch, with the C oracle's counts of each."""
    from ysb_amd import GEN_REORDER as R, GEN_COMPACT as CP
    out = []
    for v in (0, R, CP):
        g = GenParams(seed=33, events_per_sec=2000, variant=v)
        raw, off = g.events_host(0, n)
        out.append((raw, off))
    g0 = GenParams(seed=33, events_per_sec=2000)
    _, aids = g0.ids()
    return out, aids, g0.ad_campaign_index()


@pytest.mark.parametrize("busy", [True, False])
def test_alternating_producers_on_a_busy_stream(busy):
    """Device batches whose producers alternate per batch (generator layout, reordered keys,
    compact JSON, twice round) submitted back to back.  busy: a 2 GB memset is queued on the
    compute stream before every submit, so each launch is decided on the previous launch's
    sample: the first launch takes the per-tile dispatch (no earlier
    sample, no host wait), the second the previous sample's layout (nothing older to compare),
    every later one the dispatch (the last two samples disagree).  Idle (a sync after each
    submit): every launch reads its own sample -- 0, 3, 1.  Counts equal the C oracle's on
    the whole stream either way."""
    import ctypes as C
    hip = _hip()
    n = 60_000
    batches, aids, camp = _producer_batches(n)
    seq = [0, 1, 2, 0, 1, 2]
    allraw = b"".join(batches[i][0].tobytes() for i in seq)
    offs, base = [], 0
    for i in seq:
        offs.extend(int(o) + base for o in batches[i][1])
        base += batches[i][0].size
    rows, ost = oracle.run(oracle.AdMap(aids, camp), allraw, offs, threads=8)
    with make_ctx(n_campaigns=100, ads=(aids, camp)) as ctx:
        dev = []
        for raw, off in batches:
            d_b, d_o = ctx.device_alloc(raw.size + 64), ctx.device_alloc(4 * n + 64)
            ctx.h2d(d_b, raw)
            ctx.h2d(d_o, off)
            dev.append((d_b, int(raw.size), d_o))
        junk_n = 2 << 30
        junk = ctx.device_alloc(junk_n)
        stream = C.c_void_p(ctx.stream())
        ctx.sync()
        layouts = []
        for i in seq:
            if busy:
                assert hip.hipMemsetAsync(C.c_void_p(junk), 0, junk_n, stream) == 0
            d_b, nb, d_o = dev[i]
            ctx.submit_device(d_b, nb, d_o, n)
            layouts.append(ctx.launch_info()["layout"])
            if not busy:
                ctx.sync()
        st = ctx.stats()
        got = ctx.drain_buckets()
        for d_b, _, d_o in dev:
            ctx.device_free(d_b)
            ctx.device_free(d_o)
        ctx.device_free(junk)
    assert layouts == ([4, 0, 4, 4, 4, 4] if busy else [0, 3, 1, 0, 3, 1]), layouts
    for k, v in ost.items():
        assert st[k] == v, (k, st[k], v)
    assert st["deferred"] == 0
    assert got == rows


def test_raw_batch_over_its_line_capacity_is_a_sticky_error():
    """A raw batch with more lines than its slot holds (max(max_batch_events,
    max_batch_bytes / 32): here 40,000 blank lines in a 1 MiB slot that holds 32,769) is
    dropped at its launch with YSB_ERR_CAPACITY; the error is returned by every later call that
    would order work after it (ysb_sync, ysb_stream gives NULL) until ysb_reset, after which
    batches count again (a failed deferred launch was silently lost)."""
    from ysb_amd import YsbError
    from ysb_amd._lib import lib
    raw, offs = gd.events("gen_s7")
    with make_ctx(max_batch_bytes=1 << 20, max_batch_events=1000) as ctx:
        ctx.submit_raw(b"\n" * 40_000, slot=0)
        with pytest.raises(YsbError) as e:
            ctx.sync()
        assert e.value.code == -4 and "lines" in str(e.value)
        with pytest.raises(YsbError):
            ctx.submit(raw, offs, slot=1)
        assert lib().ysb_stream(ctx._h) is None
        with pytest.raises(YsbError):
            ctx.sync()
        ctx.reset()
        ctx.submit_raw(raw, slot=1)
        check_against(ctx, *gd.expected("gen_s7"))
