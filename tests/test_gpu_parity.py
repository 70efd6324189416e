"""GPU parity: the HIP path (through the C ABI) against the golden fixtures and the
CPU oracle, bit-exact on every (campaign, window) count and every counter."""
import numpy as np
import pytest

import golden_data as gd
from oracle import oracle
from ysb_amd import GenParams, YsbContext, YsbError

pytestmark = pytest.mark.gpu


def make_ctx(n_campaigns=10, ads=None, **kw):
    ctx = YsbContext(n_campaigns=n_campaigns, **kw)
    a, c = ads if ads is not None else gd.ad_arrays()
    ctx.load_ad_map(a, c)
    return ctx


def check_against(ctx, exp_rows, exp_st):
    got = ctx.drain_buckets()
    st = ctx.stats()
    for k, v in exp_st.items():
        assert st[k] == v, (k, st[k], v)
    assert st["overflow_dropped"] == 0
    assert got == exp_rows


@pytest.mark.parametrize("stem,require_ip", gd.FIXTURES)
@pytest.mark.parametrize("lds", [True, False])
def test_fixture_host_submit(stem, require_ip, lds):
    with make_ctx(require_ip=require_ip, lds_count=lds) as ctx:
        raw, offs = gd.events(stem)
        ctx.submit(raw, offs, slot=0)
        check_against(ctx, *gd.expected(stem, require_ip))


@pytest.mark.parametrize("stem,require_ip", gd.FIXTURES)
def test_fixture_device_submit(stem, require_ip):
    with make_ctx(require_ip=require_ip) as ctx:
        raw, offs = gd.events(stem)
        d_b = ctx.device_alloc(len(raw) + 64)
        d_o = ctx.device_alloc(4 * len(offs) + 64)
        ctx.h2d(d_b, np.frombuffer(raw, dtype=np.uint8))
        ctx.h2d(d_o, np.asarray(offs, dtype=np.uint32))
        ctx.submit_device(d_b, len(raw), d_o, len(offs))
        check_against(ctx, *gd.expected(stem, require_ip))
        ctx.device_free(d_b)
        ctx.device_free(d_o)


def split_batches(raw, offs, sizes):
    offs = list(offs) + [len(raw)]
    i = 0
    for s in sizes:
        j = min(i + s, len(offs) - 1)
        base = offs[i]
        yield raw[base:offs[j]], [o - base for o in offs[i:j]]
        i = j
    if i < len(offs) - 1:
        base = offs[i]
        yield raw[base:], [o - base for o in offs[i:-1]]


def test_batches_and_slots_sum_exactly():
    raw, offs = gd.events("gen_s7")
    with make_ctx() as ctx:
        for k, (b, o) in enumerate(split_batches(raw, offs, [1, 0, 7, 255, 256, 257, 300, 3])):
            ctx.submit(b, o, slot=k & 1)
        check_against(ctx, *gd.expected("gen_s7"))
        assert ctx.stats()["batches"] >= 9


def test_slot_buffers_zero_copy():
    raw, offs = gd.events("gen_s7")
    with make_ctx() as ctx:
        import ctypes as C
        for k, (b, o) in enumerate(split_batches(raw, offs, [600, 600])):
            slot = k & 1
            ctx.wait(slot)
            pb, po = ctx.slot_buffers(slot)
            C.memmove(pb, b, len(b))
            oa = np.asarray(o, dtype=np.uint32)
            C.memmove(po, oa.ctypes.data, oa.nbytes)
            from ysb_amd._lib import lib
            lib().ysb_submit(ctx._h, slot, C.c_void_p(pb), len(b), C.c_void_p(po), len(o))
        check_against(ctx, *gd.expected("gen_s7"))


def test_device_generator_matches_fixture_bytes():
    p = gd.gen_params()
    g = GenParams(seed=p["seed"], n_campaigns=p["n_campaigns"], ads_per_campaign=p["ads_per_campaign"],
                  t0_ms=p["t0_ms"], events_per_sec=p["events_per_sec"], with_skew=p["with_skew"])
    raw, offs = gd.events("gen_s7")
    with make_ctx() as ctx:
        n = p["n_events"]
        cap = n * g.max_line_bytes()
        d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n)
        nb = ctx.gen_events_device(g, 0, n, d_b, cap, d_o)
        assert nb == len(raw)
        got = ctx.d2h(np.empty(nb, dtype=np.uint8), d_b)
        got_off = ctx.d2h(np.empty(n, dtype=np.uint32), d_o)
        assert got.tobytes() == raw
        assert list(got_off) == offs


@pytest.mark.parametrize("rate,skew,ring", [(100, True, 4096), (100_000, False, 1024), (7, True, 16)])
def test_generated_stream_vs_oracle(rate, skew, ring):
    """2M events straight from the device generator vs the C oracle on the same bytes;
    ring 16 forces most windows through the exact side list."""
    g = GenParams(seed=1234, events_per_sec=rate, with_skew=skew)
    cids, aids = g.ids()
    camp = g.ad_campaign_index()
    n = 2_000_000
    with make_ctx(n_campaigns=100, ads=(aids[:950], camp[:950]), window_ring=ring,
                  overflow_capacity=1 << 22, max_batch_bytes=1 << 30) as ctx:
        cap = n * g.max_line_bytes()
        d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n)
        nb = ctx.gen_events_device(g, 0, n, d_b, cap, d_o)
        ctx.submit_device(d_b, nb, d_o, n)
        got = ctx.drain_buckets()
        st = ctx.stats()
        data = ctx.d2h(np.empty(nb, dtype=np.uint8), d_b)
        off = ctx.d2h(np.empty(n, dtype=np.uint32), d_o)
    rows, ost = oracle.run(oracle.AdMap(aids[:950], camp[:950]), data, off, threads=8)
    for k, v in ost.items():
        assert st[k] == v, (k, st[k], v)
    assert st["join_misses"] > 0 and st["overflow_dropped"] == 0
    assert st["deferred"] == 0          # generator lines all take the fast path
    assert got == rows


def test_sparse_fast_join_defers_misses_exactly():
    """Half the 36-byte keys left out of the fast-path cuckoo table (as a failed
    placement would): their views take the general path, counts unchanged."""
    g = GenParams(seed=99, events_per_sec=1000, with_skew=True)
    cids, aids = g.ids()
    camp = g.ad_campaign_index()
    n = 500_000
    with make_ctx(n_campaigns=100, ads=(aids[:900], camp[:900]), sparse_fast_join=True,
                  max_batch_bytes=1 << 28) as ctx:
        cap = n * g.max_line_bytes()
        d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n)
        nb = ctx.gen_events_device(g, 0, n, d_b, cap, d_o)
        ctx.submit_device(d_b, nb, d_o, n)
        got = ctx.drain_buckets()
        st = ctx.stats()
        data = ctx.d2h(np.empty(nb, dtype=np.uint8), d_b)
        off = ctx.d2h(np.empty(n, dtype=np.uint32), d_o)
    rows, ost = oracle.run(oracle.AdMap(aids[:900], camp[:900]), data, off, threads=8)
    for k, v in ost.items():
        assert st[k] == v, (k, st[k], v)
    assert st["deferred"] > 0 and st["join_misses"] > 0
    assert got == rows


@pytest.mark.parametrize("stem,require_ip", gd.FIXTURES)
def test_fixture_sparse_fast_join(stem, require_ip):
    with make_ctx(require_ip=require_ip, sparse_fast_join=True) as ctx:
        raw, offs = gd.events(stem)
        ctx.submit(raw, offs, slot=0)
        check_against(ctx, *gd.expected(stem, require_ip))


def test_truth_counts_at_scale():
    """30M generated events in 15M-event (3.8 GB) batches -- byte offsets past 2^31 --:
    parsed counts == generator truth (no parsing), and every line on the fast path."""
    g = GenParams(seed=77, events_per_sec=100_000)
    n, seg = 30_000_000, 15_000_000
    with make_ctx(n_campaigns=100, ads=(g.ids()[1], g.ad_campaign_index())) as ctx:
        cap = seg * g.max_line_bytes()
        d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * seg)
        for first in range(0, n, seg):
            nb = ctx.gen_events_device(g, first, seg, d_b, cap, d_o)
            ctx.submit_device(d_b, nb, d_o, seg)
            ctx.sync()
            ctx.truth_accumulate(g, first, seg)
        mism, truth, ring = ctx.truth_compare()
        st = ctx.stats()
    assert st["events"] == n and st["parse_errors"] == 0 and st["out_of_ring"] == 0
    assert st["deferred"] == 0
    assert mism == 0 and truth == ring == st["joined"]


def test_single_rank_group_reduce_scatter():
    raw, offs = gd.events("gen_s7")
    with make_ctx() as ctx:
        ctx.group_init(0, 1, YsbContext.group_unique_id())
        assert ctx.group_owned() == (0, 10)
        ctx.submit(raw[:offs[700]], offs[:700])
        ctx.group_reduce_scatter()
        ctx.submit(raw[offs[700]:], [o - offs[700] for o in offs[700:]], slot=1)
        check_against(ctx, *gd.expected("gen_s7"))


def test_drain_clear_and_ranges():
    raw, offs = gd.events("gen_s7")
    exp, _ = gd.expected("gen_s7")
    with make_ctx() as ctx:
        ctx.submit(raw, offs)
        lo, w = ctx.ring_range()
        buckets = sorted({b for _, b in exp})
        mid = buckets[len(buckets) // 2]
        first = ctx.drain(bucket_hi=mid, clear=True)
        assert {(c, t // 10000): v for (c, t), v in first.items()} == {k: v for k, v in exp.items() if k[1] < mid}
        rest = ctx.drain_buckets()
        assert rest == {k: v for k, v in exp.items() if k[1] >= mid}


def test_misaligned_device_pointer_rejected():
    with make_ctx() as ctx:
        d = ctx.device_alloc(1024)
        with pytest.raises(YsbError):
            ctx.submit_device(d + 3, 100, d, 1)


def test_submit_before_ad_map_is_an_error():
    with YsbContext(n_campaigns=10) as ctx:
        with pytest.raises(YsbError):
            ctx.submit(b"{}\n", [0])


@pytest.mark.parametrize("stem", gd.TBL_FIXTURES)
def test_tbl_fixture(stem):
    """The fork's .tbl rows (YSB_F_FORMAT_TBL) against the golden expectations."""
    ads, camp = gd.ad_arrays()
    raw, offs = gd.tbl_events(stem)
    with YsbContext(n_campaigns=10, input_format="tbl") as ctx:
        ctx.load_ad_map(ads, camp)
        ctx.submit(raw, offs)
        check_against(ctx, *gd.expected(stem))


def test_tbl_generated_stream_vs_oracle():
    g = GenParams(seed=13, n_campaigns=50, ads_per_campaign=10, events_per_sec=1000, with_skew=True)
    raw, offs = g.events_host_tbl(0, 200_000)
    _, aids = g.ids()
    rows, st = oracle.run(oracle.AdMap(aids, g.ad_campaign_index()), raw, offs, fmt="tbl", threads=8)
    with YsbContext(n_campaigns=50, window_ring=64, input_format="tbl", max_batch_bytes=64 << 20,
                    max_batch_events=1 << 18) as ctx:
        ctx.load_ad_map(aids, g.ad_campaign_index())
        ctx.submit(raw, offs)
        assert ctx.drain_buckets() == rows
        s = ctx.stats()
        for k, v in st.items():
            assert s[k] == v, k


def _oracle_vs_gpu(lines, require_ip, lds=True, fmt="json", ad_map=None, **ctx_kw):
    """Submits the lines as one batch; on a mismatch, bisects to the first line whose
    GPU counters differ from the C oracle's (for the failure message)."""
    ads, camp = ad_map or gd.ad_arrays()
    am = oracle.AdMap(ads, camp)

    def run_gpu(ls):
        raw = b"".join(ls)
        offs = np.cumsum([0] + [len(x) for x in ls[:-1]]).tolist()
        with make_ctx(ads=(ads, camp), require_ip=require_ip, lds_count=lds, input_format=fmt, **ctx_kw) as ctx:
            ctx.submit(raw, offs, slot=0)
            rows = ctx.drain_buckets()
            st = ctx.stats()
        return rows, {k: st[k] for k in ("events", "views", "joined", "join_misses", "parse_errors", "time_errors")}

    def run_cpu(ls):
        raw = b"".join(ls)
        offs = np.cumsum([0] + [len(x) for x in ls[:-1]]).tolist()
        return oracle.run(am, raw, offs, require_ip=require_ip, fmt=fmt)

    if run_gpu(lines) == run_cpu(lines):
        return
    lo, hi = 0, len(lines)   # first prefix length that differs
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if run_gpu(lines[:mid]) == run_cpu(lines[:mid]):
            lo = mid
        else:
            hi = mid
    bad = lines[hi - 1]
    raise AssertionError("GPU differs from the oracle at line %d: %r gpu=%r cpu=%r"
                         % (hi - 1, bad, run_gpu([bad]), run_cpu([bad])))


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("require_ip", [False, True])
def test_orgjson_fuzz_matches_oracle(seed, require_ip):
    """org.json's grammar (tests/orgjson_fuzz.py) through the general path: every counter
    and every (campaign, window) count equals the C restatement's."""
    import orgjson_fuzz as fz
    ads, _ = gd.ad_arrays()
    _oracle_vs_gpu(fz.lines(seed, 3000, ads), require_ip)


def test_canonical_lines_with_control_bytes_and_trailing_text():
    """The fast path must hand a generator-layout line with a NUL / CR / LF inside a value
    to the general path (org.json throws there) and must count one with text after '}'."""
    raw, offs = gd.events("gen_s7")
    offs = list(offs) + [len(raw)]
    lines = [raw[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]
    rng = np.random.default_rng(5)
    out = []
    for i, ln in enumerate(lines[:600]):
        r = i % 6
        if r == 1:                                   # a control byte inside some value
            quotes = [k for k, c in enumerate(ln) if c == 0x22]
            vals = [(quotes[k] + 1, quotes[k + 1]) for k in range(2, len(quotes) - 1, 4)]
            a, b = vals[rng.integers(len(vals))]
            p = int(rng.integers(a, b + 1))
            ln = ln[:p] + bytes([int(rng.choice([0x00, 0x0A, 0x0D, 0x09, 0x0B]))]) + ln[p:]
        elif r == 2:                                 # text after the closing brace
            ln = ln[:-1] + rng.choice([b" x", b"}", b"\x00", b"garbage{", b"\r"]) + b"\n"
        out.append(ln)
    _oracle_vs_gpu(out, False)


def test_device_tbl_generator_matches_host():
    g = GenParams(seed=21, with_skew=True, events_per_sec=3000, fmt="tbl")
    raw, offs = g.events_host(0, 300_000)
    with make_ctx() as ctx:
        n = len(offs)
        cap = n * g.max_line_bytes()
        d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n)
        nb = ctx.gen_events_device(g, 0, n, d_b, cap, d_o)
        assert nb == raw.size
        assert ctx.d2h(np.empty(nb, dtype=np.uint8), d_b).tobytes() == raw.tobytes()
        assert np.array_equal(ctx.d2h(np.empty(n, dtype=np.uint32), d_o), offs)


@pytest.mark.parametrize("seed", [1, 2])
def test_tbl_mutations_match_oracle(seed):
    """.tbl rows through the fast path and, mutated, through the deferred path: extra or
    missing '|', '}' after a '|' (a SWAR false candidate), CR / CRLF / no terminator,
    empty fields, long rows, non-digit times -- every counter equals the C oracle's."""
    g = GenParams(seed=7, n_campaigns=10, ads_per_campaign=10, fmt="tbl", events_per_sec=1000)
    _, aids = g.ids()
    amap = (aids, list(g.ad_campaign_index()))
    raw, offs = g.events_host(0, 4000)
    raw = raw.tobytes()
    bounds = list(offs) + [len(raw)]
    rows = [raw[bounds[i]:bounds[i + 1]] for i in range(len(offs))]
    rng = np.random.default_rng(seed)
    out = []
    for r in rows:
        k = int(rng.integers(12))
        body = r[:-1]
        if k == 1:
            p = int(rng.integers(len(body) + 1))
            body = body[:p] + b"|" + body[p:]
        elif k == 2:
            p = int(rng.integers(len(body)))
            body = body[:p] + body[p + 1:]
        elif k == 3:
            bars = [i for i, c in enumerate(body) if c == 0x7C]
            p = bars[int(rng.integers(len(bars)))] + 1
            body = body[:p] + b"}" + body[p:]
        elif k == 4:
            body = body + b"\r"
        elif k == 5:
            body = body.replace(b"|view|", b"||") if rng.integers(2) else body + b"|"
        elif k == 6:
            body = body + b"|x" * int(rng.integers(1, 12))
        elif k == 7:
            body = body[:-3] + bytes([int(rng.choice([0x41, 0x2D, 0x2B, 0x20]))]) + body[-2:]
        elif k == 8:
            body = body.replace(b"|", b"||", 1)
        out.append(body + (b"" if k == 9 else b"\n"))
    _oracle_vs_gpu(out, False, fmt="tbl", ad_map=amap)
    _oracle_vs_gpu(out, False, lds=False, fmt="tbl", ad_map=amap)


@pytest.mark.parametrize("seed", [3, 4])
def test_tbl_vocabulary_edges_match_oracle(seed):
    """The .tbl fast path names ad_type / event_type from the generator's sets and wants 13
    digits to the row's end: rows with near-miss values (other lengths, one byte off, a
    '|' inside, other time lengths, signs) take the bitmap branch or the deferred path --
    every counter equals the C oracle's."""
    g = GenParams(seed=9, n_campaigns=10, ads_per_campaign=10, fmt="tbl", events_per_sec=1000)
    _, aids = g.ids()
    amap = (aids, list(g.ad_campaign_index()))
    raw, offs = g.events_host(0, 3000)
    raw = raw.tobytes()
    bounds = list(offs) + [len(raw)]
    rows = [raw[bounds[i]:bounds[i + 1]] for i in range(len(offs))]
    ad_types = [b"banner", b"modal", b"sponsored-search", b"mail", b"mobile", b"banners", b"mai", b"mobilE",
                b"sponsored-searcX", b"sponsored-search-2", b"", b"x", b"b|nner", b"modal}", b"maiL"]
    ev_types = [b"view", b"click", b"purchase", b"vie", b"views", b"clic", b"clickk", b"purchas", b"purchasee",
                b"View", b"", b"v|ew"]
    rng = np.random.default_rng(seed)
    out = []
    for r in rows:
        f = r[:-1].split(b"|")
        k = int(rng.integers(6))
        if k == 1:
            f[3] = ad_types[int(rng.integers(len(ad_types)))]
        elif k == 2:
            f[4] = ev_types[int(rng.integers(len(ev_types)))]
        elif k == 3:
            t = f[5]
            f[5] = [t[:-1], t + b"7", b"-" + t[1:], b"+" + t[1:], t[:6] + b"|" + t[7:], t[:12] + b" ",
                    t[:12] + b"/"][int(rng.integers(7))]
        elif k == 4:
            f[3] = ad_types[int(rng.integers(len(ad_types)))]
            f[4] = ev_types[int(rng.integers(len(ev_types)))]
        out.append(b"|".join(f) + b"\n")
    _oracle_vs_gpu(out, False, fmt="tbl", ad_map=amap)
    _oracle_vs_gpu(out, False, lds=False, fmt="tbl", ad_map=amap)


def test_vocabulary_fast_path_edges_match_oracle():
    """Generator-layout lines whose ad_type / event_type / event_time / ip_address leave
    the generator's vocabulary (or hide a quote / backslash / control byte in it) must
    reach the general parser; every counter equals the C oracle's."""
    raw, offs = gd.events("gen_s7")
    bounds = list(offs) + [len(raw)]
    lines = [raw[bounds[i]:bounds[i + 1]] for i in range(len(offs))]
    subs = [
        (b'"ad_type": "banner"', [b'"ad_type": "bannerX"', b'"ad_type": "banne"', b'"ad_type": "Banner"',
                                  b'"ad_type": "ban\\"er"', b'"ad_type": "b\\u0061nner"', b'"ad_type": "bann\x00r"']),
        (b'"ad_type": "mail"', [b'"ad_type": "mai"', b'"ad_type": "maill"', b'"ad_type": "mobile"',
                                b'"ad_type": "moda"', b'"ad_type": "modal"']),
        (b'"ad_type": "sponsored-search"', [b'"ad_type": "sponsored-searcH"', b'"ad_type": "sponsored-searc"']),
        (b'"event_type": "view"', [b'"event_type": "viewx"', b'"event_type": "vie"', b'"event_type": "click"',
                                   b'"event_type": "purchase"', b'"event_type": "v\\"ew"', b'"event_type": "vi\rw"']),
        (b'"event_type": "click"', [b'"event_type": "clicks"', b'"event_type": "view"', b'"event_type": "clock"']),
        (b'"event_type": "purchase"', [b'"event_type": "purchas"', b'"event_type": "purchasE"']),
        (b'"ip_address": "1.2.3.4"', [b'"ip_address": "1.2.3.5"', b'"ip_address": "1.2.3.4 "',
                                      b'"ip_address": "1.2.3.4", "x": 1', b'"ip_address": 1.2']),
    ]
    rng = np.random.default_rng(11)
    out = []
    for i, ln in enumerate(lines):
        if i % 3 == 0:
            cands = [(a, b) for a, bs in subs if a in ln for b in bs]
            a, b = cands[int(rng.integers(len(cands)))]
            ln = ln.replace(a, b)
        elif i % 3 == 1:                              # the 13 time bytes: length, sign, non-digits
            j = ln.index(b'"event_time": "') + 15
            k = ln.index(b'"', j)
            t = ln[j:k]
            t = [t[:-1], t + b"7", b"-" + t[1:], t[:5] + b"\"" + t[6:], t[:5] + b"a" + t[6:],
                 t[:5] + b"\\" + t[6:], t[:7] + b"\x00" + t[8:], t[:12] + b" "][int(rng.integers(8))]
            ln = ln[:j] + t + ln[k:]
        out.append(ln)
    _oracle_vs_gpu(out, False)
    _oracle_vs_gpu(out, True, lds=False)


def _flat_lines(seed, n):
    """Generator events re-laid as flat objects: keys in a random order, whitespace and
    ',' / ';' separators as nextClean sees them, a separator before '}' -- the general
    path's flat tier -- plus, in about a third of the lines, one change that must send the
    line to org.json's full machine (a repeated / unknown / missing key, a non-string or
    single-quoted value, an escape, a control byte, NUL, a missing ':' ...)."""
    raw, offs = gd.events("gen_s7")
    bounds = list(offs) + [len(raw)]
    import json
    evs = [json.loads(raw[bounds[i]:bounds[i + 1]]) for i in range(len(offs))]
    rng = np.random.default_rng(seed)
    ws = ["", "", " ", "  ", "\t", "\x01", "\x1f ", "\r\n"]
    times = ["1700000000000", "-5", "+17", "01700000000000", "9223372036854775807", "9223372036854775808", "1e3", ""]
    out = []
    for i in range(n):
        ev = dict(evs[i % len(evs)])
        if rng.random() < 0.2:
            ev["event_time"] = times[int(rng.integers(len(times)))]
        if rng.random() < 0.2:
            ev["event_type"] = ["view", "click", "View", "view "][int(rng.integers(4))]
        keys = list(ev)
        rng.shuffle(keys)
        pairs = [[k, v] for k, v in ((k, ev[k]) for k in keys)]
        mut = int(rng.integers(30))
        w = lambda: ws[int(rng.integers(len(ws)))]
        def q(s):
            return '"' + s + '"'
        parts = None
        if mut == 0:
            pairs.append(list(pairs[int(rng.integers(len(pairs)))]))          # repeated key
        elif mut == 1:
            pairs.insert(int(rng.integers(len(pairs) + 1)), ["extra", "x"])   # another key
        elif mut == 2:
            del pairs[int(rng.integers(len(pairs)))]                           # missing key
        elif mut == 3:
            j = int(rng.integers(len(pairs)))
            parts = (j, "value", "'" + pairs[j][1] + "'")                     # single-quoted value
        elif mut == 4:
            j = int(rng.integers(len(pairs)))
            parts = (j, "value", pairs[j][1] or "1")                          # unquoted value
        elif mut == 5:
            j = int(rng.integers(len(pairs)))
            parts = (j, "key", q(pairs[j][0][:1] + "\\u00" + "%02x" % ord(pairs[j][0][1]) + pairs[j][0][2:]))
        elif mut == 6:
            j = int(rng.integers(len(pairs)))
            parts = (j, "value", q(pairs[j][1][:2] + "\\/" + pairs[j][1][2:]))
        elif mut == 7:
            j = int(rng.integers(len(pairs)))
            parts = (j, "value", q(pairs[j][1][:1] + ["\x00", "\r", "\x02", "\x7f"][int(rng.integers(4))] + pairs[j][1][1:]))
        elif mut == 8:
            j = int(rng.integers(len(pairs)))
            parts = (j, "sep", "=")                                             # no ':'
        elif mut == 9:
            j = int(rng.integers(len(pairs)))
            parts = (j, "value", '{"a": "b"}')                                  # nested value
        body = []
        for j, (k, v) in enumerate(pairs):
            ks, vs, sep = q(k), q(v), ":"
            if parts and parts[0] == j:
                if parts[1] == "value":
                    vs = parts[2]
                elif parts[1] == "key":
                    ks = parts[2]
                else:
                    sep = parts[2]
            body.append(w() + ks + w() + sep + w() + vs + w())
        sepc = [",", ";"]
        line = w() + "{" + "".join(b + (sepc[int(rng.integers(2))] if j + 1 < len(body) else "")
                                   for j, b in enumerate(body))
        if rng.random() < 0.2:
            line += sepc[int(rng.integers(2))] + w()                            # separator before '}'
        line += "}"
        if mut == 10:
            line += ["x", " {", "}", "\x00junk"][int(rng.integers(4))]           # after '}': not read
        elif mut == 11:
            line = line[: int(rng.integers(len(line)))]                          # truncated
        out.append(line.encode("utf-8") + b"\n")
    return out


@pytest.mark.parametrize("seed", [21, 22])
def test_flat_tier_matches_oracle(seed):
    """The general path's flat tier (ysb_scan.hip flat_line) and its hand-offs to the
    org.json machine: every counter and count equals the C oracle's."""
    lines = _flat_lines(seed, 6000)
    _oracle_vs_gpu(lines, False)
    _oracle_vs_gpu(lines, True)
    # the flat-first instantiation (YSB_F_FLAT_FIRST: the flat tier is the scan's only stage)
    _oracle_vs_gpu(lines, False, flat_first=True)
    _oracle_vs_gpu(lines, True, flat_first=True)
