"""GPU: the canonical tiers of the scan kernel -- lines the vocabulary fast path rejects
(other ip addresses, ad_types, event_types, event_time lengths; compact JSON) parsed in
the scan itself instead of the general path -- exact against the CPU oracle (org.json's
grammar restated) and the generator truth, with nothing deferred; and the same with the
layout hints (YSB_F_COMPACT_FIRST: the tiers reordered; YSB_F_FLAT_FIRST: the flat-object
tier as the only stage; YSB_F_LAYOUT_AUTO: the instantiation named by each host batch's
first line)."""
import numpy as np
import pytest

from oracle import oracle
from ysb_amd import GEN_COMPACT, GEN_MORE_AD_TYPES, GEN_RANDOM_IP, GEN_REORDER, GenParams, YsbContext

pytestmark = pytest.mark.gpu


def hint_kw(hint):
    """None: the default (each batch's first line picks the instantiation); "fixed": no
    sampling (the generator's layout first); else an explicit layout hint."""
    if hint is None:
        return {}
    if hint == "fixed":
        return {"layout_auto": False}
    return {hint: True}

VARIANTS = [GEN_RANDOM_IP, GEN_MORE_AD_TYPES, GEN_RANDOM_IP | GEN_MORE_AD_TYPES, GEN_COMPACT,
            GEN_COMPACT | GEN_RANDOM_IP, GEN_COMPACT | GEN_RANDOM_IP | GEN_MORE_AD_TYPES,
            GEN_REORDER, GEN_REORDER | GEN_COMPACT | GEN_RANDOM_IP]


@pytest.mark.parametrize("hint", [None, "compact_first", "flat_first", "fixed"])
@pytest.mark.parametrize("variant", VARIANTS)
def test_tier_lines_exact_and_not_deferred(variant, hint):
    g = GenParams(seed=23, n_campaigns=50, ads_per_campaign=10, events_per_sec=1000, with_skew=True,
                  variant=variant)
    _, aids = g.ids()
    raw, offs = g.events_host(0, 150_000)
    exp, est = oracle.run(oracle.AdMap(aids, g.ad_campaign_index()), raw, offs)
    with YsbContext(n_campaigns=50, window_ring=256, max_batch_bytes=raw.size + 64,
                    max_batch_events=offs.size + 1, **hint_kw(hint)) as ctx:
        ctx.load_ad_map(aids, g.ad_campaign_index())
        ctx.submit(raw, offs)
        got = ctx.drain_buckets()
        st = ctx.stats()
    assert got == exp
    for k, v in est.items():
        assert st[k] == v, k
    assert st["deferred"] == 0                # every line taken by a scan tier


@pytest.mark.parametrize("variant,hint", [(GEN_RANDOM_IP | GEN_MORE_AD_TYPES, None), (GEN_COMPACT | GEN_RANDOM_IP, None),
                                          (GEN_COMPACT | GEN_RANDOM_IP, "compact_first"), (0, "compact_first"),
                                          (GEN_RANDOM_IP | GEN_MORE_AD_TYPES, "flat_first"), (0, "flat_first"),
                                          (GEN_REORDER, None), (GEN_REORDER | GEN_RANDOM_IP, "flat_first")])
def test_tier_device_generator_truth(variant, hint):
    g = GenParams(seed=42, n_campaigns=100, ads_per_campaign=10, events_per_sec=100_000, variant=variant)
    _, aids = g.ids()
    n = 4_000_000
    hraw, _ = g.events_host(0, 20_000)
    with YsbContext(n_campaigns=100, window_ring=1024, **hint_kw(hint)) as ctx:
        ctx.load_ad_map(aids, g.ad_campaign_index())
        cap = n * g.max_line_bytes()
        d_b, d_o = ctx.device_alloc(cap), ctx.device_alloc(4 * n + 64)
        nb = ctx.gen_events_device(g, 0, n, d_b, cap, d_o)
        # the device generator writes the host generator's bytes
        assert (ctx.d2h(np.empty(hraw.size, dtype=np.uint8), d_b) == hraw).all()
        ctx.submit_device(d_b, nb, d_o, n)
        ctx.truth_accumulate(g, 0, n)
        mism, truth, ring = ctx.truth_compare()
        st = ctx.stats()
    assert mism == 0 and truth == ring > 0
    assert st["deferred"] == 0 and st["parse_errors"] == 0 and st["join_misses"] == 0


@pytest.mark.parametrize("hint", [None, "compact_first", "flat_first", "fixed"])
def test_tier_mixed_with_off_template_lines(hint):
    """Tier lines, vocabulary lines and general-path lines (whitespace, escapes, other key
    orders) interleaved in one batch: still exactly the oracle."""
    g0 = GenParams(seed=5, n_campaigns=20, ads_per_campaign=5, events_per_sec=100)
    g1 = GenParams(seed=5, n_campaigns=20, ads_per_campaign=5, events_per_sec=100,
                   variant=GEN_COMPACT | GEN_RANDOM_IP | GEN_MORE_AD_TYPES)
    _, aids = g0.ids()
    a, _ = g0.events_host(0, 3000)
    b, _ = g1.events_host(0, 3000)
    la = bytes(a).split(b"\n")[:-1]
    lb = bytes(b).split(b"\n")[:-1]
    odd = [ln.replace(b'", "', b'" , "', 1) if i % 7 == 0 else ln.replace(b'"view"', b'"vi\\u0065w"')
           for i, ln in enumerate(la[:500])]
    lines = []
    for i in range(3000):
        lines.append(la[i] if i % 3 == 0 else lb[i] if i % 3 == 1 else odd[i % 500])
    data = b"\n".join(lines) + b"\n"
    offs = np.zeros(len(lines), dtype=np.uint32)
    offs[1:] = np.cumsum([len(x) + 1 for x in lines[:-1]])
    exp, est = oracle.run(oracle.AdMap(aids, g0.ad_campaign_index()), data, offs)
    with YsbContext(n_campaigns=20, window_ring=64, **hint_kw(hint)) as ctx:
        ctx.load_ad_map(aids, g0.ad_campaign_index())
        ctx.submit(data, offs)
        got = ctx.drain_buckets()
        st = ctx.stats()
    assert got == exp
    for k, v in est.items():
        assert st[k] == v, k
    assert 0 < st["deferred"] <= 1000


@pytest.mark.parametrize("hint", [None, "compact_first", "flat_first", "fixed"])
def test_canonical_tier_other_event_types_and_times(hint):
    """Lines in the generator's layout whose event_type is none of the three or whose
    event_time is not 13 digits (the vocabulary path names both from closed sets) go to
    the canonical tier, not to the general path: exact, nothing deferred."""
    g = GenParams(seed=31, n_campaigns=40, ads_per_campaign=10, events_per_sec=1000,
                  variant=GEN_RANDOM_IP | GEN_MORE_AD_TYPES)
    _, aids = g.ids()
    raw, offs = g.events_host(0, 60_000)
    lines = bytes(raw).split(b"\n")[:-1]
    ets = [b'"impression"', b'"View"', b'"views"', b'""']
    out = []
    for i, ln in enumerate(lines):
        if i % 2 == 0:
            for et in (b'"view"', b'"click"', b'"purchase"'):
                ln = ln.replace(b'"event_type": ' + et, b'"event_type": ' + ets[(i // 2) % 4])
        if i % 3 == 0:
            j = ln.index(b'"event_time": "') + 15
            k = ln.index(b'"', j)
            t = ln[j:k]
            ln = ln[:j] + [t + b"1", t[:-2], b"-" + t, t[:5] + b"x" + t[6:], b"0" + t][(i // 3) % 5] + ln[k:]
        out.append(ln)
    data = b"\n".join(out) + b"\n"
    offs2 = np.zeros(len(out), dtype=np.uint32)
    offs2[1:] = np.cumsum([len(x) + 1 for x in out[:-1]])
    exp, est = oracle.run(oracle.AdMap(aids, g.ad_campaign_index()), data, offs2)
    with YsbContext(n_campaigns=40, window_ring=256, max_batch_bytes=len(data) + 64,
                    max_batch_events=len(out) + 1, **hint_kw(hint)) as ctx:
        ctx.load_ad_map(aids, g.ad_campaign_index())
        ctx.submit(data, offs2)
        got = ctx.drain_buckets()
        st = ctx.stats()
    assert got == exp
    for k, v in est.items():
        assert st[k] == v, k
    assert st["deferred"] == 0 and st["time_errors"] > 0


@pytest.mark.parametrize("variant", [0, GEN_COMPACT, GEN_REORDER, GEN_REORDER | GEN_COMPACT | GEN_RANDOM_IP])
def test_layout_auto_host_batches_exact(variant):
    """YSB_F_LAYOUT_AUTO over host batches whose layouts change from batch to batch (each
    batch's first line names the instantiation; a batch of mixed layouts still counts
    exactly): the oracle's counts."""
    g = GenParams(seed=41, n_campaigns=30, ads_per_campaign=10, events_per_sec=1000, variant=variant)
    g0 = GenParams(seed=42, n_campaigns=30, ads_per_campaign=10, events_per_sec=1000)
    _, aids = g.ids()
    a, _ = g.events_host(0, 6000)
    b, _ = g0.events_host(0, 6000)
    la, lb = bytes(a).split(b"\n")[:-1], bytes(b).split(b"\n")[:-1]
    batches = [la[:2000], lb[:2000], la[2000:4000] + lb[2000:3000], lb[3000:4000] + la[4000:6000]]
    exp_rows, exp_st = oracle.run(oracle.AdMap(aids, g.ad_campaign_index()),
                                  b"".join(b"\n".join(x) + b"\n" for x in batches),
                                  np.cumsum([0] + [len(ln) + 1 for x in batches for ln in x][:-1]).astype(np.uint32))
    with YsbContext(n_campaigns=30, window_ring=64, max_batch_bytes=1 << 22, max_batch_events=1 << 14,
                    layout_auto=True) as ctx:
        ctx.load_ad_map(aids, g.ad_campaign_index())
        for k, x in enumerate(batches):
            data = b"\n".join(x) + b"\n"
            offs = np.cumsum([0] + [len(ln) + 1 for ln in x[:-1]]).astype(np.uint32)
            ctx.submit(data, offs, slot=k & 1)
        got = ctx.drain_buckets()
        st = ctx.stats()
    assert got == exp_rows
    for k, v in exp_st.items():
        assert st[k] == v, k


def _batch(lines):
    data = b"\n".join(lines) + b"\n"
    offs = np.zeros(len(lines), dtype=np.uint32)
    offs[1:] = np.cumsum([len(x) + 1 for x in lines[:-1]])
    return data, offs


@pytest.mark.parametrize("variant", [GEN_REORDER, GEN_REORDER | GEN_COMPACT,
                                     GEN_REORDER | GEN_RANDOM_IP | GEN_MORE_AD_TYPES])
@pytest.mark.parametrize("device", [False, True])
def test_learned_key_order_layout(variant, device):
    """Another key order (the generator's GEN_REORDER lines, also compact and with other
    values): the batch's first line names the order (ysb_capi.cpp learn_layout) and the
    scan runs the learned-order instantiation (layout 3) -- host batches from the pinned
    slot, device batches from a sampled first line -- exact vs the oracle, nothing
    deferred."""
    g = GenParams(seed=29, n_campaigns=60, ads_per_campaign=10, events_per_sec=1000, with_skew=True,
                  variant=variant)
    _, aids = g.ids()
    raw, offs = g.events_host(0, 120_000)
    exp, est = oracle.run(oracle.AdMap(aids, g.ad_campaign_index()), raw, offs)
    with YsbContext(n_campaigns=60, window_ring=256, max_batch_bytes=raw.size + 64,
                    max_batch_events=offs.size + 1) as ctx:
        ctx.load_ad_map(aids, g.ad_campaign_index())
        if device:
            d_b, d_o = ctx.device_alloc(raw.size + 64), ctx.device_alloc(4 * offs.size + 64)
            ctx.h2d(d_b, raw)
            ctx.h2d(d_o, offs)
            ctx.submit_device(d_b, raw.size, d_o, offs.size)
        else:
            ctx.submit(raw, offs)
        assert ctx.launch_info()["layout"] == 3
        got = ctx.drain_buckets()
        st = ctx.stats()
    assert got == exp
    for k, v in est.items():
        assert st[k] == v, k
    assert st["deferred"] == 0


@pytest.mark.parametrize("require_ip", [False, True])
def test_learned_order_with_off_order_lines(require_ip):
    """A batch whose first line is in a learned order, then lines that break it in every way
    the learned check must reject -- another order, other spacing, a missing or an extra
    key, a repeated key, an id value of another length, an escape, a nested value, a
    single-quoted value, text after '}' -- interleaved with lines in the order.  The learned
    instantiation hands each off to the flat tier / the general parser: exactly the
    oracle's counts (with and without YSB_F_REQUIRE_IP)."""
    g = GenParams(seed=37, n_campaigns=20, ads_per_campaign=5, events_per_sec=100, variant=GEN_REORDER)
    g0 = GenParams(seed=37, n_campaigns=20, ads_per_campaign=5, events_per_sec=100)
    _, aids = g.ids()
    a, _ = g.events_host(0, 4000)
    b, _ = g0.events_host(0, 4000)
    la, lb = bytes(a).split(b"\n")[:-1], bytes(b).split(b"\n")[:-1]
    breaks = [
        lambda ln: ln.replace(b'", "', b'","', 1),                                  # other spacing
        lambda ln: ln.replace(b', "ip_address": "1.2.3.4"', b''),                   # a key missing
        lambda ln: ln[:-1] + b', "extra": "x"}',                                    # an extra key
        lambda ln: ln[:-1] + b', "ad_type": "x"}',                                  # a repeated key
        lambda ln: ln.replace(b'"user_id": "', b'"user_id": "z', 1),                # a 37-byte id
        lambda ln: ln.replace(b'"event_type": "view"', b'"event_type": "vi\\u0065w"'),   # an escape
        lambda ln: ln.replace(b'"ip_address": "1.2.3.4"', b'"ip_address": {"a": "1"}'),  # nested
        lambda ln: ln.replace(b'"ad_type": "', b"'ad_type': '", 1).replace(b'", "event_time"', b"', \"event_time\"", 1),
        lambda ln: ln + b' trailing',                                               # text after '}'
        lambda ln: ln.replace(b'{"ad_type"', b'{ "ad_type"', 1),                    # space after '{'
    ]
    # one line in ten off the order (the layout sample -- 64 lines, 46 must agree -- still
    # names the learned order; with 4 producers interleaved it picks the flat tier instead)
    lines = [la[0]]
    for i in range(1, 4000):
        if i % 20 == 0:
            lines.append(breaks[(i // 20) % len(breaks)](la[i]))
        elif i % 20 == 10:
            lines.append(lb[i])                                                     # generator order
        else:
            lines.append(la[i])
    data, offs = _batch(lines)
    am = oracle.AdMap(aids, g.ad_campaign_index())
    exp, est = oracle.run(am, data, offs, require_ip=require_ip) if require_ip else oracle.run(am, data, offs)
    with YsbContext(n_campaigns=20, window_ring=64, max_batch_bytes=len(data) + 64, max_batch_events=len(lines) + 1,
                    require_ip=require_ip) as ctx:
        ctx.load_ad_map(aids, g.ad_campaign_index())
        ctx.submit(data, offs)
        assert ctx.launch_info()["layout"] == 3
        got = ctx.drain_buckets()
        st = ctx.stats()
    assert got == exp
    for k, v in est.items():
        assert st[k] == v, k
    assert st["parse_errors"] > 0 and st["deferred"] > 0


def test_learned_order_subset_of_keys():
    """Lines with only DeserializeBolt's six keys (no ip_address) in another order: a learned
    order of six keys (layout 3); with YSB_F_REQUIRE_IP the same first line cannot name an
    order (ip_address is required) and the flat tier takes the batch (layout 2) -- where
    every line is a parse error, as the Storm deserializer's getString("ip_address") throws."""
    g = GenParams(seed=43, n_campaigns=20, ads_per_campaign=5, events_per_sec=100, variant=GEN_REORDER)
    _, aids = g.ids()
    a, _ = g.events_host(0, 3000)
    lines = [ln.replace(b', "ip_address": "1.2.3.4"', b'') for ln in bytes(a).split(b"\n")[:-1]]
    assert all(b"ip_address" not in ln for ln in lines)
    data, offs = _batch(lines)
    am = oracle.AdMap(aids, g.ad_campaign_index())
    for req in (False, True):
        exp, est = oracle.run(am, data, offs, require_ip=req) if req else oracle.run(am, data, offs)
        with YsbContext(n_campaigns=20, window_ring=64, max_batch_bytes=len(data) + 64,
                        max_batch_events=len(lines) + 1, require_ip=req) as ctx:
            ctx.load_ad_map(aids, g.ad_campaign_index())
            ctx.submit(data, offs)
            assert ctx.launch_info()["layout"] == (2 if req else 3)
            got = ctx.drain_buckets()
            st = ctx.stats()
        assert got == exp
        for k, v in est.items():
            assert st[k] == v, k
        assert (st["parse_errors"] == len(lines)) == req


@pytest.mark.parametrize("variant,fixed,want", [(GEN_REORDER, False, 3), (0, False, 2), (GEN_COMPACT, False, 2),
                                                 (GEN_REORDER, True, 2)])
def test_flat_first_hint_takes_a_learned_order(variant, fixed, want):
    """YSB_F_FLAT_FIRST keeps the flat-object tier first (layout 2) unless the batch's first
    line names a key order (layout 3, whose off-order lines go to the same flat tier);
    with YSB_F_LAYOUT_FIXED nothing is sampled.  Host and device batches, exact vs the oracle."""
    g = GenParams(seed=29, n_campaigns=40, ads_per_campaign=10, events_per_sec=1000, with_skew=True, variant=variant)
    _, aids = g.ids()
    raw, offs = g.events_host(0, 60_000)
    exp, est = oracle.run(oracle.AdMap(aids, g.ad_campaign_index()), raw, offs)
    kw = {"flat_first": True}
    if fixed:
        kw["layout_auto"] = False
    for device in (False, True):
        with YsbContext(n_campaigns=40, window_ring=256, max_batch_bytes=raw.size + 64,
                        max_batch_events=offs.size + 1, **kw) as ctx:
            ctx.load_ad_map(aids, g.ad_campaign_index())
            if device:
                d_b, d_o = ctx.device_alloc(raw.size + 64), ctx.device_alloc(4 * offs.size + 64)
                ctx.h2d(d_b, raw)
                ctx.h2d(d_o, offs)
                ctx.submit_device(d_b, raw.size, d_o, offs.size)
            else:
                ctx.submit(raw, offs)
            got = ctx.drain_buckets()
            st = ctx.stats()
            assert ctx.launch_info()["layout"] == want
        assert got == exp
        for k, v in est.items():
            assert st[k] == v, k
        assert st["deferred"] == 0


# short fields: a tile holds 64 lines of 272 bytes on average (a longer tile is deferred
# whole, still exact), generator lines are 249-265 bytes
EXTRA_FIELDS = [b'"src": "w", ', b'"ad_idx":"7",', b'"event":"",', b'"user_id2":"",', b'"ip_a": "", ',
                b'"k" : "v" , ']


def _with_extra(line, rng, kind):
    """One generator line with extra fields spliced in after '{' or after a pair."""
    body = line[:-1]
    cuts = [1] + [i + 3 for i in range(len(body) - 2) if body[i:i + 3] == b'", "']
    def put(b, fld):
        at = cuts[int(rng.integers(0, len(cuts)))]
        return b[:at] + fld + b[at:]
    if kind == "one":
        body = put(body, EXTRA_FIELDS[int(rng.integers(0, len(EXTRA_FIELDS)))])
    elif kind == "two":
        body = put(body, b'"a1": "x", ')
        body = body[:1] + b'"a2": "y", ' + body[1:]
    elif kind == "dup":
        body = body[:1] + b'"a1": "x", "a1": "y", ' + body[1:]
    elif kind == "number":
        body = body[:1] + b'"n": 12, ' + body[1:]
    elif kind == "nested":
        body = body[:1] + b'"o": {"p": "q"}, ' + body[1:]
    elif kind == "escaped":
        body = body[:1] + b'"a\\u0031": "x", ' + body[1:]
    elif kind == "quote_in_value":
        body = body[:1] + b'"a": "x\\"y", ' + body[1:]
    return body + b"\n"


@pytest.mark.parametrize("hint", [None, "flat_first"])
@pytest.mark.parametrize("base_variant", [0, GEN_REORDER])
def test_extra_fields_match_oracle(hint, base_variant):
    """A producer's extra fields (org.json puts them, DeserializeBolt never reads them): one
    plain-string extra pair per line is parsed by the flat tier (nothing deferred); two,
    a repeat (putOnce throws: a parse error), other value forms and escapes go to the
    general path -- all exactly as the oracle decides them."""
    g = GenParams(seed=31, n_campaigns=40, ads_per_campaign=10, events_per_sec=1000, with_skew=True,
                  variant=base_variant)
    _, aids = g.ids()
    raw, offs = g.events_host(0, 40_000)
    data = raw.tobytes()
    ends = list(offs[1:]) + [len(data)]
    base = [data[s:e] for s, e in zip(offs, ends)]
    rng = np.random.default_rng(3)
    for kinds in (["one"], ["one", "two", "dup", "number", "nested", "escaped", "quote_in_value"]):
        lines = [_with_extra(ln, rng, kinds[int(rng.integers(0, len(kinds)))]) for ln in base]
        if len(kinds) > 1:
            lines[0] = base[0]   # the first line plain: its layout (generator / learned order) is sampled
        buf = b"".join(lines)
        o = np.cumsum([0] + [len(x) for x in lines[:-1]]).astype(np.uint32)
        exp, est = oracle.run(oracle.AdMap(aids, g.ad_campaign_index()), buf, o)
        with YsbContext(n_campaigns=40, window_ring=256, max_batch_bytes=len(buf) + 64,
                        max_batch_events=o.size + 1, **hint_kw(hint)) as ctx:
            ctx.load_ad_map(aids, g.ad_campaign_index())
            ctx.submit(np.frombuffer(buf, dtype=np.uint8), o)
            got = ctx.drain_buckets()
            st = ctx.stats()
            lay = ctx.launch_info()["layout"]
        assert got == exp
        for k, v in est.items():
            assert st[k] == v, k
        if kinds == ["one"]:
            assert lay == 2 and st["deferred"] == 0    # the flat tier took every line
        else:
            assert est["parse_errors"] > 0 and st["deferred"] > 0


@pytest.mark.parametrize("hint", [None, "flat_first"])
def test_extra_field_edge_lines_match_oracle(hint):
    """Edge forms around the flat tier's one extra field: an empty key, a key named like
    one of DeserializeBolt's with more bytes, an extra pair after a repeated known key,
    the extra pair last (before '}'), compact and spaced separators -- each line in a
    batch of its own kind, exact vs the oracle."""
    g = GenParams(seed=37, n_campaigns=20, ads_per_campaign=5, events_per_sec=1000)
    _, aids = g.ids()
    raw, offs = g.events_host(0, 2000)
    data = raw.tobytes()
    ends = list(offs[1:]) + [len(data)]
    base = [data[s:e] for s, e in zip(offs, ends)]
    edits = [lambda ln: ln.replace(b'{"user_id"', b'{"": "x", "user_id"', 1),
             lambda ln: ln.replace(b'{"user_id"', b'{"event_timex": "1", "user_id"', 1),
             lambda ln: ln.replace(b'{"user_id"', b'{"ad_i": "1", "user_id"', 1),
             lambda ln: ln[:-2] + b', "zz": "last"}\n',
             lambda ln: ln[:-2] + b',"zz":"last"}\n',
             lambda ln: ln.replace(b'{"user_id"', b'{"x": "1", "user_id": "u", "user_id"', 1),
             lambda ln: ln.replace(b'{"user_id"', b'{ "x" :"1" ;"user_id"', 1)]
    for ed in edits:
        lines = [ed(ln) for ln in base]
        buf = b"".join(lines)
        o = np.cumsum([0] + [len(x) for x in lines[:-1]]).astype(np.uint32)
        exp, est = oracle.run(oracle.AdMap(aids, g.ad_campaign_index()), buf, o)
        with YsbContext(n_campaigns=20, window_ring=64, max_batch_bytes=len(buf) + 64,
                        max_batch_events=o.size + 1, **hint_kw(hint)) as ctx:
            ctx.load_ad_map(aids, g.ad_campaign_index())
            ctx.submit(np.frombuffer(buf, dtype=np.uint8), o)
            got = ctx.drain_buckets()
            st = ctx.stats()
        assert got == exp, lines[0]
        for k, v in est.items():
            assert st[k] == v, (k, lines[0])


@pytest.mark.parametrize("blocks", [False, True])
def test_mixed_producers_take_the_per_tile_dispatch(blocks):
    """Four producers interleaved line by line (GEN_MIXED) or in runs of 256 lines
    (GEN_MIXED_BLOCKS): the 64-line layout sample (32 pairs of adjacent lines) finds no layout
    46 of them agree on.  In runs (adjacent lines alike) the per-tile dispatch runs (layout 4:
    a tile of one producer takes its path -- the vocabulary paths, the learned order -- a
    mixed tile the flat tier); line by line, the flat tier (layout 2) -- host, device and raw
    batches, exact vs the oracle, nothing deferred."""
    from ysb_amd import GEN_MIXED, GEN_MIXED_BLOCKS
    g = GenParams(seed=53, n_campaigns=40, ads_per_campaign=10, events_per_sec=1000, with_skew=True,
                  variant=GEN_MIXED_BLOCKS if blocks else GEN_MIXED)
    _, aids = g.ids()
    raw, offs = g.events_host(0, 80_000)
    exp, est = oracle.run(oracle.AdMap(aids, g.ad_campaign_index()), raw, offs)
    for how in ("host", "device", "raw"):
        with YsbContext(n_campaigns=40, window_ring=256, max_batch_bytes=raw.size + 64,
                        max_batch_events=offs.size + 1) as ctx:
            ctx.load_ad_map(aids, g.ad_campaign_index())
            if how == "device":
                d_b, d_o = ctx.device_alloc(raw.size + 64), ctx.device_alloc(4 * offs.size + 64)
                ctx.h2d(d_b, raw)
                ctx.h2d(d_o, offs)
                ctx.submit_device(d_b, raw.size, d_o, offs.size)
            elif how == "raw":
                ctx.submit_raw(raw)
            else:
                ctx.submit(raw, offs)
            got = ctx.drain_buckets()
            st = ctx.stats()
            # runs: adjacent sample lines alike -> the per-tile dispatch; line by line -> the flat tier
            assert ctx.launch_info()["layout"] == (4 if blocks else 2), how
        assert got == exp, how
        for k, v in est.items():
            assert st[k] == v, (how, k)
        assert st["deferred"] == 0, how
