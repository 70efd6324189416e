"""GPU parity at volume: random byte edits of generator lines in every producer layout, a
few hundred thousand lines per batch, through every tier of the HIP path (vocabulary path,
canonical tiers, learned order / flat tier, the deferred org.json machine) against the C
oracle (oracle/ysb_oracle.c, test infrastructure) -- every (campaign, window) count and
every counter bit-exact.

The edits are the small ones a producer, a transport or a file could make to one line: a
byte replaced by one of JSON's structural characters, a quote, a backslash, a space, a
digit or a letter; a byte inserted; a byte deleted.  Most edited lines stop being
DeserializeBolt-parseable (AdvertisingTopologyNative.java:257-276: org.json throws, the
line is a parse error) or change a value (another ad_id: a join miss; another event_type:
filtered); all must be decided exactly as the reference decides them."""
import numpy as np
import pytest

from oracle import oracle
from ysb_amd import GEN_COMPACT, GEN_MORE_AD_TYPES, GEN_RANDOM_IP, GEN_REORDER, GenParams, YsbContext

pytestmark = pytest.mark.gpu

ALPHABET = np.frombuffer(b'"\\:,{}[] \t/u0123456789abcdefviewlnrt-.+eE;=#', dtype=np.uint8)
STAT_KEYS = ("events", "views", "joined", "join_misses", "parse_errors", "time_errors")


def mutate(lines, rng, frac):
    """Edits `frac` of the lines: 1-3 replacements / insertions / deletions each."""
    out = []
    for ln in lines:
        if rng.random() >= frac or len(ln) < 3:
            out.append(ln)
            continue
        b = bytearray(ln)
        for _ in range(int(rng.integers(1, 4))):
            op = rng.integers(0, 3)
            i = int(rng.integers(0, max(1, len(b) - 1)))   # never the final '\n'
            if op == 0:
                b[i] = int(ALPHABET[rng.integers(0, ALPHABET.size)])
            elif op == 1:
                b.insert(i, int(ALPHABET[rng.integers(0, ALPHABET.size)]))
            elif len(b) > 2:
                del b[i]
        out.append(bytes(b))
    return out


def lines_of(g, n):
    raw, offs = g.events_host(0, n)
    data = raw.tobytes()
    ends = list(offs[1:]) + [len(data)]
    return [data[s:e] for s, e in zip(offs, ends)]


def run_both(lines, aids, camp, n_campaigns, **kw):
    data = b"".join(lines)
    offs = np.cumsum([0] + [len(x) for x in lines[:-1]]).astype(np.uint32)
    exp, est = oracle.run(oracle.AdMap(aids, camp), data, offs, threads=8)
    raw = np.frombuffer(data, dtype=np.uint8)
    with YsbContext(n_campaigns=n_campaigns, window_ring=256, max_batch_bytes=raw.size + 64,
                    max_batch_events=offs.size + 1, **kw) as ctx:
        ctx.load_ad_map(aids, camp)
        d_b, d_o = ctx.device_alloc(raw.size + 64), ctx.device_alloc(4 * offs.size + 64)
        ctx.h2d(d_b, raw)
        ctx.h2d(d_o, offs)
        ctx.submit_device(d_b, raw.size, d_o, offs.size)   # layout sampled from line 0
        got = ctx.drain_buckets()
        st = ctx.stats()
    return exp, est, got, st


HINTS = {None: {}, "fixed": {"layout_auto": False}, "flat_first": {"flat_first": True},
         "compact_first": {"compact_first": True}}


@pytest.mark.timeout(300)
@pytest.mark.parametrize("hint", list(HINTS))
@pytest.mark.parametrize("first,seed", [(0, 1), (GEN_COMPACT, 2), (GEN_REORDER, 3), (GEN_RANDOM_IP, 4)])
def test_random_edits_every_layout_match_oracle(first, seed, hint):
    """600k lines: four producers' layouts interleaved (the batch's first line from
    `first`, which picks the instantiation unless the hint fixes it), 20 % of the lines
    edited."""
    rng = np.random.default_rng(seed)
    variants = [first] + [v for v in (0, GEN_COMPACT, GEN_REORDER, GEN_RANDOM_IP | GEN_MORE_AD_TYPES) if v != first]
    per = 150_000
    pools = []
    for v in variants:
        g = GenParams(seed=40 + seed, n_campaigns=60, ads_per_campaign=10, events_per_sec=1000, with_skew=True,
                      variant=v)
        pools.append(lines_of(g, per))
    g0 = GenParams(seed=40 + seed, n_campaigns=60, ads_per_campaign=10)
    _, aids = g0.ids()
    camp = g0.ad_campaign_index()
    order = rng.permutation(np.repeat(np.arange(len(variants)), per))
    j = int(np.argmax(order == 0))
    order[0], order[j] = order[j], order[0]   # line 0 from `first`
    idx = [0] * len(variants)
    lines = []
    for v in order:
        lines.append(pools[v][idx[v]])
        idx[v] += 1
    lines = [lines[0]] + mutate(lines[1:], rng, 0.20)
    exp, est, got, st = run_both(lines, aids, camp, 60, **HINTS[hint])
    assert est["parse_errors"] > 1000 and est["views"] > 10_000   # the edits reached every decision
    for k in STAT_KEYS:
        assert st[k] == est[k], (k, st[k], est[k])
    assert st["overflow_dropped"] == 0
    assert got == exp


@pytest.mark.timeout(300)
@pytest.mark.parametrize("seed", [5, 6])
def test_random_edits_tbl_rows_match_oracle(seed):
    """The fork's .tbl rows (MockWindowedFlatMap, AdvertisingTopologyNative.java:197-226),
    500k rows, 20 % edited (a '|' added or lost moves every field after it)."""
    rng = np.random.default_rng(seed)
    g = GenParams(seed=50 + seed, n_campaigns=60, ads_per_campaign=10, events_per_sec=1000, fmt="tbl")
    _, aids = g.ids()
    camp = g.ad_campaign_index()
    lines = lines_of(g, 500_000)
    lines = [lines[0]] + mutate(lines[1:], rng, 0.20)
    data = b"".join(lines)
    offs = np.cumsum([0] + [len(x) for x in lines[:-1]]).astype(np.uint32)
    exp, est = oracle.run(oracle.AdMap(aids, camp), data, offs, threads=8, fmt="tbl")
    raw = np.frombuffer(data, dtype=np.uint8)
    with YsbContext(n_campaigns=60, window_ring=256, input_format="tbl", max_batch_bytes=raw.size + 64,
                    max_batch_events=offs.size + 1) as ctx:
        ctx.load_ad_map(aids, camp)
        ctx.submit(raw, offs)
        got = ctx.drain_buckets()
        st = ctx.stats()
    assert est["views"] > 10_000
    for k in STAT_KEYS:
        assert st[k] == est[k], (k, st[k], est[k])
    assert got == exp


@pytest.mark.timeout(300)
def test_random_edits_hbm_table_record_mode_match_oracle():
    """configs[2]'s path: an HBM-resident bucket join table (1.2M ads) and record-mode
    counting (LDS-staged records -> partition -> per-block counts into the u8 delta ring),
    400k lines, 20 % edited."""
    rng = np.random.default_rng(9)
    g = GenParams(seed=61, n_campaigns=600_000, ads_per_campaign=2, events_per_sec=1000, with_skew=True)
    _, aids = g.ids()
    camp = g.ad_campaign_index()
    lines = lines_of(g, 400_000)
    lines = [lines[0]] + mutate(lines[1:], rng, 0.20)
    data = b"".join(lines)
    offs = np.cumsum([0] + [len(x) for x in lines[:-1]]).astype(np.uint32)
    exp, est = oracle.run(oracle.AdMap(aids, camp), data, offs, threads=8)
    raw = np.frombuffer(data, dtype=np.uint8)
    with YsbContext(n_campaigns=600_000, window_ring=128, record_count=True, timing=True,
                    max_batch_bytes=raw.size + 64, max_batch_events=offs.size + 1) as ctx:
        ctx.load_ad_map(aids, camp)
        ctx.submit(raw, offs)
        got = ctx.drain_buckets()
        st = ctx.stats()
        ctx.kernel_time()
        assert ctx.path_time()[2] == 1 and ctx.launch_info()["hbm_table"] == 1
    assert est["parse_errors"] > 1000 and est["join_misses"] > 100
    for k in STAT_KEYS:
        assert st[k] == est[k], (k, st[k], est[k])
    assert got == exp


@pytest.mark.timeout(300)
@pytest.mark.parametrize("first,want", [(GEN_COMPACT, 1), (GEN_REORDER, 3), (0, 0)])
@pytest.mark.parametrize("rec", [True, False])
def test_hbm_table_layout_instantiations_match_oracle(first, want, rec):
    """configs[2]'s HBM-resident join table with other producers' layouts (round 4): the
    batch's first line picks the compact / learned-order / generator instantiation of the
    record-mode (rec) or serial-probe kernel; 300k lines, 6 % of them from the other
    producers, 3 % edited -- exact vs the C oracle, and the instantiation is the sampled one."""
    rng = np.random.default_rng(11 + first)
    variants = [first] + [v for v in (0, GEN_COMPACT, GEN_REORDER) if v != first]
    pools = [lines_of(GenParams(seed=71, n_campaigns=600_000, ads_per_campaign=2, events_per_sec=1000,
                                with_skew=True, variant=v), 300_000) for v in variants]
    g0 = GenParams(seed=71, n_campaigns=600_000, ads_per_campaign=2)
    _, aids = g0.ids()
    camp = g0.ad_campaign_index()
    pick = rng.random(300_000)
    # 94 % in the first producer's layout (the 64-line layout sample, 46 of which must agree,
    # names it), the rest from the others, 3 % edited
    lines = [pools[0][i] if pick[i] < 0.94 or i == 0 else pools[1 + (i & 1)][i] for i in range(300_000)]
    lines = [lines[0]] + mutate(lines[1:], rng, 0.03)
    data = b"".join(lines)
    offs = np.cumsum([0] + [len(x) for x in lines[:-1]]).astype(np.uint32)
    exp, est = oracle.run(oracle.AdMap(aids, camp), data, offs, threads=8)
    raw = np.frombuffer(data, dtype=np.uint8)
    with YsbContext(n_campaigns=600_000, window_ring=128, record_count=rec, timing=True,
                    max_batch_bytes=raw.size + 64, max_batch_events=offs.size + 1) as ctx:
        ctx.load_ad_map(aids, camp)
        d_b, d_o = ctx.device_alloc(raw.size + 64), ctx.device_alloc(4 * offs.size + 64)
        ctx.h2d(d_b, raw)
        ctx.h2d(d_o, offs)
        ctx.submit_device(d_b, raw.size, d_o, offs.size)
        got = ctx.drain_buckets()
        st = ctx.stats()
        ctx.kernel_time()
        info = ctx.launch_info()
        assert info["hbm_table"] == 1 and info["layout"] == want and info["record_mode"] == int(rec)
        assert (ctx.path_time()[2] == 1) == rec
    assert est["parse_errors"] > 1000 and est["views"] > 50_000
    for k in STAT_KEYS:
        assert st[k] == est[k], (k, st[k], est[k])
    assert got == exp


@pytest.mark.timeout(300)
@pytest.mark.parametrize("rec", [True, False])
def test_hbm_table_producers_in_runs_take_the_per_tile_dispatch(rec):
    """configs[2]'s HBM-resident join table, four producers writing in runs of 256 lines
    (GEN_MIXED_BLOCKS), 3 % of the lines edited: the per-tile dispatch instantiation of the
    record-mode (rec) / serial-probe kernel (layout 4) -- exact vs the C oracle."""
    from ysb_amd import GEN_MIXED_BLOCKS
    rng = np.random.default_rng(5)
    g = GenParams(seed=73, n_campaigns=600_000, ads_per_campaign=2, events_per_sec=1000, with_skew=True,
                  variant=GEN_MIXED_BLOCKS)
    _, aids = g.ids()
    camp = g.ad_campaign_index()
    lines = lines_of(g, 200_000)
    lines = lines[:1] + mutate(lines[1:], rng, 0.03)
    data = b"".join(lines)
    offs = np.cumsum([0] + [len(x) for x in lines[:-1]]).astype(np.uint32)
    exp, est = oracle.run(oracle.AdMap(aids, camp), data, offs, threads=8)
    raw = np.frombuffer(data, dtype=np.uint8)
    with YsbContext(n_campaigns=600_000, window_ring=128, record_count=rec, max_batch_bytes=raw.size + 64,
                    max_batch_events=offs.size + 1) as ctx:
        ctx.load_ad_map(aids, camp)
        ctx.submit(raw, offs)
        got = ctx.drain_buckets()
        st = ctx.stats()
        info = ctx.launch_info()
        assert info["hbm_table"] == 1 and info["layout"] == 4 and info["record_mode"] == int(rec)
    for k in STAT_KEYS:
        assert st[k] == est[k], (k, st[k], est[k])
    assert got == exp
