"""Loading of the committed fixtures in tests/golden/ (see make_golden.py)."""
from __future__ import annotations

import csv
import json
import os

from oracle import dostats

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def path(name):
    return os.path.join(GOLDEN, name)


def campaigns():
    with open(path("gen_s7.campaign_ids.txt")) as f:
        return [ln.strip() for ln in f if ln.strip()]


def campaign_index():
    return {c: i for i, c in enumerate(campaigns())}


def ad_map():
    """ad uuid -> campaign uuid, from the core.clj:58 JSON-lines file."""
    with open(path("gen_s7.ad_to_campaign.txt"), "rb") as f:
        return dostats.load_ad_map_json_lines(f.read())


def ad_arrays():
    idx = campaign_index()
    m = ad_map()
    ads = list(m)
    return ads, [idx[m[a]] for a in ads]


def gen_params():
    with open(path("gen_s7.params.json")) as f:
        return json.load(f)


def events(stem, ext=".jsonl"):
    """(raw bytes, line offsets) of tests/golden/<stem><ext>."""
    with open(path(stem + ext), "rb") as f:
        raw = f.read()
    _, offs = dostats.split_lines(raw)
    return raw, offs


def tbl_events(stem):
    """.tbl fixture (expected-output stem, data file): gen_s7_tbl -> gen_s7.tbl."""
    return events(TBL_FILES[stem], ".tbl")


def expected(stem, require_ip=False):
    """({(campaign_idx, bucket): count}, stats dict)."""
    suf = ".ip" if require_ip else ""
    idx = campaign_index()
    rows = {}
    with open(path(stem + suf + ".expected.csv")) as f:
        for r in csv.DictReader(f):
            w = int(r["window_ms"])
            assert w % 10000 == 0
            rows[(idx[r["campaign_id"]], w // 10000)] = int(r["count"])
    with open(path(stem + suf + ".expected.json")) as f:
        st = json.load(f)
    return rows, st


FIXTURES = [("gen_s7", False), ("edge", False), ("edge", True), ("edge_orgjson", False), ("edge_orgjson", True),
            ("edge_long", False)]
# .tbl fixtures: expected-output stem -> data file stem (tests/golden/<file>.tbl)
TBL_FILES = {"gen_s7_tbl": "gen_s7", "edge_tbl": "edge_tbl"}
TBL_FIXTURES = sorted(TBL_FILES)
