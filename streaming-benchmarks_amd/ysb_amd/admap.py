"""Ad -> campaign map loading in both formats the reference uses.

  JSON lines `{ "AD": "CAMPAIGN"}`  written by data/src/setup/core.clj:58, merged
                                    left to right by dostats (core.clj:104-106)
  CSV `ad,campaign`                 read by getAdCampaignMap
                                    (flink-benchmarks/.../AdvertisingTopologyNative.java:47-56)

Both give a later duplicate precedence (HashMap.put / merge).  Campaign UUIDs are
mapped to dense indices in order of first appearance (or of a given campaign list,
e.g. campaign-ids.txt, core.clj:24-31); the index space is what the device counts in.
"""
from __future__ import annotations

import json
import re


class AdCampaignMap:
    def __init__(self, pairs, campaigns=None):
        self.campaigns = list(campaigns) if campaigns is not None else []
        self.index = {c: i for i, c in enumerate(self.campaigns)}
        self.ad_to_campaign = {}
        for ad, camp in pairs:
            if camp not in self.index:
                self.index[camp] = len(self.campaigns)
                self.campaigns.append(camp)
            self.ad_to_campaign[ad] = camp

    @classmethod
    def from_json_lines(cls, data: bytes, campaigns=None):
        pairs = []
        for ln in data.splitlines():
            if ln.strip():
                pairs.extend(json.loads(ln.decode("utf-8")).items())
        return cls(pairs, campaigns)

    @classmethod
    def from_csv(cls, data: bytes, campaigns=None):
        """readLine + String.split(",") (trailing empty items dropped) + kv[0] -> kv[1];
        a line with fewer than two items raises IndexError (ArrayIndexOutOfBounds)."""
        text = data.decode("utf-8")
        lines = re.split(r"\r\n|\r|\n", text)
        if text.endswith(("\n", "\r")) or not text:
            lines.pop()                       # readLine: no empty line after the last terminator
        pairs = []
        for ln in lines:
            kv = ln.split(",")
            while len(kv) > 1 and kv[-1] == "":
                kv.pop()
            pairs.append((kv[0], kv[1]))
        return cls(pairs, campaigns)

    def arrays(self):
        """(ad_ids, campaign_idx) for YsbContext.load_ad_map."""
        ads = list(self.ad_to_campaign)
        return ads, [self.index[self.ad_to_campaign[a]] for a in ads]

    @property
    def n_campaigns(self):
        return len(self.campaigns)
