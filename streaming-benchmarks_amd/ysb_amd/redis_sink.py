"""Redis output of the window counts, in the reference's schema, plus the generator's
readers of it.

Writer: RedisWindowWriter.write(rows) is CampaignProcessorCommon.writeWindow
(streaming-benchmark-common/.../CampaignProcessorCommon.java:69-89, commented out in
the fork) and AdvertisingSpark.writeWindow (spark-benchmarks/src/main/scala/
AdvertisingSpark.scala:184-208) for a batch of (campaign, window_ms, delta) rows as
ysb_drain returns them:

    windowUUID = HGET <campaign> <window_ms>
    if missing:  windowUUID = random UUID;  HSET <campaign> <window_ms> windowUUID
                 listUUID = HGET <campaign> "windows"
                 if missing: listUUID = random UUID;  HSET <campaign> "windows" listUUID
                 LPUSH listUUID <window_ms>
    HINCRBY windowUUID seen_count <delta>
    HSET    windowUUID time_updated <now ms>
    LPUSH   time_updated <now ms>                     (CampaignProcessorCommon only)

Batched into two pipelined round trips per flush (all reads, then all writes); the
result is the same as the per-window sequence for a single writer, which is what the
reference's one flusher thread per processor is.

Readers: get_stats (core.clj:130-149, the seen.txt / updated.txt dump) and
check_correct (core.clj:215-237, CORRECT / DIFFER per (campaign, bucket)).

The client is a minimal RESP2 implementation over a socket (no redis package is
installed here); it speaks to any Redis server.
"""
from __future__ import annotations

import socket
import time
import uuid


class RedisError(RuntimeError):
    pass


class RespClient:
    """Minimal RESP2 client with pipelining."""

    def __init__(self, host="127.0.0.1", port=6379, timeout=10.0):
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.buf = b""

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass

    @staticmethod
    def _encode(args):
        out = [b"*%d\r\n" % len(args)]
        for a in args:
            if isinstance(a, str):
                a = a.encode()
            elif isinstance(a, int):
                a = str(a).encode()
            out.append(b"$%d\r\n%s\r\n" % (len(a), a))
        return b"".join(out)

    def _line(self):
        while b"\r\n" not in self.buf:
            chunk = self.sock.recv(1 << 16)
            if not chunk:
                raise RedisError("connection closed")
            self.buf += chunk
        ln, self.buf = self.buf.split(b"\r\n", 1)
        return ln

    def _exact(self, n):
        while len(self.buf) < n + 2:
            chunk = self.sock.recv(1 << 16)
            if not chunk:
                raise RedisError("connection closed")
            self.buf += chunk
        data, self.buf = self.buf[:n], self.buf[n + 2:]
        return data

    def _reply(self):
        ln = self._line()
        t, rest = ln[:1], ln[1:]
        if t == b"+":
            return rest.decode()
        if t == b"-":
            return RedisError(rest.decode())
        if t == b":":
            return int(rest)
        if t == b"$":
            n = int(rest)
            return None if n < 0 else self._exact(n).decode()
        if t == b"*":
            n = int(rest)
            return None if n < 0 else [self._reply() for _ in range(n)]
        raise RedisError("bad reply %r" % ln)

    def pipeline(self, cmds):
        """Sends every command, then reads every reply (in order)."""
        if not cmds:
            return []
        self.sock.sendall(b"".join(self._encode(c) for c in cmds))
        out = [self._reply() for _ in cmds]
        for r in out:
            if isinstance(r, RedisError):
                raise r
        return out

    def execute(self, *args):
        return self.pipeline([args])[0]


class RedisWindowWriter:
    """writeWindow for batches of drained rows.  campaign_ids maps the library's
    campaign index to the campaign UUID string."""

    def __init__(self, client: RespClient, campaign_ids, time_updated_list=True, clock_ms=None):
        self.r = client
        self.campaign_ids = list(campaign_ids)
        self.time_updated_list = time_updated_list   # CampaignProcessorCommon.java:88
        self.clock_ms = clock_ms or (lambda: int(time.time() * 1000))
        self.window_uuid = {}   # (campaign uuid, window_ms str) -> window UUID (cache)
        self.list_uuid = {}     # campaign uuid -> windows list UUID (cache)
        self.round_trips = 0

    def write(self, rows):
        """rows: iterable of (campaign_idx, window_ms, delta) (ysb_drain output)."""
        rows = [(self.campaign_ids[c], str(int(w)), int(n)) for c, w, n in rows if n]
        if not rows:
            return 0
        # round trip 1: the window and list UUIDs not cached yet
        need_w = sorted({(c, w) for c, w, _ in rows if (c, w) not in self.window_uuid})
        need_l = sorted({c for c, w in need_w if c not in self.list_uuid})
        reads = [("HGET", c, w) for c, w in need_w] + [("HGET", c, "windows") for c in need_l]
        got = self.r.pipeline(reads)
        self.round_trips += 1 if reads else 0
        wres = dict(zip(need_w, got[:len(need_w)]))
        lres = dict(zip(need_l, got[len(need_w):]))
        writes = []
        for c in need_l:
            if lres[c] is not None:
                self.list_uuid[c] = lres[c]
        for c, w in need_w:
            if wres[(c, w)] is not None:
                self.window_uuid[(c, w)] = wres[(c, w)]
                continue
            wu = str(uuid.uuid4())
            self.window_uuid[(c, w)] = wu
            writes.append(("HSET", c, w, wu))
            if c not in self.list_uuid:
                lu = str(uuid.uuid4())
                self.list_uuid[c] = lu
                writes.append(("HSET", c, "windows", lu))
            writes.append(("LPUSH", self.list_uuid[c], w))
        # round trip 2: the deltas
        now = str(self.clock_ms())
        for c, w, n in rows:
            wu = self.window_uuid[(c, w)]
            writes.append(("HINCRBY", wu, "seen_count", n))
            writes.append(("HSET", wu, "time_updated", now))
            if self.time_updated_list:
                writes.append(("LPUSH", "time_updated", now))
        self.r.pipeline(writes)
        self.round_trips += 1
        return len(rows)


def new_setup(client: RespClient, campaign_ids):
    """do-new-setup (core.clj:209-214): FLUSHALL, then SADD campaigns."""
    client.execute("FLUSHALL")
    client.pipeline([("SADD", "campaigns", c) for c in campaign_ids])


def write_ad_map(client: RespClient, ad_to_campaign):
    """gen-ads (core.clj:151-162): SET <ad> <campaign> (what RedisAdCampaignCache.execute
    GETs on a cache miss, RedisAdCampaignCache.java:26)."""
    client.pipeline([("SET", a, c) for a, c in ad_to_campaign.items()])


def get_stats(client: RespClient):
    """get-stats (core.clj:130-149): [(seen_count, time_updated - window_ms)] over every
    campaign window, the contents of seen.txt / updated.txt."""
    out = []
    for campaign in sorted(client.execute("SMEMBERS", "campaigns")):
        wkey = client.execute("HGET", campaign, "windows")
        if wkey is None:
            continue
        n = client.execute("LLEN", wkey)
        for wt in client.execute("LRANGE", wkey, 0, n):
            wk = client.execute("HGET", campaign, wt)
            seen = client.execute("HGET", wk, "seen_count")
            upd = client.execute("HGET", wk, "time_updated")
            out.append((int(seen), int(upd) - int(wt)))
    return out


def check_correct(client: RespClient, expected, divisor=10000):
    """check-correct (core.clj:215-237).  expected: {campaign uuid: {bucket: count}}
    (dostats' shape).  Returns [(campaign, bucket, status, redis_count)] with status
    'CORRECT', 'DIFFER' or 'MISSING'."""
    out = []
    for campaign, per in expected.items():
        for bucket, val in per.items():
            key = client.execute("HGET", campaign, str(bucket * divisor))
            if key is None:
                out.append((campaign, bucket, "MISSING", None))
                continue
            seen = int(client.execute("HGET", key, "seen_count"))
            out.append((campaign, bucket, "CORRECT" if seen == val else "DIFFER", seen))
    return out
