"""In-process RESP2 server with the handful of Redis commands the YSB schema uses
(test infrastructure: no Redis server exists in this image).  Semantics follow the
Redis command reference for string / hash / list / set keys."""
from __future__ import annotations

import collections
import itertools
import socketserver
import socket
import threading


class _State:
    def __init__(self):
        self.kv = {}
        self.lock = threading.Lock()
        self.commands = 0


def _bulk(v):
    if v is None:
        return b"$-1\r\n"
    b = v.encode() if isinstance(v, str) else v
    return b"$%d\r\n%s\r\n" % (len(b), b)


def _arr(vs):
    return b"*%d\r\n" % len(vs) + b"".join(_bulk(v) for v in vs)


def _int(n):
    return b":%d\r\n" % n


class _Handler(socketserver.BaseRequestHandler):
    """RESP over one connection: every complete command in what has arrived is run, and
    their replies go back in one send (a pipelined client gets them together; replies
    written one by one would meet Nagle's algorithm and the client's delayed ACK)."""

    def handle(self):
        st = self.server.state
        sock = self.request
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        buf = b""
        pos = 0
        while True:
            chunk = sock.recv(1 << 20)
            if not chunk:
                return
            buf = buf[pos:] + chunk
            pos = 0
            out = []
            while True:
                cmd = self.parse(buf, pos)
                if cmd is None:
                    break
                args, pos = cmd
                with st.lock:
                    st.commands += 1
                    out.append(self.run(st.kv, args))
            if out:
                sock.sendall(b"".join(out))

    @staticmethod
    def parse(buf, pos):
        """(args, next position) of the command at pos, or None if it is not all here."""
        e = buf.find(b"\r\n", pos)
        if e < 0:
            return None
        assert buf[pos:pos + 1] == b"*", buf[pos:pos + 40]
        n = int(buf[pos + 1:e])
        p = e + 2
        args = []
        for _ in range(n):
            e = buf.find(b"\r\n", p)
            if e < 0:
                return None
            assert buf[p:p + 1] == b"$"
            m = int(buf[p + 1:e])
            if e + 2 + m + 2 > len(buf):
                return None
            args.append(buf[e + 2:e + 2 + m].decode())
            p = e + 2 + m + 2
        return args, p

    @staticmethod
    def run(kv, args):
        cmd = args[0].upper()
        a = args[1:]

        def typed(key, t):
            v = kv.get(key)
            if v is None:
                v = t()
                kv[key] = v
            if not isinstance(v, t):
                raise TypeError
            return v
        try:
            if cmd == "PING":
                return b"+PONG\r\n"
            if cmd == "FLUSHALL":
                kv.clear()
                return b"+OK\r\n"
            if cmd == "SET":
                kv[a[0]] = a[1]
                return b"+OK\r\n"
            if cmd == "GET":
                v = kv.get(a[0])
                return _bulk(v if isinstance(v, str) or v is None else None)
            if cmd == "SADD":
                s = typed(a[0], set)
                n = len([m for m in a[1:] if m not in s])
                s.update(a[1:])
                return _int(n)
            if cmd == "SMEMBERS":
                return _arr(sorted(kv.get(a[0], set())))
            if cmd == "HSET":
                h = typed(a[0], dict)
                n = 0
                for f, v in zip(a[1::2], a[2::2]):
                    n += f not in h
                    h[f] = v
                return _int(n)
            if cmd == "HGET":
                return _bulk(kv.get(a[0], {}).get(a[1]))
            if cmd == "HMGET":
                h = kv.get(a[0], {})
                return _arr([h.get(f) for f in a[1:]])
            if cmd == "HINCRBY":
                h = typed(a[0], dict)
                v = int(h.get(a[1], "0")) + int(a[2])
                h[a[1]] = str(v)
                return _int(v)
            if cmd == "LPUSH":   # (a deque: O(1) at the head; the time_updated list grows long)
                lst = typed(a[0], collections.deque)
                for v in a[1:]:
                    lst.appendleft(v)
                return _int(len(lst))
            if cmd == "LLEN":
                return _int(len(kv.get(a[0], [])))
            if cmd == "LRANGE":
                lst = kv.get(a[0], collections.deque())
                lo, hi = int(a[1]), int(a[2])
                hi = len(lst) - 1 if hi < 0 else hi
                return _arr(list(itertools.islice(lst, lo, hi + 1)))
            return b"-ERR unknown command '%s'\r\n" % cmd.encode()
        except TypeError:
            return b"-WRONGTYPE Operation against a key holding the wrong kind of value\r\n"


class FakeRedis:
    def __init__(self):
        self.server = socketserver.ThreadingTCPServer(("127.0.0.1", 0), _Handler)
        self.server.daemon_threads = True
        self.server.state = _State()
        self.port = self.server.server_address[1]
        self.thread = threading.Thread(target=self.server.serve_forever, daemon=True)
        self.thread.start()

    @property
    def kv(self):
        return self.server.state.kv

    def close(self):
        self.server.shutdown()
        self.server.server_close()
