"""PCIe H2D probe (diagnostic, not a result): the GPU's NUMA node, where pinned pages really
land (move_pages(2) per sampled page, tools/numa_info.py -- round 4's probe asked
get_mempolicy, which reported node 0 for every binding), and the pinned -> device copy rate of
256 MiB buffers allocated four ways:

  default        hipHostMalloc(flags 0): HIP picks the pages' node
  numa_user_nN   hipHostMalloc(hipHostMallocNumaUser) under set_mempolicy(MPOL_BIND, node N)
  register_nN    mmap + mbind(node N) + first touch, then hipHostRegister

Rates: hipMemcpyAsync on a non-blocking stream, HIP events around 8 back-to-back copies.
Run with --after-load to repeat the default allocation after the conditions bench.py's
host_staged leg meets (a 25 GB device allocation freed, 16 host threads of CPU work, a 1 GB
device-to-host copy into pageable memory)."""
import ctypes as C
import json
import mmap
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numa_info  # noqa: E402

libc = C.CDLL(None, use_errno=True)
SYS_set_mempolicy, SYS_mbind = 238, 237   # x86_64
MPOL_DEFAULT, MPOL_BIND = 0, 2
hipHostMallocNumaUser = 0x20000000
H2D = 1

hip = C.CDLL("/opt/rocm/lib/libamdhip64.so")
for f, a in (("hipHostMalloc", [C.c_void_p, C.c_size_t, C.c_uint]), ("hipHostFree", [C.c_void_p]),
             ("hipHostRegister", [C.c_void_p, C.c_size_t, C.c_uint]), ("hipHostUnregister", [C.c_void_p]),
             ("hipMalloc", [C.c_void_p, C.c_size_t]), ("hipFree", [C.c_void_p]),
             ("hipMemcpyAsync", [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]),
             ("hipMemcpy", [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]),
             ("hipStreamCreateWithFlags", [C.c_void_p, C.c_uint]), ("hipStreamSynchronize", [C.c_void_p]),
             ("hipEventCreate", [C.c_void_p]), ("hipEventRecord", [C.c_void_p, C.c_void_p]),
             ("hipEventSynchronize", [C.c_void_p]),
             ("hipEventElapsedTime", [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]), ("hipSetDevice", [C.c_int])):
    getattr(hip, f).argtypes = a
    getattr(hip, f).restype = C.c_int


def ok(rc, what):
    if rc != 0:
        raise RuntimeError("%s failed: %d" % (what, rc))


def bind(node):
    if node is None:
        return libc.syscall(SYS_set_mempolicy, MPOL_DEFAULT, None, C.c_ulong(0))
    mask = C.c_ulong(1 << node)
    return libc.syscall(SYS_set_mempolicy, MPOL_BIND, C.byref(mask), C.c_ulong(64))


class Copier:
    def __init__(self, nbytes):
        self.n = nbytes
        self.d = C.c_void_p()
        ok(hip.hipMalloc(C.byref(self.d), nbytes), "hipMalloc")
        self.s = C.c_void_p()
        ok(hip.hipStreamCreateWithFlags(C.byref(self.s), 1), "stream")
        self.e0, self.e1 = C.c_void_p(), C.c_void_p()
        ok(hip.hipEventCreate(C.byref(self.e0)), "event")
        ok(hip.hipEventCreate(C.byref(self.e1)), "event")

    def rate(self, h, reps=8):
        ok(hip.hipMemcpyAsync(self.d, h, self.n, H2D, self.s), "warm copy")
        ok(hip.hipEventRecord(self.e0, self.s), "record")
        for _ in range(reps):
            ok(hip.hipMemcpyAsync(self.d, h, self.n, H2D, self.s), "copy")
        ok(hip.hipEventRecord(self.e1, self.s), "record")
        ok(hip.hipEventSynchronize(self.e1), "sync")
        ms = C.c_float()
        ok(hip.hipEventElapsedTime(C.byref(ms), self.e0, self.e1), "elapsed")
        return round(reps * self.n / (ms.value * 1e-3) / 1e9, 2)


def host_malloc(n, flags=0, node=None):
    if node is not None:
        bind(node)
    p = C.c_void_p()
    try:
        ok(hip.hipHostMalloc(C.byref(p), n, flags), "hipHostMalloc")
    finally:
        if node is not None:
            bind(None)
    C.memset(p, 1, n)
    return p


def registered(n, node):
    m = mmap.mmap(-1, n, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    addr = C.addressof(C.c_char.from_buffer(m))
    mask = C.c_ulong(1 << node)
    rc = libc.syscall(SYS_mbind, C.c_void_p(addr), C.c_ulong(n), MPOL_BIND, C.byref(mask), C.c_ulong(64), 0)
    C.memset(addr, 1, n)
    ok(hip.hipHostRegister(C.c_void_p(addr), n, 0), "hipHostRegister")
    return m, addr, rc


def per_stream(n, p, k_streams=8, reps=8):
    """The same pinned buffer copied on k_streams streams one at a time (each stream's copies
    may run on another SDMA engine), then split over 2 and 4 streams at once."""
    d = C.c_void_p()
    ok(hip.hipMalloc(C.byref(d), n), "hipMalloc")
    ss = []
    for _ in range(k_streams):
        s = C.c_void_p()
        ok(hip.hipStreamCreateWithFlags(C.byref(s), 1), "stream")
        ss.append(s)
    e0, e1 = C.c_void_p(), C.c_void_p()
    ok(hip.hipEventCreate(C.byref(e0)), "event")
    ok(hip.hipEventCreate(C.byref(e1)), "event")
    hip.hipDeviceSynchronize.restype = C.c_int

    def timed(streams):
        ok(hip.hipDeviceSynchronize(), "sync")
        t = time.perf_counter()
        part = n // len(streams)
        for _ in range(reps):
            for j, s in enumerate(streams):
                ok(hip.hipMemcpyAsync(C.c_void_p(d.value + j * part), C.c_void_p(p.value + j * part), part, H2D, s),
                   "copy")
        ok(hip.hipDeviceSynchronize(), "sync")
        return round(reps * n / (time.perf_counter() - t) / 1e9, 2)
    def pairs(stream, small=4 << 20):
        # ysb_submit's pattern: the slot's bytes, then its offsets, on one stream
        ok(hip.hipDeviceSynchronize(), "sync")
        t = time.perf_counter()
        for _ in range(reps):
            ok(hip.hipMemcpyAsync(d, p, n, H2D, stream), "copy")
            ok(hip.hipMemcpyAsync(C.c_void_p(d.value + n - small), C.c_void_p(p.value), small, H2D, stream), "copy")
        ok(hip.hipDeviceSynchronize(), "sync")
        return round(reps * (n + small) / (time.perf_counter() - t) / 1e9, 2)
    out = {"one_stream_each": [timed([s]) for s in ss]}
    out["big_small_pairs"] = [pairs(ss[0]) for _ in range(3)]
    out["series_one_stream"] = []
    for _ in range(10):
        out["series_one_stream"].append(timed(ss[:1]))
        time.sleep(0.3)
    out["split_2"] = timed(ss[:2])
    out["split_4"] = timed(ss[:4])
    out["one_stream_again"] = timed(ss[:1])
    return out


def thp_buffer(n):
    """n bytes of anonymous memory on 2 MiB-aligned transparent huge pages (madvise), touched,
    then pinned with hipHostRegister: one IOMMU translation per 2 MiB instead of per 4 KiB."""
    MADV_HUGEPAGE = 14
    raw = mmap.mmap(-1, n + (2 << 20), flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    base = C.addressof(C.c_char.from_buffer(raw))
    addr = (base + (2 << 20) - 1) & ~((2 << 20) - 1)
    rc = libc.madvise(C.c_void_p(addr), C.c_size_t(n), MADV_HUGEPAGE)
    C.memset(addr, 1, n)
    ok(hip.hipHostRegister(C.c_void_p(addr), n, 0), "hipHostRegister")
    return raw, addr, rc


def interleaved(n, bufs, rounds=20):
    """Each buffer copied once per round, alternating, every copy timed alone (HIP events):
    the per-copy rates, so a slow episode hits every buffer alike or not."""
    d = C.c_void_p()
    ok(hip.hipMalloc(C.byref(d), n), "hipMalloc")
    s = C.c_void_p()
    ok(hip.hipStreamCreateWithFlags(C.byref(s), 1), "stream")
    ev = [C.c_void_p() for _ in range(2)]
    for e in ev:
        ok(hip.hipEventCreate(C.byref(e)), "event")
    out = {k: [] for k in bufs}
    for _ in range(rounds):
        for k, p in bufs.items():
            ok(hip.hipEventRecord(ev[0], s), "rec")
            ok(hip.hipMemcpyAsync(d, C.c_void_p(p), n, H2D, s), "copy")
            ok(hip.hipEventRecord(ev[1], s), "rec")
            ok(hip.hipEventSynchronize(ev[1]), "sync")
            ms = C.c_float()
            ok(hip.hipEventElapsedTime(C.byref(ms), ev[0], ev[1]), "elapsed")
            out[k].append(round(n / (ms.value * 1e-3) / 1e9, 1))
    return out


def after_free(n, p, gb, seconds=4.0):
    """Allocate gb GiB of HBM, touch it (memset), free it, then time single 256 MiB copies for
    `seconds`: [(ms since the free, GB/s)].  The amdgpu driver clears freed VRAM with its own
    SDMA work; copies that share the engine with it run slower until it is done."""
    hip.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
    hip.hipMemset.restype = C.c_int
    hip.hipDeviceSynchronize.restype = C.c_int
    d = C.c_void_p()
    ok(hip.hipMalloc(C.byref(d), n), "hipMalloc")
    s = C.c_void_p()
    ok(hip.hipStreamCreateWithFlags(C.byref(s), 1), "stream")
    ev = [C.c_void_p() for _ in range(2)]
    for e in ev:
        ok(hip.hipEventCreate(C.byref(e)), "event")
    if gb:
        big = C.c_void_p()
        ok(hip.hipMalloc(C.byref(big), gb << 30), "hipMalloc big")
        ok(hip.hipMemset(big, 1, gb << 30), "memset big")
        ok(hip.hipDeviceSynchronize(), "sync")
        ok(hip.hipFree(big), "hipFree big")
    t0 = time.perf_counter()
    out = []
    while time.perf_counter() - t0 < seconds:
        ok(hip.hipEventRecord(ev[0], s), "rec")
        ok(hip.hipMemcpyAsync(d, p, n, H2D, s), "copy")
        ok(hip.hipEventRecord(ev[1], s), "rec")
        ok(hip.hipEventSynchronize(ev[1]), "sync")
        ms = C.c_float()
        ok(hip.hipEventElapsedTime(C.byref(ms), ev[0], ev[1]), "elapsed")
        out.append((round((time.perf_counter() - t0) * 1e3), round(n / (ms.value * 1e-3) / 1e9, 1)))
    ok(hip.hipFree(d), "hipFree")
    return out


def one(cp, p, n):
    return {"GBs": cp.rate(p), "pages_by_node": numa_info.page_nodes(p.value if hasattr(p, "value") else p, n),
            "thp_kB": numa_info.thp_kb(p.value if hasattr(p, "value") else p)}


def load_conditions(n_dev=25 << 30, seconds=5.0):
    """What bench.py's process has done before its host_staged leg: a large device allocation
    freed, 16 host threads busy for a while, a 1 GB device -> pageable host copy."""
    d = C.c_void_p()
    ok(hip.hipMalloc(C.byref(d), n_dev), "hipMalloc big")
    big = bytearray(1 << 30)
    ok(hip.hipMemcpy(C.c_void_p(C.addressof(C.c_char.from_buffer(big))), d, 1 << 30, 2), "d2h 1 GB")
    ok(hip.hipFree(d), "hipFree big")
    stop = time.time() + seconds

    def spin():
        x = 0
        while time.time() < stop:
            x += sum(range(1000))
    th = [threading.Thread(target=spin) for _ in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    del big


def main():
    ok(hip.hipSetDevice(0), "hipSetDevice")
    n = 256 << 20
    nodes = sorted(numa_info.node_meminfo())
    out = {"gpu": numa_info.gpu_node(0), "nodes": numa_info.node_meminfo(), "thread": numa_info.thread_node(),
           "affinity_cpus": len(os.sched_getaffinity(0))}
    cp = Copier(n)
    p = host_malloc(n)
    out["default"] = one(cp, p, n)
    for nd in nodes:
        try:
            out["numa_user_n%d" % nd] = one(cp, host_malloc(n, hipHostMallocNumaUser, nd), n)
        except RuntimeError as e:
            out["numa_user_n%d" % nd] = {"error": str(e)}
        try:
            m, addr, rc = registered(n, nd)
            r = one(cp, addr, n)
            r["mbind_rc"] = rc
            out["register_n%d" % nd] = r
        except RuntimeError as e:
            out["register_n%d" % nd] = {"error": str(e)}
    if "--free-test" in sys.argv:
        for gb in (0, 25, 0, 100):
            out["after_free_%dGB" % gb + ("_b" if "after_free_%dGB" % gb in out else "")] = after_free(n, p, gb)
    if "--thp" in sys.argv:
        tb, taddr, trc = thp_buffer(n)
        out["thp_buffer"] = {"madvise_rc": trc, "thp_kB": numa_info.thp_kb(taddr),
                             "pages_by_node": numa_info.page_nodes(taddr, n)}
        try:
            out["thp_enabled"] = open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip()
        except OSError:
            pass
        out["interleaved"] = interleaved(n, {"hipHostMalloc_4k": p.value, "registered_thp": taddr})
    if "--streams" in sys.argv:
        out["streams"] = per_stream(n, p)
        out["HSA_ENABLE_SDMA"] = os.environ.get("HSA_ENABLE_SDMA")
    if "--after-load" in sys.argv:
        out["default_again_before_load"] = {"GBs": cp.rate(p)}
        load_conditions()
        out["default_old_buffer_after_load"] = {"GBs": cp.rate(p)}
        out["default_new_buffer_after_load"] = one(cp, host_malloc(n), n)
        out["thread_after_load"] = numa_info.thread_node()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
