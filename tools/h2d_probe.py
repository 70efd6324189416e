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
    if "--after-load" in sys.argv:
        out["default_again_before_load"] = {"GBs": cp.rate(p)}
        load_conditions()
        out["default_old_buffer_after_load"] = {"GBs": cp.rate(p)}
        out["default_new_buffer_after_load"] = one(cp, host_malloc(n), n)
        out["thread_after_load"] = numa_info.thread_node()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
