"""Where host memory and threads sit relative to the GPU (diagnostics for the H2D legs).

page_nodes(addr, nbytes): the NUMA node of sampled pages of a buffer, from move_pages(2) in
query mode (nodes = NULL: each page's status is its node, or -errno) -- the kernel's own
answer for those pages, whatever allocator made them.  gpu_node(device): the PCI device's
numa_node from sysfs (bus id from hipDeviceGetPCIBusId, no framework).  thread_node(): the
node of the CPU this thread runs on.  thp_kb(addr): AnonHugePages of the mapping that holds
addr (/proc/self/smaps).
"""
from __future__ import annotations

import ctypes as C
import glob
import os
from collections import Counter

_libc = C.CDLL(None, use_errno=True)
SYS_move_pages = 279   # x86_64
PAGE = os.sysconf("SC_PAGE_SIZE")


def page_nodes(addr, nbytes, samples=256):
    """{node: pages} over `samples` pages spread evenly over [addr, addr + nbytes)."""
    n = max(1, min(samples, nbytes // PAGE))
    base = addr - addr % PAGE
    pages = (C.c_void_p * n)(*[base + (nbytes * i // n) // PAGE * PAGE for i in range(n)])
    status = (C.c_int * n)()
    rc = _libc.syscall(SYS_move_pages, 0, C.c_ulong(n), pages, None, status, 0)
    if rc != 0:
        return {"error": C.get_errno()}
    return dict(Counter(int(s) for s in status))


def cpu_node(cpu):
    for p in glob.glob("/sys/devices/system/cpu/cpu%d/node[0-9]*" % cpu):
        return int(p.rsplit("node", 1)[1])
    return -1


def thread_node():
    cpu = _libc.sched_getcpu()
    return {"cpu": cpu, "node": cpu_node(cpu)}


def _kfd_gpu_bus(device):
    """The PCI address of the device-th GPU in the KFD topology (nodes with SIMDs, in node
    order: HIP's device order when no *_VISIBLE_DEVICES filter is set), or None."""
    gpus = []
    for d in glob.glob("/sys/class/kfd/kfd/topology/nodes/*"):
        try:
            props = dict(ln.split() for ln in open(os.path.join(d, "properties")) if len(ln.split()) == 2)
        except OSError:
            continue
        if int(props.get("simd_count", 0)) > 0:
            loc, dom = int(props.get("location_id", 0)), int(props.get("domain", 0))
            gpus.append((int(os.path.basename(d)), "%04x:%02x:%02x.%x" % (dom, loc >> 8, (loc >> 3) & 31, loc & 7)))
    gpus.sort()
    return gpus[device][1] if device < len(gpus) else None


def gpu_node(device=0):
    """{"bus", "node"} of the GPU: the bus id from hipDeviceGetPCIBusId when this process's
    HIP runtime sees the device, else from the KFD topology (a process whose torch bundles
    another HIP runtime may not see it through libamdhip64), and the PCI device's numa_node."""
    bus = None
    try:
        try:
            hip = C.CDLL("libamdhip64.so")
        except OSError:
            hip = C.CDLL("/opt/rocm/lib/libamdhip64.so")
        buf = C.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, device) == 0:
            bus = buf.value.decode().lower()
    except OSError:
        pass
    how = "hip"
    if bus is None:
        bus, how = _kfd_gpu_bus(device), "kfd"
    if bus is None:
        return {"bus": None, "node": -1, "from": None}
    try:
        node = int(open("/sys/bus/pci/devices/%s/numa_node" % bus).read())
    except OSError:
        node = -1
    return {"bus": bus, "node": node, "from": how}


def thp_kb(addr):
    """AnonHugePages (kB) of the mapping holding addr, -1 if not found."""
    try:
        with open("/proc/self/smaps") as f:
            inside = False
            for ln in f:
                head = ln.split()[0]
                if "-" in head and not head.endswith(":"):
                    lo, hi = (int(x, 16) for x in head.split("-"))
                    inside = lo <= addr < hi
                elif inside and head == "AnonHugePages:":
                    return int(ln.split()[1])
    except OSError:
        pass
    return -1


def node_meminfo():
    """{node: {"free_MB": .., "total_MB": ..}} from sysfs."""
    out = {}
    for p in sorted(glob.glob("/sys/devices/system/node/node[0-9]*/meminfo")):
        node = int(p.split("/node")[-1].split("/")[0])
        d = {}
        for ln in open(p):
            parts = ln.split()
            if parts[2] in ("MemTotal:", "MemFree:"):
                d[parts[2][3:-1].lower() + "_MB"] = int(parts[3]) // 1024
        out[node] = d
    return out


def placement(addr, nbytes):
    return {"pages_by_node": page_nodes(addr, nbytes), "thp_kB": thp_kb(addr), "thread": thread_node()}
