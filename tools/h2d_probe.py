"""PCIe H2D probe (diagnostic, not a result): the GPU's NUMA node, where this process's pinned
pages land, and the pinned -> device copy rate with the pinned pages bound to each NUMA node
(set_mempolicy(MPOL_BIND) around the allocation)."""
import ctypes, glob, json, os, sys, time
import torch

libc = ctypes.CDLL(None, use_errno=True)
SYS_set_mempolicy, SYS_get_mempolicy = 238, 239   # x86_64
MPOL_DEFAULT, MPOL_BIND = 0, 2


def page_node(addr):
    mode = ctypes.c_int(-1)
    rc = libc.syscall(SYS_get_mempolicy, ctypes.byref(mode), None, ctypes.c_ulong(0), ctypes.c_void_p(addr),
                      ctypes.c_ulong(3))   # MPOL_F_NODE | MPOL_F_ADDR
    return mode.value if rc == 0 else -1


def bind(node):
    if node is None:
        return libc.syscall(SYS_set_mempolicy, MPOL_DEFAULT, None, ctypes.c_ulong(0))
    mask = ctypes.c_ulong(1 << node)
    return libc.syscall(SYS_set_mempolicy, MPOL_BIND, ctypes.byref(mask), ctypes.c_ulong(64))


def h2d(mb, node, reps=8):
    bind(node)
    h = torch.empty(mb << 20, dtype=torch.uint8).pin_memory()
    bind(None)
    d = torch.empty(mb << 20, dtype=torch.uint8, device="cuda")
    d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    r = reps * (mb << 20) / (time.perf_counter() - t) / 1e9
    return {"pages_on_node": page_node(h.data_ptr()), "GBs": round(r, 2)}


if __name__ == "__main__":
    p = torch.cuda.get_device_properties(0)
    bus = "%04x:%02x:%02x.0" % (getattr(p, "pci_domain_id", 0), getattr(p, "pci_bus_id", 0), getattr(p, "pci_device_id", 0))
    gnode = -1
    try:
        gnode = int(open("/sys/bus/pci/devices/%s/numa_node" % bus).read())
    except OSError:
        pass
    nodes = sorted(int(x.rsplit("node", 1)[1]) for x in glob.glob("/sys/devices/system/node/node[0-9]*"))
    cpus = sorted(os.sched_getaffinity(0))
    out = {"gpu_bus": bus, "gpu_numa_node": gnode, "numa_nodes": nodes, "affinity_cpus": [cpus[0], cpus[-1], len(cpus)],
           "default": h2d(256, None)}
    for n in nodes:
        out["bound_node%d" % n] = h2d(256, n)
    print(json.dumps(out), flush=True)
