import sys, os, ctypes as C; os.environ['YSB_LIB_VARIANT']='stamps'; sys.path.insert(0,'streaming-benchmarks_amd')
import numpy as np
from ysb_amd import YsbContext, GenParams
from ysb_amd._lib import lib
g = GenParams(seed=42); n = 12_500_000
with YsbContext(n_campaigns=100) as ctx:
    ctx.load_ad_map(g.ids()[1], g.ad_campaign_index()); cap = n * g.max_line_bytes()
    db, do = ctx.device_alloc(cap), ctx.device_alloc(4 * n)
    nb = ctx.gen_events_device(g, 0, n, db, cap, do)
    ctx.submit_device(db, nb, do, n); st = ctx.stats(); print(st)
    L = lib(); L.ysb_debug_defer_list.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
    buf = np.zeros(n, dtype=np.uint32); L.ysb_debug_defer_list(ctx._h, buf.ctypes.data, n)
    d = np.sort(buf[:st['deferred']]); tile = d // 256; lane = d % 256
    print('n deferred', len(d)); print('tiles: min', tile.min(), 'unique', len(np.unique(tile)))
    blocks_tpb = 96; tib = tile % blocks_tpb
    print('tile-in-block histogram (first 8):', np.bincount(tib, minlength=96)[:8], 'max tib', tib.max())
    print('lane histogram by wave:', np.bincount(lane // 64, minlength=4))
    off = ctx.d2h(np.empty(n, dtype=np.uint32), do); data = ctx.d2h(np.empty(nb, dtype=np.uint8), db)
    for i in d[:3]:
        print(i, bytes(data[off[i]:off[i+1]]))
    # first tile of each block?
    print('deferred in first tile of blocks:', np.sum(tib == 0))
