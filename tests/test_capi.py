"""CPU: the C-ABI library loads, exports every symbol include/ysb_hip.h declares, its
structs match the ctypes mirror, and the host-side arithmetic shared with the
device is exact.  No compute calls (no GPU here)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from ysb_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ysb_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*[A-Za-z_][A-Za-z0-9_\s\*]*?\b(ysb_[a-z0-9_]+)\s*\(", src, flags=re.M)))


def test_header_declares_the_boundary():
    fns = declared_functions()
    for f in ("ysb_open", "ysb_load_ad_map", "ysb_submit", "ysb_submit_device", "ysb_drain", "ysb_stats_get",
              "ysb_close", "ysb_group_init", "ysb_group_reduce_scatter", "ysb_last_error"):
        assert f in fns
    assert len(fns) >= 30


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    missing = [f for f in declared_functions() if not hasattr(L, f)]
    assert missing == []


def test_ctypes_signatures_cover_header():
    assert sorted(_lib.SIGNATURES) == declared_functions()


def test_nm_shows_extern_c_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    syms = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    assert set(declared_functions()) <= syms


STRUCT_PROBE = r"""
#include <stddef.h>
#include <stdio.h>
#include "ysb_hip.h"
#define P(T, F) printf(#T "." #F " %zu\n", offsetof(T, F));
int main(void) {
  printf("ysb_config %zu\nysb_stats %zu\nysb_count %zu\nysb_gen_params %zu\nysb_exchange_info %zu\n",
         sizeof(ysb_config), sizeof(ysb_stats), sizeof(ysb_count), sizeof(ysb_gen_params), sizeof(ysb_exchange_info));
  P(ysb_config, flags) P(ysb_config, overflow_capacity) P(ysb_count, window_ms) P(ysb_count, count)
  P(ysb_gen_params, ad_subset) P(ysb_gen_params, n_ad_subset) P(ysb_stats, batches) P(ysb_stats, deferred)
  P(ysb_stats, foreign_shard) P(ysb_exchange_info, ms) P(ysb_exchange_info, last_width)
  P(ysb_exchange_info, full_ring_bytes) P(ysb_exchange_info, rs_ms) P(ysb_exchange_info, exposed_ms)
  return 0;
}
"""


def test_struct_layouts_match_ctypes(tmp_path):
    src = tmp_path / "probe.c"
    src.write_text(STRUCT_PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(ln.split() for ln in subprocess.run([str(exe)], capture_output=True, text=True).stdout.splitlines())
    assert int(got["ysb_config"]) == C.sizeof(_lib.YsbConfig)
    assert int(got["ysb_stats"]) == C.sizeof(_lib.YsbStats)
    assert int(got["ysb_count"]) == C.sizeof(_lib.YsbCount)
    assert int(got["ysb_gen_params"]) == C.sizeof(_lib.YsbGenParams)
    assert int(got["ysb_config.flags"]) == _lib.YsbConfig.flags.offset
    assert int(got["ysb_config.overflow_capacity"]) == _lib.YsbConfig.overflow_capacity.offset
    assert int(got["ysb_count.window_ms"]) == _lib.YsbCount.window_ms.offset
    assert int(got["ysb_gen_params.ad_subset"]) == _lib.YsbGenParams.ad_subset.offset
    assert int(got["ysb_stats.batches"]) == _lib.YsbStats.batches.offset
    assert int(got["ysb_stats.deferred"]) == _lib.YsbStats.deferred.offset
    assert int(got["ysb_stats.foreign_shard"]) == _lib.YsbStats.foreign_shard.offset
    assert int(got["ysb_exchange_info"]) == C.sizeof(_lib.YsbExchangeInfo)
    for f in ("ms", "last_width", "full_ring_bytes", "rs_ms", "exposed_ms"):
        assert int(got["ysb_exchange_info." + f]) == getattr(_lib.YsbExchangeInfo, f).offset


def test_abi_version_and_defaults():
    L = _lib.lib()
    assert L.ysb_abi_version() == 5 == _lib.ABI_VERSION
    # the struct the caller lays out is the library's (ysb_exchange_info grew in ABI 4)
    assert L.ysb_exchange_info_size() == C.sizeof(_lib.YsbExchangeInfo) == 64
    assert C.sizeof(_lib.YsbRebase) == 16
    cfg = _lib.YsbConfig()
    L.ysb_config_default(C.byref(cfg))
    assert cfg.time_divisor_ms == 10000          # CampaignProcessorCommon.java:28
    assert cfg.n_campaigns == 100                # core.clj:15
    assert cfg.window_ring >= 16 and cfg.window_ring & (cfg.window_ring - 1) == 0
    assert cfg.ring_base_bucket == _lib.INT64_MIN


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is present")
def test_open_without_gpu_fails_loudly():
    from ysb_amd import YsbContext, YsbError
    with pytest.raises(YsbError):
        YsbContext()


def test_bad_config_rejected_before_device_use():
    L = _lib.lib()
    cfg = _lib.YsbConfig()
    L.ysb_config_default(C.byref(cfg))
    cfg.window_ring = 1000   # not a power of two
    h = C.c_void_p()
    assert L.ysb_open(C.byref(h), 0, C.byref(cfg)) == -1
    assert b"window_ring" in L.ysb_last_error(None)


def test_host_logic_native(tmp_path):
    exe = tmp_path / "host_logic"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "streaming-benchmarks_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "host_logic.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout


def test_ad_shard_is_stable_and_balanced():
    from ysb_amd import GenParams, ad_shard
    _, aids = GenParams().ids()
    for n in (1, 2, 4, 8):
        counts = [0] * n
        for a in aids:
            s = ad_shard(a, n)
            assert 0 <= s < n and s == ad_shard(a, n)
            counts[s] += 1
        assert min(counts) > 1000 / n * 0.7


def test_config_flags_match_the_header():
    """Every YSB_F_* flag the header defines has the same value in the ctypes mirror, and
    no two flags share a bit."""
    src = open(HEADER).read()
    flags = {m.group(1): int(m.group(2), 16) for m in re.finditer(r"^#define (YSB_F_\w+)\s+0x([0-9a-fA-F]+)u", src, re.M)}
    assert "YSB_F_COMPACT_FIRST" in flags and "YSB_F_FLAT_FIRST" in flags
    for name, v in flags.items():
        assert getattr(_lib, name) == v, name
    vals = list(flags.values())
    assert all(v & (v - 1) == 0 for v in vals) and len(set(vals)) == len(vals)


def test_exchange_plan_width_and_slots():
    """ysb_exchange_plan: the touched slots ascending, and the narrowest cell width whose sum
    over the ranks cannot wrap (RCCL has no 16-bit integer type: 1, 4 or 8 bytes)."""
    import numpy as np
    from ysb_amd import YsbError, exchange_plan
    m = np.zeros(64, dtype=np.uint64)
    slots, w = exchange_plan(m, 8)
    assert slots.size == 0 and w == 1
    m[[3, 9, 63]] = [1, 31, 2]
    slots, w = exchange_plan(m, 8)
    assert slots.tolist() == [3, 9, 63] and w == 1          # 8 * 31 = 248 <= 255
    assert exchange_plan(m, 9)[1] == 4                      # 9 * 31 = 279
    m[9] = (1 << 32) // 8 - 1
    assert exchange_plan(m, 8)[1] == 4
    m[9] = 1 << 32
    assert exchange_plan(m, 8)[1] == 8
    m[9] = (1 << 63)
    with pytest.raises(YsbError):
        exchange_plan(m, 8)


def test_load_shard_arguments_checked_without_gpu():
    """The sharded loader rejects a bad shard before touching a device."""
    L = _lib.lib()
    assert L.ysb_load_ad_map_shard(None, None, None, None, 0, 0, 1) == -1


def test_route_lines_hashes_the_decoded_ad_id():
    """ysb_route_lines decodes org.json escapes in the ad_id value and the key name (and takes
    single-quoted strings), so an event routes to the same shard however its ad_id is
    written -- the shard the device's decoded-key test expects."""
    import numpy as np
    from ysb_amd import GenParams, route_lines
    g = GenParams(seed=3)
    raw, off = g.events_host(0, 3000)
    lines = [bytes(raw[a:b]) for a, b in zip(off, list(off[1:]) + [raw.size])]

    def esc(line, mode):
        i = line.index(b'"ad_id": "')
        v0 = i + 10
        val = line[v0:v0 + 36]
        if mode == 2:
            return line[:i] + b"'ad_id' : '" + val + b"'" + line[v0 + 37:]
        ev = b"".join((b"\\u%04X" % c) if k % 3 == 0 else bytes([c]) for k, c in enumerate(val))
        return line[:i] + (b'"ad\\u005Fid": "' if mode else b'"ad_id": "') + ev + line[v0 + 36:]

    for mode in (0, 1, 2):
        el = [esc(ln, mode) for ln in lines]
        for n in (2, 3, 8):
            a, _ = route_lines(np.frombuffer(b"".join(lines), dtype=np.uint8),
                               np.cumsum([0] + [len(x) for x in lines[:-1]]), n)
            b, _ = route_lines(np.frombuffer(b"".join(el), dtype=np.uint8),
                               np.cumsum([0] + [len(x) for x in el[:-1]]), n)
            assert np.array_equal(a, b), (mode, n)


def test_no_device_error_names_the_cause():
    """ysb_device_sync / ysb_open without a visible device: YSB_ERR_HIP, and the message names
    the likely cause (here: no /dev/kfd; on a GPU box: another HIP runtime opened it first)."""
    import os
    import pytest
    from ysb_amd import YsbContext, YsbError, device_sync
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU driver is present")
    with pytest.raises(YsbError, match="no /dev/kfd"):
        device_sync(0)
    with pytest.raises(YsbError, match="YSB_ERR_HIP"):
        YsbContext()


def test_generator_rejects_unknown_skew_modes():
    import pytest
    from ysb_amd import GenParams, YsbError
    with pytest.raises(ValueError):
        GenParams(with_skew=3)
    g = GenParams()
    g.c.with_skew = 7                                    # past the binding: the library refuses
    with pytest.raises(YsbError, match="YSB_ERR_ARG"):
        g.events_host(0, 10)
