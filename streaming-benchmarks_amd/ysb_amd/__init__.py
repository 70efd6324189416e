"""ysb_amd: host-side binding of the MI355X-native YSB advertising hot path.

The compute path is libysb_hip.so (HIP kernels for gfx950, C ABI in include/ysb_hip.h);
this package only binds it.  There is no CPU fallback.
"""
from ._lib import LIB_PATH, YsbError, lib  # noqa: F401
from .admap import AdCampaignMap  # noqa: F401
from .context import YsbContext, device_count, device_sync, rank_device  # noqa: F401
from .source import FileBasedDataSource  # noqa: F401
from .generator import (AD_TYPES, EVENT_TYPES, GEN_COMPACT, GEN_MIXED, GEN_MIXED_BLOCKS, GEN_MORE_AD_TYPES, GEN_RANDOM_IP, GEN_REORDER,  # noqa: F401
                        MORE_AD_TYPES, GenParams, ad_shard, json_to_tbl, layout_of_line, shard_ads, shard_packed)
from .group import (exchange_mismatches, exchange_plan, owned_block, ring_agreement, route_lines, split_batch,  # noqa: F401
                    table_rows)
