"""rlo -- MI355X-native rootless collective engine (host side).

Importing this package loads librlo_hip.so (built in-tree); there is no CPU fallback.
"""
from ._lib import load, RloError, LIB_PATH  # noqa: F401
from .world import World, topology, children, hist_percentile, bulk_plan, storm_lengths, layout_plan, pool_trim, pool_stats  # noqa: F401
from . import _lib as abi  # noqa: F401
from .host import HostWorld  # noqa: F401

load()
