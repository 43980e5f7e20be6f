"""parameter_server_amd — MI355X-native parameter-shard Add/Get (the server-side
storage hot path of tkwong/parameter_server), as hand-written gfx950 HIP kernels
behind a C ABI (include/pskv.h, libpskv.so).

Importing this package loads libpskv.so and raises if it is missing: there is
no CPU fallback on the product path.
"""
from ._lib import PskvError, lib  # noqa: F401  (fails loudly if the HIP library is absent)
from .shard import (HostFrame, Shard, device_count, host_pool_stats, host_pool_trim,  # noqa: F401
                    jump_hash, range_slice)
from .storage import (AbstractStorage, CheckError, ConsistentHashingPartitionManager, Flag,  # noqa: F401
                      HipStorage, Message, Meta, RangePartitionManager, typed)

__all__ = ["Shard", "HipStorage", "AbstractStorage", "Message", "Meta", "Flag",
           "RangePartitionManager", "ConsistentHashingPartitionManager", "range_slice", "jump_hash",
           "device_count", "CheckError", "PskvError", "HostFrame", "host_pool_stats", "host_pool_trim"]
