"""ina_amd -- MI355X-native gradient-aggregation path (drop-in for the in-switch
aggregator and worker quantise/packetise code of distributed-training-INA).

Device ops live in ina_amd.ops (libina.so via ctypes); the reference's host
surfaces are mirrored in ina_amd.communicator (communicator.py), ina_amd.
data_manager (DataManager.py), ina_amd.packet (NGAPacket.py / header_config.py)
and ina_amd.ps (launch.py's aggregate / communication_parallel / Worker); buckets that
outgrow one GPU go through ina_amd.dist (ShardedAggregator: reduce-scatter + all-gather
over RCCL; RangeAggregator: range-split worker slices, one all-gather).
"""
from ._lib import (ACT_DROP, ACT_FWD_ACK, ACT_FWD_AGG, ACT_FWD_COLLISION, ACT_FWD_OTHER,  # noqa: F401
                   C128_BYTES, C128_VALUES, FLAG_ACK, FLAG_COLLISION, FLAG_OVERFLOW,
                   FLAG_RESEND, InaError, LIB_PATH, MAX_WORKERS, NGA_HDR_BYTES, NUM_REGISTER)

__version__ = "0.1.0"
