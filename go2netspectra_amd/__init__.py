"""go2netspectra_amd -- MI355X-native sketch hot path for Go2NetSpectra.

Drop-in for the reference's per-packet sketch path (internal/engine/impl/sketch):
header parse -> flow-key encode -> d seeded MurmurHash3 -> fingerprinted
Count-Min / SuperSpread bucket updates, plus the exact per-flow aggregator
(internal/engine/impl/exact), executed by hand-written gfx950 HIP kernels
behind the C ABI in include/gns_sketch.h (libgns_sketch.so).
"""
from ._lib import GnsError, build, load
from .config import Config, ExactTaskDef, SketchTaskDef, load_config, parse_config
from .exact import ExactAggregator, ExactTask, NewExact, SnapshotData
from .factory import Manager, TaskGroup, create, register_aggregator
from .packets import (HeaderBatch, PacketBatch, SyntheticTraffic, compact_headers, ip_slot, read_pcap,
                      read_pcap_compact, write_pcap, write_pcapgen, write_pcapng)
from .sketch import CountMin, CountMinView, HeavyCount, HeavyRecord, HeavySize, SuperSpread
from .task import New, SketchTask, decode_flow

__all__ = [
    "GnsError", "build", "load", "Config", "SketchTaskDef", "load_config", "parse_config", "Manager",
    "TaskGroup", "create", "register_aggregator", "HeaderBatch", "PacketBatch", "SyntheticTraffic",
    "ip_slot", "read_pcap", "read_pcap_compact", "compact_headers", "write_pcap", "write_pcapgen", "write_pcapng", "CountMin", "CountMinView", "HeavyCount", "HeavyRecord", "HeavySize",
    "SuperSpread", "New", "SketchTask", "decode_flow", "ExactTaskDef", "ExactAggregator", "ExactTask",
    "NewExact", "SnapshotData",
]
