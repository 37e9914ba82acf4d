"""ctypes binding of libgns_sketch.so (the C ABI in include/gns_sketch.h).

The product path has no CPU fallback: if the HIP library is missing or no GPU
is present, every engine constructor raises.
"""
from __future__ import annotations

import ctypes as ct
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GNS_LIB") or os.path.join(_HERE, "libgns_sketch.so")
CSRC = os.path.join(_HERE, "csrc")

GNS_OK = 0
GNS_E_ARG, GNS_E_HIP, GNS_E_OOM, GNS_E_FULL, GNS_E_RANGE, GNS_E_NODEV = -1, -2, -3, -4, -5, -6
ERRORS = {-1: "GNS_E_ARG", -2: "GNS_E_HIP", -3: "GNS_E_OOM", -4: "GNS_E_FULL", -5: "GNS_E_RANGE",
          -6: "GNS_E_NODEV"}
MEM_HOST, MEM_DEVICE = 0, 1

FIELD_IDS = {"SrcIP": 1, "DstIP": 2, "SrcPort": 3, "DstPort": 4, "Protocol": 5}
FIELD_NAMES = {v: k for k, v in FIELD_IDS.items()}
FIELD_SIZE = {"SrcIP": 16, "DstIP": 16, "SrcPort": 2, "DstPort": 2, "Protocol": 1}

EXPORTED = [
    "gns_cm_create", "gns_cm_destroy", "gns_cm_insert_keys", "gns_cm_insert_tuples",
    "gns_cm_insert_headers", "gns_cm_flush", "gns_cm_query", "gns_cm_query_device", "gns_cm_heavy_hitters", "gns_cm_reset",
    "gns_cm_export_state", "gns_cm_stats", "gns_cm_counters", "gns_cm_set_timing", "gns_cm_stage_times", "gns_cm_stream",
    "gns_cm_view_create", "gns_cm_view_destroy", "gns_cm_view_refresh", "gns_cm_view_heavy_hitters",
    "gns_cm_view_query",
    "gns_ss_create", "gns_ss_destroy", "gns_ss_insert_keys", "gns_ss_insert_tuples",
    "gns_ss_insert_headers", "gns_ss_flush", "gns_ss_query", "gns_ss_query_device", "gns_ss_heavy_hitters", "gns_ss_reset",
    "gns_ss_export_state", "gns_ss_stats", "gns_ss_counters", "gns_ss_set_timing", "gns_ss_stage_times",
    "gns_synth_create", "gns_synth_destroy", "gns_synth_fill", "gns_synth_flows",
    "gns_ex_create", "gns_ex_destroy", "gns_ex_insert_tuples", "gns_ex_insert_headers", "gns_ex_flush",
    "gns_ex_query", "gns_ex_query_device", "gns_ex_snapshot", "gns_ex_reset", "gns_ex_counters", "gns_ex_set_timing",
    "gns_ex_stage_times",
    "gns_thrift_decode", "gns_pack_pcap", "gns_pack_pcap_ts", "gns_pack_counts", "gns_frame_record", "gns_last_error", "gns_version",
    "gns_route_create", "gns_route_destroy", "gns_route_partition",
    "gns_cm_dict_stats", "gns_ss_dict_stats", "gns_ex_dict_stats", "gns_cm_reclaim", "gns_ss_reclaim",
    "gns_cm_insert_compact", "gns_pack_pcap_compact", "gns_compact_headers", "gns_route_partition_async",
    "gns_pack_pcap_compact16", "gns_compact_headers16",
    "gns_route_owner_fields", "gns_route_create_keyed", "gns_route_owner_layout", "gns_route_owner_keys",
    "gns_device_alloc", "gns_device_free", "gns_cm_heavy_rows", "gns_hh_order_rows",
]


class GnsError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class Layout(ct.Structure):
    _fields_ = [("n_fields", ct.c_uint32), ("fields", ct.c_uint8 * 8)]

    @classmethod
    def of(cls, fields) -> "Layout":
        fields = list(fields or [])
        if len(fields) > 8:
            raise ValueError("at most 8 key fields")
        lay = cls()
        lay.n_fields = len(fields)
        for i, f in enumerate(fields):
            lay.fields[i] = FIELD_IDS.get(f, 0)  # unknown names contribute 0 bytes (task.go:335)
        return lay

    def names(self):
        return [FIELD_NAMES.get(int(self.fields[i]), "") for i in range(self.n_fields)]


class Tuples(ct.Structure):
    _fields_ = [("src16", ct.c_void_p), ("dst16", ct.c_void_p), ("sport", ct.c_void_p),
                ("dport", ct.c_void_p), ("proto", ct.c_void_p), ("length", ct.c_void_p)]


class CmParams(ct.Structure):
    _fields_ = [("width", ct.c_uint32), ("depth", ct.c_uint32), ("size_threshold", ct.c_uint32),
                ("count_threshold", ct.c_uint32), ("flow", Layout), ("key_bytes", ct.c_uint32),
                ("seeds", ct.c_void_p), ("max_flows", ct.c_uint64), ("batch_packets", ct.c_uint64),
                ("device", ct.c_int), ("bucket_lo", ct.c_uint32), ("bucket_hi", ct.c_uint32)]


class SsParams(ct.Structure):
    _fields_ = [("width", ct.c_uint32), ("depth", ct.c_uint32), ("threshold", ct.c_uint32),
                ("m", ct.c_uint32), ("size", ct.c_uint32), ("base", ct.c_double), ("b", ct.c_double),
                ("flow", Layout), ("elem", Layout), ("flow_bytes", ct.c_uint32),
                ("elem_bytes", ct.c_uint32), ("seeds", ct.c_void_p), ("hll_master", ct.c_uint64),
                ("rng_seed", ct.c_uint64), ("batch_packets", ct.c_uint64), ("max_flows", ct.c_uint64),
                ("device", ct.c_int)]


class ExParams(ct.Structure):
    _fields_ = [("key", Layout), ("max_flows", ct.c_uint64), ("batch_packets", ct.c_uint64), ("device", ct.c_int)]


class SynthParams(ct.Structure):
    _fields_ = [("flows", ct.c_uint32), ("zipf_s", ct.c_double), ("tuple_seed", ct.c_uint64),
                ("rank_seed", ct.c_uint64), ("len_seed", ct.c_uint64), ("shard", ct.c_uint32),
                ("nshards", ct.c_uint32), ("device", ct.c_int), ("fanout", ct.c_uint32)]


_lib = None


def build(verbose: bool = False) -> str:
    """Compile csrc/ for gfx950 into libgns_sketch.so (in-tree)."""
    jobs = min(8, os.cpu_count() or 1)
    out = subprocess.run(["make", "-C", CSRC, f"-j{jobs}"], capture_output=not verbose, text=True)
    if out.returncode != 0:
        raise RuntimeError("libgns_sketch build failed:\n" + (out.stdout or "") + (out.stderr or ""))
    return LIB_PATH


def load() -> ct.CDLL:
    """Load libgns_sketch.so; raises if it is not built (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing: run `make -C {CSRC}` or __graft_entry__.build()")
    L = ct.CDLL(LIB_PATH)
    vp, u32, u64, i32 = ct.c_void_p, ct.c_uint32, ct.c_uint64, ct.c_int
    sig = {
        "gns_cm_create": ([vp, vp], i32), "gns_cm_destroy": ([vp], i32),
        "gns_cm_insert_keys": ([vp, vp, u32, vp, u64, i32], i32),
        "gns_cm_insert_tuples": ([vp, vp, u64, i32], i32),
        "gns_cm_insert_headers": ([vp, vp, vp, u64, i32], i32),
        "gns_cm_flush": ([vp], i32), "gns_cm_query": ([vp, vp, u32, u64, vp], i32),
        "gns_cm_query_device": ([vp, vp, u32, u64, vp], i32),
        "gns_cm_heavy_hitters": ([vp, vp, vp, vp, vp, vp, vp], i32), "gns_cm_reset": ([vp], i32),
        "gns_cm_export_state": ([vp, vp, vp, vp, vp], i32), "gns_cm_stats": ([vp, vp], i32),
        "gns_cm_counters": ([vp, vp], i32),
        "gns_cm_set_timing": ([vp, i32], i32), "gns_cm_stage_times": ([vp, vp, vp, i32], i32),
        "gns_cm_stream": ([vp], vp),
        "gns_cm_view_create": ([vp, vp], i32), "gns_cm_view_destroy": ([vp], i32),
        "gns_cm_view_refresh": ([vp], i32), "gns_cm_view_heavy_hitters": ([vp, vp, vp, vp, vp, vp, vp], i32),
        "gns_cm_view_query": ([vp, vp, u32, u64, vp], i32),
        "gns_ss_create": ([vp, vp], i32), "gns_ss_destroy": ([vp], i32),
        "gns_ss_insert_keys": ([vp, vp, u32, vp, u32, u64, i32], i32),
        "gns_ss_insert_tuples": ([vp, vp, u64, i32], i32),
        "gns_ss_insert_headers": ([vp, vp, vp, u64, i32], i32),
        "gns_ss_flush": ([vp], i32), "gns_ss_query": ([vp, vp, u32, u64, vp], i32),
        "gns_ss_query_device": ([vp, vp, u32, u64, vp], i32),
        "gns_ss_heavy_hitters": ([vp, vp, vp, vp], i32), "gns_ss_reset": ([vp], i32),
        "gns_ss_export_state": ([vp, vp, vp, vp, vp], i32), "gns_ss_stats": ([vp, vp], i32),
        "gns_ss_counters": ([vp, vp], i32),
        "gns_ss_set_timing": ([vp, i32], i32), "gns_ss_stage_times": ([vp, vp, vp, i32], i32),
        "gns_synth_create": ([vp, vp], i32), "gns_synth_destroy": ([vp], i32),
        "gns_synth_fill": ([vp, vp, vp, u64, u64], i32), "gns_synth_flows": ([vp, vp], i32),
        "gns_ex_create": ([vp, vp], i32), "gns_ex_destroy": ([vp], i32),
        "gns_ex_insert_tuples": ([vp, vp, vp, vp, u64, i32], i32),
        "gns_ex_insert_headers": ([vp, vp, vp, vp, u64, i32], i32),
        "gns_ex_flush": ([vp], i32), "gns_ex_query": ([vp, vp, u32, u64, vp], i32),
        "gns_ex_query_device": ([vp, vp, u32, u64, vp], i32),
        "gns_ex_snapshot": ([vp, vp, vp, vp, vp, vp, vp], i32), "gns_ex_reset": ([vp], i32),
        "gns_ex_counters": ([vp, vp], i32), "gns_ex_set_timing": ([vp, i32], i32),
        "gns_ex_stage_times": ([vp, vp, vp, i32], i32),
        "gns_thrift_decode": ([vp, u64, vp, u64, vp, vp, vp, vp, i32, i32], i32),
        "gns_pack_pcap": ([ct.c_char_p, vp, vp, u64, vp], ct.c_int64),
        "gns_pack_pcap_ts": ([ct.c_char_p, vp, vp, vp, u64, vp], ct.c_int64),
        "gns_pack_counts": ([vp], ct.c_int),
        "gns_frame_record": ([vp, ct.c_uint32, ct.c_uint32, vp], ct.c_int),
        "gns_last_error": ([], ct.c_char_p), "gns_version": ([], ct.c_char_p),
        "gns_route_create": ([u32, i32, vp], i32), "gns_route_destroy": ([vp], i32),
        "gns_route_partition": ([vp, vp, vp, u64, vp, vp, vp], i32),
        "gns_cm_dict_stats": ([vp, vp], i32), "gns_ss_dict_stats": ([vp, vp], i32),
        "gns_ex_dict_stats": ([vp, vp], i32), "gns_cm_reclaim": ([vp], i32), "gns_ss_reclaim": ([vp], i32),
        "gns_cm_insert_compact": ([vp, vp, vp, u64, vp, u64, i32], i32),
        "gns_pack_pcap_compact": ([ct.c_char_p, vp, vp, u64, vp, u64, vp, vp], ct.c_int64),
        "gns_compact_headers": ([vp, vp, u64, vp, vp, u64, vp, i32], i32),
        "gns_pack_pcap_compact16": ([ct.c_char_p, vp, u64, vp, u64, vp, vp], ct.c_int64),
        "gns_compact_headers16": ([vp, vp, u64, vp, vp, u64, vp, i32], i32),
        "gns_route_partition_async": ([vp, vp, vp, u64, vp, vp, vp, vp], i32),
        "gns_route_owner_fields": ([vp, u32, vp], i32),
        "gns_route_create_keyed": ([u32, vp, i32, vp], i32),
        "gns_route_owner_layout": ([vp, vp], i32),
        "gns_route_owner_keys": ([vp, vp, vp, u32, u64, vp, i32], i32),
        "gns_device_alloc": ([u64, i32, vp], i32), "gns_device_free": ([vp, i32], i32),
        "gns_cm_heavy_rows": ([vp, vp, vp, vp, vp], i32),
        "gns_hh_order_rows": ([vp, u32, u64, vp, i32], i32),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def device_ready(*arrays) -> None:
    """Device tensors handed to the engine must be complete: the engines launch on
    their own non-blocking streams, which are not ordered after torch's stream
    that produced the data.  Synchronize torch's current stream of every device
    involved (once per device) before the call."""
    seen = set()
    for a in arrays:
        if a is None or not getattr(a, "is_cuda", False):
            continue
        d = a.device.index
        if d in seen:
            continue
        seen.add(d)
        import torch
        torch.cuda.current_stream(a.device).synchronize()


def is_device(a) -> bool:
    return bool(getattr(a, "is_cuda", False))


def query_device(fn, h, keys):
    """A *_query_device call: keys a device uint8 tensor [n, K] on the handle's GPU ->
    a device int64 tensor [n] holding the uint64 answers (no host copy either way)."""
    import torch
    n = int(keys.shape[0])
    out = torch.empty((n,), dtype=torch.int64, device=keys.device)
    if n:
        keys = keys.reshape(n, -1).contiguous()
        if keys.dtype != torch.uint8:
            raise TypeError(f"device keys must be uint8, not {keys.dtype}")
        device_ready(keys)
        check(fn(h, keys.data_ptr(), int(keys.shape[1]), n, out.data_ptr()))
    return out


DICT_STATS = ["reclaims", "dropped", "live", "claimed", "reclaim_us", "retried_batches", "slots", "growths"]


def dict_stats(fn, h) -> dict:
    out = (ct.c_uint64 * 8)()
    check(fn(h, out))
    return dict(zip(DICT_STATS, list(out)))


GNS_TIMING_MASK = 0x100


def timing_arg(on, stages, names) -> int:
    """gns_*_set_timing's argument: 0 off, 1 every stage, GNS_TIMING_MASK | bits for ``stages``."""
    if not on:
        return 0
    if stages is None:
        return 1
    bits = 0
    for s in stages:
        if s not in names:
            raise ValueError(f"unknown stage {s!r} (stages: {list(names)})")
        bits |= 1 << names.index(s)
    return GNS_TIMING_MASK | bits


def check(code: int) -> None:
    if code != GNS_OK:
        msg = (load().gns_last_error() or b"").decode(errors="replace")
        raise GnsError(code, msg)


def layout_bytes(fields) -> int:
    return sum(FIELD_SIZE.get(f, 0) for f in (fields or []))
