"""Sketch-task configuration, same YAML keys as the reference.

Reference: internal/config/config.go:56-86 (SketchTaskDef, SketchAggregatorConfig,
AggregatorConfig) and :163-186 (LoadConfig: os.ExpandEnv over the file).  The
misspelled keys `size_thereshold` / `count_thereshold` are the public keys and
are kept.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import List, Optional

import yaml


@dataclass
class SketchTaskDef:
    Name: str = ""
    SketchType: int = 0          # skt_type: 0 CountMin, 1 SuperSpread
    FlowFields: List[str] = field(default_factory=list)
    ElementFields: List[str] = field(default_factory=list)
    Width: int = 0
    Depth: int = 0
    SizeThreshold: int = 0       # size_thereshold
    CountThreshold: int = 0      # count_thereshold
    M: int = 0
    Size: int = 0
    Base: float = 0.0
    B: float = 0.0

    _YAML = {"name": "Name", "skt_type": "SketchType", "flow_fields": "FlowFields",
             "element_fields": "ElementFields", "width": "Width", "depth": "Depth",
             "size_thereshold": "SizeThreshold", "count_thereshold": "CountThreshold", "m": "M",
             "size": "Size", "base": "Base", "b": "B"}

    @classmethod
    def from_dict(cls, d: dict) -> "SketchTaskDef":
        kw = {}
        for k, v in (d or {}).items():
            attr = cls._YAML.get(k)
            if attr is not None:
                kw[attr] = v
        t = cls(**kw)
        t.FlowFields = list(t.FlowFields or [])
        t.ElementFields = list(t.ElementFields or [])
        for a in ("SketchType", "Width", "Depth", "SizeThreshold", "CountThreshold", "M", "Size"):
            setattr(t, a, int(getattr(t, a) or 0))
        t.Base, t.B = float(t.Base or 0), float(t.B or 0)
        return t


@dataclass
class ExactTaskDef:  # config.go:42-47
    Name: str = ""
    NumShards: int = 0
    KeyFields: List[str] = field(default_factory=list)

    @classmethod
    def from_dict(cls, d: dict) -> "ExactTaskDef":
        d = d or {}
        return cls(str(d.get("name", "") or ""), int(d.get("num_shards", 0) or 0), list(d.get("key_fields", []) or []))


@dataclass
class ExactAggregatorConfig:  # config.go:49-53
    Tasks: List[ExactTaskDef] = field(default_factory=list)
    Writers: List[dict] = field(default_factory=list)


@dataclass
class SketchAggregatorConfig:
    Tasks: List[SketchTaskDef] = field(default_factory=list)
    Writers: List[dict] = field(default_factory=list)  # writers are out of scope; kept verbatim


@dataclass
class AggregatorConfig:
    Types: List[str] = field(default_factory=list)
    Period: str = "720h"
    NumWorkers: int = 1
    SizeOfPacketChannel: int = 10000
    Sketch: SketchAggregatorConfig = field(default_factory=SketchAggregatorConfig)
    Exact: ExactAggregatorConfig = field(default_factory=ExactAggregatorConfig)


@dataclass
class Config:
    Aggregator: AggregatorConfig = field(default_factory=AggregatorConfig)
    raw: Optional[dict] = None


def parse_config(text: str) -> Config:
    """LoadConfig semantics: expand ${VAR} from the environment, then YAML."""
    doc = yaml.safe_load(os.path.expandvars(text)) or {}
    agg = doc.get("aggregator", {}) or {}
    sk = agg.get("sketch", {}) or {}
    ex = agg.get("exact", {}) or {}
    cfg = Config(raw=doc)
    cfg.Aggregator = AggregatorConfig(
        Types=list(agg.get("types", []) or []),
        Period=str(agg.get("period", "720h")),
        NumWorkers=int(agg.get("num_workers", 1) or 1),
        SizeOfPacketChannel=int(agg.get("size_of_packet_channel", 10000) or 10000),
        Sketch=SketchAggregatorConfig(
            Tasks=[SketchTaskDef.from_dict(t) for t in (sk.get("tasks", []) or [])],
            Writers=list(sk.get("writers", []) or [])),
        Exact=ExactAggregatorConfig(
            Tasks=[ExactTaskDef.from_dict(t) for t in (ex.get("tasks", []) or [])],
            Writers=list(ex.get("writers", []) or [])))
    return cfg


def load_config(path: str) -> Config:
    with open(path, "r", encoding="utf-8") as f:
        return parse_config(f.read())
