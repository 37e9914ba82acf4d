"""Aggregator registry and the batch Manager.

Reference: internal/factory/task_factory.go:12-52 (TaskGroup, RegisterAggregator
panics on duplicates, Create builds groups from aggregator.types) and
internal/engine/manager/manager.go (worker pool, snapshotter, resetter).

The Manager keeps the reference's lifecycle (start -> packets -> snapshot /
reset -> stop) but replaces the goroutine worker pool fed one *PacketInfo at a
time (manager.go:218-244) with batch submission: every task receives each
packet batch in arrival order on its GPU stream.  Writers (ClickHouse / text),
alerting and the timers are out of scope for this build.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List

from .config import Config
from .task import SketchTask


@dataclass
class TaskGroup:
    Tasks: List[SketchTask] = field(default_factory=list)
    Writers: List[object] = field(default_factory=list)


TaskFactory = Callable[[Config], TaskGroup]
_registry: Dict[str, TaskFactory] = {}


def register_aggregator(name: str, factory: TaskFactory) -> None:
    if name in _registry:  # task_factory.go:25-27 panics
        raise RuntimeError(f"aggregator type '{name}' already registered")
    _registry[name] = factory


def create(cfg: Config, **task_kw) -> List[TaskGroup]:
    groups = []
    for agg in cfg.Aggregator.Types:
        f = _registry.get(agg)
        if f is None:
            raise KeyError(f"unknown aggregator type: '{agg}'")
        groups.append(f(cfg, **task_kw))
    return groups


def _sketch_factory(cfg: Config, **task_kw) -> TaskGroup:  # sketch/task.go:21-65
    return TaskGroup(Tasks=[SketchTask(t, **task_kw) for t in cfg.Aggregator.Sketch.Tasks], Writers=[])


def _exact_factory(cfg: Config, device: int = 0, max_flows: int = 0, batch_packets: int = 0,
                   **_sketch_only) -> TaskGroup:  # exact/task.go:20-64
    from .exact import ExactTask
    return TaskGroup(Tasks=[ExactTask(t.Name, t.KeyFields, t.NumShards, device=device, max_flows=max_flows,
                                      batch_packets=batch_packets) for t in cfg.Aggregator.Exact.Tasks], Writers=[])


register_aggregator("sketch", _sketch_factory)
register_aggregator("exact", _exact_factory)
RegisterAggregator = register_aggregator
Create = create


def key_fields(task) -> List[str]:
    """The fields a task keys its flows on: FlowFields (sketch, task.go:265-300) or
    KeyFields (exact, exact/task.go:330-366)."""
    if hasattr(task, "flow_fields"):
        return list(task.flow_fields)
    return list(task.agg.key_fields)


class Manager:
    """Batch-submission replacement of manager.Manager."""

    def __init__(self, cfg: Config, **task_kw):
        self.groups = create(cfg, **task_kw)
        self.started = False

    def tasks(self) -> List[SketchTask]:
        return [t for g in self.groups for t in g.Tasks]

    def start(self) -> None:
        self.started = True

    def owner_fields(self) -> List[str]:
        """The owner key for sharding this Manager's tasks over GPUs (dist.owner_fields):
        every task sees every packet (manager.go:232-244), so one owner must hold
        each flow of every task.  Raises ValueError when the tasks share no key field."""
        from .dist import owner_fields
        return owner_fields([key_fields(t) for t in self.tasks()])

    def process(self, batch) -> None:
        """processPacket (manager.go:232-244) for a whole batch: fan out to every task."""
        for t in self.tasks():
            t.process_packets(batch)

    def snapshot(self) -> Dict[str, object]:
        """takeSnapshotForWriter without writers: name -> HeavyRecord (sketch) / SnapshotData (exact)."""
        return {t.name(): t.snapshot() for t in self.tasks()}

    def reset_all(self) -> None:  # resetAllTasks, manager.go:179-193
        for t in self.tasks():
            t.reset()

    def stop(self) -> Dict[str, object]:
        """Drain (flush every stream) and take the final snapshot (manager.go:196-216)."""
        for t in self.tasks():
            t.flush()
        self.started = False
        return self.snapshot()
