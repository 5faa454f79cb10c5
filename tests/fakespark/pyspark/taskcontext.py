"""TaskContext / BarrierTaskContext: ``get()`` returns the context the fake executor installed."""
from typing import Any, Optional

_current: Optional[Any] = None


def _install(ctx: Any) -> None:
    global _current
    _current = ctx


class TaskContext:
    def __init__(self, partition_id: int) -> None:
        self._pid = partition_id

    @staticmethod
    def get() -> Optional[Any]:
        return _current

    def partitionId(self) -> int:
        return self._pid

    def resources(self) -> dict:
        return {}


class BarrierTaskContext(TaskContext):
    @staticmethod
    def get() -> Optional[Any]:
        return _current
