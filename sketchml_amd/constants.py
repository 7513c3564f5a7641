"""common/Constants.java:8-43: the process-wide parallelism of the parallel* methods.

`parallelQuantize` / `parallelCompress*` read it as the number of slice sketches T
(QuantileQuantizer.java:59); the reference's thread pool has no counterpart here because the
slices run as device kernels.
"""
from __future__ import annotations

from .exceptions import SketchMLException


class Parallel:
    """Constants.Parallel (Constants.java:9-41)."""

    _parallelism = 0

    @staticmethod
    def setParallelism(parallelism: int) -> None:
        if int(parallelism) < 1:
            raise SketchMLException(f"Invalid parallelism: {parallelism}")
        Parallel._parallelism = int(parallelism)

    @staticmethod
    def getParallelism() -> int:
        if Parallel._parallelism <= 0:
            raise SketchMLException("Parallelism is not set yet")
        return Parallel._parallelism

    @staticmethod
    def shutdown() -> None:
        """No pool to stop; kept for the reference surface."""


class Constants:
    Parallel = Parallel
