"""The `ml` module's gradient containers around the codec:
DenseDoubleGradient / SparseDoubleGradient (ml/gradient/DenseDoubleGradient.scala,
SparseDoubleGradient.scala) and SketchGradient (ml/gradient/SketchGradient.scala:8-80), the
caller that compresses a worker's gradient.

Values live on the GPU (float32 or float64 tensors).  The compaction (toSparse), quantisation,
MinMax sketch and key codec run in libskml's kernels; this module is the glue the reference
keeps in Scala: which codec to use, bucketValues and its timesBy, the nnz rule of toAuto.
"""
from __future__ import annotations

from enum import Enum

import numpy as np
import torch

from .exceptions import SketchMLException
from .quantization import QuantileQuantizer
from .sparse import encode_sparse, to_sparse

EPS = 1e-8  # ml/util/Maths.scala:8


class Kind(Enum):
    DenseDouble = "DenseDouble"
    SparseDouble = "SparseDouble"
    Sketch = "Sketch"


def _jint(x: int) -> int:
    """Java int wrap-around."""
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= (1 << 31) else x


def auto_dense(nnz: int, dim: int) -> bool:
    """toAuto's rule: dense iff nnz > dim * 2 / 3 in Java int arithmetic (the product wraps for
    dim > 1,073,741,823; DenseDoubleGradient.scala:92-95)."""
    lim = _jint(dim * 2)
    lim = int(lim / 3)  # Java division truncates toward zero
    return nnz > lim


class DenseDoubleGradient:
    """ml/gradient/DenseDoubleGradient.scala."""

    def __init__(self, dim: int, values: torch.Tensor):
        self.dim = int(dim)
        self.values = values

    def _sparse(self):
        # |v| > EPS compaction on the device (k_compact; fp64 values are tested in double and kept
        # as doubles, so fromSparse bins the reference's own double values)
        return to_sparse(self.values)

    def countNNZ(self) -> int:
        return int(self._sparse()[0].numel())

    def timesBy(self, x: float) -> None:
        self.values.mul_(x)

    def toDense(self) -> "DenseDoubleGradient":
        return self

    def toSparse(self) -> "SparseDoubleGradient":
        keys, vals = self._sparse()
        return SparseDoubleGradient(self.dim, keys, vals)

    def toAuto(self):
        keys, vals = self._sparse()
        return self if auto_dense(int(keys.numel()), self.dim) else SparseDoubleGradient(self.dim, keys, vals)

    def kind(self) -> Kind:
        return Kind.DenseDouble


class SparseDoubleGradient:
    """ml/gradient/SparseDoubleGradient.scala: strictly increasing int keys and their values."""

    def __init__(self, dim: int, indices: torch.Tensor, values: torch.Tensor):
        if indices.numel() != values.numel():
            raise SketchMLException(
                f"Lengths of key array and value array do not match: {indices.numel()}, {values.numel()}")
        self.dim = int(dim)
        self.indices = indices
        self.values = values

    def _live(self) -> torch.Tensor:
        return self.values.abs() > EPS

    def countNNZ(self) -> int:
        return int(self._live().sum().item())

    def timesBy(self, x: float) -> None:
        self.values.mul_(x)

    def toDense(self) -> DenseDoubleGradient:
        dense = torch.zeros(self.dim, dtype=self.values.dtype, device=self.values.device)
        live = self._live()
        dense[self.indices[live].long()] = self.values[live]
        return DenseDoubleGradient(self.dim, dense)

    def toSparse(self) -> "SparseDoubleGradient":
        return self

    def toAuto(self):
        return self.toDense() if auto_dense(self.countNNZ(), self.dim) else self

    def kind(self) -> Kind:
        return Kind.SparseDouble


class SketchGradient:
    """ml/gradient/SketchGradient.scala:8-80.

    fromDense: QuantileQuantizer.quantize over all values, bins kept (as the device payload);
    fromSparse: quantize the values, then GroupedMinMaxSketch over (indices, bins).
    bucketValues is the host double array Quantizer.getValues() returns, scaled in place by
    timesBy exactly as the Scala loop does, so toDense / toSparse return the same doubles.
    """

    def __init__(self, grad=None, binNum: int = 256, groupNum: int = 8, rowNum: int = 2, colRatio: float = 0.3,
                 dim: int | None = None, seed: int = 0, hashSeed: int = 0):
        self.binNum, self.groupNum, self.rowNum, self.colRatio = int(binNum), int(groupNum), int(rowNum), colRatio
        self.seed, self.hashSeed = seed, hashSeed
        self.dim = int(dim if dim is not None else (grad.dim if grad is not None else 0))
        self.nnz = 0
        self.bucketValues: np.ndarray | None = None
        self.quantizer: QuantileQuantizer | None = None  # dense: the bins live in its payload
        self.sketch = None                                # sparse: the GroupedMinMaxSketch payload
        if grad is not None:
            if grad.kind() == Kind.DenseDouble:
                self.fromDense(grad)
            elif grad.kind() == Kind.SparseDouble:
                self.fromSparse(grad)
            else:
                raise SketchMLException(f"Cannot create {Kind.Sketch.value} from {grad.kind().value}")

    def fromDense(self, dense: DenseDoubleGradient) -> None:
        q = QuantileQuantizer(self.binNum, self.seed)
        q.quantize(dense.values)
        self.bucketValues = q.getValues()
        self.quantizer, self.sketch = q, None
        self.nnz = self.dim

    def fromSparse(self, sparse: SparseDoubleGradient) -> None:
        self.sketch = encode_sparse(sparse.indices, sparse.values, self.binNum, self.groupNum, self.rowNum,
                                    self.colRatio, self.seed, self.hashSeed)
        self.bucketValues = self.sketch.values()
        self.quantizer = None
        self.nnz = int(sparse.indices.numel())

    def timesBy(self, x: float) -> None:
        self.bucketValues = self.bucketValues * x  # element-wise double products, as the Scala loop

    def countNNZ(self) -> int:
        return self.nnz

    def _values_of(self, bins: torch.Tensor) -> torch.Tensor:
        lut = torch.from_numpy(np.ascontiguousarray(self.bucketValues)).to(bins.device)
        return lut[bins.long()]

    def toDense(self) -> DenseDoubleGradient:
        if self.quantizer is None:
            raise SketchMLException("toDense of a sparse SketchGradient: bins is null")
        return DenseDoubleGradient(self.dim, self._values_of(self.quantizer.getBins()))

    def toSparse(self) -> SparseDoubleGradient:
        if self.sketch is None:
            raise SketchMLException("toSparse of a dense SketchGradient: sketch is null")
        keys, bins = self.sketch.restore_bins()
        return SparseDoubleGradient(self.dim, keys, self._values_of(bins))

    def toAuto(self):
        return (self.toDense() if self.quantizer is not None else self.toSparse()).toAuto()

    def kind(self) -> Kind:
        return Kind.Sketch
