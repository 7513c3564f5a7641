"""VectorCompressor implementations (base/VectorCompressor.java:9-27) over the HIP codec."""
from __future__ import annotations

import torch

from .context import as_device_values
from .exceptions import SketchMLException
from .quantization import Quantizer, QuantizationType


class DenseVectorCompressor:
    """sample/DenseVectorCompressor.java:18-117."""

    def __init__(self, quantType=QuantizationType.QUANTILE, quantBinNum: int = Quantizer.DEFAULT_BIN_NUM,
                 seed: int = 0):
        self.quantType = quantType
        self.quantBinNum = int(quantBinNum)
        self.seed = seed
        self._size = 0
        self.quantizer = None

    def compressDense(self, values) -> None:
        x = as_device_values(values)
        self._size = x.numel()
        self.quantizer = Quantizer.newQuantizer(self.quantType, self.quantBinNum, self.seed)
        self.quantizer.quantize(x)

    def parallelCompressDense(self, values) -> None:
        x = as_device_values(values)
        self._size = x.numel()
        self.quantizer = Quantizer.newQuantizer(self.quantType, self.quantBinNum, self.seed)
        self.quantizer.parallelQuantize(x)

    def _sparse_to_dense(self, keys, values):
        keys = torch.as_tensor(keys)
        values = torch.as_tensor(values)
        if keys.numel() != values.numel():
            raise SketchMLException(
                f"Lengths of key array and value array do not match: {keys.numel()}, {values.numel()}")
        # DenseVectorCompressor.java:51-54 sizes the array maxKey (not maxKey + 1), so the
        # reference throws ArrayIndexOutOfBoundsException for any non-empty input; mirrored.
        max_key = int(keys.max().item())
        raise IndexError(f"Index {max_key} out of bounds for length {max_key}")

    def compressSparse(self, keys, values) -> None:
        self._sparse_to_dense(keys, values)

    def parallelCompressSparse(self, keys, values) -> None:
        self._sparse_to_dense(keys, values)

    def decompressDense(self) -> torch.Tensor:
        return self.quantizer.decode()

    def decompressSparse(self):
        vals = self.decompressDense()
        keys = torch.arange(vals.numel(), dtype=torch.int32, device=vals.device)
        return keys, vals

    def timesBy(self, x: float) -> None:
        self.quantizer.timesBy(x)

    def size(self) -> float:
        return float(self._size)

    def memoryBytes(self) -> int:
        """12 + serialised quantizer (DenseVectorCompressor.java:112-116; the quantizer's field
        stream without Java object-stream framing)."""
        res = 12
        if self.quantizer is not None:
            res += len(self.quantizer.writeObject())
        return res
