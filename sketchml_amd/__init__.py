"""sketchml_amd -- MI355X-native SketchML gradient codec.

The hot path (k=128 quantile sketch, bucket quantisation, packed codes, sparse key/value
codec) runs in hand-written gfx950 HIP kernels in lib/libskml.so behind the C ABI of
include/skml.h; this package mirrors the reference's Java surface over that ABI.
"""
from . import _lib
from .compressor import DenseVectorCompressor
from .constants import Constants, Parallel
from .context import Context, alloc_aligned, get_context
from .exceptions import QuantileSketchException, SketchMLException
from .gradient import DenseDoubleGradient, Kind, SketchGradient, SparseDoubleGradient
from .quantization import QuantileQuantizer, QuantizationType, Quantizer, UniformQuantizer
from .sparse import (DeltaAdaptiveEncoder, GroupedMinMaxSketch, SparsePayload, SparseVectorCompressor, decode_sum,
                     encode_dense_as_sparse, encode_sparse, to_sparse)

__all__ = ["Constants", "Parallel", "DenseDoubleGradient", "Kind", "SketchGradient", "SparseDoubleGradient", "Context", "DeltaAdaptiveEncoder", "DenseVectorCompressor", "GroupedMinMaxSketch", "SparsePayload",
           "SparseVectorCompressor", "decode_sum", "encode_dense_as_sparse", "encode_sparse", "to_sparse", "QuantileQuantizer", "QuantizationType", "Quantizer", "UniformQuantizer",
           "QuantileSketchException", "SketchMLException", "get_context", "alloc_aligned"]

LIB_PATH = _lib.LIB_PATH
