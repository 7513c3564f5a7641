"""ctypes binding of libskml.so (the C ABI in include/skml.h).

There is no CPU fallback: if the HIP library is missing or cannot be loaded, importing the
package fails loudly.  The library is built in-tree by __graft_entry__.build()
(sketchml_amd/csrc/Makefile -> sketchml_amd/lib/libskml.so).
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os

# torch first: its bundled HIP runtime must be the one in the process before libskml.so (which
# links libamdhip64) is loaded, or the two runtimes disagree about the devices.
import torch  # noqa: F401

_HERE = os.path.dirname(os.path.abspath(__file__))
# SKML_LIB selects another in-tree build of the same library (e.g. the profiling build in
# lib_prof/); there is no non-native fallback.
LIB_PATH = os.environ.get("SKML_LIB", os.path.join(_HERE, "lib", "libskml.so"))

SKML_OK = 0
SKML_E_ARG = 1
SKML_E_NAN = 2
SKML_E_ORDER = 3
SKML_E_HIP = 4
SKML_E_RCCL = 5
SKML_E_OOM = 6
SKML_E_STATE = 7
UNIQUE_ID_BYTES = 128
SKML_MAX_BINS = 65536
SKML_QUANTILE = 0
SKML_UNIFORM = 1

vp = C.c_void_p
i32 = C.c_int32
i64 = C.c_int64
i64p = C.POINTER(C.c_int64)
i32p = C.POINTER(C.c_int32)
u8p = C.POINTER(C.c_uint8)
dblp = C.POINTER(C.c_double)
szp = C.POINTER(C.c_size_t)


class Params(C.Structure):
    _fields_ = [("bin_num", C.c_int32), ("group_num", C.c_int32), ("row_num", C.c_int32),
                ("dedup", C.c_int32), ("col_ratio", C.c_double), ("seed", C.c_int64),
                ("hash_seed", C.c_int64), ("quant_type", C.c_int32), ("parallelism", C.c_int32)]


class SparseBlobHeader(C.Structure):
    """The 256-byte header of an exported sparse payload (SpBlobHeader, csrc/skml_sparse.h)."""
    _fields_ = [("magic", C.c_uint32), ("version", C.c_int32), ("total_bytes", C.c_int64), ("nnz", C.c_int64),
                ("ncells", C.c_int64), ("n_flag_words", C.c_int64), ("n_delta_words", C.c_int64),
                ("flag_bits", C.c_int64), ("delta_bits", C.c_int64), ("nvalues", C.c_int32),
                ("quant_bytes", C.c_int32), ("off_groups", C.c_int64), ("off_quant", C.c_int64),
                ("off_values", C.c_int64), ("off_tables", C.c_int64), ("off_flags", C.c_int64),
                ("off_deltas", C.c_int64), ("params", Params), ("table_width", C.c_int32), ("pad0", C.c_int32),
                ("reserved", C.c_int64 * 7)]


class DenseHeader(C.Structure):
    _fields_ = [("magic", C.c_uint32), ("status", C.c_int32), ("n", C.c_int64),
                ("bin_num", C.c_int32), ("zero_idx", C.c_int32), ("code_bits", C.c_int32),
                ("req_bins", C.c_int32), ("min", C.c_double), ("max", C.c_double),
                ("codes_offset", C.c_int64), ("reserved", C.c_int64)]


class SparseGroup(C.Structure):
    _fields_ = [("size", C.c_int32), ("col_num", C.c_int32), ("hash_ids", C.c_int32 * 8),
                ("num_intervals", C.c_int32), ("flag_kind", C.c_int32),
                ("n_flag_bits", C.c_int64), ("n_delta_bits", C.c_int64)]


# name -> (restype, argtypes)
_SIGS = {
    "skml_params_default": (None, [C.POINTER(Params)]),
    "skml_last_error": (C.c_char_p, []),
    "skml_version": (C.c_char_p, []),
    "skml_ctx_create": (C.c_int, [C.c_int, vp, C.POINTER(vp)]),
    "skml_ctx_destroy": (C.c_int, [vp]),
    "skml_ctx_sync": (C.c_int, [vp]),
    "skml_ctx_set_stream": (C.c_int, [vp, vp]),
    "skml_ctx_set_timing": (C.c_int, [vp, C.c_int]),
    "skml_ctx_kernel_stats": (C.c_int, [vp, C.c_int, i64p, C.POINTER(C.c_double)]),
    "skml_ctx_reset_stats": (C.c_int, [vp]),
    "skml_debug_leaf_stage": (C.c_int, [vp, vp, i64, C.c_int, C.c_int, C.POINTER(C.c_double)]),
    "skml_debug_sparse_scratch_fail": (C.c_int, [C.c_int]),
    "skml_debug_sparse_merge_path": (C.c_int, []),
    "skml_debug_form": (C.c_int, [C.c_int, C.c_int]),
    "skml_build_flags": (C.c_int, []),
    "skml_dense_payload_bytes": (C.c_size_t, [i64, i32]),
    "skml_dense_encode_f32": (C.c_int, [vp, vp, i64, C.POINTER(Params), vp, C.c_size_t]),
    "skml_dense_encode_with_splits_f32": (C.c_int, [vp, vp, i64, dblp, i32, C.c_double, C.c_double,
                                                    vp, C.c_size_t]),
    "skml_dense_encode_f64": (C.c_int, [vp, vp, i64, C.POINTER(Params), vp, C.c_size_t]),
    "skml_dense_encode_uniform_f32": (C.c_int, [vp, vp, i64, C.POINTER(Params), vp, C.c_size_t]),
    "skml_dense_encode_parallel_f32": (C.c_int, [vp, vp, i64, i32, C.POINTER(Params), vp, C.c_size_t]),
    "skml_dense_encode_batch_f32": (C.c_int, [vp, i32, C.POINTER(vp), i64p, C.POINTER(Params), C.POINTER(vp),
                                              C.POINTER(C.c_size_t)]),
    "skml_sketch_record_bytes": (C.c_size_t, [i32]),
    "skml_dense_encode_parallel_f64": (C.c_int, [vp, vp, i64, i32, C.POINTER(Params), vp, C.c_size_t]),
    "skml_dense_sketch_shard_f64": (C.c_int, [vp, vp, i64, i64p, i32, i32, i64, vp]),
    "skml_dense_encode_sharded_f64": (C.c_int, [vp, vp, i64, i64p, i32, i32, vp, C.POINTER(Params), vp,
                                                C.c_size_t]),
    "skml_dense_sketch_shard_f32": (C.c_int, [vp, vp, i64, i64p, i32, i32, i64, vp]),
    "skml_dense_encode_sharded_f32": (C.c_int, [vp, vp, i64, i64p, i32, i32, vp, C.POINTER(Params), vp,
                                                C.c_size_t]),
    "skml_dense_encode_uniform_f64": (C.c_int, [vp, vp, i64, C.POINTER(Params), vp, C.c_size_t]),
    "skml_dense_decode_f32": (C.c_int, [vp, vp, vp, i64]),
    "skml_dense_decode_f64": (C.c_int, [vp, vp, vp, i64]),
    "skml_dense_decode_sum_f32": (C.c_int, [vp, vp, i32, C.c_size_t, vp, i64, C.c_double]),
    "skml_dense_bins_i32": (C.c_int, [vp, vp, vp, i64]),
    "skml_dense_info": (C.c_int, [vp, vp, C.POINTER(DenseHeader), dblp, i32]),
    "skml_dense_times_by": (C.c_int, [vp, vp, C.c_double]),
    "skml_dense_serialize_ref": (C.c_int, [vp, vp, u8p, C.c_size_t, szp]),
    "skml_dense_deserialize_ref": (C.c_int, [vp, u8p, C.c_size_t, vp, C.c_size_t]),
    "skml_host_alloc": (C.c_int, [C.c_size_t, C.POINTER(vp)]),
    "skml_host_free": (C.c_int, [vp]),
    "skml_dense_encode_host_f32": (C.c_int, [vp, vp, i64, C.POINTER(Params), vp, C.c_size_t, szp]),
    "skml_dense_decode_host_f32": (C.c_int, [vp, vp, C.c_size_t, vp, i64]),
    "skml_dense_encode_host_f64": (C.c_int, [vp, vp, i64, C.POINTER(Params), vp, C.c_size_t, szp]),
    "skml_dense_decode_host_f64": (C.c_int, [vp, vp, C.c_size_t, vp, i64]),
    "skml_dense_info_host": (C.c_int, [vp, C.c_size_t, C.POINTER(DenseHeader), dblp, i32]),
    "skml_dense_bins_host": (C.c_int, [vp, C.c_size_t, vp, i64]),
    "skml_dense_times_by_host": (C.c_int, [vp, C.c_size_t, C.c_double]),
    "skml_sparse_encode_kv_host_f32": (C.c_int, [vp, vp, vp, i64, C.POINTER(Params), C.POINTER(vp)]),
    "skml_sparse_encode_kv_host_f64": (C.c_int, [vp, vp, vp, i64, C.POINTER(Params), C.POINTER(vp)]),
    "skml_sparse_decode_host_f32": (C.c_int, [vp, vp, vp, vp]),
    "skml_sparse_decode_host_f64": (C.c_int, [vp, vp, vp, vp]),
    "skml_delta_encode_host": (C.c_int, [vp, vp, i64, i32p, i32p, i64p, i64p, vp, vp, i64]),
    "skml_delta_decode_host": (C.c_int, [vp, i64, i32, i32, vp, i64, vp, i64, vp]),
    "skml_sparse_compact_f32": (C.c_int, [vp, vp, i64, vp, vp, i64p]),
    "skml_sparse_compact_f64": (C.c_int, [vp, vp, i64, vp, vp, i64p]),
    "skml_sparse_encode_kv_f32": (C.c_int, [vp, vp, vp, i64, C.POINTER(Params), C.POINTER(vp)]),
    "skml_sparse_encode_kv_f64": (C.c_int, [vp, vp, vp, i64, C.POINTER(Params), C.POINTER(vp)]),
    "skml_sparse_encode_f32": (C.c_int, [vp, vp, i64, C.POINTER(Params), C.POINTER(vp)]),
    "skml_sparse_encode_f64": (C.c_int, [vp, vp, i64, C.POINTER(Params), C.POINTER(vp)]),
    "skml_sparse_decode_f32": (C.c_int, [vp, vp, vp, vp]),
    "skml_sparse_decode_f64": (C.c_int, [vp, vp, vp, vp]),
    "skml_sparse_nnz": (C.c_int, [vp, i64p]),
    "skml_sparse_times_by": (C.c_int, [vp, C.c_double]),
    "skml_sparse_values": (C.c_int, [vp, dblp, i32]),
    "skml_sparse_quant_info": (C.c_int, [vp, C.POINTER(DenseHeader), dblp, i32]),
    "skml_sparse_group_info": (C.c_int, [vp, vp, i32, C.POINTER(SparseGroup), i32p,
                                         C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "skml_sparse_serialize": (C.c_int, [vp, vp, u8p, C.c_size_t, szp]),
    "skml_sparse_deserialize": (C.c_int, [vp, u8p, C.c_size_t, dblp, i32, C.POINTER(vp)]),
    "skml_sparse_restore_bins": (C.c_int, [vp, vp, vp, vp]),
    "skml_sparse_free": (C.c_int, [vp]),
    "skml_sparse_export_bytes": (C.c_int, [vp, szp]),
    "skml_sparse_export": (C.c_int, [vp, vp, vp, C.c_size_t]),
    "skml_sparse_import": (C.c_int, [vp, vp, C.c_size_t, C.POINTER(vp)]),
    "skml_sparse_decode_sum_f64": (C.c_int, [vp, vp, i32, C.c_size_t, i64, C.c_double, vp]),
    "skml_delta_encode": (C.c_int, [vp, vp, i64, i32p, i32p, i64p, i64p, vp, vp, i64]),
    "skml_delta_decode": (C.c_int, [vp, i64, i32, i32, vp, i64, vp, i64, vp]),
    "skml_comm_unique_id": (C.c_int, [u8p]),
    "skml_comm_init_rank": (C.c_int, [vp, u8p, i32, i32, C.POINTER(vp)]),
    "skml_comm_destroy": (C.c_int, [vp]),
    "skml_allgather": (C.c_int, [vp, vp, vp, C.c_size_t, vp]),
}

EXPORTED = tuple(_SIGS)


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"sketchml_amd: HIP library not built ({LIB_PATH}); run "
                          f"`python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)  # AttributeError here == ABI drift vs include/skml.h
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()

# skml_debug_form ids (include/skml.h SKML_FORM_*): alternative kernel forms the tests force to run
# each one against the oracle; every form gives the same results, 0 is the library's own choice.
FORMS = {"leaf_split": 0, "decode_sum": 1, "part_ballot": 2, "rs_rounds": 3, "dec_rows_serial": 4,
         "agg_tiles": 5, "agg_one_lane": 6, "run_bounds": 7, "dec_lookback": 8}


# SKML_BUILD_AB: the loaded library is the A/B build (sketchml_amd/lib_ab, `make -C
# sketchml_amd/csrc ab`), which also carries the forms measured slower than the default
AB_BUILD = bool(lib.skml_build_flags() & 1)


class FormNotBuilt(RuntimeError):
    """A kernel form only the A/B build carries (skml_debug_form returned -2)."""


@contextlib.contextmanager
def forced_forms(**values):
    """with forced_forms(rs_rounds=1, ...): the named forms forced for the duration.  Raises
    FormNotBuilt (forcing nothing) for a form this build does not carry."""
    prev = {}
    try:
        for k, v in values.items():
            r = lib.skml_debug_form(FORMS[k], int(v))
            if r == -2:
                raise FormNotBuilt(f"form {k}={v} is built only with -DSKML_AB (SKML_LIB=sketchml_amd/lib_ab/libskml.so)")
            if r < 0:
                raise ValueError(f"unknown form {k}")
            prev[k] = r
        yield
    finally:
        for k, v in prev.items():
            lib.skml_debug_form(FORMS[k], v)


def last_error() -> str:
    return (lib.skml_last_error() or b"").decode("utf-8", "replace")
