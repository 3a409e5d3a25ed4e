"""ctypes binding of libkxcodec.so (the product C-ABI, include/kxcodec.h).

Fails loudly: there is no CPU fallback anywhere in the product path. If the shared library is
missing or was built for another ABI version, import of the codec raises.
"""
from __future__ import annotations

import ctypes as C
import os

from . import _abi as A

HERE = os.path.dirname(os.path.abspath(__file__))
# KXCODEC_LIB: an alternative in-tree build of the same library (kernel-tuning experiments)
LIB_PATH = os.environ.get("KXCODEC_LIB") or os.path.join(HERE, "lib", "libkxcodec.so")

_lib = None

EXPORTS = [
    "kx_abi_version", "kx_strerror", "kx_schema_create", "kx_schema_destroy", "kx_schema_num_columns",
    "kx_schema_column_info", "kx_schema_presence_bits", "kx_schema_min_record_size", "kx_ctx_create",
    "kx_ctx_destroy", "kx_thrift_decode_batch", "kx_thrift_skip_batch", "kx_thrift_split_points", "kx_thrift_encoded_size_batch",
    "kx_thrift_encode_batch", "kx_pb_decode_batch", "kx_pb_encoded_size_batch",
    "kx_pb_encode_batch", "kx_host_decode_batch", "kx_host_pb_decode_batch",
    "kx_thrift_message_begin_length", "kx_thrift_write_message_begin", "kx_thrift_read_message_begin",
    "kx_thrift_decode_messages", "kx_pb_decode_messages", "kx_pb_meta_length", "kx_pb_write_meta",
    "kx_pb_read_meta", "kx_ctx_set_pipeline", "kx_frame_scan", "kx_thrift_decode_frames",
    "kx_pb_decode_frames", "kx_crc32c_batch", "kx_frame_crc32c_validate", "kx_ctx_set_crc32c_check",
    "kx_grpc_frame_scan", "kx_thrift_decode_grpc", "kx_pb_decode_grpc", "kx_thrift_raw_messages",
    "kx_thrift_set_seqids", "kx_thrift_encode_messages", "kx_ttstream_default_keys", "kx_ttstream_frame_scan",
    "kx_thrift_decode_extents", "kx_pb_decode_extents", "kx_schema_is_nested", "kx_thrift_decode_sizes",
    "kx_decode_workspace_bytes", "kx_thrift_decode_sizes_extents", "kx_shard_meta_words", "kx_shard_meta",
    "kx_concat_plan", "kx_concat_rebase", "kx_host_encode_batch", "kx_host_pb_encode_batch",
]


class KxError(RuntimeError):
    def __init__(self, code: int, what: str = "", record: int = None, offset: int = None):
        self.code = code
        self.record = record
        self.offset = offset
        msg = f"{what}: {A.ERROR_NAMES.get(code, code)} (code {code})"
        if record is not None:
            msg += f" at record {record} (offset {offset})"
        super().__init__(msg)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libkxcodec.so not built ({LIB_PATH}); run `python -m kitex_amd.build` "
                          "or __graft_entry__.build()")
    try:  # share torch's HIP runtime (same soname) when torch is around
        import torch  # noqa: F401
    except Exception:
        pass
    L = C.CDLL(LIB_PATH)
    vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int32
    L.kx_abi_version.restype = C.c_int
    L.kx_strerror.argtypes = [C.c_int]
    L.kx_strerror.restype = C.c_char_p
    L.kx_schema_create.argtypes = [C.POINTER(A.StructDesc), u32, C.POINTER(vp)]
    L.kx_schema_destroy.argtypes = [vp]
    L.kx_schema_destroy.restype = None
    L.kx_schema_num_columns.argtypes = [vp]
    L.kx_schema_num_columns.restype = u32
    L.kx_schema_column_info.argtypes = [vp, u32, C.POINTER(A.ColumnInfo)]
    L.kx_schema_presence_bits.argtypes = [vp]
    L.kx_schema_presence_bits.restype = u32
    L.kx_schema_min_record_size.argtypes = [vp]
    L.kx_schema_min_record_size.restype = u64
    L.kx_ctx_create.argtypes = [C.c_int, C.POINTER(vp)]
    L.kx_ctx_destroy.argtypes = [vp]
    L.kx_ctx_destroy.restype = None
    L.kx_ctx_set_pipeline.argtypes = [vp, u64, C.c_int]
    dec = [vp, vp, vp, u64, vp, u64, C.POINTER(A.Columns), vp, vp, vp]
    L.kx_thrift_decode_batch.argtypes = dec
    L.kx_schema_is_nested.argtypes = [vp]
    L.kx_schema_is_nested.restype = C.c_int
    L.kx_thrift_decode_sizes.argtypes = [vp, vp, vp, u64, vp, u64, vp, C.POINTER(A.Status), vp]
    L.kx_thrift_decode_sizes_extents.argtypes = [vp, vp, vp, u64, vp, vp, u64, vp, C.POINTER(A.Status), vp]
    L.kx_pb_decode_batch.argtypes = dec
    L.kx_decode_workspace_bytes.argtypes = [vp, u64, C.c_int, u64]
    L.kx_decode_workspace_bytes.restype = u64
    L.kx_thrift_skip_batch.argtypes = [vp, vp, u64, u64, vp, vp, vp]
    L.kx_thrift_split_points.argtypes = [vp, vp, vp, u64, u64, C.c_uint32, vp, vp, vp]
    L.kx_thrift_encoded_size_batch.argtypes = [vp, vp, C.POINTER(A.Columns), u64, vp, vp]
    L.kx_thrift_encode_batch.argtypes = [vp, vp, C.POINTER(A.Columns), u64, vp, u64, vp, vp, vp]
    L.kx_pb_encoded_size_batch.argtypes = L.kx_thrift_encoded_size_batch.argtypes
    L.kx_pb_encode_batch.argtypes = L.kx_thrift_encode_batch.argtypes
    L.kx_host_decode_batch.argtypes = [vp, vp, vp, u64, vp, u64, C.POINTER(A.Columns), vp, C.POINTER(A.Status)]
    L.kx_host_pb_decode_batch.argtypes = L.kx_host_decode_batch.argtypes
    L.kx_host_encode_batch.argtypes = [vp, vp, C.POINTER(A.Columns), u64, vp, u64, vp, vp, C.POINTER(A.Status)]
    L.kx_host_pb_encode_batch.argtypes = L.kx_host_encode_batch.argtypes
    L.kx_thrift_message_begin_length.argtypes = [u32]
    L.kx_thrift_message_begin_length.restype = u64
    L.kx_thrift_write_message_begin.argtypes = [vp, u64, C.c_char_p, u32, i32, i32, C.POINTER(u64)]
    L.kx_thrift_read_message_begin.argtypes = [vp, u64, C.POINTER(C.c_char_p), C.POINTER(u32),
                                               C.POINTER(i32), C.POINTER(i32), C.POINTER(u64)]
    L.kx_thrift_decode_messages.argtypes = [vp, vp, vp, u64, vp, u64, i32, C.POINTER(A.Column),
                                            C.POINTER(A.Columns), vp, vp, vp]
    L.kx_pb_decode_messages.argtypes = [vp, vp, vp, u64, vp, u64, C.POINTER(A.Column), C.POINTER(A.Columns),
                                        vp, vp, vp]
    L.kx_frame_scan.argtypes = [vp, vp, u64, u64, u64, vp, vp, vp, vp, vp, vp]
    L.kx_thrift_decode_frames.argtypes = [vp, vp, vp, u64, u64, i32, u64, vp, vp, C.POINTER(A.Column),
                                          C.POINTER(A.Columns), vp, vp, vp]
    L.kx_pb_decode_frames.argtypes = [vp, vp, vp, u64, u64, u64, vp, vp, C.POINTER(A.Column),
                                      C.POINTER(A.Columns), vp, vp, vp]
    L.kx_crc32c_batch.argtypes = [vp, vp, u64, vp, u64, vp, vp, vp]
    L.kx_frame_crc32c_validate.argtypes = [vp, vp, u64, vp, u64, vp, vp, vp, vp]
    L.kx_ctx_set_crc32c_check.argtypes = [vp, C.c_int]
    L.kx_ttstream_default_keys.argtypes = [C.POINTER(A.TTStreamKeys)]
    L.kx_ttstream_default_keys.restype = None
    L.kx_ttstream_frame_scan.argtypes = [vp, vp, u64, u64, C.POINTER(A.TTStreamKeys), vp, vp, vp, vp, vp, vp, vp,
                                         vp, vp]
    L.kx_thrift_decode_extents.argtypes = [vp, vp, vp, u64, vp, vp, u64, C.POINTER(A.Columns), vp, vp, vp]
    L.kx_pb_decode_extents.argtypes = L.kx_thrift_decode_extents.argtypes
    L.kx_grpc_frame_scan.argtypes = L.kx_frame_scan.argtypes
    L.kx_thrift_raw_messages.argtypes = [vp, vp, u64, vp, u64, C.POINTER(A.Column), vp, vp, vp]
    L.kx_thrift_set_seqids.argtypes = [vp, vp, u64, vp, u64, vp, vp, vp, vp]
    L.kx_thrift_encode_messages.argtypes = [vp, vp, C.POINTER(A.Columns), u64, C.c_char_p, u32, i32, vp, i32, vp,
                                            u64, vp, u64, vp, vp, vp]
    L.kx_thrift_decode_grpc.argtypes = [vp, vp, vp, u64, u64, u64, vp, C.POINTER(A.Columns), vp, vp, vp]
    L.kx_pb_decode_grpc.argtypes = L.kx_thrift_decode_grpc.argtypes
    ci = C.POINTER(A.ColumnInfo)
    L.kx_shard_meta_words.argtypes = [ci, u32]
    L.kx_shard_meta_words.restype = u32
    L.kx_shard_meta.argtypes = [vp, ci, u32, C.POINTER(A.Columns), u64, u64, vp, vp]
    L.kx_concat_plan.argtypes = [ci, u32, C.POINTER(A.Columns), C.POINTER(u64), u32, C.POINTER(A.ConcatPiece),
                                 C.POINTER(u32), C.POINTER(A.ConcatSizes)]
    L.kx_concat_rebase.argtypes = [vp, ci, u32, C.POINTER(A.ConcatPiece), u32, C.POINTER(A.Columns),
                                   C.POINTER(A.Columns), C.POINTER(A.ConcatSizes), vp]
    L.kx_pb_meta_length.argtypes = [u32]
    L.kx_pb_meta_length.restype = u64
    L.kx_pb_write_meta.argtypes = L.kx_thrift_write_message_begin.argtypes
    L.kx_pb_read_meta.argtypes = L.kx_thrift_read_message_begin.argtypes
    if L.kx_abi_version() != A.KX_ABI_VERSION:
        raise ImportError(f"libkxcodec ABI {L.kx_abi_version()} != {A.KX_ABI_VERSION}")
    _lib = L
    return L


def check(rc: int, what: str):
    if rc != 0:
        raise KxError(rc, what)
