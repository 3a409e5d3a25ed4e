"""kitex_amd — MI355X-native batch payload codec for Kitex (Thrift binary + Kitex-Protobuf).

The product is libkxcodec.so (kitex_amd/lib), a C-ABI over hand-written HIP kernels for gfx950;
this package is the host-side mirror of Kitex's payload-codec interface over that C-ABI.
"""
from . import _abi  # noqa: F401
from .schema import Field, Schema, Struct  # noqa: F401

__all__ = ["Field", "Schema", "Struct"]
