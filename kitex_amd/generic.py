"""Generic (IDL-free or IDL-at-runtime) ingress of the batch codec.

* BinaryThriftCodec mirrors binaryThriftCodec (pkg/generic/binarythrift_codec.go:41-199), the codec of
  Kitex's binary generic call: requests stay raw Thrift message bytes. Unmarshal over a batch reads only
  the method name / type / seqid of each message on the device (readBinaryMethod :185-199) and hands the
  messages on zero-copy; SetSeqID rewrites every message's seqid in place (:117-175).
* schema_from_idl compiles a request struct from a Thrift IDL (kitex_amd.idl, the descriptor model of
  pkg/generic/descriptor/descriptor.go) into a ThriftCodec, for raw bytes -> columns once the method is
  known (pkg/generic/thrift/raw.go:79-92 is the RawReader the reference uses instead).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

from . import _abi as A
from ._lib import KxError, check, lib
from .codec import ProtocolError, ThriftCodec, _ctx_for, _ptr, _stream, read_status, status_tensor


@dataclass
class RawBatch:
    """n raw messages: requests = buf[offsets[i]:offsets[i+1]] (not copied)"""
    buf: object
    offsets: object
    names: tuple            # (int64 offsets[n+1], uint8 arena)
    msg_type: object        # int32[n]
    seqid: object           # int32[n]
    record_status: object   # uint8[n]
    status: object

    def name(self, i: int) -> str:
        offs, arena = self.names
        a, b = int(offs[i]), int(offs[i + 1])
        return bytes(arena[a:b].cpu().numpy()).decode()

    def request(self, i: int):
        return self.buf[int(self.offsets[i]):int(self.offsets[i + 1])]


class BinaryThriftCodec:
    """Batch mirror of binaryThriftCodec (RawThriftBinary)."""

    def __init__(self, device: int = 0):
        self.device = device

    def Name(self) -> str:
        return "RawThriftBinary"

    def Unmarshal(self, buf, n: int, offsets, name_cap: int = None, stream=None,
                  raise_on_error: bool = True) -> RawBatch:
        import torch
        s = _stream(stream)
        name_cap = max(1, buf.numel() if name_cap is None else name_cap)
        names = (torch.zeros(n + 1, dtype=torch.int64, device=buf.device),
                 torch.empty(name_cap, dtype=torch.uint8, device=buf.device))
        mtype = torch.zeros(max(1, n), dtype=torch.int32, device=buf.device)
        seqid = torch.zeros(max(1, n), dtype=torch.int32, device=buf.device)
        mc = (A.Column * 3)()
        mc[0].data, mc[0].offsets, mc[0].capacity, mc[0].offset_bytes = names[1].data_ptr(), names[0].data_ptr(), \
            name_cap, 8
        mc[1].data = mtype.data_ptr()
        mc[2].data = seqid.data_ptr()
        rs = torch.zeros(max(1, n), dtype=torch.uint8, device=buf.device)
        st = status_tensor(buf.device)
        check(lib().kx_thrift_raw_messages(_ctx_for(self.device, s).handle, _ptr(buf), buf.numel(), _ptr(offsets), n,
                                           mc, _ptr(rs), _ptr(st), int(s.cuda_stream)), "kx_thrift_raw_messages")
        res = RawBatch(buf, offsets, names, mtype[:n], seqid[:n], rs[:n], st)
        if raise_on_error:
            stt = read_status(st, s)
            if stt.code:
                raise ProtocolError(stt.code, "binaryThriftCodec Unmarshal", stt.record, stt.offset)
        return res

    def SetSeqID(self, buf, offsets, seqids, stream=None, raise_on_error: bool = True):
        """SetSeqID of every message in place; returns the per-message codes"""
        import torch
        s = _stream(stream)
        n = offsets.numel() - 1
        rs = torch.zeros(max(1, n), dtype=torch.uint8, device=buf.device)
        st = status_tensor(buf.device)
        check(lib().kx_thrift_set_seqids(_ctx_for(self.device, s).handle, _ptr(buf), buf.numel(), _ptr(offsets), n,
                                         _ptr(seqids), _ptr(rs), _ptr(st), int(s.cuda_stream)), "kx_thrift_set_seqids")
        stt = read_status(st, s)
        if raise_on_error and stt.code:
            raise KxError(stt.code, "SetSeqID", stt.record, stt.offset)
        return rs[:n]

    name, unmarshal = Name, Unmarshal


def schema_from_idl(path_or_text: str, method: str, service: str = None, include_dirs=()):
    """The codec schema of `method`'s request record (Args field 1) compiled from an IDL."""
    from .idl import parse_idl, request_schema
    return request_schema(parse_idl(path_or_text, include_dirs), method, service)


def codec_from_idl(path_or_text: str, method: str, service: str = None, device: int = 0) -> ThriftCodec:
    return ThriftCodec(schema_from_idl(path_or_text, method, service), device=device)
