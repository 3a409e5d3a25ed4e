"""Host-side mirror of Kitex's payload-codec interface over the MI355X C-ABI.

Kitex (Go) plugs payload codecs in through `remote.PayloadCodec{Marshal, Unmarshal, Name}`
(pkg/remote/payload_codec.go:29-33) and configures the Thrift one with `CodecType` bit flags
(pkg/remote/codec/thrift/thrift.go:36-53). The classes below keep those names and meanings for a
*batch* of same-schema records held in HBM:

  ThriftCodec.Unmarshal(buf, n, offsets)  ~ n x FastRead       (codec_fast.go:60-82)
  ThriftCodec.Marshal(columns)            ~ n x FastWriteNocopy (codec_fast.go:40-58, 85-91)
  ThriftCodec.BLength(columns)            ~ n x BLength
  ThriftCodec.Skip(buf, n)                ~ skipThriftStruct    (codec_apache.go:39-68,166)

Errors surface as `ProtocolError` carrying the thrift TProtocolException type id, the way
fastUnmarshal wraps them in remote.NewTransError(remote.ProtocolError, err).

Every call goes through libkxcodec.so; there is no CPU path. Device buffers are torch tensors
(torch is only the HBM allocator and stream provider here).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from enum import IntFlag
from typing import List, Optional, Sequence

from . import _abi as A
from ._lib import KxError, check, lib
from .columns import alloc_device, alloc_host, to_kx_columns
from .schema import Schema
from .synth import ColumnSet


class CodecType(IntFlag):
    """thrift.go:36-53"""
    Basic = 0b0000
    FastWrite = 0b0001
    FastRead = 0b0010
    FastReadWrite = 0b0011
    FrugalWrite = 0b0100
    FrugalRead = 0b1000
    FrugalReadWrite = 0b1100
    EnableSkipDecoder = 0b10000


@dataclass(frozen=True)
class TypeCodec:
    """typeCodec (pkg/remote/codec/thrift/codec.go:26-47): the codecs a record type implements. Every type
    compiled into a kx schema has the generated FastCodec trio (kx_thrift_* are its batch form)."""
    FastCodec: bool = True
    Frugal: bool = False
    Apache: bool = False


def is_data_len_deterministic(codec_type: "CodecType", data_len: int) -> bool:
    """IsDataLenDeterministic (thrift.go:102-105)"""
    return data_len > 0 or bool(codec_type & CodecType.EnableSkipDecoder)


def select_unmarshal(codec_type: "CodecType", data_len: int, tc: TypeCodec = TypeCodec()) -> str:
    """unmarshalThriftData (thrift_data.go:106-127): "frugal" | "fast" | "apache". A "fast" read with
    data_len 0 is fastUnmarshal's skip-then-read (codec_fast.go:72-81): the concatenated batch decode."""
    ok = is_data_len_deterministic(codec_type, data_len)
    if ok and codec_type & CodecType.FrugalRead and tc.Frugal:
        return "frugal"
    if ok and codec_type & CodecType.FastRead and tc.FastCodec:
        return "fast"
    if tc.Apache:
        return "apache"
    if tc.FastCodec:  # fallback even though CodecType=Basic or EnableSkipDecoder not set
        return "fast"
    if tc.Frugal:
        return "frugal"
    raise KxError(A.ERR_INVALID_DATA, "decode failed, msg type not match with thriftCodec")  # errDecodeMismatchMsgType


def select_marshal(codec_type: "CodecType", tc: TypeCodec = TypeCodec()) -> str:
    """marshalThriftData (thrift_data.go:56-78)"""
    if codec_type & CodecType.FrugalWrite and tc.Frugal:
        return "frugal"
    if codec_type & CodecType.FastWrite and tc.FastCodec:
        return "fast"
    if tc.Apache:
        return "apache"
    if tc.FastCodec:
        return "fast"
    if tc.Frugal:
        return "frugal"
    raise KxError(A.ERR_INVALID_DATA, "encode failed, msg type not match with thriftCodec")


class ProtocolError(KxError):
    """remote.NewTransError(remote.ProtocolError, err) equivalent (trans_errors.go:35)."""


class DeviceSchema:
    """A Schema compiled by libkxcodec (kx_schema_create)."""

    def __init__(self, schema: Schema):
        L = lib()
        self.schema = schema
        tab, ns = schema.struct_table()
        h = C.c_void_p()
        check(L.kx_schema_create(tab, ns, C.byref(h)), "kx_schema_create")
        self.handle = h
        self.ncols = L.kx_schema_num_columns(h)
        self.infos: List[A.ColumnInfo] = []
        for c in range(self.ncols):
            ci = A.ColumnInfo()
            check(L.kx_schema_column_info(h, c, C.byref(ci)), "kx_schema_column_info")
            self.infos.append(ci)
        self.npresence = L.kx_schema_presence_bits(h)
        self.min_record_size = L.kx_schema_min_record_size(h)
        self.nested = bool(L.kx_schema_is_nested(h))   # include/kxcodec.h "Nested schemas"

    def var_columns(self) -> List[int]:
        return [c for c, ci in enumerate(self.infos) if ci.kind != A.COL_FIXED]

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                lib().kx_schema_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


class Context:
    """kx_ctx: one per host thread / stream; owns the device workspace."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        check(lib().kx_ctx_create(device, C.byref(h)), "kx_ctx_create")
        self.handle = h
        self.device = device

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                lib().kx_ctx_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


def _stream(stream):
    """The torch stream a call runs on (the caller's, else the current one)."""
    import torch
    return stream if stream is not None else torch.cuda.current_stream()


def _ptr(t) -> Optional[int]:
    return None if t is None else t.data_ptr()


def on_call_stream(fn):
    """Run the call with its `stream` argument as torch's current stream, so the outputs it allocates
    (and their zero fills) are ordered on the stream its kernels run on: the caching allocator then
    never hands a buffer a side-stream kernel still writes to another call, and no fill on the default
    stream can land after the kernel (the caller's `stream` keyword; current stream when absent)."""
    import functools

    @functools.wraps(fn)
    def run(*args, **kw):
        st = kw.get("stream")
        if st is None:
            return fn(*args, **kw)
        import torch
        with torch.cuda.stream(st):
            return fn(*args, **kw)
    return run


@dataclass
class DecodeResult:
    columns: ColumnSet
    status: "object"          # torch int64[16] on the device (kx_status)
    record_status: "object"   # torch uint8[n] or None
    stream: "object" = None   # the torch stream the decode ran on

    def read_status(self) -> A.Status:
        return read_status(self.status, self.stream)


@dataclass
class MessageBatch(DecodeResult):
    names: "object" = None     # (int64 offsets[n+1], uint8 arena) method names
    msg_type: "object" = None  # int32[n]
    seqid: "object" = None     # int32[n]
    frame_offsets: "object" = None  # UnmarshalFrames: int64[n + 1]
    kinds: "object" = None          # UnmarshalFrames: uint8[n]

    def name(self, i: int) -> str:
        o = self.names[0]
        a, b = int(o[i].item()), int(o[i + 1].item())
        return bytes(self.names[1][a:b].cpu().numpy()).decode()


@dataclass
class StreamBatch(DecodeResult):
    """UnmarshalStream: the frames of a ttstream connection buffer and the records of its DATA frames."""
    frame_offsets: "object" = None   # int64[n + 1]
    frame_types: "object" = None     # uint8[n], A.TTS_*
    stream_ids: "object" = None      # int32[n]
    method_pos: "object" = None      # int64[n] (IntInfo[ToMethod] inside buf)
    method_len: "object" = None      # int32[n]
    payload_start: "object" = None   # int64[n]
    payload_end: "object" = None     # int64[n]
    data_frames: "object" = None     # int64[records]: the DATA frame each record came from
    scan_status: "object" = None     # A.Status of the frame scan
    buf: "object" = None

    def method(self, i: int) -> str:
        p, l = int(self.method_pos[i].item()), int(self.method_len[i].item())
        return bytes(self.buf[p:p + l].cpu().numpy()).decode()


def default_ttstream_keys() -> A.TTStreamKeys:
    """kx_ttstream_default_keys: the gopkg ttheader streaming constants this library assumes"""
    k = A.TTStreamKeys()
    lib().kx_ttstream_default_keys(C.byref(k))
    return k


@on_call_stream
def ttstream_frame_scan(buf, n: int, keys: Optional[A.TTStreamKeys] = None, device: int = 0, stream=None):
    """kx_ttstream_frame_scan over a device buffer of n ttstream frames. Returns (frame offsets int64[n+1],
    payload starts int64[n], payload ends int64[n], frame types uint8[n], stream ids int32[n], method
    positions int64[n], method lengths int32[n], status tensor)."""
    import torch
    dev = torch.device("cuda", device)
    s = _stream(stream)
    ctx = _ctx_for(device, s)
    keys = keys if keys is not None else default_ttstream_keys()
    fo = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    ps = torch.zeros(max(1, n), dtype=torch.int64, device=dev)
    pe = torch.zeros(max(1, n), dtype=torch.int64, device=dev)
    ft = torch.zeros(max(1, n), dtype=torch.uint8, device=dev)
    sid = torch.zeros(max(1, n), dtype=torch.int32, device=dev)
    mp = torch.zeros(max(1, n), dtype=torch.int64, device=dev)
    ml = torch.zeros(max(1, n), dtype=torch.int32, device=dev)
    st = status_tensor(dev)
    check(lib().kx_ttstream_frame_scan(ctx.handle, _ptr(buf), buf.numel(), n, C.byref(keys), _ptr(fo), _ptr(ps),
                                       _ptr(pe), _ptr(ft), _ptr(sid), _ptr(mp), _ptr(ml), _ptr(st),
                                       int(s.cuda_stream)), "kx_ttstream_frame_scan")
    return fo, ps[:n], pe[:n], ft[:n], sid[:n], mp[:n], ml[:n], st


def status_tensor(device):
    import torch
    return torch.zeros(24, dtype=torch.int64, device=device)   # kx_status: 192 bytes


def read_status(t, stream=None) -> A.Status:
    """The kx_status a call on `stream` wrote into t: that stream is drained first (t.cpu() alone
    would copy on the current stream, possibly before a side-stream kernel has written it)."""
    _stream(stream).synchronize()
    return A.Status.from_buffer_copy(t.cpu().numpy().tobytes())


class ThriftCodec:
    """Batch Thrift-binary payload codec on one MI355X (remote.PayloadCodec mirror)."""

    _DECODE = "kx_thrift_decode_batch"
    _HOST = "kx_host_decode_batch"
    _ENCODE = "kx_thrift_encode_batch"
    _SIZE = "kx_thrift_encoded_size_batch"
    _WHAT = "thrift unmarshal"

    def __init__(self, schema: Schema, codec_type: CodecType = CodecType.FastReadWrite, device: int = 0):
        import torch
        self.codec_type = codec_type
        self.dschema = schema if isinstance(schema, DeviceSchema) else DeviceSchema(schema)
        self.device = torch.device("cuda", device)
        self._ctxs = {}           # one kx_ctx (workspace) per stream: calls on two streams never share one
        self._pipeline = None     # (chunk_bytes, ahead) applied to every ctx, None = library default
        self.ctx = self._ctx(None)

    def _ctx(self, stream) -> Context:
        key = int(_stream(stream).cuda_stream)
        c = self._ctxs.get(key)
        if c is None:
            c = self._ctxs[key] = Context(self.device.index or 0)
            if self._pipeline is not None:
                check(lib().kx_ctx_set_pipeline(c.handle, *self._pipeline), "kx_ctx_set_pipeline")
        return c

    def set_pipeline(self, chunk_bytes: int, ahead: int = 1):
        """Decode pipelining (kx_ctx_set_pipeline): chunk size in input bytes (0 = one chunk) and how
        many chunks the index pass may run ahead of emit. Results do not depend on it."""
        self._pipeline = (int(chunk_bytes), int(ahead))
        for c in self._ctxs.values():
            check(lib().kx_ctx_set_pipeline(c.handle, *self._pipeline), "kx_ctx_set_pipeline")

    # -- remote.PayloadCodec --------------------------------------------------------------------
    def Name(self) -> str:
        return "Thrift"

    @on_call_stream
    def Unmarshal(self, buf, n: int, offsets=None, out: ColumnSet = None, var_caps: Sequence[int] = None,
                  record_status: bool = False, stream=None, raise_on_error: bool = True,
                  status=None, views: bool = False) -> DecodeResult:
        """Decode n records from `buf` (uint8 tensor in HBM). offsets: int64[n+1] tensor or None.
        views: string/binary columns as zero-copy (offset, length) pairs into `buf` (KX_COLF_VIEW)."""
        import torch
        ds = self.dschema
        if out is None:
            elem_caps = sub_caps = None
            if var_caps is None and ds.nested:   # exact arenas from the measure pass
                units = self.DecodeSizes(buf, n, offsets, stream=stream)
                var_caps, elem_caps, sub_caps = units[0::3], units[1::3], units[2::3]
            if var_caps is None:
                var_caps = [0 if ci.kind == A.COL_FIXED else max(1, buf.numel()) for ci in ds.infos]
            out = alloc_device(ds.infos, n, var_caps, ds.npresence, self.device, views=views, elem_caps=elem_caps,
                               sub_caps=sub_caps)
        kc = to_kx_columns(out, ds.infos, var_caps)
        st = status if status is not None else status_tensor(self.device)
        rs = torch.empty(max(1, n), dtype=torch.uint8, device=self.device) if record_status else None
        s = _stream(stream)
        rc = getattr(lib(), self._DECODE)(self._ctx(s).handle, ds.handle, _ptr(buf), buf.numel(), _ptr(offsets), n,
                                          C.byref(kc), _ptr(rs), _ptr(st), int(s.cuda_stream))
        check(rc, self._DECODE)
        res = DecodeResult(out, st, rs, s)
        # the reference's codec choice for this call (every choice reads the same struct; the device
        # runs the batch FastRead, with the skip decoder finding the records when no dataLen is known)
        res.path = self._PATH_FN(self.codec_type, 1 if offsets is not None else 0)
        if raise_on_error:
            s = res.read_status()
            if s.code:
                raise ProtocolError(s.code, self._WHAT, s.record, s.offset)
        return res

    @on_call_stream
    def DecodeSizes(self, buf, n: int, offsets=None, stream=None, ends=None) -> List[int]:
        """Nested schemas: the arena units a decode of buf needs, 3 per column (data units, elem_offsets
        entries - 1, sub_offsets entries - 1): kx_thrift_decode_sizes (synchronous). With `ends`,
        `offsets` are the bodies' starts (explicit extents, kx_thrift_decode_sizes_extents)."""
        ds = self.dschema
        units = (C.c_uint64 * (3 * max(1, ds.ncols)))()
        st = A.Status()
        s = _stream(stream)
        if ends is not None:
            check(lib().kx_thrift_decode_sizes_extents(self._ctx(s).handle, ds.handle, _ptr(buf), buf.numel(),
                                                       _ptr(offsets), _ptr(ends), n, units, C.byref(st),
                                                       int(s.cuda_stream)), "kx_thrift_decode_sizes_extents")
        else:
            check(lib().kx_thrift_decode_sizes(self._ctx(s).handle, ds.handle, _ptr(buf), buf.numel(), _ptr(offsets),
                                               n, units, C.byref(st), int(s.cuda_stream)), "kx_thrift_decode_sizes")
        return [int(units[i]) for i in range(3 * ds.ncols)]

    def UnmarshalHost(self, wire, n: int, offsets=None, var_caps: Sequence[int] = None,
                      raise_on_error: bool = True, out: ColumnSet = None, elem_caps: Sequence[int] = None,
                      sub_caps: Sequence[int] = None, record_status: bool = False):
        """fastUnmarshal from host memory (netpoll buffers): numpy uint8 wire (+ uint64 offsets[n+1])
        -> host ColumnSet + status, via kx_host_decode_batch (H2D, device decode, D2H; with offsets
        a chunked pipeline whose copies overlap the decode). Pinned buffers reach full PCIe rate.
        Every schema: flat columns of every kind and nested schemas (var_caps / elem_caps / sub_caps: the
        units each column's arrays hold; default: the wire size, a bound for every column kind).
        record_status=True: returns (out, status, codes uint8[n]) with each record's own code."""
        import numpy as np
        ds = self.dschema
        if var_caps is None:
            var_caps = [0 if ci.kind == A.COL_FIXED else max(1, wire.size) for ci in ds.infos]
        if out is None:
            out = alloc_host(ds.infos, n, var_caps, ds.npresence, elem_caps=elem_caps, sub_caps=sub_caps)
        kc = to_kx_columns(out, ds.infos, var_caps)
        st = A.Status()
        wire = np.ascontiguousarray(wire, dtype=np.uint8)
        offp = None
        if offsets is not None:
            offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
            offp = offsets.ctypes.data
        rs = np.zeros(max(1, n), dtype=np.uint8) if record_status else None
        rc = getattr(lib(), self._HOST)(self.ctx.handle, ds.handle, wire.ctypes.data if wire.size else None,
                                        wire.size, offp, n, C.byref(kc), rs.ctypes.data if rs is not None else None,
                                        C.byref(st))
        check(rc, self._HOST)
        if raise_on_error and st.code:
            raise ProtocolError(st.code, self._WHAT, st.record, st.offset)
        return (out, st, rs[:n]) if record_status else (out, st)

    _HOST_ENCODE = "kx_host_encode_batch"

    def MarshalHost(self, cols: ColumnSet, out=None, with_offsets: bool = True, raise_on_error: bool = True,
                    record_status: bool = False):
        """fastMarshal to host memory (the reply path, codec_fast.go:40-58): host ColumnSet (numpy; pinned
        buffers reach full PCIe rate; flat or nested schemas) -> (wire uint8 numpy, offsets uint64[n+1] or
        None, status) via kx_host_encode_batch (H2D of the columns, device encode, D2H of the wire; with
        n >= 64 Ki a chunked pipeline whose copies overlap the encode). `out`: a preallocated uint8 buffer
        (default: an upper bound from the column sizes). record_status=True appends each record's code."""
        import numpy as np
        ds = self.dschema
        n = cols.n
        kc = to_kx_columns(cols, ds.infos)
        if out is None:
            out = np.empty(max(1, _host_encode_bound(cols, ds.infos, n, self._HOST_ENCODE != "kx_host_encode_batch")),
                           dtype=np.uint8)
        offs = np.empty(n + 1, dtype=np.uint64) if with_offsets else None
        rs = np.zeros(max(1, n), dtype=np.uint8) if record_status else None
        st = A.Status()
        rc = getattr(lib(), self._HOST_ENCODE)(self.ctx.handle, ds.handle, C.byref(kc), n, out.ctypes.data, out.size,
                                               offs.ctypes.data if offs is not None else None,
                                               rs.ctypes.data if rs is not None else None, C.byref(st))
        check(rc, self._HOST_ENCODE)
        if raise_on_error and st.code:
            raise ProtocolError(st.code, self._HOST_ENCODE)
        wire = out[:min(st.consumed, out.size)]
        return (wire, offs, st, rs[:n]) if record_status else (wire, offs, st)

    _MESSAGES = "kx_thrift_decode_messages"
    _FRAMES = "kx_thrift_decode_frames"
    _GRPC = "kx_thrift_decode_grpc"
    _PATH_FN = staticmethod(select_unmarshal)

    @on_call_stream
    def UnmarshalMessages(self, buf, n: int, offsets, body_field: int = 1, out: ColumnSet = None,
                          var_caps: Sequence[int] = None, name_cap: int = None, stream=None,
                          raise_on_error: bool = True) -> "MessageBatch":
        """thriftCodec.Unmarshal over n framed messages: buf[offsets[i]:offsets[i+1]] = MessageBegin +
        the method's Args (body_field 1) / Result (body_field 0) struct holding one record.
        Returns the record columns plus method name / message type / seqid columns."""
        s = _stream(stream)
        args = [self._ctx(s).handle, self.dschema.handle, _ptr(buf), buf.numel(), _ptr(offsets), n]
        if self._MESSAGES == "kx_thrift_decode_messages":
            args.append(body_field)
        return self._messages(self._MESSAGES, args, buf, n, out, var_caps, name_cap, s, raise_on_error)

    @on_call_stream
    def UnmarshalFrames(self, buf, n: int, body_field: int = 1, max_payload: int = 0, out: ColumnSet = None,
                        var_caps: Sequence[int] = None, name_cap: int = None, stream=None,
                        raise_on_error: bool = True, crc32_check: bool = False,
                        frame_offsets: bool = True) -> "MessageBatch":
        """A socket buffer of n frames (TTHeader / Mesh / Framed / PurePayload, default_codec.go:189-221)
        straight to columns: framing sniff on the device, then UnmarshalMessages on the payloads.
        The batch also carries frame_offsets (int64[n+1]) and kinds (uint8[n], transport.Protocol |
        FRAME_PB | FRAME_MESH). crc32_check: CodecConfig{CRC32Check: true} (default_codec.go:70-92), every
        TTHeader frame's "crc32c" header is checked against its payload (ERR_PAYLOAD_VALIDATION).
        frame_offsets=False passes NULL for them (the library keeps them in its scratch) and the batch
        carries none."""
        import torch
        s = _stream(stream)
        check(lib().kx_ctx_set_crc32c_check(self._ctx(s).handle, 1 if crc32_check else 0), "set crc32c check")
        fo = torch.zeros(n + 1, dtype=torch.int64, device=self.device) if frame_offsets else None
        kinds = torch.zeros(max(1, n), dtype=torch.uint8, device=self.device)
        args = [self._ctx(s).handle, self.dschema.handle, _ptr(buf), buf.numel(), n]
        if self._FRAMES == "kx_thrift_decode_frames":
            args.append(body_field)
        args += [max_payload, _ptr(fo) if fo is not None else None, _ptr(kinds)]
        res = self._messages(self._FRAMES, args, buf, n, out, var_caps, name_cap, s, raise_on_error)
        res.frame_offsets, res.kinds = fo, kinds[:n]
        return res

    @on_call_stream
    def UnmarshalGRPC(self, buf, n: int, max_payload: int = 0, out: ColumnSet = None,
                      var_caps: Sequence[int] = None, stream=None, raise_on_error: bool = True) -> "DecodeResult":
        """grpcCodec.Decode (pkg/remote/codec/grpc/grpc.go:202-270) over n gRPC messages back to back
        ([u8 compressed][u32 BE length][payload], decodeGRPCFrame grpc_compress.go:37-60): each payload is
        one record. The result also carries frame_offsets (int64[n+1]); a compressed message's code is
        ERR_NOT_IMPLEMENTED (no decompressor on the device)."""
        import torch
        s = _stream(stream)
        ds = self.dschema
        if out is None:
            if var_caps is None:
                var_caps = [0 if ci.kind == A.COL_FIXED else max(1, buf.numel()) for ci in ds.infos]
            out = alloc_device(ds.infos, n, var_caps, ds.npresence, self.device)
        kc = to_kx_columns(out, ds.infos, var_caps)
        fo = torch.zeros(n + 1, dtype=torch.int64, device=self.device)
        st = status_tensor(self.device)
        rs = torch.empty(max(1, n), dtype=torch.uint8, device=self.device)
        fn = self._GRPC
        rc = getattr(lib(), fn)(self._ctx(s).handle, ds.handle, _ptr(buf), buf.numel(), n, max_payload, _ptr(fo),
                                C.byref(kc), _ptr(rs), _ptr(st), int(s.cuda_stream))
        check(rc, fn)
        res = DecodeResult(out, st, rs, s)
        res.frame_offsets = fo
        if raise_on_error:
            stt = res.read_status()
            if stt.code:
                raise ProtocolError(stt.code, self._WHAT, stt.record, stt.offset)
        return res

    _EXTENTS = "kx_thrift_decode_extents"

    @on_call_stream
    def UnmarshalExtents(self, buf, starts, ends, out: ColumnSet = None, var_caps: Sequence[int] = None,
                         stream=None, raise_on_error: bool = True) -> DecodeResult:
        """FastUnmarshal of n bare bodies at explicit extents buf[starts[i]:ends[i]) (int64 device tensors;
        ttstream DecodePayload, frame.go:223-233). record_status per body."""
        import torch
        ds = self.dschema
        n = int(starts.numel())
        starts = starts.to(torch.int64).contiguous()
        ends = ends.to(torch.int64).contiguous()
        if out is None:
            elem_caps = sub_caps = None
            if var_caps is None and ds.nested:
                # exact arenas from the measure pass over the same extents (a connection buffer's worth of
                # buf-sized arenas per column would not fit for wide nested schemas)
                units = self.DecodeSizes(buf, n, starts, stream=stream, ends=ends)
                var_caps, elem_caps, sub_caps = units[0::3], units[1::3], units[2::3]
            if var_caps is None:
                var_caps = [0 if ci.kind == A.COL_FIXED else max(1, buf.numel()) for ci in ds.infos]
            out = alloc_device(ds.infos, n, var_caps, ds.npresence, self.device, elem_caps=elem_caps,
                               sub_caps=sub_caps)
        kc = to_kx_columns(out, ds.infos, var_caps)
        st = status_tensor(self.device)
        rs = torch.empty(max(1, n), dtype=torch.uint8, device=self.device)
        s = _stream(stream)
        rc = getattr(lib(), self._EXTENTS)(self._ctx(s).handle, ds.handle, _ptr(buf), buf.numel(), _ptr(starts),
                                           _ptr(ends), n, C.byref(kc), _ptr(rs), _ptr(st), int(s.cuda_stream))
        check(rc, self._EXTENTS)
        res = DecodeResult(out, st, rs, s)
        if raise_on_error:
            stt = res.read_status()
            if stt.code:
                raise ProtocolError(stt.code, self._WHAT, stt.record, stt.offset)
        return res

    @on_call_stream
    def UnmarshalStream(self, buf, n_frames: int, keys: Optional[A.TTStreamKeys] = None, stream=None,
                        raise_on_error: bool = True) -> "StreamBatch":
        """ttstream's receive side over a connection buffer of n TTHeader streaming frames (DecodeFrame,
        pkg/remote/trans/ttstream/frame.go:137-185): every frame located and classified on the device
        (kx_ttstream_frame_scan), then the DATA frames' payloads decoded as records (DecodePayload ->
        FastUnmarshal, :223-233; kx_*_decode_extents). Records are in DATA-frame order; data_frames[j]
        is the frame record j came from."""
        import torch
        s = _stream(stream)
        fo, ps, pe, ft, sid, mp, ml, st = ttstream_frame_scan(buf, n_frames, keys, self.device.index or 0, s)
        stt = read_status(st, s)
        if stt.code and raise_on_error:
            raise ProtocolError(stt.code, "ttstream DecodeFrame", stt.record, stt.offset)
        nf = stt.n_records if stt.code else n_frames
        data = torch.nonzero(ft[:nf] == A.TTS_DATA).flatten()
        res = self.UnmarshalExtents(buf, ps[data], pe[data], stream=s, raise_on_error=raise_on_error)
        return StreamBatch(res.columns, res.status, res.record_status, s, frame_offsets=fo, frame_types=ft,
                           stream_ids=sid, method_pos=mp, method_len=ml, payload_start=ps, payload_end=pe,
                           data_frames=data, scan_status=stt, buf=buf)

    def _messages(self, fn, args, buf, n, out, var_caps, name_cap, s, raise_on_error):
        import torch
        ds = self.dschema
        if out is None:
            if var_caps is None:
                var_caps = [0 if ci.kind == A.COL_FIXED else max(1, buf.numel()) for ci in ds.infos]
            out = alloc_device(ds.infos, n, var_caps, ds.npresence, self.device)
        kc = to_kx_columns(out, ds.infos, var_caps)
        name_cap = max(1, buf.numel() if name_cap is None else name_cap)
        names = (torch.zeros(n + 1, dtype=torch.int64, device=self.device),
                 torch.empty(name_cap, dtype=torch.uint8, device=self.device))
        mtype = torch.zeros(max(1, n), dtype=torch.int32, device=self.device)
        seqid = torch.zeros(max(1, n), dtype=torch.int32, device=self.device)
        mc = (A.Column * 3)()
        mc[0].data, mc[0].offsets, mc[0].capacity, mc[0].offset_bytes = names[1].data_ptr(), names[0].data_ptr(), \
            name_cap, 8
        mc[1].data = mtype.data_ptr()
        mc[2].data = seqid.data_ptr()
        st = status_tensor(self.device)
        rs = torch.empty(max(1, n), dtype=torch.uint8, device=self.device)
        rc = getattr(lib(), fn)(*args, mc, C.byref(kc), _ptr(rs), _ptr(st), int(s.cuda_stream))
        check(rc, fn)
        res = MessageBatch(out, st, rs, s, names, mtype[:n], seqid[:n])
        if raise_on_error:
            stt = res.read_status()
            if stt.code:
                raise ProtocolError(stt.code, self._WHAT, stt.record, stt.offset)
        return res

    @on_call_stream
    def Marshal(self, cols: ColumnSet, with_offsets: bool = True, stream=None, out=None, status=None,
                check_status: bool = True):
        """Encode the columns; returns (wire uint8 tensor, record offsets int64[n+1] or None).
        check_status=False (with `out` and `status` given) leaves the call asynchronous: the wire is
        the whole `out` and the caller reads `status` later."""
        import torch
        ds = self.dschema
        n = cols.n
        kc = to_kx_columns(cols, ds.infos)
        if out is None:
            sizes = self.BLength(cols, stream=stream)
            total = int(sizes.sum().item()) if n else 0
            out = torch.empty(max(1, total), dtype=torch.uint8, device=self.device)
        else:
            total = out.numel()
        offs = torch.empty(n + 1, dtype=torch.int64, device=self.device) if with_offsets else None
        st = status if status is not None else status_tensor(self.device)
        ss = _stream(stream)
        rc = getattr(lib(), self._ENCODE)(self._ctx(ss).handle, ds.handle, C.byref(kc), n, _ptr(out), out.numel(),
                                          _ptr(offs), _ptr(st), int(ss.cuda_stream))
        check(rc, self._ENCODE)
        if not check_status:
            return out, offs
        s = read_status(st, ss)
        if s.code:
            raise ProtocolError(s.code, self._ENCODE)
        return out[:s.consumed], offs

    @on_call_stream
    def MarshalMessages(self, cols: ColumnSet, method: str, seqids, msg_type: int = 1, body_field: int = 1,
                        stream=None):
        """fastMarshal (codec_fast.go:40-58) of n messages: MessageBegin(method, msg_type, seqids[i]) + the
        Args{body_field: record i} (or Result{0: success}) struct + STOP, on the device. Returns (messages
        uint8 tensor, message offsets int64[n+1])."""
        import torch
        if self._ENCODE != "kx_thrift_encode_batch":
            raise KxError(A.ERR_NOT_IMPLEMENTED, "MarshalMessages: Thrift only")
        ds = self.dschema
        n = cols.n
        # the kernel reads int32[n] seqids from device memory: anything else is converted or refused here
        if not isinstance(seqids, torch.Tensor):
            seqids = torch.as_tensor(seqids, dtype=torch.int32)
        if seqids.dtype != torch.int32:
            if seqids.dtype.is_floating_point or seqids.dtype == torch.bool:
                raise KxError(A.ERR_INVALID_ARG, f"MarshalMessages: seqids must be integers, got {seqids.dtype}")
            if n and (int(seqids.min()) < -(1 << 31) or int(seqids.max()) >= (1 << 31)):
                raise KxError(A.ERR_INVALID_ARG, "MarshalMessages: a seqid does not fit in int32")
            seqids = seqids.to(torch.int32)
        if seqids.dim() != 1 or seqids.numel() < n:
            raise KxError(A.ERR_INVALID_ARG, f"MarshalMessages: need {n} seqids, got shape {tuple(seqids.shape)}")
        seqids = seqids.to(self.device).contiguous()
        kc = to_kx_columns(cols, ds.infos)
        body = int(self.BLength(cols, stream=stream).sum().item()) if n else 0
        nb = method.encode()
        total = body + n * (16 + len(nb))
        scratch = torch.empty(max(1, body), dtype=torch.uint8, device=self.device)
        out = torch.empty(max(1, total), dtype=torch.uint8, device=self.device)
        offs = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        st = status_tensor(self.device)
        ss = _stream(stream)
        rc = lib().kx_thrift_encode_messages(self._ctx(ss).handle, ds.handle, C.byref(kc), n, nb, len(nb), msg_type,
                                             _ptr(seqids), body_field, _ptr(scratch), scratch.numel(), _ptr(out),
                                             out.numel(), _ptr(offs), _ptr(st), int(ss.cuda_stream))
        check(rc, "kx_thrift_encode_messages")
        s = read_status(st, ss)
        if s.code:
            raise ProtocolError(s.code, "fastMarshal")
        return out[:s.consumed], offs

    @on_call_stream
    def BLength(self, cols: ColumnSet, stream=None):
        import torch
        ds = self.dschema
        kc = to_kx_columns(cols, ds.infos)
        sizes = torch.empty(max(1, cols.n), dtype=torch.int64, device=self.device)
        ss = _stream(stream)
        rc = getattr(lib(), self._SIZE)(self._ctx(ss).handle, ds.handle, C.byref(kc), cols.n, _ptr(sizes),
                                        int(ss.cuda_stream))
        check(rc, self._SIZE)
        return sizes[:cols.n]

    @on_call_stream
    def Skip(self, buf, n: int, stream=None):
        """skipThriftStruct over n concatenated records -> int64[n+1] record offsets."""
        import torch
        offs = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        st = status_tensor(self.device)
        ss = _stream(stream)
        rc = lib().kx_thrift_skip_batch(self._ctx(ss).handle, _ptr(buf), buf.numel(), n, _ptr(offs), _ptr(st),
                                        int(ss.cuda_stream))
        check(rc, "kx_thrift_skip_batch")
        s = read_status(st, ss)
        if s.code:
            raise ProtocolError(s.code, "skipThriftStruct", s.record, s.offset)
        return offs

    @on_call_stream
    def SplitPoints(self, buf, n: int, parts: int, stream=None):
        """kx_thrift_split_points: the parts + 1 record boundaries that cut n concatenated records into
        `parts` shards of equal record counts (shard k holds floor((k+1)n/parts) - floor(kn/parts) records)
        -> int64[parts + 1]. The index and chain passes of a decode, no emit (SURVEY.md §8e pass A)."""
        import torch
        pts = torch.empty(parts + 1, dtype=torch.int64, device=self.device)
        st = status_tensor(self.device)
        ss = _stream(stream)
        rc = lib().kx_thrift_split_points(self._ctx(ss).handle, self.dschema.handle, _ptr(buf), buf.numel(), n,
                                          parts, _ptr(pts), _ptr(st), int(ss.cuda_stream))
        check(rc, "kx_thrift_split_points")
        s = read_status(st, ss)
        if s.code:
            raise ProtocolError(s.code, "split points", s.record, s.offset)
        return pts

    # lower-case aliases
    name, unmarshal, marshal, blength, skip = Name, Unmarshal, Marshal, BLength, Skip
    split_points = SplitPoints


def _host_encode_bound(cols: ColumnSet, infos, n: int, pb: bool) -> int:
    """an upper bound of the encoded size of host columns: per record 16 bytes per column (header, length,
    list header, STOP / frame) plus 16 per fixed value, plus per var column its payload bytes and 16 bytes
    per element of every level (headers, lengths, element STOPs; elements at up to 10 bytes as proto
    varints)"""
    import numpy as np
    total = n * (16 * (len(infos) + 2) + 16)
    for c, ci in enumerate(infos):
        if ci.kind == A.COL_FIXED:
            total += n * 16
            continue
        parts = cols.cols[c]
        hi = n
        for arr in parts[:-1]:            # walk the offsets chain: the units of every level
            hi = int(np.asarray(arr)[hi])
            total += 16 * hi
        width = 1 if ci.kind in (A.COL_BYTES, A.COL_LIST_BYTES, A.COL_LIST2_BYTES) else ci.width
        total += hi * (max(width, 10) if pb and width > 1 else width)
    return total


class ProtobufCodec(ThriftCodec):
    """Batch Kitex-Protobuf payload codec (pkg/remote/codec/protobuf/protobuf.go:49-61).

    Unmarshal = proto.Unmarshal of each record body (protobuf.go:135-170 -> service.go:358-365):
    with offsets, n bare proto3 bodies with known extents; without, the body of
    `message Batch { repeated Rec recs = 1; }` (record boundaries found on the GPU)."""

    _DECODE = "kx_pb_decode_batch"
    _HOST = "kx_host_pb_decode_batch"
    _HOST_ENCODE = "kx_host_pb_encode_batch"
    _MESSAGES = "kx_pb_decode_messages"
    _FRAMES = "kx_pb_decode_frames"
    _GRPC = "kx_pb_decode_grpc"
    _PATH_FN = staticmethod(lambda codec_type, data_len: "protobuf")
    _EXTENTS = "kx_pb_decode_extents"
    _ENCODE = "kx_pb_encode_batch"
    _SIZE = "kx_pb_encoded_size_batch"
    _WHAT = "protobuf unmarshal"

    def __init__(self, schema: Schema, device: int = 0):
        super().__init__(schema, CodecType.Basic, device)

    def Name(self) -> str:
        return "protobuf"

    @on_call_stream
    def Skip(self, buf, n: int, stream=None):
        raise KxError(A.ERR_NOT_IMPLEMENTED, "protobuf has no skip decoder")

    @on_call_stream
    def SplitPoints(self, buf, n: int, parts: int, stream=None):
        """kx_thrift_split_points walks Thrift records; a flat proto3 schema carries no wire-format mark the
        library could refuse it by (its calls choose the format), so the codec refuses it here"""
        raise KxError(A.ERR_NOT_IMPLEMENTED, "split points: Thrift records only")

    name, skip, split_points = Name, Skip, SplitPoints


def write_message_begin(name: str, msg_type: int, seqid: int) -> bytes:
    """thrift.Binary.WriteMessageBegin (binary_test.go:387-457) via the C-ABI."""
    nb = name.encode()
    buf = (C.c_uint8 * (12 + len(nb)))()
    w = C.c_uint64()
    check(lib().kx_thrift_write_message_begin(buf, len(buf), nb, len(nb), msg_type, seqid, C.byref(w)),
          "WriteMessageBegin")
    return bytes(buf[:w.value])


def read_message_begin(data: bytes):
    L = lib()
    arr = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    name, nl, t, s, u = C.c_char_p(), C.c_uint32(), C.c_int32(), C.c_int32(), C.c_uint64()
    rc = L.kx_thrift_read_message_begin(arr, len(data), C.byref(name), C.byref(nl), C.byref(t), C.byref(s),
                                        C.byref(u))
    if rc:
        raise ProtocolError(rc, "ReadMessageBegin")
    off = C.cast(name, C.c_void_p).value - C.addressof(arr)
    return bytes(data[off:off + nl.value]).decode(), t.value, s.value, u.value


def write_pb_meta(name: str, msg_type: int, seqid: int) -> bytes:
    """Kitex-Protobuf meta header (protobuf.go:77-90) via the C-ABI."""
    nb = name.encode()
    buf = (C.c_uint8 * (12 + len(nb)))()
    w = C.c_uint64()
    check(lib().kx_pb_write_meta(buf, len(buf), nb, len(nb), msg_type, seqid, C.byref(w)), "pb write meta")
    return bytes(buf[:w.value])


def read_pb_meta(data: bytes):
    arr = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    name, nl, t, s, u = C.c_char_p(), C.c_uint32(), C.c_int32(), C.c_int32(), C.c_uint64()
    rc = lib().kx_pb_read_meta(arr, len(data), C.byref(name), C.byref(nl), C.byref(t), C.byref(s), C.byref(u))
    if rc:
        raise ProtocolError(rc, "pb read meta")
    off = C.cast(name, C.c_void_p).value - C.addressof(arr)
    return bytes(data[off:off + nl.value]).decode(), t.value, s.value, u.value


@on_call_stream
def grpc_frame_scan(buf, n: int, max_payload: int = 0, device: int = 0, stream=None):
    """kx_grpc_frame_scan over a device buffer of n gRPC messages. Returns (frame offsets int64[n+1],
    payload starts int64[n], payload ends int64[n], compressed flags uint8[n], status tensor)."""
    import torch
    dev = torch.device("cuda", device)
    s = _stream(stream)
    ctx = _ctx_for(device, s)
    fo = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    ps = torch.zeros(max(1, n), dtype=torch.int64, device=dev)
    pe = torch.zeros(max(1, n), dtype=torch.int64, device=dev)
    fl = torch.zeros(max(1, n), dtype=torch.uint8, device=dev)
    st = status_tensor(dev)
    check(lib().kx_grpc_frame_scan(ctx.handle, _ptr(buf), buf.numel(), n, max_payload, _ptr(fo), _ptr(ps),
                                   _ptr(pe), _ptr(fl), _ptr(st), int(s.cuda_stream)), "kx_grpc_frame_scan")
    return fo, ps[:n], pe[:n], fl[:n], st


@on_call_stream
def frame_scan(buf, n: int, max_payload: int = 0, device: int = 0, stream=None):
    """kx_frame_scan: the framing sniff alone over a device buffer of n frames. Returns (frame offsets
    int64[n+1], payload starts int64[n], payload ends int64[n], kinds uint8[n], status tensor)."""
    import torch
    dev = torch.device("cuda", device)
    s = _stream(stream)
    key = (device, int(s.cuda_stream))
    ctx = _SCAN_CTX.get(key)
    if ctx is None:
        ctx = _SCAN_CTX[key] = Context(device)
    fo = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    ps = torch.zeros(max(1, n), dtype=torch.int64, device=dev)
    pe = torch.zeros(max(1, n), dtype=torch.int64, device=dev)
    kinds = torch.zeros(max(1, n), dtype=torch.uint8, device=dev)
    st = status_tensor(dev)
    check(lib().kx_frame_scan(ctx.handle, _ptr(buf), buf.numel(), n, max_payload, _ptr(fo), _ptr(ps), _ptr(pe),
                              _ptr(kinds), _ptr(st), int(s.cuda_stream)), "kx_frame_scan")
    return fo, ps[:n], pe[:n], kinds[:n], st


_SCAN_CTX = {}


def _ctx_for(device, s):
    key = (device, int(s.cuda_stream))
    ctx = _SCAN_CTX.get(key)
    if ctx is None:
        ctx = _SCAN_CTX[key] = Context(device)
    return ctx


class CRC32PayloadValidator:
    """crcPayloadValidator (pkg/remote/codec/validate.go:168-217) over batches on the device.

    Generate(buf, offsets) = getCRC32C of each payload buf[offsets[i]:offsets[i+1]] (:187-189, :208-217),
    as uint32 values (the header value is their big-endian lowercase hex, `hex_value`). ValidateFrames
    runs payloadChecksumValidate (:91-127) over n TTHeader frames located by frame_scan."""

    KEY = "crc32c"  # transmeta.HeaderCRC32C

    def __init__(self, device: int = 0):
        self.device = device

    def Key(self) -> str:
        return self.KEY

    @staticmethod
    def hex_value(crc: int) -> str:
        return "%08x" % (crc & 0xFFFFFFFF)

    @on_call_stream
    def Generate(self, buf, offsets, stream=None):
        """-> int64 tensor of CRC-32C values (0..2^32-1), one per range"""
        import torch
        s = _stream(stream)
        n = offsets.numel() - 1
        out = torch.zeros(max(1, n), dtype=torch.int32, device=buf.device)
        st = status_tensor(buf.device)
        check(lib().kx_crc32c_batch(_ctx_for(self.device, s).handle, _ptr(buf), buf.numel(), _ptr(offsets), n,
                                    _ptr(out), _ptr(st), int(s.cuda_stream)), "kx_crc32c_batch")
        stt = read_status(st, s)
        if stt.code:
            raise KxError(stt.code, "crc32c generate", stt.record, stt.offset)
        return out[:n].to(torch.int64) & 0xFFFFFFFF

    @on_call_stream
    def ValidateFrames(self, buf, frame_offsets, n: int, stream=None, raise_on_error: bool = False):
        """-> (per-frame codes uint8[n], per-frame payload CRC int64[n], kx_status)"""
        import torch
        s = _stream(stream)
        crc = torch.zeros(max(1, n), dtype=torch.int32, device=buf.device)
        rs = torch.zeros(max(1, n), dtype=torch.uint8, device=buf.device)
        st = status_tensor(buf.device)
        check(lib().kx_frame_crc32c_validate(_ctx_for(self.device, s).handle, _ptr(buf), buf.numel(),
                                             _ptr(frame_offsets), n, _ptr(crc), _ptr(rs), _ptr(st),
                                             int(s.cuda_stream)), "kx_frame_crc32c_validate")
        stt = read_status(st, s)
        if raise_on_error and stt.code:
            raise ProtocolError(stt.code, "payload validation", stt.record, stt.offset)
        return rs[:n], crc[:n].to(torch.int64) & 0xFFFFFFFF, stt
