/*
 * kx_oracle.c — TEST INFRASTRUCTURE ONLY (see kx_oracle.h). A plain-C restatement of the reference
 * algorithms; each function cites the reference file:line it follows. Written for clarity first, but
 * kept allocation-free per record so that the multi-threaded build is a fair CPU baseline.
 */
#include "kx_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------------
 * Byte helpers: thrift is big-endian two's complement (binary_test.go:215-276).
 * ---------------------------------------------------------------------------------------------- */
static inline uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
static inline uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
static inline uint64_t be64(const uint8_t* p) { return ((uint64_t)be32(p) << 32) | be32(p + 4); }
static inline void put16(uint8_t* p, uint16_t v) { p[0] = v >> 8; p[1] = (uint8_t)v; }
static inline void put32(uint8_t* p, uint32_t v) {
  p[0] = v >> 24; p[1] = v >> 16; p[2] = v >> 8; p[3] = (uint8_t)v;
}
static inline void put64(uint8_t* p, uint64_t v) { put32(p, (uint32_t)(v >> 32)); put32(p + 4, (uint32_t)v); }

/* kx_column offsets are 4 (default) or 8 bytes wide; a 4-byte column never wraps (SIZE_LIMIT) */
static int off_w(const kx_column* c) { return c->offset_bytes == 8 ? 8 : 4; }
static uint64_t off_get(const kx_column* c, uint64_t i) {
  return off_w(c) == 8 ? ((const uint64_t*)c->offsets)[i] : ((const uint32_t*)c->offsets)[i];
}
static void off_set(const kx_column* c, uint64_t i, uint64_t v) {
  if (off_w(c) == 8) ((uint64_t*)c->offsets)[i] = v;
  else ((uint32_t*)c->offsets)[i] = (uint32_t)v;
}
static uint64_t arena_lim(const kx_column* c) {
  return off_w(c) == 8 || c->capacity < 0xffffffffull ? c->capacity : 0xffffffffull;
}
/* LIST_BYTES: element byte offsets (same width as the record offsets), element capacity */
static void eoff_set(const kx_column* c, uint64_t i, uint64_t v) {
  if (off_w(c) == 8) ((uint64_t*)c->elem_offsets)[i] = v;
  else ((uint32_t*)c->elem_offsets)[i] = (uint32_t)v;
}
static uint64_t eoff_get(const kx_column* c, uint64_t i) {
  return off_w(c) == 8 ? ((const uint64_t*)c->elem_offsets)[i] : ((const uint32_t*)c->elem_offsets)[i];
}
static uint64_t elem_lim(const kx_column* c) {
  return off_w(c) == 8 || c->elem_capacity < 0xffffffffull ? c->elem_capacity : 0xffffffffull;
}

/* typeToSize (codec_apache.go:182-189) */
static int type_size(uint8_t t) {
  switch (t) {
    case KX_T_BOOL: case KX_T_BYTE: return 1;
    case KX_T_I16: return 2;
    case KX_T_I32: return 4;
    case KX_T_DOUBLE: case KX_T_I64: return 8;
    default: return 0;
  }
}
/* golang.IsFixedLengthType as used by reorderStructFields (patcher.go:503-522): base scalar types. */
static int is_fixed_length(uint8_t t) { return type_size(t) > 0; }

/* ------------------------------------------------------------------------------------------------
 * Primitives (gopkg thrift.Binary; byte layouts pinned by pkg/protocol/bthrift/binary_test.go)
 * ---------------------------------------------------------------------------------------------- */
size_t kxo_write_field_begin(uint8_t* b, uint8_t t, int16_t id) { b[0] = t; put16(b + 1, (uint16_t)id); return 3; }
size_t kxo_write_field_stop(uint8_t* b) { b[0] = KX_T_STOP; return 1; }
size_t kxo_write_map_begin(uint8_t* b, uint8_t kt, uint8_t vt, int32_t n) { b[0] = kt; b[1] = vt; put32(b + 2, (uint32_t)n); return 6; }
size_t kxo_write_list_begin(uint8_t* b, uint8_t et, int32_t n) { b[0] = et; put32(b + 1, (uint32_t)n); return 5; }
size_t kxo_write_set_begin(uint8_t* b, uint8_t et, int32_t n) { return kxo_write_list_begin(b, et, n); }
size_t kxo_write_bool(uint8_t* b, int v) { b[0] = v ? 1 : 0; return 1; }
size_t kxo_write_byte(uint8_t* b, int8_t v) { b[0] = (uint8_t)v; return 1; }
size_t kxo_write_i16(uint8_t* b, int16_t v) { put16(b, (uint16_t)v); return 2; }
size_t kxo_write_i32(uint8_t* b, int32_t v) { put32(b, (uint32_t)v); return 4; }
size_t kxo_write_i64(uint8_t* b, int64_t v) { put64(b, (uint64_t)v); return 8; }
size_t kxo_write_double(uint8_t* b, double v) { uint64_t u; memcpy(&u, &v, 8); put64(b, u); return 8; }
size_t kxo_write_string(uint8_t* b, const uint8_t* s, uint32_t n) { put32(b, n); if (n) memcpy(b + 4, s, n); return 4 + (size_t)n; }

/* WriteMessageBegin: u32(0x80010000|type) u32(len) name i32(seqid)  (binary_test.go:389-393) */
size_t kxo_write_message_begin(uint8_t* b, const char* name, uint32_t n, int32_t type, int32_t seqid) {
  put32(b, 0x80010000u | ((uint32_t)type & 0xffu));
  put32(b + 4, n);
  if (n) memcpy(b + 8, name, n);
  put32(b + 8 + n, (uint32_t)seqid);
  return 12 + (size_t)n;
}
size_t kxo_message_begin_length(uint32_t n) { return 12 + (size_t)n; } /* binary_test.go:338 */

/* ReadMessageBegin. Strict (versioned) form only; a non-strict header is rejected with BAD_VERSION
 * (parity unpinned: gopkg has no in-tree test; the generic binary path also rejects it,
 * pkg/generic/binarythrift_codec.go:153-156). */
int kxo_read_message_begin(const uint8_t* b, size_t len, uint32_t* name_off, uint32_t* name_len,
                           int32_t* type, int32_t* seqid, size_t* used) {
  if (len < 4) return KX_ERR_EOF;
  uint32_t v = be32(b);
  if ((v & 0xffff0000u) != 0x80010000u) return KX_ERR_BAD_VERSION;
  if (len < 8) return KX_ERR_EOF;
  int32_t n = (int32_t)be32(b + 4);
  if (n < 0) return KX_ERR_NEGATIVE_SIZE;
  if ((uint64_t)len < 12 + (uint64_t)n) return KX_ERR_EOF;
  *type = (int32_t)(v & 0xffu);
  *name_off = 8; *name_len = (uint32_t)n;
  *seqid = (int32_t)be32(b + 8 + n);
  *used = 12 + (size_t)n;
  return KX_OK;
}

/* ------------------------------------------------------------------------------------------------
 * Skip decoder: netpollSkipDecoder.skipType (pkg/remote/codec/thrift/codec_apache.go:191-293)
 * restated over a byte slice. skipn() beyond the slice is the reader's EOF.
 * ---------------------------------------------------------------------------------------------- */
typedef struct { const uint8_t* b; size_t len; size_t n; } skipper;

static int skipn(skipper* s, uint64_t k) {
  if ((uint64_t)s->n + k > (uint64_t)s->len) return KX_ERR_EOF;
  s->n += (size_t)k;
  return KX_OK;
}

static int skip_type(skipper* s, uint8_t t, int maxdepth) {
  if (maxdepth == 0) return KX_ERR_DEPTH_LIMIT;                 /* :192-194 */
  int sz = type_size(t);
  if (sz > 0) return skipn(s, (uint64_t)sz);                     /* :195-197 */
  int rc;
  switch (t) {
    case KX_T_STRING: {                                          /* :199-209 */
      if ((rc = skipn(s, 4))) return rc;
      int32_t l = (int32_t)be32(s->b + s->n - 4);
      if (l < 0) return KX_ERR_INVALID_DATA;                     /* errDataLength */
      return skipn(s, (uint64_t)l);
    }
    case KX_T_STRUCT:                                            /* :210-234 */
      for (;;) {
        if ((rc = skipn(s, 1))) return rc;
        uint8_t tp = s->b[s->n - 1];
        if (tp == KX_T_STOP) break;
        int fsz = type_size(tp);
        if (fsz > 0) { if ((rc = skipn(s, 2 + (uint64_t)fsz))) return rc; continue; }
        if ((rc = skipn(s, 2))) return rc;
        if ((rc = skip_type(s, tp, maxdepth - 1))) return rc;
      }
      return KX_OK;
    case KX_T_MAP: {                                             /* :235-268 */
      if ((rc = skipn(s, 6))) return rc;
      const uint8_t* h = s->b + s->n - 6;
      uint8_t kt = h[0], vt = h[1];
      int32_t n = (int32_t)be32(h + 2);
      if (n < 0) return KX_ERR_INVALID_DATA;
      int ks = type_size(kt), vs = type_size(vt);
      if (ks > 0 && vs > 0) return skipn(s, (uint64_t)n * (uint64_t)(ks + vs));
      for (int32_t i = 0; i < n; i++) {
        rc = ks > 0 ? skipn(s, (uint64_t)ks) : skip_type(s, kt, maxdepth - 1);
        if (rc) return rc;
        rc = vs > 0 ? skipn(s, (uint64_t)vs) : skip_type(s, vt, maxdepth - 1);
        if (rc) return rc;
      }
      return KX_OK;
    }
    case KX_T_SET: case KX_T_LIST: {                             /* :269-286 */
      if ((rc = skipn(s, 5))) return rc;
      const uint8_t* h = s->b + s->n - 5;
      uint8_t vt = h[0];
      int32_t n = (int32_t)be32(h + 1);
      if (n < 0) return KX_ERR_INVALID_DATA;
      int vs = type_size(vt);
      if (vs > 0) return skipn(s, (uint64_t)n * (uint64_t)vs);
      for (int32_t i = 0; i < n; i++)
        if ((rc = skip_type(s, vt, maxdepth - 1))) return rc;
      return KX_OK;
    }
    default:                                                     /* :287-290 unknown data type */
      return KX_ERR_INVALID_DATA;
  }
}

int kxo_skip(const uint8_t* b, size_t len, uint8_t ttype, int maxdepth, size_t* used) {
  skipper s = {b, len, 0};
  int rc = skip_type(&s, ttype, maxdepth);
  *used = s.n;
  return rc;
}

int kxo_skip_batch(const uint8_t* b, size_t len, uint64_t n, uint64_t* offsets_out, uint64_t* n_done) {
  size_t pos = 0;
  for (uint64_t i = 0; i < n; i++) {
    offsets_out[i] = pos;
    size_t u = 0;
    int rc = kxo_skip(b + pos, len - pos, KX_T_STRUCT, 64, &u);  /* SkipStruct, codec_apache.go:166-172 */
    if (rc) { *n_done = i; return rc; }
    pos += u;
  }
  offsets_out[n] = pos;
  *n_done = n;
  return KX_OK;
}

/* ------------------------------------------------------------------------------------------------
 * Framing sniff over a socket buffer of n messages: defaultCodec.DecodeMeta + checkPayload
 * (pkg/remote/codec/default_codec.go:189-221, 328-427), the Mesh header (header_codec.go:192-212,
 * readStrKVInfo :115-138) and the TTHeader meta / info blocks. TTHeader decoding itself lives in the
 * un-vendored github.com/cloudwego/gopkg v0.2.0 (protocol/ttheader); restated from its published
 * layout: u32 LENGTH (bytes after this field), u16 magic 0x1000, u16 flags, u32 seqid, u16 header
 * size in 4-byte words (2..65536 bytes), then protocol id (0 binary, 3 compact v2, 4 Kitex-PB),
 * transform count + ids, and info blocks (0x00 padding, 0x01 string KVs, 0x10 int KVs, 0x11 ACL
 * token). Parity unpinned beyond the reference's sniff-matrix tests (default_codec_test.go:58-199).
 *
 * Per frame: its extent, its payload [start, end) (what the payload codec sees: MessageBegin or the
 * Kitex-PB meta header first) and kind = transport.Protocol (0 PurePayload, 2 TTHeader, 4 Framed,
 * 6 TTHeaderFramed; transport/keys.go:24-53) | 0x10 Kitex-Protobuf | 0x20 Mesh header.
 * A payload longer than max_payload (> 0) is INVALID_DATA (checkPayloadSize, :429-434; a PurePayload
 * length is unknown at that point and never checked). A frame cut short is EOF.
 * ---------------------------------------------------------------------------------------------- */
#define KXO_MASK 0xffff0000u
static int kv_strings(const uint8_t* b, uint64_t len, uint64_t* i) { /* readStrKVInfo */
  if (*i + 2 > len) return KX_ERR_UNKNOWN_PROTOCOL;
  uint32_t k = be16(b + *i);
  *i += 2;
  for (uint32_t j = 0; j < 2 * k; j++) {  /* key, value: ReadString2BLen */
    if (*i + 2 > len) return KX_ERR_UNKNOWN_PROTOCOL;
    uint64_t l = be16(b + *i);
    if (*i + 2 + l > len) return KX_ERR_UNKNOWN_PROTOCOL;
    *i += 2 + l;
  }
  return KX_OK;
}

static int tth_info(const uint8_t* b, uint64_t len) {
  uint8_t proto = b[0];
  if (proto != 0 && proto != 3 && proto != 4) return KX_ERR_UNKNOWN_PROTOCOL;  /* checkProtocolID */
  uint64_t nt = b[1], i = 2;
  if (len - 2 < nt) return KX_ERR_UNKNOWN_PROTOCOL;  /* transform ids */
  i += nt;
  while (i < len) {
    uint8_t id = b[i++];
    if (id == 0x00) continue;  /* padding */
    int rc;
    if (id == 0x01) {
      rc = kv_strings(b, len, &i);
    } else if (id == 0x10) {  /* int KVs: u16 count, (u16 key, u16-length string) */
      if (i + 2 > len) return KX_ERR_UNKNOWN_PROTOCOL;
      uint32_t k = be16(b + i);
      i += 2;
      rc = KX_OK;
      for (uint32_t j = 0; j < k && !rc; j++) {
        if (i + 4 > len) { rc = KX_ERR_UNKNOWN_PROTOCOL; break; }
        uint64_t l = be16(b + i + 2);
        if (i + 4 + l > len) rc = KX_ERR_UNKNOWN_PROTOCOL;
        else i += 4 + l;
      }
    } else if (id == 0x11) {  /* ACL token: u16-length string */
      if (i + 2 > len) return KX_ERR_UNKNOWN_PROTOCOL;
      uint64_t l = be16(b + i);
      rc = i + 2 + l > len ? KX_ERR_UNKNOWN_PROTOCOL : KX_OK;
      i += 2 + l;
    } else {
      rc = KX_ERR_UNKNOWN_PROTOCOL;  /* invalid info id */
    }
    if (rc) return rc;
  }
  return KX_OK;
}

int kxo_frame_one(const uint8_t* b, uint64_t len, uint64_t max_payload, uint64_t* flen, uint64_t* ps,
                  uint64_t* pe, uint8_t* kind) {
  if (len < 8) return KX_ERR_EOF;  /* in.Peek(2 * Size32), :191 */
  uint32_t a = be32(b), c = be32(b + 4);
  uint64_t p = 0, fend = 0, plen = 0;
  int tth = 0, mesh = 0;
  if ((c & KXO_MASK) == 0x10000000u) {  /* IsTTHeader, :328-330 */
    tth = 1;
    if (len < 14) return KX_ERR_EOF;
    uint64_t hs = (uint64_t)be16(b + 12) * 4;
    if (hs > 65536 || hs < 2) return KX_ERR_UNKNOWN_PROTOCOL;
    if (14 + hs > len) return KX_ERR_EOF;
    int rc = tth_info(b + 14, hs);
    if (rc) return rc;
    fend = 4 + (uint64_t)a;
    if (fend < 14 + hs) return KX_ERR_UNKNOWN_PROTOCOL;  /* negative payload length */
    p = 14 + hs;
    plen = fend - p;  /* PayloadLen = LENGTH - header size + 4 - 14 */
  } else if ((a & KXO_MASK) == 0xFFAF0000u) {  /* isMeshHeader, :339-341 */
    mesh = 1;
    uint64_t hl = a & 0xffffu;
    if (4 + hl > len) return KX_ERR_EOF;
    uint64_t i = 0;
    int rc = kv_strings(b + 4, hl, &i);
    if (rc) return rc;
    p = 4 + hl;
  }
  const uint64_t avail = tth ? fend : len;
  if (tth && fend > len) return KX_ERR_EOF;
  if (p + 8 > avail) return KX_ERR_EOF;  /* Peek(8) of the payload, :202-204 / :216-218 */
  uint32_t x = be32(b + p), y = be32(b + p + 4);
  uint8_t k;
  if ((x & KXO_MASK) == 0x80010000u) {  /* isThriftBinary: TTHeader / PurePayload, :380-386 */
    k = tth ? 2 : 0;
    if (tth) {
      *ps = p; *pe = fend;
    } else {  /* the message delimits itself: MessageBegin + the struct after it */
      uint32_t no, nl; int32_t ty, sq; size_t u = 0, u2 = 0;
      int rc = kxo_read_message_begin(b + p, len - p, &no, &nl, &ty, &sq, &u);
      if (rc) return rc;
      rc = kxo_skip(b + p + u, len - p - u, KX_T_STRUCT, 64, &u2);
      if (rc) return rc;
      *ps = p; *pe = p + u + u2;
      fend = *pe;
      plen = 0;  /* unknown when checkPayloadSize runs */
    }
  } else if ((y & KXO_MASK) == 0x80010000u || (y & KXO_MASK) == 0x90010000u) {  /* Framed, :387-410 */
    k = (uint8_t)((tth ? 6 : 4) | ((y & KXO_MASK) == 0x90010000u ? 0x10 : 0));
    plen = x;
    if (tth) {
      if (p + 4 + plen > fend) return KX_ERR_EOF;
    } else {
      fend = p + 4 + plen;
      if (fend > len) return KX_ERR_EOF;
    }
    *ps = p + 4; *pe = p + 4 + plen;
  } else {
    return KX_ERR_UNKNOWN_PROTOCOL;  /* invalid payload, :411-416 */
  }
  if (max_payload && plen > max_payload) return KX_ERR_INVALID_DATA;  /* checkPayloadSize */
  *flen = fend;
  *kind = (uint8_t)(k | (mesh ? 0x20 : 0));
  return KX_OK;
}

/* ttstream DecodeFrame (pkg/remote/trans/ttstream/frame.go:137-185) of the frame at b: ttheader.Decode
 * (the same TTHeader layout as above; checkProtocolID also admits the streaming struct protocols 0x10
 * ThriftStruct / 0x11 ProtobufStruct), the streaming flag check (:143-145), IntInfo[frame type key] ->
 * frame type (:151-168; unknown -> error), IntInfo[ToMethod] (:169; readIntKVInfo: the last occurrence of
 * a key wins), the TTHeader seqid as the stream id (:170), payload = the PayloadLen bytes after the
 * header (:173-182). Keys / values of the un-vendored gopkg are the caller's (kx_ttstream_keys). */
static int tts_match(const uint8_t* v, uint64_t l, const char* name) {
  uint64_t nl = 0;
  while (nl < 8 && name[nl]) nl++;
  return nl == l && memcmp(v, name, l) == 0;
}

int kxo_ttstream_frame_one(const uint8_t* b, uint64_t len, const kx_ttstream_keys* keys, uint64_t* flen,
                           uint64_t* ps, uint64_t* pe, uint8_t* ftype, int32_t* sid, uint64_t* mpos,
                           uint32_t* mlen) {
  if (len < 8) return KX_ERR_EOF;
  uint32_t a = be32(b), c = be32(b + 4);
  if ((c & KXO_MASK) != 0x10000000u) return KX_ERR_UNKNOWN_PROTOCOL;  /* not a TTHeader */
  if (len < 14) return KX_ERR_EOF;
  uint64_t hs = (uint64_t)be16(b + 12) * 4;
  if (hs > 65536 || hs < 2) return KX_ERR_UNKNOWN_PROTOCOL;
  if (14 + hs > len) return KX_ERR_EOF;
  const uint8_t* h = b + 14;
  uint8_t proto = h[0];
  if (proto != 0 && proto != 3 && proto != 4 && proto != 0x10 && proto != 0x11) return KX_ERR_UNKNOWN_PROTOCOL;
  uint64_t nt = h[1], i = 2;
  if (hs - 2 < nt) return KX_ERR_UNKNOWN_PROTOCOL;
  i += nt;
  const uint8_t* ftv = NULL;
  uint64_t ftl = 0;
  *mpos = 0;
  *mlen = 0;
  while (i < hs) {
    uint8_t id = h[i++];
    if (id == 0x00) continue;
    if (id == 0x01) {
      int rc = kv_strings(h, hs, &i);
      if (rc) return rc;
    } else if (id == 0x10) {
      if (i + 2 > hs) return KX_ERR_UNKNOWN_PROTOCOL;
      uint32_t k = be16(h + i);
      i += 2;
      for (uint32_t j = 0; j < k; j++) {
        if (i + 4 > hs) return KX_ERR_UNKNOWN_PROTOCOL;
        uint32_t key = be16(h + i);
        uint64_t l = be16(h + i + 2);
        if (i + 4 + l > hs) return KX_ERR_UNKNOWN_PROTOCOL;
        if (key == keys->frame_type_key) { ftv = h + i + 4; ftl = l; }
        if (key == keys->to_method_key) { *mpos = 14 + i + 4; *mlen = (uint32_t)l; }
        i += 4 + l;
      }
    } else if (id == 0x11) {
      if (i + 2 > hs) return KX_ERR_UNKNOWN_PROTOCOL;
      uint64_t l = be16(h + i);
      if (i + 2 + l > hs) return KX_ERR_UNKNOWN_PROTOCOL;
      i += 2 + l;
    } else {
      return KX_ERR_UNKNOWN_PROTOCOL;
    }
  }
  uint64_t fend = 4 + (uint64_t)a;
  if (fend < 14 + hs) return KX_ERR_UNKNOWN_PROTOCOL;
  if ((c & 0xffffu & keys->streaming_flag) == 0) return KX_ERR_INVALID_DATA;  /* unexpected header flags */
  uint8_t t = 0;
  for (int k = 0; k < 5 && !t; k++)
    if (ftv && tts_match(ftv, ftl, keys->type_names[k])) t = (uint8_t)(k + 1);
  if (!t) return KX_ERR_INVALID_DATA;  /* unexpected frame type */
  if (fend > len) return KX_ERR_EOF;   /* reader.ReadBinary(payload) */
  *flen = fend;
  *ps = 14 + hs;
  *pe = fend;
  *ftype = t;
  *sid = (int32_t)be32(b + 8);
  return KX_OK;
}

int kxo_ttstream_frame_scan(const uint8_t* in, uint64_t in_len, uint64_t n, const kx_ttstream_keys* keys,
                            uint64_t* frame_offsets, uint64_t* pay_start, uint64_t* pay_end, uint8_t* ftypes,
                            int32_t* sids, uint64_t* mpos, uint32_t* mlen, uint64_t* n_done) {
  uint64_t pos = 0;
  for (uint64_t i = 0; i < n; i++) {
    frame_offsets[i] = pos;
    uint64_t fl = 0, ps = 0, pe = 0, mp = 0;
    uint32_t ml = 0;
    uint8_t t = 0;
    int32_t sd = 0;
    int rc = kxo_ttstream_frame_one(in + pos, in_len - pos, keys, &fl, &ps, &pe, &t, &sd, &mp, &ml);
    if (rc) { *n_done = i; return rc; }
    pay_start[i] = pos + ps; pay_end[i] = pos + pe; ftypes[i] = t; sids[i] = sd;
    mpos[i] = ml ? pos + mp : 0; mlen[i] = ml;
    pos += fl;
  }
  frame_offsets[n] = pos;
  *n_done = n;
  return KX_OK;
}

/* n frames back to back from in[0]; stops at the first failing frame (n_done = its index) */
int kxo_frame_scan(const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t max_payload, uint64_t* frame_offsets,
                   uint64_t* pay_start, uint64_t* pay_end, uint8_t* kinds, uint64_t* n_done) {
  uint64_t pos = 0;
  for (uint64_t i = 0; i < n; i++) {
    frame_offsets[i] = pos;
    uint64_t fl = 0, ps = 0, pe = 0;
    uint8_t k = 0;
    int rc = kxo_frame_one(in + pos, in_len - pos, max_payload, &fl, &ps, &pe, &k);
    if (rc) { *n_done = i; return rc; }
    pay_start[i] = pos + ps; pay_end[i] = pos + pe; kinds[i] = k;
    pos += fl;
  }
  frame_offsets[n] = pos;
  *n_done = n;
  return KX_OK;
}

/* Binary generic ingress (pkg/generic/binarythrift_codec.go). Unmarshal (:83-115): PeekUint32 &
 * FrontMask (0xffff, codec/util.go:31) == Exception -> the regular thrift path (APPLICATION_EXCEPTION
 * here); readBinaryMethod (:185-199): size >= 8, methodLen = u32 [4, 8), 0 < methodLen <= size - 8.
 * The seqid reported is the u32 after the name when present (GetSeqID's position, :137-175). */
int kxo_raw_messages(const uint8_t* in, uint64_t in_len, const uint64_t* offsets, uint64_t n, uint64_t* name_pos,
                     uint64_t* name_len, int32_t* msg_type, int32_t* seqid, uint8_t* rs) {
  int first = KX_OK;
  for (uint64_t i = 0; i < n; i++) {
    uint64_t p = offsets[i], e = offsets[i + 1];
    int rc = KX_OK;
    uint32_t ty = 0, sq = 0;
    uint64_t ml = 0;
    if (p > e || e > in_len) rc = KX_ERR_INVALID_ARG;
    else if (e - p < 4) rc = KX_ERR_EOF;
    else {
      ty = be32(in + p) & 0xffffu;
      if (ty == KX_MSG_EXCEPTION) rc = KX_ERR_APPLICATION_EXCEPTION;
      else if (e - p < 8) rc = KX_ERR_INVALID_DATA;
      else {
        ml = be32(in + p + 4);
        if (ml == 0 || ml > 0x7fffffffu || e - p - 8 < ml) rc = KX_ERR_INVALID_DATA;
        else if (e - p - 8 - ml >= 4) sq = be32(in + p + 8 + ml);
      }
    }
    if (rc) { ty = 0; sq = 0; ml = 0; }
    name_pos[i] = p + 8; name_len[i] = ml; msg_type[i] = (int32_t)ty; seqid[i] = (int32_t)sq; rs[i] = (uint8_t)rc;
    if (rc && !first) first = rc;
  }
  return first;
}

/* SetSeqID (:117-134) via getSeqID4Bytes (:147-175), in place */
int kxo_set_seqids(uint8_t* in, uint64_t in_len, const uint64_t* offsets, uint64_t n, const int32_t* seqids,
                   uint8_t* rs) {
  int first = KX_OK;
  for (uint64_t i = 0; i < n; i++) {
    uint64_t p = offsets[i], e = offsets[i + 1];
    int rc = KX_OK;
    if (p > e || e > in_len) rc = KX_ERR_INVALID_ARG;
    else if (e - p < 4) rc = KX_ERR_INVALID_DATA;
    else {
      int32_t f = (int32_t)be32(in + p);
      if (f > 0) rc = KX_ERR_INVALID_DATA;                            /* missing version */
      else if (((uint32_t)f & KXO_MASK) != 0x80010000u) rc = KX_ERR_BAD_VERSION;
      else if (e - p < 8) rc = KX_ERR_INVALID_DATA;
      else {
        int32_t nl = (int32_t)be32(in + p + 4);
        if (nl < 0 || e - p < 12ull + (uint64_t)nl) rc = KX_ERR_INVALID_DATA;
        else put32(in + p + 8 + nl, (uint32_t)seqids[i]);
      }
    }
    rs[i] = (uint8_t)rc;
    if (rc && !first) first = rc;
  }
  return first;
}

/* gRPC messages (decodeGRPCFrame, pkg/remote/codec/grpc/grpc_compress.go:37-60): in.Next(5) -> u8
 * compressed flag, u32 BE length; in.Next(dLen) -> payload (EOF when short). flags[i] = the flag byte.
 * max_payload > 0: a longer payload is INVALID_DATA. Stops at the first message that cannot be read. */
int kxo_grpc_frame_scan(const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t max_payload,
                        uint64_t* frame_offsets, uint64_t* pay_start, uint64_t* pay_end, uint8_t* flags,
                        uint64_t* n_done) {
  uint64_t pos = 0;
  for (uint64_t i = 0; i < n; i++) {
    frame_offsets[i] = pos;
    if (in_len - pos < 5) { *n_done = i; return KX_ERR_EOF; }
    uint64_t len = be32(in + pos + 1);
    if (len > in_len - pos - 5) { *n_done = i; return KX_ERR_EOF; }
    if (max_payload && len > max_payload) { *n_done = i; return KX_ERR_INVALID_DATA; }
    flags[i] = in[pos];
    pay_start[i] = pos + 5;
    pay_end[i] = pos + 5 + len;
    pos += 5 + len;
  }
  frame_offsets[n] = pos;
  *n_done = n;
  return KX_OK;
}

/* ------------------------------------------------------------------------------------------------
 * CRC32C payload validator: crcPayloadValidator (pkg/remote/codec/validate.go:168-217). getCRC32C
 * (:208-217) = crc32.Update(0, crc32.MakeTable(crc32.Castagnoli), payload), Go's hash/crc32 (standard
 * library, not in the reference tree): the reflected CRC-32 over polynomial 0x82F63B78, pre- and
 * post-inverted. Restated bit by bit (no tables) so that the device's slicing-by-8 tables and chunk
 * combination are checked against the definition; pinned by the RFC 3720 B.4 / "123456789" check
 * values in tests/test_oracle_crc.py. kxo_crc32c(crc, p, n) continues crc like crc32.Update.
 * ---------------------------------------------------------------------------------------------- */
uint32_t kxo_crc32c(uint32_t crc, const uint8_t* p, uint64_t n) {
  crc = ~crc;
  for (uint64_t i = 0; i < n; i++) {
    crc ^= p[i];
    for (int k = 0; k < 8; k++) crc = (crc & 1) ? (crc >> 1) ^ 0x82F63B78u : crc >> 1;
  }
  return ~crc;
}

/* Generate over n ranges [offsets[i], offsets[i+1]) (crcPayloadValidator.Generate, :187-189) */
int kxo_crc32c_batch(const uint8_t* in, uint64_t in_len, const uint64_t* offsets, uint64_t n, uint32_t* crc_out) {
  int rc = KX_OK;
  for (uint64_t i = 0; i < n; i++) {
    uint64_t a = offsets[i], b = offsets[i + 1];
    if (a > b || b > in_len) { crc_out[i] = 0; if (!rc) rc = KX_ERR_INVALID_ARG; continue; }
    crc_out[i] = kxo_crc32c(0, in + a, b - a);
  }
  return rc;
}

/* payloadChecksumValidate (:91-127) for one frame at b (DecodeMeta runs it right after the TTHeader,
 * default_codec.go:205-209): expectedValue = strInfo["crc32c"] (transmeta.HeaderCRC32C; the TTHeader
 * string-KV info, last pair wins like the map assignment), payload = PayloadLen bytes after the TTHeader
 * (the Framed length prefix included). Validate (:190-201): "" passes, else hex(BE crc) == value. */
static int frame_crc_one(const uint8_t* b, uint64_t len, uint32_t* crc) {
  *crc = 0;
  if (len < 14 || (be32(b + 4) & KXO_MASK) != 0x10000000u) return KX_OK;  /* not TTHeader: no validator */
  uint64_t flen = (uint64_t)be32(b) + 4, hs = (uint64_t)be16(b + 12) * 4;
  if (hs < 2 || 14 + hs > flen || flen > len) return KX_ERR_UNKNOWN_PROTOCOL;
  const uint8_t* info = b + 14;
  const uint8_t* want = NULL;
  uint64_t want_len = 0, i = 2 + (uint64_t)info[1];
  if (i > hs) return KX_ERR_UNKNOWN_PROTOCOL;
  while (i < hs) {
    uint8_t id = info[i++];
    if (id == 0x00) continue;
    if (id == 0x01) {
      if (i + 2 > hs) return KX_ERR_UNKNOWN_PROTOCOL;
      uint32_t k = be16(info + i);
      i += 2;
      for (uint32_t j = 0; j < k; j++) {
        if (i + 2 > hs) return KX_ERR_UNKNOWN_PROTOCOL;
        uint64_t kl = be16(info + i);
        if (i + 2 + kl + 2 > hs) return KX_ERR_UNKNOWN_PROTOCOL;
        const uint8_t* key = info + i + 2;
        i += 2 + kl;
        uint64_t vl = be16(info + i);
        if (i + 2 + vl > hs) return KX_ERR_UNKNOWN_PROTOCOL;
        if (kl == 6 && memcmp(key, "crc32c", 6) == 0) { want = info + i + 2; want_len = vl; }
        i += 2 + vl;
      }
    } else if (id == 0x10) {
      if (i + 2 > hs) return KX_ERR_UNKNOWN_PROTOCOL;
      uint32_t k = be16(info + i);
      i += 2;
      for (uint32_t j = 0; j < k; j++) {
        if (i + 4 > hs) return KX_ERR_UNKNOWN_PROTOCOL;
        uint64_t l = be16(info + i + 2);
        if (i + 4 + l > hs) return KX_ERR_UNKNOWN_PROTOCOL;
        i += 4 + l;
      }
    } else if (id == 0x11) {
      if (i + 2 > hs) return KX_ERR_UNKNOWN_PROTOCOL;
      uint64_t l = be16(info + i);
      if (i + 2 + l > hs) return KX_ERR_UNKNOWN_PROTOCOL;
      i += 2 + l;
    } else {
      return KX_ERR_UNKNOWN_PROTOCOL;
    }
  }
  *crc = kxo_crc32c(0, b + 14 + hs, flen - 14 - hs);
  if (!want || want_len == 0) return KX_OK;
  static const char hexd[] = "0123456789abcdef";
  char real[8];
  for (int q = 0; q < 8; q++) real[q] = hexd[(*crc >> (28 - 4 * q)) & 15];  /* hex.EncodeToString(BE) */
  return want_len == 8 && memcmp(real, want, 8) == 0 ? KX_OK : KX_ERR_PAYLOAD_VALIDATION;
}

int kxo_frame_crc32c_validate(const uint8_t* in, uint64_t in_len, const uint64_t* frame_offsets, uint64_t n,
                              uint32_t* crc_out, uint8_t* record_status, uint64_t* first_bad) {
  int first = KX_OK;
  *first_bad = n;
  for (uint64_t i = 0; i < n; i++) {
    uint64_t f = frame_offsets[i];
    uint32_t crc = 0;
    int rc = f > in_len ? KX_OK : frame_crc_one(in + f, in_len - f, &crc);
    if (crc_out) crc_out[i] = rc == KX_ERR_UNKNOWN_PROTOCOL ? 0 : crc;
    if (record_status) record_status[i] = (uint8_t)rc;
    if (rc && !first) { first = rc; *first_bad = i; }
  }
  return first;
}

/* ------------------------------------------------------------------------------------------------
 * Schema flattening: depth-first over the IDL, struct fields inlined, a presence bit for every
 * optional / struct / container field (Go represents those as nil-able; struct_tpl.go:405-450).
 * ---------------------------------------------------------------------------------------------- */
#define MAXF 64
#define MAXINST 32
typedef struct { int col; int inst; int pbit; } fmap_t;
typedef struct { int sidx; fmap_t fm[MAXF]; } inst_t;
typedef struct {
  const kx_struct_desc* structs;
  uint32_t nstructs;
  inst_t inst[MAXINST];
  int ninst;
  kx_column_info cols[KX_MAX_COLUMNS];
  uint32_t ncols, npres;
  int nvar;
  int varidx[KX_MAX_COLUMNS]; /* column -> var slot (elements / bytes), -1 for fixed */
  int varidx2[KX_MAX_COLUMNS]; /* LIST_BYTES column -> its bytes slot, else -1 */
  uint8_t mside[KX_MAX_COLUMNS]; /* 1: map key column, 2: map value column, 0: neither */
  uint8_t mkt[KX_MAX_COLUMNS], mvt[KX_MAX_COLUMNS]; /* map key / value types (map columns) */
  uint8_t sside[KX_MAX_COLUMNS];  /* list<struct> element field column: 1 + index of the field in S */
  const kx_struct_desc* ssd[KX_MAX_COLUMNS];  /* ... and S */
  int is_pb;
} plan_t;

static int flatten_rec(plan_t* p, int sidx, int depth, int16_t* path, int* stack, int* out_inst) {
  if (sidx < 0 || (uint32_t)sidx >= p->nstructs) return KX_ERR_INVALID_ARG;
  if (depth >= 8) return KX_ERR_NOT_IMPLEMENTED;
  for (int i = 0; i < depth; i++) if (stack[i] == sidx) return KX_ERR_NOT_IMPLEMENTED; /* recursive type */
  if (p->ninst >= MAXINST) return KX_ERR_NOT_IMPLEMENTED;
  const kx_struct_desc* sd = &p->structs[sidx];
  if (sd->nfields > MAXF) return KX_ERR_NOT_IMPLEMENTED;
  int me = p->ninst++;
  p->inst[me].sidx = sidx;
  stack[depth] = sidx;
  for (uint32_t i = 0; i < sd->nfields; i++) {
    const kx_field_desc* f = &sd->fields[i];
    fmap_t* m = &p->inst[me].fm[i];
    m->col = -1; m->inst = -1; m->pbit = -1;
    for (uint32_t j = 0; j < i; j++) if (sd->fields[j].id == f->id) return KX_ERR_INVALID_ARG;
    int container = f->ttype == KX_T_STRUCT || f->ttype == KX_T_LIST || f->ttype == KX_T_SET || f->ttype == KX_T_MAP;
    if (f->req > KX_REQ_OPTIONAL) return KX_ERR_INVALID_ARG;
    if (f->req == KX_REQ_OPTIONAL || container) {
      if (p->npres >= 64) return KX_ERR_NOT_IMPLEMENTED;
      m->pbit = (int)p->npres++;
    }
    path[depth] = f->id;
    kx_column_info ci;
    memset(&ci, 0, sizeof ci);
    ci.ttype = f->ttype; ci.field_id = f->id; ci.presence_bit = m->pbit; ci.depth = (uint32_t)depth;
    for (int d = 0; d <= depth; d++) ci.path[d] = path[d];
    switch (f->ttype) {
      case KX_T_BOOL: case KX_T_BYTE: case KX_T_I16: case KX_T_I32: case KX_T_I64: case KX_T_DOUBLE:
        ci.kind = KX_COL_FIXED; ci.width = (uint32_t)type_size(f->ttype); break;
      case KX_T_STRING:
        if ((f->reserved0 & KX_FIELD_STRING_DEFAULT) && f->default_bits && *(const char*)(intptr_t)f->default_bits)
          return KX_ERR_NOT_IMPLEMENTED;                   /* a string default: nested */
        ci.kind = KX_COL_BYTES; ci.width = 1; break;
      case KX_T_LIST: case KX_T_SET:
        if (f->elem_ttype == KX_T_STRING) {                /* list/set<string>: FieldFastReadList (:582-625) */
          ci.kind = KX_COL_LIST_BYTES; ci.width = 1; ci.elem_ttype = KX_T_STRING; break;
        }
        if (f->elem_ttype == KX_T_STRUCT) {                /* list/set<S>: one LIST column per field of S */
          if (f->child < 0 || (uint32_t)f->child >= p->nstructs || depth + 1 >= 8) return KX_ERR_NOT_IMPLEMENTED;
          const kx_struct_desc* es = &p->structs[f->child];
          if (es->nfields == 0 || es->nfields > 8 || p->ncols + es->nfields > KX_MAX_COLUMNS)
            return KX_ERR_NOT_IMPLEMENTED;
          for (uint32_t k = 0; k < es->nfields; k++) {
            const kx_field_desc* g = &es->fields[k];
            for (uint32_t j = 0; j < k; j++) if (es->fields[j].id == g->id) return KX_ERR_INVALID_ARG;
            if (type_size(g->ttype) == 0 || g->req == KX_REQ_OPTIONAL) return KX_ERR_NOT_IMPLEMENTED;
            if (g->req > KX_REQ_OPTIONAL) return KX_ERR_INVALID_ARG;
          }
          m->col = (int)p->ncols;
          for (uint32_t k = 0; k < es->nfields; k++) {
            const kx_field_desc* g = &es->fields[k];
            kx_column_info cs = ci;
            cs.kind = KX_COL_LIST; cs.width = (uint32_t)type_size(g->ttype);
            cs.elem_ttype = (uint8_t)(g->ttype | KX_ELEM_STRUCT_FIELD);
            cs.field_id = g->id; cs.depth = (uint32_t)depth + 1; cs.path[depth + 1] = g->id;
            p->sside[p->ncols] = (uint8_t)(1 + k); p->ssd[p->ncols] = es;
            p->cols[p->ncols++] = cs;
          }
          continue;
        }
        if (type_size(f->elem_ttype) == 0) return KX_ERR_NOT_IMPLEMENTED;  /* list<container> */
        ci.kind = KX_COL_LIST; ci.width = (uint32_t)type_size(f->elem_ttype); ci.elem_ttype = f->elem_ttype; break;
      case KX_T_MAP: {                                     /* FieldFastReadMap (:466-533): keys, values columns */
        const uint8_t kt = f->elem_ttype & 15, vt = (uint8_t)(f->elem_ttype >> 4);
        if ((type_size(kt) == 0 && kt != KX_T_STRING) || (type_size(vt) == 0 && vt != KX_T_STRING))
          return KX_ERR_NOT_IMPLEMENTED;                   /* map<.., struct|container> */
        if (p->ncols + 2 > KX_MAX_COLUMNS) return KX_ERR_NOT_IMPLEMENTED;
        m->col = (int)p->ncols;
        for (int side = 0; side < 2; side++) {
          const uint8_t t = side ? vt : kt;
          kx_column_info cm = ci;
          cm.kind = t == KX_T_STRING ? KX_COL_LIST_BYTES : KX_COL_LIST;
          cm.width = t == KX_T_STRING ? 1u : (uint32_t)type_size(t);
          cm.elem_ttype = (uint8_t)(t | (side ? KX_ELEM_MAP_VALUE : 0));
          p->mside[p->ncols] = (uint8_t)(1 + side); p->mkt[p->ncols] = kt; p->mvt[p->ncols] = vt;
          p->cols[p->ncols++] = cm;
        }
        continue;
      }
      case KX_T_STRUCT: {
        int child = -1;
        int rc = flatten_rec(p, f->child, depth + 1, path, stack, &child);
        if (rc) return rc;
        m->inst = child;
        continue;
      }
      default: return KX_ERR_INVALID_ARG;
    }
    if (p->ncols >= KX_MAX_COLUMNS) return KX_ERR_NOT_IMPLEMENTED;
    m->col = (int)p->ncols;
    p->cols[p->ncols++] = ci;
  }
  *out_inst = me;
  return KX_OK;
}

static int plan_build(plan_t* p, const kx_struct_desc* structs, uint32_t nstructs) {
  memset(p, 0, sizeof *p);
  if (!structs || nstructs == 0 || nstructs > KX_MAX_STRUCTS) return KX_ERR_INVALID_ARG;
  p->structs = structs; p->nstructs = nstructs;
  int16_t path[8]; int stack[8]; int root = -1;
  int rc = flatten_rec(p, 0, 0, path, stack, &root);
  if (rc) return rc;
  /* the flat model's limits (the library's kx_program.h): beyond them a schema is nested */
  int nfields = 0;
  for (int i = 0; i < p->ninst; i++) nfields += (int)p->structs[p->inst[i].sidx].nfields;
  if (p->ncols > 32 || p->ninst > 16 || nfields > 64) return KX_ERR_NOT_IMPLEMENTED;
  p->nvar = 0;
  for (uint32_t c = 0; c < p->ncols; c++) {  /* var slots in column order; LIST_BYTES: elements, bytes */
    p->varidx[c] = p->cols[c].kind == KX_COL_FIXED ? -1 : p->nvar++;
    p->varidx2[c] = p->cols[c].kind == KX_COL_LIST_BYTES ? p->nvar++ : -1;
  }
  if (p->nvar > 16) return KX_ERR_NOT_IMPLEMENTED;   /* KXP_NV_MAX */
  return KX_OK;
}

/* a Kitex-Protobuf schema the flat proto path does not read (the layout rule of include/kxcodec.h,
 * KX_STRUCT_PROTOBUF): anything but one flat message of natural-kind scalars and strings */
static int pb_nested(const kx_struct_desc* structs, uint32_t nstructs) {
  if (!structs || nstructs == 0 || !(structs[0].reserved0 & KX_STRUCT_PROTOBUF)) return 0;
  if (nstructs != 1) return 1;
  int nstr = 0;
  for (uint32_t i = 0; i < structs[0].nfields; i++) {
    const kx_field_desc* f = &structs[0].fields[i];
    const int t = f->ttype;
    if (!(t == KX_T_BOOL || t == KX_T_I32 || t == KX_T_I64 || t == KX_T_DOUBLE || t == KX_T_STRING)) return 1;
    if ((f->default_bits & 0xffff) != 0 || f->req == KX_REQ_REQUIRED) return 1;
    nstr += t == KX_T_STRING;
  }
  return nstr > 8;   /* the library's flat proto path stops at 8 strings (kx_capi.cpp pb_flat_ok) */
}

int kxo_is_nested(const kx_struct_desc* structs, uint32_t nstructs) {
  if (pb_nested(structs, nstructs)) return 1;
  plan_t* p = (plan_t*)malloc(sizeof(plan_t));
  const int rc = plan_build(p, structs, nstructs);
  free(p);
  return rc == KX_ERR_NOT_IMPLEMENTED;
}

int kxo_flatten(const kx_struct_desc* structs, uint32_t nstructs, kx_column_info* cols,
                uint32_t* ncols, uint32_t* npresence) {
  if (pb_nested(structs, nstructs)) return kxo_nflatten(structs, nstructs, cols, ncols, npresence);
  plan_t* p = (plan_t*)malloc(sizeof(plan_t));
  int rc = plan_build(p, structs, nstructs);
  if (!rc) {
    memcpy(cols, p->cols, sizeof(kx_column_info) * p->ncols);
    *ncols = p->ncols; *npresence = p->npres;
  }
  free(p);
  if (rc == KX_ERR_NOT_IMPLEMENTED) return kxo_nflatten(structs, nstructs, cols, ncols, npresence);
  return rc;
}

/* ------------------------------------------------------------------------------------------------
 * Generated FastRead (struct_tpl.go:41-149 field loop; :425-450 base types; :582-625 lists;
 * :405-422 nested struct = NewX() + FastRead, so a repeated struct field replaces the old value).
 * Var-length fields are buffered per record and emitted when the root record ends, so that a
 * repeated field id keeps only its last occurrence (Go assigns p.Field = _field each time).
 * ---------------------------------------------------------------------------------------------- */
typedef struct {
  const plan_t* p;
  const kx_columns* out;
  uint64_t rec;
  int emit;
  uint64_t presence;
  const uint8_t* in0;               /* start of the call's input (KX_COLF_VIEW offsets) */
  const uint8_t* vptr[KX_MAX_COLUMNS];
  uint64_t vlen[KX_MAX_COLUMNS];    /* bytes / elements */
  uint64_t vbytes[KX_MAX_COLUMNS];  /* LIST_BYTES: payload bytes of the elements */
} dec_t;

static void store_fixed(const dec_t* d, int col, uint64_t v) {
  if (!d->emit) return;
  uint32_t w = d->p->cols[col].width;
  uint8_t* dst = (uint8_t*)d->out->cols[col].data + d->rec * w;
  switch (w) { /* host little-endian */
    case 1: *dst = (uint8_t)v; break;
    case 2: { uint16_t x = (uint16_t)v; memcpy(dst, &x, 2); break; }
    case 4: { uint32_t x = (uint32_t)v; memcpy(dst, &x, 4); break; }
    default: memcpy(dst, &v, 8); break;
  }
}

static void set_defaults(dec_t* d, int inst) {
  const inst_t* in = &d->p->inst[inst];
  const kx_struct_desc* sd = &d->p->structs[in->sidx];
  for (uint32_t i = 0; i < sd->nfields; i++) {
    const fmap_t* m = &in->fm[i];
    if (m->pbit >= 0) d->presence &= ~(1ull << m->pbit);
    if (m->inst >= 0) { set_defaults(d, m->inst); continue; }
    if (d->p->cols[m->col].kind == KX_COL_FIXED) store_fixed(d, m->col, (uint64_t)sd->fields[i].default_bits);
    else {
      const kx_field_desc* f = &sd->fields[i];
      const int nc = f->ttype == KX_T_MAP ? 2
                   : (f->ttype == KX_T_LIST || f->ttype == KX_T_SET) && f->elem_ttype == KX_T_STRUCT
                     ? (int)d->p->structs[f->child].nfields : 1;
      for (int k = 0; k < nc; k++) { d->vptr[m->col + k] = NULL; d->vlen[m->col + k] = 0; d->vbytes[m->col + k] = 0; }
    }
  }
}

static int find_field(const kx_struct_desc* sd, int16_t id) {
  for (uint32_t i = 0; i < sd->nfields; i++) if (sd->fields[i].id == id) return (int)i;
  return -1;
}

/* one scalar in host order from big-endian wire bytes; BOOL is `b == 1` (parity unpinned) */
static uint64_t read_scalar(uint8_t t, const uint8_t* b) {
  switch (t) {
    case KX_T_BOOL: return b[0] == 1;
    case KX_T_BYTE: return b[0];
    case KX_T_I16: return be16(b);
    case KX_T_I32: return be32(b);
    default: return be64(b);
  }
}

/* One element of a list<S> (S: fixed-width scalar fields): S's FastRead (struct_tpl.go:41-149) over
 * [b, b + len): fields until STOP, unknown / mistyped ids skipped, the last duplicate wins, required
 * fields checked. want >= 0: *val = the value of S's field `want`, or its default when absent. */
static int read_elem_struct(const kx_struct_desc* es, const uint8_t* b, size_t len, size_t* used, int want,
                            uint64_t* val) {
  uint64_t isset = 0;
  size_t off = 0;
  if (want >= 0) *val = (uint64_t)es->fields[want].default_bits;
  for (;;) {
    if (len - off < 1) return KX_ERR_EOF;
    uint8_t t = b[off];
    if (t == KX_T_STOP) { off += 1; break; }
    if (len - off < 3) return KX_ERR_EOF;
    int16_t id = (int16_t)be16(b + off + 1);
    off += 3;
    int fi = find_field(es, id);
    if (fi < 0 || es->fields[fi].ttype != t) {
      size_t u = 0;
      int rc = kxo_skip(b + off, len - off, t, 64, &u);
      if (rc) return rc;
      off += u;
      continue;
    }
    size_t w = (size_t)type_size(t);
    if (len - off < w) return KX_ERR_EOF;
    if (fi == want) *val = read_scalar(t, b + off);
    off += w;
    isset |= 1ull << fi;
  }
  for (uint32_t i = 0; i < es->nfields; i++)
    if (es->fields[i].req == KX_REQ_REQUIRED && !(isset & (1ull << i))) return KX_ERR_INVALID_DATA;
  *used = off;
  return KX_OK;
}

static int read_struct(dec_t* d, int inst, const uint8_t* b, size_t len, size_t* used) {
  const inst_t* in = &d->p->inst[inst];
  const kx_struct_desc* sd = &d->p->structs[in->sidx];
  set_defaults(d, inst);                                   /* NewX() / InitDefault */
  uint64_t isset = 0;
  size_t off = 0;
  for (;;) {
    if (len - off < 1) return KX_ERR_EOF;                  /* ReadFieldBegin */
    uint8_t t = b[off];
    if (t == KX_T_STOP) { off += 1; break; }
    if (len - off < 3) return KX_ERR_EOF;
    int16_t id = (int16_t)be16(b + off + 1);
    off += 3;
    int fi = find_field(sd, id);
    if (fi < 0 || sd->fields[fi].ttype != t) {             /* default: / type mismatch -> Skip */
      size_t u = 0;
      int rc = kxo_skip(b + off, len - off, t, 64, &u);
      if (rc) return rc;
      off += u;
      continue;
    }
    const kx_field_desc* f = &sd->fields[fi];
    const fmap_t* m = &in->fm[fi];
    const uint8_t* v = b + off;
    size_t rem = len - off;
    switch (t) {
      case KX_T_BOOL: case KX_T_BYTE: case KX_T_I16: case KX_T_I32: case KX_T_I64: case KX_T_DOUBLE: {
        size_t w = (size_t)type_size(t);
        if (rem < w) return KX_ERR_EOF;
        store_fixed(d, m->col, read_scalar(t, v));
        off += w;
        break;
      }
      case KX_T_STRING: {                                  /* ReadString: copy */
        if (rem < 4) return KX_ERR_EOF;
        int32_t n = (int32_t)be32(v);
        if (n < 0) return KX_ERR_NEGATIVE_SIZE;
        if ((uint64_t)rem < 4 + (uint64_t)n) return KX_ERR_EOF;
        d->vptr[m->col] = v + 4; d->vlen[m->col] = (uint64_t)n;
        off += 4 + (size_t)n;
        break;
      }
      case KX_T_LIST: case KX_T_SET: {                     /* ReadListBegin; elem type ignored (:587) */
        if (rem < 5) return KX_ERR_EOF;
        int32_t n = (int32_t)be32(v + 1);
        if (n < 0) return KX_ERR_NEGATIVE_SIZE;
        if (f->elem_ttype == KX_T_STRUCT) {                /* n x S.FastRead (FieldFastReadList :583-625) */
          const kx_struct_desc* es = &d->p->structs[f->child];
          size_t q = 5;
          for (int32_t j = 0; j < n; j++) {
            size_t u = 0;
            uint64_t dummy;
            int rc = read_elem_struct(es, v + q, rem - q, &u, -1, &dummy);
            if (rc) return rc;
            q += u;
          }
          for (uint32_t k = 0; k < es->nfields; k++) {
            d->vptr[m->col + k] = v + 5; d->vlen[m->col + k] = (uint64_t)n; d->vbytes[m->col + k] = 0;
          }
          off += q;
          break;
        }
        if (f->elem_ttype == KX_T_STRING) {                /* n x ReadString */
          size_t q = 5;
          uint64_t bytes = 0;
          for (int32_t j = 0; j < n; j++) {
            if (rem - q < 4) return KX_ERR_EOF;
            int32_t l = (int32_t)be32(v + q);
            if (l < 0) return KX_ERR_NEGATIVE_SIZE;
            if ((uint64_t)(rem - q - 4) < (uint64_t)l) return KX_ERR_EOF;
            bytes += (uint64_t)l;
            q += 4 + (size_t)l;
          }
          d->vptr[m->col] = v + 5; d->vlen[m->col] = (uint64_t)n; d->vbytes[m->col] = bytes;
          off += q;
          break;
        }
        uint64_t w = (uint64_t)type_size(f->elem_ttype);
        if ((uint64_t)rem < 5 + (uint64_t)n * w) return KX_ERR_EOF;
        d->vptr[m->col] = v + 5; d->vlen[m->col] = (uint64_t)n;
        off += 5 + (size_t)((uint64_t)n * w);
        break;
      }
      case KX_T_MAP: {                                     /* ReadMapBegin; key/value types ignored */
        if (rem < 6) return KX_ERR_EOF;
        int32_t n = (int32_t)be32(v + 2);
        if (n < 0) return KX_ERR_NEGATIVE_SIZE;
        const uint8_t kt = f->elem_ttype & 15, vt = (uint8_t)(f->elem_ttype >> 4);
        size_t q = 6;
        uint64_t kb = 0, vb = 0;
        for (int32_t j = 0; j < n; j++) {
          for (int side = 0; side < 2; side++) {
            const uint8_t t = side ? vt : kt;
            if (t == KX_T_STRING) {
              if (rem - q < 4) return KX_ERR_EOF;
              int32_t l = (int32_t)be32(v + q);
              if (l < 0) return KX_ERR_NEGATIVE_SIZE;
              if ((uint64_t)(rem - q - 4) < (uint64_t)l) return KX_ERR_EOF;
              if (side) vb += (uint64_t)l; else kb += (uint64_t)l;
              q += 4 + (size_t)l;
            } else {
              const size_t w = (size_t)type_size(t);
              if (rem - q < w) return KX_ERR_EOF;
              q += w;
            }
          }
        }
        d->vptr[m->col] = d->vptr[m->col + 1] = v + 6;
        d->vlen[m->col] = d->vlen[m->col + 1] = (uint64_t)n;
        d->vbytes[m->col] = kb; d->vbytes[m->col + 1] = vb;
        off += q;
        break;
      }
      case KX_T_STRUCT: {
        size_t u = 0;
        int rc = read_struct(d, m->inst, v, rem, &u);
        if (rc) return rc;
        off += u;
        break;
      }
      default: return KX_ERR_INVALID_DATA;
    }
    if (m->pbit >= 0) d->presence |= 1ull << m->pbit;
    isset |= 1ull << fi;
  }
  for (uint32_t i = 0; i < sd->nfields; i++)               /* RequiredFieldNotSetError (:124-145) */
    if (sd->fields[i].req == KX_REQ_REQUIRED && !(isset & (1ull << i))) return KX_ERR_INVALID_DATA;
  *used = off;
  return KX_OK;
}

/* One element of wire type t at q: its payload (a string's bytes, a scalar's wire bytes). */
static const uint8_t* elem_at(const uint8_t* q, uint8_t t, const uint8_t** data, uint64_t* len) {
  if (t == KX_T_STRING) { *len = be32(q); *data = q + 4; return q + 4 + *len; }
  *len = (uint64_t)type_size(t); *data = q; return q + *len;
}

/* A list<string> / set<string> column or one side of a map: record offsets in elements, element
 * byte offsets (LIST_BYTES) or host-order scalars (a map's fixed side), cursors per slot. */
static void emit_container(dec_t* d, uint32_t c, uint64_t* cursor, int* overflow) {
  const plan_t* p = d->p;
  const kx_column* col = &d->out->cols[c];
  const int vs = p->varidx[c], vs2 = p->varidx2[c];
  const uint64_t n = d->vlen[c], nb = vs2 >= 0 ? d->vbytes[c] : 0;
  const uint64_t E = cursor[vs], B = vs2 >= 0 ? cursor[vs2] : 0;
  const int lb = p->cols[c].kind == KX_COL_LIST_BYTES;
  const int fits = lb ? (E + n <= elem_lim(col) && B + nb <= arena_lim(col)) : E + n <= arena_lim(col);
  if (d->emit && fits) {
    off_set(col, d->rec, E);
    const uint8_t* q = d->vptr[c];
    uint64_t acc = 0;
    for (uint64_t j = 0; j < n; j++) {
      const uint8_t *kd, *vd, *x;
      uint64_t kl, vl, xl;
      if (p->sside[c]) {  /* list<S>: this column's field of element j, or its default */
        size_t u = 0;
        uint64_t v = 0;
        (void)read_elem_struct(p->ssd[c], q, (size_t)-1 / 2, &u, p->sside[c] - 1, &v);  /* validated */
        q += u;
        const uint32_t w = p->cols[c].width;
        memcpy((uint8_t*)col->data + (E + j) * w, &v, w);
        continue;
      }
      if (p->mside[c]) {
        q = elem_at(q, p->mkt[c], &kd, &kl);
        q = elem_at(q, p->mvt[c], &vd, &vl);
        x = p->mside[c] == 1 ? kd : vd;
        xl = p->mside[c] == 1 ? kl : vl;
      } else {
        q = elem_at(q, KX_T_STRING, &x, &xl);
      }
      if (lb) {
        eoff_set(col, E + j, B + acc);
        if (xl) memcpy((uint8_t*)col->data + B + acc, x, xl);
        acc += xl;
      } else {
        const uint32_t w = p->cols[c].width;
        uint64_t v = read_scalar(p->cols[c].elem_ttype & 15, x);
        memcpy((uint8_t*)col->data + (E + j) * w, &v, w);
      }
    }
  } else if (!fits) {
    *overflow = 1;
  }
  cursor[vs] += n;
  if (vs2 >= 0) cursor[vs2] += nb;
}

/* Emit buffered var fields + presence for record d->rec. cursors: arena cursor per var slot. */
static int emit_record_tail(dec_t* d, uint64_t* cursor, int* overflow) {
  const plan_t* p = d->p;
  for (uint32_t c = 0; c < p->ncols; c++) {
    int vs = p->varidx[c];
    if (vs < 0) continue;
    const kx_column* col = &d->out->cols[c];
    uint64_t n = d->vlen[c];
    if (p->cols[c].kind == KX_COL_LIST_BYTES || p->mside[c] || p->sside[c]) {  /* element by element */
      emit_container(d, c, cursor, overflow);
      continue;
    }
    if (col->flags & KX_COLF_VIEW) {  /* zero-copy view: (offset into the input, length), empty -> (0, 0) */
      if (d->emit) {
        const uint64_t o = n ? (uint64_t)(d->vptr[c] - d->in0) : 0;
        if (col->offset_bytes == 8) {
          ((uint64_t*)col->offsets)[2 * d->rec] = o;
          ((uint64_t*)col->offsets)[2 * d->rec + 1] = n;
        } else {
          ((uint32_t*)col->offsets)[2 * d->rec] = (uint32_t)o;
          ((uint32_t*)col->offsets)[2 * d->rec + 1] = (uint32_t)n;
        }
      }
      cursor[vs] += n;
      continue;
    }
    const uint64_t lim = arena_lim(col);
    if (d->emit && cursor[vs] + n <= lim) {
      off_set(col, d->rec, cursor[vs]);
      if (p->cols[c].kind == KX_COL_BYTES) {
        if (n) memcpy((uint8_t*)col->data + cursor[vs], d->vptr[c], n);
      } else {
        uint32_t w = p->cols[c].width;
        uint8_t et = p->cols[c].elem_ttype;
        uint8_t* dst = (uint8_t*)col->data + cursor[vs] * w;
        for (uint64_t i = 0; i < n; i++) {
          uint64_t x = read_scalar(et, d->vptr[c] + i * w);
          memcpy(dst + i * w, &x, w);
        }
      }
    } else if (cursor[vs] + n > lim) {
      *overflow = 1;
    }
    cursor[vs] += n;
  }
  if (d->emit && d->out->presence) d->out->presence[d->rec] = d->presence;
  return KX_OK;
}

static int check_out(const plan_t* p, const kx_columns* out) {
  if (!out || out->ncols != p->ncols) return KX_ERR_INVALID_ARG;
  if (p->npres && !out->presence) return KX_ERR_INVALID_ARG;
  for (uint32_t c = 0; c < p->ncols; c++) {
    if (!out->cols[c].data && p->cols[c].kind == KX_COL_FIXED) return KX_ERR_INVALID_ARG;
    if (p->cols[c].kind != KX_COL_FIXED && !out->cols[c].offsets) return KX_ERR_INVALID_ARG;
    if (p->cols[c].kind == KX_COL_LIST_BYTES && !out->cols[c].elem_offsets) return KX_ERR_INVALID_ARG;
  }
  return KX_OK;
}

/* decode records [r0, r1) (offsets mode) or n consecutive records from `start` (offsets == NULL) */
typedef int (*rec_reader)(dec_t* d, const uint8_t* b, size_t len, size_t* used);

static int thrift_reader(dec_t* d, const uint8_t* b, size_t len, size_t* used) {
  return read_struct(d, 0, b, len, used);
}

static int decode_range(const plan_t* p, rec_reader rd, const uint8_t* in, uint64_t in_len,
                        const uint64_t* offsets, uint64_t r0, uint64_t r1, uint64_t start,
                        const kx_columns* out, uint8_t* record_status, kx_status* st,
                        uint64_t* cursor, int emit, int* overflow) {
  dec_t d;
  memset(&d, 0, sizeof d);
  d.p = p; d.out = out; d.emit = emit; d.in0 = in;
  uint64_t pos = start;
  for (uint64_t r = r0; r < r1; r++) {
    d.rec = r;
    const uint8_t* b; size_t len;
    if (offsets) {
      if (offsets[r] > offsets[r + 1] || offsets[r + 1] > in_len) return KX_ERR_INVALID_ARG;
      b = in + offsets[r]; len = (size_t)(offsets[r + 1] - offsets[r]);
    } else {
      b = in + pos; len = (size_t)(in_len - pos);
    }
    size_t used = 0;
    d.presence = 0;
    int rc = rd(&d, b, len, &used);
    if (rc) {
      if (record_status) record_status[r] = (uint8_t)rc;
      if (st && (st->code == 0 || r < st->record)) {
        st->code = rc; st->record = r; st->offset = offsets ? offsets[r] : pos;
      }
      /* a failing record decodes to defaults */
      d.presence = 0;
      set_defaults(&d, 0);
      emit_record_tail(&d, cursor, overflow);
      if (!offsets) { if (st) { st->n_records = r; st->consumed = pos; } return rc; }
      continue;
    }
    if (record_status) record_status[r] = 0;
    emit_record_tail(&d, cursor, overflow);
    pos += used;
  }
  if (!offsets && st) { st->n_records = r1; st->consumed = pos; }
  return KX_OK;
}

static void finish_status(const plan_t* p, const kx_columns* out, kx_status* st, const uint64_t* cursor,
                          uint64_t n_rec, int overflow) {
  int k = 0;
  for (uint32_t c = 0; c < p->ncols; c++) {
    int vs = p->varidx[c], vs2 = p->varidx2[c];
    if (vs < 0) continue;
    const kx_column* col = &out->cols[c];
    if (col->offsets && !(col->flags & KX_COLF_VIEW)) {
      const uint64_t lim = vs2 >= 0 ? elem_lim(col) : arena_lim(col);
      if (cursor[vs] <= lim) off_set(col, n_rec, cursor[vs]);
      else overflow = 1;
    }
    if (vs2 >= 0 && col->elem_offsets) {  /* elem_offsets[elements] closes the byte arena */
      if (cursor[vs] <= elem_lim(col) && cursor[vs2] <= arena_lim(col)) eoff_set(col, cursor[vs], cursor[vs2]);
      else overflow = 1;
    }
    if (k < 16) st->var_total[k++] = cursor[vs];
    if (vs2 >= 0 && k < 16) st->var_total[k++] = cursor[vs2];
  }
  if (overflow && st->code == 0) st->code = KX_ERR_SIZE_LIMIT;
}

static int decode_common(const kx_struct_desc* structs, uint32_t nstructs, rec_reader rd, int is_pb,
                         const uint8_t* in, uint64_t in_len, const uint64_t* offsets, uint64_t n,
                         const kx_columns* out, uint8_t* record_status, kx_status* st) {
  plan_t* p = (plan_t*)malloc(sizeof(plan_t));
  int rc = plan_build(p, structs, nstructs);
  if (!rc) rc = check_out(p, out);
  if (rc) { free(p); return rc; }
  p->is_pb = is_pb;
  memset(st, 0, sizeof *st);
  uint64_t cursor[KX_MAX_COLUMNS] = {0};
  int overflow = 0;
  rc = decode_range(p, rd, in, in_len, offsets, 0, n, 0, out, record_status, st, cursor, 1, &overflow);
  if (rc == KX_ERR_INVALID_ARG) { free(p); return rc; }
  uint64_t n_rec = offsets ? n : st->n_records;
  if (offsets) st->n_records = n;
  /* concatenated mode stops at the failing record: offsets[n_rec] closes the decoded prefix */
  finish_status(p, out, st, cursor, n_rec, overflow);
  free(p);
  return st->code;
}

int kxo_thrift_decode(const kx_struct_desc* structs, uint32_t nstructs, const uint8_t* in,
                      uint64_t in_len, const uint64_t* offsets, uint64_t n, const kx_columns* out,
                      uint8_t* record_status, kx_status* st) {
  if (kxo_is_nested(structs, nstructs))
    return kxo_nthrift_decode(structs, nstructs, in, in_len, offsets, n, out, record_status, st);
  return decode_common(structs, nstructs, thrift_reader, 0, in, in_len, offsets, n, out, record_status, st);
}

/* ---- multi-threaded CPU baseline: size pass -> prefix -> emit pass, record ranges per thread ---- */
typedef struct {
  const plan_t* p; rec_reader rd; const uint8_t* in; uint64_t in_len; const uint64_t* offsets;
  uint64_t r0, r1; const kx_columns* out; kx_status st; uint64_t cursor[KX_MAX_COLUMNS];
  int emit; int overflow; int rc;
} mt_job;

static void* mt_worker(void* arg) {
  mt_job* j = (mt_job*)arg;
  memset(&j->st, 0, sizeof j->st);
  j->rc = decode_range(j->p, j->rd, j->in, j->in_len, j->offsets, j->r0, j->r1, 0, j->out, NULL,
                       &j->st, j->cursor, j->emit, &j->overflow);
  return NULL;
}

static int decode_mt(const kx_struct_desc* structs, uint32_t nstructs, rec_reader rd, int is_pb,
                     const uint8_t* in, uint64_t in_len, const uint64_t* offsets, uint64_t n,
                     const kx_columns* out, kx_status* st, int threads) {
  if (!offsets) return KX_ERR_INVALID_ARG;
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  plan_t* p = (plan_t*)malloc(sizeof(plan_t));
  int rc = plan_build(p, structs, nstructs);
  if (!rc) rc = check_out(p, out);
  if (rc) { free(p); return rc; }
  p->is_pb = is_pb;
  mt_job* jobs = (mt_job*)calloc((size_t)threads, sizeof(mt_job));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; t++) {
    jobs[t].p = p; jobs[t].rd = rd; jobs[t].in = in; jobs[t].in_len = in_len; jobs[t].offsets = offsets;
    jobs[t].r0 = n * (uint64_t)t / (uint64_t)threads; jobs[t].r1 = n * (uint64_t)(t + 1) / (uint64_t)threads;
    jobs[t].out = out;
  }
  /* pass 1: sizes */
  for (int t = 0; t < threads; t++) { jobs[t].emit = 0; pthread_create(&th[t], NULL, mt_worker, &jobs[t]); }
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  uint64_t run[KX_MAX_COLUMNS] = {0};
  for (int t = 0; t < threads; t++) {
    uint64_t sz[KX_MAX_COLUMNS];
    memcpy(sz, jobs[t].cursor, sizeof sz);
    for (int v = 0; v < p->nvar; v++) { jobs[t].cursor[v] = run[v]; run[v] += sz[v]; }
  }
  /* pass 2: emit */
  for (int t = 0; t < threads; t++) { jobs[t].emit = 1; jobs[t].overflow = 0; pthread_create(&th[t], NULL, mt_worker, &jobs[t]); }
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  memset(st, 0, sizeof *st);
  int overflow = 0;
  for (int t = 0; t < threads; t++) {
    if (jobs[t].rc == KX_ERR_INVALID_ARG) rc = KX_ERR_INVALID_ARG;
    if (jobs[t].st.code && (st->code == 0 || jobs[t].st.record < st->record)) {
      st->code = jobs[t].st.code; st->record = jobs[t].st.record; st->offset = jobs[t].st.offset;
    }
    overflow |= jobs[t].overflow;
  }
  st->n_records = n;
  finish_status(p, out, st, run, n, overflow);
  free(th); free(jobs); free(p);
  return rc ? rc : st->code;
}

int kxo_thrift_decode_mt(const kx_struct_desc* structs, uint32_t nstructs, const uint8_t* in,
                         uint64_t in_len, const uint64_t* offsets, uint64_t n, const kx_columns* out,
                         kx_status* st, int threads) {
  if (kxo_is_nested(structs, nstructs))
    return kxo_nthrift_decode(structs, nstructs, in, in_len, offsets, n, out, NULL, st);
  return decode_mt(structs, nstructs, thrift_reader, 0, in, in_len, offsets, n, out, st, threads);
}

/* ------------------------------------------------------------------------------------------------
 * Generated BLength / FastWriteNocopy (struct_tpl.go:225-391, 948-1061): fixed-length fields first,
 * then the rest, IDL order inside each group (reorderStructFields, patcher.go:503-522); optional
 * fields only when set (:313-340); a nil struct writes only STOP (k-mock.go:190-199); a list writes
 * its header (elem type, count) then the elements (:1011-1036); STOP at the end.
 * ---------------------------------------------------------------------------------------------- */
typedef struct { const plan_t* p; const kx_columns* in; uint64_t rec; uint8_t* out; } enc_t;

static uint64_t col_len(const enc_t* e, int col) {
  const kx_column* c = &e->in->cols[col];
  return off_get(c, e->rec + 1) - off_get(c, e->rec);
}

static uint64_t fixed_val(const enc_t* e, int col) {
  uint32_t w = e->p->cols[col].width;
  const uint8_t* s = (const uint8_t*)e->in->cols[col].data + e->rec * w;
  uint64_t v = 0;
  memcpy(&v, s, w);
  return v;
}

static int field_written(const enc_t* e, const kx_field_desc* f, const fmap_t* m, uint64_t pres) {
  if (f->req != KX_REQ_OPTIONAL) return 1;
  return (pres >> m->pbit) & 1;
}

/* returns bytes; writes when e->out != NULL */
static uint64_t write_struct(enc_t* e, int inst, uint64_t pres, uint8_t* b) {
  const inst_t* in = &e->p->inst[inst];
  const kx_struct_desc* sd = &e->p->structs[in->sidx];
  uint64_t off = 0;
  for (int pass = 0; pass < 2; pass++) {
    for (uint32_t i = 0; i < sd->nfields; i++) {
      const kx_field_desc* f = &sd->fields[i];
      if (is_fixed_length(f->ttype) != (pass == 0)) continue;
      const fmap_t* m = &in->fm[i];
      if (!field_written(e, f, m, pres)) continue;
      if (b) kxo_write_field_begin(b + off, f->ttype, f->id);
      off += 3;
      switch (f->ttype) {
        case KX_T_BOOL: case KX_T_BYTE: case KX_T_I16: case KX_T_I32: case KX_T_I64: case KX_T_DOUBLE: {
          uint64_t v = fixed_val(e, m->col);
          int w = type_size(f->ttype);
          if (b) {
            if (f->ttype == KX_T_BOOL) b[off] = v ? 1 : 0;
            else if (w == 1) b[off] = (uint8_t)v;
            else if (w == 2) put16(b + off, (uint16_t)v);
            else if (w == 4) put32(b + off, (uint32_t)v);
            else put64(b + off, v);
          }
          off += (uint64_t)w;
          break;
        }
        case KX_T_STRING: {
          uint64_t n = col_len(e, m->col);
          if (b) {
            const kx_column* c = &e->in->cols[m->col];
            kxo_write_string(b + off, (const uint8_t*)c->data + off_get(c, e->rec), (uint32_t)n);
          }
          off += 4 + n;
          break;
        }
        case KX_T_LIST: case KX_T_SET: {
          uint64_t n = col_len(e, m->col);
          if (f->elem_ttype == KX_T_STRING) {                  /* FieldFastWriteList of strings */
            const kx_column* c = &e->in->cols[m->col];
            const uint64_t E = off_get(c, e->rec);
            if (b) kxo_write_list_begin(b + off, KX_T_STRING, (int32_t)n);
            off += 5;
            for (uint64_t k = 0; k < n; k++) {
              const uint64_t a0 = eoff_get(c, E + k), l = eoff_get(c, E + k + 1) - a0;
              if (b) kxo_write_string(b + off, (const uint8_t*)c->data + a0, (uint32_t)l);
              off += 4 + l;
            }
            break;
          }
          if (f->elem_ttype == KX_T_STRUCT) {                  /* FieldFastWriteList of S: fields, STOP */
            const kx_struct_desc* es = &e->p->structs[f->child];
            if (b) kxo_write_list_begin(b + off, KX_T_STRUCT, (int32_t)n);
            off += 5;
            for (uint64_t k = 0; k < n; k++) {
              for (uint32_t g = 0; g < es->nfields; g++) {
                const kx_column* c = &e->in->cols[m->col + g];
                const uint8_t t = es->fields[g].ttype;
                const int w = type_size(t);
                uint64_t v = 0;
                memcpy(&v, (const uint8_t*)c->data + (off_get(c, e->rec) + k) * (uint64_t)w, (size_t)w);
                if (b) {
                  kxo_write_field_begin(b + off, t, es->fields[g].id);
                  uint8_t* q = b + off + 3;
                  if (t == KX_T_BOOL) q[0] = v ? 1 : 0;
                  else if (w == 1) q[0] = (uint8_t)v;
                  else if (w == 2) put16(q, (uint16_t)v);
                  else if (w == 4) put32(q, (uint32_t)v);
                  else put64(q, v);
                }
                off += 3 + (uint64_t)w;
              }
              if (b) b[off] = KX_T_STOP;
              off += 1;
            }
            break;
          }
          uint32_t w = e->p->cols[m->col].width;
          if (b) {
            const kx_column* c = &e->in->cols[m->col];
            kxo_write_list_begin(b + off, f->elem_ttype, (int32_t)n);
            const uint8_t* s = (const uint8_t*)c->data + off_get(c, e->rec) * w;
            uint8_t* d = b + off + 5;
            for (uint64_t k = 0; k < n; k++) {
              uint64_t v = 0;
              memcpy(&v, s + k * w, w);
              if (f->elem_ttype == KX_T_BOOL) d[k] = v ? 1 : 0;
              else if (w == 1) d[k] = (uint8_t)v;
              else if (w == 2) put16(d + k * 2, (uint16_t)v);
              else if (w == 4) put32(d + k * 4, (uint32_t)v);
              else put64(d + k * 8, v);
            }
          }
          off += 5 + n * w;
          break;
        }
        case KX_T_MAP: {  /* FieldFastWriteMap (:875-912) in stored order (Go's map order is random) */
          const kx_column* kc = &e->in->cols[m->col];
          const kx_column* vc = &e->in->cols[m->col + 1];
          const uint8_t kt = f->elem_ttype & 15, vt = (uint8_t)(f->elem_ttype >> 4);
          const uint64_t n = col_len(e, m->col), EK = off_get(kc, e->rec), EV = off_get(vc, e->rec);
          if (b) kxo_write_map_begin(b + off, kt, vt, (int32_t)n);
          off += 6;
          for (uint64_t k = 0; k < n; k++) {
            for (int side = 0; side < 2; side++) {
              const kx_column* c = side ? vc : kc;
              const uint8_t t = side ? vt : kt;
              const uint64_t E = side ? EV : EK;
              if (t == KX_T_STRING) {
                const uint64_t a0 = eoff_get(c, E + k), l = eoff_get(c, E + k + 1) - a0;
                if (b) kxo_write_string(b + off, (const uint8_t*)c->data + a0, (uint32_t)l);
                off += 4 + l;
              } else {
                const int w = type_size(t);
                uint64_t v = 0;
                memcpy(&v, (const uint8_t*)c->data + (E + k) * (uint64_t)w, (size_t)w);
                if (b) {
                  if (t == KX_T_BOOL) b[off] = v ? 1 : 0;
                  else if (w == 1) b[off] = (uint8_t)v;
                  else if (w == 2) put16(b + off, (uint16_t)v);
                  else if (w == 4) put32(b + off, (uint32_t)v);
                  else put64(b + off, v);
                }
                off += (uint64_t)w;
              }
            }
          }
          break;
        }
        case KX_T_STRUCT: {
          if ((pres >> m->pbit) & 1) off += write_struct(e, m->inst, pres, b ? b + off : NULL);
          else { if (b) b[off] = KX_T_STOP; off += 1; }          /* nil *T -> STOP only */
          break;
        }
        default: break;
      }
    }
  }
  if (b) b[off] = KX_T_STOP;
  return off + 1;
}

static uint64_t rec_presence(const enc_t* e) { return e->in->presence ? e->in->presence[e->rec] : 0; }

int kxo_thrift_sizes(const kx_struct_desc* structs, uint32_t nstructs, const kx_columns* in,
                     uint64_t n, uint64_t* sizes) {
  if (kxo_is_nested(structs, nstructs)) {
    uint64_t total = 0;
    return kxo_nthrift_encode(structs, nstructs, in, n, NULL, 0, sizes, NULL, &total);
  }
  plan_t* p = (plan_t*)malloc(sizeof(plan_t));
  int rc = plan_build(p, structs, nstructs);
  if (!rc) rc = check_out(p, in);
  if (rc) { free(p); return rc; }
  enc_t e = {p, in, 0, NULL};
  for (uint64_t r = 0; r < n; r++) { e.rec = r; sizes[r] = write_struct(&e, 0, rec_presence(&e), NULL); }
  free(p);
  return KX_OK;
}

typedef struct { const plan_t* p; const kx_columns* in; uint64_t r0, r1; uint8_t* out; uint64_t* offs; uint64_t base; uint64_t size; } enc_job;

static void* enc_worker(void* arg) {
  enc_job* j = (enc_job*)arg;
  enc_t e = {j->p, j->in, 0, NULL};
  uint64_t pos = j->base;
  for (uint64_t r = j->r0; r < j->r1; r++) {
    e.rec = r;
    if (j->offs && j->out) j->offs[r] = pos;
    pos += write_struct(&e, 0, rec_presence(&e), j->out ? j->out + pos : NULL);
  }
  j->size = pos - j->base;
  return NULL;
}

int kxo_thrift_encode_mt(const kx_struct_desc* structs, uint32_t nstructs, const kx_columns* in,
                         uint64_t n, uint8_t* out, uint64_t cap, uint64_t* offsets_out,
                         uint64_t* total, int threads) {
  if (kxo_is_nested(structs, nstructs))
    return kxo_nthrift_encode(structs, nstructs, in, n, out, cap, NULL, offsets_out, total);
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  plan_t* p = (plan_t*)malloc(sizeof(plan_t));
  int rc = plan_build(p, structs, nstructs);
  if (!rc) rc = check_out(p, in);
  if (rc) { free(p); return rc; }
  enc_job* jobs = (enc_job*)calloc((size_t)threads, sizeof(enc_job));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; t++) {
    jobs[t].p = p; jobs[t].in = in; jobs[t].offs = offsets_out; jobs[t].out = NULL;
    jobs[t].r0 = n * (uint64_t)t / (uint64_t)threads; jobs[t].r1 = n * (uint64_t)(t + 1) / (uint64_t)threads;
  }
  for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, enc_worker, &jobs[t]); /* BLength */
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  uint64_t run = 0;
  for (int t = 0; t < threads; t++) { jobs[t].base = run; run += jobs[t].size; }
  *total = run;
  if (run > cap) { free(th); free(jobs); free(p); return KX_ERR_SIZE_LIMIT; }
  for (int t = 0; t < threads; t++) { jobs[t].out = out; pthread_create(&th[t], NULL, enc_worker, &jobs[t]); }
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  if (offsets_out) offsets_out[n] = run;
  free(th); free(jobs); free(p);
  return KX_OK;
}

int kxo_thrift_encode(const kx_struct_desc* structs, uint32_t nstructs, const kx_columns* in,
                      uint64_t n, uint8_t* out, uint64_t cap, uint64_t* offsets_out, uint64_t* total) {
  return kxo_thrift_encode_mt(structs, nstructs, in, n, out, cap, offsets_out, total, 1);
}

/* ------------------------------------------------------------------------------------------------
 * Kitex-Protobuf. Meta header (protobuf.go:24-47, Marshal :77-90, Unmarshal :136-165):
 *   u32 BE (0x90010000 + msgType) | u32 BE len(method) | method | u32 BE seqID | proto3 body
 * Body: proto3 wire format (google.golang.org/protobuf v1.33.0 / prutal v0.1.3 — not vendored;
 * the published encoding is restated): varint tags, zero values omitted on encode, fields in
 * number order, last occurrence wins for singular fields, mismatched wire types are unknown fields.
 * ---------------------------------------------------------------------------------------------- */
size_t kxo_pb_write_meta(uint8_t* b, const char* method, uint32_t n, int32_t msg_type, int32_t seqid) {
  put32(b, 0x90010000u + (uint32_t)msg_type);
  put32(b + 4, n);
  if (n) memcpy(b + 8, method, n);
  put32(b + 8 + n, (uint32_t)seqid);
  return 12 + (size_t)n;
}

int kxo_pb_read_meta(const uint8_t* b, size_t len, uint32_t* method_off, uint32_t* method_len,
                     int32_t* msg_type, int32_t* seqid, size_t* used) {
  if (len < 4) return KX_ERR_EOF;
  uint32_t v = be32(b);
  if ((v & 0xffff0000u) != 0x90010000u) return KX_ERR_BAD_VERSION;  /* MagicMask, :142-144 */
  if (len < 8) return KX_ERR_EOF;
  uint32_t n = be32(b + 4);
  if (n == 0) return KX_ERR_INVALID_DATA;                            /* empty method (bytebuf_util.go:125-135) */
  if ((uint64_t)len < 12 + (uint64_t)n) return KX_ERR_EOF;
  *msg_type = (int32_t)(v & 0x0000ffffu);                            /* FrontMask */
  *method_off = 8; *method_len = n;
  *seqid = (int32_t)be32(b + 8 + n);
  *used = 12 + (size_t)n;
  return KX_OK;
}

size_t kxo_put_uvarint(uint8_t* b, uint64_t v) {
  size_t i = 0;
  while (v >= 0x80) { b[i++] = (uint8_t)(v | 0x80); v >>= 7; }
  b[i++] = (uint8_t)v;
  return i;
}

/* protowire.ConsumeVarint: at most 10 bytes, the 10th must be <= 1 */
int kxo_get_uvarint(const uint8_t* b, size_t len, uint64_t* v, size_t* used) {
  uint64_t x = 0;
  for (size_t i = 0; i < 10; i++) {
    if (i >= len) return KX_ERR_EOF;
    uint8_t c = b[i];
    if (i == 9 && c > 1) return KX_ERR_INVALID_DATA;
    x |= (uint64_t)(c & 0x7f) << (7 * i);
    if (c < 0x80) { *v = x; *used = i + 1; return KX_OK; }
  }
  return KX_ERR_INVALID_DATA;
}

/* UTF-8 validity as enforced by protobuf-go for proto3 `string` fields (utf8.Valid) */
static int utf8_valid(const uint8_t* s, uint64_t n) {
  uint64_t i = 0;
  while (i < n) {
    uint8_t c = s[i];
    if (c < 0x80) { i++; continue; }
    int k; uint32_t cp;
    if ((c & 0xe0) == 0xc0) { k = 1; cp = c & 0x1f; }
    else if ((c & 0xf0) == 0xe0) { k = 2; cp = c & 0x0f; }
    else if ((c & 0xf8) == 0xf0) { k = 3; cp = c & 0x07; }
    else return 0;
    if (i + (uint64_t)k >= n) return 0;                 /* truncated sequence */
    for (int j = 1; j <= k; j++) {
      uint8_t d = s[i + (uint64_t)j];
      if ((d & 0xc0) != 0x80) return 0;
      cp = (cp << 6) | (d & 0x3f);
    }
    if ((k == 1 && cp < 0x80) || (k == 2 && cp < 0x800) || (k == 3 && cp < 0x10000)) return 0;
    if (cp > 0x10ffff || (cp >= 0xd800 && cp <= 0xdfff)) return 0;
    i += (uint64_t)k + 1;
  }
  return 1;
}

#define KX_FIELD_BINARY 1  /* kx_field_desc.reserved0 bit: bytes, not string (no UTF-8 check) */

static int pb_wiretype(uint8_t t) {
  switch (t) {
    case KX_T_BOOL: case KX_T_BYTE: case KX_T_I16: case KX_T_I32: case KX_T_I64: return 0;
    case KX_T_DOUBLE: return 1;
    case KX_T_STRING: return 2;
    default: return -1;
  }
}

static int pb_skip(int wt, const uint8_t* b, size_t len, size_t* used) {
  uint64_t v; size_t u;
  int rc;
  switch (wt) {
    case 0: rc = kxo_get_uvarint(b, len, &v, &u); if (rc) return rc; *used = u; return KX_OK;
    case 1: if (len < 8) return KX_ERR_EOF; *used = 8; return KX_OK;
    case 2:
      rc = kxo_get_uvarint(b, len, &v, &u); if (rc) return rc;
      if (v > (uint64_t)(len - u)) return KX_ERR_EOF;
      *used = u + (size_t)v; return KX_OK;
    case 5: if (len < 4) return KX_ERR_EOF; *used = 4; return KX_OK;
    default: return KX_ERR_INVALID_DATA;  /* groups (3,4) and 6,7: rejected (parity unpinned) */
  }
}

static int pb_reader(dec_t* d, const uint8_t* b, size_t len, size_t* used) {
  const inst_t* in = &d->p->inst[0];
  const kx_struct_desc* sd = &d->p->structs[in->sidx];
  set_defaults(d, 0);
  size_t off = 0;
  while (off < len) {
    uint64_t tag; size_t u;
    int rc = kxo_get_uvarint(b + off, len - off, &tag, &u);
    if (rc) return rc;
    off += u;
    uint64_t num = tag >> 3;
    int wt = (int)(tag & 7);
    if (num == 0 || num > 536870911ull) return KX_ERR_INVALID_DATA;
    int fi = num <= 32767 ? find_field(sd, (int16_t)num) : -1;
    if (fi < 0 || pb_wiretype(sd->fields[fi].ttype) != wt) {
      rc = pb_skip(wt, b + off, len - off, &u);
      if (rc) return rc;
      off += u;
      continue;
    }
    const kx_field_desc* f = &sd->fields[fi];
    const fmap_t* m = &in->fm[fi];
    if (wt == 0) {
      uint64_t v;
      rc = kxo_get_uvarint(b + off, len - off, &v, &u);
      if (rc) return rc;
      off += u;
      if (f->ttype == KX_T_BOOL) v = v != 0;
      store_fixed(d, m->col, v);                   /* int32: low 32 bits; int64: all 64 */
    } else if (wt == 1) {
      if (len - off < 8) return KX_ERR_EOF;
      uint64_t v; memcpy(&v, b + off, 8);           /* little-endian fixed64 */
      store_fixed(d, m->col, v);
      off += 8;
    } else {
      uint64_t n;
      rc = kxo_get_uvarint(b + off, len - off, &n, &u);
      if (rc) return rc;
      off += u;
      if (n > (uint64_t)(len - off)) return KX_ERR_EOF;
      if (!(f->reserved0 & KX_FIELD_BINARY) && !utf8_valid(b + off, n)) return KX_ERR_INVALID_DATA;
      d->vptr[m->col] = b + off; d->vlen[m->col] = n;
      off += (size_t)n;
    }
    if (m->pbit >= 0) d->presence |= 1ull << m->pbit;
  }
  *used = off;
  return KX_OK;
}

static int pb_check_schema(const kx_struct_desc* structs, uint32_t nstructs) {
  if (!structs || nstructs == 0) return KX_ERR_INVALID_ARG;
  for (uint32_t i = 0; i < structs[0].nfields; i++)
    if (pb_wiretype(structs[0].fields[i].ttype) < 0) return KX_ERR_NOT_IMPLEMENTED;
  return KX_OK;
}

/* Batch framing: each record is field 1 / wire type 2: 0x0A, uvarint(len), body. */
static int pb_batch_offsets(const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t* body_off,
                            uint64_t* body_end, uint64_t* consumed, uint64_t* n_ok, int* rc_out) {
  uint64_t pos = 0;
  for (uint64_t i = 0; i < n; i++) {
    if (pos >= in_len) { *n_ok = i; *consumed = pos; *rc_out = KX_ERR_EOF; return 0; }
    if (in[pos] != 0x0A) { *n_ok = i; *consumed = pos; *rc_out = KX_ERR_INVALID_DATA; return 0; }
    uint64_t l; size_t u;
    int rc = kxo_get_uvarint(in + pos + 1, (size_t)(in_len - pos - 1), &l, &u);
    if (rc == KX_OK && l > in_len - pos - 1 - u) rc = KX_ERR_EOF;
    if (rc) { *n_ok = i; *consumed = pos; *rc_out = rc; return 0; }
    body_off[i] = pos + 1 + u;
    body_end[i] = body_off[i] + l;
    pos = body_end[i];
  }
  *n_ok = n; *consumed = pos; *rc_out = KX_OK;
  return 1;
}

int kxo_pb_decode(const kx_struct_desc* structs, uint32_t nstructs, const uint8_t* in,
                  uint64_t in_len, const uint64_t* offsets, uint64_t n, const kx_columns* out,
                  uint8_t* record_status, kx_status* st) {
  if (pb_nested(structs, nstructs))
    return kxo_npb_decode(structs, nstructs, in, in_len, offsets, n, out, record_status, st);
  int rc = pb_check_schema(structs, nstructs);
  if (rc) return rc;
  if (offsets) return decode_common(structs, nstructs, pb_reader, 1, in, in_len, offsets, n, out, record_status, st);
  /* concatenated: resolve the Batch framing first, then decode each body (offsets pairs) */
  uint64_t* bo = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
  uint64_t* be = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
  uint64_t consumed = 0, n_ok = 0;
  int frc = KX_OK;
  pb_batch_offsets(in, in_len, n, bo, be, &consumed, &n_ok, &frc);
  /* decode bodies: build a compact (start,end) walk */
  plan_t* p = (plan_t*)malloc(sizeof(plan_t));
  rc = plan_build(p, structs, nstructs);
  if (!rc) rc = check_out(p, out);
  if (rc) { free(p); free(bo); free(be); return rc; }
  memset(st, 0, sizeof *st);
  uint64_t cursor[KX_MAX_COLUMNS] = {0};
  int overflow = 0;
  dec_t d; memset(&d, 0, sizeof d);
  d.p = p; d.out = out; d.emit = 1; d.in0 = in;
  uint64_t r = 0;
  for (; r < n_ok; r++) {
    d.rec = r; d.presence = 0;
    size_t used;
    int e = pb_reader(&d, in + bo[r], (size_t)(be[r] - bo[r]), &used);
    if (e) {
      st->code = e; st->record = r; st->offset = bo[r];
      if (record_status) record_status[r] = (uint8_t)e;
      break;
    }
    if (record_status) record_status[r] = 0;
    emit_record_tail(&d, cursor, &overflow);
  }
  if (r == n_ok && frc) { st->code = frc; st->record = n_ok; }
  (void)consumed;
  if (st->code) st->offset = r ? be[r - 1] : 0;   /* start of the failing record's frame */
  st->n_records = r;
  st->consumed = r ? be[r - 1] : 0;
  finish_status(p, out, st, cursor, r, overflow);
  free(p); free(bo); free(be);
  return st->code;
}

int kxo_pb_decode_mt(const kx_struct_desc* structs, uint32_t nstructs, const uint8_t* in,
                     uint64_t in_len, const uint64_t* offsets, uint64_t n, const kx_columns* out,
                     kx_status* st, int threads) {
  if (pb_nested(structs, nstructs))
    return kxo_npb_decode(structs, nstructs, in, in_len, offsets, n, out, NULL, st);
  int rc = pb_check_schema(structs, nstructs);
  if (rc) return rc;
  return decode_mt(structs, nstructs, pb_reader, 1, in, in_len, offsets, n, out, st, threads);
}

static uint64_t pb_write_record(const plan_t* p, const kx_columns* in, uint64_t rec, uint8_t* b) {
  const kx_struct_desc* sd = &p->structs[0];
  const inst_t* ins = &p->inst[0];
  /* field-number order */
  int order[MAXF];
  for (uint32_t i = 0; i < sd->nfields; i++) order[i] = (int)i;
  for (uint32_t i = 1; i < sd->nfields; i++)
    for (uint32_t j = i; j > 0 && sd->fields[order[j]].id < sd->fields[order[j - 1]].id; j--) {
      int t = order[j]; order[j] = order[j - 1]; order[j - 1] = t;
    }
  uint64_t pres = in->presence ? in->presence[rec] : 0;
  uint64_t off = 0;
  uint8_t tmp[16];
  for (uint32_t k = 0; k < sd->nfields; k++) {
    const kx_field_desc* f = &sd->fields[order[k]];
    const fmap_t* m = &ins->fm[order[k]];
    int explicit_presence = f->req == KX_REQ_OPTIONAL;
    if (explicit_presence && !((pres >> m->pbit) & 1)) continue;
    int wt = pb_wiretype(f->ttype);
    uint64_t tag = ((uint64_t)(uint16_t)f->id << 3) | (uint64_t)wt;
    if (wt == 2) {
      const kx_column* c = &in->cols[m->col];
      uint64_t n = off_get(c, rec + 1) - off_get(c, rec);
      if (n == 0 && !explicit_presence) continue;
      size_t u = kxo_put_uvarint(tmp, tag);
      if (b) memcpy(b + off, tmp, u);
      off += u;
      u = kxo_put_uvarint(tmp, n);
      if (b) memcpy(b + off, tmp, u);
      off += u;
      if (b && n) memcpy(b + off, (const uint8_t*)c->data + off_get(c, rec), n);
      off += n;
      continue;
    }
    uint32_t w = p->cols[m->col].width;
    uint64_t v = 0;
    memcpy(&v, (const uint8_t*)in->cols[m->col].data + rec * w, w);
    if (wt == 0 && w == 4) v = (uint64_t)(int64_t)(int32_t)(uint32_t)v;   /* int32 sign-extends */
    if (wt == 0 && w == 2) v = (uint64_t)(int64_t)(int16_t)(uint16_t)v;
    if (wt == 0 && w == 1) v = f->ttype == KX_T_BOOL ? (v & 0xff ? 1 : 0) : (uint64_t)(int64_t)(int8_t)(uint8_t)v;
    if (v == 0 && !explicit_presence) continue;                          /* proto3 zero omitted */
    size_t u = kxo_put_uvarint(tmp, tag);
    if (b) memcpy(b + off, tmp, u);
    off += u;
    if (wt == 0) { u = kxo_put_uvarint(tmp, v); if (b) memcpy(b + off, tmp, u); off += u; }
    else { if (b) memcpy(b + off, &v, 8); off += 8; }
  }
  return off;
}

int kxo_pb_encode(const kx_struct_desc* structs, uint32_t nstructs, const kx_columns* in,
                  uint64_t n, uint8_t* out, uint64_t cap, uint64_t* offsets_out, uint64_t* total) {
  if (pb_nested(structs, nstructs)) return kxo_npb_encode(structs, nstructs, in, n, out, cap, offsets_out, total);
  int rc = pb_check_schema(structs, nstructs);
  if (rc) return rc;
  plan_t* p = (plan_t*)malloc(sizeof(plan_t));
  rc = plan_build(p, structs, nstructs);
  if (!rc) rc = check_out(p, in);
  if (rc) { free(p); return rc; }
  uint64_t pos = 0;
  uint8_t tmp[16];
  for (uint64_t r = 0; r < n; r++) {
    uint64_t body = pb_write_record(p, in, r, NULL);
    size_t u = kxo_put_uvarint(tmp, body);
    if (pos + 1 + u + body > cap) { free(p); *total = pos; return KX_ERR_SIZE_LIMIT; }
    out[pos] = 0x0A;
    memcpy(out + pos + 1, tmp, u);
    if (offsets_out) offsets_out[r] = pos + 1 + u;
    pb_write_record(p, in, r, out + pos + 1 + u);
    pos += 1 + u + body;
  }
  if (offsets_out) offsets_out[n] = pos;
  *total = pos;
  free(p);
  return KX_OK;
}

uint64_t kxo_splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
