// kx_message.hip — message level of an RPC batch on CDNA4 / gfx950: N framed messages, each
// MessageBegin + the method's argument (or result) struct, whose one field holds the record; or each
// a Kitex-Protobuf meta header + the proto body (protobuf.go:77-90,136-165: u32 0x9001_0000 + type,
// u32-length method name, u32 seqid).
//
// Reference semantics: thriftCodec.Unmarshal (pkg/remote/codec/thrift/thrift.go:180-225):
// ReadMessageBegin (strict binary: i32 0x8001_00TT, string name, i32 seqid; binary_test.go:387-457),
// an EXCEPTION message carries a TApplicationException instead of the arguments (thrift.go:192-195),
// then the generated Args/Result FastRead (internal/mocks/thrift/k-mock.go:422-517): fields until
// STOP, field `body` (1 = Args.Req, 0 = Result.Success) of type STRUCT is the record, every other
// field goes through the skip decoder (codec_apache.go:191-293, depth 64).
//
// Pipeline (all stream-ordered, lane = message):
//   header_kernel  MessageBegin + Args walk -> type / seqid columns, name extents, the record's
//                  extent [req_start, req_end) (an absent record field -> the Args STOP byte, i.e.
//                  an empty struct), a per-message header code
//   bsum / bscan / apply  exclusive scan of the name lengths: block sums of 4096-entry blocks, one workgroup
//                  over the block sums, then each block's own scan (was one workgroup over all n: 58 ms
//                  at 16 M messages on the MI355X)
//   name_kernel    method names copied into the name arena
//   (the record bodies: kx_launch_decode in known-offsets mode with explicit ends)
//   merge_kernel   per-message code = header code, else body code; first failing message -> status
// Header walks read global memory byte-wise: headers are tens of bytes, the bodies are the work.
#include <hip/hip_runtime.h>

#include "kx_internal.h"
#include "kx_mem.h"

namespace {

constexpr int MT = 256;       // threads per workgroup (lane = message)
constexpr int ST = 1024;      // scan kernel: one workgroup
constexpr int MAXDEPTH = 64;  // skip recursion depth (codec_apache.go:167)

__device__ __forceinline__ uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

__device__ __forceinline__ int fixed_size(uint32_t t) {
  switch (t) {
    case KX_T_BOOL: case KX_T_BYTE: return 1;
    case KX_T_I16: return 2;
    case KX_T_I32: return 4;
    case KX_T_I64: case KX_T_DOUBLE: return 8;
    default: return 0;
  }
}

// skipType (codec_apache.go:191-293) of one value of type t at pos, bounded by end; an explicit
// stack of struct / list / map frames instead of recursion (depth limit as the reference)
struct Frame {
  uint8_t kind, t1, t2, phase;  // kind 0 struct, 1 list/set, 2 map (phase 0 key, 1 value)
  uint32_t left;
};

// The header walk's bytes through a 16-byte aligned block held in registers: a field's type byte, ids and
// lengths mostly lie in the block the previous field's read loaded, so the walk's chain of dependent global
// byte loads (one per field) becomes one 16-byte load per block crossed. A read that straddles the block's
// end is made byte by byte (and leaves the block as it is). An aligned 16-byte block never crosses a page,
// so its bytes past the input are readable (and never used).
struct HWin {
  const uint8_t* in;
  uint64_t base;        // absolute address of the block (16-aligned), ~0 before the first read
  uint32_t d0, d1, d2, d3;
  __device__ __forceinline__ uint32_t dw(uint32_t i) const { return i == 0 ? d0 : i == 1 ? d1 : i == 2 ? d2 : d3; }
  __device__ __forceinline__ void fill(uint64_t a) {
    base = a & ~15ull;
    const uint4 v = kx_ld16((const void*)base);
    d0 = v.x; d1 = v.y; d2 = v.z; d3 = v.w;
  }
  __device__ __forceinline__ uint32_t b(uint64_t p) {
    const uint64_t a = (uint64_t)in + p;
    if (a - base >= 16) fill(a);
    const uint32_t o = (uint32_t)(a - base);
    return (dw(o >> 2) >> (8 * (o & 3))) & 0xffu;
  }
  // 4 bytes at p, big-endian
  __device__ __forceinline__ uint32_t be32(uint64_t p) {
    const uint64_t a = (uint64_t)in + p;
    if (a - base >= 16) fill(a);
    const uint32_t o = (uint32_t)(a - base);
    if (o + 4 <= 16) {
      const uint32_t i = o >> 2;
      const uint32_t lo = dw(i), hi = i < 3 ? dw(i + 1) : 0u;
      return __builtin_bswap32(__builtin_amdgcn_alignbyte(hi, lo, o & 3));
    }
    const uint8_t* q = in + p;
    return ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
};

// The innermost open frame lives in registers (`top`); only the frames below it go to the stack array,
// which is private (scratch) memory: a record nested one level deep never touches it (with every frame
// in the array, each field re-read its frame from scratch, a memory round trip per field).
__device__ __forceinline__ int skip_value(HWin& in, uint64_t& pos, uint64_t end, uint32_t t) {
  Frame st[MAXDEPTH];
  Frame top = Frame{0, 0, 0, 0, 0};
  int sp = 0;  // open frames: st[0 .. sp - 2], then top
  auto push = [&](const Frame& f) {
    if (sp > 0) st[sp - 1] = top;
    top = f;
    sp++;
  };
  auto pop = [&]() {
    sp--;
    if (sp > 0) top = st[sp - 1];
  };
  uint32_t cur = t;
  for (;;) {
    const int w = fixed_size(cur);
    if (w) {
      if (end - pos < (uint64_t)w) return KX_ERR_EOF;
      pos += w;
    } else if (cur == KX_T_STRING) {
      if (end - pos < 4) return KX_ERR_EOF;
      const int32_t l = (int32_t)in.be32(pos);
      if (l < 0) return KX_ERR_NEGATIVE_SIZE;
      if (end - pos - 4 < (uint64_t)l) return KX_ERR_EOF;
      pos += 4 + (uint64_t)l;
    } else if (cur == KX_T_STRUCT) {
      if (sp == MAXDEPTH) return KX_ERR_DEPTH_LIMIT;
      push(Frame{0, 0, 0, 0, 0});
    } else if (cur == KX_T_LIST || cur == KX_T_SET) {
      if (end - pos < 5) return KX_ERR_EOF;
      const uint32_t et = in.b(pos);
      const int32_t sz = (int32_t)in.be32(pos + 1);
      pos += 5;
      if (sz < 0) return KX_ERR_NEGATIVE_SIZE;
      const int ew = fixed_size(et);
      if (ew) {
        if ((end - pos) / (uint64_t)ew < (uint64_t)sz) return KX_ERR_EOF;
        pos += (uint64_t)sz * ew;
      } else if (sz) {
        if (sp == MAXDEPTH) return KX_ERR_DEPTH_LIMIT;
        push(Frame{1, (uint8_t)et, 0, 0, (uint32_t)sz});
      }
    } else if (cur == KX_T_MAP) {
      if (end - pos < 6) return KX_ERR_EOF;
      const uint32_t kt = in.b(pos), vt = in.b(pos + 1);
      const int32_t sz = (int32_t)in.be32(pos + 2);
      pos += 6;
      if (sz < 0) return KX_ERR_NEGATIVE_SIZE;
      const int kw = fixed_size(kt), vw = fixed_size(vt);
      if (kw && vw) {
        if ((end - pos) / (uint64_t)(kw + vw) < (uint64_t)sz) return KX_ERR_EOF;
        pos += (uint64_t)sz * (kw + vw);
      } else if (sz) {
        if (sp == MAXDEPTH) return KX_ERR_DEPTH_LIMIT;
        push(Frame{2, (uint8_t)kt, (uint8_t)vt, 0, (uint32_t)sz});
      }
    } else {
      return KX_ERR_INVALID_DATA;  // unknown data type
    }
    // the next value to skip, from the innermost open frame
    for (;;) {
      if (sp == 0) return KX_OK;
      if (top.kind == 0) {
        if (pos >= end) return KX_ERR_EOF;
        const uint32_t ft = in.b(pos);
        if (ft == KX_T_STOP) { pos++; pop(); continue; }
        if (end - pos < 3) return KX_ERR_EOF;
        pos += 3;
        cur = ft;
        break;
      }
      if (top.left == 0) { pop(); continue; }
      if (top.kind == 1) {
        top.left--;
        cur = top.t1;
      } else if (top.phase == 0) {
        top.phase = 1;
        cur = top.t1;
      } else {
        top.phase = 0;
        top.left--;
        cur = top.t2;
      }
      break;
    }
  }
}

struct MsgParams {
  const uint8_t* in;
  uint64_t in_len;
  const uint64_t* offsets;   // n + 1 message boundaries (with ends: n message starts)
  const uint64_t* ends;      // message i ends at ends[i] (framed payloads), else offsets[i + 1]
  const kx_status* pre;      // framing-scan status: messages from its failing frame on are not read
  const uint8_t* pre_rc;     // per-frame code found before the payload is read (CRC32C validation)
  uint64_t n;
  int32_t body_field;        // 1: Args{1: req}, 0: Result{0: success}
  int pb;                    // Kitex-Protobuf meta header (magic 0x9001, 16-bit type), body = the rest
  const uint8_t* raw_flags;  // raw mode (gRPC): no message header, the body is the whole payload;
  int raw;                   // a message whose compressed flag is 1 cannot be decoded here
  KxMsgOut mo;
  uint64_t* req_start;       // n + 1 (req_start[n] = in_len)
  uint64_t* req_end;
  uint64_t* name_pos;
  uint64_t* name_len;        // n + 1, scanned in place into the name offsets
  uint8_t* hdr_rc;
  unsigned long long* errkey;
  uint32_t* overflow;
};

__global__ void __launch_bounds__(MT) header_kernel(MsgParams mp) {
  const uint64_t i = (uint64_t)blockIdx.x * MT + threadIdx.x;
  if (i >= mp.n) {
    if (i == mp.n) { mp.req_start[i] = mp.in_len; mp.name_len[i] = 0; }
    return;
  }
  const uint8_t* in = mp.in;
  const bool cut = mp.pre && mp.pre->code && i >= (uint64_t)mp.pre->record;
  const uint64_t p = cut ? 0 : mp.offsets[i], e = cut ? 0 : mp.ends ? mp.ends[i] : mp.offsets[i + 1];
  int rc = KX_OK;
  uint32_t type = 0;
  int32_t seqid = 0, nl = 0;
  uint64_t rs = p, re = p;
  if (cut) {
    rc = mp.pre->code;  // the frame could not be delimited: neither it nor any later one is decoded
  } else if (mp.pre_rc && mp.pre_rc[i]) {
    rc = mp.pre_rc[i];  // DecodeMeta failed (payload checksum): the payload codec never runs
  } else if (p > e || e > mp.in_len) {
    rc = KX_ERR_INVALID_ARG;
  } else if (mp.raw == 2) {
    // binary generic ingress (binaryThriftCodec.Unmarshal, pkg/generic/binarythrift_codec.go:83-115): the
    // request stays the raw message; PeekUint32 & FrontMask == Exception takes the regular thrift path;
    // readBinaryMethod (:185-199): u32 length at [4, 8), 0 < length <= size - 8, name at [8, 8 + length)
    if (e - p < 4) {
      rc = KX_ERR_EOF;
    } else {
      const uint32_t v = be32(in + p);
      type = v & 0xffffu;
      if (type == KX_MSG_EXCEPTION) {
        rc = KX_ERR_APPLICATION_EXCEPTION;
      } else if (e - p < 8) {
        rc = KX_ERR_INVALID_DATA;
      } else {
        const uint64_t ml = be32(in + p + 4);
        if (ml == 0 || ml > 0x7fffffffull || e - p - 8 < ml) {
          rc = KX_ERR_INVALID_DATA;
        } else {
          nl = (int32_t)ml;
          seqid = e - p - 8 - ml >= 4 ? (int32_t)be32(in + p + 8 + ml) : 0;
        }
      }
    }
    rs = p;
    re = p;
  } else if (mp.raw) {
    // decodeGRPCFrame (grpc_compress.go:53-58): a compressed message needs a registered decompressor
    if (mp.raw_flags && mp.raw_flags[i] == 1) rc = KX_ERR_NOT_IMPLEMENTED;
    rs = p;
    re = e;
  } else if (e - p < 4) {
    rc = KX_ERR_EOF;
  } else {
    const uint32_t v = be32(in + p);
    if ((v & 0xffff0000u) != (mp.pb ? 0x90010000u : 0x80010000u)) {
      rc = KX_ERR_BAD_VERSION;
    } else if (e - p < 8) {
      rc = KX_ERR_EOF;
    } else {
      nl = (int32_t)be32(in + p + 4);
      if (nl < 0) rc = KX_ERR_NEGATIVE_SIZE;
      else if (e - p < 12ull + (uint64_t)nl) rc = KX_ERR_EOF;
      else {
        type = v & (mp.pb ? 0xffffu : 0xffu);
        seqid = (int32_t)be32(in + p + 8 + nl);
      }
    }
  }
  if (!rc && type == KX_MSG_EXCEPTION) rc = KX_ERR_APPLICATION_EXCEPTION;
  if (mp.raw) {
  } else if (!rc && mp.pb) {  // protobuf.go:136-165: the body is the rest of the payload
    rs = p + 12 + (uint64_t)nl;
    re = e;
  } else if (!rc) {  // the Args / Result struct: fields until STOP, the record field kept, the rest skipped
    uint64_t pos = p + 12 + (uint64_t)nl;
    bool have = false;
    HWin hw{in, ~0ull, 0u, 0u, 0u, 0u};
    for (;;) {
      if (pos >= e) { rc = KX_ERR_EOF; break; }
      const uint32_t t = hw.b(pos);
      if (t == KX_T_STOP) {
        if (!have) { rs = pos; re = pos + 1; }  // no record field: an empty struct (the STOP byte)
        break;
      }
      if (e - pos < 3) { rc = KX_ERR_EOF; break; }
      const int32_t id = (int16_t)((hw.b(pos + 1) << 8) | hw.b(pos + 2));
      pos += 3;
      const uint64_t s0 = pos;
      rc = skip_value(hw, pos, e, t);
      if (rc) break;
      if (id == mp.body_field && t == KX_T_STRUCT) { rs = s0; re = pos; have = true; }
    }
  }
  if (rc) { rs = re = p; nl = 0; type = 0; seqid = 0; }
  mp.req_start[i] = rs;
  mp.req_end[i] = re;
  mp.name_pos[i] = p + 8;
  mp.name_len[i] = (uint64_t)nl;
  mp.hdr_rc[i] = (uint8_t)rc;
  if (mp.mo.msg_type) mp.mo.msg_type[i] = (int32_t)type;
  if (mp.mo.seqid) mp.mo.seqid[i] = seqid;
}

// SetSeqID (binarythrift_codec.go:117-134 via getSeqID4Bytes :147-175) of raw message i in place
__global__ void __launch_bounds__(MT) setseq_kernel(uint8_t* in, uint64_t in_len, const uint64_t* offsets,
                                                    uint64_t n, const int32_t* seqids, uint8_t* rs,
                                                    unsigned long long* errkey) {
  const uint64_t i = (uint64_t)blockIdx.x * MT + threadIdx.x;
  if (i >= n) return;
  const uint64_t p = offsets[i], e = offsets[i + 1];
  int rc = KX_OK;
  if (p > e || e > in_len) {
    rc = KX_ERR_INVALID_ARG;
  } else if (e - p < 4) {
    rc = KX_ERR_INVALID_DATA;
  } else {
    const int32_t first = (int32_t)be32(in + p);
    if (first > 0) rc = KX_ERR_INVALID_DATA;                                  // missing version
    else if (((uint32_t)first & 0xffff0000u) != 0x80010000u) rc = KX_ERR_BAD_VERSION;
    else if (e - p < 8) rc = KX_ERR_INVALID_DATA;
    else {
      const int32_t nl = (int32_t)be32(in + p + 4);
      if (nl < 0) rc = KX_ERR_INVALID_DATA;                                    // perrors.InvalidDataLength
      else if (e - p < 12ull + (uint64_t)nl) rc = KX_ERR_INVALID_DATA;         // invalid trans buffer
      else {
        const uint32_t v = (uint32_t)seqids[i];
        uint8_t* q = in + p + 8 + nl;
        q[0] = (uint8_t)(v >> 24); q[1] = (uint8_t)(v >> 16); q[2] = (uint8_t)(v >> 8); q[3] = (uint8_t)v;
      }
    }
  }
  if (rs) rs[i] = (uint8_t)rc;
  if (rc) atomicMin(errkey, (unsigned long long)((i << 8) | (uint64_t)(rc & 0xff)));
}

// fastMarshal (codec_fast.go:40-58) of message i: WriteMessageBegin(name, type, seqid[i]) + the Args /
// Result struct whose field `body_field` holds record i (STRUCT header) + the record + STOP. Every
// message adds the same H + 1 bytes around its record, so its position is body_off[i] + i * (H + 1): no
// scan. Lane = message; the record's bytes are copied from the encoder's output.
struct MsgEnc {
  const uint8_t* bodies;
  const uint64_t* body_off;  // n + 1
  uint64_t scratch_cap;      // bytes readable at `bodies`
  uint64_t n;
  const uint8_t* name;       // device copy of the method name
  uint32_t name_len;
  int32_t msg_type;
  const int32_t* seqids;
  int32_t body_field;
  uint8_t* out;
  uint64_t out_cap;
  uint64_t* offsets_out;     // n + 1 (optional)
  kx_status* status;
};

__global__ void __launch_bounds__(MT) msgenc_kernel(MsgEnc me) {
  const uint64_t i = (uint64_t)blockIdx.x * MT + threadIdx.x;
  const int lane = threadIdx.x & 63;
  // the record encoder failed (SIZE_LIMIT: the scratch is too small, or a record error): its offsets were
  // never written, so nothing here may read them; the status keeps the encoder's code and counts
  if (me.status->code != 0) return;  // uniform
  const uint64_t H = 12ull + me.name_len + 3ull;
  bool ok = i <= me.n;
  const uint64_t bo = ok ? me.body_off[i] : 0;
  if (ok && (bo > me.scratch_cap || me.body_off[me.n] > me.scratch_cap)) {  // never read past the offsets
    if (i == me.n) me.status->code = KX_ERR_SIZE_LIMIT;
    ok = false;
  }
  const uint64_t at = bo + i * (H + 1);
  if (ok && me.offsets_out) me.offsets_out[i] = at;
  if (ok && i == me.n) {
    me.status->n_records = me.n;
    me.status->consumed = at;
    if (at > me.out_cap) me.status->code = KX_ERR_SIZE_LIMIT;
    ok = false;
  }
  uint64_t bl = 0;
  if (ok) {
    const uint64_t bn = me.body_off[i + 1];
    ok = bn >= bo && bn <= me.scratch_cap;                       // (thread n reports the inconsistency)
    bl = ok ? bn - bo : 0;
    ok = ok && at <= me.out_cap && me.out_cap - at >= H + bl + 1;  // else SIZE_LIMIT (thread n)
  }
  uint8_t* d = nullptr;
  if (ok) {
    uint8_t* o = me.out + at;
    const uint32_t v = 0x80010000u | ((uint32_t)me.msg_type & 0xffu);  // strict version | type
    const uint32_t nl = me.name_len, sq = (uint32_t)me.seqids[i];
    o[0] = (uint8_t)(v >> 24); o[1] = (uint8_t)(v >> 16); o[2] = (uint8_t)(v >> 8); o[3] = (uint8_t)v;
    o[4] = (uint8_t)(nl >> 24); o[5] = (uint8_t)(nl >> 16); o[6] = (uint8_t)(nl >> 8); o[7] = (uint8_t)nl;
    for (uint32_t k = 0; k < nl; k++) o[8 + k] = me.name[k];
    uint8_t* q = o + 8 + nl;
    q[0] = (uint8_t)(sq >> 24); q[1] = (uint8_t)(sq >> 16); q[2] = (uint8_t)(sq >> 8); q[3] = (uint8_t)sq;
    q[4] = KX_T_STRUCT; q[5] = (uint8_t)((uint32_t)me.body_field >> 8); q[6] = (uint8_t)me.body_field;
    d = q + 7;
    d[bl] = KX_T_STOP;
  }
  // the records' bytes: copied by the whole wave, one message after the other, 64 adjacent bytes per
  // store instruction (a lane copying its own record would touch 64 records' lines per instruction)
  const uint64_t src = ok ? (uint64_t)(me.bodies + bo) : 0, dst = (uint64_t)d, len = ok ? bl : 0;
  for (int j = 0; j < 64; j++) {
    const uint64_t lj = (uint64_t)__shfl((long long)len, j, 64);
    if (lj == 0) continue;
    const uint8_t* sj = (const uint8_t*)(uint64_t)__shfl((long long)src, j, 64);
    uint8_t* dj = (uint8_t*)(uint64_t)__shfl((long long)dst, j, 64);
    for (uint64_t k = (uint64_t)lane; k < lj; k += 64) dj[k] = sj[k];
  }
}

// exclusive scan of name_len[0..n] in place, three passes: SB entries per block (MT threads x SPT
// consecutive entries each, so a wave covers 64 x SPT contiguous words)
constexpr int SPT = 16;
constexpr uint64_t SB = (uint64_t)MT * SPT;

__device__ __forceinline__ uint64_t wave_incl_u64(uint64_t v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

// block exclusive prefix of x (MT threads); *tot = the block's sum
__device__ __forceinline__ uint64_t block_excl(uint64_t x, uint64_t* tot) {
  __shared__ uint64_t wsum[MT / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t inc = wave_incl_u64(x, lane);
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  uint64_t base = 0, t = 0;
#pragma unroll
  for (int k = 0; k < MT / 64; k++) {
    if (k < wv) base += wsum[k];
    t += wsum[k];
  }
  __syncthreads();
  *tot = t;
  return base + inc - x;
}

__global__ void __launch_bounds__(MT) scan_bsum_kernel(const uint64_t* v, uint64_t n1, uint64_t* bs) {
  const uint64_t lo = (uint64_t)blockIdx.x * SB;
  uint64_t s = 0;
  for (int k = 0; k < SPT; k++) {
    const uint64_t i = lo + (uint64_t)k * MT + threadIdx.x;   // coalesced
    if (i < n1) s += v[i];
  }
  uint64_t tot;
  (void)block_excl(s, &tot);
  if (threadIdx.x == 0) bs[blockIdx.x] = tot;
}

// one workgroup: the block sums -> exclusive block bases
__global__ void __launch_bounds__(ST) scan_bases_kernel(uint64_t* bs, uint64_t nb) {
  __shared__ uint64_t part[ST];
  const uint64_t per = (nb + ST - 1) / ST;
  const uint64_t lo = kmin64((uint64_t)threadIdx.x * per, nb), hi = kmin64(lo + per, nb);
  uint64_t s = 0;
  for (uint64_t k = lo; k < hi; k++) s += bs[k];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int d = 1; d < ST; d <<= 1) {
    const uint64_t x = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0;
    __syncthreads();
    part[threadIdx.x] += x;
    __syncthreads();
  }
  uint64_t run = part[threadIdx.x] - s;
  for (uint64_t k = lo; k < hi; k++) {
    const uint64_t x = bs[k];
    bs[k] = run;
    run += x;
  }
}

__global__ void __launch_bounds__(MT) scan_apply_kernel(uint64_t* v, uint64_t n1, const uint64_t* bs) {
  const uint64_t lo = (uint64_t)blockIdx.x * SB + (uint64_t)threadIdx.x * SPT;
  uint64_t x[SPT], s = 0;
#pragma unroll
  for (int k = 0; k < SPT; k++) {
    x[k] = lo + k < n1 ? v[lo + k] : 0;
    s += x[k];
  }
  uint64_t tot;
  uint64_t run = bs[blockIdx.x] + block_excl(s, &tot);
#pragma unroll
  for (int k = 0; k < SPT; k++) {
    if (lo + k < n1) v[lo + k] = run;
    run += x[k];
  }
}

__global__ void __launch_bounds__(MT) name_kernel(MsgParams mp) {
  const uint64_t i = (uint64_t)blockIdx.x * MT + threadIdx.x;
  if (i > mp.n) return;
  const uint64_t at = mp.name_len[i];  // exclusive prefix after the scan
  const bool wide = mp.mo.name_owide != 0;
  const uint64_t lim = wide ? mp.mo.name_cap : kmin64(mp.mo.name_cap, 0xffffffffull);
  if (mp.mo.name_offs) {
    if (at <= lim) {
      if (wide) ((uint64_t*)mp.mo.name_offs)[i] = at;
      else ((uint32_t*)mp.mo.name_offs)[i] = (uint32_t)at;
    } else if (i == mp.n) {
      atomicOr(mp.overflow, 1u);
    }
  }
  if (i == mp.n || !mp.mo.name_data) return;
  const uint64_t len = mp.name_len[i + 1] - at;
  if (at + len > lim) return;
  const uint8_t* src = mp.in + mp.name_pos[i];
  for (uint64_t k = 0; k < len; k++) mp.mo.name_data[at + k] = src[k];
}

__global__ void __launch_bounds__(MT) merge_kernel(const uint8_t* hdr_rc, const uint8_t* body_rc,
                                                   uint8_t* record_status, uint64_t n, unsigned long long* errkey) {
  const uint64_t i = (uint64_t)blockIdx.x * MT + threadIdx.x;
  if (i >= n) return;
  const int rc = hdr_rc[i] ? hdr_rc[i] : body_rc[i];
  if (record_status) record_status[i] = (uint8_t)rc;
  if (rc) atomicMin(errkey, (unsigned long long)((i << 8) | (uint64_t)(rc & 0xff)));
}

// the call's status: the first failing message (header or body) wins; else the body decode's own
// code (an arena overflow), else a name-arena overflow
__global__ void final_kernel(kx_status* st, const uint64_t* offsets, uint64_t n, unsigned long long* errkey,
                             uint32_t* overflow, const kx_status* pre) {
  if (threadIdx.x != 0) return;
  const unsigned long long k = *errkey;
  if (pre && pre->code) {  // a framing error ends the batch at its frame
    st->code = pre->code;
    st->record = pre->record;
    st->offset = pre->offset;
    st->n_records = n;
    st->consumed = pre->offset;
    *errkey = ~0ull;
    *overflow = 0;
    return;
  }
  if (k != ~0ull) {
    st->code = (int32_t)(k & 0xff);
    st->record = k >> 8;
    st->offset = offsets[k >> 8];
  } else if (st->code != KX_ERR_SIZE_LIMIT && st->code != KX_ERR_INTERNAL) {
    st->code = 0;
    st->record = 0;
    st->offset = 0;
  }
  if (*overflow && st->code == 0) st->code = KX_ERR_SIZE_LIMIT;
  st->n_records = n;
  st->consumed = offsets[n];
  *errkey = ~0ull;
  *overflow = 0;
}

// message workspace: [0] errkey, [8] overflow, then req_start, req_end, name_pos, name_len, hdr_rc, body_rc,
// the name scan's block sums
struct MsgWs {
  size_t req_start, req_end, name_pos, name_len, hdr_rc, body_rc, name_bsum, total;
};

MsgWs msg_ws(uint64_t n) {
  MsgWs L{};
  size_t o = 256;
  auto take = [&](size_t bytes) { const size_t at = o; o += (bytes + 255) & ~(size_t)255; return at; };
  L.req_start = take((n + 1) * 8);
  L.req_end = take((n + 1) * 8);
  L.name_pos = take((n + 1) * 8);
  L.name_len = take((n + 1) * 8);
  L.hdr_rc = take(n + 1);
  L.body_rc = take(n + 1);
  L.name_bsum = take(((n + 1 + SB - 1) / SB) * 8);
  L.total = o;
  return L;
}

}  // namespace

size_t kx_message_ws_bytes(uint64_t n) { return msg_ws(n).total; }

int kx_launch_message_headers(const uint8_t* in, uint64_t in_len, const uint64_t* offsets, uint64_t n,
                              int32_t body_field, bool pb, const KxMsgOut& mo, void* mws, uint64_t** req_start,
                              uint64_t** req_end, uint8_t** hdr_rc, uint8_t** body_rc, hipStream_t stream,
                              const uint64_t* ends, const kx_status* pre, const uint8_t* pre_rc,
                              const uint8_t* raw_flags, int raw) {
  const MsgWs L = msg_ws(n);
  char* b = (char*)mws;
  MsgParams mp{};
  mp.in = in; mp.in_len = in_len; mp.offsets = offsets; mp.n = n; mp.body_field = body_field; mp.mo = mo;
  mp.ends = ends; mp.pre = pre; mp.pre_rc = pre_rc;
  mp.raw = raw; mp.raw_flags = raw_flags;
  mp.pb = pb;
  mp.req_start = (uint64_t*)(b + L.req_start);
  mp.req_end = (uint64_t*)(b + L.req_end);
  mp.name_pos = (uint64_t*)(b + L.name_pos);
  mp.name_len = (uint64_t*)(b + L.name_len);
  mp.hdr_rc = (uint8_t*)(b + L.hdr_rc);
  mp.errkey = (unsigned long long*)b;
  mp.overflow = (uint32_t*)(b + 8);
  const unsigned grid = (unsigned)((n + 1 + MT - 1) / MT);
  hipLaunchKernelGGL(header_kernel, dim3(grid), dim3(MT), 0, stream, mp);
  KX_HIP_CHECK(hipGetLastError());
  {
    const uint64_t nb = (n + 1 + SB - 1) / SB;
    uint64_t* bs = (uint64_t*)(b + L.name_bsum);
    hipLaunchKernelGGL(scan_bsum_kernel, dim3((unsigned)nb), dim3(MT), 0, stream, mp.name_len, n + 1, bs);
    KX_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(scan_bases_kernel, dim3(1), dim3(ST), 0, stream, bs, nb);
    KX_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(scan_apply_kernel, dim3((unsigned)nb), dim3(MT), 0, stream, mp.name_len, n + 1, bs);
    KX_HIP_CHECK(hipGetLastError());
  }
  hipLaunchKernelGGL(name_kernel, dim3(grid), dim3(MT), 0, stream, mp);
  KX_HIP_CHECK(hipGetLastError());
  *req_start = mp.req_start;
  *req_end = mp.req_end;
  *hdr_rc = mp.hdr_rc;
  *body_rc = (uint8_t*)(b + L.body_rc);
  return KX_OK;
}

int kx_launch_set_seqids(uint8_t* in, uint64_t in_len, const uint64_t* offsets, uint64_t n, const int32_t* seqids,
                         uint8_t* record_status, kx_status* status, void* mws, hipStream_t stream) {
  unsigned long long* errkey = (unsigned long long*)mws;
  uint32_t* overflow = (uint32_t*)((char*)mws + 8);
  const unsigned grid = (unsigned)((n + MT - 1) / MT);
  if (grid) {
    hipLaunchKernelGGL(setseq_kernel, dim3(grid), dim3(MT), 0, stream, in, in_len, offsets, n, seqids, record_status,
                       errkey);
    KX_HIP_CHECK(hipGetLastError());
  }
  KX_HIP_CHECK(hipMemsetAsync(status, 0, sizeof(kx_status), stream));
  hipLaunchKernelGGL(final_kernel, dim3(1), dim3(64), 0, stream, status, offsets, n, errkey, overflow,
                     (const kx_status*)nullptr);
  KX_HIP_CHECK(hipGetLastError());
  return KX_OK;
}

int kx_launch_message_encode(const uint8_t* bodies, const uint64_t* body_off, uint64_t scratch_cap, uint64_t n,
                             const uint8_t* name,
                             uint32_t name_len, int32_t msg_type, const int32_t* seqids, int32_t body_field,
                             uint8_t* out, uint64_t out_cap, uint64_t* offsets_out, kx_status* status,
                             hipStream_t stream) {
  MsgEnc me{bodies, body_off, scratch_cap, n, name, name_len, msg_type, seqids, body_field, out, out_cap, offsets_out, status};
  const unsigned grid = (unsigned)((n + 1 + MT - 1) / MT);
  hipLaunchKernelGGL(msgenc_kernel, dim3(grid), dim3(MT), 0, stream, me);
  KX_HIP_CHECK(hipGetLastError());
  return KX_OK;
}

int kx_launch_message_merge(const uint64_t* offsets, uint64_t n, const uint8_t* hdr_rc, const uint8_t* body_rc,
                            uint8_t* record_status, kx_status* status, void* mws, hipStream_t stream,
                            const kx_status* pre) {
  unsigned long long* errkey = (unsigned long long*)mws;
  uint32_t* overflow = (uint32_t*)((char*)mws + 8);
  const unsigned grid = (unsigned)((n + MT - 1) / MT);
  hipLaunchKernelGGL(merge_kernel, dim3(grid), dim3(MT), 0, stream, hdr_rc, body_rc, record_status, n, errkey);
  KX_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(final_kernel, dim3(1), dim3(64), 0, stream, status, offsets, n, errkey, overflow, pre);
  KX_HIP_CHECK(hipGetLastError());
  return KX_OK;
}
