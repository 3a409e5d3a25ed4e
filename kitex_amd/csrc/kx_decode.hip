// kx_decode.hip — batched Thrift-binary FastRead (and the skip decoder) on CDNA4 / gfx950.
//
// Reference semantics: generated FastRead (tool/internal_pkg/pluginmode/thriftgo/struct_tpl.go:41-149,
// 405-625; instance internal/mocks/thrift/k-mock.go:39-184) over N records, as fastUnmarshal does per
// message (pkg/remote/codec/thrift/codec_fast.go:60-82) or as the element loop of a list<Struct>;
// unknown / mistyped fields go through the skip decoder (codec_apache.go:191-293).
//
// Design: ONE pass over HBM. A workgroup owns a 32 KiB tile of the input:
//   1. stage the tile (+2 KiB halo) into LDS with 16-byte loads;
//   2. every lane speculatively finds the first canonical record signature in its 128-byte segment
//      and walks records (schema-aware FastRead lengths) until it leaves the segment ("walk 1");
//   3. links between segments are validated in LDS (exit of the previous walking lane == entry);
//   4. the tile aggregate (records, var bytes, speculative entry, exit) is published and a
//      decoupled look-back over predecessor tiles yields the true entry, record base and arena
//      bases; a wrong speculation falls back to a serial walk from the true entry;
//   5. "walk 2" re-parses the tile from LDS and scatters: fixed-width columns are stored as they are
//      parsed (lanes = consecutive records, coalesced), strings / lists are copied at record end.
// Known-offsets mode (fastUnmarshal with dataLen) uses the same pipeline with one record per lane.
// No MFMA anywhere: this is byte movement, bounded by HBM bandwidth.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "kx_internal.h"

#define LDS __attribute__((address_space(3)))
#define GLB __attribute__((address_space(1)))

namespace {

constexpr int NT = 256;                 // threads per workgroup (4 waves)
constexpr int SEG = 128;                // bytes per lane segment
constexpr int TILE = NT * SEG;          // 32 KiB of input per workgroup
constexpr int HALO = 512;               // records straddling the tile end are read from LDS up to here
constexpr int WINB = TILE + HALO + 16;  // LDS window bytes (16 for the aligned-down start)
constexpr int WIN_CHUNKS = WINB / 16;
constexpr int DSTRIDE = 24;             // u64 words per tile descriptor

constexpr uint64_t X_ERR = ~0ull;       // chain terminated by a decode error
constexpr uint64_t X_DONE = ~0ull - 1;  // chain reached n records
constexpr uint64_t X_NONE = ~0ull - 2;  // no candidate in this tile / lane

// descriptor words
constexpr int D_AGG_CNT = 0, D_AGG_ENT = 1, D_AGG_EXIT = 2, D_AGG_VAR = 3;
constexpr int D_INC_CNT = 11, D_INC_EXIT = 12, D_INC_VAR = 13;

enum Mode { M_THRIFT = 0, M_SKIP = 1 };

// opt-in phase timing (KX_PHASE_TIMING=1): cycles per phase summed over tiles, lane 0 of wave 0
__device__ unsigned long long g_phase[10];

struct DecParams {
  const uint8_t* in;
  uint64_t in_len;
  const uint64_t* offsets;   // known-offsets mode when non-null
  uint64_t n;
  const KxProgram* prog;
  KxLaunchCols cols;
  uint8_t* rstat;
  kx_status* status;
  uint64_t* skip_out;        // M_SKIP: record start offsets
  uint32_t* counter;         // dynamic tile counter
  uint32_t* flags;           // per-tile look-back flag
  uint64_t* desc;            // per-tile look-back payload
  unsigned long long* errkey;  // offsets mode: min((record << 8) | code)
  uint32_t* overflow;        // an arena capacity was exceeded
  uint64_t ntiles;
  int timing;
  int ablate;   // diagnostics only (KX_ABLATE): 1 no walk2, 2 no var copies, 4 walk2 without stores, 8 no walk1
};

// ---------------------------------------------------------------------------------------------
// byte access: LDS window first, global memory (aligned dword loads, never past the granule that
// holds the last input byte) for anything outside it.
// ---------------------------------------------------------------------------------------------
struct Win {
  const uint8_t* in;
  uint64_t in_len;
  uint64_t wlo;        // absolute address of LDS byte 0 (16-aligned)
  uint32_t wlen;       // bytes valid in LDS
  const LDS uint32_t* lds;
  const KxpStep* steps;  // canonical plan (global memory; uniform index -> scalar loads)
  uint32_t nsteps;
  uint64_t canon_pres;
};

__device__ __forceinline__ uint32_t gld4(const Win& w, uint64_t p) {
  uint64_t a = (uint64_t)w.in + p;
  uint64_t A = a & ~3ull;
  uint32_t sh = (uint32_t)(a & 3);
  uint64_t end = (uint64_t)w.in + w.in_len;
  uint32_t x0 = A < end ? *(const GLB uint32_t*)A : 0u;
  uint32_t x1 = A + 4 < end ? *(const GLB uint32_t*)(A + 4) : 0u;
  return __builtin_amdgcn_alignbyte(x1, x0, sh);
}

// 4 bytes starting at input offset p, byte p in bits 0..7
__device__ __forceinline__ uint32_t ld4(const Win& w, uint64_t p) {
  uint64_t r = (uint64_t)w.in + p - w.wlo;
  if (r + 4 <= w.wlen) {
    uint32_t q = (uint32_t)r >> 2, sh = (uint32_t)r & 3;
    return __builtin_amdgcn_alignbyte(w.lds[q + 1], w.lds[q], sh);
  }
  return gld4(w, p);
}

__device__ __forceinline__ uint32_t ld1(const Win& w, uint64_t p) {
  uint64_t r = (uint64_t)w.in + p - w.wlo;
  if (r < w.wlen) return ((const LDS uint8_t*)w.lds)[r];
  return ((const GLB uint8_t*)w.in)[p];
}

__device__ __forceinline__ uint32_t be32(const Win& w, uint64_t p) { return __builtin_bswap32(ld4(w, p)); }
__device__ __forceinline__ uint64_t be64(const Win& w, uint64_t p) {
  return ((uint64_t)be32(w, p) << 32) | be32(w, p + 4);
}

__device__ __forceinline__ int tsize(uint32_t t) {
  // typeToSize (codec_apache.go:182-189)
  switch (t) {
    case KX_T_BOOL: case KX_T_BYTE: return 1;
    case KX_T_I16: return 2;
    case KX_T_I32: return 4;
    case KX_T_DOUBLE: case KX_T_I64: return 8;
    default: return 0;
  }
}

// scalar in host order from its big-endian wire bytes (BOOL: b == 1, parity unpinned)
__device__ __forceinline__ uint64_t load_scalar(const Win& w, uint64_t p, uint32_t t) {
  switch (t) {
    case KX_T_BOOL: return ld1(w, p) == 1 ? 1u : 0u;
    case KX_T_BYTE: return ld1(w, p);
    case KX_T_I16: { uint32_t x = ld4(w, p); return ((x & 0xff) << 8) | ((x >> 8) & 0xff); }
    case KX_T_I32: return be32(w, p);
    default: return be64(w, p);
  }
}

// ---------------------------------------------------------------------------------------------
// skip decoder: netpollSkipDecoder.skipType (codec_apache.go:191-293), iterative with an explicit
// frame stack (rare path; lives in scratch). Frame: t:4 kt:4 vt:4 st:2 ph:1 md:7 | rem:31 << 32.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t canon_t(uint32_t t) {
  switch (t) {
    case KX_T_BOOL: case KX_T_BYTE: case KX_T_DOUBLE: case KX_T_I16: case KX_T_I32: case KX_T_I64:
    case KX_T_STRING: case KX_T_STRUCT: case KX_T_MAP: case KX_T_SET: case KX_T_LIST: return t;
    default: return 1;  // any invalid id (also STOP) -> "unknown data type"
  }
}

__device__ __forceinline__ int dskip_body(const Win& w, uint64_t& pos, uint64_t limit, uint32_t t0, int md0) {
  uint64_t stk[66];
  int sp = 0;
  auto mk = [](uint32_t t, uint32_t md) -> uint64_t { return (uint64_t)(canon_t(t) | (md << 15)); };
  stk[sp++] = mk(t0, (uint32_t)md0);
  while (sp > 0) {
    uint64_t fr = stk[sp - 1];
    uint32_t t = fr & 15, kt = (fr >> 4) & 15, vt = (fr >> 8) & 15, st = (fr >> 12) & 3;
    uint32_t ph = (fr >> 14) & 1, md = (fr >> 15) & 127;
    uint32_t rem = (uint32_t)(fr >> 32);
    if (st == 0) {
      if (md == 0) return KX_ERR_DEPTH_LIMIT;
      int sz = tsize(t);
      if (sz > 0) {
        if (limit - pos < (uint64_t)sz) return KX_ERR_EOF;
        pos += sz; sp--; continue;
      }
      switch (t) {
        case KX_T_STRING: {
          if (limit - pos < 4) return KX_ERR_EOF;
          int32_t l = (int32_t)be32(w, pos);
          if (l < 0) return KX_ERR_INVALID_DATA;
          if (limit - pos - 4 < (uint64_t)l) return KX_ERR_EOF;
          pos += 4 + (uint64_t)l; sp--; continue;
        }
        case KX_T_STRUCT:
          stk[sp - 1] = (fr & ~(3ull << 12)) | (1ull << 12); continue;
        case KX_T_MAP: {
          if (limit - pos < 6) return KX_ERR_EOF;
          uint32_t h = ld4(w, pos);
          uint32_t k = h & 0xff, v = (h >> 8) & 0xff;
          int32_t cnt = (int32_t)be32(w, pos + 2);
          if (cnt < 0) return KX_ERR_INVALID_DATA;
          int ks = tsize(k), vs = tsize(v);
          if (ks > 0 && vs > 0) {
            uint64_t b = (uint64_t)cnt * (uint64_t)(ks + vs);
            if (limit - pos - 6 < b) return KX_ERR_EOF;
            pos += 6 + b; sp--; continue;
          }
          pos += 6;
          stk[sp - 1] = (uint64_t)t | ((uint64_t)canon_t(k) << 4) | ((uint64_t)canon_t(v) << 8) |
                        (3ull << 12) | ((uint64_t)md << 15) | ((uint64_t)(uint32_t)cnt << 32);
          continue;
        }
        case KX_T_SET: case KX_T_LIST: {
          if (limit - pos < 5) return KX_ERR_EOF;
          uint32_t v = ld1(w, pos);
          int32_t cnt = (int32_t)be32(w, pos + 1);
          if (cnt < 0) return KX_ERR_INVALID_DATA;
          int vs = tsize(v);
          if (vs > 0) {
            uint64_t b = (uint64_t)cnt * (uint64_t)vs;
            if (limit - pos - 5 < b) return KX_ERR_EOF;
            pos += 5 + b; sp--; continue;
          }
          pos += 5;
          stk[sp - 1] = (uint64_t)t | ((uint64_t)canon_t(v) << 8) | (2ull << 12) | ((uint64_t)md << 15) |
                        ((uint64_t)(uint32_t)cnt << 32);
          continue;
        }
        default:
          return KX_ERR_INVALID_DATA;
      }
    } else if (st == 1) {  // struct field loop
      if (limit - pos < 1) return KX_ERR_EOF;
      uint32_t tp = ld1(w, pos);
      pos += 1;
      if (tp == KX_T_STOP) { sp--; continue; }
      int fsz = tsize(tp);
      if (fsz > 0) {
        if (limit - pos < 2 + (uint64_t)fsz) return KX_ERR_EOF;
        pos += 2 + fsz; continue;
      }
      if (limit - pos < 2) return KX_ERR_EOF;
      pos += 2;
      stk[sp++] = mk(tp, md - 1);
    } else if (st == 2) {  // list / set elements
      if (rem == 0) { sp--; continue; }
      stk[sp - 1] = (fr & 0xffffffffull) | ((uint64_t)(rem - 1) << 32);
      stk[sp++] = mk(vt, md - 1);
    } else {  // map: key then value
      if (rem == 0) { sp--; continue; }
      uint32_t et = ph ? vt : kt;
      uint64_t nf = ph ? ((fr & ~(1ull << 14)) & 0xffffffffull) | ((uint64_t)(rem - 1) << 32)
                       : (fr | (1ull << 14));
      stk[sp - 1] = nf;
      int es = tsize(et);
      if (es > 0) {  // fixed-size element: skipn (only reached when the other side is not)
        if (limit - pos < (uint64_t)es) return KX_ERR_EOF;
        pos += es;
      } else {
        stk[sp++] = mk(et, md - 1);
      }
    }
  }
  return KX_OK;
}

struct SkipRes {
  uint64_t pos;
  int rc;
};

// (pos is passed and returned by value: a reference would pin the caller's loop-carried position
// to scratch memory)
__device__ __noinline__ SkipRes dskip_v(const Win w, uint64_t pos, uint64_t limit, uint32_t t0, int md0) {
  int rc_ = dskip_body(w, pos, limit, t0, md0);
  return SkipRes{pos, rc_};
}

__device__ __forceinline__ int dskip(const Win& w, uint64_t& pos, uint64_t limit, uint32_t t0, int md0) {
  SkipRes r = dskip_v(w, pos, limit, t0, md0);
  pos = r.pos;
  return r.rc;
}


// ---------------------------------------------------------------------------------------------
// per-record FastRead. EMIT=false: measure (length, var lengths); EMIT=true: also store columns.
// ---------------------------------------------------------------------------------------------

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// struct reads from the LDS-resident program (no implicit copy across address spaces)
__device__ __forceinline__ KxpField ld_field(const LDS KxProgram* P, int i) {
  u32x4 v = *(const LDS u32x4*)&P->f[i];
  KxpField F;
  __builtin_memcpy(&F, &v, sizeof F);
  return F;
}
__device__ __forceinline__ KxpInst ld_inst(const LDS KxProgram* P, int i) {
  u32x4 v[2];
  v[0] = ((const LDS u32x4*)&P->inst[i])[0];
  v[1] = ((const LDS u32x4*)&P->inst[i])[1];
  KxpInst I;
  __builtin_memcpy(&I, v, sizeof I);
  return I;
}
__device__ __forceinline__ KxpCol ld_col(const LDS KxProgram* P, int i) {
  u32x4 v = *(const LDS u32x4*)&P->col[i];
  KxpCol K;
  __builtin_memcpy(&K, &v, sizeof K);
  return K;
}

template <int NV>
struct VarState {
  uint64_t pos[NV > 0 ? NV : 1];
  uint32_t len[NV > 0 ? NV : 1];
};

template <int NV>
__device__ __forceinline__ void vset(VarState<NV>& v, uint32_t slot, uint64_t p, uint32_t l) {
#pragma unroll
  for (int i = 0; i < NV; i++)
    if ((uint32_t)i == slot) { v.pos[i] = p; v.len[i] = l; }
}

struct Shared;  // fwd

__device__ __forceinline__ void store_col(void* base, uint32_t width, uint64_t rec, uint64_t v) {
  switch (width) {
    case 1: ((GLB uint8_t*)base)[rec] = (uint8_t)v; break;
    case 2: ((GLB uint16_t*)base)[rec] = (uint16_t)v; break;
    case 4: ((GLB uint32_t*)base)[rec] = (uint32_t)v; break;
    default: ((GLB uint64_t*)base)[rec] = v; break;
  }
}

// 12 wire bytes starting at p, byte p in bits 0..7 of w0: one LDS round trip (4 independent
// ds_read_b32 + v_alignbyte) when the bytes are in the window, global dword loads otherwise.
struct Fetch {
  uint32_t w0, w1, w2;
};

__device__ __forceinline__ Fetch fetch12(const Win& w, uint64_t p) {
  uint64_t r = (uint64_t)w.in + p - w.wlo;
  Fetch f;
  if (r + 16 <= w.wlen) {
    uint32_t q = (uint32_t)r >> 2, sh = (uint32_t)r & 3;
    uint32_t x0 = w.lds[q], x1 = w.lds[q + 1], x2 = w.lds[q + 2], x3 = w.lds[q + 3];
    f.w0 = __builtin_amdgcn_alignbyte(x1, x0, sh);
    f.w1 = __builtin_amdgcn_alignbyte(x2, x1, sh);
    f.w2 = __builtin_amdgcn_alignbyte(x3, x2, sh);
  } else {
    f.w0 = ld4(w, p);
    f.w1 = ld4(w, p + 4);
    f.w2 = ld4(w, p + 8);
  }
  return f;
}

// fetch12 for a window byte offset already known to be inside the window (no branch)
__device__ __forceinline__ Fetch fetch12_lds(const Win& w, uint32_t r) {
  uint32_t q = r >> 2, sh = r & 3;
  uint32_t x0 = w.lds[q], x1 = w.lds[q + 1], x2 = w.lds[q + 2], x3 = w.lds[q + 3];
  Fetch f;
  f.w0 = __builtin_amdgcn_alignbyte(x1, x0, sh);
  f.w1 = __builtin_amdgcn_alignbyte(x2, x1, sh);
  f.w2 = __builtin_amdgcn_alignbyte(x3, x2, sh);
  return f;
}

// the field value that follows a 3-byte field header (wire bytes p+3 ...), host order
__device__ __forceinline__ uint64_t fixed_after_header(const Fetch& f, uint32_t t) {
  switch (t) {
    case KX_T_BOOL: return (f.w0 >> 24) == 1 ? 1u : 0u;
    case KX_T_BYTE: return f.w0 >> 24;
    case KX_T_I16: return ((f.w0 >> 24) << 8) | (f.w1 & 0xff);
    case KX_T_I32: return __builtin_bswap32(__builtin_amdgcn_alignbyte(f.w1, f.w0, 3));
    default:
      return ((uint64_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(f.w1, f.w0, 3)) << 32) |
             __builtin_bswap32(__builtin_amdgcn_alignbyte(f.w2, f.w1, 3));
  }
}

// Canonical fast path: the record is checked against the schema's canonical plan (header bytes in
// encoder order, STOP bytes) step by step; the step is wave-uniform, so the only divergence is a
// lane whose record deviates, which returns false and is re-parsed by the generic loop below.
template <int NV, bool EMIT>
__device__ __forceinline__ bool canon_record(const Win& w, void* const LDS* colp, uint64_t start, uint64_t limit,
                                             uint64_t rec, uint64_t* endp, VarState<NV>& vs, uint64_t& pres) {
  uint64_t pos = start;
  const KxpStep* __restrict__ steps = w.steps;
  uint32_t k = 0;
  while (k < w.nsteps) {
    const KxpStep st = steps[k];
    const uint64_t rem = limit - pos;
    if (st.kind == KXP_S_FIXED) {
      // up to 4 consecutive fixed-width fields: positions are known without waiting for data, so
      // all their bytes are fetched in one LDS round trip
      const uint32_t m = min(st.hdr >> 24, 4u);
      const KxpStep s1 = steps[k + (m > 1 ? 1 : 0)];
      const KxpStep s2 = steps[k + (m > 2 ? 2 : 0)];
      const KxpStep s3 = steps[k + (m > 3 ? 3 : 0)];
      const uint32_t o1 = 3 + st.width, o2 = o1 + 3 + s1.width, o3 = o2 + 3 + s2.width;
      const uint32_t len = m == 1 ? o1 : m == 2 ? o2 : m == 3 ? o3 : o3 + 3 + s3.width;
      if (rem < len) return false;
      const uint64_t r = (uint64_t)w.in + pos - w.wlo;
      Fetch f0, f1, f2, f3;
      if (r + o3 + 16 <= w.wlen) {
        f0 = fetch12_lds(w, (uint32_t)r);
        f1 = fetch12_lds(w, (uint32_t)r + o1);
        f2 = fetch12_lds(w, (uint32_t)r + o2);
        f3 = fetch12_lds(w, (uint32_t)r + o3);
      } else {
        f0 = fetch12(w, pos);
        f1 = fetch12(w, pos + o1);
        f2 = fetch12(w, pos + o2);
        f3 = fetch12(w, pos + o3);
      }
      bool ok = (f0.w0 & 0xffffffu) == (st.hdr & 0xffffffu);
      if (m > 1) ok &= (f1.w0 & 0xffffffu) == (s1.hdr & 0xffffffu);
      if (m > 2) ok &= (f2.w0 & 0xffffffu) == (s2.hdr & 0xffffffu);
      if (m > 3) ok &= (f3.w0 & 0xffffffu) == (s3.hdr & 0xffffffu);
      if (!ok) return false;
      if (EMIT) {
        store_col(colp[st.col], st.width, rec, fixed_after_header(f0, st.hdr & 0xff));
        if (m > 1) store_col(colp[s1.col], s1.width, rec, fixed_after_header(f1, s1.hdr & 0xff));
        if (m > 2) store_col(colp[s2.col], s2.width, rec, fixed_after_header(f2, s2.hdr & 0xff));
        if (m > 3) store_col(colp[s3.col], s3.width, rec, fixed_after_header(f3, s3.hdr & 0xff));
      }
      pos += len;
      k += m;
      continue;
    }
    const Fetch fx = fetch12(w, pos);
    k++;
    if (st.kind == KXP_S_END) {
      if (rem < 1 || (fx.w0 & 0xff) != KX_T_STOP) return false;
      pos += 1;
      continue;
    }
    if (rem < 3 || (fx.w0 & 0xffffffu) != (st.hdr & 0xffffffu)) return false;
    const uint64_t vp = pos + 3, vrem = rem - 3;
    if (st.kind == KXP_S_BYTES) {
      if (vrem < 4) return false;
      const int32_t l = (int32_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(fx.w1, fx.w0, 3));
      if (l < 0 || vrem - 4 < (uint64_t)l) return false;
      vset<NV>(vs, st.vslot, vp + 4, (uint32_t)l);
      pos = vp + 4 + (uint64_t)l;
    } else if (st.kind == KXP_S_LIST) {
      if (vrem < 5) return false;
      const int32_t l = (int32_t)__builtin_bswap32(fx.w1);
      const uint64_t b = (uint64_t)(l < 0 ? 0 : l) * st.width;
      if (l < 0 || vrem - 5 < b) return false;
      vset<NV>(vs, st.vslot, vp + 5, (uint32_t)l);
      pos = vp + 5 + b;
    } else {  // KXP_S_STRUCT: header only, its fields follow
      pos = vp;
    }
  }
  pres = w.canon_pres;
  *endp = pos;
  return true;
}

// One record's FastRead. EMIT=false: measure (length, var lengths); EMIT=true: also store the
// fixed-width columns as they are parsed. In canonical order every field costs one LDS round trip:
// the 12 bytes at the cursor and the predicted field descriptor are fetched together.
template <int NV, bool EMIT>
__device__ int thrift_record(const Win& w, const LDS KxProgram* P, void* const LDS* colp, uint64_t start,
                             uint64_t limit, uint64_t rec, uint64_t* endp, VarState<NV>& vs,
                             uint64_t& pres) {
#pragma unroll
  for (int i = 0; i < NV; i++) { vs.len[i] = 0; vs.pos[i] = 0; }
  if (w.nsteps && canon_record<NV, EMIT>(w, colp, start, limit, rec, endp, vs, pres)) return KX_OK;
#pragma unroll
  for (int i = 0; i < NV; i++) { vs.len[i] = 0; vs.pos[i] = 0; }
  uint64_t pos = start;
  int inst = 0;
  int pred = P->inst[0].enc_first;
  uint64_t seen = 0;
  pres = 0;
  for (;;) {
    if (pos >= limit) return KX_ERR_EOF;
    const Fetch fx = fetch12(w, pos);
    KxpField F = ld_field(P, pred >= 0 ? pred : 0);
    const uint32_t t = fx.w0 & 0xff;
    if (t == KX_T_STOP) {
      pos += 1;
      uint64_t rq = P->inst[inst].req_mask;
      if ((seen & rq) != rq) return KX_ERR_INVALID_DATA;   // RequiredFieldNotSetError
      if (inst == 0) break;
      pred = P->inst[inst].ret_pred;
      inst = P->inst[inst].parent;
      continue;
    }
    if (limit - pos < 3) return KX_ERR_EOF;
    const int id = (int)(int16_t)((((fx.w0 >> 8) & 0xffu) << 8) | ((fx.w0 >> 16) & 0xffu));
    int fi = -1;
    if (pred >= 0 && F.id == id) {
      fi = pred;
    } else {
      int f0 = P->inst[inst].first, nf = P->inst[inst].nfields;
      for (int k = 0; k < nf; k++)
        if (P->f[f0 + k].id == id) { fi = f0 + k; break; }
      if (fi >= 0) F = ld_field(P, fi);
    }
    const uint64_t vp = pos + 3;
    if (fi < 0 || F.ttype != t) {                            // default: / mismatched type -> Skip
      SkipRes r = dskip_v(w, vp, limit, t, 64);
      if (r.rc) return r.rc;
      pos = r.pos;
      continue;
    }
    pred = F.enc_next;
    if (F.kind == KXP_K_FIXED) {
      const uint32_t wd = F.width;
      if (limit - vp < wd) return KX_ERR_EOF;
      if (EMIT) store_col(colp[F.col], wd, rec, fixed_after_header(fx, t));
      pos = vp + wd;
    } else if (F.kind == KXP_K_BYTES) {                      // ReadString (copies)
      if (limit - vp < 4) return KX_ERR_EOF;
      const int32_t l = (int32_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(fx.w1, fx.w0, 3));
      if (l < 0) return KX_ERR_NEGATIVE_SIZE;
      if (limit - vp - 4 < (uint64_t)l) return KX_ERR_EOF;
      vset<NV>(vs, F.vslot, vp + 4, (uint32_t)l);
      pos = vp + 4 + (uint64_t)l;
    } else if (F.kind == KXP_K_LIST) {                       // ReadListBegin: elem type ignored
      if (limit - vp < 5) return KX_ERR_EOF;
      const int32_t l = (int32_t)__builtin_bswap32(fx.w1);
      if (l < 0) return KX_ERR_NEGATIVE_SIZE;
      const uint64_t b = (uint64_t)l * F.width;
      if (limit - vp - 5 < b) return KX_ERR_EOF;
      vset<NV>(vs, F.vslot, vp + 5, (uint32_t)l);
      pos = vp + 5 + b;
    } else {                                                 // nested struct: NewX() + FastRead
      const KxpInst C = ld_inst(P, F.child);
      seen &= ~C.subtree_mask;
      pres &= ~C.pres_mask;
#pragma unroll
      for (int i = 0; i < NV; i++)
        if ((C.vslot_mask >> i) & 1) vs.len[i] = 0;
      seen |= 1ull << fi;
      if (F.pbit >= 0) pres |= 1ull << F.pbit;
      inst = F.child;
      pred = C.enc_first;
      pos = vp;
      continue;
    }
    seen |= 1ull << fi;
    if (F.pbit >= 0) pres |= 1ull << F.pbit;
  }
  if (EMIT) {
    // fields never seen (or reset by a repeated struct field) take their default
    for (uint32_t c = 0; c < P->ncols; c++) {
      const KxpCol K = ld_col(P, c);
      if (K.kind == KXP_K_FIXED && !((seen >> K.field) & 1)) store_col(colp[c], K.width, rec, (uint64_t)K.defv);
    }
  }
  *endp = pos;
  return KX_OK;
}

template <int NV>
__device__ void emit_defaults(const LDS KxProgram* P, void* const LDS* colp, uint64_t rec) {
  for (uint32_t c = 0; c < P->ncols; c++) {
    const KxpCol K = ld_col(P, c);
    if (K.kind == KXP_K_FIXED) store_col(colp[c], K.width, rec, (uint64_t)K.defv);
  }
}

// copy one var field payload (n units of `width` bytes) from the input to its arena
__device__ void copy_var_slow(const Win& w, const KxpCol& K, uint64_t src, uint32_t n, uint8_t* dst_) {
  GLB uint8_t* dst = (GLB uint8_t*)dst_;
  if (K.kind == KXP_K_BYTES) {
    uint32_t i = 0;
    while (i < n && (((uintptr_t)(dst_ + i)) & 3)) { dst[i] = (uint8_t)ld1(w, src + i); i++; }
    for (; i + 4 <= n; i += 4) *(GLB uint32_t*)(dst + i) = ld4(w, src + i);
    for (; i < n; i++) dst[i] = (uint8_t)ld1(w, src + i);
    return;
  }
  switch (K.width) {
    case 1:
      for (uint32_t i = 0; i < n; i++) {
        uint32_t b = ld1(w, src + i);
        dst[i] = (uint8_t)(K.elem == KX_T_BOOL ? (b == 1) : b);
      }
      break;
    case 2:
      for (uint32_t i = 0; i < n; i++) {
        uint32_t x = ld4(w, src + 2ull * i);
        ((GLB uint16_t*)dst)[i] = (uint16_t)(((x & 0xff) << 8) | ((x >> 8) & 0xff));
      }
      break;
    case 4:
      for (uint32_t i = 0; i < n; i++) ((GLB uint32_t*)dst)[i] = be32(w, src + 4ull * i);
      break;
    default:
      for (uint32_t i = 0; i < n; i++) ((GLB uint64_t*)dst)[i] = be64(w, src + 8ull * i);
      break;
  }
}

// Fast path: the payload is inside the LDS window. 16 output bytes per step: 5 independent LDS
// dwords, v_alignbyte to the source skew, byte swap for big-endian elements, one 16-byte store
// when the destination allows it.
__device__ void copy_var(const Win& w, const KxpCol& K, uint64_t src, uint32_t n, uint8_t* dst_) {
  const uint64_t nbytes = (uint64_t)n * K.width;
  const uint64_t r = (uint64_t)w.in + src - w.wlo;
  const bool bswap = K.kind == KXP_K_LIST && K.width > 1;
  if (r + nbytes + 20 > w.wlen || (K.kind == KXP_K_LIST && K.elem == KX_T_BOOL)) {
    copy_var_slow(w, K, src, n, dst_);
    return;
  }
  GLB uint8_t* dst = (GLB uint8_t*)dst_;
  uint32_t i = 0;
  if (!bswap) {
    while (i < nbytes && (((uintptr_t)(dst_ + i)) & 15)) {
      dst[i] = ((const LDS uint8_t*)w.lds)[r + i];
      i++;
    }
  } else if (((uintptr_t)dst_) & 3) {
    copy_var_slow(w, K, src, n, dst_);
    return;
  }
  const bool a16 = ((((uintptr_t)dst_) + i) & 15) == 0;
  const uint32_t sh = (uint32_t)((r + i) & 3);
  uint32_t q = (uint32_t)((r + i) >> 2);
  for (; i + 16 <= nbytes; i += 16, q += 4) {
    uint32_t x0 = w.lds[q], x1 = w.lds[q + 1], x2 = w.lds[q + 2], x3 = w.lds[q + 3], x4 = w.lds[q + 4];
    uint32_t a0 = __builtin_amdgcn_alignbyte(x1, x0, sh), a1 = __builtin_amdgcn_alignbyte(x2, x1, sh);
    uint32_t a2 = __builtin_amdgcn_alignbyte(x3, x2, sh), a3 = __builtin_amdgcn_alignbyte(x4, x3, sh);
    if (bswap) {
      if (K.width == 8) {
        uint32_t t0 = __builtin_bswap32(a1), t1 = __builtin_bswap32(a0);
        uint32_t t2 = __builtin_bswap32(a3), t3 = __builtin_bswap32(a2);
        a0 = t0; a1 = t1; a2 = t2; a3 = t3;
      } else if (K.width == 4) {
        a0 = __builtin_bswap32(a0); a1 = __builtin_bswap32(a1);
        a2 = __builtin_bswap32(a2); a3 = __builtin_bswap32(a3);
      } else {
        a0 = __builtin_amdgcn_perm(a0, a0, 0x02030001u); a1 = __builtin_amdgcn_perm(a1, a1, 0x02030001u);
        a2 = __builtin_amdgcn_perm(a2, a2, 0x02030001u); a3 = __builtin_amdgcn_perm(a3, a3, 0x02030001u);
      }
    }
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    if (a16) {
      v4u v = {a0, a1, a2, a3};
      *(GLB v4u*)(dst + i) = v;
    } else {
      GLB uint32_t* d32 = (GLB uint32_t*)(dst + i);
      d32[0] = a0; d32[1] = a1; d32[2] = a2; d32[3] = a3;
    }
  }
  if (i < nbytes) {
    if (bswap) {
      copy_var_slow(w, K, src + i, (uint32_t)((nbytes - i) / K.width), dst_ + i);
    } else {
      for (; i + 4 <= nbytes; i += 4, q++)
        *(GLB uint32_t*)(dst + i) = __builtin_amdgcn_alignbyte(w.lds[q + 1], w.lds[q], sh);
      for (; i < nbytes; i++) dst[i] = ((const LDS uint8_t*)w.lds)[r + i];
    }
  }
}


// First canonical record signature (3 bytes) in a lane's 128-byte segment: the segment (plus the
// 2 bytes a match may straddle) is read with 9 x ds_read_b128 + 1 x ds_read_b32 in one round trip
// and searched in registers, byte-equality SWAR on the first signature byte.
__device__ __forceinline__ uint64_t scan_segment(const LDS uint32_t* win, uint32_t r0w, uint64_t seg_lo,
                                                 uint64_t plim, uint32_t sig) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const uint32_t skew = r0w & 15;
  const LDS v4u* src = (const LDS v4u*)(win + ((r0w & ~15u) >> 2));
  uint32_t d[37];
#pragma unroll
  for (int i = 0; i < 9; i++) {
    v4u v = src[i];
    d[4 * i] = v.x; d[4 * i + 1] = v.y; d[4 * i + 2] = v.z; d[4 * i + 3] = v.w;
  }
  d[36] = ((const LDS uint32_t*)src)[36];
  const uint64_t base = seg_lo - skew;  // input position of d[0] byte 0
  const uint32_t b0 = (sig & 0xff) * 0x01010101u;
  uint64_t found = ~0ull - 2;
  bool done = false;
#pragma unroll
  for (int i = 0; i < 36; i++) {
    const uint32_t t = d[i] ^ b0;
    uint32_t z = (t - 0x01010101u) & ~t & 0x80808080u;   // bytes equal to the first sig byte
    if (!done && z) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint64_t pp = base + 4 * i + j;
        if (!done && pp >= seg_lo && pp < plim && (__builtin_amdgcn_alignbyte(d[i + 1], d[i], j) & 0xffffffu) == sig) {
          found = pp;
          done = true;
        }
      }
    }
  }
  return found;
}

// ---------------------------------------------------------------------------------------------
// shared memory layout
// ---------------------------------------------------------------------------------------------
struct Shared {
  uint32_t win[WINB / 4 + 4];         // staged input window (+ pad for the q+1 read)
  KxProgram prog;
  void* colp[KX_MAX_COLUMNS];
  uint64_t ent[NT];                   // lane speculative entry / true entry
  uint64_t ext[NT];                   // lane exit
  int32_t scan_i[NT / 64];
  uint64_t scan_u[NT / 64];
  uint64_t red[KXP_NV_MAX + 2];
  // look-back results
  uint64_t e_in, base_cnt, tile_cnt, tile_exit, spec_ent;
  uint64_t base_var[KXP_NV_MAX];
  uint64_t tile_var[KXP_NV_MAX];
  uint32_t tile_id;
  int32_t ok;
  int32_t first_err_lane;
  int32_t changed;
};

// ---- block scans (256 threads = 4 waves) ----
__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

// exclusive block scan; returns the block total through *tot. All threads must call.
__device__ uint64_t block_excl_scan_u64(uint64_t v, uint64_t* tot, uint64_t* scratch) {
  int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t inc = wave_incl_scan_u64(v, lane);
  __syncthreads();
  if (lane == 63) scratch[wv] = inc;
  __syncthreads();
  uint64_t base = 0, t = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; i++) {
    uint64_t s = scratch[i];
    if (i < wv) base += s;
    t += s;
  }
  *tot = t;
  return base + inc - v;
}

// exclusive max-scan of lane indices (-1 when none)
__device__ int block_excl_maxscan_i32(int v, int32_t* scratch) {
  int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int o = __shfl_up(inc, d, 64);
    if (lane >= d) inc = max(inc, o);
  }
  int exc = __shfl_up(inc, 1, 64);
  if (lane == 0) exc = -1;
  __syncthreads();
  if (lane == 63) scratch[wv] = inc;
  __syncthreads();
  int pre = -1;
#pragma unroll
  for (int i = 0; i < NT / 64; i++)
    if (i < wv) pre = max(pre, scratch[i]);
  return max(pre, exc);
}

__device__ __forceinline__ uint32_t aload32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t aload64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void astore64(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void astore32(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// publish a descriptor (one lane): sc1 payload stores, drain, then the flag (Guideline 16 R1)
__device__ void publish(const DecParams& dp, uint64_t t, uint32_t flag, const uint64_t* words, int first,
                        int nwords) {
  uint64_t* d = dp.desc + t * DSTRIDE;
  for (int i = 0; i < nwords; i++) astore64(d + first + i, words[i]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  astore32(dp.flags + t, flag);
}

__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
  uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
  uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t now_ns() { return __builtin_amdgcn_s_memrealtime() * 10; }  // 100 MHz

// Decoupled look-back, executed by wave 0 (64 predecessors per window, newest in lane 0).
// Walks back window by window, summing aggregates, until an inclusive predecessor is found; the
// speculative chain is verified on the way: for consecutive candidate-bearing tiles a < b,
// exit(a) == entry(b), and the inclusive tile's exit equals the entry of the oldest candidate tile
// after it. Tiles without a candidate pass the chain through (implied by the entry check of the
// next candidate tile, or by the caller's own check). Any mismatch: wait for tile t-1 to publish
// its inclusive prefix (it validates itself and repairs by a serial walk).
// Writes S.e_in / S.base_cnt / S.base_var.
template <int NV>
__device__ void lookback(const DecParams& dp, Shared& S, uint64_t t, bool chain) {
  const int lane = threadIdx.x & 63;
  if (t == 0) {
    if (lane == 0) {
      S.e_in = 0; S.base_cnt = 0;
      for (int v = 0; v < KXP_NV_MAX; v++) S.base_var[v] = 0;
    }
    return;
  }
  const uint64_t t0 = now_ns();
  bool ok = true, done = false, timed_out = false;
  bool have_pending = false, have_newest = false;
  uint64_t pending_ent = 0, newest_ex = 0, E = 0, cnt = 0;
  uint64_t var[KXP_NV_MAX];
#pragma unroll
  for (int v = 0; v < KXP_NV_MAX; v++) var[v] = 0;
  int64_t wend = (int64_t)t;  // exclusive end of the current window
  while (ok && !done) {
    const int64_t j = wend - 1 - lane;
    uint32_t f = j >= 0 ? aload32(dp.flags + j) : 2u;
    while (__ballot(f == 0)) {
      __builtin_amdgcn_s_sleep(1);
      if (f == 0) f = aload32(dp.flags + j);
      if (now_ns() - t0 > 4000000000ull) { timed_out = true; break; }
    }
    if (timed_out) { ok = false; break; }
    const uint64_t incl = __ballot(f == 2);
    const int p = incl ? __ffsll((long long)incl) - 1 : 64;
    uint64_t c = 0, en = X_NONE, ex = 0;
    uint64_t vv[KXP_NV_MAX];
#pragma unroll
    for (int v = 0; v < KXP_NV_MAX; v++) vv[v] = 0;
    if (lane <= p && j >= 0) {
      const uint64_t* d = dp.desc + (uint64_t)j * DSTRIDE;
      if (lane == p) {
        c = aload64(d + D_INC_CNT); ex = aload64(d + D_INC_EXIT);
#pragma unroll
        for (int v = 0; v < NV; v++) vv[v] = aload64(d + D_INC_VAR + v);
      } else {
        c = aload64(d + D_AGG_CNT); en = aload64(d + D_AGG_ENT); ex = aload64(d + D_AGG_EXIT);
#pragma unroll
        for (int v = 0; v < NV; v++) vv[v] = aload64(d + D_AGG_VAR + v);
      }
    }
    // window sums over lanes <= p (lane p: inclusive prefix)
    uint64_t sc = lane <= p ? c : 0;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) sc += __shfl_xor(sc, d, 64);
    cnt += sc;
#pragma unroll
    for (int v = 0; v < NV; v++) {
      uint64_t sv = lane <= p ? vv[v] : 0;
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) sv += __shfl_xor(sv, d, 64);
      var[v] += sv;
    }
    if (chain) {
      // candidate-bearing AGG lanes in this window
      const bool cand = lane < p && en != X_NONE;
      const uint64_t cm = __ballot(cand);
      // each candidate lane links to the next older candidate lane inside the window
      const uint64_t older_mask = lane < 63 ? cm & ~((2ull << lane) - 1) : 0ull;
      const int older = older_mask ? __ffsll((long long)older_mask) - 1 : -1;
      const uint64_t older_ex = __shfl(ex, older < 0 ? lane : older, 64);
      const bool link_bad = cand && older >= 0 && older_ex != en;
      if (__ballot(link_bad)) ok = false;
      if (cm) {
        const int newest = __ffsll((long long)cm) - 1;
        const int oldest = 63 - __clzll((long long)cm);
        const uint64_t newest_exv = rl64(ex, newest);
        const uint64_t oldest_en = rl64(en, oldest);
        if (have_pending && newest_exv != pending_ent) ok = false;
        if (!have_newest) { newest_ex = newest_exv; have_newest = true; }
        pending_ent = oldest_en;
        have_pending = true;
      }
    }
    if (p < 64) {
      const uint64_t xp = rl64(ex, p);
      if (xp == X_ERR || xp == X_DONE) {
        E = xp;
      } else if (chain) {
        if (have_pending && xp != pending_ent) ok = false;
        E = have_newest ? newest_ex : xp;
      } else {
        E = xp;
      }
      done = true;
    } else {
      wend -= 64;
    }
  }
  if (!ok) {
    if (lane == 0) atomicAdd((unsigned long long*)&dp.status->diag[1], 1ull);
    // wait for the immediate predecessor's inclusive prefix
    const uint64_t* d = dp.desc + (t - 1) * DSTRIDE;
    uint32_t g = aload32(dp.flags + t - 1);
    while (g != 2) {
      __builtin_amdgcn_s_sleep(2);
      g = aload32(dp.flags + t - 1);
      if (now_ns() - t0 > 4000000000ull) break;
    }
    if (g != 2) {
      E = X_ERR;  // give up: reported as an internal error
      if (lane == 0) atomicCAS((int*)&dp.status->code, 0, KX_ERR_INTERNAL);
    } else {
      E = aload64(d + D_INC_EXIT);
      cnt = aload64(d + D_INC_CNT);
#pragma unroll
      for (int v = 0; v < NV; v++) var[v] = aload64(d + D_INC_VAR + v);
    }
  }
  if (lane == 0) {
    S.e_in = E; S.base_cnt = cnt;
    for (int v = 0; v < KXP_NV_MAX; v++) S.base_var[v] = v < NV ? var[v] : 0;
  }
}

// ---------------------------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------------------------
template <int NV, int MODE>
__global__ void __launch_bounds__(NT) decode_kernel(DecParams dp) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  Shared& S = *reinterpret_cast<Shared*>(smem_raw);
  const int tid = threadIdx.x;
  const bool known = dp.offsets != nullptr;
  uint64_t tp_last = dp.timing ? __builtin_amdgcn_s_memtime() : 0;
  auto phase = [&](int k) {
    if (dp.timing && tid == 0) {
      uint64_t now = __builtin_amdgcn_s_memtime();
      atomicAdd(&g_phase[k], (unsigned long long)(now - tp_last));
      tp_last = now;
    }
  };

  // ---- tile id in dispatch order (forward progress of the look-back) + program into LDS ----
  if (tid == 0) S.tile_id = atomicAdd(dp.counter, 1u);
  if (MODE == M_THRIFT) {
    const uint32_t* src = (const uint32_t*)dp.prog;
    uint32_t* dst = (uint32_t*)&S.prog;
    for (int i = tid; i < (int)(sizeof(KxProgram) / 4); i += NT) dst[i] = src[i];
    if (tid < KX_MAX_COLUMNS) S.colp[tid] = dp.cols.data[tid];
  } else if (tid == 0) {
    S.prog.nvar = 0; S.prog.ncols = 0;
  }
  __syncthreads();
  const uint64_t t = S.tile_id;
  const LDS KxProgram* P = (const LDS KxProgram*)&S.prog;
  void* const LDS* colp = (void* const LDS*)S.colp;

  // ---- this tile's byte range and the LDS window ----
  uint64_t r0 = 0, r1 = 0, tlo, thi;
  if (known) {
    r0 = t * NT;
    r1 = min(r0 + NT, dp.n);
    tlo = dp.offsets[r0];
    thi = dp.offsets[r1];
  } else {
    tlo = t * (uint64_t)TILE;
    thi = min(tlo + TILE, dp.in_len);
  }
  const uint64_t abs_in = (uint64_t)dp.in;
  const uint64_t wlo = (abs_in + min(tlo, dp.in_len)) & ~15ull;
  const uint64_t gend = (abs_in + dp.in_len + 15) & ~15ull;
  const uint32_t wlen = dp.in_len == 0 ? 0u : (uint32_t)min((uint64_t)WINB, gend > wlo ? gend - wlo : 0ull);
  {
    // LDS-DMA: every 16-byte chunk goes HBM -> LDS without touching registers; all loads of the
    // tile are in flight together (global_load_lds_dwordx4, wave-uniform LDS base + lane * 16).
    const GLB uint8_t* g = (const GLB uint8_t*)wlo;
    const int nch = (int)(wlen >> 4);
    const int wv = tid >> 6;
    constexpr int KW = (WIN_CHUNKS + NT - 1) / NT;
#pragma unroll
    for (int k = 0; k < KW; k++) {
      const int c = tid + k * NT;
      if (c < nch) {
        LDS void* dst = (LDS void*)((LDS uint8_t*)S.win + (size_t)(k * NT + wv * 64) * 16);
        __builtin_amdgcn_global_load_lds((const GLB void*)(g + (size_t)c * 16), dst, 16, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  Win w{dp.in, dp.in_len, wlo, wlen, (const LDS uint32_t*)S.win,
        MODE == M_THRIFT ? dp.prog->steps : nullptr, MODE == M_THRIFT ? dp.prog->nsteps : 0u,
        MODE == M_THRIFT ? dp.prog->canon_pres : 0ull};

  phase(0);
  // ---- walk 1: speculative entry + measure ----
  uint64_t ent = X_NONE, ex = X_NONE, cnt = 0;
  uint64_t vsum[KXP_NV_MAX];
#pragma unroll
  for (int v = 0; v < KXP_NV_MAX; v++) vsum[v] = 0;
  int err = 0;
  uint64_t seg_lo, seg_hi;
  if (known) {
    seg_lo = 0; seg_hi = 0;
    uint64_t r = r0 + tid;
    if (r < r1) {
      uint64_t a = dp.offsets[r], b = dp.offsets[r + 1];
      ent = a;
      if (a > b || b > dp.in_len) {
        err = KX_ERR_INVALID_ARG;
      } else {
        VarState<NV> vs; uint64_t pres, end;
        if (MODE == M_THRIFT) err = thrift_record<NV, false>(w, P, colp, a, b, r, &end, vs, pres);
        else { end = a; err = dskip(w, end, b, KX_T_STRUCT, 64); }
        if (!err) {
#pragma unroll
          for (int v = 0; v < NV; v++) vsum[v] = vs.len[v];
        }
      }
      cnt = 1;
    }
  } else {
    seg_lo = tlo + (uint64_t)tid * SEG;
    seg_hi = min(seg_lo + SEG, thi);
    if (seg_lo < thi) {
      // first canonical signature in [seg_lo, seg_hi)
      const uint32_t sig = MODE == M_THRIFT ? P->sig : (uint32_t)KX_T_STOP;
      const uint32_t smask = (MODE == M_THRIFT && P->sig_len == 3) ? 0xffffffu : 0xffu;
      const uint64_t slen = (MODE == M_THRIFT && P->sig_len == 3) ? 3 : 1;
      const uint64_t plim = min(seg_hi, dp.in_len >= slen ? dp.in_len - slen + 1 : 0ull);
      const uint64_t r0w = abs_in + seg_lo - wlo;   // window byte of seg_lo
      if (slen == 3 && seg_hi - seg_lo == SEG) {
        ent = scan_segment((const LDS uint32_t*)S.win, (uint32_t)r0w, seg_lo, plim, sig);
      } else {
        // short (last) segment or 1-byte signature: dword-at-a-time
        uint32_t q = (uint32_t)(r0w >> 2);
        uint64_t pbase = seg_lo - (r0w & 3);          // input position of window byte 4q
        uint32_t x0 = S.win[q];
        for (; pbase < plim; pbase += 4, q++) {
          const uint32_t x1 = S.win[q + 1];
          uint32_t hit = 0;
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const uint64_t pp = pbase + j;
            if (pp >= seg_lo && pp < plim && (__builtin_amdgcn_alignbyte(x1, x0, j) & smask) == sig) hit |= 1u << j;
          }
          if (hit) { ent = pbase + __builtin_ctz(hit); break; }
          x0 = x1;
        }
      }
    }
  }
  // (re)walk from `ent` through the segment; used for speculation and for the serial fallback
  auto walk_measure = [&](uint64_t e) {
    ex = e; cnt = 0; err = 0;
#pragma unroll
    for (int v = 0; v < KXP_NV_MAX; v++) vsum[v] = 0;
    if (e == X_NONE) { ex = X_NONE; return; }
    uint64_t pos = e;
    while (pos < seg_hi && pos < dp.in_len) {
      VarState<NV> vs; uint64_t pres, end;
      int rc;
      if (MODE == M_THRIFT) rc = thrift_record<NV, false>(w, P, colp, pos, dp.in_len, 0, &end, vs, pres);
      else { end = pos; rc = dskip(w, end, dp.in_len, KX_T_STRUCT, 64); }
      if (rc) { err = rc; ex = X_ERR; return; }
#pragma unroll
      for (int v = 0; v < NV; v++) vsum[v] += vs.len[v];
      cnt++;
      pos = end;
    }
    ex = pos;
  };
  if (!known) walk_measure(ent);

  phase(1);
  // ---- link repair (concatenated mode) ----
  // Every lane must start walking at the first true record start in its segment. Given the exit
  // of the previous walking lane (or the tile's entry `seed`), each lane adopts the position that
  // exit implies and re-walks; rounds repeat until nothing changes (normally 0-1 rounds: a false
  // signature hit is corrected by its neighbour's exit). seed == X_NONE: the tile's entry is not
  // known yet and the first candidate lane is trusted.
  S.ent[tid] = ent;
  S.ext[tid] = ex;
  if (tid == 0) { S.first_err_lane = NT; S.ok = 1; }
  __syncthreads();
  auto relax = [&](uint64_t seed, int max_rounds) -> int {  // rounds used, -1 if not converged
    for (int it = 0; it <= max_rounds; it++) {
      const bool has = ent != X_NONE;
      const int pc = block_excl_maxscan_i32(has ? tid : -1, S.scan_i);
      const uint64_t pe = pc >= 0 ? S.ext[pc] : seed;
      uint64_t want = ent;
      if (pe != X_NONE) {
        if (pe == X_ERR || pe == X_DONE || seg_lo >= thi || pe >= seg_hi) want = X_NONE;
        else if (pe >= seg_lo) want = pe;
        // pe < seg_lo: an earlier lane adopts pe first; revisit next round
      }
      if (tid == 0) S.changed = 0;
      __syncthreads();
      if (want != ent) {
        if (it == max_rounds) { S.changed = 2; }
        else {
          ent = want;
          walk_measure(ent);
          S.ent[tid] = ent;
          S.ext[tid] = ex;
          S.changed = 1;
        }
      }
      __syncthreads();
      const int ch = S.changed;
      __syncthreads();
      if (ch == 0) return it;
      if (ch == 2) return -1;
    }
    return -1;
  };
  auto find_first_err = [&]() {
    if (tid == 0) S.first_err_lane = NT;
    __syncthreads();
    if (ent != X_NONE && ex == X_ERR) atomicMin(&S.first_err_lane, tid);
    __syncthreads();
  };
  if (!known) {
    int r = relax(X_NONE, 16);
    if (r != 0 && tid == 0) atomicAdd((unsigned long long*)&dp.status->diag[2], 1ull);
    if (r < 0 && tid == 0) S.ok = 0;
    find_first_err();
  }

  // lanes after the first failing walk hold no valid records
  uint64_t cpre = 0;
  uint64_t vpre[KXP_NV_MAX];
  auto scan_tile = [&]() {
    bool live = known || (ent != X_NONE && tid <= S.first_err_lane);
    uint64_t tot;
    cpre = block_excl_scan_u64(live ? cnt : 0, &tot, S.scan_u);
    if (tid == 0) S.tile_cnt = tot;
#pragma unroll
    for (int v = 0; v < NV; v++) {
      vpre[v] = block_excl_scan_u64(live ? vsum[v] : 0, &tot, S.scan_u);
      if (tid == 0) S.tile_var[v] = tot;
    }
  };
  // tile entry / exit from the lane table; `pass` is the exit when no lane holds a record start
  auto tile_ends = [&](uint64_t pass) {
    if (tid == 0) {
      uint64_t se = X_NONE, sx = pass;
      for (int i = 0; i < NT; i++)
        if (S.ent[i] != X_NONE) { se = S.ent[i]; break; }
      if (S.first_err_lane < NT) sx = X_ERR;
      else
        for (int i = NT - 1; i >= 0; i--)
          if (S.ent[i] != X_NONE) { sx = S.ext[i]; break; }
      S.spec_ent = se;
      S.tile_exit = sx;
    }
    __syncthreads();
  };
  scan_tile();
  if (!known) tile_ends(X_NONE);
  __syncthreads();

  phase(2);
  // ---- publish the aggregate, then look back ----
  if (tid == 0 && (known || S.ok)) {
    uint64_t words[3 + KXP_NV_MAX];
    words[0] = S.tile_cnt;
    words[1] = known ? X_NONE : S.spec_ent;
    words[2] = known ? 0 : S.tile_exit;
    for (int v = 0; v < KXP_NV_MAX; v++) words[3 + v] = v < NV ? S.tile_var[v] : 0;
    publish(dp, t, 1u, words, D_AGG_CNT, 3 + NV);
  }
  if (tid < 64) lookback<NV>(dp, S, t, !known);
  __syncthreads();

  phase(3);
  uint64_t E = S.e_in;
  bool terminal = E == X_ERR || E == X_DONE || (!known && S.base_cnt >= dp.n);
  if (!known && !terminal) {
    bool valid = S.ok && (S.spec_ent == X_NONE ? E >= thi : E == S.spec_ent);
    if (!valid) {
      if (tid == 0) atomicAdd((unsigned long long*)&dp.status->diag[0], 1ull);
      // repair from the true entry
      int r = relax(E, 64);
      if (r < 0) {
        // last resort: one lane walks from the true entry, assigning each record start to its lane
        __syncthreads();
        S.ent[tid] = X_NONE;
        __syncthreads();
        if (tid == 0) {
          uint64_t pos = E;
          while (pos < thi && pos < dp.in_len) {
            uint64_t lane_of = (pos - tlo) / SEG;
            if (S.ent[lane_of] == X_NONE) S.ent[lane_of] = pos;
            VarState<NV> vs; uint64_t pres, end;
            int rc;
            if (MODE == M_THRIFT) rc = thrift_record<NV, false>(w, P, colp, pos, dp.in_len, 0, &end, vs, pres);
            else { end = pos; rc = dskip(w, end, dp.in_len, KX_T_STRUCT, 64); }
            if (rc) break;
            pos = end;
          }
        }
        __syncthreads();
        ent = S.ent[tid];
        walk_measure(ent);
        S.ext[tid] = ex;
        __syncthreads();
      }
      find_first_err();
      scan_tile();
      tile_ends(E);
    } else if (S.spec_ent == X_NONE && tid == 0) {
      S.tile_exit = E;  // pass-through tile
    }
  }
  __syncthreads();

  phase(4);
  // ---- publish the inclusive prefix ----
  const uint64_t base = S.base_cnt;
  if (tid == 0) {
    uint64_t words[2 + KXP_NV_MAX];
    uint64_t xo;
    if (known) {
      xo = 0;
      words[0] = base + S.tile_cnt;
    } else if (terminal) {
      xo = E == X_DONE || base >= dp.n ? X_DONE : X_ERR;
      words[0] = base;
    } else {
      uint64_t tot = base + S.tile_cnt;
      xo = S.tile_exit;
      if (tot >= dp.n) xo = X_DONE;
      else if (xo == dp.in_len) {
        // the input ends before n records: EOF at record `tot`
        xo = X_ERR;
        kx_status* st = dp.status;
        st->code = KX_ERR_EOF; st->record = tot; st->offset = dp.in_len;
        st->n_records = tot; st->consumed = dp.in_len;
        for (int v = 0; v < NV && v < (int)P->nvar; v++) {
          uint64_t vt = S.base_var[v] + S.tile_var[v];
          if (v < 8) st->var_total[v] = vt;
          if (MODE == M_THRIFT) dp.cols.offs[P->var_col[v]][tot] = (uint32_t)vt;
        }
        if (MODE == M_SKIP) dp.skip_out[tot] = dp.in_len;
      }
      words[0] = tot;
    }
    words[1] = xo;
    for (int v = 0; v < KXP_NV_MAX; v++) words[2 + v] = v < NV ? S.base_var[v] + S.tile_var[v] : 0;
    publish(dp, t, 2u, words, D_INC_CNT, 2 + NV);
  }
  if (!known && terminal) return;

  phase(5);
  // ---- walk 2: re-parse from LDS and scatter ----
  bool live = known || (ent != X_NONE && tid <= S.first_err_lane);
  if (!live || (dp.ablate & 1)) goto walk2_done;
  {
  uint64_t rec = base + cpre;
  uint64_t run[KXP_NV_MAX];
#pragma unroll
  for (int v = 0; v < NV; v++) run[v] = S.base_var[v] + vpre[v];
  uint64_t pres = 0;

  auto finish_record = [&](const VarState<NV>& vs, uint64_t r) {
    if (MODE != M_THRIFT) return;
#pragma unroll
    for (int v = 0; v < NV; v++) {
      if (v >= (int)P->nvar) break;
      uint32_t c = P->var_col[v];
      const KxpCol K = ld_col(P, c);
      dp.cols.offs[c][r] = (uint32_t)run[v];
      uint32_t n = vs.len[v];
      if (run[v] + n <= dp.cols.cap[c]) {
        if (n && !(dp.ablate & 2)) copy_var(w, K, vs.pos[v], n, (uint8_t*)colp[c] + run[v] * K.width);
      } else {
        atomicOr(dp.overflow, 1u);
      }
      run[v] += n;
    }
    if (dp.cols.presence) dp.cols.presence[r] = pres;
  };
  auto write_final = [&](uint64_t nrec, uint64_t consumed) {
    kx_status* st = dp.status;
    st->n_records = nrec;
    st->consumed = consumed;
#pragma unroll
    for (int v = 0; v < NV; v++) {
      if (v >= (int)P->nvar) break;
      if (v < 8) st->var_total[v] = run[v];
      if (MODE == M_THRIFT) dp.cols.offs[P->var_col[v]][nrec] = (uint32_t)run[v];
    }
  };

  if (known) {
    uint64_t r = r0 + tid;
    if (r >= r1) goto walk2_done;
    uint64_t a = dp.offsets[r], b = dp.offsets[r + 1];
    VarState<NV> vs;
    uint64_t end;
    int rc = err;
    if (!rc) {
      if (MODE == M_THRIFT) rc = thrift_record<NV, true>(w, P, colp, a, b, r, &end, vs, pres);
      else { end = a; rc = dskip(w, end, b, KX_T_STRUCT, 64); }
    }
    if (rc) {
      if (MODE == M_THRIFT) emit_defaults<NV>(P, colp, r);
#pragma unroll
      for (int v = 0; v < NV; v++) vs.len[v] = 0;
      pres = 0;
      atomicMin(dp.errkey, (unsigned long long)((r << 8) | (uint64_t)(rc & 0xff)));
    }
    if (dp.rstat) dp.rstat[r] = (uint8_t)rc;
    finish_record(vs, r);
    if (r == dp.n - 1) write_final(dp.n, dp.offsets[dp.n]);
    goto walk2_done;
  }

  if (ent == X_NONE) goto walk2_done;
  uint64_t pos = ent;
  while (pos < seg_hi && pos < dp.in_len && rec < dp.n) {
    VarState<NV> vs;
    uint64_t end;
    int rc;
    if (MODE == M_THRIFT) {
      if (dp.ablate & 4) rc = thrift_record<NV, false>(w, P, colp, pos, dp.in_len, rec, &end, vs, pres);
      else rc = thrift_record<NV, true>(w, P, colp, pos, dp.in_len, rec, &end, vs, pres);
    }
    else {
      end = pos;
      rc = dskip(w, end, dp.in_len, KX_T_STRUCT, 64);
      if (!rc) dp.skip_out[rec] = pos;
    }
    if (rc) {
      // the validated chain stops here: report it (single writer: the only error on the chain)
      kx_status* st = dp.status;
      st->code = rc; st->record = rec; st->offset = pos;
      write_final(rec, pos);
      if (MODE == M_SKIP) dp.skip_out[rec] = pos;
      goto walk2_done;
    }
    finish_record(vs, rec);
    rec++;
    pos = end;
    if (rec == dp.n) {
      write_final(dp.n, pos);
      if (MODE == M_SKIP) dp.skip_out[dp.n] = pos;
    }
  }
  }
walk2_done:
  if (dp.timing) {
    __syncthreads();
    phase(6);
  }
}

__global__ void finalize_kernel(kx_status* st, const unsigned long long* errkey, const uint32_t* overflow,
                                const uint64_t* offsets, uint64_t n) {
  if (threadIdx.x != 0) return;
  unsigned long long k = *errkey;
  if (k != ~0ull && st->code == 0) {
    st->code = (int32_t)(k & 0xff);
    st->record = k >> 8;
    st->offset = offsets ? offsets[k >> 8] : 0;
  }
  if (*overflow && st->code == 0) st->code = KX_ERR_SIZE_LIMIT;
  if (offsets) st->n_records = n;
}

// workspace layout: [0] tile counter u32, [8] errkey u64, [16] overflow u32, [256...) flags, then desc
struct WsLayout {
  size_t flags_off, desc_off, total;
};

WsLayout ws_layout(uint64_t ntiles) {
  WsLayout L;
  L.flags_off = 256;
  L.desc_off = (L.flags_off + ntiles * 4 + 255) & ~(size_t)255;
  L.total = L.desc_off + ntiles * DSTRIDE * 8;
  return L;
}

uint64_t tiles_for(uint64_t in_len, const uint64_t* offsets, uint64_t n) {
  return offsets ? (n + NT - 1) / NT : (in_len + TILE - 1) / TILE;
}

template <int NV, int MODE>
int launch_t(const DecParams& dp0, void* ws, hipStream_t stream) {
  DecParams dp = dp0;
  WsLayout L = ws_layout(dp.ntiles);
  char* base = (char*)ws;
  dp.counter = (uint32_t*)base;
  dp.errkey = (unsigned long long*)(base + 8);
  dp.overflow = (uint32_t*)(base + 16);
  dp.flags = (uint32_t*)(base + L.flags_off);
  dp.desc = (uint64_t*)(base + L.desc_off);
  KX_HIP_CHECK(hipMemsetAsync(base, 0, L.desc_off, stream));
  KX_HIP_CHECK(hipMemsetAsync(base + 8, 0xff, 8, stream));
  KX_HIP_CHECK(hipMemsetAsync(dp.status, 0, sizeof(kx_status), stream));
  size_t shmem = sizeof(Shared);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)decode_kernel<NV, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)shmem);
    attr_set = true;
  }
  hipLaunchKernelGGL((decode_kernel<NV, MODE>), dim3((unsigned)dp.ntiles), dim3(NT), shmem, stream, dp);
  KX_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(64), 0, stream, dp.status, dp.errkey, dp.overflow,
                     dp.offsets, dp.n);
  KX_HIP_CHECK(hipGetLastError());
  return KX_OK;
}

}  // namespace

size_t kx_decode_ws_bytes(const KxProgram&, uint64_t in_len, const uint64_t* offsets, uint64_t n) {
  return ws_layout(tiles_for(in_len, offsets, n)).total;
}

// diagnostics (not part of the public ABI): read and reset the phase-timing accumulators
extern "C" int kx_debug_phase_cycles(unsigned long long* out, int n) {
  if (n > 10) n = 10;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), sizeof(unsigned long long) * n) != hipSuccess) return KX_ERR_HIP;
  unsigned long long z[10] = {0};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof z) != hipSuccess) return KX_ERR_HIP;
  return KX_OK;
}

size_t kx_skip_ws_bytes(uint64_t in_len) { return ws_layout(tiles_for(in_len, nullptr, 0)).total; }

int kx_launch_decode(const KxProgram* dprog, const KxProgram& hprog, const uint8_t* in, uint64_t in_len,
                     const uint64_t* offsets, uint64_t n, const KxLaunchCols& cols, uint8_t* record_status,
                     kx_status* status, void* ws, size_t ws_size, hipStream_t stream, bool pb) {
  if (pb) return KX_ERR_NOT_IMPLEMENTED;
  DecParams dp{};
  static int timing = -1, ablate = -1;
  if (timing < 0) { const char* e = getenv("KX_PHASE_TIMING"); timing = e && e[0] == '1'; }
  if (ablate < 0) { const char* e = getenv("KX_ABLATE"); ablate = e ? atoi(e) : 0; }
  dp.timing = timing;
  dp.ablate = ablate;
  dp.in = in; dp.in_len = in_len; dp.offsets = offsets; dp.n = n; dp.prog = dprog;
  dp.cols = cols; dp.rstat = record_status; dp.status = status;
  dp.ntiles = tiles_for(in_len, offsets, n);
  if (dp.ntiles == 0) dp.ntiles = 1;
  if (ws_size < ws_layout(dp.ntiles).total) return KX_ERR_INVALID_ARG;
  switch (hprog.nvar) {
    case 0: return launch_t<0, M_THRIFT>(dp, ws, stream);
    case 1: return launch_t<1, M_THRIFT>(dp, ws, stream);
    case 2: return launch_t<2, M_THRIFT>(dp, ws, stream);
    case 3: case 4: return launch_t<4, M_THRIFT>(dp, ws, stream);
    default: return launch_t<8, M_THRIFT>(dp, ws, stream);
  }
}

int kx_launch_skip(const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t* offsets_out, kx_status* status,
                   void* ws, size_t ws_size, hipStream_t stream) {
  DecParams dp{};
  dp.in = in; dp.in_len = in_len; dp.offsets = nullptr; dp.n = n; dp.prog = nullptr;
  dp.status = status; dp.skip_out = offsets_out;
  dp.ntiles = tiles_for(in_len, nullptr, n);
  if (dp.ntiles == 0) dp.ntiles = 1;
  if (ws_size < ws_layout(dp.ntiles).total) return KX_ERR_INVALID_ARG;
  return launch_t<0, M_SKIP>(dp, ws, stream);
}
