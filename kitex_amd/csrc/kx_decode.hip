// kx_decode.hip — batched Thrift-binary FastRead (and the skip decoder) on CDNA4 / gfx950.
//
// Reference semantics: generated FastRead (tool/internal_pkg/pluginmode/thriftgo/struct_tpl.go:41-149,
// 405-625; instance internal/mocks/thrift/k-mock.go:39-184) over N records, as fastUnmarshal does per
// message (pkg/remote/codec/thrift/codec_fast.go:60-82) or as the element loop of a list<Struct>;
// unknown / mistyped fields go through the skip decoder (codec_apache.go:191-293).
//
// Design — ONE pass over HBM, one WAVE per tile, no workgroup barriers:
//   * concatenated mode: a tile is 8 KiB of input. The wave pulls the tile (+ a 512-byte halo for
//     the record straddling its end) into its own LDS window with LDS-DMA (global_load_lds_dwordx4:
//     HBM -> LDS without registers, 9 loads in flight per lane). Lane l owns the 128-byte segment
//     l: it finds the first canonical record signature in its segment and walks records
//     (schema-aware FastRead lengths) until it leaves the segment ("walk 1").
//   * lanes repair each other's entries with wave shuffles until the chain is consistent; record
//     counts and arena bytes are prefix-summed across the wave;
//   * the tile aggregate is published as self-tagged 64-bit words (16-bit call epoch + 48-bit value:
//     no flag, no fence, no per-call memset) and a decoupled look-back over predecessor tiles yields
//     the true entry, record base and arena bases; a wrong speculation is repaired from the true
//     entry (more shuffle rounds) before the inclusive prefix is published;
//   * "walk 2" re-parses from LDS and scatters: fixed-width columns are stored as parsed (lanes =
//     consecutive records), strings / lists are copied from LDS with 16-byte stores.
//   * known-offsets mode (fastUnmarshal with dataLen): a tile is up to 64 records, one per lane.
// Walk 1, the repair rounds and walk 2 run through ONE instance of the record parser (a small
// state machine around it), which keeps the kernel's code inside the instruction cache.
// Canonical records (the encoder's layout) take a straight-line step plan compiled from the schema;
// anything else takes the generic field loop. Records or strings reaching past the LDS window are
// read from global memory (same code, other source).
// No MFMA anywhere: this is byte movement, bounded by HBM bandwidth and memory latency.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "kx_internal.h"

#define LDS __attribute__((address_space(3)))
#define GLB __attribute__((address_space(1)))

namespace {

constexpr int NT = 256;                  // threads per workgroup (4 independent waves)
constexpr int WAVES = NT / 64;
constexpr int SEG = 128;                 // bytes per lane segment
constexpr int TILE = 64 * SEG;           // 8 KiB of input per wave
constexpr int HALO = 512;                // the record straddling the tile end is read from LDS up to here
constexpr int WINB = TILE + HALO + 16;   // LDS window bytes (+16 for the aligned-down start)
constexpr int WINW = WINB / 4 + 4;       // window dwords (+ pad for the last aligned read pair)
constexpr int WIN_LOADS = (WINB / 16 + 63) / 64;
constexpr int DFIELDS = 21;              // look-back word arrays (structure of arrays over tiles)

constexpr uint64_t V48 = (1ull << 48) - 1;
constexpr uint64_t X_ERR = V48;          // chain terminated by a decode error
constexpr uint64_t X_DONE = V48 - 1;     // chain reached n records
constexpr uint64_t X_NONE = V48 - 2;     // no candidate in this tile / lane

// descriptor words (each = epoch << 48 | value); word f of tile t lives at desc[f * ntiles + t], so a
// wave reading 64 consecutive tiles' word f touches a few contiguous cache lines
constexpr int D_AGG_CNT = 0, D_AGG_ENT = 1, D_AGG_EXIT = 2, D_AGG_VAR = 3;  // 3 + 8
constexpr int D_INC_CNT = 11, D_INC_EXIT = 12, D_INC_VAR = 13;              // 2 + 8

enum Mode { M_THRIFT = 0, M_SKIP = 1 };

// opt-in phase timing (KX_PHASE_TIMING=1): shader cycles per phase summed over tiles (lane 0)
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
  uint32_t* counter;         // dynamic tile counter (reset by finalize)
  uint64_t* desc;            // per-tile look-back words
  unsigned long long* errkey;  // offsets mode: min((record << 8) | code)
  uint32_t* overflow;        // an arena capacity was exceeded
  uint64_t ntiles;
  uint64_t epoch;            // 16-bit call epoch (never 0)
  uint32_t krec;             // offsets mode: records per tile (<= 64)
  int timing;
  int nolds;                 // diagnostics (KX_NOLDS=1): read every byte from global memory
};

// ---------------------------------------------------------------------------------------------
// byte access: the wave's LDS window, or global memory outside it
// ---------------------------------------------------------------------------------------------
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v4u_a4 __attribute__((ext_vector_type(4), aligned(4)));

struct Src {
  const uint8_t* in;
  uint64_t len;
  uint64_t wpos;             // input position of window byte 0 (mod 2^64: may precede 0)
  int32_t wlen;              // valid bytes in the window
  const LDS uint32_t* win;
  const KxpStep* steps;      // canonical plan (uniform index -> scalar loads)
  uint32_t nsteps;
  uint64_t canon_pres;
};

// window offset of p, or -1 when [p, p + need) is not entirely inside the window
__device__ __forceinline__ int32_t wofs(const Src& w, uint64_t p, uint32_t need) {
  const int64_t q = (int64_t)(p - w.wpos);
  return (q >= 0 && q + (int64_t)need <= (int64_t)w.wlen) ? (int32_t)q : -1;
}

// 4 bytes at p from global memory; never reads past the dword holding the last input byte
__device__ __forceinline__ uint32_t gld4(const Src& w, uint64_t p) {
  uint64_t a = (uint64_t)w.in + p;
  uint64_t A = a & ~3ull;
  uint32_t sh = (uint32_t)(a & 3);
  uint64_t end = (uint64_t)w.in + w.len;
  uint32_t x0 = A < end ? *(const GLB uint32_t*)A : 0u;
  uint32_t x1 = A + 4 < end ? *(const GLB uint32_t*)(A + 4) : 0u;
  return __builtin_amdgcn_alignbyte(x1, x0, sh);
}

// 4 bytes at p (byte p in bits 0..7)
__device__ __forceinline__ uint32_t ld4(const Src& w, uint64_t p) {
  const int32_t q = wofs(w, p, 8);
  if (q >= 0) return __builtin_amdgcn_alignbyte(w.win[(q >> 2) + 1], w.win[q >> 2], q & 3);
  return gld4(w, p);
}

__device__ __forceinline__ uint32_t ld1(const Src& w, uint64_t p) {
  const int32_t q = wofs(w, p, 1);
  if (q >= 0) return ((const LDS uint8_t*)w.win)[q];
  return ((const GLB uint8_t*)w.in)[p];
}
__device__ __forceinline__ uint32_t be32(const Src& w, uint64_t p) { return __builtin_bswap32(ld4(w, p)); }
__device__ __forceinline__ uint64_t be64(const Src& w, uint64_t p) {
  return ((uint64_t)be32(w, p) << 32) | be32(w, p + 4);
}

// 12 bytes at p
struct Fetch {
  uint32_t w0, w1, w2;
};

__device__ __forceinline__ Fetch fetch12(const Src& w, uint64_t p) {
  Fetch f;
  const int32_t q = wofs(w, p, 16);
  if (q >= 0) {
    const LDS uint32_t* s = w.win + (q >> 2);
    const uint32_t sh = q & 3;
    const uint32_t x0 = s[0], x1 = s[1], x2 = s[2], x3 = s[3];
    f.w0 = __builtin_amdgcn_alignbyte(x1, x0, sh);
    f.w1 = __builtin_amdgcn_alignbyte(x2, x1, sh);
    f.w2 = __builtin_amdgcn_alignbyte(x3, x2, sh);
  } else if (p + 16 <= w.len) {
    uint64_t a = (uint64_t)w.in + p;
    v4u v = *(const GLB v4u_a4*)(a & ~3ull);  // dword alignment suffices
    uint32_t sh = (uint32_t)(a & 3);
    f.w0 = __builtin_amdgcn_alignbyte(v.y, v.x, sh);
    f.w1 = __builtin_amdgcn_alignbyte(v.z, v.y, sh);
    f.w2 = __builtin_amdgcn_alignbyte(v.w, v.z, sh);
  } else {
    f.w0 = gld4(w, p);
    f.w1 = gld4(w, p + 4);
    f.w2 = gld4(w, p + 8);
  }
  return f;
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

// the field value that follows a 3-byte field header (wire bytes p+3 ...), host order
// (BOOL is `b == 1`: parity unpinned, matches the oracle)
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

__device__ __forceinline__ int dskip_body(const Src& w, uint64_t& pos, uint64_t limit, uint32_t t0, int md0) {
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

// ---------------------------------------------------------------------------------------------
// per-record FastRead
// ---------------------------------------------------------------------------------------------
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

__device__ __forceinline__ void store_col(void* base, uint32_t width, uint64_t rec, uint64_t v) {
  switch (width) {
    case 1: ((GLB uint8_t*)base)[rec] = (uint8_t)v; break;
    case 2: ((GLB uint16_t*)base)[rec] = (uint16_t)v; break;
    case 4: ((GLB uint32_t*)base)[rec] = (uint32_t)v; break;
    default: ((GLB uint64_t*)base)[rec] = v; break;
  }
}

// program tables are read from global memory (a few KiB, L1/L2-resident)
__device__ __forceinline__ KxpField ld_field(const KxProgram* P, int i) {
  v4u v = *(const GLB v4u_a4*)&P->f[i];
  KxpField F;
  __builtin_memcpy(&F, &v, sizeof F);
  return F;
}
__device__ __forceinline__ KxpInst ld_inst(const KxProgram* P, int i) {
  v4u v[2];
  v[0] = ((const GLB v4u_a4*)&P->inst[i])[0];
  v[1] = ((const GLB v4u_a4*)&P->inst[i])[1];
  KxpInst I;
  __builtin_memcpy(&I, v, sizeof I);
  return I;
}
__device__ __forceinline__ KxpCol ld_col(const KxProgram* P, int i) {
  v4u v = *(const GLB v4u_a4*)&P->col[i];
  KxpCol K;
  __builtin_memcpy(&K, &v, sizeof K);
  return K;
}

// Canonical fast path: the record is checked against the schema's canonical plan (header bytes in
// encoder order, STOP bytes). The step index is wave-uniform (scalar loads); a lane whose record
// deviates returns false and the record is re-parsed by the generic loop.
template <int NV>
__device__ __forceinline__ bool canon_record(const Src& w, const KxLaunchCols& cols, uint64_t start, uint64_t limit,
                                             uint64_t rec, bool emit, uint64_t* endp, VarState<NV>& vs) {
  uint64_t pos = start;
  const KxpStep* __restrict__ steps = w.steps;
  uint32_t k = 0;
  while (k < w.nsteps) {
    const KxpStep st = steps[k];
    const uint64_t rem = limit - pos;
    if (st.kind == KXP_S_FIXED) {
      // up to 4 consecutive fixed-width fields: their positions do not depend on data
      const uint32_t m = min(st.hdr >> 24, 4u);
      const KxpStep s1 = steps[k + (m > 1 ? 1 : 0)];
      const KxpStep s2 = steps[k + (m > 2 ? 2 : 0)];
      const KxpStep s3 = steps[k + (m > 3 ? 3 : 0)];
      const uint32_t o1 = 3 + st.width, o2 = o1 + 3 + s1.width, o3 = o2 + 3 + s2.width;
      const uint32_t len = m == 1 ? o1 : m == 2 ? o2 : m == 3 ? o3 : o3 + 3 + s3.width;
      if (rem < len) return false;
      const Fetch f0 = fetch12(w, pos);
      const Fetch f1 = fetch12(w, pos + o1);
      const Fetch f2 = fetch12(w, pos + o2);
      const Fetch f3 = fetch12(w, pos + o3);
      bool ok = (f0.w0 & 0xffffffu) == (st.hdr & 0xffffffu);
      if (m > 1) ok &= (f1.w0 & 0xffffffu) == (s1.hdr & 0xffffffu);
      if (m > 2) ok &= (f2.w0 & 0xffffffu) == (s2.hdr & 0xffffffu);
      if (m > 3) ok &= (f3.w0 & 0xffffffu) == (s3.hdr & 0xffffffu);
      if (!ok) return false;
      if (emit) {
        store_col(cols.data[st.col], st.width, rec, fixed_after_header(f0, st.hdr & 0xff));
        if (m > 1) store_col(cols.data[s1.col], s1.width, rec, fixed_after_header(f1, s1.hdr & 0xff));
        if (m > 2) store_col(cols.data[s2.col], s2.width, rec, fixed_after_header(f2, s2.hdr & 0xff));
        if (m > 3) store_col(cols.data[s3.col], s3.width, rec, fixed_after_header(f3, s3.hdr & 0xff));
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
  *endp = pos;
  return true;
}

// Generic FastRead field loop: any field order, unknown / mistyped fields skipped, repeated ids
// (last wins; a repeated struct field is a fresh NewX()), required fields checked.
template <int NV>
__device__ __forceinline__ int generic_record(const Src& w, const KxProgram* P, const KxLaunchCols& cols,
                                              uint64_t start, uint64_t limit, uint64_t rec, bool emit,
                                              uint64_t* endp, VarState<NV>& vs, uint64_t& pres_out) {
#pragma unroll
  for (int i = 0; i < NV; i++) { vs.len[i] = 0; vs.pos[i] = 0; }
  uint64_t pres = 0;
  uint64_t pos = start;
  int inst = 0;
  int pred = P->inst[0].enc_first;
  uint64_t seen = 0;
  for (;;) {
    if (pos >= limit) return KX_ERR_EOF;
    const Fetch fx = fetch12(w, pos);
    KxpField F = ld_field(P, pred >= 0 ? pred : 0);
    const uint32_t t = fx.w0 & 0xff;
    if (t == KX_T_STOP) {
      pos += 1;
      const KxpInst I = ld_inst(P, inst);
      if ((seen & I.req_mask) != I.req_mask) return KX_ERR_INVALID_DATA;  // RequiredFieldNotSetError (struct_tpl.go:124-145)
      if (inst == 0) break;
      pred = I.ret_pred;
      inst = I.parent;
      continue;
    }
    if (limit - pos < 3) return KX_ERR_EOF;
    const int id = (int)(int16_t)((((fx.w0 >> 8) & 0xffu) << 8) | ((fx.w0 >> 16) & 0xffu));
    int fi = -1;
    if (pred >= 0 && F.id == id) {
      fi = pred;
    } else {
      const KxpInst I = ld_inst(P, inst);
      for (int k = 0; k < I.nfields; k++)
        if (P->f[I.first + k].id == id) { fi = I.first + k; break; }
      if (fi >= 0) F = ld_field(P, fi);
    }
    const uint64_t vp = pos + 3;
    if (fi < 0 || F.ttype != t) {                            // default: / mismatched type -> Skip
      pos = vp;
      const int rc = dskip_body(w, pos, limit, t, 64);
      if (rc) return rc;
      continue;
    }
    pred = F.enc_next;
    if (F.kind == KXP_K_FIXED) {
      const uint32_t wd = F.width;
      if (limit - vp < wd) return KX_ERR_EOF;
      if (emit) store_col(cols.data[F.col], wd, rec, fixed_after_header(fx, t));
      pos = vp + wd;
    } else if (F.kind == KXP_K_BYTES) {                      // ReadString (copies)
      if (limit - vp < 4) return KX_ERR_EOF;
      const int32_t l = (int32_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(fx.w1, fx.w0, 3));
      if (l < 0) return KX_ERR_NEGATIVE_SIZE;
      if (limit - vp - 4 < (uint64_t)l) return KX_ERR_EOF;
      vset<NV>(vs, F.vslot, vp + 4, (uint32_t)l);
      pos = vp + 4 + (uint64_t)l;
    } else if (F.kind == KXP_K_LIST) {                       // ReadListBegin: elem type ignored (:587)
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
  if (emit) {
    // fields never seen (or reset by a repeated struct field) take their default
    for (uint32_t c = 0; c < P->ncols; c++) {
      const KxpCol K = ld_col(P, c);
      if (K.kind == KXP_K_FIXED && !((seen >> K.field) & 1)) store_col(cols.data[c], K.width, rec, (uint64_t)K.defv);
    }
  }
  pres_out = pres;
  *endp = pos;
  return KX_OK;
}

__device__ __forceinline__ void emit_defaults(const KxProgram* P, const KxLaunchCols& cols, uint64_t rec) {
  for (uint32_t c = 0; c < P->ncols; c++) {
    const KxpCol K = ld_col(P, c);
    if (K.kind == KXP_K_FIXED) store_col(cols.data[c], K.width, rec, (uint64_t)K.defv);
  }
}

// ---------------------------------------------------------------------------------------------
// variable-length payload copy (strings: raw bytes; lists: big-endian elements -> host order)
// ---------------------------------------------------------------------------------------------
__device__ __noinline__ void copy_var_slow(const Src w, KxpCol K, uint64_t src, uint32_t n, uint8_t* dst_) {
  GLB uint8_t* dst = (GLB uint8_t*)dst_;
  if (K.kind == KXP_K_BYTES) {
    for (uint32_t i = 0; i < n; i++) dst[i] = (uint8_t)ld1(w, src + i);
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

// 16 bytes at p (4 dwords, byte p in bits 0..7 of the first): LDS window or global
struct Q16 {
  uint32_t a0, a1, a2, a3;
};
__device__ __forceinline__ Q16 ld16(const Src& w, uint64_t p, bool inwin) {
  uint32_t x0, x1, x2, x3, x4, sh;
  if (inwin) {
    const uint32_t q = (uint32_t)(p - w.wpos);
    const LDS uint32_t* s = w.win + (q >> 2);
    x0 = s[0]; x1 = s[1]; x2 = s[2]; x3 = s[3]; x4 = s[4];
    sh = q & 3;
  } else {
    const uint64_t a = (uint64_t)w.in + p;
    const v4u v = *(const GLB v4u_a4*)(a & ~3ull);
    x4 = *(const GLB uint32_t*)((a & ~3ull) + 16);
    x0 = v.x; x1 = v.y; x2 = v.z; x3 = v.w;
    sh = (uint32_t)(a & 3);
  }
  Q16 r;
  r.a0 = __builtin_amdgcn_alignbyte(x1, x0, sh);
  r.a1 = __builtin_amdgcn_alignbyte(x2, x1, sh);
  r.a2 = __builtin_amdgcn_alignbyte(x3, x2, sh);
  r.a3 = __builtin_amdgcn_alignbyte(x4, x3, sh);
  return r;
}

// Fast path: up to 3 head bytes to reach a dword-aligned destination, then 16-byte pieces stored
// with dwordx4 (dword alignment suffices for global stores), then a dword / byte tail.
__device__ __forceinline__ void copy_var(const Src& w, const KxpCol& K, uint64_t src, uint32_t n, uint8_t* dst_) {
  const uint64_t nbytes = (uint64_t)n * K.width;
  const bool bswap = K.kind == KXP_K_LIST && K.width > 1;
  const bool inwin = wofs(w, src, (uint32_t)min(nbytes + 20, (uint64_t)0x7fffffff)) >= 0;
  if ((!inwin && src + nbytes + 20 > w.len) || (K.kind == KXP_K_LIST && K.elem == KX_T_BOOL) ||
      (bswap && (((uintptr_t)dst_) & 3))) {
    copy_var_slow(w, K, src, n, dst_);
    return;
  }
  GLB uint8_t* dst = (GLB uint8_t*)dst_;
  uint64_t i = 0;
  if (!bswap)
    for (; i < nbytes && (((uintptr_t)(dst_ + i)) & 3); i++) dst[i] = (uint8_t)ld1(w, src + i);
  for (; i + 16 <= nbytes; i += 16) {
    Q16 r = ld16(w, src + i, inwin);
    if (bswap) {
      if (K.width == 8) {
        const uint32_t t0 = __builtin_bswap32(r.a1), t1 = __builtin_bswap32(r.a0);
        const uint32_t t2 = __builtin_bswap32(r.a3), t3 = __builtin_bswap32(r.a2);
        r.a0 = t0; r.a1 = t1; r.a2 = t2; r.a3 = t3;
      } else if (K.width == 4) {
        r.a0 = __builtin_bswap32(r.a0); r.a1 = __builtin_bswap32(r.a1);
        r.a2 = __builtin_bswap32(r.a2); r.a3 = __builtin_bswap32(r.a3);
      } else {
        r.a0 = __builtin_amdgcn_perm(r.a0, r.a0, 0x02030001u); r.a1 = __builtin_amdgcn_perm(r.a1, r.a1, 0x02030001u);
        r.a2 = __builtin_amdgcn_perm(r.a2, r.a2, 0x02030001u); r.a3 = __builtin_amdgcn_perm(r.a3, r.a3, 0x02030001u);
      }
    }
    v4u_a4 o = {r.a0, r.a1, r.a2, r.a3};
    *(GLB v4u_a4*)(dst + i) = o;
  }
  if (i < nbytes) {
    if (bswap) {
      copy_var_slow(w, K, src + i, (uint32_t)((nbytes - i) / K.width), dst_ + i);
    } else {
      for (; i + 4 <= nbytes; i += 4) *(GLB uint32_t*)(dst + i) = ld4(w, src + i);
      for (; i < nbytes; i++) dst[i] = (uint8_t)ld1(w, src + i);
    }
  }
}
// ---------------------------------------------------------------------------------------------
// wave helpers
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
  uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
  uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t aload64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void astore64(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t now_ns() { return __builtin_amdgcn_s_memrealtime() * 10; }  // 100 MHz

struct LB {
  uint64_t e, cnt;
  uint64_t var[KXP_NV_MAX];
};

// Decoupled look-back by one wave (64 predecessors per window, newest in lane 0). Every word is
// self-tagged with the call epoch, so no flag / fence protocol is needed: a word is valid iff its
// tag is this call's. Polling touches only the two head words of each predecessor (INCL count,
// AGG count) with exponential back-off; the remaining words of the tiles that matter are read once
// they are ready (re-polled in the rare case one of them is not visible yet).
// The speculative chain is verified on the way back: for consecutive candidate-bearing tiles
// a < b, exit(a) == entry(b); the inclusive tile's exit equals the entry of the oldest candidate
// tile after it. Any mismatch: wait for tile t-1's inclusive prefix.
template <int NV>
__device__ __forceinline__ LB lookback(const DecParams& dp, uint64_t t, bool chain, int lane) {
  LB out;
  out.e = 0; out.cnt = 0;
#pragma unroll
  for (int v = 0; v < KXP_NV_MAX; v++) out.var[v] = 0;
  if (t == 0) return out;
  const uint64_t ep = dp.epoch;
  const uint64_t t0 = now_ns();
  bool ok = true, done = false;
  bool have_pending = false, have_newest = false;
  uint64_t pending_ent = 0, newest_ex = 0, E = 0, cnt = 0;
  uint64_t var[KXP_NV_MAX];
#pragma unroll
  for (int v = 0; v < KXP_NV_MAX; v++) var[v] = 0;
  int64_t wend = (int64_t)t;
  while (ok && !done) {
    const int64_t j = wend - 1 - lane;
    const uint64_t* d = dp.desc + (uint64_t)(j < 0 ? 0 : j);
    const uint64_t nt = dp.ntiles;
    int state = j < 0 ? 2 : 0;  // 0 not ready, 1 AGG, 2 INCL
    uint64_t c = 0, en = X_NONE, ex = 0;
    uint64_t vv[KXP_NV_MAX];
#pragma unroll
    for (int v = 0; v < KXP_NV_MAX; v++) vv[v] = 0;
    int backoff = 1;
    for (;;) {
      // heads: lanes still unknown poll the INCL and AGG count words
      if (state == 0) {
        const uint64_t ic = aload64(d + D_INC_CNT * nt);
        const uint64_t ac = aload64(d + D_AGG_CNT * nt);
        if ((ic >> 48) == ep) { state = 2; c = ic & V48; }
        else if ((ac >> 48) == ep) { state = 1; c = ac & V48; }
      }
      uint64_t inclm = __ballot(state == 2);
      int p = inclm ? __ffsll((long long)inclm) - 1 : 64;
      if (!__ballot(state == 0 && lane <= p)) {
        // bodies of the tiles that matter (lanes <= p), one round trip
        bool bad = false;
        if (j >= 0 && lane <= p) {
          if (state == 2) {
            const uint64_t ix = aload64(d + D_INC_EXIT * nt);
            bad |= (ix >> 48) != ep;
            ex = ix & V48;
#pragma unroll
            for (int v = 0; v < NV; v++) {
              const uint64_t iv = aload64(d + (D_INC_VAR + v) * nt);
              bad |= (iv >> 48) != ep;
              vv[v] = iv & V48;
            }
          } else {
            const uint64_t ae = aload64(d + D_AGG_ENT * nt), ax = aload64(d + D_AGG_EXIT * nt);
            bad |= (ae >> 48) != ep || (ax >> 48) != ep;
            en = ae & V48;
            ex = ax & V48;
#pragma unroll
            for (int v = 0; v < NV; v++) {
              const uint64_t av = aload64(d + (D_AGG_VAR + v) * nt);
              bad |= (av >> 48) != ep;
              vv[v] = av & V48;
            }
          }
        }
        if (!__ballot(bad)) break;
        if (bad) state = 0;  // a word not visible yet: poll again
      }
      if (now_ns() - t0 > 4000000000ull) { ok = false; break; }
      __builtin_amdgcn_s_sleep(1);
      for (int k = 1; k < backoff; k++) __builtin_amdgcn_s_sleep(1);
      backoff = backoff < 32 ? backoff * 2 : 32;
    }
    if (!ok) break;
    const uint64_t inclm = __ballot(state == 2);
    const int p = inclm ? __ffsll((long long)inclm) - 1 : 64;
    uint64_t sc = lane <= p ? c : 0;
#pragma unroll
    for (int dd = 32; dd >= 1; dd >>= 1) sc += __shfl_xor(sc, dd, 64);
    cnt += sc;
#pragma unroll
    for (int v = 0; v < NV; v++) {
      uint64_t sv = lane <= p ? vv[v] : 0;
#pragma unroll
      for (int dd = 32; dd >= 1; dd >>= 1) sv += __shfl_xor(sv, dd, 64);
      var[v] += sv;
    }
    if (chain) {
      const bool cand = lane < p && state == 1 && en != X_NONE;
      const uint64_t cm = __ballot(cand);
      const uint64_t older_mask = lane < 63 ? cm & ~((2ull << lane) - 1) : 0ull;
      const int older = older_mask ? __ffsll((long long)older_mask) - 1 : -1;
      const uint64_t older_ex = __shfl(ex, older < 0 ? lane : older, 64);
      if (__ballot(cand && older >= 0 && older_ex != en)) ok = false;
      if (cm) {
        const int newest = __ffsll((long long)cm) - 1;
        const int oldest = 63 - __clzll((long long)cm);
        const uint64_t newest_exv = rl64(ex, newest);
        if (have_pending && newest_exv != pending_ent) ok = false;
        if (!have_newest) { newest_ex = newest_exv; have_newest = true; }
        pending_ent = rl64(en, oldest);
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
    const uint64_t* d = dp.desc + (t - 1);
    const uint64_t nt = dp.ntiles;
    bool got = false;
    int backoff = 1;
    for (;;) {
      const uint64_t ic = aload64(d + D_INC_CNT * nt), ix = aload64(d + D_INC_EXIT * nt);
      uint64_t iv[KXP_NV_MAX];
      bool incl = (ic >> 48) == ep && (ix >> 48) == ep;
#pragma unroll
      for (int v = 0; v < NV; v++) {
        iv[v] = aload64(d + (D_INC_VAR + v) * nt);
        incl &= (iv[v] >> 48) == ep;
      }
      if (incl) {
        E = ix & V48; cnt = ic & V48;
#pragma unroll
        for (int v = 0; v < NV; v++) var[v] = iv[v] & V48;
        got = true;
        break;
      }
      if (now_ns() - t0 > 4000000000ull) break;
      for (int k = 0; k < backoff; k++) __builtin_amdgcn_s_sleep(1);
      backoff = backoff < 32 ? backoff * 2 : 32;
    }
    if (!got) {
      E = X_ERR;  // give up: reported as an internal error
      if (lane == 0) atomicCAS((int*)&dp.status->code, 0, KX_ERR_INTERNAL);
    }
  }
  out.e = E;
  out.cnt = cnt;
#pragma unroll
  for (int v = 0; v < NV; v++) out.var[v] = var[v];
  return out;
}

// one lane publishes a set of self-tagged words
__device__ __forceinline__ void publish_words(const DecParams& dp, uint64_t t, int first, const uint64_t* vals,
                                              int nwords) {
  uint64_t* d = dp.desc + t + (uint64_t)first * dp.ntiles;
  const uint64_t ep = dp.epoch << 48;
  for (int i = 0; i < nwords; i++) astore64(d + (uint64_t)i * dp.ntiles, ep | (vals[i] & V48));
}

// ---------------------------------------------------------------------------------------------
// the kernel: 4 independent waves per workgroup, one tile per wave
// ---------------------------------------------------------------------------------------------
// (the lane builtins return int: keep both halves unsigned so bit 31 never sign-extends)
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// first canonical signature (3 bytes) in a lane's 128-byte segment, read from the LDS window:
// 35 dwords in registers, SWAR test for the first signature byte, exact 3-byte check on hits
__device__ __forceinline__ uint64_t scan_segment(const Src& w, int32_t q0, uint64_t seg_lo, uint64_t plim,
                                                 uint32_t sig) {
  const LDS uint32_t* s = w.win + (q0 >> 2);
  const int sh0 = q0 & 3;
  uint32_t d[35];
#pragma unroll
  for (int i = 0; i < 35; i++) d[i] = s[i];
  const uint32_t b0 = (sig & 0xff) * 0x01010101u;
  uint64_t found = X_NONE;
#pragma unroll
  for (int i = 0; i < 34; i++) {
    const uint32_t t = d[i] ^ b0;
    const uint32_t z = (t - 0x01010101u) & ~t & 0x80808080u;   // bytes equal to the first sig byte
    if (found == X_NONE && z) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int rel = 4 * i + j - sh0;
        if (found == X_NONE && rel >= 0 && rel < SEG && seg_lo + rel < plim &&
            (__builtin_amdgcn_alignbyte(d[i + 1], d[i], j) & 0xffffffu) == sig)
          found = seg_lo + rel;
      }
    }
  }
  return found;
}

template <int NV, int MODE>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) decode_kernel(DecParams dp) {
  __shared__ __attribute__((aligned(16))) uint32_t WIN[WAVES][WINW];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const bool known = dp.offsets != nullptr;
  const KxProgram* P = dp.prog;
  const uint32_t nvar = MODE == M_THRIFT ? P->nvar : 0u;

  // ---- tile ids in claim order (forward progress of the look-back): one claim per workgroup ----
  __shared__ uint32_t wg_claim;
  if (threadIdx.x == 0) wg_claim = atomicAdd(dp.counter, 1u);
  __syncthreads();
  const uint64_t t = (uint64_t)wg_claim * WAVES + wv;
  if (t >= dp.ntiles) return;
  uint64_t tp_last = dp.timing ? __builtin_amdgcn_s_memtime() : 0;
  auto phase = [&](int k) {
    if (dp.timing && lane == 0) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      atomicAdd(&g_phase[k], (unsigned long long)(now - tp_last));
      tp_last = now;
    }
  };

  // ---- this tile's range ----
  uint64_t tlo, thi = 0, r0 = 0, r1 = 0;
  if (known) {
    r0 = t * dp.krec;
    r1 = min(r0 + dp.krec, dp.n);
    tlo = dp.offsets[r0];
  } else {
    tlo = t * (uint64_t)TILE;
    thi = min(tlo + TILE, dp.in_len);
  }

  // ---- LDS window: HBM -> LDS by DMA, all chunks in flight together ----
  LDS uint32_t* win = (LDS uint32_t*)WIN[wv];
  const uint64_t abs_in = (uint64_t)dp.in;
  const uint64_t wbase = (abs_in + min(tlo, dp.in_len)) & ~15ull;
  const int32_t wlen = dp.nolds ? 0 : (int32_t)min((uint64_t)WINB, abs_in + dp.in_len - wbase);
  {
    const int nch = (wlen + 15) >> 4;
    const GLB uint8_t* g = (const GLB uint8_t*)wbase;
#pragma unroll
    for (int k = 0; k < WIN_LOADS; k++) {
      const int c = k * 64 + lane;
      if (c < nch)
        __builtin_amdgcn_global_load_lds((const GLB void*)(g + (size_t)c * 16), (LDS void*)(win + k * 256), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  const Src w{dp.in, dp.in_len, wbase - abs_in, wlen, win,
              MODE == M_THRIFT ? P->steps : nullptr, MODE == M_THRIFT ? P->nsteps : 0u,
              MODE == M_THRIFT ? P->canon_pres : 0ull};
  phase(0);

  // ---- per-lane segment (concatenated) or record (offsets) ----
  uint64_t seg_lo = 0, seg_hi = 0, lim = dp.in_len, rrec = 0;
  bool mine = false;
  int kerr = 0;
  uint64_t ent = X_NONE;
  if (known) {
    rrec = r0 + lane;
    mine = rrec < r1;
    if (mine) {
      const uint64_t a = dp.offsets[rrec], b = dp.offsets[rrec + 1];
      ent = a;
      lim = b;
      if (a > b || b > dp.in_len) kerr = KX_ERR_INVALID_ARG;
    }
  } else {
    seg_lo = tlo + (uint64_t)lane * SEG;
    seg_hi = min(seg_lo + SEG, thi);
    if (seg_lo < thi) {
      const uint32_t sig = MODE == M_THRIFT ? P->sig : (uint32_t)KX_T_STOP;
      const uint32_t slen = (MODE == M_THRIFT && P->sig_len == 3) ? 3u : 1u;
      const uint64_t plim = min(seg_hi, dp.in_len >= slen ? dp.in_len - slen + 1 : 0ull);
      const int32_t q0 = wofs(w, seg_lo, SEG + 12);
      if (slen == 3 && seg_hi - seg_lo == SEG && q0 >= 0) {
        ent = scan_segment(w, q0, seg_lo, plim, sig);
      } else {
        const uint32_t smask = slen == 3 ? 0xffffffu : 0xffu;
        for (uint64_t p = seg_lo; p < plim; p++)
          if ((ld4(w, p) & smask) == sig) { ent = p; break; }
      }
    }
  }

  // ---- walks: ONE instance of the record loop serves walk 1 (measure), the repair rounds and
  //      walk 2 (emit); the state machine around it decides who walks next ----
  uint64_t ex = X_NONE, cnt = 0;
  uint64_t vsum[NV > 0 ? NV : 1];
#pragma unroll
  for (int v = 0; v < (NV > 0 ? NV : 1); v++) vsum[v] = 0;
  bool need = known ? mine : ent != X_NONE;
  int stage = 0;            // 0 speculative walk 1, 1 repair from the true entry, 2 emit
  int rounds = 0;
  uint64_t seed = X_NONE;
  bool ok = true;
  int fel = 64;
  uint64_t cpre = 0, tile_cnt = 0;
  uint64_t vpre[NV > 0 ? NV : 1], tile_var[NV > 0 ? NV : 1];
  uint64_t spec_ent = X_NONE, tile_exit = X_NONE;
  LB lb;
  lb.e = 0; lb.cnt = 0;
  uint64_t rec = 0;
  uint64_t run[NV > 0 ? NV : 1];
  bool terminal = false;

  auto write_final = [&](uint64_t nrec, uint64_t consumed) {
    kx_status* st = dp.status;
    st->n_records = nrec;
    st->consumed = consumed;
#pragma unroll
    for (int v = 0; v < NV; v++) {
      if (v >= (int)nvar) break;
      st->var_total[v] = run[v];
      dp.cols.offs[P->var_col[v]][nrec] = (uint32_t)run[v];
    }
  };

  for (;;) {
    if (need) {
      const bool emit = stage == 2;
      uint64_t pos = ent, c = 0;
      uint64_t acc[NV > 0 ? NV : 1];
#pragma unroll
      for (int v = 0; v < (NV > 0 ? NV : 1); v++) acc[v] = 0;
      int e = 0;
      for (;;) {
        if (!known && !(pos < seg_hi && pos < dp.in_len)) break;
        if (emit && !known && rec >= dp.n) break;
        const uint64_t r = known ? rrec : rec;
        VarState<NV> vs;
#pragma unroll
        for (int v = 0; v < NV; v++) { vs.len[v] = 0; vs.pos[v] = 0; }
        uint64_t pres = 0, end = pos;
        int rc = kerr;
        if (!rc) {
          if (MODE == M_THRIFT) {
            const bool canon = w.nsteps && canon_record<NV>(w, dp.cols, pos, lim, r, emit, &end, vs);
            if (canon) pres = w.canon_pres;
            else rc = generic_record<NV>(w, P, dp.cols, pos, lim, r, emit, &end, vs, pres);
          } else {
            uint64_t p2 = pos;
            rc = dskip_body(w, p2, lim, KX_T_STRUCT, 64);
            end = p2;
            if (emit && !rc) dp.skip_out[r] = pos;
          }
        }
        if (rc) {
          e = rc;
          if (!known) break;
          // offsets mode: the failed record reads as all defaults, empty payloads
#pragma unroll
          for (int v = 0; v < NV; v++) vs.len[v] = 0;
          pres = 0;
          if (emit && MODE == M_THRIFT) emit_defaults(P, dp.cols, r);
        }
        if (emit && MODE == M_THRIFT) {
#pragma unroll
          for (int v = 0; v < NV; v++) {
            if (v >= (int)nvar) break;
            const uint32_t cc = P->var_col[v];
            dp.cols.offs[cc][r] = (uint32_t)run[v];
            const uint32_t nn = vs.len[v];
            if (run[v] + nn <= dp.cols.cap[cc]) {
              if (nn) {
                const KxpCol K = ld_col(P, cc);
                copy_var(w, K, vs.pos[v], nn, (uint8_t*)dp.cols.data[cc] + run[v] * K.width);
              }
            } else {
              atomicOr(dp.overflow, 1u);
            }
            run[v] += nn;
          }
          if (dp.cols.presence) dp.cols.presence[r] = pres;
        }
        c++;
#pragma unroll
        for (int v = 0; v < NV; v++) acc[v] += vs.len[v];
        pos = end;
        if (emit && !known) {
          rec++;
          if (rec == dp.n) {
            write_final(dp.n, pos);
            if (MODE == M_SKIP) dp.skip_out[dp.n] = pos;
          }
        }
        if (known) break;
      }
      if (emit) {
        if (known) {
          if (e) atomicMin(dp.errkey, (unsigned long long)((rrec << 8) | (uint64_t)(e & 0xff)));
          if (dp.rstat) dp.rstat[rrec] = (uint8_t)e;
          if (rrec == dp.n - 1) write_final(dp.n, dp.offsets[dp.n]);
        } else if (e) {
          // the validated chain stops here (single writer: the only error on the chain)
          kx_status* st = dp.status;
          st->code = e; st->record = rec; st->offset = pos;
          write_final(rec, pos);
          if (MODE == M_SKIP) dp.skip_out[rec] = pos;
        }
      }
      ex = e ? X_ERR : pos;
      cnt = c;
#pragma unroll
      for (int v = 0; v < NV; v++) vsum[v] = acc[v];
    }
    need = false;
    if (stage == 2) break;

    if (!known) {
      // ---- one repair round: every lane must start at the first true record start in its
      //      segment, i.e. where the previous walking lane's chain (or `seed`) leaves off ----
      const uint64_t hm = __ballot(ent != X_NONE);
      const uint64_t below = hm & ((1ull << lane) - 1);
      const int pc = below ? 63 - __clzll((long long)below) : -1;
      const uint64_t pex = __shfl(ex, pc < 0 ? 0 : pc, 64);
      const uint64_t pe = pc >= 0 ? pex : seed;
      uint64_t want = ent;
      if (pe != X_NONE) {
        if (pe == X_ERR || pe == X_DONE || seg_lo >= thi || pe >= seg_hi) want = X_NONE;
        else if (pe >= seg_lo) want = pe;
      }
      const bool ch = want != ent;
      if (__ballot(ch)) {
        if (++rounds <= (stage == 0 ? 8 : 70)) {
          if (ch) {
            ent = want;
            need = ent != X_NONE;
            ex = X_NONE;
            cnt = 0;
#pragma unroll
            for (int v = 0; v < NV; v++) vsum[v] = 0;
          }
          continue;
        }
        if (stage == 1) {  // cannot happen: from the true entry the chain settles in <= 65 rounds
          if (lane == 0) atomicCAS((int*)&dp.status->code, 0, KX_ERR_INTERNAL);
          ent = X_NONE;
        }
        ok = false;
      }
      if (stage == 0 && rounds && lane == 0) atomicAdd((unsigned long long*)&dp.status->diag[2], 1ull);
    }
    if (stage == 0) phase(1);

    // ---- wave prefix sums of record counts and arena bytes ----
    {
      const uint64_t em = known ? 0ull : __ballot(ent != X_NONE && ex == X_ERR);
      fel = em ? __ffsll((long long)em) - 1 : 64;
      const bool live = known ? mine : (ent != X_NONE && lane <= fel);
      const uint64_t c0 = live ? cnt : 0;
      const uint64_t inc = wave_incl_scan(c0, lane);
      cpre = inc - c0;
      tile_cnt = rl64(inc, 63);
#pragma unroll
      for (int v = 0; v < NV; v++) {
        const uint64_t x = live ? vsum[v] : 0;
        const uint64_t vi = wave_incl_scan(x, lane);
        vpre[v] = vi - x;
        tile_var[v] = rl64(vi, 63);
      }
      if (!known) {
        const uint64_t hm = __ballot(ent != X_NONE);
        spec_ent = hm ? rl64(ent, __ffsll((long long)hm) - 1) : X_NONE;
        tile_exit = fel < 64 ? X_ERR : hm ? rl64(ex, 63 - __clzll((long long)hm)) : (stage == 0 ? X_NONE : seed);
      }
    }

    if (stage == 0) {
      // ---- publish the aggregate, then look back ----
      if (lane == 0 && (known || ok)) {
        uint64_t words[3 + KXP_NV_MAX];
        words[0] = tile_cnt;
        words[1] = known ? X_NONE : spec_ent;
        words[2] = known ? 0 : tile_exit;
#pragma unroll
        for (int v = 0; v < NV; v++) words[3 + v] = tile_var[v];
        publish_words(dp, t, D_AGG_CNT, words, 3 + NV);
      }
      phase(2);
      lb = lookback<NV>(dp, t, !known, lane);
      lb.e = rfl64(lb.e);
      lb.cnt = rfl64(lb.cnt);
#pragma unroll
      for (int v = 0; v < NV; v++) lb.var[v] = rfl64(lb.var[v]);
      phase(3);
      terminal = lb.e == X_ERR || lb.e == X_DONE || (!known && lb.cnt >= dp.n);
      if (!known && !terminal) {
        const bool valid = ok && (spec_ent == X_NONE ? lb.e >= thi : lb.e == spec_ent);
        if (!valid) {
          if (lane == 0) atomicAdd((unsigned long long*)&dp.status->diag[0], 1ull);
          stage = 1;
          seed = lb.e;
          rounds = 0;
          ok = true;
          continue;
        }
        if (spec_ent == X_NONE) tile_exit = lb.e;  // pass-through tile
      }
    }

    // ---- publish the inclusive prefix ----
    if (lane == 0) {
      uint64_t words[2 + KXP_NV_MAX];
      uint64_t xo;
      const uint64_t base = lb.cnt;
      if (known) {
        xo = 0;
        words[0] = base + tile_cnt;
      } else if (terminal) {
        xo = lb.e == X_DONE || base >= dp.n ? X_DONE : X_ERR;
        words[0] = base;
      } else {
        const uint64_t tot = base + tile_cnt;
        xo = tile_exit;
        if (tot >= dp.n) {
          xo = X_DONE;
        } else if (xo == dp.in_len) {
          // the input ends before n records: EOF at record `tot`
          xo = X_ERR;
          kx_status* st = dp.status;
          st->code = KX_ERR_EOF; st->record = tot; st->offset = dp.in_len;
          st->n_records = tot; st->consumed = dp.in_len;
#pragma unroll
          for (int v = 0; v < NV; v++) {
            if (v >= (int)nvar) break;
            const uint64_t vt = lb.var[v] + tile_var[v];
            st->var_total[v] = vt;
            dp.cols.offs[P->var_col[v]][tot] = (uint32_t)vt;
          }
          if (MODE == M_SKIP) dp.skip_out[tot] = dp.in_len;
        }
        words[0] = tot;
      }
      words[1] = xo;
#pragma unroll
      for (int v = 0; v < NV; v++) words[2 + v] = lb.var[v] + tile_var[v];
      publish_words(dp, t, D_INC_CNT, words, 2 + NV);
    }
    phase(4);
    if (!known && terminal) break;

    // ---- walk 2 ----
    need = known ? mine : (ent != X_NONE && lane <= fel);
    rec = lb.cnt + cpre;
#pragma unroll
    for (int v = 0; v < NV; v++) run[v] = lb.var[v] + vpre[v];
    stage = 2;
  }
  phase(5);
}

// Completes a call and re-arms the workspace for the next one (tile counter, error key, overflow).
__global__ void finalize_kernel(kx_status* st, unsigned long long* errkey, uint32_t* overflow, uint32_t* counter,
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
  *errkey = ~0ull;
  *overflow = 0;
  *counter = 0;
}

// workspace: [0] tile counter u32, [8] errkey u64, [16] overflow u32, [256...) tile descriptors
constexpr size_t WS_DESC = 256;

size_t ws_total(uint64_t ntiles) { return WS_DESC + ntiles * DFIELDS * 8; }

// offsets mode: records per tile so that a tile's bytes fit the LDS window on average
uint32_t krec_for(uint64_t in_len, uint64_t n) {
  if (n == 0) return 64;
  const uint64_t avg = (in_len + n - 1) / n;
  const uint64_t k = avg ? (uint64_t)TILE / avg : 64;
  return (uint32_t)(k < 1 ? 1 : k > 64 ? 64 : k);
}

uint64_t tiles_for(uint64_t in_len, const uint64_t* offsets, uint64_t n) {
  const uint64_t nt = offsets ? (n + krec_for(in_len, n) - 1) / krec_for(in_len, n) : (in_len + TILE - 1) / TILE;
  return nt ? nt : 1;
}

template <int NV, int MODE>
int launch_t(const DecParams& dp0, void* ws, hipStream_t stream) {
  DecParams dp = dp0;
  char* base = (char*)ws;
  dp.counter = (uint32_t*)base;
  dp.errkey = (unsigned long long*)(base + 8);
  dp.overflow = (uint32_t*)(base + 16);
  dp.desc = (uint64_t*)(base + WS_DESC);
  KX_HIP_CHECK(hipMemsetAsync(dp.status, 0, sizeof(kx_status), stream));
  const unsigned grid = (unsigned)((dp.ntiles + WAVES - 1) / WAVES);
  hipLaunchKernelGGL((decode_kernel<NV, MODE>), dim3(grid), dim3(NT), 0, stream, dp);
  KX_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(64), 0, stream, dp.status, dp.errkey, dp.overflow,
                     dp.counter, dp.offsets, dp.n);
  KX_HIP_CHECK(hipGetLastError());
  return KX_OK;
}

void fill_diag_flags(DecParams& dp) {
  static int timing = -1, nolds = -1;
  if (timing < 0) { const char* e = getenv("KX_PHASE_TIMING"); timing = e && e[0] == '1'; }
  if (nolds < 0) { const char* e = getenv("KX_NOLDS"); nolds = e && e[0] == '1'; }
  dp.timing = timing;
  dp.nolds = nolds;
}

}  // namespace

size_t kx_decode_ws_bytes(const KxProgram&, uint64_t in_len, const uint64_t* offsets, uint64_t n) {
  return ws_total(tiles_for(in_len, offsets, n));
}

size_t kx_skip_ws_bytes(uint64_t in_len) { return ws_total(tiles_for(in_len, nullptr, 0)); }

// diagnostics (not part of the public ABI): read and reset the phase-timing accumulators
extern "C" int kx_debug_phase_cycles(unsigned long long* out, int n) {
  if (n > 10) n = 10;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), sizeof(unsigned long long) * n) != hipSuccess) return KX_ERR_HIP;
  unsigned long long z[10] = {0};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof z) != hipSuccess) return KX_ERR_HIP;
  return KX_OK;
}

int kx_launch_decode(const KxProgram* dprog, const KxProgram& hprog, const uint8_t* in, uint64_t in_len,
                     const uint64_t* offsets, uint64_t n, const KxLaunchCols& cols, uint8_t* record_status,
                     kx_status* status, void* ws, size_t ws_size, uint64_t epoch, hipStream_t stream, bool pb) {
  if (pb) return KX_ERR_NOT_IMPLEMENTED;
  DecParams dp{};
  fill_diag_flags(dp);
  dp.in = in; dp.in_len = in_len; dp.offsets = offsets; dp.n = n; dp.prog = dprog;
  dp.cols = cols; dp.rstat = record_status; dp.status = status; dp.epoch = epoch;
  dp.krec = krec_for(in_len, n);
  dp.ntiles = tiles_for(in_len, offsets, n);
  if (ws_size < ws_total(dp.ntiles)) return KX_ERR_INVALID_ARG;
  switch (hprog.nvar) {
    case 0: return launch_t<0, M_THRIFT>(dp, ws, stream);
    case 1: return launch_t<1, M_THRIFT>(dp, ws, stream);
    case 2: return launch_t<2, M_THRIFT>(dp, ws, stream);
    case 3: case 4: return launch_t<4, M_THRIFT>(dp, ws, stream);
    default: return launch_t<8, M_THRIFT>(dp, ws, stream);
  }
}

int kx_launch_skip(const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t* offsets_out, kx_status* status,
                   void* ws, size_t ws_size, uint64_t epoch, hipStream_t stream) {
  DecParams dp{};
  fill_diag_flags(dp);
  dp.in = in; dp.in_len = in_len; dp.offsets = nullptr; dp.n = n; dp.prog = nullptr;
  dp.status = status; dp.skip_out = offsets_out; dp.epoch = epoch;
  dp.krec = 64;
  dp.ntiles = tiles_for(in_len, nullptr, n);
  if (ws_size < ws_total(dp.ntiles)) return KX_ERR_INVALID_ARG;
  return launch_t<0, M_SKIP>(dp, ws, stream);
}
