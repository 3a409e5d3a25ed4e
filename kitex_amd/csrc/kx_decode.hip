// kx_decode.hip — batched Thrift-binary FastRead (and the skip decoder) on CDNA4 / gfx950.
//
// Reference semantics: generated FastRead (tool/internal_pkg/pluginmode/thriftgo/struct_tpl.go:41-149,
// 405-625; instance internal/mocks/thrift/k-mock.go:39-184) over N records, as fastUnmarshal does per
// message (pkg/remote/codec/thrift/codec_fast.go:60-82) or as the element loop of a list<Struct>;
// unknown / mistyped fields go through the skip decoder (codec_apache.go:191-293).
//
// Design: ONE persistent kernel; every input byte is read from HBM once.
//   A workgroup of 8 waves owns a super-tile (ST) of 8 tiles x 8 KiB at a time (persistent grid,
//   super-tiles dealt round-robin). Each wave pulls its tile (+ a 512-byte halo for the record
//   straddling its end) into LDS by LDS-DMA (global_load_lds_dwordx4) and walks it speculatively:
//   lane l owns the 128-byte segment l, starts at the first canonical record signature in it and
//   walks records (schema-aware FastRead lengths) until it leaves the segment; lanes repair each
//   other with wave shuffles until the chain is consistent. The 8 tile aggregates are chained in
//   LDS into the ST aggregate (entry, exit, records, arena bytes, first error), which is published
//   as epoch-tagged words; a decoupled look-back over the preceding STs (with a chain-consistency
//   check at every boundary: a tile's speculative entry must be where the chain below exits) gives
//   the ST's true entry and its record / arena bases. A tile whose speculation was wrong is re-walked
//   from its true entry out of LDS. Then every wave emits its tile from LDS (lane = segment):
//   fixed-width fields are stored as parsed, strings / lists are copied with 16-byte stores.
//   Known-offsets mode (fastUnmarshal with dataLen): a tile is up to 64 records, lane = record; the
//   look-back carries only arena bytes (none at all when the schema has no var columns).
// Canonical records (the encoder's layout) take a straight-line step plan compiled from the schema;
// anything else takes the generic field loop. Records or strings reaching past the LDS window are
// read from global memory (same code, other source).
// No MFMA anywhere: this is byte movement, bounded by HBM bandwidth.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "kx_internal.h"

#define LDS __attribute__((address_space(3)))
#define GLB __attribute__((address_space(1)))
#define KAS __attribute__((address_space(4)))  // kernarg segment (read in place, never copied to scratch)

namespace {

constexpr int WGW = 8;                   // waves per workgroup = tiles per super-tile
constexpr int NT = WGW * 64;
constexpr int SEG = 128;                 // bytes per lane segment
constexpr int TILE = 64 * SEG;           // 8 KiB of input per wave
constexpr int HALO = 256;                // the record straddling the tile end is read from LDS up to here
constexpr int WINB = TILE + HALO + 16;   // LDS window bytes (+16 for the aligned-down start)
constexpr int WINW = WINB / 4 + 4;       // window dwords (+ pad for the last aligned read pair)
constexpr int WIN_LOADS = (WINB / 16 + 63) / 64;

constexpr uint64_t V48 = (1ull << 48) - 1;
constexpr uint64_t X_ERR = V48;          // chain terminated by a decode error
constexpr uint64_t X_NONE = V48 - 2;     // no record start (candidate / entry / exit unknown)

// super-tile descriptor words (structure of arrays over STs, epoch-tagged):
//   A = the ST's speculative aggregate, P = the inclusive prefix through the ST
enum { A_S = 0, A_X, A_C, A_EC, A_EP, A_V, P_X = A_V + KXP_NV_MAX, P_C, P_EC, P_EP, P_V,
       S_NF = P_V + KXP_NV_MAX };

enum Mode { M_THRIFT = 0, M_SKIP = 1, M_PB = 2 };

struct DecParams {
  const uint8_t* in;
  uint64_t in_len;
  const uint64_t* offsets;   // known-offsets mode when non-null
  uint64_t n;
  const KAS KxProgram* prog;  // compiled schema (constant address space: scalar loads when uniform)
  KxLaunchCols cols;
  uint8_t* rstat;
  kx_status* status;
  uint64_t* skip_out;        // M_SKIP: record start offsets
  uint64_t* sdesc;           // super-tile words
  unsigned long long* errkey;  // offsets mode: min((record << 8) | code)
  uint32_t* overflow;        // an arena capacity (or the 4-byte offset range) was exceeded
  uint32_t* abort;           // a look-back wait timed out: every other wait gives up at once
  unsigned long long* ticket;  // super-tiles handed out so far (claimed in order: deadlock-free look-back)
  unsigned long long* progress;  // inclusive prefixes published so far (the look-back watchdog's clock)
  uint64_t ntiles, nst;
  uint64_t epoch;            // 16-bit call epoch (never 0)
  uint32_t krec;             // offsets mode: records per tile (<= 64)
  int direct;                // offsets mode without var columns: no look-back
  int nolds;                 // diagnostics (KX_NOLDS=1): read every byte from global memory
  int diag;
};

// Kernels read their parameter block in place from the kernarg segment: indexing a by-value
// parameter (cols.data[c]) would otherwise make the compiler copy the whole block to scratch per lane.
typedef const KAS DecParams KParams;
#define KX_PARAMS() (*(KParams*)__builtin_amdgcn_kernarg_segment_ptr())

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
  const KAS KxpStep* steps;  // canonical plan (uniform index -> scalar loads)
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
  return p < w.len ? ((const GLB uint8_t*)w.in)[p] : 0u;
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

// refused out-of-range device accesses (never expected; a bit per site lands in kx_status.diag[2])
enum { G_ROUNDS = 1, G_LB_WAIT = 2, G_LB_SLOW = 4, G_NFIX = 8, G_COMBINE = 16, G_COLUMN = 32, G_OFFSET = 64,
       G_ROWS = 128, G_WORD = 256 };

__device__ __forceinline__ void store_col_(void* base, uint32_t width, uint64_t rec, uint64_t v);
// store value v of record rec into fixed column col
__device__ __forceinline__ void store_col(const KAS KxLaunchCols& cols, int col, uint32_t width, uint64_t rec,
                                          uint64_t v) {
  if (rec >= cols.nrec || col < 0 || col >= KX_MAX_COLUMNS) {
    atomicOr(cols.guard, (unsigned long long)G_COLUMN);
    return;
  }
  store_col_(cols.data[col], width, rec, v);
}

__device__ __forceinline__ void store_col_(void* base, uint32_t width, uint64_t rec, uint64_t v) {
  switch (width) {
    case 1: ((GLB uint8_t*)base)[rec] = (uint8_t)v; break;
    case 2: ((GLB uint16_t*)base)[rec] = (uint16_t)v; break;
    case 4: ((GLB uint32_t*)base)[rec] = (uint32_t)v; break;
    default: ((GLB uint64_t*)base)[rec] = v; break;
  }
}

// program tables live in the constant address space: a uniform index becomes a scalar load
template <typename T>
__device__ __forceinline__ T ldk(const KAS T* p) {
  static_assert(sizeof(T) % 4 == 0, "dword-sized tables");
  uint32_t w[sizeof(T) / 4];
  const KAS uint32_t* q = (const KAS uint32_t*)p;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); i++) w[i] = q[i];
  T v;
  __builtin_memcpy(&v, w, sizeof(T));
  return v;
}
__device__ __forceinline__ KxpField ld_field(const KAS KxProgram* P, int i) { return ldk(&P->f[i]); }
__device__ __forceinline__ KxpInst ld_inst(const KAS KxProgram* P, int i) { return ldk(&P->inst[i]); }
__device__ __forceinline__ KxpCol ld_col(const KAS KxProgram* P, int i) { return ldk(&P->col[i]); }

// Canonical fast path: the record is checked against the schema's canonical plan (header bytes in
// encoder order, STOP bytes). The step index is wave-uniform (scalar loads); a lane whose record
// deviates returns false and the record is re-parsed by the generic loop.
template <int NV>
__device__ __forceinline__ bool canon_record(const Src& w, const KAS KxLaunchCols& cols, uint64_t start, uint64_t limit,
                                             uint64_t rec, bool emit, uint64_t* endp, VarState<NV>& vs) {
  uint64_t pos = start;
  const KAS KxpStep* __restrict__ steps = w.steps;
  uint32_t k = 0;
  while (k < w.nsteps) {
    // every lane still on the plan is at the same step: make that explicit so the plan is read
    // with scalar loads (a per-lane index would turn each step into a vector memory round trip)
    k = __builtin_amdgcn_readfirstlane(k);
    const KxpStep st = ldk(&steps[k]);
    const uint64_t rem = limit - pos;
    if (st.kind == KXP_S_FIXED) {
      // up to 4 consecutive fixed-width fields: their positions do not depend on data
      const uint32_t m = min(st.hdr >> 24, 4u);
      const KxpStep s1 = ldk(&steps[k + (m > 1 ? 1 : 0)]);
      const KxpStep s2 = ldk(&steps[k + (m > 2 ? 2 : 0)]);
      const KxpStep s3 = ldk(&steps[k + (m > 3 ? 3 : 0)]);
      const uint32_t o1 = 3 + st.width, o2 = o1 + 3 + s1.width, o3 = o2 + 3 + s2.width;
      const uint32_t len = m == 1 ? o1 : m == 2 ? o2 : m == 3 ? o3 : o3 + 3 + s3.width;
      if (rem < len) return false;
      // the walk (measure) pass only checks the headers: 2 dwords per field instead of 4
      Fetch f0, f1, f2, f3;
      if (emit) {
        f0 = fetch12(w, pos); f1 = fetch12(w, pos + o1); f2 = fetch12(w, pos + o2); f3 = fetch12(w, pos + o3);
      } else {
        f0.w0 = ld4(w, pos); f1.w0 = ld4(w, pos + o1); f2.w0 = ld4(w, pos + o2); f3.w0 = ld4(w, pos + o3);
        f0.w1 = f0.w2 = f1.w1 = f1.w2 = f2.w1 = f2.w2 = f3.w1 = f3.w2 = 0;
      }
      bool ok = (f0.w0 & 0xffffffu) == (st.hdr & 0xffffffu);
      if (m > 1) ok &= (f1.w0 & 0xffffffu) == (s1.hdr & 0xffffffu);
      if (m > 2) ok &= (f2.w0 & 0xffffffu) == (s2.hdr & 0xffffffu);
      if (m > 3) ok &= (f3.w0 & 0xffffffu) == (s3.hdr & 0xffffffu);
      if (!ok) return false;
      if (emit) {
        store_col(cols, st.col, st.width, rec, fixed_after_header(f0, st.hdr & 0xff));
        if (m > 1) store_col(cols, s1.col, s1.width, rec, fixed_after_header(f1, s1.hdr & 0xff));
        if (m > 2) store_col(cols, s2.col, s2.width, rec, fixed_after_header(f2, s2.hdr & 0xff));
        if (m > 3) store_col(cols, s3.col, s3.width, rec, fixed_after_header(f3, s3.hdr & 0xff));
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
__device__ __forceinline__ int generic_record(const Src& w, const KAS KxProgram* P, const KAS KxLaunchCols& cols,
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
      if (emit) store_col(cols, F.col, wd, rec, fixed_after_header(fx, t));
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
      if (K.kind == KXP_K_FIXED && !((seen >> K.field) & 1)) store_col(cols, (int)c, K.width, rec, (uint64_t)K.defv);
    }
  }
  pres_out = pres;
  *endp = pos;
  return KX_OK;
}

__device__ __forceinline__ void emit_defaults(const KAS KxProgram* P, const KAS KxLaunchCols& cols, uint64_t rec) {
  for (uint32_t c = 0; c < P->ncols; c++) {
    const KxpCol K = ld_col(P, c);
    if (K.kind == KXP_K_FIXED) store_col(cols, (int)c, K.width, rec, (uint64_t)K.defv);
  }
}

// ---------------------------------------------------------------------------------------------
// Kitex-Protobuf body: proto.Unmarshal of a flat proto3 message
// (protobuf.go:135-170; protowire rules as restated in oracle/kx_oracle.c pb_reader): fields in any
// order, unknown numbers and mismatched wire types skipped, the last occurrence wins, `string`
// fields UTF-8 validated, groups (wire types 3/4) rejected.
// ---------------------------------------------------------------------------------------------
// protowire.ConsumeVarint of the varint starting at byte 0 of f: at most 10 bytes, the 10th <= 1;
// `rem` bytes are available. Branch-free SWAR: the terminator is the first byte with bit 7 clear,
// the 7-bit groups of the first 8 bytes are compacted in three shift/mask steps.
__device__ __forceinline__ int pb_varint_f(const Fetch& f, uint64_t rem, uint64_t& v, uint32_t& used) {
  if (!(f.w0 & 0x80u)) {  // one byte: tags, lengths < 128, small values (usually wave-uniform)
    if (rem < 1) return KX_ERR_EOF;
    v = f.w0 & 0x7fu;
    used = 1;
    return KX_OK;
  }
  const uint64_t lo = (uint64_t)f.w0 | ((uint64_t)f.w1 << 32);
  const uint64_t stop = ~lo & 0x8080808080808080ull;
  const uint32_t b8 = f.w2 & 0xffu, b9 = (f.w2 >> 8) & 0xffu;
  const uint32_t k = stop ? (uint32_t)__builtin_ctzll(stop) >> 3 : b8 < 0x80 ? 8u : b9 < 0x80 ? 9u : 10u;
  if (k >= 9) {  // the 10th byte decides: it must exist, and be <= 1
    if (rem <= 9) return KX_ERR_EOF;
    if (b9 > 1) return KX_ERR_INVALID_DATA;
  } else if ((uint64_t)k >= rem) {
    return KX_ERR_EOF;
  }
  const uint64_t keep = k >= 7 ? ~0ull : (2ull << (8 * k + 7)) - 1;  // bytes 0..k
  uint64_t x = lo & keep & 0x7f7f7f7f7f7f7f7full;
  x = (x & 0x007f007f007f007full) | ((x & 0x7f007f007f007f00ull) >> 1);
  x = (x & 0x00003fff00003fffull) | ((x & 0x3fff00003fff0000ull) >> 2);
  x = (x & 0x000000000fffffffull) | ((x & 0x0fffffff00000000ull) >> 4);
  if (k >= 8) x |= (uint64_t)(b8 & 0x7f) << 56;
  if (k >= 9) x |= (uint64_t)(b9 & 0x01) << 63;
  v = x;
  used = k + 1;
  return KX_OK;
}

__device__ __forceinline__ int pb_varint(const Src& w, uint64_t p, uint64_t rem, uint64_t& v, uint32_t& used) {
  return pb_varint_f(fetch12(w, p), rem, v, used);
}

// the 12-byte fetch advanced by u (<= 2) bytes: the value after a 1- or 2-byte tag
__device__ __forceinline__ Fetch fetch_skip(const Fetch& f, uint32_t u) {
  Fetch g;
  g.w0 = __builtin_amdgcn_alignbyte(f.w1, f.w0, u);
  g.w1 = __builtin_amdgcn_alignbyte(f.w2, f.w1, u);
  g.w2 = __builtin_amdgcn_alignbyte(0u, f.w2, u);
  return g;
}

// utf8.Valid (what protobuf-go enforces on proto3 `string` fields), byte by byte
__device__ __forceinline__ bool pb_utf8_slow(const Src w, uint64_t p, uint64_t n) {
  uint64_t i = 0;
  while (i < n) {
    const uint32_t c = ld1(w, p + i);
    if (c < 0x80) { i++; continue; }
    uint32_t k, cp;
    if ((c & 0xe0) == 0xc0) { k = 1; cp = c & 0x1f; }
    else if ((c & 0xf0) == 0xe0) { k = 2; cp = c & 0x0f; }
    else if ((c & 0xf8) == 0xf0) { k = 3; cp = c & 0x07; }
    else return false;
    if (i + k >= n) return false;  // truncated sequence
    for (uint32_t j = 1; j <= k; j++) {
      const uint32_t d = ld1(w, p + i + j);
      if ((d & 0xc0) != 0x80) return false;
      cp = (cp << 6) | (d & 0x3f);
    }
    if ((k == 1 && cp < 0x80) || (k == 2 && cp < 0x800) || (k == 3 && cp < 0x10000)) return false;
    if (cp > 0x10ffff || (cp >= 0xd800 && cp <= 0xdfff)) return false;
    i += k + 1;
  }
  return true;
}

// ASCII fast path from the LDS window (OR of the covering dwords), else the full check
__device__ __forceinline__ bool pb_utf8_ok(const Src& w, uint64_t p, uint64_t n) {
  if (n == 0) return true;
  const int32_t q = n <= 4096 ? wofs(w, p, (uint32_t)n) : -1;
  if (q >= 0) {
    const LDS uint32_t* s = w.win + (q >> 2);
    const int sh = q & 3;
    const int nd = (sh + (int)n + 3) >> 2;
    const int tail = (sh + (int)n) & 3;
    uint32_t acc = 0;
    for (int i = 0; i < nd; i++) {
      uint32_t m = 0xffffffffu;
      if (i == 0) m &= 0xffffffffu << (8 * sh);
      if (i == nd - 1 && tail) m &= 0xffffffffu >> (8 * (4 - tail));
      acc |= s[i] & m;
    }
    if (!(acc & 0x80808080u)) return true;
  }
  return pb_utf8_slow(w, p, n);
}

template <int NV>
__device__ __forceinline__ int pb_body(const Src& w, const KAS KxProgram* P, const KAS KxLaunchCols& cols,
                                       uint64_t start, uint64_t limit, uint64_t rec, bool emit,
                                       VarState<NV>& vs, uint64_t& pres_out, bool utf8 = true) {
  uint64_t pos = start, seen = 0, pres = 0;
  const int nf = (int)P->nfields;
  int pred = 0;  // fields usually arrive in field-number order: try the one after the last match first
  while (pos < limit) {
    uint64_t tag;
    uint32_t u;
    const Fetch ft = fetch12(w, pos);
    int rc = pb_varint_f(ft, limit - pos, tag, u);
    if (rc) return rc;
    pos += u;
    // value bytes: from the same fetch when the tag is short (value varints need <= 10 of the
    // remaining 12 - u bytes)
    const Fetch fv = u <= 2 ? fetch_skip(ft, u) : fetch12(w, pos);
    const uint64_t num = tag >> 3;
    const uint32_t wt = (uint32_t)tag & 7u;
    if (num == 0 || num > 536870911ull) return KX_ERR_INVALID_DATA;
    const int id = num <= 32767 ? (int)num : -1;
    int fi = -1;
    KxpField F = ld_field(P, pred);
    if (id >= 0 && pred < nf && F.id == id) {
      fi = pred;
    } else if (id >= 0) {
      for (int k = 0; k < nf; k++)
        if (P->f[k].id == id) { fi = k; break; }
      if (fi >= 0) F = ld_field(P, fi);
    }
    const uint64_t rem = limit - pos;
    if (fi < 0 || F.pb_wt != wt) {  // unknown number / other wire type: skipped (ConsumeFieldValue)
      if (wt == 0) {
        uint64_t v;
        if ((rc = pb_varint_f(fv, rem, v, u))) return rc;
        pos += u;
      } else if (wt == 1 || wt == 5) {
        const uint32_t k = wt == 1 ? 8u : 4u;
        if (rem < k) return KX_ERR_EOF;
        pos += k;
      } else if (wt == 2) {
        uint64_t l;
        if ((rc = pb_varint_f(fv, rem, l, u))) return rc;
        if (l > rem - u) return KX_ERR_EOF;
        pos += u + l;
      } else {
        return KX_ERR_INVALID_DATA;  // groups and reserved wire types
      }
      continue;
    }
    pred = fi + 1 < nf ? fi + 1 : 0;
    if (wt == 0) {
      uint64_t v;
      if ((rc = pb_varint_f(fv, rem, v, u))) return rc;
      pos += u;
      if (F.ttype == KX_T_BOOL) v = v != 0;
      if (emit) store_col(cols, F.col, F.width, rec, v);  // int32: low 32 bits
    } else if (wt == 1) {
      if (rem < 8) return KX_ERR_EOF;
      if (emit) store_col(cols, F.col, F.width, rec, (uint64_t)fv.w0 | ((uint64_t)fv.w1 << 32));
      pos += 8;
    } else {
      uint64_t l;
      if ((rc = pb_varint_f(fv, rem, l, u))) return rc;
      pos += u;
      if (l > rem - u) return KX_ERR_EOF;
      if (utf8 && !(F.flags & 1) && !pb_utf8_ok(w, pos, l)) return KX_ERR_INVALID_DATA;
      vset<NV>(vs, F.vslot, pos, (uint32_t)l);
      pos += l;
    }
    seen |= 1ull << fi;
    if (F.pbit >= 0) pres |= 1ull << F.pbit;
  }
  if (emit) {
    // fields never seen keep their (proto3 zero / schema) default
    for (uint32_t c = 0; c < P->ncols; c++) {
      const KxpCol K = ld_col(P, c);
      if (K.kind == KXP_K_FIXED && !((seen >> K.field) & 1)) store_col(cols, (int)c, K.width, rec, (uint64_t)K.defv);
    }
  }
  pres_out = pres;
  return KX_OK;
}

// ---------------------------------------------------------------------------------------------
// variable-length payload copy (strings: raw bytes; lists: big-endian elements -> host order)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void copy_var_slow(const Src w, KxpCol K, uint64_t src, uint32_t n, uint8_t* dst_) {
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

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
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

// ---------------------------------------------------------------------------------------------
// self-tagged descriptor words (16-bit call epoch << 48 | 48-bit value), structure of arrays:
// word f of item i lives at base[f * nitems + i]. A word is valid iff its tag is this call's, so no
// per-call clearing and no fences: a reader polls the words it needs until their tags match.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void put_word(uint64_t* base, uint64_t nitems, int f, uint64_t i, uint64_t ep,
                                         uint64_t v) {
  astore64(base + (uint64_t)f * nitems + i, (ep << 48) | (v & V48));
}

// 0x80 in the lowest byte of v that is 0x00 (bytes above it may be flagged spuriously)
__device__ __forceinline__ uint32_t low_zero_byte(uint32_t v) { return (v - 0x01010101u) & ~v & 0x80808080u; }

// 0x80 in every byte of v that is 0x00, nothing elsewhere (exact, no borrow false positives)
__device__ __forceinline__ uint32_t zero_bytes(uint32_t v) {
  return ~(((v & 0x7f7f7f7fu) + 0x7f7f7f7fu) | v | 0x7f7f7f7fu);
}

// bytes j of the stream x0|x1 (little-endian dwords) where bytes j, j+1, j+2 equal the signature
// (the lowest flagged byte of the borrow-based zero test is exact, and only the lowest is used)
__device__ __forceinline__ uint32_t sig_hits(uint32_t x0, uint32_t x1, uint32_t b0, uint32_t b1, uint32_t b2) {
  return low_zero_byte((x0 ^ b0) | (__builtin_amdgcn_alignbyte(x1, x0, 1) ^ b1) |
                    (__builtin_amdgcn_alignbyte(x1, x0, 2) ^ b2));
}

// byte index of the lowest hit, or >= 0x1fffffff when there is none (v_ffbl returns -1 for 0)
__device__ __forceinline__ uint32_t first_hit(uint32_t m) { return (uint32_t)(__builtin_ffs((int)m) - 1) >> 3; }

// first canonical signature (3 bytes) in a lane's 128-byte segment, read from the LDS window. All
// four alignments of a dword are tested at once (byte j matches iff bytes j, j+1, j+2 equal the
// signature: OR of the three XORs is zero), so the loop is branch- and select-free whatever the data
// (the first signature byte alone, e.g. 0x0A = T_I64, occurs every few bytes). Segments are 128 B
// apart, so lanes reading dword i of their segment together would all hit one LDS bank; each lane
// starts at dword (lane mod 33) and rotates through its 33 dwords (conflict-free), keeping the lowest
// hit. Hits before the segment start wrap to huge unsigned offsets and lose every min; a hit of the
// first dword that sits above such a one is missed, which only costs a repair round (the candidate
// is speculation: the chain from the lane / tile below decides).
__device__ __forceinline__ uint64_t scan_segment(const Src& w, int32_t q0, uint64_t seg_lo, uint64_t plim,
                                                 uint32_t sig, int lane) {
  const LDS uint32_t* s = w.win + (q0 >> 2);
  const uint32_t sh0 = q0 & 3;
  const uint32_t b0 = (sig & 0xff) * 0x01010101u, b1 = ((sig >> 8) & 0xff) * 0x01010101u;
  const uint32_t b2 = ((sig >> 16) & 0xff) * 0x01010101u;
  uint32_t best = SEG;
  int idx = lane % 33;
#pragma unroll 3
  for (int i = 0; i < 33; i++) {
    const uint32_t m = sig_hits(s[idx], s[idx + 1], b0, b1, b2);
    best = min(best, (uint32_t)(4 * idx) - sh0 + first_hit(m));
    idx = idx == 32 ? 0 : idx + 1;
  }
  return (best < (uint32_t)SEG && seg_lo + best < plim) ? seg_lo + best : X_NONE;
}

// the two lowest signature offsets of the segment (same scan; >= SEG when absent), for schemas
// whose signature also starts a nested struct
__device__ __forceinline__ void scan_segment2(const Src& w, int32_t q0, uint32_t sig, int lane, uint32_t& c1,
                                              uint32_t& c2) {
  const LDS uint32_t* s = w.win + (q0 >> 2);
  const uint32_t sh0 = q0 & 3;
  const uint32_t b0 = (sig & 0xff) * 0x01010101u, b1 = ((sig >> 8) & 0xff) * 0x01010101u;
  const uint32_t b2 = ((sig >> 16) & 0xff) * 0x01010101u;
  c1 = ~0u;
  c2 = ~0u;
  int idx = lane % 33;
  for (int i = 0; i < 33; i++) {
    const uint32_t x0 = s[idx], x1 = s[idx + 1];
    uint32_t m = zero_bytes((x0 ^ b0) | (__builtin_amdgcn_alignbyte(x1, x0, 1) ^ b1) |
                            (__builtin_amdgcn_alignbyte(x1, x0, 2) ^ b2));
    const uint32_t base = (uint32_t)(4 * idx) - sh0;
    const uint32_t h1 = base + first_hit(m);
    m &= m - 1;
    const uint32_t h2 = base + first_hit(m);
    const uint32_t lo = min(c1, h1);
    c2 = min(min(c2, h2), max(c1, h1));
    c1 = lo;
    idx = idx == 32 ? 0 : idx + 1;
  }
}

// Kitex-Protobuf record candidate at p: a Batch frame header (0x0A, uvarint length) whose body fits
// the input, starts with a plausible tag, and is followed by the next frame's 0x0A (or the end).
__device__ __forceinline__ int pb_varint(const Src& w, uint64_t p, uint64_t rem, uint64_t& v, uint32_t& used);
__device__ __forceinline__ bool pb_frame_ok(const Src& w, uint64_t p, uint64_t len) {
  uint64_t l;
  uint32_t u;
  if (p + 1 >= len || pb_varint(w, p + 1, len - p - 1, l, u) || u > 5 || l > len - p - 1 - u) return false;
  const uint64_t b = p + 1 + u, e = b + l;
  if (l) {
    const uint32_t t = ld1(w, b), wt = t & 7;
    if (t < 8 || wt == 3 || wt == 4 || wt > 5) return false;
  }
  return e == len || ld1(w, e) == 0x0Au;
}

// Kitex-Protobuf candidate in a lane's segment [seg_lo, seg_hi): the rotated, conflict-free scan
// (as scan_segment) keeps the two lowest 0x0A bytes, then only those two are validated as frame
// headers. Frame validation is a varint decode plus two probes, far too costly to run for every
// 0x0A byte inside the scan loop (a divergent branch taken by the whole wave). If neither validates
// the lane has no candidate and takes its entry from the chain below (speculation only).
__device__ __forceinline__ uint64_t pb_scan_segment(const Src& w, uint64_t seg_lo, uint64_t seg_hi, uint64_t len,
                                                    int lane) {
  const int32_t q0 = wofs(w, seg_lo, SEG + 8);
  const uint32_t n = (uint32_t)(seg_hi - seg_lo);
  uint32_t c1 = ~0u, c2 = ~0u;  // the two lowest 0x0A offsets in the segment
  if (q0 >= 0 && n == SEG) {
    const LDS uint32_t* s = w.win + (q0 >> 2);
    const uint32_t sh0 = q0 & 3;
    int idx = lane % 33;
#pragma unroll 3
    for (int i = 0; i < 33; i++) {
      uint32_t m = zero_bytes(s[idx] ^ 0x0A0A0A0Au);
      const uint32_t base = (uint32_t)(4 * idx) - sh0;  // bytes before the segment wrap to huge offsets
      const uint32_t h1 = base + first_hit(m);
      m &= m - 1;
      const uint32_t h2 = base + first_hit(m);
      const uint32_t lo = min(c1, h1);
      c2 = min(min(c2, h2), max(c1, h1));
      c1 = lo;
      idx = idx == 32 ? 0 : idx + 1;
    }
  } else {
    for (uint32_t rel = 0; rel < n; rel++)
      if (ld1(w, seg_lo + rel) == 0x0Au) {
        if (c1 == ~0u) c1 = rel;
        else { c2 = rel; break; }
      }
  }
  if (c1 < n && pb_frame_ok(w, seg_lo + c1, len)) return seg_lo + c1;
  if (c2 < n && pb_frame_ok(w, seg_lo + c2, len)) return seg_lo + c2;
  return X_NONE;
}

// ---------------------------------------------------------------------------------------------
// the decode pipeline
// ---------------------------------------------------------------------------------------------
// HBM -> LDS window for input position `lo` (all DMA chunks in flight together)
// the window descriptor for input position `lo` (what load_window DMA'd there; cheap to recompute)
// (whole 16-byte chunks inside the input only: the last < 16 bytes of the input are read from HBM)
__device__ __forceinline__ int32_t window_len(KParams& dp, uint64_t wbase) {
  const uint64_t end = (uint64_t)dp.in + dp.in_len;
  return dp.nolds || end < wbase + 16 ? 0 : (int32_t)min((uint64_t)WINB, (end - wbase) & ~15ull);
}

__device__ __forceinline__ Src window_src(KParams& dp, LDS uint32_t* win, uint64_t lo, bool thrift) {
  const uint64_t abs_in = (uint64_t)dp.in;
  const uint64_t wbase = (abs_in + min(lo, dp.in_len)) & ~15ull;
  const int32_t wlen = window_len(dp, wbase);
  const KAS KxProgram* P = dp.prog;
  return Src{dp.in, dp.in_len, wbase - abs_in, wlen, win, thrift ? P->steps : nullptr, thrift ? P->nsteps : 0u,
             thrift ? P->canon_pres : 0ull};
}

// HBM -> LDS window for input position `lo` (all DMA chunks in flight together)
__device__ __forceinline__ void load_window(KParams& dp, LDS uint32_t* win, uint64_t lo, int lane) {
  const uint64_t abs_in = (uint64_t)dp.in;
  const uint64_t wbase = (abs_in + min(lo, dp.in_len)) & ~15ull;
  const int32_t wlen = window_len(dp, wbase);
  const int nch = wlen >> 4;
  const GLB uint8_t* g = (const GLB uint8_t*)wbase;
  // the window is reused tile after tile: the wave's reads of the previous tile complete first
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int k = 0; k < WIN_LOADS; k++) {
    const int c = k * 64 + lane;
    if (c < nch)
      __builtin_amdgcn_global_load_lds((const GLB void*)(g + (size_t)c * 16), (LDS void*)(win + k * 256), 16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// One record: FastRead (emit) or its length / var extents only (measure).
template <int NV, int MODE>
__device__ __forceinline__ int parse_record(KParams& dp, const Src& w, uint64_t pos, uint64_t lim, uint64_t r,
                                            bool emit, uint64_t* end, VarState<NV>& vs, uint64_t& pres) {
#pragma unroll
  for (int v = 0; v < NV; v++) { vs.len[v] = 0; vs.pos[v] = 0; }
  pres = 0;
  if (MODE == M_THRIFT) {
    if (w.nsteps && canon_record<NV>(w, dp.cols, pos, lim, r, emit, end, vs)) {
      pres = w.canon_pres;
      return KX_OK;
    }
    return generic_record<NV>(w, dp.prog, dp.cols, pos, lim, r, emit, end, vs, pres);
  }
  if (MODE == M_PB) {
    uint64_t b = pos, e = lim;
    if (!dp.offsets) {  // Batch framing: 0x0A, uvarint(len), body
      if (pos >= lim) return KX_ERR_EOF;
      if (ld1(w, pos) != 0x0Au) return KX_ERR_INVALID_DATA;
      uint64_t l;
      uint32_t u;
      const int rc = pb_varint(w, pos + 1, lim - pos - 1, l, u);
      if (rc) return rc;
      if (l > lim - pos - 1 - u) return KX_ERR_EOF;
      b = pos + 1 + u;
      e = b + l;
    }
    *end = e;
    // concatenated mode: the index pass already validated every record the chain reaches, so the
    // emit pass skips the UTF-8 check; with known extents the emit pass is the validator
    return pb_body<NV>(w, dp.prog, dp.cols, b, e, r, emit, vs, pres, !emit || dp.offsets != nullptr);
  }
  uint64_t p2 = pos;
  const int rc = dskip_body(w, p2, lim, KX_T_STRUCT, 64);
  *end = p2;
  return rc;
}

// ---------------------------------------------------------------------------------------------
// output offsets: 4 or 8 bytes per entry (kx_column.offset_bytes); a 4-byte column never wraps
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void put_off(KParams& dp, uint32_t c, uint64_t r, uint64_t v) {
  if (r > dp.n || c >= KX_MAX_COLUMNS) { atomicOr(dp.cols.guard, (unsigned long long)G_OFFSET); return; }
  if ((dp.cols.owide >> c) & 1) ((GLB uint64_t*)dp.cols.offs[c])[r] = v;
  else ((GLB uint32_t*)dp.cols.offs[c])[r] = (uint32_t)v;
}
// arena limit of column c in arena units: its capacity, and the 4-byte offset range
__device__ __forceinline__ uint64_t arena_lim(KParams& dp, uint32_t c) {
  const uint64_t cap = dp.cols.cap[c];
  return ((dp.cols.owide >> c) & 1) ? cap : min(cap, 0xffffffffull);
}
// offsets[i] = v for a record that ends the decoded prefix (n, or the failing record)
__device__ __forceinline__ void put_total(KParams& dp, uint32_t c, uint64_t i, uint64_t v) {
  if (v <= arena_lim(dp, c)) put_off(dp, c, i, v);
  else atomicOr(dp.overflow, 1u);
}

// ---------------------------------------------------------------------------------------------
// aggregates: lane / tile / super-tile
// ---------------------------------------------------------------------------------------------
constexpr uint32_t NOREL = 0xffffu;  // no tile-relative position

// A lane's walk, kept in LDS between the walk and the emit (so nothing of it stays live in
// registers across the super-tile's chaining and look-back). Positions are tile-relative, counts
// per lane / tile fit 16 bits; arena prefixes are kept modulo 2^32 (exact unless the tile's own
// records carry >= 4 GiB of payload, which the tile flags and the emit then recomputes).
template <int NV>
struct LaneS {
  uint16_t cand;            // first record signature in the lane's segment, or NOREL
  uint16_t ent;             // where the lane's records start, or NOREL
  uint16_t cnt;             // records the lane emits (0 unless live)
  uint16_t cpre;            // records of the live lanes below it
  uint32_t vpre[NV > 0 ? NV : 1];  // arena units of the live lanes below it (mod 2^32), per var slot
};

struct TAgg {               // a tile's chain: entry, exit (X_ERR: ends in an error), records, arena units
  uint64_t ent, ex, cnt, errc, errp;
  uint64_t var[KXP_NV_MAX];
  uint32_t wide;            // a var slot's total reaches 2^32: the emit recomputes the lane prefixes
  uint32_t pad;
};

// A composite of consecutive super-tiles, or an inclusive prefix (kind 2, S unused).
// kind 0: nothing; 1: no record start anywhere (the chain must pass over it: entry >= maxhi);
// 2: records from entry S to exit X (X_ERR: the chain ends in error ec at byte ep, after C records).
template <int NV>
struct Comp {
  uint32_t kind, ec;
  uint64_t S, X, C, ep, maxhi;
  uint64_t V[NV > 0 ? NV : 1];
};

// L then H (H covers the input right after L). False when the speculative entries disagree.
template <int NV>
__device__ __forceinline__ bool combine(const Comp<NV> L, const Comp<NV> H, Comp<NV>& out) {  // by value: out may alias
  if (L.kind == 0) { out = H; return true; }
  if (H.kind == 0 || (L.kind == 2 && L.X == X_ERR)) { out = L; return true; }
  if (H.kind == 1) {
    if (L.kind == 1) { out = L; out.maxhi = max(L.maxhi, H.maxhi); return true; }
    if (L.X >= H.maxhi) { out = L; return true; }
    return false;
  }
  if (L.kind == 1) { out = H; return true; }  // H.S lies past everything L covers
  if (L.X != H.S) return false;
  out = L;
  out.X = H.X;
  out.C = L.C + H.C;
  out.ec = H.ec;
  out.ep = H.ep;
#pragma unroll
  for (int v = 0; v < NV; v++) out.V[v] = L.V[v] + H.V[v];
  return true;
}

// ---------------------------------------------------------------------------------------------
// concatenated mode: candidates, lane walks, the tile walk with in-wave repair
// ---------------------------------------------------------------------------------------------
// The record signature is the first 3 bytes of a record. The schema's canonical one (the encoder's
// first field header) is used when the batch's first record starts with it; otherwise (an
// IDL-order producer, an unset optional first field, the schema-less skip decoder) the first
// record's own first 3 bytes are: records of one batch normally start alike.
__device__ __forceinline__ uint32_t data_sig(KParams& dp) {
  if (dp.in_len < 3) return 0;
  const GLB uint8_t* p = (const GLB uint8_t*)dp.in;
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
}

#define P_SIG(P, MODE) ((MODE) == M_THRIFT ? (P)->sig : ~0u)

// does the record at c parse, and is it followed by the signature again (or the end of the input)?
template <int NV, int MODE>
__device__ __forceinline__ bool succ_ok(KParams& dp, const Src& w, uint64_t c, uint32_t sig) {
  VarState<NV> vs;
  uint64_t e = c, pres;
  if (parse_record<NV, MODE>(dp, w, c, dp.in_len, 0, false, &e, vs, pres)) return false;
  return e == dp.in_len || (dp.in_len - e >= 3 && (ld4(w, e) & 0xffffffu) == sig);
}

// first plausible record start in the lane's segment [seg_lo, seg_hi) (speculation only)
template <int NV, int MODE>
__device__ __forceinline__ uint64_t lane_candidate(KParams& dp, const Src& w, uint64_t seg_lo, uint64_t seg_hi,
                                                   uint32_t dsig, int lane) {
  if (seg_lo >= seg_hi) return X_NONE;
  if (MODE == M_PB) return pb_scan_segment(w, seg_lo, seg_hi, dp.in_len, lane);
  const KAS KxProgram* P = dp.prog;
  const bool dok = dsig != 0 && canon_t(dsig & 0xff) != 1;  // the first record starts with a field header
  uint32_t sig, slen;
  bool ambig = false;
  if (MODE == M_THRIFT && P->sig_len == 3 && (!dok || dsig == P->sig)) {
    sig = P->sig; slen = 3; ambig = P->sig_ambig && w.nsteps;
  } else if (dok) {
    sig = dsig; slen = 3;
  } else if (MODE == M_THRIFT) {
    sig = P->sig; slen = P->sig_len;
  } else {
    sig = KX_T_STOP; slen = 1;
  }
  const uint64_t plim = min(seg_hi, dp.in_len >= slen ? dp.in_len - slen + 1 : 0ull);
  const int32_t q0 = wofs(w, seg_lo, SEG + 12);
  uint64_t ent = X_NONE;
  if (slen == 3 && seg_hi - seg_lo == SEG && q0 >= 0 && MODE == M_THRIFT && ambig) {
    // the signature also starts a nested struct: keep the lowest of the two lowest hits that parses
    // as a canonical record (a nested-struct start does not), else no candidate
    uint32_t c1, c2;
    scan_segment2(w, q0, sig, lane, c1, c2);
    VarState<NV> vs0;
    uint64_t e0;
    if (c1 < (uint32_t)SEG && seg_lo + c1 < plim &&
        canon_record<NV>(w, dp.cols, seg_lo + c1, dp.in_len, 0, false, &e0, vs0))
      ent = seg_lo + c1;
    else if (c2 < (uint32_t)SEG && seg_lo + c2 < plim &&
             canon_record<NV>(w, dp.cols, seg_lo + c2, dp.in_len, 0, false, &e0, vs0))
      ent = seg_lo + c2;
  } else if (slen == 3 && seg_hi - seg_lo == SEG && q0 >= 0 && sig != P_SIG(P, MODE)) {
    // a signature taken from the data may also start nested structs: keep the lowest of the two
    // lowest hits whose record is followed by the signature again (or ends the input)
    uint32_t c1, c2;
    scan_segment2(w, q0, sig, lane, c1, c2);
    if (c1 < (uint32_t)SEG && seg_lo + c1 < plim && succ_ok<NV, MODE>(dp, w, seg_lo + c1, sig)) ent = seg_lo + c1;
    else if (c2 < (uint32_t)SEG && seg_lo + c2 < plim && succ_ok<NV, MODE>(dp, w, seg_lo + c2, sig)) ent = seg_lo + c2;
  } else if (slen == 3 && seg_hi - seg_lo == SEG && q0 >= 0) {
    ent = scan_segment(w, q0, seg_lo, plim, sig, lane);
  } else {
    const uint32_t smask = slen == 3 ? 0xffffffu : 0xffu;
    for (uint64_t p = seg_lo; p < plim; p++)
      if ((ld4(w, p) & smask) == sig) { ent = p; break; }
  }
  return ent;
}

// walk records from `ent` until the lane's segment is left (measure only); on a decode error ex =
// X_ERR and errp = the failing record's start
template <int NV, int MODE>
__device__ __forceinline__ void walk_lane(KParams& dp, const Src& w, uint64_t ent, uint64_t seg_hi, uint64_t& ex,
                                          uint64_t& cnt, uint32_t& errc, uint64_t& errp, uint64_t* vsum) {
  uint64_t pos = ent, c = 0;
  int e = 0;
#pragma unroll
  for (int v = 0; v < NV; v++) vsum[v] = 0;
  while (pos < seg_hi && pos < dp.in_len) {
    VarState<NV> vs;
    uint64_t end = pos, pres;
    const int rc = parse_record<NV, MODE>(dp, w, pos, dp.in_len, 0, false, &end, vs, pres);
    if (rc) { e = rc; break; }
    c++;
#pragma unroll
    for (int v = 0; v < NV; v++) vsum[v] += vs.len[v];
    pos = end;
  }
  ex = e ? X_ERR : pos;
  cnt = c;
  errc = (uint32_t)e;
  errp = pos;
}

// One wave, tile [tlo, thi) in the LDS window. Every lane starts at its candidate (ls[lane].cand) or
// where the chain of the nearest lower walking lane (or `seed`, the tile's true entry when known)
// enters its segment, and walks until it leaves it; lanes re-walk until the chain is consistent.
// While speculating (seed unknown) a candidate whose own walk fails is dropped, so a false signature
// hit does not end the tile's chain. Returns the tile aggregate (uniform) and leaves every lane's
// emit state (entry, records, prefixes among the live lanes) in ls[lane].
template <int NV, int MODE>
__device__ __forceinline__ TAgg walk_tile(KParams& dp, const Src& w, uint64_t tlo, uint64_t thi, uint64_t seed,
                                          int lane, LDS LaneS<NV>* ls) {
  const uint64_t seg_lo = tlo + (uint64_t)lane * SEG;
  const uint64_t seg_hi = min(seg_lo + SEG, thi);
  const uint32_t c0 = ls[lane].cand;  // (NOREL: none)
  uint64_t ent = c0 == NOREL ? X_NONE : tlo + c0;
  uint64_t ex = X_NONE, cnt = 0, errp = 0;
  uint32_t errc = 0;
  uint64_t vsum[NV > 0 ? NV : 1];
#pragma unroll
  for (int v = 0; v < (NV > 0 ? NV : 1); v++) vsum[v] = 0;
  bool need = ent != X_NONE;
  int rounds = 0;
  bool first = true;
  uint64_t hm;
  for (;;) {
    if (need) walk_lane<NV, MODE>(dp, w, ent, seg_hi, ex, cnt, errc, errp, vsum);
    need = false;
    if (first && seed == X_NONE && ent != X_NONE && ex == X_ERR) {
      ent = X_NONE; ex = X_NONE; cnt = 0; errc = 0;
#pragma unroll
      for (int v = 0; v < NV; v++) vsum[v] = 0;
    }
    first = false;
    hm = __ballot(ent != X_NONE);
    const uint64_t below = hm & ((1ull << lane) - 1);
    const int pc = below ? 63 - __clzll((long long)below) : -1;
    const uint64_t pex = __shfl(ex, pc < 0 ? 0 : pc, 64);
    const uint64_t pe = pc >= 0 ? pex : seed;
    uint64_t want = ent;
    if (pe != X_NONE) {
      if (pe == X_ERR || seg_lo >= thi || pe >= seg_hi) want = X_NONE;
      else if (pe >= seg_lo) want = pe;
    }
    const bool ch = want != ent;
    if (!__ballot(ch)) break;
    if (++rounds > 70) {  // from a fixed lowest entry the chain settles in <= 65 rounds
      if (lane == 0) {
        atomicCAS((int*)&dp.status->code, 0, KX_ERR_INTERNAL);
        atomicOr((unsigned long long*)&dp.status->diag[2], (unsigned long long)G_ROUNDS);
      }
      break;
    }
    if (ch) {
      ent = want;
      need = want != X_NONE;
      ex = X_NONE; cnt = 0; errc = 0;
#pragma unroll
      for (int v = 0; v < NV; v++) vsum[v] = 0;
    }
  }
  const uint64_t em = __ballot(ent != X_NONE && ex == X_ERR);
  const int fel = em ? __ffsll((long long)em) - 1 : 64;
  const bool live = ent != X_NONE && lane <= fel;
  TAgg a;
  a.wide = 0;
  const uint64_t lc = live ? cnt : 0;
  const uint64_t ci = wave_incl_scan(lc, lane);
  a.cnt = rl64(ci, 63);
  ls[lane].ent = live ? (uint16_t)(ent - tlo) : (uint16_t)NOREL;
  ls[lane].cnt = (uint16_t)lc;
  ls[lane].cpre = (uint16_t)(ci - lc);
#pragma unroll
  for (int v = 0; v < NV; v++) {
    const uint64_t x0 = live ? vsum[v] : 0;
    const uint64_t xi = wave_incl_scan(x0, lane);
    ls[lane].vpre[v] = (uint32_t)(xi - x0);
    a.var[v] = rl64(xi, 63);
    a.wide |= a.var[v] >> 32 ? 1u : 0u;
  }
  a.ent = hm ? rl64(ent, __ffsll((long long)hm) - 1) : X_NONE;
  a.ex = fel < 64 ? X_ERR : hm ? rl64(ex, 63 - __clzll((long long)hm)) : seed;
  a.errc = fel < 64 ? (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)errc, fel) : 0;
  a.errp = fel < 64 ? rl64(errp, fel) : 0;
  return a;
}

// Known-offsets mode: lane = record. Measures the var extents (failed records count as empty).
template <int NV, int MODE>
__device__ __forceinline__ TAgg measure_records(KParams& dp, const Src& w, uint64_t r0, uint64_t r1, int lane) {
  const uint64_t r = r0 + lane;
  VarState<NV> vs;
#pragma unroll
  for (int v = 0; v < NV; v++) vs.len[v] = 0;
  if (r < r1) {
    const uint64_t a = dp.offsets[r], b = dp.offsets[r + 1];
    uint64_t end, pres;
    int rc = (a > b || b > dp.in_len) ? KX_ERR_INVALID_ARG : parse_record<NV, MODE>(dp, w, a, b, r, false, &end, vs, pres);
    if (rc) {
#pragma unroll
      for (int v = 0; v < NV; v++) vs.len[v] = 0;
    }
  }
  TAgg g;
  g.ent = 0; g.ex = 0; g.errc = 0; g.errp = 0; g.wide = 0;
  g.cnt = r1 - r0;
#pragma unroll
  for (int v = 0; v < NV; v++) g.var[v] = wave_sum(vs.len[v]);
  return g;
}

// tile geometry: bytes (concatenated) or records (known offsets)
__device__ __forceinline__ void tile_range(KParams& dp, uint64_t t, uint64_t& lo, uint64_t& hi) {
  if (dp.offsets) {
    lo = t * dp.krec;
    hi = min(lo + dp.krec, dp.n);
  } else {
    lo = t * (uint64_t)TILE;
    hi = min(lo + TILE, dp.in_len);
  }
}
__device__ __forceinline__ uint64_t st_hi(KParams& dp, uint64_t s) {
  return min((s + 1) * (uint64_t)WGW * TILE, dp.in_len);
}
// the input position of a tile's window
__device__ __forceinline__ uint64_t tile_pos(KParams& dp, uint64_t lo) { return dp.offsets ? dp.offsets[lo] : lo; }

// ---------------------------------------------------------------------------------------------
// super-tile: chaining the tiles of one workgroup (LDS), publishing, decoupled look-back
// ---------------------------------------------------------------------------------------------
// super-tile state machine (decode_kernel, st_step)
enum { ST_SPEC = 0, ST_LB = 1, ST_TRUE = 2, ST_DONE = 3 };

template <int NV>
struct StShared {
  TAgg ta[WGW];               // tile aggregates
  uint64_t tbc[WGW];          // records of the ST's chain before tile k
  uint64_t tbv[WGW][KXP_NV_MAX];
  int on[WGW];                // tile k is on the chain
  int fix;                    // tile to re-walk (-1: none)
  int state;                  // ST_* (decode_kernel)
  int nfix;                   // re-walks of this super-tile so far
  uint64_t fixE;              // ... from this entry
  uint64_t tk, tkn[2];        // first ticket; the next one (prefetched; by iteration parity)
  Comp<NV> agg, fin, pre;     // speculative / true ST aggregate, prefix before the ST
};

// Chains the tile aggregates of super-tile s from entry Ein (X_NONE = speculative: the first tile
// with a record start is trusted). Returns the first tile that disagrees with the chain (to be
// re-walked from *fixE), or -1 with the ST aggregate in `out` and each tile's base / membership.
template <int NV>
__device__ __forceinline__ int st_fold(KParams& dp, StShared<NV>* sh, uint64_t s, uint64_t Ein, Comp<NV>& out,
                                       uint64_t* fixE) {
  Comp<NV> cur;
  cur.kind = Ein == X_NONE ? 0u : 2u;
  cur.S = Ein; cur.X = Ein; cur.C = 0; cur.ec = 0; cur.ep = 0; cur.maxhi = 0;
#pragma unroll
  for (int v = 0; v < (NV > 0 ? NV : 1); v++) cur.V[v] = 0;
  const bool known = dp.offsets != nullptr;
  for (int k = 0; k < WGW; k++) {
    const uint64_t t = s * WGW + k;
    sh->tbc[k] = cur.C;
#pragma unroll
    for (int v = 0; v < NV; v++) sh->tbv[k][v] = cur.V[v];
    sh->on[k] = 0;
    if (t >= dp.ntiles) continue;
    const TAgg& a = sh->ta[k];
    if (!known) {
      uint64_t lo, hi;
      tile_range(dp, t, lo, hi);
      if (cur.kind == 2 && cur.X == X_ERR) continue;
      if (cur.kind != 2) {
        if (a.ent == X_NONE) continue;
        cur.kind = 2;
        cur.S = a.ent;
      } else {
        if (cur.X >= hi) continue;  // the chain passes over this tile
        if (a.ent != cur.X) { *fixE = cur.X; return k; }
      }
      cur.X = a.ex;
      if (a.ex == X_ERR) { cur.ec = (uint32_t)a.errc; cur.ep = a.errp; }
    }
    sh->on[k] = 1;
    cur.C += a.cnt;
#pragma unroll
    for (int v = 0; v < NV; v++) cur.V[v] += a.var[v];
  }
  if (cur.kind != 2) {
    cur.kind = 1;
    cur.S = cur.X = X_NONE;
    cur.maxhi = st_hi(dp, s);
  }
  out = cur;
  return -1;
}

__device__ __forceinline__ uint64_t sword(KParams& dp, int f, uint64_t j) {
  if (j >= dp.nst) { atomicOr(dp.cols.guard, (unsigned long long)G_WORD); return 0; }
  return aload64(dp.sdesc + (uint64_t)f * dp.nst + j);
}

template <int NV>
__device__ __forceinline__ void publish(KParams& dp, uint64_t s, const Comp<NV>& c, bool inclusive) {
  const uint64_t ep = dp.epoch, ns = dp.nst;
  if (s >= ns) { atomicOr(dp.cols.guard, (unsigned long long)G_WORD); return; }
  if (inclusive) {
    put_word(dp.sdesc, ns, P_C, s, ep, c.C);
    put_word(dp.sdesc, ns, P_EC, s, ep, c.ec);
    put_word(dp.sdesc, ns, P_EP, s, ep, c.ep);
#pragma unroll
    for (int v = 0; v < NV; v++) put_word(dp.sdesc, ns, P_V + v, s, ep, c.V[v]);
    put_word(dp.sdesc, ns, P_X, s, ep, c.X);
  } else {
    const bool pass = c.kind != 2;
    put_word(dp.sdesc, ns, A_X, s, ep, pass ? X_NONE : c.X);
    put_word(dp.sdesc, ns, A_C, s, ep, c.C);
    put_word(dp.sdesc, ns, A_EC, s, ep, c.ec);
    put_word(dp.sdesc, ns, A_EP, s, ep, c.ep);
#pragma unroll
    for (int v = 0; v < NV; v++) put_word(dp.sdesc, ns, A_V + v, s, ep, c.V[v]);
    put_word(dp.sdesc, ns, A_S, s, ep, pass ? X_NONE : c.S);
  }
}

// the A (speculative) or P (inclusive) words of super-tile j; false unless all carry this epoch
template <int NV>
__device__ __forceinline__ bool load_st(KParams& dp, uint64_t j, bool inclusive, Comp<NV>& c) {
  const uint64_t ep = dp.epoch;
  bool ok = true;
  uint64_t x;
  if (inclusive) {
    x = sword(dp, P_X, j); ok &= (x >> 48) == ep; c.X = x & V48;
    x = sword(dp, P_C, j); ok &= (x >> 48) == ep; c.C = x & V48;
    x = sword(dp, P_EC, j); ok &= (x >> 48) == ep; c.ec = (uint32_t)(x & V48);
    x = sword(dp, P_EP, j); ok &= (x >> 48) == ep; c.ep = x & V48;
#pragma unroll
    for (int v = 0; v < NV; v++) { x = sword(dp, P_V + v, j); ok &= (x >> 48) == ep; c.V[v] = x & V48; }
    c.kind = 2;
    c.S = 0;
  } else {
    x = sword(dp, A_S, j); ok &= (x >> 48) == ep; c.S = x & V48;
    x = sword(dp, A_X, j); ok &= (x >> 48) == ep; c.X = x & V48;
    x = sword(dp, A_C, j); ok &= (x >> 48) == ep; c.C = x & V48;
    x = sword(dp, A_EC, j); ok &= (x >> 48) == ep; c.ec = (uint32_t)(x & V48);
    x = sword(dp, A_EP, j); ok &= (x >> 48) == ep; c.ep = x & V48;
#pragma unroll
    for (int v = 0; v < NV; v++) { x = sword(dp, A_V + v, j); ok &= (x >> 48) == ep; c.V[v] = x & V48; }
    c.kind = c.S == X_NONE ? 1u : 2u;
  }
  c.maxhi = dp.offsets ? 0 : st_hi(dp, j);
  return ok;
}

// Watchdog of the look-back waits: a wait gives up (the call fails with KX_ERR_INTERNAL, the returned
// prefix ends the chain) only when no super-tile anywhere has published its prefix for 2 s (a long
// but moving serial chain is not a hang), or when another wait already gave up.
__device__ __forceinline__ bool wait_expired(KParams& dp, uint64_t& t0, uint64_t& prog) {
  if (__hip_atomic_load(dp.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return true;
  const uint64_t p = aload64((const uint64_t*)dp.progress);
  const uint64_t now = now_ns();
  if (p != prog) { prog = p; t0 = now; return false; }
  if (now - t0 <= 2000000000ull) return false;
  __hip_atomic_store(dp.abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

template <int NV>
__device__ __forceinline__ Comp<NV> bcast(const Comp<NV>& c, int l) {
  Comp<NV> r;
  r.kind = (uint32_t)__builtin_amdgcn_readlane((int)c.kind, l);
  r.ec = (uint32_t)__builtin_amdgcn_readlane((int)c.ec, l);
  r.S = rl64(c.S, l); r.X = rl64(c.X, l); r.C = rl64(c.C, l); r.ep = rl64(c.ep, l); r.maxhi = rl64(c.maxhi, l);
#pragma unroll
  for (int v = 0; v < NV; v++) r.V[v] = rl64(c.V[v], l);
  return r;
}

template <int NV>
__device__ __forceinline__ Comp<NV> failed_prefix(KParams& dp, int lane, uint64_t why) {
  if (lane == 0) {
    atomicCAS((int*)&dp.status->code, 0, KX_ERR_INTERNAL);
    atomicOr((unsigned long long*)&dp.status->diag[2], why);
  }
  Comp<NV> e;
  e.kind = 2; e.ec = KX_ERR_INTERNAL; e.S = 0; e.X = X_ERR; e.C = 0; e.ep = 0; e.maxhi = 0;
#pragma unroll
  for (int v = 0; v < (NV > 0 ? NV : 1); v++) e.V[v] = 0;
  return e;
}

// Decoupled look-back (one wave): the inclusive prefix of the chain before super-tile s. Lane l
// reads super-tile jhi - l (its inclusive prefix P when published, else its speculative aggregate A);
// the window's A are combined up to the nearest P, every boundary checked for chain consistency. If
// the speculation disagrees anywhere, the predecessor's own P is awaited (it re-walks itself from
// its true entry).
template <int NV>
__device__ __forceinline__ Comp<NV> lookback(KParams& dp, uint64_t s, int lane) {
  Comp<NV> base0;
  base0.kind = 2; base0.ec = 0; base0.S = 0; base0.X = 0; base0.C = 0; base0.ep = 0; base0.maxhi = 0;
#pragma unroll
  for (int v = 0; v < (NV > 0 ? NV : 1); v++) base0.V[v] = 0;
  if (s == 0) return base0;
  Comp<NV> acc;
  acc.kind = 0;
  uint64_t jhi = s - 1;
  int wsz = 16;
  uint64_t t0 = now_ns(), prog = ~0ull;
  int backoff = 1;
  bool ok = true;
  for (;;) {
    const bool inwin = lane < wsz;
    const bool v = inwin && jhi >= (uint64_t)lane;
    Comp<NV> c;
    bool hp = false, ha = false;
    if (v) {
      hp = load_st<NV>(dp, jhi - lane, true, c);
      if (!hp) ha = load_st<NV>(dp, jhi - lane, false, c);
    }
    const uint64_t pm = __ballot(hp || (inwin && !v));
    const int p = pm ? __ffsll((long long)pm) - 1 : wsz;
    const uint64_t need = p >= 64 ? ~0ull : ((1ull << p) - 1);
    if ((__ballot(ha) & need) != need) {
      if (__ballot(wait_expired(dp, t0, prog))) return failed_prefix<NV>(dp, lane, G_LB_WAIT);
      for (int k = 0; k < backoff; k++) __builtin_amdgcn_s_sleep(1);
      backoff = backoff < 32 ? backoff * 2 : 32;
      continue;
    }
    Comp<NV> wc;
    wc.kind = 0;
    for (int k = p - 1; k >= 0 && ok; k--) ok = combine(wc, bcast(c, k), wc);
    if (ok) ok = combine(wc, acc, acc);
    if (!ok) break;
    if (p < wsz || jhi < (uint64_t)wsz) {  // a published prefix, or the window reached super-tile 0
      const Comp<NV> base = p < wsz && jhi >= (uint64_t)p ? bcast(c, p) : base0;
      Comp<NV> r;
      if (combine(base, acc, r) && r.kind == 2) return r;
      break;
    }
    jhi -= (uint64_t)wsz;
    wsz = 64;
  }
  if (lane == 0) atomicAdd((unsigned long long*)&dp.status->diag[1], 1ull);
  // the speculation disagrees below s: the predecessor resolves itself; take its inclusive prefix
  backoff = 1;
  for (;;) {
    Comp<NV> P;
    const bool hp = load_st<NV>(dp, s - 1, true, P);
    if (__ballot(hp) & 1ull) return bcast(P, 0);
    if (__ballot(wait_expired(dp, t0, prog))) return failed_prefix<NV>(dp, lane, G_LB_SLOW);
    for (int k = 0; k < backoff; k++) __builtin_amdgcn_s_sleep(1);
    backoff = backoff < 32 ? backoff * 2 : 32;
  }
}

// ---------------------------------------------------------------------------------------------
// emit
// ---------------------------------------------------------------------------------------------
// the var payloads of record r at the running arena positions
template <int NV>
__device__ __forceinline__ void emit_vars(KParams& dp, const Src& w, const VarState<NV>& vs, uint64_t r, uint64_t* run) {
  const KAS KxProgram* P = dp.prog;
#pragma unroll
  for (int v = 0; v < NV; v++) {
    if (v >= (int)P->nvar) break;
    const uint32_t c = P->var_col[v];
    const uint32_t nn = vs.len[v];
    const uint64_t at = run[v];
    if (at + nn <= arena_lim(dp, c)) {
      put_off(dp, c, r, at);
      if (nn) {
        const KxpCol K = ld_col(P, c);
        copy_var(w, K, vs.pos[v], nn, (uint8_t*)dp.cols.data[c] + at * K.width);
      }
    } else {
      atomicOr(dp.overflow, 1u);
    }
    run[v] = at + nn;
  }
}

// record n-1 was decoded: the call's final status
template <int NV, int MODE>
__device__ __forceinline__ void finish_ok(KParams& dp, uint64_t consumed, const uint64_t* run) {
  const KAS KxProgram* P = dp.prog;
  kx_status* st = dp.status;
  st->n_records = dp.n;
  st->consumed = consumed;
  if (MODE == M_SKIP) dp.skip_out[dp.n] = consumed;
#pragma unroll
  for (int v = 0; v < NV; v++) {
    if (v >= (int)P->nvar) break;
    st->var_total[v] = run[v];
    put_total(dp, P->var_col[v], dp.n, run[v]);
  }
}

// concatenated mode, lane = segment: every live lane re-walks its records from its entry, emitting
template <int NV, int MODE>
__device__ __forceinline__ void emit_concat(KParams& dp, const Src& w, uint64_t tlo, uint64_t thi,
                                            const LDS LaneS<NV>* ls, bool wide, uint64_t rbase,
                                            const uint64_t* vbase, int lane) {
  const uint32_t e0 = ls[lane].ent, cnt = ls[lane].cnt;
  uint64_t run[NV > 0 ? NV : 1];
  if (wide) {  // >= 4 GiB of payload in this tile: re-measure the lanes for exact 64-bit prefixes
    uint64_t ex, c, ep, vsum[NV > 0 ? NV : 1];
    uint32_t ec;
#pragma unroll
    for (int v = 0; v < (NV > 0 ? NV : 1); v++) vsum[v] = 0;
    const uint64_t seg_hi = min(tlo + (uint64_t)lane * SEG + SEG, thi);
    if (e0 != NOREL && cnt) walk_lane<NV, MODE>(dp, w, tlo + e0, seg_hi, ex, c, ec, ep, vsum);
#pragma unroll
    for (int v = 0; v < NV; v++) {
      const uint64_t x0 = (e0 != NOREL && cnt) ? vsum[v] : 0;
      run[v] = vbase[v] + wave_incl_scan(x0, lane) - x0;
    }
  } else {
#pragma unroll
    for (int v = 0; v < NV; v++) run[v] = vbase[v] + ls[lane].vpre[v];
  }
  if (e0 == NOREL || cnt == 0) return;
  uint64_t r = rbase + ls[lane].cpre;
  uint64_t pos = tlo + e0;
  for (uint32_t j = 0; j < cnt && r < dp.n; j++, r++) {
    VarState<NV> vs;
    uint64_t end = pos, pres = 0;
    (void)parse_record<NV, MODE>(dp, w, pos, dp.in_len, r, MODE != M_SKIP, &end, vs, pres);
    if (r >= dp.n) { atomicOr(dp.cols.guard, (unsigned long long)G_ROWS); break; }
    if (MODE == M_SKIP) dp.skip_out[r] = pos;
    else if (dp.cols.presence) dp.cols.presence[r] = pres;
    emit_vars<NV>(dp, w, vs, r, run);
    if (r == dp.n - 1) finish_ok<NV, MODE>(dp, end, run);
    pos = end;
  }
}

// known-offsets mode, lane = record (<= 64 per tile)
template <int NV, int MODE>
__device__ __forceinline__ void emit_offsets(KParams& dp, const Src& w, uint64_t r0, uint64_t r1, const uint64_t* vbase,
                                             int lane) {
  const uint64_t r = r0 + lane;
  const bool act = r < r1;
  VarState<NV> vs;
#pragma unroll
  for (int v = 0; v < NV; v++) { vs.len[v] = 0; vs.pos[v] = 0; }
  if (act) {
    const uint64_t pos = dp.offsets[r], lim = dp.offsets[r + 1];
    uint64_t end = 0, pres = 0;
    int rc = (pos > lim || lim > dp.in_len) ? KX_ERR_INVALID_ARG : KX_OK;
    if (!rc) rc = parse_record<NV, MODE>(dp, w, pos, lim, r, MODE != M_SKIP, &end, vs, pres);
    if (rc) {  // the failed record reads as all defaults, empty payloads
#pragma unroll
      for (int v = 0; v < NV; v++) vs.len[v] = 0;
      pres = 0;
      if (MODE != M_SKIP) emit_defaults(dp.prog, dp.cols, r);
      atomicMin(dp.errkey, (unsigned long long)((r << 8) | (uint64_t)(rc & 0xff)));
    }
    if (dp.rstat) dp.rstat[r] = (uint8_t)rc;
    if (MODE == M_SKIP) dp.skip_out[r] = pos;
    else if (dp.cols.presence) dp.cols.presence[r] = pres;
  }
  uint64_t run[NV > 0 ? NV : 1];
#pragma unroll
  for (int v = 0; v < NV; v++) {
    const uint64_t x0 = act ? vs.len[v] : 0;
    run[v] = vbase[v] + wave_incl_scan(x0, lane) - x0;
  }
  if (act) {
    emit_vars<NV>(dp, w, vs, r, run);
    if (r == dp.n - 1) finish_ok<NV, MODE>(dp, dp.offsets[dp.n], run);
  }
}

// the chain ended in super-tile s before record n (decode error or input exhausted): final status
template <int NV, int MODE>
__device__ __forceinline__ void finish_short(KParams& dp, const Comp<NV>& fin, int code, uint64_t offset) {
  const KAS KxProgram* P = dp.prog;
  kx_status* st = dp.status;
  st->code = code;
  st->record = fin.C;
  st->offset = offset;
  st->n_records = fin.C;
  st->consumed = offset;
  if (fin.C > dp.n) { atomicOr(dp.cols.guard, (unsigned long long)G_ROWS); return; }
  if (MODE == M_SKIP) dp.skip_out[fin.C] = offset;
#pragma unroll
  for (int v = 0; v < NV; v++) {
    if (v >= (int)P->nvar) break;
    st->var_total[v] = fin.V[v];
    put_total(dp, P->var_col[v], fin.C, fin.V[v]);
  }
}

// One step of the super-tile state machine (thread 0; see decode_kernel). Sets sh->fix to the tile
// to re-walk from sh->fixE (or -1), advances sh->state.
template <int NV, int MODE>
__device__ __forceinline__ void st_step(KParams& dp, StShared<NV>* sh, uint64_t s) {
  const bool known = dp.offsets != nullptr;
  uint64_t fe = 0;
  int k;
  if (sh->fix >= 0 && ++sh->nfix > 4 * WGW) {  // each fold fixes one tile for good: cannot happen
    atomicCAS((int*)&dp.status->code, 0, KX_ERR_INTERNAL);
    atomicOr((unsigned long long*)&dp.status->diag[2], (unsigned long long)G_NFIX);
    sh->fix = -1;
    sh->state = ST_DONE;
    Comp<NV> e = sh->agg;
    e.kind = 2; e.X = X_ERR; e.ec = KX_ERR_INTERNAL;
    publish<NV>(dp, s, e, true);
    atomicAdd(dp.progress, 1ull);
    sh->pre = e;  // nothing is emitted
    return;
  }
  switch (sh->state) {
    case ST_SPEC:
      k = st_fold<NV>(dp, sh, s, (s == 0 || known) ? 0ull : X_NONE, sh->agg, &fe);
      sh->fix = k;
      sh->fixE = fe;
      if (k < 0) {
        publish<NV>(dp, s, sh->agg, false);
        sh->state = ST_LB;  // wave 0 looks back before the next step
      }
      return;
    case ST_LB: {
      const Comp<NV>& pre = sh->pre;
      // the speculative chain stands when it starts at the true entry (always, known offsets)
      if (known || s == 0 || pre.X == X_ERR || (sh->agg.kind == 2 && sh->agg.S == pre.X)) {
        sh->fin = sh->agg;
        break;
      }
      sh->state = ST_TRUE;
    }
    // fallthrough
    case ST_TRUE:
      k = st_fold<NV>(dp, sh, s, sh->pre.X, sh->fin, &fe);
      sh->fix = k;
      sh->fixE = fe;
      if (k >= 0) return;
      break;
    default:
      return;
  }
  // the ST's true chain is known: publish the inclusive prefix, settle the call's status
  sh->fix = -1;
  sh->state = ST_DONE;
  const Comp<NV> pre = sh->pre;
  Comp<NV> fin;
  if (!combine(pre, sh->fin, fin)) {  // cannot happen: sh->fin starts at pre.X
    atomicCAS((int*)&dp.status->code, 0, KX_ERR_INTERNAL);
    atomicOr((unsigned long long*)&dp.status->diag[2], (unsigned long long)G_COMBINE);
    fin = pre;
    fin.X = X_ERR;
    fin.ec = KX_ERR_INTERNAL;
  }
  publish<NV>(dp, s, fin, true);
  atomicAdd(dp.progress, 1ull);
  if (!known && pre.X != X_ERR && pre.C < dp.n) {
    if (fin.X == X_ERR && fin.C < dp.n) finish_short<NV, MODE>(dp, fin, (int)fin.ec, fin.ep);
    else if (s == dp.nst - 1 && fin.X != X_ERR && fin.C < dp.n) finish_short<NV, MODE>(dp, fin, KX_ERR_EOF, dp.in_len);
  }
}

// ---- the persistent decode kernel ----
// Super-tiles are claimed in order from one counter (the next claim is issued a whole super-tile
// ahead of its use), so a look-back only ever waits on super-tiles that running workgroups hold.
// Per super-tile, a small state machine run by thread 0 between workgroup barriers decides who
// walks next (every walk of a tile goes through one call site):
//   SPEC: chain the tiles speculatively, re-walking tiles that disagree inside the ST; publish A
//   LB:   wave 0 looks back for the true prefix; TRUE: re-chain from the true entry (re-walks out of
//   LDS where the speculation was wrong); publish P and the final status; then every wave emits.
// Without var columns in offsets mode nothing is chained: tiles are dealt round-robin, emit only.
// Everything is inlined: out-of-line calls from divergent code (lane 0 / a subset of lanes) lose
// inactive lanes' registers on this toolchain.
template <int NV, int MODE>
__global__ void __launch_bounds__(NT, 4) decode_kernel(DecParams dp_) {
  KParams& dp = KX_PARAMS();
  (void)dp_;
  __shared__ __attribute__((aligned(16))) uint32_t WIN[WGW][WINW];
  __shared__ LaneS<NV> LSA[WGW][64];
  __shared__ StShared<NV> SH;
  StShared<NV>* sh = &SH;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  LDS uint32_t* win = (LDS uint32_t*)WIN[wv];
  LDS LaneS<NV>* ls = (LDS LaneS<NV>*)LSA[wv];
  const bool known = dp.offsets != nullptr;
  const bool thrift = MODE == M_THRIFT;
  const uint32_t dsig = known ? 0u : data_sig(dp);
  if (threadIdx.x == 0) sh->tk = dp.direct ? blockIdx.x : atomicAdd(dp.ticket, 1ull);
  __syncthreads();
  uint32_t it = 0;
  for (uint64_t s = sh->tk; s < dp.nst; it ^= 1) {
    if (threadIdx.x == 0 && !dp.direct) sh->tkn[it] = atomicAdd(dp.ticket, 1ull);
    const uint64_t t = s * WGW + wv;
    const bool has = t < dp.ntiles;
    uint64_t lo = 0, hi = 0;
    if (has) {
      tile_range(dp, t, lo, hi);
      load_window(dp, win, tile_pos(dp, lo), lane);
      if (dp.direct) {
        uint64_t zero[NV > 0 ? NV : 1];
#pragma unroll
        for (int v = 0; v < (NV > 0 ? NV : 1); v++) zero[v] = 0;
        emit_offsets<NV, MODE>(dp, window_src(dp, win, tile_pos(dp, lo), thrift), lo, hi, zero, lane);
      } else if (!known) {
        const uint64_t seg_lo = lo + (uint64_t)lane * SEG;
        const uint64_t c = lane_candidate<NV, MODE>(dp, window_src(dp, win, lo, thrift), seg_lo,
                                                    min(seg_lo + SEG, hi), dsig, lane);
        ls[lane].cand = c == X_NONE ? (uint16_t)NOREL : (uint16_t)(c - lo);
      }
    }
    if (dp.direct) {
      s += gridDim.x;
      continue;
    }
    if (threadIdx.x == 0) { sh->state = ST_SPEC; sh->fix = -1; sh->nfix = 0; }
    bool walk = has;
    uint64_t seed = (t == 0 && !known) ? 0ull : X_NONE;
    for (;;) {
      if (walk) {
        const Src w = window_src(dp, win, tile_pos(dp, lo), thrift);
        const TAgg a = known ? measure_records<NV, MODE>(dp, w, lo, hi, lane)
                             : walk_tile<NV, MODE>(dp, w, lo, hi, seed, lane, ls);
        if (lane == 0) sh->ta[wv] = a;
      } else if (!has && lane == 0) {
        TAgg a;
        a.ent = X_NONE; a.ex = X_NONE; a.cnt = 0; a.errc = 0; a.errp = 0; a.wide = 0;
#pragma unroll
        for (int v = 0; v < KXP_NV_MAX; v++) a.var[v] = 0;
        sh->ta[wv] = a;
      }
      __syncthreads();
      if (wv == 0 && __shfl(sh->state, 0, 64) == ST_LB) {  // lane 0's read: it runs st_step next
        const Comp<NV> pre = lookback<NV>(dp, s, lane);
        if (lane == 0) sh->pre = pre;
      }
      if (threadIdx.x == 0) st_step<NV, MODE>(dp, sh, s);
      __syncthreads();
      const int k = sh->fix;
      if (sh->state == ST_DONE) break;
      walk = k == wv;
      if (walk) {
        seed = sh->fixE;
        if (lane == 0) atomicAdd((unsigned long long*)&dp.status->diag[0], 1ull);
      }
    }
    // emit this wave's tile
    if (has && sh->on[wv] && sh->pre.X != X_ERR) {
      const uint64_t rbase = sh->pre.C + sh->tbc[wv];
      uint64_t vbase[NV > 0 ? NV : 1];
#pragma unroll
      for (int v = 0; v < NV; v++) vbase[v] = sh->pre.V[v] + sh->tbv[wv][v];
      const Src w = window_src(dp, win, tile_pos(dp, lo), thrift);
      if (known) emit_offsets<NV, MODE>(dp, w, lo, hi, vbase, lane);
      else if (rbase < dp.n) emit_concat<NV, MODE>(dp, w, lo, hi, ls, sh->ta[wv].wide != 0, rbase, vbase, lane);
    }
    __syncthreads();
    s = sh->tkn[it];
  }
}

// Completes a call and re-arms the workspace for the next one (error key, overflow).
__global__ void finalize_kernel(kx_status* st, unsigned long long* errkey, uint32_t* overflow, uint32_t* abort,
                                unsigned long long* ticket, const uint64_t* offsets, uint64_t n) {
  unsigned long long* progress = ticket + 1;
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
  *abort = 0;
  *ticket = 0;
  *progress = 0;
}

// ---- workspace: [8] errkey u64, [16] overflow u32, [32] abort u32, [40] ticket u64, [48] progress
//      u64, then the super-tile words ----
constexpr size_t WS_HDR = 256;

struct WsLayout {
  uint64_t ntiles, nst;
  size_t sdesc, total;
};

uint32_t krec_for(uint64_t in_len, uint64_t n) {
  if (n == 0) return 64;
  const uint64_t avg = (in_len + n - 1) / n;
  const uint64_t k = avg ? (uint64_t)TILE / avg : 64;
  return (uint32_t)(k < 1 ? 1 : k > 64 ? 64 : k);
}

WsLayout ws_layout(uint64_t in_len, const uint64_t* offsets, uint64_t n) {
  WsLayout L{};
  if (offsets) {
    const uint64_t k = krec_for(in_len, n);
    L.ntiles = (n + k - 1) / k;
  } else {
    L.ntiles = (in_len + TILE - 1) / TILE;
  }
  if (!L.ntiles) L.ntiles = 1;
  L.nst = (L.ntiles + WGW - 1) / WGW;
  L.sdesc = WS_HDR;
  L.total = WS_HDR + (size_t)L.nst * S_NF * 8;
  return L;
}

// workgroups of this kernel that are resident at once on device `dev` (the persistent grid: every
// workgroup of it must be co-resident, since a super-tile's look-back waits on earlier ones)
template <int NV, int MODE>
unsigned resident_grid() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (!cache[dev]) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, decode_kernel<NV, MODE>, NT, 0) != hipSuccess ||
        per_cu < 1)
      per_cu = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 1;
    cache[dev] = per_cu * cus;
  }
  return (unsigned)cache[dev];
}

template <int NV, int MODE>
int launch_t(const DecParams& dp0, const WsLayout& L, void* ws, hipStream_t stream) {
  DecParams dp = dp0;
  char* base = (char*)ws;
  dp.errkey = (unsigned long long*)(base + 8);
  dp.overflow = (uint32_t*)(base + 16);
  dp.abort = (uint32_t*)(base + 32);
  dp.ticket = (unsigned long long*)(base + 40);
  dp.progress = (unsigned long long*)(base + 48);
  dp.sdesc = (uint64_t*)(base + L.sdesc);
  dp.ntiles = L.ntiles;
  dp.nst = L.nst;
  dp.direct = dp.offsets && NV == 0;
  KX_HIP_CHECK(hipMemsetAsync(dp.status, 0, sizeof(kx_status), stream));
  static int grid_cap = -1;  // diagnostics: KX_GRID caps the persistent grid
  if (grid_cap < 0) { const char* e = getenv("KX_GRID"); grid_cap = e ? atoi(e) : 0; }
  uint64_t g = min((uint64_t)resident_grid<NV, MODE>(), dp.nst);
  if (grid_cap > 0) g = min(g, (uint64_t)grid_cap);
  hipLaunchKernelGGL((decode_kernel<NV, MODE>), dim3((unsigned)g), dim3(NT), 0, stream, dp);
  KX_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(64), 0, stream, dp.status, dp.errkey, dp.overflow, dp.abort,
                     dp.ticket, dp.offsets, dp.n);
  KX_HIP_CHECK(hipGetLastError());
  return KX_OK;
}

template <int MODE>
int launch_nv(const DecParams& dp, const WsLayout& L, void* ws, hipStream_t stream, uint32_t nvar) {
  switch (nvar) {
    case 0: return launch_t<0, MODE>(dp, L, ws, stream);
    case 1: return launch_t<1, MODE>(dp, L, ws, stream);
    case 2: return launch_t<2, MODE>(dp, L, ws, stream);
    case 3: case 4: return launch_t<4, MODE>(dp, L, ws, stream);
    default: return launch_t<8, MODE>(dp, L, ws, stream);
  }
}

void fill_diag_flags(DecParams& dp) {
  static int nolds = -1;
  if (nolds < 0) { const char* e = getenv("KX_NOLDS"); nolds = e && e[0] == '1'; }
  dp.nolds = nolds;
  dp.diag = 0;
}

}  // namespace

size_t kx_decode_ws_bytes(const KxProgram& hprog, uint64_t in_len, const uint64_t* offsets, uint64_t n) {
  (void)hprog;
  return ws_layout(in_len, offsets, n).total;
}

size_t kx_skip_ws_bytes(uint64_t in_len) { return ws_layout(in_len, nullptr, 0).total; }

int kx_launch_decode(const KxProgram* dprog, const KxProgram& hprog, const uint8_t* in, uint64_t in_len,
                     const uint64_t* offsets, uint64_t n, const KxLaunchCols& cols, uint8_t* record_status,
                     kx_status* status, void* ws, size_t ws_size, uint64_t epoch, hipStream_t stream, bool pb) {
  DecParams dp{};
  fill_diag_flags(dp);
  dp.in = in; dp.in_len = in_len; dp.offsets = offsets; dp.n = n; dp.prog = (const KAS KxProgram*)dprog;
  dp.cols = cols; dp.rstat = record_status; dp.status = status; dp.epoch = epoch;
  dp.cols.nrec = n;
  dp.cols.guard = (unsigned long long*)&status->diag[2];
  dp.krec = krec_for(in_len, n);
  const WsLayout L = ws_layout(in_len, offsets, n);
  if (ws_size < L.total) return KX_ERR_INVALID_ARG;
  return pb ? launch_nv<M_PB>(dp, L, ws, stream, hprog.nvar) : launch_nv<M_THRIFT>(dp, L, ws, stream, hprog.nvar);
}

int kx_launch_skip(const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t* offsets_out, kx_status* status,
                   void* ws, size_t ws_size, uint64_t epoch, hipStream_t stream) {
  DecParams dp{};
  fill_diag_flags(dp);
  dp.in = in; dp.in_len = in_len; dp.offsets = nullptr; dp.n = n; dp.prog = nullptr;
  dp.status = status; dp.skip_out = offsets_out; dp.epoch = epoch;
  dp.cols.nrec = n;
  dp.cols.guard = (unsigned long long*)&status->diag[2];
  dp.krec = 64;
  const WsLayout L = ws_layout(in_len, nullptr, n);
  if (ws_size < L.total) return KX_ERR_INVALID_ARG;
  return launch_t<0, M_SKIP>(dp, L, ws, stream);
}
