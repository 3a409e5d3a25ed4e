// kx_decode.hip — batched Thrift-binary FastRead (and the skip decoder) on CDNA4 / gfx950.
//
// Reference semantics: generated FastRead (tool/internal_pkg/pluginmode/thriftgo/struct_tpl.go:41-149,
// 405-625; instance internal/mocks/thrift/k-mock.go:39-184) over N records, as fastUnmarshal does per
// message (pkg/remote/codec/thrift/codec_fast.go:60-82) or as the element loop of a list<Struct>;
// unknown / mistyped fields go through the skip decoder (codec_apache.go:191-293).
//
// Design: three stream-ordered kernels, no wave ever waits for another tile's work.
//   1. index pass — one WAVE per 8 KiB tile. The tile (+ a 512-byte halo for the record straddling
//      its end) is pulled into the wave's LDS window by LDS-DMA (global_load_lds_dwordx4). Lane l owns
//      the 128-byte segment l: it finds the first canonical record signature in it and walks records
//      (schema-aware FastRead lengths) until it leaves the segment; lanes repair each other with wave
//      shuffles until the chain is consistent. The tile writes its record starts (u16 list) and an
//      aggregate (speculative entry, exit, count, arena bytes, first error) as epoch-tagged words.
//      The last wave to finish a group of 64 tiles validates the chain between them (re-walking a
//      tile from its true entry where the speculation was wrong) and scans the group.
//   2. chain pass — one workgroup resolves the chain over the groups from offset 0 and writes every
//      group's record / arena base and the number of records to emit (errors, EOF, n).
//   3. emit pass — one wave per tile again (the tile is re-read, mostly from the Infinity Cache when
//      it fits), lane = record: fixed-width fields are stored as parsed (lanes = consecutive records,
//      coalesced), strings / lists are copied from LDS with 16-byte stores at scanned arena offsets.
//   Known-offsets mode (fastUnmarshal with dataLen): a tile is up to 64 records, lane = record; the
//   index pass only measures arena bytes (skipped entirely when the schema has no var columns).
// Canonical records (the encoder's layout) take a straight-line step plan compiled from the schema;
// anything else takes the generic field loop. Records or strings reaching past the LDS window are
// read from global memory (same code, other source).
// No MFMA anywhere: this is byte movement, bounded by HBM bandwidth and memory latency.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "kx_internal.h"
#include "kx_crc.h"
#include "kx_knobs.h"

#define LDS __attribute__((address_space(3)))
#define GLB __attribute__((address_space(1)))
#define KAS __attribute__((address_space(4)))  // kernarg segment (read in place, never copied to scratch)

namespace {

constexpr int NT = 256;                  // threads per workgroup (4 independent waves)
constexpr int WAVES = NT / 64;
#ifndef KX_SEG
#define KX_SEG 128
#endif
constexpr int SEG = KX_SEG;              // bytes per lane segment
constexpr int TILE = 64 * SEG;           // 8 KiB of input per wave
static_assert(TILE <= 65536, "record starts are uint16 offsets from the tile start");
constexpr int HALO = 512;                // default halo: the record straddling the tile end is read from LDS
constexpr int HALO_MAX = 1536;           // up to here (the halo grows with the batch's mean record size)
constexpr int WINB = TILE + HALO_MAX + 16;  // LDS window bytes allocated (+16 for the aligned-down start)
constexpr int WINW = WINB / 4 + 4;       // window dwords (+ pad for the last aligned read pair)
constexpr int GT = 64;                   // tiles per group (one group-scan lane per tile)
#ifndef KX_CT
#define KX_CT 256
#endif
constexpr int CT = KX_CT, CW = CT / 64;  // chain pass: one workgroup, lane = group (1024 measured: the launch fails on the MI355X)

constexpr uint64_t V48 = (1ull << 48) - 1;
constexpr int KX_STATUS_VT = 16;         // kx_status.var_total slots
constexpr uint64_t X_ERR = V48;          // chain terminated by a decode error
constexpr uint64_t X_DONE = V48 - 1;     // chain already ended (no records to emit)
constexpr uint64_t X_NONE = V48 - 2;     // no candidate in this tile / lane
constexpr uint64_t X_BAD = V48 - 3;      // group whose speculative tile chain disagrees (chain pass repairs)

// tile words (structure of arrays over tiles, epoch-tagged): aggregate of the index pass, then the
// exclusive prefix inside the group written by the group scan
enum { T_ENT = 0, T_EXIT, T_CNT, T_ERRC, T_ERRP, T_VAR, T_PCNT = T_VAR + KXP_NV_MAX, T_PVAR,
       T_NF = T_PVAR + KXP_NV_MAX };
// T_ERRC of a tile indexed by the fast path (no error possible): its records are canonical and inside the
// window, so the emit pass reads them with the plan alone (emit_canon)
constexpr uint64_t T_CANON = 0x100;
// group words: group aggregate, then the global exclusive base written by the chain pass
enum { G_ENT = 0, G_EXIT, G_CNT, G_ERRC, G_ERRP, G_VAR, G_BCNT = G_VAR + KXP_NV_MAX, G_BVAR,
       G_NF = G_BVAR + KXP_NV_MAX };
// chain carry between chunks: E, record count, var units per slot, nstop, error | done << 1
enum { CY_E = 0, CY_CNT, CY_VAR, CY_NSTOP = CY_VAR + KXP_NV_MAX, CY_FLAGS, CY_WORDS };

// M_FRAME: framing sniff; M_THRIFT_LS: Thrift with list<struct> fields (its own instantiation, so that the
// element loop does not change the register allocation of every other schema's kernels)
enum Mode { M_THRIFT = 0, M_SKIP = 1, M_PB = 2, M_FRAME = 3, M_THRIFT_LS = 4, M_PBB = 5 };
// M_PBB: Kitex-PB Batch frames (0x0A, uvarint length; the nested walker's record boundaries) on the frame
// pipeline, an instantiation of its own: its candidate test (two frames, later 0x0A bytes) inlined into
// the M_FRAME index kernel took it from 4 to 2 waves per SIMD (248 VGPRs), round 5's frames regression
constexpr bool is_frame(int m) { return m == M_FRAME || m == M_PBB; }
__host__ __device__ constexpr bool is_thrift(int m) { return m == M_THRIFT || m == M_THRIFT_LS; }

// diagnostics (KX_DIAG & 64): shader-clock cycles per index-pass phase, summed over tiles (lane 0), in a
// device buffer every decode part shares (DecParams::phase; a __device__ array would be one per part)


struct DecParams {
  const uint8_t* in;
  uint64_t in_len;
  const uint64_t* offsets;   // known-offsets mode when non-null
  const uint64_t* ends;      // known-offsets mode: record r ends at ends[r] (else offsets[r + 1])
  uint64_t n;
  const KAS KxProgram* prog;  // compiled schema (constant address space: scalar loads when uniform)
  KxLaunchCols cols;
  uint8_t* rstat;
  kx_status* status;
  uint64_t* skip_out;        // M_SKIP / M_FRAME: record (frame) start offsets
  uint64_t* fr_ps;           // M_FRAME: payload start / end per frame, kind per frame
  uint64_t* fr_pe;
  uint8_t* fr_kind;
  uint64_t fr_max;           // M_FRAME: payload size limit (0: none)
  int fr_grpc;               // M_FRAME: 0 default-codec sniff, 1 gRPC length-prefixed messages, 2 ttstream,
                             // 3 Kitex-PB Batch frames (nested proto schemas' record extents)
  int32_t* fr_sid;           // ttstream: stream id (TTHeader seqid), method position / length per frame
  uint64_t* fr_mpos;
  uint32_t* fr_mlen;
  uint32_t tts_keys;         // ttstream: frame-type key | ToMethod key << 16
  uint32_t tts_flag;         // ttstream: HeaderFlagsStreaming
  uint64_t tts_name[5];      // ttstream: frame-type values (little-endian packed, NUL-padded)
  uint32_t tts_nlen[5];
  uint8_t* fr_crc;           // M_FRAME with CRC32Check: per-frame code of the fused payload checksum
  uint64_t* tdesc;           // tile words
  uint64_t* gdesc;           // group words
  uint16_t* starts;          // concatenated mode: record starts per tile (slotcap slots each)
  unsigned long long* errkey;  // offsets mode: min((record << 8) | code)
  uint32_t* overflow;        // an arena capacity was exceeded
  uint64_t* nstop;           // records to emit (chain pass)
  uint64_t* nstop_ring;      // chunked pipeline: nstop of chunk k at [k % KX_PIPE_EV] (chain runs ahead of emit)
  uint32_t* redo_n;          // fast index kernel: tiles it could not index (count, then their ids)
  uint32_t* redo;
  int gate_reset;            // chain_kernel zeroes *gate when it ends
  uint32_t* gate;            // chain_kernel runs only when *gate != 0 (chain_fast_kernel's fallback flag)
  uint64_t* split_out;       // kx_thrift_split_points: nsplit + 1 record starts (no emit pass)
  uint32_t nsplit;
  uint64_t var_base[KXP_NV_MAX];  // arena positions start here (a chunk of a larger batch)
  const uint64_t* var_base_dev;   // ... plus these device words (the previous chunk's status->var_total)
  KxpFast fp;                // the canonical plan in segment form (fast_record_fp), fp.ok = 0: none
  KxpEmit ep;                // ... in emit form (emit_fast_kernel), ep.ok = 0: none
  uint64_t ntiles, ngroups, slotcap;
  // chunked pipeline (launch_t): this launch covers tiles [t_lo, t_hi) and groups [g_lo, g_hi); the
  // chain pass carries its state between chunks in `carry`
  uint64_t t_lo, t_hi, g_lo, g_hi;
  uint64_t* carry;
  int chunk_first, chunk_last;
  uint64_t epoch;            // 16-bit call epoch (never 0)
  uint32_t krec;             // offsets mode: records per tile (<= 64)
  uint32_t winb;             // window bytes loaded per tile: TILE + halo + 16 (<= WINB)
  uint32_t nlist;            // numeric list columns (thrift): emit copies them wave-cooperatively
  int direct;                // offsets mode without var columns: emit pass only
  int fast;                  // concatenated Thrift with a canonical plan: fast_tile before walk_tile
  int all_view;              // every var column is a zero-copy view (no arena to lay out)
  int nolds;                 // diagnostics (KX_NOLDS=1): read every byte from global memory
  unsigned long long* phase; // diagnostics (KX_DIAG & 64): the phase-cycle accumulators
  int diag;                  // diagnostics (KX_DIAG bits, timing experiments only; output is wrong):
                             // 1 no walk, 2 no group arrival, 4 no tile words, 256 index pass only
};

// Kernels read their parameter block in place from the kernarg segment: indexing a by-value
// parameter (cols.data[c]) would otherwise make the compiler copy the whole block to scratch per lane.
typedef const KAS DecParams KParams;
#define KX_PARAMS() (*(KParams*)__builtin_amdgcn_kernarg_segment_ptr())

// known-offsets mode: where record r ends (message bodies: an explicit end per record)
__device__ __forceinline__ uint64_t rec_end(KParams& dp, uint64_t r) {
  return dp.ends ? dp.ends[r] : dp.offsets[r + 1];
}

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

// the aligned input dword at A, which holds an input byte below `end`: an aligned dword never crosses a
// page, so its bytes past the input are readable (and ignored by every caller). The CPU emulation
// (tests/emu/build_emu.sh) replaces the read with one of the input bytes alone, the rest poisoned.
__device__ __forceinline__ uint32_t gdword(uint64_t A, uint64_t end) {
  (void)end;
  return *(const GLB uint32_t*)A;  // input tail dword
}

// 4 bytes at p from global memory; never reads past the dword holding the last input byte
__device__ __forceinline__ uint32_t gld4(const Src& w, uint64_t p) {
  uint64_t a = (uint64_t)w.in + p;
  uint64_t A = a & ~3ull;
  uint32_t sh = (uint32_t)(a & 3);
  uint64_t end = (uint64_t)w.in + w.len;
  uint32_t x0 = A < end ? gdword(A, end) : 0u;
  uint32_t x1 = A + 4 < end ? gdword(A + 4, end) : 0u;
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

// Strings, and lists / sets / maps whose elements are strings or fixed-size, are skipped where they are met
// (at a depth that leaves their elements inside the limit) instead of through a frame each: the frame stack
// lives in scratch, and a store + load per string field / element was most of the skip pass's memory traffic
// on nested records
__device__ __forceinline__ int dskip_str(const Src& w, uint64_t& pos, uint64_t limit) {
  if (limit - pos < 4) return KX_ERR_EOF;
  const int32_t l = (int32_t)be32(w, pos);
  if (l < 0) return KX_ERR_INVALID_DATA;
  if (limit - pos - 4 < (uint64_t)l) return KX_ERR_EOF;
  pos += 4 + (uint64_t)l;
  return KX_OK;
}

// a leaf element (a string or fixed-size type, the caller checked which)
__device__ __forceinline__ int dskip_leaf(const Src& w, uint64_t& pos, uint64_t limit, int sz) {
  if (sz > 0) {
    if (limit - pos < (uint64_t)sz) return KX_ERR_EOF;
    pos += (uint64_t)sz;
    return KX_OK;
  }
  return dskip_str(w, pos, limit);
}

// a list / set / map field whose elements are leaves, skipped whole (*done); else nothing is consumed and the
// frame path takes it (also for a header past the limit, so that its error is the frame path's)
__device__ __forceinline__ int dskip_flat(const Src& w, uint64_t& pos, uint64_t limit, uint32_t t, bool& done) {
  done = false;
  const bool map = t == KX_T_MAP;
  const uint64_t hl = map ? 6 : 5;
  if (limit - pos < hl) return KX_OK;
  const uint32_t h = ld4(w, pos);
  const uint32_t k = h & 0xff, v = map ? (h >> 8) & 0xff : k;
  const int ks = tsize(k), vs = tsize(v);
  if (!(ks > 0 || k == KX_T_STRING) || !(vs > 0 || v == KX_T_STRING)) return KX_OK;
  const int32_t cnt = (int32_t)be32(w, pos + (map ? 2 : 1));
  if (cnt < 0) return KX_ERR_INVALID_DATA;
  done = true;
  pos += hl;
  if (map ? ks > 0 && vs > 0 : ks > 0) {
    const uint64_t b = (uint64_t)cnt * (uint64_t)(map ? ks + vs : ks);
    if (limit - pos < b) return KX_ERR_EOF;
    pos += b;
    return KX_OK;
  }
  for (int32_t i = 0; i < cnt; i++) {
    int rc = dskip_leaf(w, pos, limit, ks);
    if (!rc && map) rc = dskip_leaf(w, pos, limit, vs);
    if (rc) return rc;
  }
  return KX_OK;
}

// LEAF: the in-place skips above (the skip decoder's record walk and the field loops' unknown fields); the frame
// walker's PurePayload skip keeps the plain form, whose registers and scratch its TTHeader index kernel shares
template <bool LEAF = true>
__device__ __forceinline__ int dskip_body(const Src& w, uint64_t& pos, uint64_t limit, uint32_t t0, int md0) {
  uint64_t stk[66];
  int sp = 0;
  auto mk = [](uint32_t t, uint32_t md) -> uint64_t { return (uint64_t)(canon_t(t) | (md << 15)); };
  // the top frame in a register (stk holds the frames below it): the field loop of a struct reads and the
  // element loops update it at every step
  uint64_t top = mk(t0, (uint32_t)md0);
  sp = 1;
  while (sp > 0) {
    uint64_t fr = top;
    uint32_t t = fr & 15, kt = (fr >> 4) & 15, vt = (fr >> 8) & 15, st = (fr >> 12) & 3;
    uint32_t ph = (fr >> 14) & 1, md = (fr >> 15) & 127;
    uint32_t rem = (uint32_t)(fr >> 32);
    if (st == 0) {
      if (md == 0) return KX_ERR_DEPTH_LIMIT;
      int sz = tsize(t);
      if (sz > 0) {
        if (limit - pos < (uint64_t)sz) return KX_ERR_EOF;
        pos += sz; if (--sp) top = stk[sp - 1]; continue;
      }
      switch (t) {
        case KX_T_STRING: {
          if (limit - pos < 4) return KX_ERR_EOF;
          int32_t l = (int32_t)be32(w, pos);
          if (l < 0) return KX_ERR_INVALID_DATA;
          if (limit - pos - 4 < (uint64_t)l) return KX_ERR_EOF;
          pos += 4 + (uint64_t)l; if (--sp) top = stk[sp - 1]; continue;
        }
        case KX_T_STRUCT:
          top = (fr & ~(3ull << 12)) | (1ull << 12); continue;
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
            pos += 6 + b; if (--sp) top = stk[sp - 1]; continue;
          }
          pos += 6;
          if (LEAF && md > 1 && (ks > 0 || k == KX_T_STRING) && (vs > 0 || v == KX_T_STRING)) {
            for (int32_t i = 0; i < cnt; i++) {
              int rc = dskip_leaf(w, pos, limit, ks);
              if (!rc) rc = dskip_leaf(w, pos, limit, vs);
              if (rc) return rc;
            }
            if (--sp) top = stk[sp - 1];
            continue;
          }
          top = (uint64_t)t | ((uint64_t)canon_t(k) << 4) | ((uint64_t)canon_t(v) << 8) |
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
            pos += 5 + b; if (--sp) top = stk[sp - 1]; continue;
          }
          pos += 5;
          if (LEAF && md > 1 && v == KX_T_STRING) {
            for (int32_t i = 0; i < cnt; i++) {
              const int rc = dskip_str(w, pos, limit);
              if (rc) return rc;
            }
            if (--sp) top = stk[sp - 1];
            continue;
          }
          top = (uint64_t)t | ((uint64_t)canon_t(v) << 8) | (2ull << 12) | ((uint64_t)md << 15) |
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
      if (tp == KX_T_STOP) { if (--sp) top = stk[sp - 1]; continue; }
      int fsz = tsize(tp);
      if (fsz > 0) {
        if (limit - pos < 2 + (uint64_t)fsz) return KX_ERR_EOF;
        pos += 2 + fsz; continue;
      }
      if (limit - pos < 2) return KX_ERR_EOF;
      pos += 2;
      if (LEAF && tp == KX_T_STRING && md > 1) {
        const int rc = dskip_str(w, pos, limit);
        if (rc) return rc;
        continue;
      }
      if (LEAF && (tp == KX_T_LIST || tp == KX_T_SET || tp == KX_T_MAP) && md > 2) {
        bool done;
        const int rc = dskip_flat(w, pos, limit, tp, done);
        if (rc) return rc;
        if (done) continue;
      }
      stk[sp - 1] = top; top = mk(tp, md - 1); sp++;
    } else if (st == 2) {  // list / set elements
      if (rem == 0) { if (--sp) top = stk[sp - 1]; continue; }
      top = (fr & 0xffffffffull) | ((uint64_t)(rem - 1) << 32);
      stk[sp - 1] = top; top = mk(vt, md - 1); sp++;
    } else {  // map: key then value
      if (rem == 0) { if (--sp) top = stk[sp - 1]; continue; }
      uint32_t et = ph ? vt : kt;
      uint64_t nf = ph ? ((fr & ~(1ull << 14)) & 0xffffffffull) | ((uint64_t)(rem - 1) << 32)
                       : (fr | (1ull << 14));
      top = nf;
      int es = tsize(et);
      if (es > 0) {  // fixed-size element: skipn (only reached when the other side is not)
        if (limit - pos < (uint64_t)es) return KX_ERR_EOF;
        pos += es;
      } else {
        stk[sp - 1] = top; top = mk(et, md - 1); sp++;
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

// record offsets: 4 or 8 bytes per entry (kx_column.offset_bytes). A 4-byte column never wraps: an
// arena position past 2^32 - 1 counts as an overflow (KX_ERR_SIZE_LIMIT), like one past the capacity.
__device__ __forceinline__ void put_off(const KAS KxLaunchCols& cols, uint32_t c, uint64_t r, uint64_t v) {
  if ((cols.owide >> c) & 1) ((GLB uint64_t*)cols.offs[c])[r] = v;
  else ((GLB uint32_t*)cols.offs[c])[r] = (uint32_t)v;
}
// zero-copy view of record r's string (KX_COLF_VIEW): (offset into the input, length); empty -> (0, 0)
__device__ __forceinline__ void put_view(const KAS KxLaunchCols& cols, uint32_t c, uint64_t r, uint64_t pos,
                                         uint64_t len) {
  const uint64_t o = len ? pos : 0;
  if ((cols.owide >> c) & 1) {
    ((GLB uint64_t*)cols.offs[c])[2 * r] = o;
    ((GLB uint64_t*)cols.offs[c])[2 * r + 1] = len;
  } else {
    ((GLB uint64_t*)cols.offs[c])[r] = (o & 0xffffffffull) | (len << 32);  // one 8-byte store per pair
  }
}
// the arena limit of column c in arena units: its capacity, and the 4-byte offset range
__device__ __forceinline__ uint64_t arena_lim(const KAS KxLaunchCols& cols, uint32_t c) {
  return ((cols.owide >> c) & 1) ? cols.cap[c] : kmin64(cols.cap[c], 0xffffffffull);
}
// offsets[i] = v for the record that ends the decoded prefix (n, or the failing record)
__device__ __forceinline__ void put_total(const KAS KxLaunchCols& cols, uint32_t* overflow, uint32_t c, uint64_t i,
                                          uint64_t v) {
  if (v <= arena_lim(cols, c)) put_off(cols, c, i, v);
  else atomicOr(overflow, 1u);
}

// LIST_BYTES: element byte offsets (the record offsets' width), the element limit
__device__ __forceinline__ void put_eoff(const KAS KxLaunchCols& cols, uint32_t c, uint64_t i, uint64_t v) {
  if ((cols.owide >> c) & 1) ((GLB uint64_t*)cols.eoffs[c])[i] = v;
  else ((GLB uint32_t*)cols.eoffs[c])[i] = (uint32_t)v;
}
__device__ __forceinline__ uint64_t elem_lim(const KAS KxLaunchCols& cols, uint32_t c) {
  const uint64_t cap = cols.ecap[c];
  return ((cols.owide >> c) & 1) ? cap : kmin64(cap, 0xffffffffull);
}


__device__ __forceinline__ void store_col(void* base, uint32_t width, uint64_t rec, uint64_t v) {
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

// The decoded prefix ends at record i with per-slot arena totals tot[]: offsets[i] of every var column
// (in elements for a container column) and, for LIST_BYTES, elem_offsets[elements] = bytes.
template <int NV>
__device__ __forceinline__ void close_slots(const KAS KxProgram* P, const KAS KxLaunchCols& cols, uint32_t* overflow,
                                            uint64_t i, const uint64_t* tot) {
#pragma unroll
  for (int v = 0; v < NV; v++) {
    if (v >= (int)P->nvar) break;
    const uint32_t c = P->var_col[v];
    if ((cols.view >> c) & 1) continue;  // views have no closing offset
    const KxpCol K = ld_col(P, c);
    if (K.kind == KXP_K_LISTB) {
      if ((uint32_t)v != K.vslot) continue;
      uint64_t nb = 0;
#pragma unroll
      for (int u = 0; u < NV; u++) if ((uint32_t)u == K.vslot2) nb = tot[u];
      if (tot[v] <= elem_lim(cols, c) && nb <= arena_lim(cols, c)) {
        put_off(cols, c, i, tot[v]);
        put_eoff(cols, c, tot[v], nb);
      } else {
        atomicOr(overflow, 1u);
      }
    } else {
      put_total(cols, overflow, c, i, tot[v]);
    }
  }
}

// One element of a list<S> (S of fixed-width scalars) at q: S's FastRead (struct_tpl.go:41-149): fields
// until STOP, unknown / mistyped ids skipped, the last duplicate wins, required fields checked. S's fields
// are the columns c0 .. c0 + ns - 1 (sel_id / sel_req / elem / width / defv). want >= 0: *val = the value
// of S's field `want` (host order), or its default when the element lacks it. *qe = the element's end.
__device__ __forceinline__ int elem_struct(const Src& w, const KAS KxProgram* P, uint32_t c0, uint32_t ns, uint64_t q,
                                           uint64_t limit, uint64_t* qe, int want, uint64_t* val) {
  uint32_t isset = 0;
  if (want >= 0) *val = (uint64_t)ldk(&P->col[c0 + want]).defv;
  for (;;) {
    if (q >= limit) return KX_ERR_EOF;
    const uint32_t h = ld4(w, q);
    const uint32_t t = h & 0xff;
    if (t == KX_T_STOP) { q += 1; break; }
    if (limit - q < 3) return KX_ERR_EOF;
    const int16_t id = (int16_t)((((h >> 8) & 0xffu) << 8) | ((h >> 16) & 0xffu));
    q += 3;
    int k = -1;
    for (uint32_t j = 0; j < ns; j++)
      if (P->sel_id[c0 + j] == id) { k = (int)j; break; }
    const KxpCol K = ldk(&P->col[c0 + (k < 0 ? 0 : k)]);
    if (k < 0 || K.elem != t) {
      const int rc = dskip_body(w, q, limit, t, 64);
      if (rc) return rc;
      continue;
    }
    if (limit - q < K.width) return KX_ERR_EOF;
    if (k == want) {
      uint64_t v;
      if (K.width == 1) v = t == KX_T_BOOL ? (ld1(w, q) == 1) : ld1(w, q);
      else if (K.width == 2) v = __builtin_bswap32(ld4(w, q)) >> 16;
      else if (K.width == 4) v = __builtin_bswap32(ld4(w, q));
      else v = be64(w, q);
      *val = v;
    }
    q += K.width;
    isset |= 1u << k;
  }
  for (uint32_t j = 0; j < ns; j++)
    if (P->sel_req[c0 + j] && !((isset >> j) & 1)) return KX_ERR_INVALID_DATA;
  *qe = q;
  return KX_OK;
}

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
template <int NV, bool LS>
__device__ __forceinline__ int generic_record(const Src& w, const KAS KxProgram* P, const KAS KxLaunchCols& cols,
                                              uint64_t start, uint64_t limit, uint64_t rec, bool emit,
                                              uint64_t* endp, VarState<NV>& vs, uint64_t& pres_out) {
#pragma unroll
  for (int i = 0; i < NV; i++) { vs.len[i] = 0; vs.pos[i] = 0; }
  uint64_t pres = 0;
  uint64_t pos = start;
  int inst = 0;
  int pred = P->inst[0].enc_first;
  int ipred = -1;   // IDL-order guess: the field after the last one read
  uint64_t seen = 0;
  // inside a list<S> field (S of fixed scalars): its elements are read by this same loop (one skip
  // decoder instance per kernel: a second inlined copy doubled the index pass's scratch and halved it)
  uint32_t lrem = 0, lisset = 0, lcnt = 0, lcol = 0, lns = 0;
  int lfi = 0, lpbit = -1;
  uint64_t lstart = 0;
  for (;;) {
    if (pos >= limit) return KX_ERR_EOF;
    const Fetch fx = fetch12(w, pos);
    KxpField F = ld_field(P, pred >= 0 ? pred : 0);
    const uint32_t t = fx.w0 & 0xff;
    int fi = -1;
    if (LS && lrem) {  // an element of list<S>: S.FastRead (struct_tpl.go:41-149)
      if (t == KX_T_STOP) {
        pos += 1;
        for (uint32_t j = 0; j < lns; j++)
          if (P->sel_req[lcol + j] && !((lisset >> j) & 1)) return KX_ERR_INVALID_DATA;
        lisset = 0;
        if (--lrem == 0) {
          for (uint32_t k = 0; k < lns; k++) vset<NV>(vs, ldk(&P->col[lcol + k]).vslot, lstart, lcnt);
          seen |= 1ull << lfi;
          if (lpbit >= 0) pres |= 1ull << lpbit;
        }
        continue;
      }
      if (limit - pos < 3) return KX_ERR_EOF;
      const int16_t eid = (int16_t)((((fx.w0 >> 8) & 0xffu) << 8) | ((fx.w0 >> 16) & 0xffu));
      int k = -1;
      for (uint32_t j = 0; j < lns; j++)
        if (P->sel_id[lcol + j] == eid) { k = (int)j; break; }
      if (k >= 0) {
        const KxpCol K = ldk(&P->col[lcol + k]);
        if (K.elem == t) {
          if (limit - pos - 3 < K.width) return KX_ERR_EOF;
          pos += 3 + K.width;
          lisset |= 1u << k;
          continue;
        }
      }
      // an unknown or mistyped element field: the skip decoder below
    } else if (t == KX_T_STOP) {
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
    if (LS && lrem) {
    } else if (pred >= 0 && F.id == id) {
      fi = pred;
    } else {
      // the encoder-order guess missed: the field after the last one in IDL order (a producer writing IDL
      // order, e.g. Apache Thrift), else a scan of the instance's fields
      const KxpInst I = ld_inst(P, inst);
      if (ipred >= I.first && ipred < I.first + I.nfields && P->f[ipred].id == id) {
        fi = ipred;
      } else {
        for (int k = 0; k < I.nfields; k++)
          if (P->f[I.first + k].id == id) { fi = I.first + k; break; }
      }
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
    ipred = fi + 1;
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
    } else if (F.kind == KXP_K_LISTB) {                      // list/set<string>: size x ReadString (:582-625)
      if (limit - vp < 5) return KX_ERR_EOF;
      const int32_t l = (int32_t)__builtin_bswap32(fx.w1);
      if (l < 0) return KX_ERR_NEGATIVE_SIZE;
      uint64_t q = vp + 5, nb = 0;
      for (int32_t j = 0; j < l; j++) {
        if (limit - q < 4) return KX_ERR_EOF;
        const int32_t sl = (int32_t)__builtin_bswap32(ld4(w, q));
        if (sl < 0) return KX_ERR_NEGATIVE_SIZE;
        if (limit - q - 4 < (uint64_t)sl) return KX_ERR_EOF;
        nb += (uint64_t)sl;
        q += 4 + (uint64_t)sl;
      }
      const KxpCol K = ld_col(P, F.col);
      vset<NV>(vs, K.vslot, vp + 5, (uint32_t)l);
      vset<NV>(vs, K.vslot2, vp + 5, (uint32_t)nb);
      pos = q;
    } else if (F.kind == KXP_K_MAP) {                        // ReadMapBegin + size x (key, value) (:466-533)
      if (limit - vp < 6) return KX_ERR_EOF;
      const int32_t l = (int32_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(fx.w2, fx.w1, 1));
      if (l < 0) return KX_ERR_NEGATIVE_SIZE;
      const uint32_t kt = F.elem & 15u, vt = F.elem >> 4;
      const uint32_t kw = (uint32_t)tsize(kt), vw = (uint32_t)tsize(vt);
      uint64_t q = vp + 6, nb[2] = {0, 0};
      if (kw && vw) {
        if ((limit - q) / (kw + vw) < (uint64_t)l) return KX_ERR_EOF;
        q += (uint64_t)l * (kw + vw);
      } else {
        for (int32_t j = 0; j < l; j++) {
#pragma unroll
          for (int side = 0; side < 2; side++) {
            const uint32_t sw = side ? vw : kw;
            if (sw) {
              if (limit - q < sw) return KX_ERR_EOF;
              q += sw;
            } else {
              if (limit - q < 4) return KX_ERR_EOF;
              const int32_t sl = (int32_t)__builtin_bswap32(ld4(w, q));
              if (sl < 0) return KX_ERR_NEGATIVE_SIZE;
              if (limit - q - 4 < (uint64_t)sl) return KX_ERR_EOF;
              nb[side] += (uint64_t)sl;
              q += 4 + (uint64_t)sl;
            }
          }
        }
      }
#pragma unroll
      for (int side = 0; side < 2; side++) {
        const KxpCol K = ld_col(P, F.col + side);
        vset<NV>(vs, K.vslot, vp + 6, (uint32_t)l);
        if (K.vslot2 != 0xff) vset<NV>(vs, K.vslot2, vp + 6, (uint32_t)nb[side]);
      }
      pos = q;
    } else if (LS && F.kind == KXP_K_LSTRUCT) {              // list/set<S>: size x S.FastRead (:583-625)
      if (limit - vp < 5) return KX_ERR_EOF;
      const int32_t l = (int32_t)__builtin_bswap32(fx.w1);
      if (l < 0) return KX_ERR_NEGATIVE_SIZE;
      pos = vp + 5;
      if (l > 0) {  // the elements follow through this loop; the list is recorded after its last one
        lrem = (uint32_t)l; lcnt = (uint32_t)l; lisset = 0;
        lcol = (uint32_t)F.col; lns = F.width; lfi = fi; lpbit = F.pbit; lstart = pos;
        continue;
      }
      for (uint32_t k = 0; k < F.width; k++) vset<NV>(vs, ldk(&P->col[F.col + k]).vslot, pos, 0u);
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

__device__ __forceinline__ void emit_defaults(const KAS KxProgram* P, const KAS KxLaunchCols& cols, uint64_t rec) {
  for (uint32_t c = 0; c < P->ncols; c++) {
    const KxpCol K = ld_col(P, c);
    if (K.kind == KXP_K_FIXED) store_col(cols.data[c], K.width, rec, (uint64_t)K.defv);
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
template <bool EARLY = true>
__device__ __forceinline__ int pb_varint_f(const Fetch& f, uint64_t rem, uint64_t& v, uint32_t& used) {
  if (EARLY && !(f.w0 & 0x80u)) {  // one byte: tags, lengths < 128, small values (usually wave-uniform)
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

// the same checks as pb_varint_f, the length alone (the index pass measures records: values unused)
__device__ __forceinline__ int pb_varint_len_f(const Fetch& f, uint64_t rem, uint32_t& used) {
  const uint64_t lo = (uint64_t)f.w0 | ((uint64_t)f.w1 << 32);
  const uint64_t stop = ~lo & 0x8080808080808080ull;
  const uint32_t b8 = f.w2 & 0xffu, b9 = (f.w2 >> 8) & 0xffu;
  const uint32_t k = stop ? (uint32_t)__builtin_ctzll(stop) >> 3 : b8 < 0x80 ? 8u : b9 < 0x80 ? 9u : 10u;
  if (k >= 9) {
    if (rem <= 9) return KX_ERR_EOF;
    if (b9 > 1) return KX_ERR_INVALID_DATA;
  } else if ((uint64_t)k >= rem) {
    return KX_ERR_EOF;
  }
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
__device__ __noinline__ bool pb_utf8_slow(const Src w, uint64_t p, uint64_t n) {
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
    const uint32_t lm = tail ? 0xffffffffu >> (8 * (4 - tail)) : 0xffffffffu;
    const uint32_t first = s[0] & (0xffffffffu << (8 * sh));
    uint32_t acc;
    if (nd == 1) {
      acc = first & lm;
    } else {  // the masked edge dwords, then the ones between with four independent ORs
      uint32_t a0 = first, a1 = s[nd - 1] & lm, a2 = 0, a3 = 0;
      int i = 1;
      for (; i + 4 <= nd - 1; i += 4) { a0 |= s[i]; a1 |= s[i + 1]; a2 |= s[i + 2]; a3 |= s[i + 3]; }
      for (; i < nd - 1; i++) a0 |= s[i];
      acc = a0 | a1 | a2 | a3;
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
      if (emit) store_col(cols.data[F.col], F.width, rec, v);  // int32: low 32 bits
    } else if (wt == 1) {
      if (rem < 8) return KX_ERR_EOF;
      if (emit) store_col(cols.data[F.col], F.width, rec, (uint64_t)fv.w0 | ((uint64_t)fv.w1 << 32));
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
      if (K.kind == KXP_K_FIXED && !((seen >> K.field) & 1)) store_col(cols.data[c], K.width, rec, (uint64_t)K.defv);
    }
  }
  pres_out = pres;
  return KX_OK;
}

// Protobuf canonical plan (the PB counterpart of canon_record): the steps are the root fields in
// field-number order, the order proto.Marshal writes (protobuf.go:209-216 -> proto.Marshal); every
// lane runs the same step at once, so each step's descriptor is a scalar load, and a lane whose next
// tag is not the step's tag has that field absent (proto3 omits zero values) and keeps its default.
// False when the record has anything else left at the end (unknown or out-of-order fields, a
// repeated field, a malformed value): the generic field loop then decodes it from the start and
// reports the error.
#ifndef KX_PB_NOEARLY
#define KX_PB_NOEARLY 1   // A/B knob: plan varint values decoded without the one-byte early exit
#endif
// The same plan over a record that lies in the LDS window with 16 bytes to spare (the usual case): positions
// are 32-bit window offsets, every fetch is four LDS reads with no window test and no global-memory branch.
template <int NV>
__device__ __forceinline__ bool pb_canon_lds(const Src& w, const KAS KxProgram* P, const KAS KxLaunchCols& cols,
                                             uint64_t start, uint32_t q0, uint32_t qlim, uint64_t rec, bool emit,
                                             bool utf8, VarState<NV>& vs, uint64_t& pres_out) {
  uint32_t q = q0;
  uint64_t pres = 0;
  const uint32_t ns = P->npbsteps;
  for (uint32_t k = 0; k < ns; k++) {
    const KxpStep S = ldk(&P->pbsteps[k]);
    const uint32_t tl = (S.hdr >> 16) & 3u;
    bool present = false;
    if (q < qlim) {
      const LDS uint32_t* sw = w.win + (q >> 2);
      const uint32_t sh = q & 3;
      const uint32_t x0 = sw[0], x1 = sw[1], x2 = sw[2], x3 = sw[3];
      Fetch f;
      f.w0 = __builtin_amdgcn_alignbyte(x1, x0, sh);
      f.w1 = __builtin_amdgcn_alignbyte(x2, x1, sh);
      f.w2 = __builtin_amdgcn_alignbyte(x3, x2, sh);
      present = (f.w0 & (tl == 1 ? 0xffu : 0xffffu)) == (S.hdr & 0xffffu) && qlim - q > tl;
      if (present) {
        const uint32_t rem = qlim - q - tl;
        const Fetch fv = fetch_skip(f, tl);
        uint64_t v;
        uint32_t u;
        if (S.kind == KXP_S_PB_VARINT) {
          if (!emit) {
            if (pb_varint_len_f(fv, rem, u)) return false;
          } else {
            // values of any length: the one-byte early exit would split the wave (both paths run)
            if (pb_varint_f<!KX_PB_NOEARLY>(fv, rem, v, u)) return false;
            if ((S.hdr >> 24) & 1u) v = v != 0;
            store_col(cols.data[S.col], S.width, rec, v);
          }
          q += tl + u;
        } else if (S.kind == KXP_S_PB_FIXED64) {
          if (rem < 8) return false;
          if (emit) store_col(cols.data[S.col], S.width, rec, (uint64_t)fv.w0 | ((uint64_t)fv.w1 << 32));
          q += tl + 8;
        } else {
          if (pb_varint_f(fv, rem, v, u) || v > rem - u) return false;
          const uint32_t b = q + tl + u;
          const uint64_t pb = start + (b - q0);
          if (utf8 && !((S.hdr >> 25) & 1u) && !pb_utf8_ok(w, pb, v)) return false;
          vset<NV>(vs, S.vslot, pb, (uint32_t)v);
          q = b + (uint32_t)v;
        }
        const int pbit = (int)(S.kind == KXP_S_PB_LEN ? S.width : S.vslot) - 1;  // kx_schema.cpp
        if (pbit >= 0) pres |= 1ull << pbit;
      }
    }
    if (!present && emit && S.kind != KXP_S_PB_LEN)
      store_col(cols.data[S.col], S.width, rec, (uint64_t)ld_col(P, S.col).defv);
  }
  if (q != qlim) return false;
  pres_out = pres;
  return true;
}

template <int NV>
__device__ __forceinline__ bool pb_canon(const Src& w, const KAS KxProgram* P, const KAS KxLaunchCols& cols,
                                         uint64_t start, uint64_t limit, uint64_t rec, bool emit, bool utf8,
                                         VarState<NV>& vs, uint64_t& pres_out) {
#ifndef KX_PB_LDS
#define KX_PB_LDS 1   // A/B knob: the window-offset walk above
#endif
  if (KX_PB_LDS && limit >= start && limit - start <= 65536) {
    const int32_t q0 = wofs(w, start, (uint32_t)(limit - start) + 16);
    if (q0 >= 0) return pb_canon_lds<NV>(w, P, cols, start, (uint32_t)q0, (uint32_t)q0 + (uint32_t)(limit - start),
                                         rec, emit, utf8, vs, pres_out);
  }
  uint64_t pos = start, pres = 0;
  const uint32_t ns = P->npbsteps;
  for (uint32_t k = 0; k < ns; k++) {
    const KxpStep S = ldk(&P->pbsteps[k]);
    const uint32_t tl = (S.hdr >> 16) & 3u;
    bool present = false;
    if (pos < limit) {
      const Fetch f = fetch12(w, pos);
      present = (f.w0 & (tl == 1 ? 0xffu : 0xffffu)) == (S.hdr & 0xffffu) && limit - pos > tl;
      if (present) {
        const uint64_t rem = limit - pos - tl;
        const Fetch fv = fetch_skip(f, tl);
        uint64_t v;
        uint32_t u;
        if (S.kind == KXP_S_PB_VARINT) {
          if (!emit) {  // measuring: the value is not needed
            if (pb_varint_len_f(fv, rem, u)) return false;
          } else {
            if (pb_varint_f(fv, rem, v, u)) return false;
            if ((S.hdr >> 24) & 1u) v = v != 0;
            store_col(cols.data[S.col], S.width, rec, v);  // int32: low 32 bits
          }
          pos += tl + u;
        } else if (S.kind == KXP_S_PB_FIXED64) {
          if (rem < 8) return false;
          if (emit) store_col(cols.data[S.col], S.width, rec, (uint64_t)fv.w0 | ((uint64_t)fv.w1 << 32));
          pos += tl + 8;
        } else {
          if (pb_varint_f(fv, rem, v, u) || v > rem - u) return false;
          const uint64_t b = pos + tl + u;
          if (utf8 && !((S.hdr >> 25) & 1u) && !pb_utf8_ok(w, b, v)) return false;
          vset<NV>(vs, S.vslot, b, (uint32_t)v);
          pos = b + v;
        }
        const int pb = (int)(S.kind == KXP_S_PB_LEN ? S.width : S.vslot) - 1;  // kx_schema.cpp
        if (pb >= 0) pres |= 1ull << pb;
      }
    }
    if (!present && emit && S.kind != KXP_S_PB_LEN)
      store_col(cols.data[S.col], S.width, rec, (uint64_t)ld_col(P, S.col).defv);
  }
  if (pos != limit) return false;
  pres_out = pres;
  return true;
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
#ifndef KX_SCAN32
#define KX_SCAN32 1   // A/B knob: emit_tile's arena scan with DPP moves when the wave's lengths allow
#endif
// Inclusive scan of 32-bit values over the wave with DPP moves (row shifts, then the row broadcasts): no
// LDS traffic, unlike the bpermute-based wave_incl_scan
__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

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

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int l) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, l, 64);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), l, 64);
  return ((uint64_t)hi << 32) | lo;
}

// ---- long strings: copied by the whole wave (bimodal record sizes) ----
// A string of KX_WAVE_COPY bytes or more costs one lane n/16 dependent 16-byte round trips; a batch with 1 %
// of its records at 64 KiB spent 11x the canonical time per byte in them. Lanes holding one defer it, and
// the wave copies the deferred strings one after another, lane k taking 16-byte pieces k, k + 64, ... of
// the 16-byte-aligned destination body (four pieces in flight per lane). For strings of this size the wave
// form never needs more rounds than the lanes would (n/1024 per string, 64 strings: n/16).
#define KX_WAVE_COPY 1024u
__device__ __forceinline__ void wave_copy_one(const Src& w, uint64_t src, uint32_t n, GLB uint8_t* dst,
                                              int lane, bool inwin) {
  const uint32_t h = min((uint32_t)((16u - ((uint32_t)(uintptr_t)dst & 15u)) & 15u), n);
  const bool body_ok = inwin || src + n + 20 <= w.len;   // ld16's global form reads 4 bytes past the piece
  if (!body_ok) {
    for (uint32_t i = lane; i < n; i += 64) dst[i] = (uint8_t)ld1(w, src + i);
    return;
  }
  if ((uint32_t)lane < h) dst[lane] = (uint8_t)ld1(w, src + lane);
  const uint32_t nb = (n - h) & ~15u;
  GLB uint8_t* d = dst + h;
  const uint64_t s = src + h;
  uint32_t i = (uint32_t)lane * 16u;
  for (; i + 3 * 1024 + 16 <= nb; i += 4 * 1024) {
    const Q16 a = ld16(w, s + i, inwin), b = ld16(w, s + i + 1024, inwin);
    const Q16 c = ld16(w, s + i + 2048, inwin), e = ld16(w, s + i + 3072, inwin);
    *(GLB v4u*)(d + i) = v4u{a.a0, a.a1, a.a2, a.a3};
    *(GLB v4u*)(d + i + 1024) = v4u{b.a0, b.a1, b.a2, b.a3};
    *(GLB v4u*)(d + i + 2048) = v4u{c.a0, c.a1, c.a2, c.a3};
    *(GLB v4u*)(d + i + 3072) = v4u{e.a0, e.a1, e.a2, e.a3};
  }
  for (; i < nb; i += 1024) {
    const Q16 a = ld16(w, s + i, inwin);
    *(GLB v4u*)(d + i) = v4u{a.a0, a.a1, a.a2, a.a3};
  }
  const uint32_t tl = n - h - nb;   // < 16
  if ((uint32_t)lane < tl) d[nb + lane] = (uint8_t)ld1(w, s + nb + lane);
}
// every lane with big set hands its string (src, n -> dst) to the wave; uniform control flow
__device__ __forceinline__ void wave_copy_deferred(const Src& w, bool big, uint64_t src, uint32_t n, uint8_t* dst,
                                                   int lane, bool inwin) {
  uint64_t m = __ballot(big);
  while (m) {
    const int l = __builtin_ctzll(m);
    m &= m - 1;
    const uint64_t s = rl64(src, l);
    const uint32_t nn = __builtin_amdgcn_readlane(n, l);
    GLB uint8_t* d = (GLB uint8_t*)rl64((uint64_t)(uintptr_t)dst, l);
    wave_copy_one(w, s, nn, d, lane, inwin);
  }
}

// emit: numeric list columns copied by the whole wave, one element per lane (1), or record by record (0)
#ifndef KX_EMIT_COOP
#define KX_EMIT_COOP 1
#endif


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

// Polls `nw` words of item i (fields f0.. of `fields`), lanes with !act skip. Returns false on timeout.
template <int NW>
__device__ __forceinline__ bool get_words(const uint64_t* base, uint64_t nitems, const int* fields, int nw, uint64_t i,
                                          uint64_t ep, bool act, uint64_t* out) {
  const uint64_t t0 = now_ns();
  int backoff = 1;
  for (;;) {
    bool ok = true;
    if (act) {
#pragma unroll
      for (int k = 0; k < NW; k++) {
        if (k >= nw) break;
        const uint64_t x = aload64(base + (uint64_t)fields[k] * nitems + i);
        ok &= (x >> 48) == ep;
        out[k] = x & V48;
      }
    }
    if (!__ballot(!ok)) return true;
    if (now_ns() - t0 > 2000000000ull) return false;
    for (int k = 0; k < backoff; k++) __builtin_amdgcn_s_sleep(1);
    backoff = backoff < 16 ? backoff * 2 : 16;
  }
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

// the two lowest signature offsets of the segment (>= SEG when absent), for the canonical-record
// candidate checks. The 33-dword loop only records which dwords hold a hit (one bit per dword); the
// hit positions are then recomputed for the (one or two) lowest such dwords. Positions are exact: bytes
// of dword 0 below the segment start and bytes of dword 32 at or past its end are masked off.
__device__ __forceinline__ void scan_segment2(const Src& w, int32_t q0, uint32_t sig, int lane, uint32_t& c1,
                                              uint32_t& c2) {
  const LDS uint32_t* s = w.win + (q0 >> 2);
  const uint32_t sh0 = q0 & 3;
  const uint32_t b0 = (sig & 0xff) * 0x01010101u, b1 = ((sig >> 8) & 0xff) * 0x01010101u;
  const uint32_t b2 = ((sig >> 16) & 0xff) * 0x01010101u;
  uint64_t hb = 0;
  int idx = lane % 33;
  for (int i = 0; i < 33; i++) {
    const uint32_t x0 = s[idx], x1 = s[idx + 1];
    const uint32_t m = zero_bytes((x0 ^ b0) | (__builtin_amdgcn_alignbyte(x1, x0, 1) ^ b1) |
                                  (__builtin_amdgcn_alignbyte(x1, x0, 2) ^ b2));
    hb |= (uint64_t)(m != 0) << idx;
    idx = idx == 32 ? 0 : idx + 1;
  }
  c1 = ~0u;
  c2 = ~0u;
  const uint32_t lowm = sh0 ? (0xffffffffu >> (32 - 8 * sh0)) : 0u;  // bytes j < sh0 of a dword
  while (hb) {
    const int d = __ffsll((long long)hb) - 1;
    hb &= hb - 1;
    const uint32_t x0 = s[d], x1 = s[d + 1];
    uint32_t m = zero_bytes((x0 ^ b0) | (__builtin_amdgcn_alignbyte(x1, x0, 1) ^ b1) |
                            (__builtin_amdgcn_alignbyte(x1, x0, 2) ^ b2));
    if (d == 0) m &= ~lowm;
    else if (d == 32) m &= lowm;
    while (m) {
      const uint32_t h = (uint32_t)(4 * d) - sh0 + first_hit(m);
      m &= m - 1;
      if (c1 == ~0u) {
        c1 = h;
      } else {
        c2 = h;
        break;
      }
    }
    if (c2 != ~0u) break;
  }
}

// Kitex-Protobuf record candidate at p: a Batch frame header (0x0A, uvarint length) whose body fits
// the input, starts with a plausible tag, and is followed by the next frame's 0x0A (or the end).
__device__ __forceinline__ int pb_varint(const Src& w, uint64_t p, uint64_t rem, uint64_t& v, uint32_t& used);
// one Batch frame at p (0x0A there): its length and its body's first tag are plausible; *e = its end
__device__ __forceinline__ bool pb_frame_at(const Src& w, uint64_t p, uint64_t len, uint64_t* e) {
  uint64_t l;
  uint32_t u;
  if (p + 1 >= len || pb_varint(w, p + 1, len - p - 1, l, u) || u > 5 || l > len - p - 1 - u) return false;
  const uint64_t b = p + 1 + u;
  *e = b + l;
  if (l) {
    const uint32_t t = ld1(w, b), wt = t & 7;
    if (t < 8 || wt == 3 || wt == 4 || wt > 5) return false;
  }
  return true;
}
// A candidate frame: it and the frame after it check out (or it ends the input). One frame alone let
// 0x0A bytes inside nested messages through (a map<string, V> entry, a repeated field-1 message): their
// false chains merged into the true one a record late, and the chain pass re-scanned group after group
// (1 M PN records: 61 ms of the 77 ms decode in the chain kernel before this, round 5).
// The candidate's body must also open with up to 3 well-formed fields (tag varint with a field number and a
// wire type of 0 / 1 / 2 / 5, its value inside the body): a 0x0A inside a record whose next byte happens to
// be the length to the next record's start passed the frame checks, and the chain pass re-scanned its group
// (1 M PN records tiled from 4 096: 28 groups, 0.58 ms of a 10.4 ms decode, round 6).
__device__ __forceinline__ bool pb_body_plausible(const Src& w, uint64_t b, uint64_t e) {
  uint64_t q = b;
  for (int k = 0; k < 3 && q < e; k++) {
    uint64_t tag, v;
    uint32_t u;
    if (pb_varint(w, q, e - q, tag, u) || u > 5 || (tag >> 3) == 0) return false;
    q += u;
    switch (tag & 7) {
      case 0:
        if (pb_varint(w, q, e - q, v, u)) return false;
        q += u;
        break;
      case 1: q += 8; break;
      case 5: q += 4; break;
      case 2:
        if (pb_varint(w, q, e - q, v, u) || v > e - q - u) return false;
        q += u + v;
        break;
      default: return false;
    }
    if (q > e) return false;
  }
  return true;
}
// BODY: also the body check (M_PBB, nested messages; flat M_PB records keep the two frame checks alone: the
// body check cost the PF index pass 1.7 ms for nothing)
template <bool BODY>
__device__ __forceinline__ bool pb_frame_ok(const Src& w, uint64_t p, uint64_t len) {
  uint64_t e, e2;
  if (!pb_frame_at(w, p, len, &e)) return false;
  if (e != len && !(ld1(w, e) == 0x0Au && pb_frame_at(w, e, len, &e2) && (e2 == len || ld1(w, e2) == 0x0Au)))
    return false;
  if (!BODY) return true;
  uint64_t l;
  uint32_t u;
  (void)pb_varint(w, p + 1, len - p - 1, l, u);   // (pb_frame_at checked it)
  return pb_body_plausible(w, p + 1 + u, e);   // last: true frames all reach it
}

// Kitex-Protobuf candidate in a lane's segment [seg_lo, seg_hi): the rotated, conflict-free scan
// (as scan_segment) keeps the two lowest 0x0A bytes, then only those two are validated as frame
// headers. Frame validation is a varint decode plus two probes, far too costly to run for every
// 0x0A byte inside the scan loop (a divergent branch taken by the whole wave). If neither validates
// the lane has no candidate and takes its entry from the chain below (speculation only).
template <bool BODY>
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
  if (c1 < n && pb_frame_ok<BODY>(w, seg_lo + c1, len)) return seg_lo + c1;
  if (c2 >= n) return X_NONE;
  if (pb_frame_ok<BODY>(w, seg_lo + c2, len)) return seg_lo + c2;
  // both lowest were false (0x0A bytes in the previous record's tail): the segment's later 0x0A bytes in
  // order, so the tile's first frame is still its entry (a later one would send the group to the chain
  // pass's serial re-scan)
  if (q0 >= 0 && n == SEG) {   // dword by dword from the window: only the 0x0A bytes are probed
    const LDS uint32_t* s = w.win + (q0 >> 2);
    const uint32_t sh0 = q0 & 3;
    for (uint32_t d = (c2 + 1 + sh0) >> 2; d < 33; d++) {
      uint32_t m = zero_bytes(s[d] ^ 0x0A0A0A0Au);
      while (m) {
        const uint32_t rel = 4 * d + first_hit(m) - sh0;
        m &= m - 1;
        if (rel <= c2 || rel >= n) continue;
        if (pb_frame_ok<BODY>(w, seg_lo + rel, len)) return seg_lo + rel;
      }
    }
    return X_NONE;
  }
  for (uint32_t rel = c2 + 1; rel < n; rel++)
    if (ld1(w, seg_lo + rel) == 0x0Au && pb_frame_ok<BODY>(w, seg_lo + rel, len)) return seg_lo + rel;
  return X_NONE;
}

// ---------------------------------------------------------------------------------------------
// the decode pipeline
// ---------------------------------------------------------------------------------------------
// HBM -> LDS window for input position `lo`: buffer LDS-DMA, every chunk in flight together. Only
// whole 16-byte chunks inside the input are loaded (the input buffer may end right there); the last
// < 16 bytes of the input are read from global memory. The descriptor is built from wave-uniform
// values (SGPRs); a chunk past num_records still writes its LDS slot (zeros), so the issue loop masks
// the lanes past the window's end.
#ifndef KX_DMA_AUX
#define KX_DMA_AUX 0   // cache policy of the window DMA (2: nt, MI355X_MICROARCH.md "nt-weights"); A/B knob
#endif
template <int WB = WINB>
__device__ __forceinline__ Src load_window(KParams& dp, LDS uint32_t* win, uint64_t lo, int lane, bool thrift,
                                           bool wait = true) {
  constexpr int WL = (WB / 16 + 63) / 64;
  const uint64_t abs_in = (uint64_t)dp.in;
  const uint64_t wbase = (abs_in + kmin64(lo, dp.in_len)) & ~15ull;
  const uint64_t end = abs_in + dp.in_len;
  const int32_t wlen = dp.nolds || end < wbase + 16 ? 0 : (int32_t)kmin64((uint64_t)dp.winb, (end - wbase) & ~15ull);
  const uint32_t blo = __builtin_amdgcn_readfirstlane((uint32_t)wbase);
  const uint32_t bhi = __builtin_amdgcn_readfirstlane((uint32_t)(wbase >> 32));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((uint64_t)bhi << 32) | blo), (short)0, __builtin_amdgcn_readfirstlane(wlen), 0x00020000);
#pragma unroll
  for (int k = 0; k < WL; k++)
    if ((k + 1) * 64 <= WB / 16 || k * 64 + lane < WB / 16)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS void*)(win + k * 256), 16, lane * 16, k * 1024, 0,
                                               KX_DMA_AUX);
  if (wait) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const KAS KxProgram* P = dp.prog;
  return Src{dp.in, dp.in_len, wbase - abs_in, wlen, win, thrift ? P->steps : nullptr, thrift ? P->nsteps : 0u,
             thrift ? P->canon_pres : 0ull};
}

// ---------------------------------------------------------------------------------------------
// Framing sniff (M_FRAME): one socket-buffer frame at pos. defaultCodec.DecodeMeta + checkPayload
// (default_codec.go:189-221, 328-427), Mesh header (header_codec.go:192-212), TTHeader meta + info
// blocks (gopkg protocol/ttheader, un-vendored; same restatement as oracle kxo_frame_one).
// kind = transport.Protocol (0 PurePayload, 2 TTHeader, 4 Framed, 6 TTHeaderFramed) | 0x10 Kitex-PB
// | 0x20 Mesh. Lane-serial per frame: headers are short and rarely repeated within a wave.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t be16s(const Src& w, uint64_t p) { return __builtin_bswap32(ld4(w, p)) >> 16; }

// readStrKVInfo (header_codec.go:115-138) over [b, b + len); *i advanced
__device__ __forceinline__ int fr_kv_strings(const Src& w, uint64_t b, uint64_t len, uint64_t& i) {
  if (i + 2 > len) return KX_ERR_UNKNOWN_PROTOCOL;
  const uint32_t k = be16s(w, b + i);
  i += 2;
  for (uint32_t j = 0; j < 2 * k; j++) {
    if (i + 2 > len) return KX_ERR_UNKNOWN_PROTOCOL;
    const uint64_t l = be16s(w, b + i);
    if (i + 2 + l > len) return KX_ERR_UNKNOWN_PROTOCOL;
    i += 2 + l;
  }
  return KX_OK;
}

__device__ __forceinline__ int fr_tth_info(const Src& w, uint64_t b, uint64_t len) {
  const uint32_t proto = ld1(w, b);
  if (proto != 0 && proto != 3 && proto != 4) return KX_ERR_UNKNOWN_PROTOCOL;  // checkProtocolID
  const uint64_t nt = ld1(w, b + 1);
  if (len - 2 < nt) return KX_ERR_UNKNOWN_PROTOCOL;
  uint64_t i = 2 + nt;
  while (i < len) {
    const uint32_t id = ld1(w, b + i++);
    if (id == 0x00) continue;  // padding
    int rc = KX_OK;
    if (id == 0x01) {
      rc = fr_kv_strings(w, b, len, i);
    } else if (id == 0x10) {  // int KVs: u16 count, (u16 key, u16-length string)
      if (i + 2 > len) return KX_ERR_UNKNOWN_PROTOCOL;
      const uint32_t k = be16s(w, b + i);
      i += 2;
      for (uint32_t j = 0; j < k; j++) {
        if (i + 4 > len) return KX_ERR_UNKNOWN_PROTOCOL;
        const uint64_t l = be16s(w, b + i + 2);
        if (i + 4 + l > len) return KX_ERR_UNKNOWN_PROTOCOL;
        i += 4 + l;
      }
    } else if (id == 0x11) {  // ACL token
      if (i + 2 > len) return KX_ERR_UNKNOWN_PROTOCOL;
      const uint64_t l = be16s(w, b + i);
      if (i + 2 + l > len) return KX_ERR_UNKNOWN_PROTOCOL;
      i += 2 + l;
    } else {
      rc = KX_ERR_UNKNOWN_PROTOCOL;
    }
    if (rc) return rc;
  }
  return KX_OK;
}

__device__ __forceinline__ int frame_one(const Src& w, uint64_t pos, uint64_t lim, uint64_t maxp, uint64_t* end,
                                         uint64_t& ps, uint64_t& pe, uint32_t& kind) {
  if (pos > lim || lim - pos < 8) return KX_ERR_EOF;
  const uint64_t len = lim - pos;
  const uint32_t a = be32(w, pos), c = be32(w, pos + 4);
  uint64_t p = 0, fend = 0, plen = 0;
  bool tth = false, mesh = false;
  if ((c & 0xffff0000u) == 0x10000000u) {  // IsTTHeader
    tth = true;
    if (len < 14) return KX_ERR_EOF;
    const uint64_t hs = (uint64_t)be16s(w, pos + 12) * 4;
    if (hs > 65536 || hs < 2) return KX_ERR_UNKNOWN_PROTOCOL;
    if (14 + hs > len) return KX_ERR_EOF;
    const int rc = fr_tth_info(w, pos + 14, hs);
    if (rc) return rc;
    fend = 4 + (uint64_t)a;
    if (fend < 14 + hs) return KX_ERR_UNKNOWN_PROTOCOL;
    p = 14 + hs;
    plen = fend - p;
  } else if ((a & 0xffff0000u) == 0xFFAF0000u) {  // isMeshHeader
    mesh = true;
    const uint64_t hl = a & 0xffffu;
    if (4 + hl > len) return KX_ERR_EOF;
    uint64_t i = 0;
    const int rc = fr_kv_strings(w, pos + 4, hl, i);
    if (rc) return rc;
    p = 4 + hl;
  }
  const uint64_t avail = tth ? fend : len;
  if (tth && fend > len) return KX_ERR_EOF;
  if (p + 8 > avail) return KX_ERR_EOF;
  const uint32_t x = be32(w, pos + p), y = be32(w, pos + p + 4);
  uint32_t k;
  if ((x & 0xffff0000u) == 0x80010000u) {  // isThriftBinary: TTHeader / PurePayload
    k = tth ? 2u : 0u;
    if (tth) {
      ps = p; pe = fend;
    } else {  // the message delimits itself: strict MessageBegin + the struct after it
      const int32_t nl = (int32_t)be32(w, pos + p + 4);
      if (nl < 0) return KX_ERR_NEGATIVE_SIZE;
      if (len - p < 12 + (uint64_t)nl) return KX_ERR_EOF;
      uint64_t q = pos + p + 12 + (uint64_t)nl;
      const int rc = dskip_body<false>(w, q, lim, KX_T_STRUCT, 64);
      if (rc) return rc;
      ps = p; pe = q - pos;
      fend = pe;
      plen = 0;  // unknown when checkPayloadSize runs
    }
  } else if ((y & 0xffff0000u) == 0x80010000u || (y & 0xffff0000u) == 0x90010000u) {  // Framed
    k = (tth ? 6u : 4u) | ((y & 0xffff0000u) == 0x90010000u ? 0x10u : 0u);
    plen = x;
    if (tth) {
      if (p + 4 + plen > fend) return KX_ERR_EOF;
    } else {
      fend = p + 4 + plen;
      if (fend > len) return KX_ERR_EOF;
    }
    ps = p + 4; pe = p + 4 + plen;
  } else {
    return KX_ERR_UNKNOWN_PROTOCOL;  // invalid payload (default_codec.go:411-416)
  }
  if (maxp && plen > maxp) return KX_ERR_INVALID_DATA;  // checkPayloadSize
  *end = pos + fend;
  ps += pos; pe += pos;
  kind = k | (mesh ? 0x20u : 0u);
  return KX_OK;
}

// gRPC message (decodeGRPCFrame, pkg/remote/codec/grpc/grpc_compress.go:37-60): u8 compressed flag,
// u32 BE length, payload. kind = the flag byte (1 = compressed; the reference treats every other value as
// uncompressed). A payload over maxp (> 0) is INVALID_DATA.
__device__ __forceinline__ int frame_grpc(const Src& w, uint64_t pos, uint64_t lim, uint64_t maxp, uint64_t* end,
                                          uint64_t& ps, uint64_t& pe, uint32_t& kind) {
  if (pos > lim || lim - pos < 5) return KX_ERR_EOF;  // in.Next(5)
  const uint64_t len = ((uint64_t)ld1(w, pos + 1) << 24) | ((uint64_t)ld1(w, pos + 2) << 16) |
                       ((uint64_t)ld1(w, pos + 3) << 8) | ld1(w, pos + 4);
  if (len > lim - pos - 5) return KX_ERR_EOF;  // in.Next(dLen)
  if (maxp && len > maxp) return KX_ERR_INVALID_DATA;
  kind = ld1(w, pos);
  ps = pos + 5;
  pe = pos + 5 + len;
  *end = pe;
  return KX_OK;
}

// Kitex-Protobuf Batch frame (`message Batch { repeated Rec recs = 1; }`): 0x0A, uvarint body length,
// body; payload = the body (the nested proto walker's record extent)
__device__ __forceinline__ int frame_pbb(const Src& w, uint64_t pos, uint64_t lim, uint64_t* end, uint64_t& ps,
                                         uint64_t& pe, uint32_t& kind) {
  if (pos >= lim) return KX_ERR_EOF;
  if (ld1(w, pos) != 0x0Au) return KX_ERR_INVALID_DATA;
  uint64_t l;
  uint32_t u;
  const int rc = pb_varint(w, pos + 1, lim - pos - 1, l, u);
  if (rc) return rc;
  if (l > lim - pos - 1 - u) return KX_ERR_EOF;
  kind = 0;
  ps = pos + 1 + u;
  pe = ps + l;
  *end = pe;
  return KX_OK;
}

// ttstream DecodeFrame (pkg/remote/trans/ttstream/frame.go:137-185): a TTHeader whose payload is a bare
// struct. kind = the frame type (KX_TTS_*, from IntInfo[frame type key]); *sid the TTHeader seqid, *mp /
// *ml IntInfo[ToMethod] (input position, 0 / 0 when absent); the last occurrence of a key wins. Same
// restatement as oracle kxo_ttstream_frame_one.
__device__ __forceinline__ int frame_tts(KParams& dp, const Src& w, uint64_t pos, uint64_t lim, uint64_t* end,
                                         uint64_t& ps, uint64_t& pe, uint32_t& kind, int32_t& sid, uint64_t& mp,
                                         uint32_t& ml) {
  if (pos > lim || lim - pos < 8) return KX_ERR_EOF;
  const uint64_t len = lim - pos;
  const uint32_t a = be32(w, pos), c = be32(w, pos + 4);
  if ((c & 0xffff0000u) != 0x10000000u) return KX_ERR_UNKNOWN_PROTOCOL;
  if (len < 14) return KX_ERR_EOF;
  const uint64_t hs = (uint64_t)be16s(w, pos + 12) * 4;
  if (hs > 65536 || hs < 2) return KX_ERR_UNKNOWN_PROTOCOL;
  if (14 + hs > len) return KX_ERR_EOF;
  const uint64_t b = pos + 14;
  const uint32_t proto = ld1(w, b);
  if (proto != 0 && proto != 3 && proto != 4 && proto != 0x10 && proto != 0x11) return KX_ERR_UNKNOWN_PROTOCOL;
  const uint64_t nt = ld1(w, b + 1);
  if (hs - 2 < nt) return KX_ERR_UNKNOWN_PROTOCOL;
  uint64_t i = 2 + nt, ftp = 0, ftl = ~0ull;
  mp = 0;
  ml = 0;
  const uint32_t ftk = dp.tts_keys & 0xffffu, tmk = dp.tts_keys >> 16;
  while (i < hs) {
    const uint32_t id = ld1(w, b + i++);
    if (id == 0x00) continue;
    if (id == 0x01) {
      const int rc = fr_kv_strings(w, b, hs, i);
      if (rc) return rc;
    } else if (id == 0x10) {
      if (i + 2 > hs) return KX_ERR_UNKNOWN_PROTOCOL;
      const uint32_t k = be16s(w, b + i);
      i += 2;
      for (uint32_t j = 0; j < k; j++) {
        if (i + 4 > hs) return KX_ERR_UNKNOWN_PROTOCOL;
        const uint32_t key = be16s(w, b + i);
        const uint64_t l = be16s(w, b + i + 2);
        if (i + 4 + l > hs) return KX_ERR_UNKNOWN_PROTOCOL;
        if (key == ftk) { ftp = b + i + 4; ftl = l; }
        if (key == tmk) { mp = b + i + 4; ml = (uint32_t)l; }
        i += 4 + l;
      }
    } else if (id == 0x11) {
      if (i + 2 > hs) return KX_ERR_UNKNOWN_PROTOCOL;
      const uint64_t l = be16s(w, b + i);
      if (i + 2 + l > hs) return KX_ERR_UNKNOWN_PROTOCOL;
      i += 2 + l;
    } else {
      return KX_ERR_UNKNOWN_PROTOCOL;
    }
  }
  const uint64_t fend = 4 + (uint64_t)a;
  if (fend < 14 + hs) return KX_ERR_UNKNOWN_PROTOCOL;
  if (!(c & 0xffffu & dp.tts_flag)) return KX_ERR_INVALID_DATA;  // unexpected header flags
  kind = 0;
  if (ftl <= 8) {
    uint64_t v = 0;
    for (uint64_t j = 0; j < ftl; j++) v |= (uint64_t)ld1(w, ftp + j) << (8 * j);
    for (int k = 0; k < 5; k++)
      if (!kind && dp.tts_nlen[k] == ftl && dp.tts_name[k] == v) kind = (uint32_t)(k + 1);
  }
  if (!kind) return KX_ERR_INVALID_DATA;  // unexpected frame type
  if (fend > len) return KX_ERR_EOF;
  sid = (int32_t)be32(w, pos + 8);
  ps = pos + 14 + hs;
  pe = pos + fend;
  *end = pos + fend;
  if (!ml) mp = 0;
  return KX_OK;
}

// One record: FastRead (emit) or its length / var extents only (measure).
template <int NV, int MODE>
__device__ __forceinline__ int parse_record(KParams& dp, const Src& w, uint64_t pos, uint64_t lim, uint64_t r,
                                            bool emit, uint64_t* end, VarState<NV>& vs, uint64_t& pres,
                                            bool canon_only = false) {
#pragma unroll
  for (int v = 0; v < NV; v++) { vs.len[v] = 0; vs.pos[v] = 0; }
  pres = 0;
  if (is_thrift(MODE)) {
    if (w.nsteps && canon_record<NV>(w, dp.cols, pos, lim, r, emit, end, vs)) {
      pres = w.canon_pres;
      return KX_OK;
    }
    if (canon_only) return KX_ERR_INVALID_DATA;
    return generic_record<NV, MODE == M_THRIFT_LS>(w, dp.prog, dp.cols, pos, lim, r, emit, end, vs, pres);
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
    const bool utf8 = !emit || dp.offsets != nullptr;
    if (dp.prog->npbsteps && pb_canon<NV>(w, dp.prog, dp.cols, b, e, r, emit, utf8, vs, pres)) return KX_OK;
    return pb_body<NV>(w, dp.prog, dp.cols, b, e, r, emit, vs, pres, utf8);
  }
  if (is_frame(MODE)) {
    uint64_t ps, pe, mp = 0;
    uint32_t kind, ml = 0;
    int32_t sid = 0;
    const int rc = MODE == M_PBB ? frame_pbb(w, pos, lim, end, ps, pe, kind)
                   : dp.fr_grpc == 2 ? frame_tts(dp, w, pos, lim, end, ps, pe, kind, sid, mp, ml)
                   : dp.fr_grpc ? frame_grpc(w, pos, lim, dp.fr_max, end, ps, pe, kind)
                                : frame_one(w, pos, lim, dp.fr_max, end, ps, pe, kind);
    if (emit && !rc) {
      dp.fr_ps[r] = ps;
      dp.fr_pe[r] = pe;
      if (dp.fr_kind) dp.fr_kind[r] = (uint8_t)kind;
      if (dp.fr_sid) dp.fr_sid[r] = sid;
      if (dp.fr_mpos) dp.fr_mpos[r] = mp;
      if (dp.fr_mlen) dp.fr_mlen[r] = ml;
    }
    return rc;
  }
  uint64_t p2 = pos;
  const int rc = dskip_body(w, p2, lim, KX_T_STRUCT, 64);
  *end = p2;
  return rc;
}

struct Agg {
  uint64_t ent, ex, cnt, errc, errp;
  uint64_t var[KXP_NV_MAX];
};

// Record signature taken from the data: the first record's first 3 bytes. The schema's canonical
// signature (encoder-first field header) is used when the batch's first record starts with it;
// otherwise (an IDL-order producer, an unset optional first field, the schema-less skip decoder) the
// first record's own header is: records of one batch normally start alike.
__device__ __forceinline__ uint32_t data_sig(KParams& dp) {
  if (dp.in_len < 3 || dp.offsets) return 0;
  const GLB uint8_t* p = (const GLB uint8_t*)dp.in;
  return __builtin_amdgcn_readfirstlane((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16));
}

// data_sig by one scalar load (uniform; inputs of 4 bytes and more, whose buffer holds the dword)
__device__ __forceinline__ uint32_t data_sig_s(KParams& dp) {
  if (dp.in_len < 4 || dp.offsets) return data_sig(dp);
  return *(const KAS uint32_t*)dp.in & 0xffffffu;
}

// A second data-derived signature for batches without the schema's own one (the skip decoder; producers
// whose records start with another field): the header that follows the batch's first record's leading
// fixed-size fields (up to three), at its offset. Records that start alike share it; a nested struct
// whose first fields coincide with the record's usually does not (Kitex's encoder writes a Nesting
// record's double, i32 and i64 first, the way its Simple elements start: before this, every Simple
// element was a candidate record start, and 1 M re-encoded Nesting records sent the chain pass into
// serial repair for minutes). s2o = 0: none.
__device__ __forceinline__ void data_sig2(KParams& dp, uint32_t& s2o, uint32_t& s2) {
  s2o = 0;
  s2 = 0;
  if (dp.offsets) return;
  const GLB uint8_t* p = (const GLB uint8_t*)dp.in;
  uint64_t pos = 0;
  for (int k = 0; k < 3; k++) {
    if (pos + 3 > dp.in_len) break;
    const int sz = tsize(p[pos]);
    if (sz <= 0) break;
    pos += 3 + (uint64_t)sz;
    if (pos + 3 > dp.in_len || p[pos] == KX_T_STOP || pos > 256) break;
    s2o = (uint32_t)pos;
    s2 = (uint32_t)p[pos] | ((uint32_t)p[pos + 1] << 8) | ((uint32_t)p[pos + 2] << 16);
  }
  s2o = __builtin_amdgcn_readfirstlane(s2o);
  s2 = __builtin_amdgcn_readfirstlane(s2);
}

// The lane's speculation: its segment's boundary signature, and the first signature hit. A hit is
// a guess; a guess whose own walk fails is replaced by the next hit (walk_tile), so payload bytes
// that contain the signature (binary strings saturated with it, strings holding serialized records)
// cost extra walks of the lanes they fall in, never the serial chain repair.
struct Cand {
  uint64_t ent;     // first hit (X_NONE: none)
  uint64_t plim;    // hits are < plim
  uint32_t sig, smask;
  uint32_t s2o, s2; // canonical second-header pre-check for later hits (s2o = 0: none)
  bool strict;      // several hits in the segment: a guess must parse as a canonical record
};

// M_FRAME candidates: positions that start a frame of the batch's first frame's class (batches from
// one connection are homogeneous; frames of another class are still reached by the chain walk)
__device__ __forceinline__ uint64_t frame_scan_segment(KParams& dp, const Src& w, uint64_t lo, uint64_t hi) {
  const GLB uint8_t* g = (const GLB uint8_t*)dp.in;
  if (dp.fr_grpc == 1) {
    // gRPC: the first message's flag byte, the top byte of its length, and the first (up to) 3 bytes of
    // its payload (records of one stream start alike: the Thrift field header / proto tag)
    if (dp.in_len < 5) return lo < hi && lo == 0 ? 0 : X_NONE;
    const uint32_t f0 = __builtin_amdgcn_readfirstlane((uint32_t)g[0]);
    const uint32_t l0 = __builtin_amdgcn_readfirstlane(((uint32_t)g[1] << 24) | ((uint32_t)g[2] << 16) |
                                                       ((uint32_t)g[3] << 8) | g[4]);
    const uint32_t np = l0 < 3 ? l0 : 3u;
    const uint32_t nb = dp.in_len - 5 < np ? 0u : np;
    uint32_t sig = 0;
    for (uint32_t k = 0; k < nb; k++) sig |= (uint32_t)g[5 + k] << (8 * k);
    sig = __builtin_amdgcn_readfirstlane(sig);
    const uint64_t plim = kmin64(hi, dp.in_len - 4);
    for (uint64_t p = lo; p < plim; p++) {
      if (ld1(w, p) != f0 || ld1(w, p + 1) != (l0 >> 24)) continue;
      const uint64_t l = be32(w, p + 1);
      if (l + 5 > dp.in_len - p || (l < nb && l != l0)) continue;
      if (l >= nb) {
        uint32_t s2 = 0;
        for (uint32_t k = 0; k < nb; k++) s2 |= ld1(w, p + 5 + k) << (8 * k);
        if (s2 != sig) continue;
      }
      return p;
    }
    return X_NONE;
  }
  if (dp.in_len < 8) return lo < hi && lo == 0 ? 0 : X_NONE;
  const uint32_t a0 = __builtin_amdgcn_readfirstlane(((uint32_t)g[0] << 24) | ((uint32_t)g[1] << 16) |
                                                     ((uint32_t)g[2] << 8) | g[3]);
  const uint32_t c0 = __builtin_amdgcn_readfirstlane(((uint32_t)g[4] << 24) | ((uint32_t)g[5] << 16) |
                                                     ((uint32_t)g[6] << 8) | g[7]);
  // class: 0 length-prefixed (TTHeader / Framed: magic in bytes 4-5), 1 Mesh, 2 PurePayload
  const uint32_t cls = (c0 >> 16) == 0x1000u ? 0u : (a0 >> 16) == 0xFFAFu ? 1u : (a0 >> 16) == 0x8001u ? 2u : 0u;
  const uint32_t m0 = cls == 0 ? (c0 >> 16) : (a0 >> 16);
  const uint64_t plim = kmin64(hi, dp.in_len - 7);
  // a candidate at p: its magic word; class 0 also needs a length that fits and the frame it would be
  // followed by another of its class (or the buffer's end): two magic words a length apart, where one
  // alone occurs in payload bytes every 64 Ki positions
  auto cand = [&](uint64_t p) -> bool {
    const uint32_t a = be32(w, p);
    if (cls != 0) return (a >> 16) == m0;
    if ((be32(w, p + 4) >> 16) != m0 || (uint64_t)a + 4 > dp.in_len - p) return false;
    const uint64_t nx = p + 4 + (uint64_t)a;
    return nx == dp.in_len || (nx + 8 <= dp.in_len && (be32(w, nx + 4) >> 16) == m0);
  };
  const uint32_t mo = cls == 0 ? 4u : 0u;   // the magic's offset in a frame
  const int32_t q0 = hi - lo == SEG ? wofs(w, lo + mo, SEG + 8) : -1;
  if (q0 >= 0) {
    // the rotated, conflict-free 33-dword pass of scan_segment2 with the 2-byte magic: one bit per
    // dword holding a match, then the matches in order, each tested in full
    const LDS uint32_t* s = w.win + (q0 >> 2);
    const uint32_t sh0 = q0 & 3;
    const uint32_t B0 = (m0 >> 8) * 0x01010101u, B1 = (m0 & 0xffu) * 0x01010101u;
    const int lane = (int)(threadIdx.x & 63);
    uint64_t hb = 0;
    int idx = lane % 33;
    for (int i = 0; i < 33; i++) {
      const uint32_t x0 = s[idx], x1 = s[idx + 1];
      const uint32_t m = zero_bytes((x0 ^ B0) | (__builtin_amdgcn_alignbyte(x1, x0, 1) ^ B1));
      hb |= (uint64_t)(m != 0) << idx;
      idx = idx == 32 ? 0 : idx + 1;
    }
    while (hb) {
      const int d = __ffsll((long long)hb) - 1;
      hb &= hb - 1;
      const uint32_t x0 = s[d], x1 = s[d + 1];
      uint32_t m = zero_bytes((x0 ^ B0) | (__builtin_amdgcn_alignbyte(x1, x0, 1) ^ B1));
      while (m) {
        const uint32_t j = first_hit(m);
        m &= m - 1;
        const uint32_t off = 4u * (uint32_t)d + j;
        if (off < sh0 || off - sh0 >= (uint32_t)SEG) continue;
        const uint64_t p = lo + (off - sh0);
        if (p >= plim) return X_NONE;
        if (cand(p)) return p;
      }
    }
    return X_NONE;
  }
  for (uint64_t p = lo; p < plim; p++)
    if (cand(p)) return p;
  return X_NONE;
}

__device__ __forceinline__ uint64_t next_hit(KParams& dp, const Src& w, const Cand& cd, uint64_t p);

template <int NV, int MODE>
__device__ __forceinline__ Cand lane_candidate(KParams& dp, const Src& w, uint64_t seg_lo, uint64_t seg_hi, int lane,
                                               uint32_t dsig) {
  Cand cd;
  cd.ent = X_NONE; cd.plim = seg_lo; cd.sig = 0; cd.smask = 0xffu; cd.s2o = 0; cd.s2 = 0; cd.strict = false;
  if (seg_lo >= seg_hi) return cd;
  if (MODE == M_PB || MODE == M_PBB) {   // Kitex-PB Batch frames
    cd.ent = pb_scan_segment<MODE == M_PBB>(w, seg_lo, seg_hi, dp.in_len, lane);
    return cd;
  }
  if (MODE == M_FRAME) {
    cd.ent = frame_scan_segment(dp, w, seg_lo, seg_hi);
    return cd;
  }
  const KAS KxProgram* P = dp.prog;
  const bool dok = dsig != 0 && canon_t(dsig & 0xff) != 1;  // the first record starts with a field header
  uint32_t sig, slen;
  bool own = false;
  if (is_thrift(MODE) && P->sig_len == 3 && (!dok || dsig == P->sig)) {
    sig = P->sig; slen = 3; own = true;
  } else if (dok) {
    sig = dsig; slen = 3;
  } else if (is_thrift(MODE)) {
    sig = P->sig; slen = P->sig_len;
  } else {
    sig = KX_T_STOP; slen = 1;
  }
  const uint64_t plim = kmin64(seg_hi, dp.in_len >= slen ? dp.in_len - slen + 1 : 0ull);
  cd.plim = plim; cd.sig = sig; cd.smask = slen == 3 ? 0xffffffu : 0xffu;
  if (own && w.nsteps) { cd.s2o = P->sig2_off; cd.s2 = P->sig2; }
  const int32_t q0 = wofs(w, seg_lo, SEG + 12);
  if (slen == 3 && seg_hi - seg_lo == SEG && q0 >= 0 && own && P->sig_ambig && w.nsteps) {
    // the signature also starts a nested struct (whose walk would succeed): keep the lowest of the
    // two lowest hits that parses as a canonical record, else no candidate
    uint32_t c1, c2;
    scan_segment2(w, q0, sig, lane, c1, c2);
    VarState<NV> vs0;
    uint64_t e0;
    if (c1 < (uint32_t)SEG && seg_lo + c1 < plim &&
        canon_record<NV>(w, dp.cols, seg_lo + c1, dp.in_len, 0, false, &e0, vs0))
      cd.ent = seg_lo + c1;
    else if (c2 < (uint32_t)SEG && seg_lo + c2 < plim &&
             canon_record<NV>(w, dp.cols, seg_lo + c2, dp.in_len, 0, false, &e0, vs0))
      cd.ent = seg_lo + c2;
    cd.plim = seg_lo;  // no further hits are tried
  } else if (slen == 3 && seg_hi - seg_lo == SEG && q0 >= 0 && own && w.nsteps) {
    // a second hit means the signature also occurs inside payload bytes: a guess must then parse as a
    // canonical record (a run of fields that merely parses, e.g. a serialized record held in a
    // string, would be followed and would merge into the true chain a record late)
    uint32_t c1, c2;
    scan_segment2(w, q0, sig, lane, c1, c2);
    cd.ent = c1 < (uint32_t)SEG && seg_lo + c1 < plim ? seg_lo + c1 : X_NONE;
    cd.strict = c2 < (uint32_t)SEG;
  } else if (slen == 3 && seg_hi - seg_lo == SEG && q0 >= 0) {
    cd.ent = scan_segment(w, q0, seg_lo, plim, sig, lane);
  } else {
    for (uint64_t p = seg_lo; p < plim; p++)
      if ((ld4(w, p) & cd.smask) == sig) { cd.ent = p; break; }
  }
  // a data-derived signature of a batch that can nest structs (the skip decoder, list<S> schemas): its
  // second header too (data_sig2); a flat schema's typed walk rejects a nested struct's fields itself
  if ((MODE == M_SKIP || MODE == M_THRIFT_LS) && !own && slen == 3) {
    data_sig2(dp, cd.s2o, cd.s2);
    if (cd.s2o && cd.ent != X_NONE &&
        (cd.ent + cd.s2o + 3 > dp.in_len || (ld4(w, cd.ent + cd.s2o) & 0xffffffu) != cd.s2))
      cd.ent = next_hit(dp, w, cd, cd.ent);
  }
  return cd;
}

// the next signature hit after p (exclusive) in the lane's segment, or X_NONE
__device__ __forceinline__ uint64_t next_hit(KParams& dp, const Src& w, const Cand& cd, uint64_t p) {
  for (uint64_t q = p + 1; q < cd.plim; q++) {
    if ((ld4(w, q) & cd.smask) != cd.sig) continue;
    if (cd.s2o && (q + cd.s2o + 3 > dp.in_len || (ld4(w, q + cd.s2o) & 0xffffffu) != cd.s2)) continue;
    return q;
  }
  return X_NONE;
}

// Concatenated mode, one wave, one tile [tlo, thi) in the LDS window. Lane l owns the 128-byte
// segment l: it starts at the first canonical record signature in its segment (or where the chain
// of the lane below enters it) and walks records until it leaves the segment. Lanes re-walk until
// the chain is consistent (`seed` = the tile's true entry when known, else the lowest lane's
// candidate is trusted). The record starts of the tile are written to `starts` (u16, relative to
// tlo). Returns the tile aggregate (uniform).
template <int NV, int MODE>
__device__ Agg walk_tile(KParams& dp, const Src& w, uint64_t tlo, uint64_t thi, uint64_t seed, int lane,
                         uint16_t* starts, uint32_t dsig) {
  // (skipping the plan attempt here for batches that do not start on it, as the emit pass does, tipped the
  // general index kernel from 128 to 232 VGPRs: the known-offsets decode's index pass went 0.6 -> 1.5 ms)
  const uint64_t seg_lo = tlo + (uint64_t)lane * SEG;
  const uint64_t seg_hi = kmin64(seg_lo + SEG, thi);
  const Cand cd = lane_candidate<NV, MODE>(dp, w, seg_lo, seg_hi, lane, dsig);
  uint64_t ent = cd.ent;
  if (dp.diag & 512) {  // diagnostics: DMA + candidate scan only
    Agg a;
    a.ent = __ballot(ent != X_NONE) ? ent : X_NONE; a.ex = thi; a.cnt = 0; a.errc = 0; a.errp = 0;
    for (int v = 0; v < NV; v++) a.var[v] = 0;
    return a;
  }
  uint64_t tp = (dp.diag & 64) ? __builtin_amdgcn_s_memtime() : 0;
  auto phase = [&](int k) {
    if (dp.diag & 64) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      if (lane == 0) atomicAdd(&dp.phase[k], (unsigned long long)(now - tp));
      tp = now;
    }
  };
  phase(1);
  uint64_t ex = X_NONE, cnt = 0, errp = 0;
  int errc = 0;
  uint64_t vsum[NV > 0 ? NV : 1];
#pragma unroll
  for (int v = 0; v < (NV > 0 ? NV : 1); v++) vsum[v] = 0;
  uint64_t st0 = 0, st1 = 0, st2 = 0, st3 = 0;  // the lane's first record starts
  bool need = ent != X_NONE;
  int rounds = 0;
  bool enumerate = false;   // second pass: lanes with > 4 records write the rest of their starts
  uint64_t sbase = 0;
  Agg a;
  for (;;) {
    if (need) {
      uint64_t pos = ent, c = 0;
      int e = 0;
      uint64_t acc[NV > 0 ? NV : 1];
#pragma unroll
      for (int v = 0; v < (NV > 0 ? NV : 1); v++) acc[v] = 0;
      while (pos < seg_hi && pos < dp.in_len) {
        VarState<NV> vs;
        uint64_t end = pos, pres;
        const bool strict = cd.strict && c == 0 && rounds == 0 && seed == X_NONE && !enumerate;
        const int rc = parse_record<NV, MODE>(dp, w, pos, dp.in_len, 0, false, &end, vs, pres, strict);
        if (rc) { e = rc; break; }
        if (!enumerate) {
          st0 = c == 0 ? pos : st0; st1 = c == 1 ? pos : st1;
          st2 = c == 2 ? pos : st2; st3 = c == 3 ? pos : st3;
        } else if (c >= 4 && sbase + c < dp.slotcap) {
          starts[sbase + c] = (uint16_t)(pos - tlo);
        }
        c++;
#pragma unroll
        for (int v = 0; v < NV; v++) acc[v] += vs.len[v];
        pos = end;
      }
      ex = e ? X_ERR : pos;
      cnt = c;
      errc = e;
      errp = pos;
#pragma unroll
      for (int v = 0; v < NV; v++) vsum[v] = acc[v];
    }
    need = false;
    if (enumerate) break;
    if (rounds == 0 && seed == X_NONE && ent != X_NONE && ex == X_ERR) {
      // speculating: a candidate whose own walk fails was a false signature hit, not the chain's end;
      // the lane tries its next hit (or has no candidate)
      ent = next_hit(dp, w, cd, ent);
      need = ent != X_NONE;
      ex = X_NONE; cnt = 0; errc = 0;
#pragma unroll
      for (int v = 0; v < NV; v++) vsum[v] = 0;
    }
    if (__ballot(need)) continue;  // uniform: lanes re-walk their next hit before the repair round
    phase(2);

    // ---- one repair round: every lane must start at the first true record start in its segment,
    //      i.e. where the chain of the nearest lower walking lane (or `seed`) enters it ----
    const uint64_t hm = __ballot(ent != X_NONE);
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
    if (__ballot(ch)) {
      if (++rounds <= 70) {  // from a fixed lowest entry the chain settles in <= 65 rounds
        if (ch) {
          ent = want;
          need = ent != X_NONE;
          ex = X_NONE; cnt = 0; errc = 0;
#pragma unroll
          for (int v = 0; v < NV; v++) vsum[v] = 0;
        }
        continue;
      }
      if (lane == 0) atomicCAS((int*)&dp.status->code, 0, KX_ERR_INTERNAL);
    }

    // ---- converged: the tile aggregate ----
    const uint64_t em = __ballot(ent != X_NONE && ex == X_ERR);
    const int fel = em ? __ffsll((long long)em) - 1 : 64;
    const bool live = ent != X_NONE && lane <= fel;
    const uint64_t c0 = live ? cnt : 0;
    const uint64_t inc = wave_incl_scan(c0, lane);
    const uint64_t cpre = inc - c0;
    a.cnt = rl64(inc, 63);
#pragma unroll
    for (int v = 0; v < NV; v++) a.var[v] = wave_sum(live ? vsum[v] : 0);
    a.ent = hm ? rl64(ent, __ffsll((long long)hm) - 1) : X_NONE;
    a.ex = fel < 64 ? X_ERR : hm ? rl64(ex, 63 - __clzll((long long)hm)) : seed;
    a.errc = fel < 64 ? (uint64_t)__builtin_amdgcn_readlane(errc, fel) : 0;
    a.errp = fel < 64 ? rl64(errp, fel) : 0;
    phase(3);
    if (live) {  // slots past slotcap are not kept (emit_tile follows the chain past them)
      const uint64_t b = cpre, sc = dp.slotcap;
      if (cnt > 0 && b + 0 < sc) starts[b + 0] = (uint16_t)(st0 - tlo);
      if (cnt > 1 && b + 1 < sc) starts[b + 1] = (uint16_t)(st1 - tlo);
      if (cnt > 2 && b + 2 < sc) starts[b + 2] = (uint16_t)(st2 - tlo);
      if (cnt > 3 && b + 3 < sc) starts[b + 3] = (uint16_t)(st3 - tlo);
    }
    if (__ballot(live && cnt > 4 && cpre + 4 < dp.slotcap)) {
      enumerate = true;
      need = live && cnt > 4 && cpre + 4 < dp.slotcap;
      sbase = cpre;
      continue;
    }
    break;
  }
  phase(4);
  return a;
}

// ---------------------------------------------------------------------------------------------
// Fast index path (concatenated Thrift, batches whose records start with the schema's canonical
// signature): the same tile aggregate and record starts as walk_tile, for tiles whose records are all
// canonical and whose speculation is right the first time, at a fraction of the instructions:
//  * segments on the window's dword grid (segment s = window dwords D0 + 32 s .. + 31, the last one
//    runs to the tile end); the signature scan is interleaved (iteration k: lane l tests dword
//    D0 + 64 k + l) and a ballot per iteration hands segment 2k / 2k + 1 its dword-hit mask
//    (a select per lane), so every LDS read is conflict-free and no lane loops over its own bytes;
//  * a lane walks from its first hit (its second one when the first does not parse canonically: a
//    nested struct with the same first header) with `fast_record`: the canonical plan's headers and
//    lengths only, one window bounds check per step;
//  * one consistency check (every lane's entry = the exit of the walking lane below it). Anything
//    else (a non-canonical record, a false signature hit, a record leaving the window, > 4 records in
//    a segment) returns false and the tile takes walk_tile from scratch.
// ---------------------------------------------------------------------------------------------
// iteration K of the interleaved signature scan: lane l tests window dword D0 + 64 K + l; the ballot's
// halves are the dword-hit masks of segments 2K and 2K + 1, picked up by those lanes (kk = lane / 2,
// sh = 32 * (lane % 2)). (v_writelane would save an instruction, but from inline assembly the compiler
// cannot see its SGPR read-after-VALU-write hazard.)
template <int K>
__device__ __forceinline__ void fast_scan(const Src& w, uint32_t D0, uint32_t b0, uint32_t b1, uint32_t b2, int lane,
                                          uint32_t kk, uint32_t sh, uint32_t& hm) {
  const uint32_t d = D0 + 64u * K + (uint32_t)lane;
  const uint32_t x0 = w.win[d], x1 = w.win[d + 1];
  const uint32_t e = (x0 ^ b0) | (__builtin_amdgcn_alignbyte(x1, x0, 1) ^ b1) |
                     (__builtin_amdgcn_alignbyte(x1, x0, 2) ^ b2);
  const uint64_t bal = __ballot(low_zero_byte(e) != 0);
  hm = kk == (uint32_t)K ? (uint32_t)(bal >> sh) : hm;
  if constexpr (K + 1 < 32) fast_scan<K + 1>(w, D0, b0, b1, b2, lane, kk, sh, hm);
}

__device__ __forceinline__ uint32_t win_ld(const Src& w, uint32_t q) {  // 4 bytes at window offset q
  return __builtin_amdgcn_alignbyte(w.win[(q >> 2) + 1], w.win[q >> 2], q & 3);
}

// one canonical record at window offset q from the segment plan: the header checks of a segment are
// independent LDS reads, so a record costs one LDS round trip per var field (its length moves the next
// segment) instead of a scalar-load chain per step
template <int NV>
__device__ __forceinline__ bool fast_record_fp(KParams& dp, const Src& w, uint32_t& q, uint64_t* vl) {
  const uint32_t wl = (uint32_t)w.wlen;
  bool ok = true;
  // the plan is re-read per record (a handful of independent scalar loads): hoisted out of the walk it
  // would hold ~100 SGPRs for the whole kernel
  uint32_t z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));   // an opaque 0: the loads below stay in the loop
  const KAS KxpFast* fp = (const KAS KxpFast*)((const KAS char*)&dp.fp + z);
  const uint32_t nseg = fp->nseg;
#pragma unroll
  for (int s = 0; s < KXF_SEG; s++) {
    if (s >= (int)nseg) break;
    const KAS KxpFastSeg& G = fp->seg[s];
    ok &= q + G.flen + 16 <= wl;            // the run, the var header and length stay in the window
    const uint32_t qq = ok ? q : 0u;
    const uint32_t ng = G.nchk;
#pragma unroll
    for (int g = 0; g < KXF_CHK; g += 4) {  // groups of 4 independent checks: one LDS round trip each group
      if (g >= (int)ng) break;
#pragma unroll
      for (int c = g; c < g + 4; c++) {
        const uint32_t cv = G.chval[c];
        const uint32_t m = (cv >> 31) ? 0xffu : ((cv >> 30) & 1u) ? 0u : 0xffffffu;
        ok &= ((win_ld(w, qq + G.choff[c]) ^ cv) & m) == 0;
      }
    }
    uint32_t q2 = qq + G.flen;
    if (G.vkind) {
      const bool list = G.vkind == 2;
      ok &= ((win_ld(w, q2) ^ G.vhdr) & 0xffffffu) == 0;
      const uint32_t l = __builtin_bswap32(win_ld(w, q2 + (list ? 4u : 3u)));
      const uint64_t b = (uint64_t)l * (list ? G.vwidth : 1u);
      ok &= l <= wl && b <= wl;             // also rejects a negative length (the generic path reports it)
#pragma unroll
      for (int v = 0; v < NV; v++)
        if ((uint32_t)v == G.vslot) vl[v] += ok ? l : 0u;
      q2 += (list ? 8u : 7u) + (ok ? (uint32_t)b : 0u);
    }
    q = q2;
  }
  return ok;
}

// After fast_record failed on the record at window offset q: did it fail only because the record runs on
// past the window (every header up to there matches the plan)? A canonical record longer than the window
// (a 64 KiB string) is then a record start the fast path cannot walk, not a false signature hit: its tile
// takes the general walk instead of reading as one with no record start (such a tile
// used to send its whole group to the chain pass's repair). Off the hot path: failing lanes only.
__device__ __forceinline__ bool record_leaves_window(const Src& w, uint32_t q) {
  const KAS KxpStep* __restrict__ steps = w.steps;
  const uint32_t wl = (uint32_t)w.wlen;
  for (uint32_t k = 0; k < w.nsteps; k++) {
    const KxpStep st = ldk(&steps[k]);
    if (q + 64 > wl) return true;
    const uint32_t h = win_ld(w, q);
    if (st.kind == KXP_S_END) return false;
    if ((h ^ st.hdr) & 0xffffffu) return false;
    if (st.kind == KXP_S_FIXED) { q += 3 + st.width; continue; }
    if (st.kind == KXP_S_STRUCT) { q += 3; continue; }
    const bool list = st.kind == KXP_S_LIST;
    const uint32_t l = __builtin_bswap32(win_ld(w, q + (list ? 4u : 3u)));
    if (l > 0x7fffffffu) return false;
    const uint64_t b = (uint64_t)l * (list ? st.width : 1u);
    if ((uint64_t)q + (list ? 8u : 7u) + b + 64 > wl) return true;
    q += (list ? 8u : 7u) + (uint32_t)b;
  }
  return false;
}

// one canonical record at window offset q (measure: headers, lengths, STOP); var lengths added to vl
template <int NV>
__device__ __forceinline__ bool fast_record(KParams& dp, const Src& w, uint32_t& q, uint64_t* vl) {
#ifdef KX_FASTPLAN
  if (dp.fp.ok) return fast_record_fp<NV>(dp, w, q, vl);
#endif
  const KAS KxpStep* __restrict__ steps = w.steps;
  const uint32_t wl = (uint32_t)w.wlen;
  bool ok = true;
  uint32_t k = 0;
  while (k < w.nsteps) {
    k = __builtin_amdgcn_readfirstlane(k);
    // steps k .. k + 3 in one scalar load (the table has room past the plan's end): a FIXED run's
    // headers do not wait for a second load that depends on the run length
#ifdef KX_STEP4
    struct Q4 { KxpStep s[4]; };
    const Q4 st4 = ldk((const KAS Q4*)&steps[k < KXP_MAX_STEPS - 3 ? k : KXP_MAX_STEPS - 4]);
    const uint32_t kb = k < KXP_MAX_STEPS - 3 ? 0u : k - (KXP_MAX_STEPS - 4);
    const KxpStep st = st4.s[kb];
#else
    const KxpStep st = ldk(&steps[k]);
#endif
    ok &= q + 64 <= wl;             // a step reads < 64 bytes from q
    const uint32_t qq = ok ? q : 0u;
    if (st.kind == KXP_S_FIXED) {
      const uint32_t m = min(st.hdr >> 24, 4u);
#ifdef KX_STEP4
      // a run of m > 1 FIXED steps starts at k <= nsteps - m, so kb == 0 whenever s1.. are used
      const KxpStep s1 = st4.s[m > 1 ? 1 : 0];
      const KxpStep s2 = st4.s[m > 2 ? 2 : 0];
      const KxpStep s3 = st4.s[m > 3 ? 3 : 0];
#else
      const KxpStep s1 = ldk(&steps[k + (m > 1 ? 1 : 0)]);
      const KxpStep s2 = ldk(&steps[k + (m > 2 ? 2 : 0)]);
      const KxpStep s3 = ldk(&steps[k + (m > 3 ? 3 : 0)]);
#endif
      const uint32_t o1 = 3 + st.width, o2 = o1 + 3 + s1.width, o3 = o2 + 3 + s2.width;
      const uint32_t len = m == 1 ? o1 : m == 2 ? o2 : m == 3 ? o3 : o3 + 3 + s3.width;
      ok &= ((win_ld(w, qq) ^ st.hdr) & 0xffffffu) == 0;
      if (m > 1) ok &= ((win_ld(w, qq + o1) ^ s1.hdr) & 0xffffffu) == 0;
      if (m > 2) ok &= ((win_ld(w, qq + o2) ^ s2.hdr) & 0xffffffu) == 0;
      if (m > 3) ok &= ((win_ld(w, qq + o3) ^ s3.hdr) & 0xffffffu) == 0;
      q += len;
      k += m;
      continue;
    }
    k++;
    const uint32_t h = win_ld(w, qq);
    if (st.kind == KXP_S_END) {
      ok &= (h & 0xffu) == KX_T_STOP;
      q += 1;
      continue;
    }
    ok &= ((h ^ st.hdr) & 0xffffffu) == 0;
    if (st.kind == KXP_S_STRUCT) {
      q += 3;
      continue;
    }
    const bool list = st.kind == KXP_S_LIST;
    const uint32_t l = __builtin_bswap32(win_ld(w, qq + (list ? 4u : 3u)));
    const uint64_t b = (uint64_t)l * (list ? st.width : 1u);
    ok &= l <= wl && b <= wl;       // also rejects a negative length (the generic path reports it)
#pragma unroll
    for (int v = 0; v < NV; v++)
      if ((uint32_t)v == st.vslot) vl[v] += ok ? l : 0u;
    q += (list ? 8u : 7u) + (ok ? (uint32_t)b : 0u);
  }
  return ok;
}

template <int NV>
__device__ __forceinline__ bool fast_tile(KParams& dp, const Src& w, uint64_t tlo, uint64_t thi, uint64_t seed,
                                          int lane, uint16_t* starts, Agg& a) {
  const KAS KxProgram* P = dp.prog;
  const uint32_t sig = P->sig;
  const uint32_t b0 = (sig & 0xff) * 0x01010101u, b1 = ((sig >> 8) & 0xff) * 0x01010101u;
  const uint32_t b2 = ((sig >> 16) & 0xff) * 0x01010101u;
  const uint32_t q0 = (uint32_t)(tlo - w.wpos);   // < 16
  const uint32_t D0 = q0 >> 2;
  // ---- interleaved scan: hm = the dword-hit mask of this lane's segment ----
  uint64_t tp = (dp.diag & 64) ? __builtin_amdgcn_s_memtime() : 0;
  auto phase = [&](int k) {   // diagnostics (KX_DIAG & 64): cycles per phase, summed over tiles
    if (dp.diag & 64) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      if (lane == 0) atomicAdd(&dp.phase[k], (unsigned long long)(now - tp));
      tp = now;
    }
  };
  uint32_t hm = 0;
  fast_scan<0>(w, D0, b0, b1, b2, lane, (uint32_t)lane >> 1, 32u * ((uint32_t)lane & 1u), hm);
  phase(1);
  // diagnostics (timing only, output wrong): stop after a phase, keeping its result live
  auto stop_here = [&](uint64_t live) {
    a.ent = tlo; a.ex = thi; a.cnt = __ballot(live != 0) & 1; a.errc = T_CANON; a.errp = 0;
    for (int v = 0; v < NV; v++) a.var[v] = 0;
  };
  if (dp.diag & 1024) { stop_here(hm); return true; }
  const uint32_t sq = 4 * D0 + 128u * (uint32_t)lane;   // window offset of the segment's first dword
  const uint64_t seg_lo = lane == 0 ? tlo : w.wpos + sq;
  const uint64_t seg_hi = lane == 63 ? thi : kmin64(w.wpos + sq + 128, thi);
  const uint64_t plim = kmin64(seg_hi, dp.in_len >= 3 ? dp.in_len - 2 : 0ull);
  // ---- the first two hits in [seg_lo, plim) (lane 63 also tests dword 32: the up to 3 bytes of the
  //      tile past the dword grid) ----
  uint64_t c1 = X_NONE, c2 = X_NONE, c3 = X_NONE;
  {
    // a hit whose second field header (at the plan's fixed offset) does not match is not a candidate:
    // payload bytes saturated with the signature cost a few compares instead of failed walks
    const uint32_t s2o = P->sig2_off, s2 = P->sig2;
    uint64_t hb = (uint64_t)hm | (lane == 63 ? (1ull << 32) : 0ull);   // lane 63 also looks at dword 32
    while (hb && c3 == X_NONE) {
      const int di = __ffsll((long long)hb) - 1;
      hb &= hb - 1;
      const uint32_t dq = sq + 4u * (uint32_t)di;
      const uint32_t x0 = w.win[dq >> 2], x1 = w.win[(dq >> 2) + 1];
      uint32_t m = zero_bytes((x0 ^ b0) | (__builtin_amdgcn_alignbyte(x1, x0, 1) ^ b1) |
                              (__builtin_amdgcn_alignbyte(x1, x0, 2) ^ b2));
      while (m) {
        const uint64_t p = w.wpos + dq + first_hit(m);
        m &= m - 1;
        if (p < seg_lo || p >= plim) continue;
        const uint32_t pq = (uint32_t)(p - w.wpos) + s2o;
        if (s2o && pq + 8 <= (uint32_t)w.wlen && ((win_ld(w, pq) ^ s2) & 0xffffffu)) continue;
        if (c1 == X_NONE) c1 = p;
        else if (c2 == X_NONE) c2 = p;
        else { c3 = p; break; }
      }
    }
  }
  phase(2);
  if (dp.diag & 2048) { stop_here(c1 ^ c2 ^ c3); return true; }
  // ---- walk: records of the segment from c1, else c2, else c3: a candidate whose walk fails anywhere
  //      (not canonical, or a record nested in a payload: it parses, but the bytes after it do not) is
  //      replaced by the next; the consistency check below accepts only an unbroken chain ----
  uint64_t ent = c1, ex = X_NONE, cnt = 0, st0 = 0, st1 = 0, st2 = 0, st3 = 0;
  uint64_t vsum[NV > 0 ? NV : 1];
#pragma unroll
  for (int v = 0; v < (NV > 0 ? NV : 1); v++) vsum[v] = 0;
  bool bad = false, wf = false;   // wf: a walk met a record that runs on past the window
  for (int attempt = 0; attempt < 3; attempt++) {
    bool again = false;
    if (ent != X_NONE) {
      uint32_t q = (uint32_t)(ent - w.wpos);
      uint64_t acc[NV > 0 ? NV : 1];
#pragma unroll
      for (int v = 0; v < (NV > 0 ? NV : 1); v++) acc[v] = 0;
      uint64_t c = 0;
      bool ok = true;
      while (ok && w.wpos + q < seg_hi) {
        const uint64_t start = w.wpos + q;
        ok = fast_record<NV>(dp, w, q, acc);
        if (!ok) {
          wf |= record_leaves_window(w, (uint32_t)(start - w.wpos));
          break;
        }
        st0 = c == 0 ? start : st0; st1 = c == 1 ? start : st1;
        st2 = c == 2 ? start : st2; st3 = c == 3 ? start : st3;
        c++;
      }
      if (!ok) {
        // not a record start of a canonical chain (a nested struct's header, a false hit, a record inside
        // a binary payload): try the segment's next hit, else the lane has no candidate (the consistency
        // check below then catches a record start that is there but not canonical)
        ent = attempt == 0 ? c2 : attempt == 1 ? c3 : X_NONE;
        again = ent != X_NONE;
        if (!again) { ex = X_NONE; cnt = 0; }
      } else {
        bad = c > 4;
        ex = w.wpos + q;
        cnt = c;
#pragma unroll
        for (int v = 0; v < NV; v++) vsum[v] = acc[v];
      }
    }
    if (!__ballot(again)) break;
  }
  phase(3);
  if (dp.diag & 4096) { stop_here(ex ^ cnt ^ st0 ^ st1 ^ vsum[0]); return true; }
  if (__ballot(bad || wf)) return false;
  // ---- consistency: every walking lane starts where the chain of the walking lane below it exits ----
  const uint64_t hmk = __ballot(ent != X_NONE);
  const uint64_t below = hmk & ((1ull << lane) - 1);
  const int pc = below ? 63 - __clzll((long long)below) : -1;
  const uint64_t pex = __shfl(ex, pc < 0 ? 0 : pc, 64);
  const uint64_t E = pc >= 0 ? pex : seed;
  const bool agree = E == X_NONE || (ent != X_NONE ? E == ent : E >= seg_hi);
  if (__ballot(!agree)) return false;
  // ---- tile aggregate and record starts (as walk_tile) ----
  const uint64_t inc = wave_incl_scan(cnt, lane);
  const uint64_t cpre = inc - cnt;
  a.cnt = rl64(inc, 63);
#pragma unroll
  for (int v = 0; v < NV; v++) a.var[v] = wave_sum(vsum[v]);
  a.ent = hmk ? rl64(ent, __ffsll((long long)hmk) - 1) : X_NONE;
  a.ex = hmk ? rl64(ex, 63 - __clzll((long long)hmk)) : seed;
  a.errc = T_CANON;   // every record of the tile is canonical and inside the window: emit trusts the plan
  a.errp = 0;
  const uint64_t sc = dp.slotcap;
  if (cnt > 0 && cpre + 0 < sc) starts[cpre + 0] = (uint16_t)(st0 - tlo);
  if (cnt > 1 && cpre + 1 < sc) starts[cpre + 1] = (uint16_t)(st1 - tlo);
  if (cnt > 2 && cpre + 2 < sc) starts[cpre + 2] = (uint16_t)(st2 - tlo);
  if (cnt > 3 && cpre + 3 < sc) starts[cpre + 3] = (uint16_t)(st3 - tlo);
  phase(4);
  return true;
}

// Known-offsets mode: lane = record. Measures the var extents (failed records count as empty). A record
// that lies in the window and parses canonically is measured with fast_record (headers and lengths of
// the plan); any other takes parse_record, which also reports its error.
template <int NV, int MODE>
__device__ __forceinline__ Agg measure_records(KParams& dp, const Src& w, uint64_t r0, uint64_t r1, int lane) {
  const uint64_t r = r0 + lane;
  VarState<NV> vs;
#pragma unroll
  for (int v = 0; v < NV; v++) vs.len[v] = 0;
  bool done = false;
  if (r < r1) {
    const uint64_t a = dp.offsets[r], b = rec_end(dp, r);
    if constexpr (MODE == M_THRIFT) {
      if (dp.fast && a <= b && b <= dp.in_len && a >= w.wpos && a - w.wpos < (uint64_t)w.wlen) {
        uint64_t vl[NV > 0 ? NV : 1];
#pragma unroll
        for (int v = 0; v < (NV > 0 ? NV : 1); v++) vl[v] = 0;
        uint32_t q = (uint32_t)(a - w.wpos);
        if (fast_record<NV>(dp, w, q, vl) && w.wpos + q <= b) {
#pragma unroll
          for (int v = 0; v < NV; v++) vs.len[v] = (uint32_t)vl[v];
          done = true;
        }
      }
    }
    if (!done) {
      uint64_t end, pres;
      int rc = (a > b || b > dp.in_len) ? KX_ERR_INVALID_ARG
                                        : parse_record<NV, MODE>(dp, w, a, b, r, false, &end, vs, pres);
      if (rc) {
#pragma unroll
        for (int v = 0; v < NV; v++) vs.len[v] = 0;
      }
    }
  }
  Agg g;
  g.ent = X_NONE; g.ex = X_NONE; g.errp = 0;
  // every record of the tile measured by the plan inside the window: the emit pass reads them with the
  // plan alone (emit_canon), as for a fast-path tile of a concatenated batch
  g.errc = __ballot(r < r1 && !done) == 0 ? T_CANON : 0;
  g.cnt = r1 - r0;
#pragma unroll
  for (int v = 0; v < NV; v++) g.var[v] = wave_sum(vs.len[v]);
  return g;
}

// tile geometry
__device__ __forceinline__ void tile_range(KParams& dp, uint64_t t, uint64_t& lo, uint64_t& hi) {
  if (dp.offsets) {
    const uint64_t r0 = t * dp.krec, r1 = kmin64(r0 + dp.krec, dp.n);
    lo = r0; hi = r1;  // records
  } else {
    lo = t * (uint64_t)TILE;
    hi = kmin64(lo + TILE, dp.in_len);
  }
}

// (re)walk tile t of a concatenated batch with the wave's LDS window
template <int NV, int MODE>
__device__ Agg tile_agg(KParams& dp, LDS uint32_t* win, uint64_t t, uint64_t seed, int lane) {
  uint64_t lo, hi;
  tile_range(dp, t, lo, hi);
  if (dp.offsets) {
    const Src w = load_window(dp, win, dp.offsets[lo], lane, is_thrift(MODE));
    return measure_records<NV, MODE>(dp, w, lo, hi, lane);
  }
  const uint64_t t0 = (dp.diag & 64) ? __builtin_amdgcn_s_memtime() : 0;
  // the window DMA is issued first and the batch signature's load behind it, so both round trips overlap
  const Src w = load_window(dp, win, lo, lane, is_thrift(MODE), false);
  const uint32_t dsig = data_sig(dp);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if ((dp.diag & 64) && lane == 0) atomicAdd(&dp.phase[0], (unsigned long long)(__builtin_amdgcn_s_memtime() - t0));
  if constexpr (MODE == M_THRIFT) {
    if (dp.fast && !dp.offsets && dsig == dp.prog->sig && w.wlen >= TILE + 64) {
      Agg a;
      if (fast_tile<NV>(dp, w, lo, hi, seed, lane, dp.starts + t * dp.slotcap, a)) return a;
      if (lane == 0) atomicAdd((unsigned long long*)&dp.status->diag[2], 1ull);  // fell back to walk_tile
    }
  }
  return walk_tile<NV, MODE>(dp, w, lo, hi, seed, lane, dp.starts + t * dp.slotcap, dsig);
}

__device__ __forceinline__ void put_tile(KParams& dp, uint64_t t, const Agg& a, int nv) {
  const uint64_t ep = dp.epoch, nt = dp.ntiles;
  put_word(dp.tdesc, nt, T_ENT, t, ep, a.ent);
  put_word(dp.tdesc, nt, T_EXIT, t, ep, a.ex);
  put_word(dp.tdesc, nt, T_CNT, t, ep, a.cnt);
  put_word(dp.tdesc, nt, T_ERRC, t, ep, a.errc);
  put_word(dp.tdesc, nt, T_ERRP, t, ep, a.errp);
  for (int v = 0; v < nv; v++) put_word(dp.tdesc, nt, T_VAR + v, t, ep, a.var[v]);
}

// Does a chain arriving at `E` agree with an item whose speculative entry is `ent`? (An item with no
// record start is a pass-through: the chain must jump over it.)
__device__ __forceinline__ bool chain_ok(uint64_t E, uint64_t ent, uint64_t hi) {
  if (E == X_ERR || E == X_DONE) return true;  // the chain already ended
  if (ent == X_BAD) return false;
  return ent == X_NONE ? E >= hi : ent == E;
}

// Group scan, one wave, lane = tile of group g. Validates the speculative chain between the tiles
// (`entry` = the group's true entry when known, else X_NONE = trust the first tile that has a record
// start), then writes each tile's exclusive prefix inside the group and the group aggregate.
// REPAIR: a tile that disagrees is re-walked from its true entry; otherwise the group is marked
// X_BAD and left to the chain pass (keeps the re-walk out of the index pass's registers).
template <int NV, int MODE, bool REPAIR>
__device__ void group_scan(KParams& dp, LDS uint32_t* win, uint64_t g, uint64_t entry, int lane) {
  const uint64_t t0 = g * GT;
  const uint64_t ntg = kmin64((uint64_t)GT, dp.ntiles - t0);
  const bool act = (uint64_t)lane < ntg;
  const uint64_t t = t0 + lane;
  const uint64_t ep = dp.epoch;
  constexpr int NW = 5 + NV;
  int fields[NW];
#pragma unroll
  for (int k = 0; k < NW; k++) fields[k] = k < 5 ? k : T_VAR + (k - 5);
  uint64_t x[NW];
  if (!get_words<NW>(dp.tdesc, dp.ntiles, fields, NW, act ? t : 0, ep, act, x)) {
    if (lane == 0) atomicCAS((int*)&dp.status->code, 0, KX_ERR_INTERNAL);
    return;
  }
  uint64_t ent = act ? x[0] : X_NONE, ex = act ? x[1] : X_NONE, cnt = act ? x[2] : 0;
  uint64_t errc = act ? x[3] : 0, errp = act ? x[4] : 0;
  uint64_t var[NV > 0 ? NV : 1];
#pragma unroll
  for (int v = 0; v < NV; v++) var[v] = act ? x[5 + v] : 0;
  uint64_t lo, hi;
  tile_range(dp, act ? t : t0, lo, hi);
  if (!dp.offsets) {
    // effective exit of every tile: its own, or (pass-through) the one it inherits
    for (int guard = 0; guard < 4 * GT + 8; guard++) {
      const uint64_t hm = __ballot(act && ent != X_NONE);
      // expected entry of each tile = exit of the nearest lower tile with a record start, else `entry`
      const uint64_t below = hm & ((1ull << lane) - 1);
      const int pc = below ? 63 - __clzll((long long)below) : -1;
      const uint64_t pex = __shfl(ex, pc < 0 ? 0 : pc, 64);
      const uint64_t E = pc >= 0 ? pex : entry;
      const bool bad = act && E != X_NONE && !chain_ok(E, ent, hi);
      const uint64_t bm = __ballot(bad);
      if (!bm) break;
      if (!REPAIR) {
        if (lane == 0) {
          const uint64_t ng = dp.ngroups;
          put_word(dp.gdesc, ng, G_EXIT, g, ep, X_NONE);
          put_word(dp.gdesc, ng, G_CNT, g, ep, 0);
          put_word(dp.gdesc, ng, G_ERRC, g, ep, 0);
          put_word(dp.gdesc, ng, G_ERRP, g, ep, 0);
          for (int v = 0; v < NV; v++) put_word(dp.gdesc, ng, G_VAR + v, g, ep, 0);
          put_word(dp.gdesc, ng, G_ENT, g, ep, X_BAD);
        }
        return;
      }
      // re-walk the first disagreeing tile from its true entry
      const int b = __ffsll((long long)bm) - 1;
      const uint64_t Eb = rl64(E, b);
      if (lane == 0) atomicAdd((unsigned long long*)&dp.status->diag[0], 1ull);
      const Agg a = tile_agg<NV, MODE>(dp, win, t0 + b, Eb, lane);
      put_tile(dp, t0 + b, a, NV);
      if (lane == b) {
        ent = a.ent; ex = a.ex; cnt = a.cnt; errc = a.errc; errp = a.errp;
#pragma unroll
        for (int v = 0; v < NV; v++) var[v] = a.var[v];
      }
    }
  }
  // the chain stops at the first erroring tile
  const uint64_t em = __ballot(act && ex == X_ERR);
  const int fe = em ? __ffsll((long long)em) - 1 : 64;
  const bool live = act && lane <= fe;
  const uint64_t c0 = live ? cnt : 0;
  const uint64_t ci = wave_incl_scan(c0, lane);
  uint64_t vpre[NV > 0 ? NV : 1], vtot[NV > 0 ? NV : 1];
#pragma unroll
  for (int v = 0; v < NV; v++) {
    const uint64_t x0 = live ? var[v] : 0;
    const uint64_t vi = wave_incl_scan(x0, lane);
    vpre[v] = vi - x0;
    vtot[v] = rl64(vi, 63);
  }
  if (act) {
    put_word(dp.tdesc, dp.ntiles, T_PCNT, t, ep, ci - c0);
#pragma unroll
    for (int v = 0; v < NV; v++) put_word(dp.tdesc, dp.ntiles, T_PVAR + v, t, ep, vpre[v]);
  }
  const uint64_t hm = __ballot(act && ent != X_NONE);
  const uint64_t gent = hm ? rl64(ent, __ffsll((long long)hm) - 1) : X_NONE;
  const uint64_t gex = fe < 64 ? X_ERR : hm ? rl64(ex, 63 - __clzll((long long)hm)) : entry;
  const uint64_t gcnt = rl64(ci, 63);
  const uint64_t gerrc = fe < 64 ? rl64(errc, fe) & 0xff : 0;
  const uint64_t gerrp = fe < 64 ? rl64(errp, fe) : 0;
  if (lane == 0) {
    const uint64_t ng = dp.ngroups;
    put_word(dp.gdesc, ng, G_ENT, g, ep, gent);
    put_word(dp.gdesc, ng, G_EXIT, g, ep, gex);
    put_word(dp.gdesc, ng, G_CNT, g, ep, gcnt);
    put_word(dp.gdesc, ng, G_ERRC, g, ep, gerrc);
    put_word(dp.gdesc, ng, G_ERRP, g, ep, gerrp);
#pragma unroll
    for (int v = 0; v < NV; v++) put_word(dp.gdesc, ng, G_VAR + v, g, ep, vtot[v]);
  }
}

// ---- kernel 1: index pass (one wave per tile) ----
template <int NV, int MODE>
__device__ __forceinline__ void index_tile(KParams& dp, LDS uint32_t* win, uint64_t t, int lane) {
  const uint64_t t_start = (dp.diag & 64) ? __builtin_amdgcn_s_memtime() : 0;
  Agg a;
  if (dp.diag & 1) {
    uint64_t lo, hi;
    tile_range(dp, t, lo, hi);
    const Src w = load_window(dp, win, dp.offsets ? dp.offsets[lo] : lo, lane, is_thrift(MODE));
    a.ent = lo + (w.win[lane] & 1); a.ex = hi; a.cnt = 0; a.errc = 0; a.errp = 0;
    for (int v = 0; v < NV; v++) a.var[v] = 0;
  } else {
    a = tile_agg<NV, MODE>(dp, win, t, t == 0 ? 0ull : X_NONE, lane);
  }
  if (lane == 0 && !(dp.diag & 4)) put_tile(dp, t, a, NV);
  if ((dp.diag & 64) && lane == 0) atomicAdd(&dp.phase[5], (unsigned long long)(__builtin_amdgcn_s_memtime() - t_start));
}

template <int NV, int MODE>
__global__ void __launch_bounds__(NT, 4) index_kernel(DecParams dp_) {  // 4 waves per SIMD: <= 128 VGPRs
  KParams& dp = KX_PARAMS();
  (void)dp_;
  __shared__ __attribute__((aligned(16))) uint32_t WIN[WAVES][WINW];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const uint64_t t = dp.t_lo + (uint64_t)blockIdx.x * WAVES + wv;
  if (t >= dp.t_hi) return;
  index_tile<NV, MODE>(dp, (LDS uint32_t*)WIN[wv], t, lane);
}

// ---- kernel 1, fast form (concatenated Thrift with a canonical plan): the fast index path alone, in a
// kernel of its own so that its registers are not those of the general walk; a tile the fast path
// cannot index (a non-canonical record, a false-hit chain, a batch that starts with another signature,
// the last partial tile) is queued for redo_kernel, which walks it with the general field loop ----
// NARROW: batches whose halo is the default (dp.winb <= FWINB) take a window sized for it and 2-wave
// workgroups, so that 18 waves fit a CU's LDS instead of 16
constexpr int FWINB = TILE + HALO + 16, FWINW = FWINB / 4 + 4, FNT = 128, FWAVES = FNT / 64;
template <int NV, bool NARROW>
__global__ void __launch_bounds__(NARROW ? FNT : NT) index_fast_kernel(DecParams dp_) {
  KParams& dp = KX_PARAMS();
  (void)dp_;
  constexpr int WV = NARROW ? FWAVES : WAVES, WW = NARROW ? FWINW : WINW;
  __shared__ __attribute__((aligned(16))) uint32_t WIN[WV][WW];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const uint64_t t = dp.t_lo + (uint64_t)blockIdx.x * WV + wv;
  if (t >= dp.t_hi) return;
  // a batch whose first record does not start with the canonical signature is left to redo_kernel whole
  // (no DMA here): the batch signature is one scalar load, a scalar-cache hit for all but a CU's first wave
  if (data_sig_s(dp) != dp.prog->sig) return;
  uint64_t lo, hi;
  tile_range(dp, t, lo, hi);
  const Src w = load_window<NARROW ? FWINB : WINB>(dp, (LDS uint32_t*)WIN[wv], lo, lane, true, true);
  Agg a;
  if (w.wlen >= TILE + 64 &&
      fast_tile<NV>(dp, w, lo, hi, t == 0 ? 0ull : X_NONE, lane, dp.starts + t * dp.slotcap, a)) {
    if (lane == 0 && !(dp.diag & 4)) put_tile(dp, t, a, NV);
  } else if (lane == 0) {
    dp.redo[atomicAdd(dp.redo_n, 1u)] = (uint32_t)t;
  }
}

// one queued tile (an out-of-line call from uniform control flow: the persistent loop around it keeps the
// general walk's register allocation of a one-tile kernel)
template <int NV, int MODE>
__device__ __noinline__ void redo_tile(KParams& dp, LDS uint32_t* win, uint32_t t, int lane) {
  uint64_t lo, hi;
  tile_range(dp, t, lo, hi);
  const Src w = load_window(dp, win, lo, lane, is_thrift(MODE), false);
  const uint32_t dsig = data_sig(dp);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0 && dsig == dp.prog->sig) atomicAdd((unsigned long long*)&dp.status->diag[2], 1ull);
  const Agg a = walk_tile<NV, MODE>(dp, w, lo, hi, t == 0 ? 0ull : X_NONE, lane, dp.starts + (uint64_t)t * dp.slotcap, dsig);
  if (lane == 0) put_tile(dp, t, a, NV);
}

// ---- kernel 1, redo: the queued tiles, general walk (one persistent grid; exits at once when none) ----
template <int NV, int MODE>
__global__ void __launch_bounds__(NT, 4) redo_kernel(DecParams dp_) {
  KParams& dp = KX_PARAMS();
  (void)dp_;
  __shared__ __attribute__((aligned(16))) uint32_t WIN[WAVES][WINW];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const uint32_t W = gridDim.x * WAVES;
  if (data_sig_s(dp) != dp.prog->sig) {   // index_fast_kernel left the whole batch: every tile
    for (uint64_t t = dp.t_lo + blockIdx.x * WAVES + wv; t < dp.t_hi; t += W)
      redo_tile<NV, MODE>(dp, (LDS uint32_t*)WIN[wv], (uint32_t)t, lane);
    return;
  }
  const uint32_t n = __builtin_amdgcn_readfirstlane(*(volatile uint32_t*)dp.redo_n);
  for (uint32_t i = blockIdx.x * WAVES + wv; i < n; i += W)
    redo_tile<NV, MODE>(dp, (LDS uint32_t*)WIN[wv], __builtin_amdgcn_readfirstlane(dp.redo[i]), lane);
}

// ---- kernel 1b: group scan (one wave per group of 64 tiles) ----
template <int NV, int MODE>
__global__ void __launch_bounds__(NT) group_kernel(DecParams dp_) {
  KParams& dp = KX_PARAMS();
  (void)dp_;
  __shared__ __attribute__((aligned(16))) uint32_t WIN[WAVES][WINW];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const uint64_t g = dp.g_lo + (uint64_t)blockIdx.x * WAVES + wv;
  if (g >= dp.g_hi) return;
  group_scan<NV, MODE, false>(dp, (LDS uint32_t*)WIN[wv], g, g == 0 && !dp.offsets ? 0ull : X_NONE, lane);
}

// exclusive scan of v over the CT threads of the chain workgroup (*tot = the sum); every thread calls it
__device__ __forceinline__ uint64_t block_scan_u64(uint64_t v, uint64_t* tot, uint64_t* sc, int tid) {
  const int lane = tid & 63, wv = tid >> 6;
  const uint64_t inc = wave_incl_scan(v, lane);
  if (lane == 63) sc[wv] = inc;
  __syncthreads();
  uint64_t before = 0, all = 0;
  for (int k = 0; k < CW; k++) {
    const uint64_t x = sc[k];
    before += k < wv ? x : 0;
    all += x;
  }
  __syncthreads();
  *tot = all;
  return before + inc - v;
}

// ---- kernel 2: chain + scan over the groups (one workgroup of 4 waves, lane = group) ----
// Resolves the group chain from offset 0 (re-scanning a group from its true entry where the
// speculation disagreed), writes every group's exclusive record / arena base, the number of records
// to emit, and the final status when the chain ends early (decode error, input exhausted).
template <int NV, int MODE>
__global__ void __launch_bounds__(CT) chain_kernel(DecParams dp_) {
  KParams& dp = KX_PARAMS();
  (void)dp_;
  if (dp.gate && !(*(volatile uint32_t*)dp.gate & 1u)) return;
  __shared__ __attribute__((aligned(16))) uint32_t WIN0[WINW];
  __shared__ uint64_t s_wcnt[CW], s_wvar[CW][KXP_NV_MAX], s_wlast[CW];
  __shared__ int s_werr[CW];
  __shared__ uint64_t s_E, s_cnt, s_var[KXP_NV_MAX], s_nstop, s_badE;
  __shared__ int s_bad, s_err, s_done, s_fast, s_fok;
  __shared__ uint64_t s_scan[CW];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint64_t ep = dp.epoch, ng = dp.ngroups;
  const bool chain = !dp.offsets;
  uint64_t* const cy = dp.carry;  // chain state between chunks (CY_*)
  if (tid == 0) {
    if (dp.chunk_first) {
      s_E = 0;  // the chain enters group 0 at offset 0
      s_cnt = 0;
      for (int v = 0; v < KXP_NV_MAX; v++)   // arena units before this call
        s_var[v] = dp.var_base[v] + (dp.var_base_dev ? dp.var_base_dev[v] : 0);
      s_nstop = dp.n;
      s_err = 0;
      s_done = 0;
    } else {
      s_E = cy[CY_E];
      s_cnt = cy[CY_CNT];
      for (int v = 0; v < KXP_NV_MAX; v++) s_var[v] = cy[CY_VAR + v];
      s_nstop = cy[CY_NSTOP];
      s_err = (int)(cy[CY_FLAGS] & 1);
      s_done = (int)(cy[CY_FLAGS] >> 1);
    }
  }
  __syncthreads();
  const uint64_t gend = dp.g_hi;
  // Fast path: when every group of the call (or chunk) has a record start, no group ended in an error and
  // each group's entry is where the group below it exits (the first one: where the chain carried in from
  // the previous chunk, offset 0 for the first), the pass is a plain scan of the group totals: a thread
  // takes a contiguous run of groups, checks and sums it, one block scan gives every run its base, the
  // carry moves on. Anything else (and a chain that already ended) takes the batch loop below.
  if (tid == 0) {
    s_fast = !s_err && !s_done;
    s_fok = 1;
  }
  __syncthreads();
  bool fast = false;   // the fast path resolved the whole call
  if (s_fast) {
    // the group words were written by the group kernel (an earlier launch): plain loads, issued four
    // groups at a time so that their latencies overlap
    const uint64_t* gw = dp.gdesc;
    const uint64_t gl = dp.g_lo, gn = dp.g_hi - dp.g_lo;
    const uint64_t per = (gn + CT - 1) / CT;
    const uint64_t lo = gl + kmin64((uint64_t)tid * per, gn), hi = kmin64(lo + per, dp.g_hi);
    bool ok = true;
    uint64_t c = 0, vs[NV > 0 ? NV : 1];
#pragma unroll
    for (int v = 0; v < NV; v++) vs[v] = 0;
    uint64_t E = s_E;   // the chain enters the call's first group where the previous chunk left it
    if (lo > gl && lo < hi) {
      const uint64_t x = gw[(uint64_t)G_EXIT * ng + lo - 1];
      ok &= (x >> 48) == ep;
      E = x & V48;
    }
    constexpr int U = 4;
    for (uint64_t g0 = lo; g0 < hi; g0 += U) {
      uint64_t xe[U], xx[U], xc[U], xv[U][NV > 0 ? NV : 1];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t g = kmin64(g0 + u, hi - 1);
        xe[u] = gw[(uint64_t)G_ENT * ng + g];
        xx[u] = gw[(uint64_t)G_EXIT * ng + g];
        xc[u] = gw[(uint64_t)G_CNT * ng + g];
#pragma unroll
        for (int v = 0; v < NV; v++) xv[u][v] = gw[(uint64_t)(G_VAR + v) * ng + g];
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t g = g0 + u;
        if (g >= hi) break;
        ok &= (xe[u] >> 48) == ep && (xx[u] >> 48) == ep && (xc[u] >> 48) == ep;
        const uint64_t gent = xe[u] & V48, gex = xx[u] & V48;
        if (chain) {
          ok &= gent != X_NONE && gent != X_BAD && gex != X_ERR;
          ok &= chain_ok(E, gent, kmin64((g + 1) * (uint64_t)GT * TILE, dp.in_len));
        }
        E = gex;
        c += xc[u] & V48;
#pragma unroll
        for (int v = 0; v < NV; v++) {
          ok &= (xv[u][v] >> 48) == ep;
          vs[v] += xv[u][v] & V48;
        }
      }
    }
    if (!ok) s_fok = 0;
    __syncthreads();
    fast = s_fok != 0;
    if (fast) {
      uint64_t vb[NV > 0 ? NV : 1], vt[NV > 0 ? NV : 1];
#pragma unroll
      for (int v = 0; v < NV; v++) vb[v] = s_var[v];   // arena units before this call (or chunk)
      uint64_t tot;
      uint64_t base = s_cnt + block_scan_u64(c, &tot, s_scan, tid);
#pragma unroll
      for (int v = 0; v < NV; v++) vb[v] += block_scan_u64(vs[v], &vt[v], s_scan, tid);
      for (uint64_t g0 = lo; g0 < hi; g0 += U) {
        uint64_t xc[U], xv[U][NV > 0 ? NV : 1];
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint64_t g = kmin64(g0 + u, hi - 1);
          xc[u] = gw[(uint64_t)G_CNT * ng + g] & V48;
#pragma unroll
          for (int v = 0; v < NV; v++) xv[u][v] = gw[(uint64_t)(G_VAR + v) * ng + g] & V48;
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint64_t g = g0 + u;
          if (g >= hi) break;
          put_word(dp.gdesc, ng, G_BCNT, g, ep, base);
          base += xc[u];
#pragma unroll
          for (int v = 0; v < NV; v++) {
            put_word(dp.gdesc, ng, G_BVAR + v, g, ep, vb[v]);
            vb[v] += xv[u][v];
          }
        }
      }
      if (tid == 0) {
        s_cnt += tot;
#pragma unroll
        for (int v = 0; v < NV; v++) s_var[v] += vt[v];
        s_done = s_cnt >= dp.n;
        if (chain && dp.g_hi > dp.g_lo) s_E = gw[(uint64_t)G_EXIT * ng + dp.g_hi - 1] & V48;   // the carry
      }
      __syncthreads();
    }
  }
  for (uint64_t b0 = dp.g_lo; b0 < gend && !fast; b0 += CT) {
    if (s_err || s_done) {  // the chain already ended: later groups emit nothing
      const uint64_t g = b0 + tid;
      if (g < gend) put_word(dp.gdesc, ng, G_BCNT, g, ep, X_DONE);
      continue;
    }
    const uint64_t g = b0 + tid;
    const bool act = g < gend;
    uint64_t gent, gex, cnt, errc, errp, var[NV > 0 ? NV : 1];
    uint64_t base, vbase[NV > 0 ? NV : 1], c0, vx[NV > 0 ? NV : 1];
    bool live, dead;
    int fe;
    for (;;) {
      constexpr int NW = 5 + NV;
      int fields[NW];
#pragma unroll
      for (int k = 0; k < NW; k++) fields[k] = k < 5 ? k : G_VAR + (k - 5);
      uint64_t x[NW];
      if (!get_words<NW>(dp.gdesc, ng, fields, NW, act ? g : 0, ep, act, x) && lane == 0)
        atomicCAS((int*)&dp.status->code, 0, KX_ERR_INTERNAL);
      gent = act ? x[0] : X_NONE; gex = act ? x[1] : X_NONE; cnt = act ? x[2] : 0;
      errc = act ? x[3] : 0; errp = act ? x[4] : 0;
#pragma unroll
      for (int v = 0; v < NV; v++) var[v] = act ? x[5 + v] : 0;
      // the chain stops at the first erroring group
      const uint64_t em = __ballot(act && chain && gex == X_ERR);
      fe = em ? __ffsll((long long)em) - 1 : 64;
      live = act && lane <= fe;
      c0 = live ? cnt : 0;
      const uint64_t ci = wave_incl_scan(c0, lane);
#pragma unroll
      for (int v = 0; v < NV; v++) {
        const uint64_t x0 = live ? var[v] : 0;
        const uint64_t vi = wave_incl_scan(x0, lane);
        vx[v] = vi - x0;
        if (lane == 63) s_wvar[wv][v] = vi;
      }
      const uint64_t hm = __ballot(act && gent != X_NONE && gent != X_BAD);
      if (lane == 63) s_wcnt[wv] = ci;
      const uint64_t wlast = hm ? rl64(gex, 63 - __clzll((long long)hm)) : X_NONE;
      if (lane == 0) {
        s_wlast[wv] = wlast;
        s_werr[wv] = em != 0;
      }
      if (tid == 0) s_bad = 1 << 30;
      __syncthreads();
      base = s_cnt + ci - c0;
      dead = false;
#pragma unroll
      for (int v = 0; v < NV; v++) vbase[v] = s_var[v] + vx[v];
      uint64_t Ein = s_E;
      for (int k = 0; k < wv; k++) {
        base += s_wcnt[k];
#pragma unroll
        for (int v = 0; v < NV; v++) vbase[v] += s_wvar[k][v];
        dead |= s_werr[k] != 0;
        if (s_wlast[k] != X_NONE) Ein = s_wlast[k];
      }
      if (!chain) break;
      // expected entry = effective exit of the nearest lower group with a record start
      const uint64_t below = hm & ((1ull << lane) - 1);
      const int pc = below ? 63 - __clzll((long long)below) : -1;
      const uint64_t pex = __shfl(gex, pc < 0 ? 0 : pc, 64);
      const uint64_t E = pc >= 0 ? pex : Ein;
      const uint64_t hi = kmin64((g + 1) * (uint64_t)GT * TILE, dp.in_len);
      const bool bad = live && !dead && base < dp.n && !chain_ok(E, gent, hi);
      if (bad) atomicMin(&s_bad, tid);
      __syncthreads();
      const int b = s_bad;
      if (b == (1 << 30)) break;
      if (tid == b) s_badE = E;
      __syncthreads();
      if (wv == 0) {  // re-scan the first disagreeing group from its true entry, then re-check
        if (lane == 0) atomicAdd((unsigned long long*)&dp.status->diag[1], 1ull);
        group_scan<NV, MODE, true>(dp, (LDS uint32_t*)WIN0, b0 + b, s_badE, lane);
      }
      __syncthreads();
    }
    if (act) {
      put_word(dp.gdesc, ng, G_BCNT, g, ep, (dead || !live) ? X_DONE : base);
#pragma unroll
      for (int v = 0; v < NV; v++) put_word(dp.gdesc, ng, G_BVAR + v, g, ep, vbase[v]);
    }
    // a decode error ends the chain (reported only when it falls before record n)
    if (chain && !dead && fe < 64 && lane == fe) {
      const uint64_t rec = base + cnt;  // records decoded before the failing one
      if (rec < dp.n) {
        kx_status* st = dp.status;
        st->code = (int32_t)errc; st->record = rec; st->offset = errp;
        st->n_records = rec; st->consumed = errp;
        uint64_t tot[NV > 0 ? NV : 1];
#pragma unroll
        for (int v = 0; v < NV; v++) {
          tot[v] = vbase[v] + var[v];
          if (v < (int)dp.prog->nvar && v < KX_STATUS_VT) st->var_total[v] = tot[v];
        }
        close_slots<NV>(dp.prog, dp.cols, dp.overflow, rec, tot);
        if (MODE == M_SKIP || is_frame(MODE)) dp.skip_out[rec] = errp;
        s_nstop = rec;
      }
      s_err = 1;
    }
    __syncthreads();
    if (tid == 0) {  // carry into the next batch
      bool stop = false;
      for (int k = 0; k < CW && !stop; k++) {
        s_cnt += s_wcnt[k];
        for (int v = 0; v < NV; v++) s_var[v] += s_wvar[k][v];
        if (s_wlast[k] != X_NONE) s_E = s_wlast[k];
        stop = s_werr[k] != 0;
      }
      if (s_cnt >= dp.n) s_done = 1;
    }
    __syncthreads();
  }
  // the chain ran out of input before n records: EOF at the record after the last one
  if (tid == 0) {
    const uint64_t tot = s_cnt;
    if (dp.chunk_last && chain && !s_err && tot < dp.n) {
      kx_status* st = dp.status;
      st->code = KX_ERR_EOF; st->record = tot; st->offset = dp.in_len;
      st->n_records = tot; st->consumed = dp.in_len;
      uint64_t vt[NV > 0 ? NV : 1];
      for (int v = 0; v < NV; v++) {
        vt[v] = s_var[v];
        if (v < (int)dp.prog->nvar && v < KX_STATUS_VT) st->var_total[v] = s_var[v];
      }
      close_slots<NV>(dp.prog, dp.cols, dp.overflow, tot, vt);
      if (MODE == M_SKIP || is_frame(MODE)) dp.skip_out[tot] = dp.in_len;
      s_nstop = tot;
    }
    // emit of this chunk bounds itself by nstop: final once the chain has ended, else unbounded
    *dp.nstop = (dp.chunk_last || s_err || s_done) ? s_nstop : ~0ull;
    if (dp.gate_reset) *(volatile uint32_t*)dp.gate = 0u;   // re-armed for the next call (chain_fast_kernel)
    if (!dp.chunk_last) {
      cy[CY_E] = s_E;
      cy[CY_CNT] = s_cnt;
      for (int v = 0; v < KXP_NV_MAX; v++) cy[CY_VAR + v] = s_var[v];
      cy[CY_NSTOP] = s_nstop;
      cy[CY_FLAGS] = (uint64_t)(s_err != 0) | (uint64_t)(s_done != 0) << 1;
    }
  }
}

// ---- kernel 2, fast form: the chain pass's fast path alone (round 5). The general chain kernel holds the
// serial repair loop and the group re-scan (268 VGPRs, scratch, one 256-thread workgroup: ~65 us for 16 M
// R2 records, most of it the latency of each thread's run of 21 groups). This kernel has 1024 threads and
// no repair: when every group of the call (chunk) chains, it writes the bases, the nstop and the carry;
// otherwise it raises *dp.gate and chain_kernel (launched right behind it, gated) does the whole pass.
constexpr int CFT = 1024, CFW = CFT / 64;
__device__ __forceinline__ uint64_t block_scan_cf(uint64_t v, uint64_t* tot, uint64_t* sc, int tid) {
  const int lane = tid & 63, wv = tid >> 6;
  const uint64_t inc = wave_incl_scan(v, lane);
  if (lane == 63) sc[wv] = inc;
  __syncthreads();
  uint64_t before = 0, all = 0;
#pragma unroll
  for (int k = 0; k < CFW; k++) {
    const uint64_t x = sc[k];
    before += k < wv ? x : 0;
    all += x;
  }
  __syncthreads();
  *tot = all;
  return before + inc - v;
}

template <int NV, int MODE>
__global__ void __launch_bounds__(CFT) chain_fast_kernel(DecParams dp_) {
  KParams& dp = KX_PARAMS();
  (void)dp_;
  __shared__ uint64_t s_E, s_cnt, s_var[KXP_NV_MAX], s_nstop;
  __shared__ int s_err, s_done, s_fok;
  __shared__ uint64_t s_scan[CFW];
  const int tid = threadIdx.x;
  const uint64_t ep = dp.epoch, ng = dp.ngroups;
  const bool chain = !dp.offsets;
  uint64_t* const cy = dp.carry;
  if (tid == 0) {
    if (dp.chunk_first) {
      s_E = 0;
      s_cnt = 0;
      for (int v = 0; v < KXP_NV_MAX; v++) s_var[v] = dp.var_base[v] + (dp.var_base_dev ? dp.var_base_dev[v] : 0);
      s_nstop = dp.n;
      s_err = 0;
      s_done = 0;
    } else {
      s_E = cy[CY_E];
      s_cnt = cy[CY_CNT];
      for (int v = 0; v < KXP_NV_MAX; v++) s_var[v] = cy[CY_VAR + v];
      s_nstop = cy[CY_NSTOP];
      s_err = (int)(cy[CY_FLAGS] & 1);
      s_done = (int)(cy[CY_FLAGS] >> 1);
    }
    s_fok = 1;
  }
  __syncthreads();
  if (s_err || s_done) {   // the chain already ended in an earlier chunk: the general pass marks the groups
    if (tid == 0) *(volatile uint32_t*)dp.gate = 1u;
    return;
  }
  const uint64_t* gw = dp.gdesc;
  const uint64_t gl = dp.g_lo, gn = dp.g_hi - dp.g_lo;
  const uint64_t per = (gn + CFT - 1) / CFT;
  const uint64_t lo = gl + kmin64((uint64_t)tid * per, gn), hi = kmin64(lo + per, dp.g_hi);
  bool ok = true;
  uint64_t c = 0, vs[NV > 0 ? NV : 1];
#pragma unroll
  for (int v = 0; v < NV; v++) vs[v] = 0;
  uint64_t E = s_E;
  if (lo > gl && lo < hi) {
    const uint64_t x = gw[(uint64_t)G_EXIT * ng + lo - 1];
    ok &= (x >> 48) == ep;
    E = x & V48;
  }
  for (uint64_t g = lo; g < hi; g++) {
    const uint64_t xe = gw[(uint64_t)G_ENT * ng + g], xx = gw[(uint64_t)G_EXIT * ng + g];
    const uint64_t xc = gw[(uint64_t)G_CNT * ng + g];
    ok &= (xe >> 48) == ep && (xx >> 48) == ep && (xc >> 48) == ep;
    const uint64_t gent = xe & V48, gex = xx & V48;
    if (chain) {
      ok &= gent != X_NONE && gent != X_BAD && gex != X_ERR;
      ok &= chain_ok(E, gent, kmin64((g + 1) * (uint64_t)GT * TILE, dp.in_len));
    }
    E = gex;
    c += xc & V48;
#pragma unroll
    for (int v = 0; v < NV; v++) {
      const uint64_t xv = gw[(uint64_t)(G_VAR + v) * ng + g];
      ok &= (xv >> 48) == ep;
      vs[v] += xv & V48;
    }
  }
  if (!ok) s_fok = 0;
  __syncthreads();
  if (!s_fok) {
    if (tid == 0) *(volatile uint32_t*)dp.gate = 1u;
    return;
  }
  uint64_t tot, vt[NV > 0 ? NV : 1], vb[NV > 0 ? NV : 1];
  uint64_t base = s_cnt + block_scan_cf(c, &tot, s_scan, tid);
#pragma unroll
  for (int v = 0; v < NV; v++) vb[v] = s_var[v] + block_scan_cf(vs[v], &vt[v], s_scan, tid);
  for (uint64_t g = lo; g < hi; g++) {
    put_word(dp.gdesc, ng, G_BCNT, g, ep, base);
    base += gw[(uint64_t)G_CNT * ng + g] & V48;
#pragma unroll
    for (int v = 0; v < NV; v++) {
      put_word(dp.gdesc, ng, G_BVAR + v, g, ep, vb[v]);
      vb[v] += gw[(uint64_t)(G_VAR + v) * ng + g] & V48;
    }
  }
  if (tid == 0) {
    const uint64_t cnt = s_cnt + tot;
    uint64_t var[NV > 0 ? NV : 1];
#pragma unroll
    for (int v = 0; v < NV; v++) var[v] = s_var[v] + vt[v];
    const bool done = cnt >= dp.n;
    const uint64_t ex = chain && gn ? gw[(uint64_t)G_EXIT * ng + dp.g_hi - 1] & V48 : s_E;
    uint64_t nstop = s_nstop;
    if (dp.chunk_last && chain && cnt < dp.n) {   // the chain ran out of input before n records: EOF
      kx_status* st = dp.status;
      st->code = KX_ERR_EOF; st->record = cnt; st->offset = dp.in_len;
      st->n_records = cnt; st->consumed = dp.in_len;
      for (int v = 0; v < NV; v++)
        if (v < (int)dp.prog->nvar && v < KX_STATUS_VT) st->var_total[v] = var[v];
      close_slots<NV>(dp.prog, dp.cols, dp.overflow, cnt, var);
      if (MODE == M_SKIP || is_frame(MODE)) dp.skip_out[cnt] = dp.in_len;
      nstop = cnt;
    }
    *dp.nstop = (dp.chunk_last || done) ? nstop : ~0ull;
    if (!dp.chunk_last) {
      cy[CY_E] = ex;
      cy[CY_CNT] = cnt;
      for (int v = 0; v < KXP_NV_MAX; v++) cy[CY_VAR + v] = v < NV ? var[v] : s_var[v];
      cy[CY_NSTOP] = nstop;
      cy[CY_FLAGS] = (uint64_t)(done ? 1 : 0) << 1;
    }
  }
}

// Emit of a record the fast index path validated (T_CANON tile): the canonical plan alone, no header
// checks and no bounds checks (every step of the record lies inside the window). Fixed fields are
// stored, var fields recorded for the copy; returns the record's end.
template <int NV>
__device__ __forceinline__ uint64_t emit_canon(const Src& w, const KAS KxLaunchCols& cols, uint64_t pos, uint64_t r,
                                               VarState<NV>& vs) {
  const KAS KxpStep* __restrict__ steps = w.steps;
  uint32_t q = (uint32_t)(pos - w.wpos);
  uint32_t k = 0;
  while (k < w.nsteps) {
    const KxpStep st = ldk(&steps[k]);
    if (st.kind == KXP_S_FIXED) {
      const uint32_t m = min(st.hdr >> 24, 4u);
#pragma unroll
      for (uint32_t j = 0; j < 4; j++) {
        if (j >= m) break;
        const KxpStep sj = j == 0 ? st : ldk(&steps[k + j]);
        const LDS uint32_t* s0 = w.win + (q >> 2);
        const uint32_t sh = q & 3;
        Fetch f;
        f.w0 = __builtin_amdgcn_alignbyte(s0[1], s0[0], sh);
        f.w1 = __builtin_amdgcn_alignbyte(s0[2], s0[1], sh);
        f.w2 = __builtin_amdgcn_alignbyte(s0[3], s0[2], sh);
        store_col(cols.data[sj.col], sj.width, r, fixed_after_header(f, sj.hdr & 0xff));
        q += 3 + sj.width;
      }
      k += m;
      continue;
    }
    k++;
    if (st.kind == KXP_S_END) { q += 1; continue; }
    if (st.kind == KXP_S_STRUCT) { q += 3; continue; }
    const bool list = st.kind == KXP_S_LIST;
    const uint32_t l = __builtin_bswap32(win_ld(w, q + (list ? 4u : 3u)));
    const uint32_t vp = q + (list ? 8u : 7u);
    vset<NV>(vs, st.vslot, w.wpos + vp, l);
    q = vp + l * (list ? st.width : 1u);
  }
  return w.wpos + q;
}

// one element of wire type t at q: its payload position and length (strings) or width (scalars)
__device__ __forceinline__ uint64_t elem_at(const Src& w, uint64_t q, uint32_t t, uint64_t& xp, uint32_t& xl) {
  if (t == KX_T_STRING) {
    xl = __builtin_bswap32(ld4(w, q));
    xp = q + 4;
    return q + 4 + xl;
  }
  xl = (uint32_t)tsize(t);
  xp = q;
  return q + xl;
}

// A list/set<string> column or one side of a map for record r: record offsets in elements at E,
// element byte offsets from B (LIST_BYTES) or host-order scalars (a map's fixed side). The record's
// walk already checked every length against its extent.
template <bool LS>
__device__ __forceinline__ void emit_container(const Src& w, const KAS KxProgram* P, const KAS KxLaunchCols& cols,
                                               uint32_t c, const KxpCol& K, uint64_t pos, uint32_t n, uint64_t E,
                                               uint64_t B, uint64_t nb, uint64_t r, uint32_t* overflow) {
  const bool lb = K.kind == KXP_K_LISTB;
  const bool fits = lb ? (E + n <= elem_lim(cols, c) && B + nb <= arena_lim(cols, c)) : E + n <= arena_lim(cols, c);
  if (!fits) { atomicOr(overflow, 1u); return; }
  put_off(cols, c, r, E);
  if (LS && K.mside == 3) {  // a field of list<S>: walk each element for this column's field
    const uint32_t c0 = P->sel_first[c], ns = P->sel_n[c];
    uint64_t q = pos;
    for (uint32_t j = 0; j < n; j++) {
      uint64_t v = 0;
      (void)elem_struct(w, P, c0, ns, q, ~0ull, &q, (int)(c - c0), &v);  // validated by the record's walk
      store_col(cols.data[c], K.width, E + j, v);
    }
    return;
  }
  uint32_t kt = KX_T_STRING, vt = KX_T_STRING;
  if (K.mside) {
    const KxpField F = ld_field(P, K.field);
    kt = F.elem & 15u;
    vt = F.elem >> 4;
  }
  KxpCol KB = K;
  KB.kind = KXP_K_BYTES;
  KB.width = 1;
  uint64_t q = pos, acc = 0;
  for (uint32_t j = 0; j < n; j++) {
    uint64_t xp, kp, vp;
    uint32_t xl, kl, vl;
    if (K.mside) {
      q = elem_at(w, q, kt, kp, kl);
      q = elem_at(w, q, vt, vp, vl);
      xp = K.mside == 1 ? kp : vp;
      xl = K.mside == 1 ? kl : vl;
    } else {
      q = elem_at(w, q, KX_T_STRING, xp, xl);
    }
    if (lb) {
      put_eoff(cols, c, E + j, B + acc);
      if (xl) copy_var(w, KB, xp, xl, (uint8_t*)cols.data[c] + B + acc);
      acc += xl;
    } else {
      uint64_t v;
      if (K.width == 1) v = K.elem == KX_T_BOOL ? (ld1(w, xp) == 1) : ld1(w, xp);
      else if (K.width == 2) v = __builtin_bswap32(ld4(w, xp)) >> 16;
      else if (K.width == 4) v = __builtin_bswap32(ld4(w, xp));
      else v = be64(w, xp);
      store_col(cols.data[c], K.width, E + j, v);
    }
  }
}

// ---- CRC32Check fused into the frame walk: the frame pipeline's emit pass checks each
// TTHeader frame's "crc32c" (crcPayloadValidator.Validate, validate.go:183-201) while the frame is in the
// LDS window, instead of a second kernel re-reading every payload from HBM (kx_crc.hip) ----
__shared__ uint32_t g_crct[8][256];   // slicing-by-8 tables, built by the frame emit kernel

struct SrcBytes {
  const Src& w;
  __device__ __forceinline__ uint32_t operator()(uint64_t p) const { return ld1(w, p); }
};

// the payload check of frame f: 0, KX_ERR_PAYLOAD_VALIDATION, or the header's UNKNOWN_PROTOCOL
__device__ __noinline__ uint8_t frame_crc_check(const Src w, uint64_t in_len, uint64_t f) {
  uint64_t a, b;
  int want;
  uint32_t exp = 0;
  const int rc = kx_frame_expect(SrcBytes{w}, in_len, f, &a, &b, &want, &exp);
  if (rc) return (uint8_t)rc;
  if (want != 1) return want == 2 ? (uint8_t)KX_ERR_PAYLOAD_VALIDATION : 0;
  uint32_t c = ~0u;
  uint64_t p = a;
  const int32_t q = b - a <= (uint64_t)WINB ? wofs(w, a, (uint32_t)(b - a) + 8) : -1;
  if (q >= 0 && b - a >= 8) {
    // inside the window: the head up to a dword boundary, then two aligned dwords per step
    const uint32_t h = (4u - ((uint32_t)q & 3u)) & 3u;
    if (h) {
      c = kx_crc_upd_k(g_crct, c, ld4(w, p) & ((1u << (8 * h)) - 1), h);
      p += h;
    }
    const LDS uint32_t* s = w.win + ((uint32_t)q + h) / 4;
    for (; p + 8 <= b; p += 8, s += 2) c = kx_crc_upd_k(g_crct, c, (uint64_t)s[0] | ((uint64_t)s[1] << 32), 8);
  }
  for (; p + 8 <= b; p += 8)
    c = kx_crc_upd_k(g_crct, c, (uint64_t)ld4(w, p) | ((uint64_t)ld4(w, p + 4) << 32), 8);
  if (p < b) {
    const uint32_t k = (uint32_t)(b - p);
    uint64_t d = (uint64_t)ld4(w, p) | ((uint64_t)(k > 4 ? ld4(w, p + 4) : 0u) << 32);
    d &= (1ull << (8 * k)) - 1;
    c = kx_crc_upd_k(g_crct, c, d, k);
  }
  return ~c == exp ? 0 : (uint8_t)KX_ERR_PAYLOAD_VALIDATION;
}

// ---- kernel 3: emit pass (one wave per tile, lane = record) ----
// COOP: numeric list columns are copied by the whole wave (its own instantiation, so that schemas
// without such a column keep the record-by-record kernel's code)
template <int NV, int MODE, bool COOP>
__device__ __forceinline__ void emit_tile(KParams& dp, LDS uint32_t* win, uint64_t t, int lane, bool plan = true) {
  const KAS KxProgram* P = dp.prog;
  const bool known = dp.offsets != nullptr;
  const uint64_t nstop = known ? dp.n : *(volatile uint64_t*)dp.nstop;
  uint64_t lo, hi;
  tile_range(dp, t, lo, hi);
  // the window DMA is issued first; the tile's bases are read while it is in flight
  const uint16_t* starts = dp.starts + t * dp.slotcap;
  Src w = load_window(dp, win, known ? dp.offsets[lo] : lo, lane, is_thrift(MODE), false);
  if (!plan) w.nsteps = 0;   // records known not to start on the plan (walk_tile): the generic loop alone
  uint64_t base = 0, cnt = 0, run[NV > 0 ? NV : 1];
#pragma unroll
  for (int v = 0; v < (NV > 0 ? NV : 1); v++) run[v] = 0;
  if (dp.direct) {  // offsets mode without arena columns: no index pass
    base = lo;
    cnt = hi - lo;
  } else {
    const uint64_t g = t / GT;
    // written by earlier kernels of this call: plain (cached) loads suffice
    const uint64_t* gd = dp.gdesc;
    const uint64_t* td = dp.tdesc;
    const uint64_t gb = gd[(uint64_t)G_BCNT * dp.ngroups + g] & V48;
    base = gb + (td[(uint64_t)T_PCNT * dp.ntiles + t] & V48);
    cnt = gb == X_DONE ? 0 : td[(uint64_t)T_CNT * dp.ntiles + t] & V48;
#pragma unroll
    for (int v = 0; v < NV; v++)
      run[v] = (gd[(uint64_t)(G_BVAR + v) * dp.ngroups + g] & V48) + (td[(uint64_t)(T_PVAR + v) * dp.ntiles + t] & V48);
  }
  // a tile the fast index path validated: records are read with the plan alone
  const bool canon = is_thrift(MODE) && !dp.direct && MODE != M_THRIFT_LS &&
                     ((dp.tdesc[(uint64_t)T_ERRC * dp.ntiles + t] & V48) == T_CANON);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (cnt == 0 || base >= nstop) return;
  cnt = kmin64(cnt, nstop - base);
  // records past the tile's slots (slotcap, a multiple of 64; ws_layout) are emitted one per round,
  // each starting where the previous one ended
  uint64_t chain = 0;
  uint64_t step = 64;
  for (uint64_t j0 = 0; j0 < cnt; j0 += step) {
    const bool past = !known && j0 >= dp.slotcap;
    step = past ? 1 : 64;
    const uint64_t j = j0 + lane;
    const bool act = j < cnt && (uint64_t)lane < step;
    const uint64_t r = base + j;
    VarState<NV> vs;
#pragma unroll
    for (int v = 0; v < NV; v++) { vs.len[v] = 0; vs.pos[v] = 0; }
    uint64_t pos = 0, lim = dp.in_len, end = 0, pres = 0;
    int rc = 0;
    if (act) {
      if (known) {
        pos = dp.offsets[r];
        lim = rec_end(dp, r);
        if (pos > lim || lim > dp.in_len) rc = KX_ERR_INVALID_ARG;
      } else {
        pos = past ? chain : lo + starts[j];
      }
      if (canon) {
        end = emit_canon<NV>(w, dp.cols, pos, r, vs);
        pres = w.canon_pres;
      } else if (MODE == M_SKIP && !known && !past && r != nstop - 1 && !(j + 1 == dp.slotcap && cnt > dp.slotcap)) {
        // the skip decoder's boundaries: the index pass walked every record before nstop and left its start
        // in the slots, which is all this pass writes (the end is read only where the chain goes on from it:
        // the last slotted record of a tile with more, and the batch's last record)
      } else if (!rc) {
        rc = parse_record<NV, MODE>(dp, w, pos, lim, r, MODE != M_SKIP, &end, vs, pres);
      }
      if (rc) {  // offsets mode: the failed record reads as all defaults, empty payloads
#pragma unroll
        for (int v = 0; v < NV; v++) vs.len[v] = 0;
        pres = 0;
        if (MODE != M_SKIP && !is_frame(MODE)) emit_defaults(P, dp.cols, r);
      }
      if (MODE == M_SKIP || is_frame(MODE)) dp.skip_out[r] = pos;
      if constexpr (is_frame(MODE)) {
        if (dp.fr_crc) dp.fr_crc[r] = rc ? 0 : frame_crc_check(w, dp.in_len, pos);
      }
      if (MODE != M_SKIP && !is_frame(MODE) && dp.cols.presence) dp.cols.presence[r] = pres;
      if (known) {
        if (rc) atomicMin(dp.errkey, (unsigned long long)((r << 8) | (uint64_t)(rc & 0xff)));
        if (dp.rstat) dp.rstat[r] = (uint8_t)rc;
      }
    }
    // arena positions: wave exclusive scan of the var lengths (per slot)
    uint64_t atv[NV > 0 ? NV : 1];
#pragma unroll
    for (int v = 0; v < NV; v++) {
      if (v >= (int)P->nvar) break;
      const uint64_t x0 = act ? vs.len[v] : 0;
      uint64_t xi;
      if (KX_SCAN32 && !__ballot(x0 >= (1u << 26))) xi = wave_incl_scan32((uint32_t)x0);   // 64 lengths < 2^26: the sum fits
      else xi = wave_incl_scan(x0, lane);
      atv[v] = run[v] + xi - x0;
      run[v] += rl64(xi, 63);
    }
#pragma unroll
    for (int v = 0; v < NV; v++) {
      if (v >= (int)P->nvar) break;
      const uint64_t at = atv[v];
      const uint32_t cc = P->var_col[v];
      const KxpCol K = ld_col(P, cc);
      if (K.kind == KXP_K_LISTB || K.mside) {   // containers: element by element, with both slots
        if ((uint32_t)v == K.vslot && act) {
          uint64_t B = 0, nb = 0;
#pragma unroll
          for (int u = 0; u < NV; u++)
            if ((uint32_t)u == K.vslot2) { B = atv[u]; nb = vs.len[u]; }
          emit_container<MODE == M_THRIFT_LS>(w, P, dp.cols, cc, K, vs.pos[v], vs.len[v], at, B, nb, r, dp.overflow);
        }
      } else if ((dp.cols.view >> cc) & 1) {
        if (act) put_view(dp.cols, cc, r, vs.pos[v], vs.len[v]);
      } else if (COOP && K.kind == KXP_K_LIST && K.width > 1 && !((dp.cols.view >> cc) & 1)) {
        // wave-cooperative list copy: the wave's elements are one contiguous arena run [at0, at0 + T);
        // lane e copies element e of it, finding its record by a binary search over the lanes' starts
        const uint32_t nn = act ? vs.len[v] : 0;
        const bool fits = act && at + nn <= arena_lim(dp.cols, cc);
        if (act) {
          if (fits) put_off(dp.cols, cc, r, at);
          else atomicOr(dp.overflow, 1u);
        }
        const uint64_t at0 = rl64(at, 0);
        const uint64_t rel = at - at0;
        const uint64_t T = rl64(at + nn, 63) - at0;
        const uint32_t okm = fits ? 1u : 0u;
        const uint64_t psrc = vs.pos[v];
        GLB uint8_t* cbase = (GLB uint8_t*)dp.cols.data[cc];
        for (uint64_t e0 = 0; e0 < T; e0 += 64) {
          const uint64_t e = e0 + lane;
          int sl = 0;
#pragma unroll
          for (int step = 32; step >= 1; step >>= 1) {
            const int c = sl + step;
            if (shfl64(rel, c) <= e) sl = c;
          }
          const uint64_t rr = shfl64(rel, sl);
          const uint64_t pr = shfl64(psrc, sl);
          const uint32_t ok = (uint32_t)__shfl((int)okm, sl, 64);
          if (e < T && ok) {
            const uint64_t s = pr + (e - rr) * K.width;
            const uint64_t d = at0 + e;
            if (K.width == 8) ((GLB uint64_t*)cbase)[d] = be64(w, s);
            else if (K.width == 4) ((GLB uint32_t*)cbase)[d] = be32(w, s);
            else {
              const uint32_t x = ld1(w, s) << 8 | ld1(w, s + 1);
              ((GLB uint16_t*)cbase)[d] = (uint16_t)x;
            }
          }
        }
      } else {
        const uint32_t nn = act ? vs.len[v] : 0u;
        uint8_t* dst = (uint8_t*)dp.cols.data[cc] + at * K.width;
        bool big = false;
        if (act) {
          if (at + nn <= arena_lim(dp.cols, cc)) {
            put_off(dp.cols, cc, r, at);
            big = K.kind == KXP_K_BYTES && nn >= KX_WAVE_COPY;
            if (nn && !big)
              copy_var(w, K, vs.pos[v], nn, dst);
          } else {
            atomicOr(dp.overflow, 1u);
          }
        }
        wave_copy_deferred(w, big, vs.pos[v], nn, dst, lane, false);
      }
    }
    if (act && r == nstop - 1 && nstop == dp.n) {
      uint64_t tot[NV > 0 ? NV : 1];
#pragma unroll
      for (int v = 0; v < NV; v++) {
        tot[v] = (v < (int)P->nvar) ? atv[v] + vs.len[v] : 0;
        if (v < (int)P->nvar && v < KX_STATUS_VT) dp.status->var_total[v] = tot[v];
      }
      close_slots<NV>(P, dp.cols, dp.overflow, dp.n, tot);
    }
    if (act && r == nstop - 1 && nstop == dp.n) {
      kx_status* st = dp.status;
      st->n_records = dp.n;
      st->consumed = known ? rec_end(dp, dp.n - 1) : end;
      if (MODE == M_SKIP || is_frame(MODE)) dp.skip_out[dp.n] = end;
    }
    if (!known) chain = rl64(end, (int)(kmin64(step, cnt - j0) - 1));   // the round's last record ends here
  }
}

// Split points of a concatenated batch (kx_thrift_split_points; SURVEY.md §8e "pass A emits G split
// points", the partition the reference leaves to its caller, codec_apache.go:166-172): lane k of the grid
// finds the start of record floor(k·n/G) from what the index, group and chain passes left (the tile's
// global record base = group base + tile prefix, then the tile's record-start slot; past the slots the
// records are skipped one by one from the last slot), and lane G the end of record n − 1. Nothing else
// is read: no emit pass. A chain that ended early (decode error, EOF) leaves its status and no points.
template <int NV, int MODE>
__global__ void __launch_bounds__(64) split_kernel(DecParams dp_) {
  KParams& dp = KX_PARAMS();
  (void)dp_;
  const uint64_t k = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  const uint64_t G = dp.nsplit, n = dp.n;
  if (k > G || *(volatile uint64_t*)dp.nstop < n) return;
  const bool last = k == G;
  // floor(k·n / G) without a 128-bit product (G <= 2^16)
  const uint64_t i = last ? n - 1 : (n / G) * k + ((n % G) * k) / G;
  const uint64_t nt = dp.ntiles, ng = dp.ngroups;
  auto tbase = [&](uint64_t t) -> uint64_t {   // first record of tile t (tiles past the chain: none)
    const uint64_t gb = dp.gdesc[(uint64_t)G_BCNT * ng + t / GT] & V48;
    return gb == X_DONE ? ~0ull : gb + (dp.tdesc[(uint64_t)T_PCNT * nt + t] & V48);
  };
  uint64_t lo = 0, hi = nt;                    // tbase(lo) <= i < tbase(hi)
  while (hi - lo > 1) {
    const uint64_t mid = lo + (hi - lo) / 2;
    if (tbase(mid) <= i) lo = mid;
    else hi = mid;
  }
  const uint64_t t = lo, j = i - tbase(t), sc = dp.slotcap;
  const uint16_t* st = dp.starts + t * sc;
  const Src w{dp.in, dp.in_len, 0, 0, nullptr, nullptr, 0u, 0ull};   // global reads only
  auto skip = [&](uint64_t p, uint64_t r) -> uint64_t {
    VarState<NV> vs;
    uint64_t end = p, pres = 0;
    parse_record<NV, MODE>(dp, w, p, dp.in_len, r, false, &end, vs, pres);
    return end;
  };
  const uint64_t t0 = t * (uint64_t)TILE;
  uint64_t pos;
  if (j < sc) {
    pos = t0 + st[j];
  } else {
    pos = t0 + st[sc - 1];
    for (uint64_t m = sc - 1; m < j; m++) pos = skip(pos, i - j + m);
  }
  if (last) {
    pos = skip(pos, i);
    dp.status->n_records = n;
    dp.status->consumed = pos;
  }
  dp.split_out[k] = pos;
}

template <int NV, int MODE, bool COOP = false>
__global__ void __launch_bounds__(NT, 4) emit_kernel(DecParams dp_) {
  KParams& dp = KX_PARAMS();
  (void)dp_;
  __shared__ __attribute__((aligned(16))) uint32_t WIN[WAVES][WINW];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  if constexpr (is_frame(MODE)) {
    if (dp.fr_crc) {   // the CRC-32C slicing tables, one column per thread (NT = 256)
      const uint32_t c0 = kx_crc_t0(g_crct, (int)threadIdx.x);
      __syncthreads();
      kx_crc_tk(g_crct, (int)threadIdx.x, c0);
      __syncthreads();
    }
  }
  const uint64_t t = dp.t_lo + (uint64_t)blockIdx.x * WAVES + wv;
  if (t >= dp.t_hi) return;
  emit_tile<NV, MODE, COOP>(dp, (LDS uint32_t*)WIN[wv], t, lane);
}

// ---- kernel 3, fast form ----

// n string bytes at window offset x -> dst (global): head bytes up to a dword-aligned destination, then
// 16-byte stores assembled from 5 window dwords, then a dword / byte tail. The bytes lie in the window (a
// T_CANON record).
__device__ __forceinline__ void copy_str_win(const Src& w, uint32_t x, uint32_t n, uint8_t* dst_) {
  GLB uint8_t* dst = (GLB uint8_t*)dst_;
  const LDS uint8_t* wb = (const LDS uint8_t*)w.win;
  uint32_t i = 0;
  const uint32_t h = min((4u - ((uint32_t)(uintptr_t)dst_ & 3u)) & 3u, n);
#pragma clang loop vectorize(disable) unroll(disable)
  for (; i < h; i++) dst[i] = wb[x + i];
  for (; i + 16 <= n; i += 16) {
    const uint32_t q = x + i;
    const LDS uint32_t* s = w.win + (q >> 2);
    const uint32_t sh = q & 3;
    const uint32_t x0 = s[0], x1 = s[1], x2 = s[2], x3 = s[3], x4 = s[4];
    const v4u_a4 o = {__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh),
                      __builtin_amdgcn_alignbyte(x3, x2, sh), __builtin_amdgcn_alignbyte(x4, x3, sh)};
    *(GLB v4u_a4*)(dst + i) = o;
  }
  for (; i + 4 <= n; i += 4) *(GLB uint32_t*)(dst + i) = win_ld(w, x + i);
#pragma clang loop vectorize(disable) unroll(disable)
  for (; i < n; i++) dst[i] = wb[x + i];   // < 4 bytes
}

// the fixed value of wire type t at window offset x (big-endian) -> column c, record r
__device__ __forceinline__ void emit_fixed_at(const Src& w, const KAS KxLaunchCols& cols, uint32_t t, uint32_t c,
                                              uint32_t x, uint64_t r) {
  const LDS uint32_t* s0 = w.win + (x >> 2);
  const uint32_t sh = x & 3;
  const uint32_t lo4 = __builtin_amdgcn_alignbyte(s0[1], s0[0], sh);
  void* colp = cols.data[c];
  switch (t) {
    case KX_T_I64: case KX_T_DOUBLE: {
      const uint32_t hi4 = __builtin_amdgcn_alignbyte(s0[2], s0[1], sh);
      ((GLB uint64_t*)colp)[r] = ((uint64_t)__builtin_bswap32(lo4) << 32) | __builtin_bswap32(hi4);
      break;
    }
    case KX_T_I32: ((GLB uint32_t*)colp)[r] = __builtin_bswap32(lo4); break;
    case KX_T_I16: ((GLB uint16_t*)colp)[r] = (uint16_t)(__builtin_bswap32(lo4) >> 16); break;
    case KX_T_BOOL: ((GLB uint8_t*)colp)[r] = (lo4 & 0xffu) == 1u ? 1 : 0; break;
    default: ((GLB uint8_t*)colp)[r] = (uint8_t)lo4; break;   // BYTE
  }
}

// One T_CANON tile, lane = record: the segment bases first (only the string lengths chain them), then every
// fixed value at its constant offset in its segment, then the arena positions (a DPP scan per var slot) and
// the string copies. Same stores as emit_tile's emit_canon path.
template <int NV>
__device__ __forceinline__ void emit_fast_tile(KParams& dp, const Src& w, uint64_t lo, uint64_t base, uint64_t cnt,
                                               uint64_t nstop, uint64_t* run, const uint16_t* starts, int lane) {
  const KAS KxProgram* P = dp.prog;
  const uint32_t q0 = (uint32_t)(lo - w.wpos);
  const uint32_t nseg = dp.ep.nseg, nvar = P->nvar;
  for (uint64_t j0 = 0; j0 < cnt; j0 += 64) {
    const uint64_t j = j0 + lane;
    const bool act = j < cnt;
    const uint64_t r = base + j;
    const uint32_t q = q0 + starts[act ? j : j0];   // an idle lane parses the round's first record (no stores)
    uint32_t sb[KXE_SEG];
    uint32_t vp[NV > 0 ? NV : 1], vl[NV > 0 ? NV : 1];
#pragma unroll
    for (int v = 0; v < (NV > 0 ? NV : 1); v++) { vp[v] = 0; vl[v] = 0; }
    uint32_t qs = q;
#pragma unroll
    for (int s = 0; s < KXE_SEG; s++) {
      sb[s] = qs;
      if (s >= (int)nseg) continue;
      const uint32_t fl = dp.ep.seg[s].flen;
      if (dp.ep.seg[s].vkind) {
        const uint32_t x = qs + fl;
        const uint32_t l = __builtin_bswap32(win_ld(w, x + 3));
        const uint32_t slot = dp.ep.seg[s].vslot;
#pragma unroll
        for (int v = 0; v < NV; v++)
          if ((uint32_t)v == slot) { vp[v] = x + 7; vl[v] = l; }
        qs = x + 7 + l;
      } else {
        qs += fl;
      }
    }
    if (act) {
#pragma unroll
      for (int s = 0; s < KXE_SEG; s++) {
        if (s >= (int)nseg) break;
        const uint32_t nf = dp.ep.seg[s].nfix;
#pragma unroll
        for (int f = 0; f < KXE_FIX; f++) {
          if (f >= (int)nf) break;
          const KxpEmitFix F = ldk(&dp.ep.seg[s].fix[f]);
          emit_fixed_at(w, dp.cols, F.ttype, F.col, sb[s] + F.off, r);
        }
      }
      if (dp.cols.presence) dp.cols.presence[r] = w.canon_pres;
    }
    uint64_t atv[NV > 0 ? NV : 1];
#pragma unroll
    for (int v = 0; v < NV; v++) {
      if (v >= (int)nvar) break;
      const uint32_t x0 = act ? vl[v] : 0u;
      const uint32_t inc = wave_incl_scan32(x0);
      const uint64_t at = run[v] + (inc - x0);
      atv[v] = at;
      run[v] += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
      const uint32_t cc = P->var_col[v];
      if ((dp.cols.view >> cc) & 1) {
        if (act) put_view(dp.cols, cc, r, w.wpos + vp[v], vl[v]);
      } else {
        uint8_t* dst = (uint8_t*)dp.cols.data[cc] + at;
        bool big = false;
        if (act) {
          if (at + vl[v] <= arena_lim(dp.cols, cc)) {
            put_off(dp.cols, cc, r, at);
            big = vl[v] >= KX_WAVE_COPY;
            if (vl[v] && !big) copy_str_win(w, vp[v], vl[v], dst);
          } else {
            atomicOr(dp.overflow, 1u);
          }
        }
        wave_copy_deferred(w, big, w.wpos + vp[v], act ? vl[v] : 0u, dst, lane, true);
      }
    }
    if (act && r == nstop - 1 && nstop == dp.n) {   // the batch's last record closes the var columns
      uint64_t tot[NV > 0 ? NV : 1];
#pragma unroll
      for (int v = 0; v < NV; v++) {
        tot[v] = v < (int)nvar ? atv[v] + vl[v] : 0;
        if (v < (int)nvar && v < KX_STATUS_VT) dp.status->var_total[v] = tot[v];
      }
      close_slots<NV>(P, dp.cols, dp.overflow, dp.n, tot);
      dp.status->n_records = dp.n;
      dp.status->consumed = w.wpos + qs;
    }
  }
}

// T_CANON tiles of a concatenated Thrift batch whose canonical plan has an emit form (dp.ep.ok): a kernel of
// its own, so its registers are not those of the general field loop; any other tile (walked by the redo
// index pass, or more records than record-start slots) is queued for emit_redo_kernel. NARROW as
// index_fast_kernel (the same window the index pass validated the records in).
template <int NV, bool NARROW>
__global__ void __launch_bounds__(NARROW ? FNT : NT) emit_fast_kernel(DecParams dp_) {
  KParams& dp = KX_PARAMS();
  (void)dp_;
  constexpr int WV = NARROW ? FWAVES : WAVES, WW = NARROW ? FWINW : WINW;
  __shared__ __attribute__((aligned(16))) uint32_t WIN[WV][WW];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const uint64_t t = dp.t_lo + (uint64_t)blockIdx.x * WV + wv;
  if (t >= dp.t_hi) return;
  // a batch the fast index path left whole (its first record is not canonical: no tile is T_CANON) goes to
  // emit_redo_kernel whole, with no DMA here (one scalar load, as index_fast_kernel)
  if (data_sig_s(dp) != dp.prog->sig) return;
  uint64_t lo, hi;
  tile_range(dp, t, lo, hi);
  const Src w = load_window<NARROW ? FWINB : WINB>(dp, (LDS uint32_t*)WIN[wv], lo, lane, true, false);
  const uint64_t nstop = *(volatile uint64_t*)dp.nstop;
  const uint64_t g = t / GT;
  const uint64_t* gd = dp.gdesc;
  const uint64_t* td = dp.tdesc;
  const uint64_t gb = gd[(uint64_t)G_BCNT * dp.ngroups + g] & V48;
  const uint64_t base = gb + (td[(uint64_t)T_PCNT * dp.ntiles + t] & V48);
  uint64_t cnt = gb == X_DONE ? 0 : td[(uint64_t)T_CNT * dp.ntiles + t] & V48;
  const bool canon = (td[(uint64_t)T_ERRC * dp.ntiles + t] & V48) == T_CANON;
  uint64_t run[NV > 0 ? NV : 1];
#pragma unroll
  for (int v = 0; v < (NV > 0 ? NV : 1); v++)
    run[v] = NV > 0 ? (gd[(uint64_t)(G_BVAR + v) * dp.ngroups + g] & V48) + (td[(uint64_t)(T_PVAR + v) * dp.ntiles + t] & V48)
                    : 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (cnt == 0 || base >= nstop) return;
  if (!canon || cnt > dp.slotcap) {   // the general emit pass takes it
    if (lane == 0) dp.redo[atomicAdd(dp.redo_n + 2, 1u)] = (uint32_t)t;
    return;
  }
  emit_fast_tile<NV>(dp, w, lo, base, kmin64(cnt, nstop - base), nstop, run, dp.starts + t * dp.slotcap, lane);
}

// the tiles emit_fast_kernel queued, with the general emit pass (one resident grid; exits at once when none)
template <int NV, int MODE, bool COOP = false>
__global__ void __launch_bounds__(NT, 4) emit_redo_kernel(DecParams dp_) {
  KParams& dp = KX_PARAMS();
  (void)dp_;
  __shared__ __attribute__((aligned(16))) uint32_t WIN[WAVES][WINW];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const uint32_t W = gridDim.x * WAVES;
  if (data_sig_s(dp) != dp.prog->sig) {   // emit_fast_kernel left the whole batch: every tile
    for (uint64_t t = dp.t_lo + blockIdx.x * WAVES + wv; t < dp.t_hi; t += W)
      emit_tile<NV, MODE, COOP>(dp, (LDS uint32_t*)WIN[wv], t, lane, false);
    return;
  }
  const uint32_t n = __builtin_amdgcn_readfirstlane(*(volatile uint32_t*)(dp.redo_n + 2));
  for (uint32_t i = blockIdx.x * WAVES + wv; i < n; i += W)
    emit_tile<NV, MODE, COOP>(dp, (LDS uint32_t*)WIN[wv], __builtin_amdgcn_readfirstlane(dp.redo[i]), lane);
}

// Completes a call and re-arms the workspace for the next one (error key, overflow, nstop).
__global__ void finalize_kernel(kx_status* st, unsigned long long* errkey, uint32_t* overflow, uint64_t* nstop,
                                const uint64_t* offsets, uint64_t n, uint32_t* redo_n) {
  if (threadIdx.x != 0) return;
  redo_n[0] = 0;
  redo_n[2] = 0;   // the emit queue (emit_fast_kernel -> emit_redo_kernel)
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
  *nstop = ~0ull;
}

// ---- workspace: [8] errkey u64, [16] overflow u32, [24] nstop u64, then tile words, group words,
//      record-start slots ----
constexpr size_t WS_HDR = 512;
// header words: [8] errkey, [16] overflow, [24] nstop, [64..) chain carry (CY_WORDS), [256..) nstop ring
// (KX_PIPE_EV words), [448] redo count (u32), [452] unused (u32), [456] emit queue count (u32),
// [460] chain fallback flag (u32)
constexpr size_t WS_CARRY = 64, WS_RING = 256, WS_REDO = 448;
static_assert(WS_CARRY + 8 * CY_WORDS <= WS_RING && WS_RING + 8 * KX_PIPE_EV <= WS_REDO && WS_REDO + 16 <= WS_HDR,
              "workspace header layout");

struct WsLayout {
  uint64_t ntiles, ngroups, slotcap;
  size_t tdesc, gdesc, starts, redo, qcnt, total;
};

uint32_t krec_for(uint64_t in_len, uint64_t n) {
  if (n == 0) return 64;
  const uint64_t avg = (in_len + n - 1) / n;
  const uint64_t k = avg ? (uint64_t)TILE / avg : 64;
  return (uint32_t)(k < 1 ? 1 : k > 64 ? 64 : k);
}

// record-start slots per tile (concatenated modes), a multiple of 64: four times the records a tile
// holds at the batch's mean record size (in_len / n) plus a wave, at most one per byte (a record can be a
// single STOP byte). A tile with more records than slots keeps the first slotcap starts and the emit
// pass follows the chain record by record past them (emit_tile), so the cap bounds the workspace, not
// what decodes: 16 M R2 records (2.8 GB) need 0.22 GB of slots instead of 5.6 GB at one slot per byte.
// KX_SLOTCAP overrides it (tests force the record-by-record path with 64).
uint64_t slot_cap(uint64_t in_len, uint64_t n) {
  const long long forced = kx_knob(KXK_SLOTCAP);
  const uint64_t full = ((uint64_t)TILE + 1 + 63) & ~63ull;
  uint64_t cap = full;
  if (forced > 0) {
    cap = (uint64_t)forced;
  } else if (n) {
    const uint64_t mean = in_len / n;
    if (mean >= 4) cap = 4 * ((uint64_t)TILE / mean) + 64;
  }
  cap = (cap + 63) & ~63ull;
  return cap < 64 ? 64 : cap > full ? full : cap;
}

WsLayout ws_layout(uint64_t min_rec, uint64_t in_len, const uint64_t* offsets, uint64_t n) {
  WsLayout L{};
  if (offsets) {
    const uint64_t k = krec_for(in_len, n);
    L.ntiles = (n + k - 1) / k;
    L.slotcap = 0;
  } else {
    L.ntiles = (in_len + TILE - 1) / TILE;
    L.slotcap = slot_cap(in_len, n);
  }
  (void)min_rec;
  if (!L.ntiles) L.ntiles = 1;
  L.ngroups = (L.ntiles + GT - 1) / GT;
  size_t o = WS_HDR;
  L.tdesc = o; o += (size_t)L.ntiles * T_NF * 8;
  L.gdesc = o; o += (size_t)L.ngroups * G_NF * 8;
  L.starts = o; o += ((size_t)L.ntiles * L.slotcap * 2 + 255) & ~(size_t)255;
  L.redo = o; o += offsets ? 0 : ((size_t)L.ntiles * 4 + 255) & ~(size_t)255;   // fast index: redo queue
  // chunked pipeline: per chunk the index and emit queue counts (u32 [0] and [2] of a 16-byte block)
  L.qcnt = o; o += offsets ? 0 : ((size_t)L.ngroups * 16 + 255) & ~(size_t)255;
  L.total = o;
  return L;
}

// chunk k of a chunked call: tiles [k·cht, (k+1)·cht) and the groups they make up
DecParams chunk_params(const DecParams& dp, uint64_t k, uint64_t nch, uint64_t cht) {
  DecParams c = dp;
  c.t_lo = k * cht;
  c.t_hi = kmin64(dp.ntiles, c.t_lo + cht);
  c.g_lo = c.t_lo / GT;
  c.g_hi = (c.t_hi + GT - 1) / GT;
  c.chunk_first = k == 0;
  c.chunk_last = k + 1 == nch;
  return c;
}

template <int NV, int MODE>
void launch_emit(dim3 grid, hipStream_t stream, const DecParams& dp) {
  if constexpr (is_thrift(MODE) && NV > 0) {
    if (KX_EMIT_COOP && dp.nlist) {
      hipLaunchKernelGGL((emit_kernel<NV, MODE, true>), grid, dim3(NT), 0, stream, dp);
      return;
    }
  }
  hipLaunchKernelGGL((emit_kernel<NV, MODE>), grid, dim3(NT), 0, stream, dp);
}

// compute units of the current device (the resident redo grids' size; 64 when the runtime cannot tell)
static int resident_cus() {
  int dev = 0;
  const int n = hipGetDevice(&dev) == hipSuccess ? kx_device_cus(dev) : 0;
  return n > 0 ? n : 64;
}

// the chain pass: chain_fast_kernel, then chain_kernel gated on its fallback flag (ws header word
// redo_n[3]); KX_CHAIN_FAST=0 launches chain_kernel alone
template <int NV, int MODE>
int launch_chain(const DecParams& dp, hipStream_t stream) {
  if (dp.gate || !kx_knob(KXK_CHAIN_FAST)) {
    hipLaunchKernelGGL((chain_kernel<NV, MODE>), dim3(1), dim3(CT), 0, stream, dp);
    return hipGetLastError() != hipSuccess ? KX_ERR_HIP : KX_OK;
  }
  DecParams f = dp;
  f.gate = dp.redo_n + 3;
  hipLaunchKernelGGL((chain_fast_kernel<NV, MODE>), dim3(1), dim3(CFT), 0, stream, f);
  KX_HIP_CHECK(hipGetLastError());
  f.gate_reset = 1;
  hipLaunchKernelGGL((chain_kernel<NV, MODE>), dim3(1), dim3(CT), 0, stream, f);
  return hipGetLastError() != hipSuccess ? KX_ERR_HIP : KX_OK;
}

// the split fast emit pass (emit_fast_kernel + emit_redo_kernel) when it applies: 1 launched, 0 not, -1 error.
// It needs the fast index pass's T_CANON tiles (concatenated Thrift with a canonical plan) and a plan in emit
// form (strings and fixed scalars only); KX_EMIT_FAST=0 keeps the general emit pass (A/B)
template <int NV, int MODE>
int launch_fast_emit(const DecParams& dp, unsigned grid, hipStream_t stream) {
  if constexpr (MODE != M_THRIFT) {
    return 0;
  } else {
    if (!kx_knob(KXK_EMIT_FAST) || !dp.fast || dp.offsets || !dp.ep.ok || dp.diag || dp.split_out) return 0;
    const int ncu = resident_cus();
    const bool narrow = kx_knob(KXK_FAST_NARROW) && dp.winb <= (uint32_t)FWINB;
    const unsigned tiles = (unsigned)(dp.t_hi - dp.t_lo);
    if (narrow)
      hipLaunchKernelGGL((emit_fast_kernel<NV, true>), dim3((tiles + FWAVES - 1) / FWAVES), dim3(FNT), 0, stream, dp);
    else
      hipLaunchKernelGGL((emit_fast_kernel<NV, false>), dim3((tiles + WAVES - 1) / WAVES), dim3(NT), 0, stream, dp);
    if (hipGetLastError() != hipSuccess) return -1;
    const unsigned rgrid = (unsigned)kmin64(grid, (uint64_t)ncu * (uint64_t)kmax64(1, kx_knob(KXK_REDO_WG)));
    if (KX_EMIT_COOP && dp.nlist)
      hipLaunchKernelGGL((emit_redo_kernel<NV, MODE, true>), dim3(rgrid), dim3(NT), 0, stream, dp);
    else
      hipLaunchKernelGGL((emit_redo_kernel<NV, MODE, false>), dim3(rgrid), dim3(NT), 0, stream, dp);
    return hipGetLastError() != hipSuccess ? -1 : 1;
  }
}

// the split fast index pass (index_fast_kernel + redo_kernel) when it applies: 1 launched, 0 not, -1 error
template <int NV, int MODE>
int launch_fast_index(const DecParams& dp, unsigned grid, hipStream_t stream) {
  if constexpr (MODE != M_THRIFT) {
    return 0;
  } else {
    if (!kx_knob(KXK_FAST_SPLIT) || !dp.fast || dp.offsets || (dp.diag & ~(64 | 256 | 1024 | 2048 | 4096))) return 0;
    const int ncu = resident_cus();
    const uint64_t tiles = dp.t_hi - dp.t_lo;
    if (kx_knob(KXK_FAST_NARROW) && dp.winb <= (uint32_t)FWINB) {
      const unsigned fgrid = (unsigned)((tiles + FWAVES - 1) / FWAVES);
      hipLaunchKernelGGL((index_fast_kernel<NV, true>), dim3(fgrid), dim3(FNT), 0, stream, dp);
    } else {
      hipLaunchKernelGGL((index_fast_kernel<NV, false>), dim3((unsigned)((tiles + WAVES - 1) / WAVES)), dim3(NT), 0,
                         stream, dp);
    }
    if (hipGetLastError() != hipSuccess) return -1;
    // the queued tiles: one resident grid's worth of waves at most (4 workgroups per CU)
    const unsigned rgrid = (unsigned)kmin64(grid, (uint64_t)ncu * (uint64_t)kmax64(1, kx_knob(KXK_REDO_WG)));
    hipLaunchKernelGGL((redo_kernel<NV, MODE>), dim3(rgrid), dim3(NT), 0, stream, dp);
    return hipGetLastError() != hipSuccess ? -1 : 1;
  }
}

template <int NV, int MODE>
int launch_t(const DecParams& dp0, const WsLayout& L, void* ws, hipStream_t stream, const KxPipe* pp) {
  DecParams dp = dp0;
  char* base = (char*)ws;
  dp.errkey = (unsigned long long*)(base + 8);
  dp.overflow = (uint32_t*)(base + 16);
  dp.nstop = (uint64_t*)(base + 24);
  dp.nstop_ring = (uint64_t*)(base + WS_RING);
  dp.redo_n = (uint32_t*)(base + WS_REDO);  // reset by finalize_kernel
  dp.redo = (uint32_t*)(base + L.redo);
  dp.carry = (uint64_t*)(base + WS_CARRY);
  dp.tdesc = (uint64_t*)(base + L.tdesc);
  dp.gdesc = (uint64_t*)(base + L.gdesc);
  dp.starts = (uint16_t*)(base + L.starts);
  dp.ntiles = L.ntiles;
  dp.ngroups = L.ngroups;
  dp.slotcap = L.slotcap;
  dp.direct = dp.offsets && (NV == 0 || dp.all_view);  // no arena positions to scan: emit alone
  dp.t_lo = 0; dp.t_hi = dp.ntiles; dp.g_lo = 0; dp.g_hi = dp.ngroups;
  dp.chunk_first = dp.chunk_last = 1;
  KX_HIP_CHECK(hipMemsetAsync(dp.status, 0, sizeof(kx_status), stream));
  const unsigned grid = (unsigned)((dp.ntiles + WAVES - 1) / WAVES);
  const unsigned ggrid = (unsigned)((dp.ngroups + WAVES - 1) / WAVES);
  if (dp.diag & 256) {
    const int lr = launch_fast_index<NV, MODE>(dp, grid, stream);
    if (lr < 0) return KX_ERR_HIP;
    if (lr == 0) hipLaunchKernelGGL((index_kernel<NV, MODE>), dim3(grid), dim3(NT), 0, stream, dp);
    return KX_OK;
  }
  const uint64_t cht = pp && pp->aux ? pp->chunk_tiles : 0;
  if (!dp.direct && cht && dp.ntiles >= 2 * cht) {
    // chunked pipeline: aux stream index + group + chain(k) | caller's stream emit(k - ahead). The chain
    // pass of chunk k runs on the aux stream right after its group pass (it carries its state from chunk
    // k - 1 there) and leaves the chunk's nstop in its own ring slot, so the caller's stream runs nothing
    // but emit passes, each behind the event of its chunk's chain
    const uint64_t nch = (dp.ntiles + cht - 1) / cht;
    const uint64_t D = (uint64_t)(pp->ahead < 0 ? 0 : pp->ahead > KX_PIPE_EV - 2 ? KX_PIPE_EV - 2 : pp->ahead);
    // each chunk queues the tiles its fast index / emit kernels leave in its own part of the redo list,
    // counted in its own block (zeroed here)
    uint32_t* const qcnt = (uint32_t*)(base + L.qcnt);
    uint32_t* const qlist = dp.redo;
    KX_HIP_CHECK(hipMemsetAsync(qcnt, 0, (size_t)nch * 16, stream));
    auto chunk = [&](uint64_t k) {
      DecParams c = chunk_params(dp, k, nch, cht);
      c.nstop = dp.nstop_ring + k % KX_PIPE_EV;
      c.redo = qlist + c.t_lo;
      c.redo_n = qcnt + 4 * k;
      return c;
    };
    KX_HIP_CHECK(hipEventRecord(pp->fork, stream));
    KX_HIP_CHECK(hipStreamWaitEvent(pp->aux, pp->fork, 0));
    for (uint64_t s = 0; s < nch + D; s++) {
      if (s < nch) {
        const uint64_t k = s;
        // the index pass runs at most `ahead` chunks in front of emit (Infinity-Cache residency; the
        // nstop ring slot k % KX_PIPE_EV is free again once emit(k - D - 1) has read it)
        if (k >= D + 1) KX_HIP_CHECK(hipStreamWaitEvent(pp->aux, pp->ev_emit[(k - D - 1) % KX_PIPE_EV], 0));
        const DecParams c = chunk(k);
        const unsigned cg = (unsigned)((c.t_hi - c.t_lo + WAVES - 1) / WAVES);
        const unsigned gg = (unsigned)((c.g_hi - c.g_lo + WAVES - 1) / WAVES);
        const int lr = launch_fast_index<NV, MODE>(c, cg, pp->aux);
        if (lr < 0) return KX_ERR_HIP;
        if (lr == 0) hipLaunchKernelGGL((index_kernel<NV, MODE>), dim3(cg), dim3(NT), 0, pp->aux, c);
        KX_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL((group_kernel<NV, MODE>), dim3(gg), dim3(NT), 0, pp->aux, c);
        KX_HIP_CHECK(hipGetLastError());
        if (int rc = launch_chain<NV, MODE>(c, pp->aux)) return rc;
        KX_HIP_CHECK(hipEventRecord(pp->ev_idx[k % KX_PIPE_EV], pp->aux));
      }
      if (s >= D) {
        const uint64_t k = s - D;
        const DecParams c = chunk(k);
        const unsigned cg = (unsigned)((c.t_hi - c.t_lo + WAVES - 1) / WAVES);
        KX_HIP_CHECK(hipStreamWaitEvent(stream, pp->ev_idx[k % KX_PIPE_EV], 0));
        const int fe = launch_fast_emit<NV, MODE>(c, cg, stream);
        if (fe < 0) return KX_ERR_HIP;
        if (fe == 0) launch_emit<NV, MODE>(dim3(cg), stream, c);
        KX_HIP_CHECK(hipGetLastError());
        KX_HIP_CHECK(hipEventRecord(pp->ev_emit[k % KX_PIPE_EV], stream));
      }
    }
    hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(64), 0, stream, dp.status, dp.errkey, dp.overflow, dp.nstop,
                       dp.offsets, dp.n, dp.redo_n);
    KX_HIP_CHECK(hipGetLastError());
    return KX_OK;
  }
  if (!dp.direct) {
    const int lr = launch_fast_index<NV, MODE>(dp, grid, stream);
    if (lr < 0) return KX_ERR_HIP;
    if (lr == 0) hipLaunchKernelGGL((index_kernel<NV, MODE>), dim3(grid), dim3(NT), 0, stream, dp);
    KX_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL((group_kernel<NV, MODE>), dim3(ggrid), dim3(NT), 0, stream, dp);
    KX_HIP_CHECK(hipGetLastError());
    if (int rc = launch_chain<NV, MODE>(dp, stream)) return rc;
  }
  if constexpr (is_thrift(MODE) || MODE == M_SKIP) {
    if (dp.split_out) {   // split points: the chain pass's tile bases and slots, no emit
      hipLaunchKernelGGL((split_kernel<NV, MODE>), dim3((dp.nsplit + 64) / 64), dim3(64), 0, stream, dp);
      KX_HIP_CHECK(hipGetLastError());
      goto done;
    }
  }
  {
    const int fe = launch_fast_emit<NV, MODE>(dp, grid, stream);
    if (fe < 0) return KX_ERR_HIP;
    if (fe == 0) launch_emit<NV, MODE>(dim3(grid), stream, dp);
  }
  KX_HIP_CHECK(hipGetLastError());
done:
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(64), 0, stream, dp.status, dp.errkey, dp.overflow, dp.nstop,
                     dp.offsets, dp.n, dp.redo_n);
  KX_HIP_CHECK(hipGetLastError());
  return KX_OK;
}

}  // namespace
unsigned long long* kx_phase_buf(int diag);
namespace {
void fill_diag_flags(DecParams& dp) {
  const int diag = kx_knob(KXK_DIAG);
  dp.nolds = kx_knob(KXK_NOLDS) == 1;
  dp.diag = diag;
  dp.phase = kx_phase_buf(diag);
}

}  // namespace

// Split compilation: build.py compiles this file once per part (-DKX_DEC_PART=k, k = 0..7); each
// part instantiates its share of the decode kernels, part 0 also holds the host entry points.
// Without KX_DEC_PART (one translation unit: the emulator build) everything is instantiated here.
#ifndef KX_DEC_PART
#define KX_DEC_PART -1
#endif
#define KX_OWNS(p) (KX_DEC_PART < 0 || KX_DEC_PART == (p))

template <int NV, int MODE>
int kx_dec_launch(const void* dp, const void* L, void* ws, hipStream_t stream, const KxPipe* pp) {
  return launch_t<NV, MODE>(*(const DecParams*)dp, *(const WsLayout*)L, ws, stream, pp);
}
#define KX_DEF(NV, MODE) \
  template int kx_dec_launch<NV, MODE>(const void*, const void*, void*, hipStream_t, const KxPipe*);
#define KX_EXT(NV, MODE) \
  extern template int kx_dec_launch<NV, MODE>(const void*, const void*, void*, hipStream_t, const KxPipe*);
#if KX_OWNS(0)
KX_DEF(0, M_THRIFT) KX_DEF(1, M_THRIFT) KX_DEF(1, M_THRIFT_LS)
#else
KX_EXT(0, M_THRIFT) KX_EXT(1, M_THRIFT) KX_EXT(1, M_THRIFT_LS)
#endif
#if KX_OWNS(1)
KX_DEF(2, M_THRIFT) KX_DEF(0, M_SKIP) KX_DEF(0, M_FRAME)
#else
KX_EXT(2, M_THRIFT) KX_EXT(0, M_SKIP) KX_EXT(0, M_FRAME)
#endif
#if KX_OWNS(2)
KX_DEF(4, M_THRIFT) KX_DEF(2, M_THRIFT_LS)
#else
KX_EXT(4, M_THRIFT) KX_EXT(2, M_THRIFT_LS)
#endif
#if KX_OWNS(3)
KX_DEF(8, M_THRIFT) KX_DEF(4, M_THRIFT_LS)
#else
KX_EXT(8, M_THRIFT) KX_EXT(4, M_THRIFT_LS)
#endif
#if KX_OWNS(5)
KX_DEF(8, M_THRIFT_LS)
#else
KX_EXT(8, M_THRIFT_LS)
#endif
#if KX_OWNS(6)
KX_DEF(16, M_THRIFT)
#else
KX_EXT(16, M_THRIFT)
#endif
#if KX_OWNS(7)
KX_DEF(16, M_THRIFT_LS)
#else
KX_EXT(16, M_THRIFT_LS)
#endif
#if KX_OWNS(4)
KX_DEF(0, M_PB) KX_DEF(1, M_PB) KX_DEF(2, M_PB) KX_DEF(0, M_PBB)
#else
KX_EXT(0, M_PB) KX_EXT(1, M_PB) KX_EXT(2, M_PB) KX_EXT(0, M_PBB)
#endif
#if KX_OWNS(5)
KX_DEF(4, M_PB) KX_DEF(8, M_PB)
#else
KX_EXT(4, M_PB) KX_EXT(8, M_PB)
#endif

#if KX_DEC_PART <= 0
template <int MODE>
static int launch_nv(const DecParams& dp, const WsLayout& L, void* ws, hipStream_t stream, uint32_t nvar,
                     const KxPipe* pp) {
  if constexpr (MODE == M_THRIFT_LS) {  // a list<struct> field holds >= 1 var slot
    switch (nvar) {
      case 0: case 1: return kx_dec_launch<1, M_THRIFT_LS>(&dp, &L, ws, stream, pp);
      case 2: return kx_dec_launch<2, M_THRIFT_LS>(&dp, &L, ws, stream, pp);
      case 3: case 4: return kx_dec_launch<4, M_THRIFT_LS>(&dp, &L, ws, stream, pp);
      case 5: case 6: case 7: case 8: return kx_dec_launch<8, M_THRIFT_LS>(&dp, &L, ws, stream, pp);
      default: return kx_dec_launch<16, M_THRIFT_LS>(&dp, &L, ws, stream, pp);
    }
  } else {
    switch (nvar) {
      case 0: return kx_dec_launch<0, MODE>(&dp, &L, ws, stream, pp);
      case 1: return kx_dec_launch<1, MODE>(&dp, &L, ws, stream, pp);
      case 2: return kx_dec_launch<2, MODE>(&dp, &L, ws, stream, pp);
      case 3: case 4: return kx_dec_launch<4, MODE>(&dp, &L, ws, stream, pp);
      case 5: case 6: case 7: case 8: return kx_dec_launch<8, MODE>(&dp, &L, ws, stream, pp);
      default:   // 9..16 var slots: Thrift only (Kitex-Protobuf flat schemas keep <= 8, kx_capi.cpp pb_flat_ok)
        if constexpr (MODE == M_THRIFT) return kx_dec_launch<16, MODE>(&dp, &L, ws, stream, pp);
        else return KX_ERR_NOT_IMPLEMENTED;
    }
  }
}

size_t kx_decode_ws_bytes(const KxProgram& hprog, uint64_t in_len, const uint64_t* offsets, uint64_t n) {
  return ws_layout(hprog.fixed_min, in_len, offsets, n).total;
}

// diagnostics (not part of the public ABI): read and reset the phase-timing accumulators
unsigned long long* kx_phase_buf(int diag) {
  static unsigned long long* buf = nullptr;
  if (!buf && (diag & 64)) {
    if (hipMalloc((void**)&buf, 8 * sizeof(unsigned long long)) != hipSuccess) return nullptr;
    if (hipMemset(buf, 0, 8 * sizeof(unsigned long long)) != hipSuccess) return nullptr;
  }
  return buf;
}

extern "C" int kx_debug_phase_cycles(unsigned long long* out, int n) {
  if (n > 8) n = 8;
  unsigned long long* b = kx_phase_buf(64);
  if (!b) return KX_ERR_HIP;
  if (hipMemcpy(out, b, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost) != hipSuccess) return KX_ERR_HIP;
  if (hipMemset(b, 0, 8 * sizeof(unsigned long long)) != hipSuccess) return KX_ERR_HIP;
  return KX_OK;
}

size_t kx_skip_ws_bytes(uint64_t in_len, uint64_t n) { return ws_layout(1, in_len, nullptr, n).total; }

// window bytes per tile: a halo of about two mean records (the walk of a tile's last records stays in
// LDS: R3's 576-byte records left the 512-byte halo and walked global memory), 512 .. HALO_MAX
static uint32_t win_bytes(uint64_t in_len, uint64_t n) {
  const uint64_t mean = n ? in_len / n : 0;
  uint64_t h = (2 * mean + 255) & ~255ull;
  h = h < (uint64_t)HALO ? (uint64_t)HALO : h > (uint64_t)HALO_MAX ? (uint64_t)HALO_MAX : h;
  return (uint32_t)(TILE + h + 16);
}

int kx_launch_decode(const KxProgram* dprog, const KxProgram& hprog, const uint8_t* in, uint64_t in_len,
                     const uint64_t* offsets, uint64_t n, const KxLaunchCols& cols, uint8_t* record_status,
                     kx_status* status, void* ws, size_t ws_size, uint64_t epoch, hipStream_t stream, bool pb,
                     const uint64_t* ends, const uint64_t* var_base, const KxPipe* pipe,
                     const uint64_t* var_base_dev) {
  DecParams dp{};
  fill_diag_flags(dp);
  if (var_base)
    for (int v = 0; v < KXP_NV_MAX; v++) dp.var_base[v] = var_base[v];
  dp.var_base_dev = var_base_dev;
  dp.in = in; dp.in_len = in_len; dp.offsets = offsets; dp.ends = offsets ? ends : nullptr; dp.n = n;
  dp.prog = (const KAS KxProgram*)dprog;
  dp.cols = cols; dp.rstat = record_status; dp.status = status; dp.epoch = epoch;
  dp.krec = krec_for(in_len, n);
  dp.winb = win_bytes(in_len, n);
  dp.all_view = 1;
  for (uint32_t v = 0; v < hprog.nvar; v++) dp.all_view &= (int)((cols.view >> hprog.var_col[v]) & 1);
  {
    // concatenated: the fast index path; known offsets: the fast record measure (index) pass
    dp.fast = kx_knob(KXK_FAST) && !pb && hprog.nsteps && (offsets || hprog.sig_len == 3);
    if (dp.fast && kx_knob(KXK_FASTPLAN)) kxp_fast_plan(hprog, dp.fp);
    if (dp.fast && !pb && !offsets) {
      kxp_emit_plan(hprog, dp.ep);
      // every var slot is a string, or a numeric list absent from the plan (its records hold none): the
      // fast emit pass writes each slot's record offsets with no container logic
      for (uint32_t v = 0; v < hprog.nvar && dp.ep.ok; v++) {
        const KxpCol& K = hprog.col[hprog.var_col[v]];
        if (!(K.kind == KXP_K_BYTES || (K.kind == KXP_K_LIST && !K.mside))) dp.ep.ok = 0;
      }
    }
  }
  for (uint32_t c = 0; c < hprog.ncols; c++) {
    const KxpCol& K = hprog.col[c];
    dp.nlist += K.kind == KXP_K_LIST && K.width > 1 && !K.mside && !((cols.view >> c) & 1);
  }
  const WsLayout L = ws_layout(hprog.fixed_min, in_len, offsets, n);
  if (ws_size < L.total) return KX_ERR_INVALID_ARG;
  bool ls = false;
  for (uint32_t f = 0; f < hprog.nfields; f++) ls |= hprog.f[f].kind == KXP_K_LSTRUCT;
  return pb ? launch_nv<M_PB>(dp, L, ws, stream, hprog.nvar, pipe)
            : ls ? launch_nv<M_THRIFT_LS>(dp, L, ws, stream, hprog.nvar, pipe)
                 : launch_nv<M_THRIFT>(dp, L, ws, stream, hprog.nvar, pipe);
}

// split points: a flat Thrift schema's own index pass (its fast path included), or the schema-free skip
// walker (dprog null: nested schemas); every column a view, so no pass writes a column
int kx_launch_split(const KxProgram* dprog, const KxProgram* hprog, const uint8_t* in, uint64_t in_len, uint64_t n,
                    uint32_t parts, uint64_t* points, kx_status* status, void* ws, size_t ws_size, uint64_t epoch,
                    hipStream_t stream) {
  DecParams dp{};
  fill_diag_flags(dp);
  dp.in = in; dp.in_len = in_len; dp.n = n; dp.status = status; dp.epoch = epoch;
  dp.split_out = points; dp.nsplit = parts;
  dp.krec = 64;
  dp.cols.view = ~0u;
  const WsLayout L = ws_layout(1, in_len, nullptr, n);
  if (ws_size < L.total) return KX_ERR_INVALID_ARG;
  if (!dprog) {
    dp.winb = TILE + HALO + 16;
    return kx_dec_launch<0, M_SKIP>(&dp, &L, ws, stream, nullptr);
  }
  dp.prog = (const KAS KxProgram*)dprog;
  dp.winb = win_bytes(in_len, n);
  dp.fast = kx_knob(KXK_FAST) && hprog->nsteps && hprog->sig_len == 3;
  bool ls = false;
  for (uint32_t f = 0; f < hprog->nfields; f++) ls |= hprog->f[f].kind == KXP_K_LSTRUCT;
  return ls ? launch_nv<M_THRIFT_LS>(dp, L, ws, stream, hprog->nvar, nullptr)
            : launch_nv<M_THRIFT>(dp, L, ws, stream, hprog->nvar, nullptr);
}

int kx_launch_skip(const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t* offsets_out, kx_status* status,
                   void* ws, size_t ws_size, uint64_t epoch, hipStream_t stream) {
  DecParams dp{};
  fill_diag_flags(dp);
  dp.in = in; dp.in_len = in_len; dp.offsets = nullptr; dp.n = n; dp.prog = nullptr;
  dp.status = status; dp.skip_out = offsets_out; dp.epoch = epoch;
  dp.krec = 64;
  dp.winb = TILE + HALO + 16;
  const WsLayout L = ws_layout(1, in_len, nullptr, n);
  if (ws_size < L.total) return KX_ERR_INVALID_ARG;
  return kx_dec_launch<0, M_SKIP>(&dp, &L, ws, stream, nullptr);
}

int kx_launch_pb_frames(const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t* frame_offsets, uint64_t* body_start,
                        uint64_t* body_end, kx_status* status, void* ws, size_t ws_size, uint64_t epoch,
                        hipStream_t stream) {
  DecParams dp{};
  fill_diag_flags(dp);
  dp.in = in; dp.in_len = in_len; dp.offsets = nullptr; dp.n = n; dp.prog = nullptr;
  dp.status = status; dp.skip_out = frame_offsets; dp.epoch = epoch;
  dp.fr_ps = body_start; dp.fr_pe = body_end; dp.fr_grpc = 3;
  dp.krec = 64;
  dp.winb = TILE + HALO + 16;
  const WsLayout L = ws_layout(1, in_len, nullptr, n);
  if (ws_size < L.total) return KX_ERR_INVALID_ARG;
  return kx_dec_launch<0, M_PBB>(&dp, &L, ws, stream, nullptr);
}

int kx_launch_frames(const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t max_payload, uint64_t* frame_offsets,
                     uint64_t* pay_start, uint64_t* pay_end, uint8_t* kinds, kx_status* status, void* ws,
                     size_t ws_size, uint64_t epoch, hipStream_t stream, bool grpc, const kx_ttstream_keys* tts,
                     int32_t* sids, uint64_t* mpos, uint32_t* mlen, uint8_t* crc_codes) {
  DecParams dp{};
  dp.fr_crc = crc_codes;
  fill_diag_flags(dp);
  dp.in = in; dp.in_len = in_len; dp.offsets = nullptr; dp.n = n; dp.prog = nullptr;
  dp.status = status; dp.skip_out = frame_offsets; dp.epoch = epoch;
  dp.fr_ps = pay_start; dp.fr_pe = pay_end; dp.fr_kind = kinds; dp.fr_max = max_payload;
  dp.fr_grpc = tts ? 2 : grpc ? 1 : 0;
  if (tts) {
    dp.fr_sid = sids; dp.fr_mpos = mpos; dp.fr_mlen = mlen;
    dp.tts_keys = (uint32_t)tts->frame_type_key | ((uint32_t)tts->to_method_key << 16);
    dp.tts_flag = tts->streaming_flag;
    for (int k = 0; k < 5; k++) {
      uint64_t v = 0;
      uint32_t l = 0;
      while (l < 8 && tts->type_names[k][l]) { v |= (uint64_t)(uint8_t)tts->type_names[k][l] << (8 * l); l++; }
      dp.tts_name[k] = v;
      dp.tts_nlen[k] = l;
    }
  }
  dp.krec = 64;
  dp.winb = TILE + HALO + 16;
  const WsLayout L = ws_layout(1, in_len, nullptr, n);
  if (ws_size < L.total) return KX_ERR_INVALID_ARG;
  return kx_dec_launch<0, M_FRAME>(&dp, &L, ws, stream, nullptr);
}
#endif  // KX_DEC_PART <= 0
