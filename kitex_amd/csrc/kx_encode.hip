// kx_encode.hip — batched BLength + FastWriteNocopy (Thrift binary) on CDNA4 / gfx950.
//
// Reference: generated FastWriteNocopy / BLength (tool/internal_pkg/pluginmode/thriftgo/
// struct_tpl.go:225-391, 948-1061; instance internal/mocks/thrift/k-mock.go:190-277): fields in
// encoder order (fixed-length first, reorderStructFields patcher.go:503-522), optional fields only
// when set, a nil struct as STOP, lists as header + elements, STOP last.
//
// Pipeline (the reference's size -> write structure mapped onto the GPU):
//   1. size_kernel: one lane per record computes BLength from the columns (offset diffs, presence);
//      per 1024-record block totals go to the workspace (sizes_out optional);
//   2. scan_kernel: one workgroup turns block totals into block bases;
//   3. write_kernel: each workgroup re-derives its records' sizes, scans them and writes as many
//      records as fit into an LDS image aligned like the destination (mod 16), then streams the
//      image to HBM with 16-byte stores. Bytes inside a record are packed into dwords in registers
//      before they touch LDS.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "kx_internal.h"
#include "kx_mem.h"

namespace {

constexpr int NT = 256;
constexpr int RB = 1024;             // records per block
#ifndef KX_ENC_WT
#define KX_ENC_WT 256
#endif
// tuning switches (A/B builds): list elements loaded in blocks of 4 (on: R3 encode 9.35 -> 6.35 ms on the
// MI355X, R2 unchanged) / min waves per SIMD of the write pass (4 spills registers: no gain)
// output dwords per lane in flight in the direct path's payload copy
#ifndef KX_ENC_WCU
#define KX_ENC_WCU 4
#endif
// 16-byte output chunks per lane in flight in the chunked payload copy (KX_ENC_WCU=16)
#ifndef KX_ENC_WCU16
#define KX_ENC_WCU16 4
#endif
// list<scalar> elements per block in the canonical writer (loads of a block all issued before the first
// element is written)
#ifndef KX_ENC_LISTB
#define KX_ENC_LISTB 4
#endif
#ifndef KX_ENC_LISTPF
#define KX_ENC_LISTPF 1
#endif
// the write pass stages a round through the LDS image when at least cnt >> KX_ENC_MINTAKE of its records fit
// (round 3, 2 = a quarter: R3 encode 5.91 -> 5.34 ms while the direct path copied one payload at a time;
// round 4, 1 = half: with the streamed payload copy the direct path takes R3 in 3.22 ms against the
// image's 5.30, R2 (303-byte records) stays on the image, 2.30 ms against 6.60 direct)
#ifndef KX_ENC_MINTAKE
#define KX_ENC_MINTAKE 1
#endif
#ifndef KX_ENC_OUTB
#define KX_ENC_OUTB (48 * 1024)
#endif
constexpr int WT = KX_ENC_WT;        // write pass: threads per workgroup (records per round)
constexpr int OUTB = KX_ENC_OUTB;    // LDS image bytes per round

struct EncParams {
  const KxProgram* prog;
  KxLaunchCols cols;
  uint64_t n;
  uint8_t* out;
  uint64_t out_cap;
  uint64_t* sizes_out;
  uint64_t* offsets_out;
  kx_status* status;
  uint64_t* block_tot;   // workspace: per-block total size, then (after scan) block base
  const uint64_t* out_base;  // device: where this call's first record goes in `out` (a chunk of a larger
                             // batch: the previous chunk's status->consumed), null = 0
  uint64_t nblocks;
  bool pb;               // Kitex-Protobuf records (Batch framing) instead of Thrift binary
  int direct;            // tuning (KX_ENC_DIRECT=1): every round writes straight to HBM
  int wcu;               // tuning (KX_ENC_WCU): the queue copy: 16 (default) 16-byte chunks, 4 dwords, 1 per item
};

// record offsets are 4 or 8 bytes wide (kx_column.offset_bytes)
__device__ __forceinline__ uint64_t off_at(const KxLaunchCols& C, int col, uint64_t r) {
  return ((C.owide >> col) & 1) ? kx_ld((const uint64_t*)C.offs[col] + r) : (uint64_t)kx_ld((const uint32_t*)C.offs[col] + r);
}

__device__ __forceinline__ uint64_t var_len(const KxLaunchCols& C, int col, uint64_t r) {
  return off_at(C, col, r + 1) - off_at(C, col, r);
}

// LIST_BYTES columns: element byte offsets (same width as the record offsets)
__device__ __forceinline__ uint64_t eoff_at(const KxLaunchCols& C, int col, uint64_t i) {
  return ((C.owide >> col) & 1) ? kx_ld((const uint64_t*)C.eoffs[col] + i) : (uint64_t)kx_ld((const uint32_t*)C.eoffs[col] + i);
}

// encoded bytes of elements [E, E + cnt) of a container column side: fixed width or strings
__device__ __forceinline__ uint64_t side_bytes(const KxProgram& P, const KxLaunchCols& C, int col, uint64_t E,
                                               uint64_t cnt) {
  const KxpCol& K = P.col[col];
  if (K.kind == KXP_K_LISTB) return 4 * cnt + eoff_at(C, col, E + cnt) - eoff_at(C, col, E);
  return cnt * K.width;
}

// BLength (struct_tpl.go:266-391)
// LS: the schema has list<struct> fields (a separate instantiation: the extra branch changes the
// register allocation of the write pass, which ran 2.4x slower for every schema with it compiled in)
template <bool LS>
__device__ __forceinline__ uint64_t record_size(const KxProgram& P, const KxLaunchCols& C, uint64_t r) {
  uint64_t pres = C.presence ? kx_ld(C.presence + r) : 0;
  int inst = 0;
  int f = P.inst[0].enc_first;
  uint64_t sz = 0;
  for (;;) {
    if (f < 0) {
      sz += 1;                                   // STOP
      if (inst == 0) break;
      f = P.inst[inst].ret_pred;
      inst = P.inst[inst].parent;
      continue;
    }
    const KxpField F = P.f[f];
    if (F.req == KX_REQ_OPTIONAL && !((pres >> F.pbit) & 1)) { f = F.enc_next; continue; }
    sz += 3;
    if (F.kind == KXP_K_FIXED) sz += F.width;
    else if (F.kind == KXP_K_BYTES) sz += 4 + var_len(C, F.col, r);
    else if (F.kind == KXP_K_LIST) sz += 5 + var_len(C, F.col, r) * F.width;
    else if (LS && F.kind == KXP_K_LSTRUCT) {  // list/set<S>: every field of S + STOP per element
      uint64_t es = 1;
      for (int c = F.col; c < F.col + F.width; c++) es += 3 + P.col[c].width;
      sz += 5 + var_len(C, F.col, r) * es;
    } else if (F.kind == KXP_K_LISTB)  // list/set<string> (FieldListLength, struct_tpl.go:1038-1061)
      sz += 5 + side_bytes(P, C, F.col, off_at(C, F.col, r), var_len(C, F.col, r));
    else if (F.kind == KXP_K_MAP) {  // map (FieldMapLength): both sides, the keys' entry count
      const uint64_t cnt = var_len(C, F.col, r);
      sz += 6 + side_bytes(P, C, F.col, off_at(C, F.col, r), cnt) +
            side_bytes(P, C, F.col + 1, off_at(C, F.col + 1, r), cnt);
    } else {
      if ((pres >> F.pbit) & 1) { inst = F.child; f = P.inst[inst].enc_first; continue; }
      sz += 1;                                   // nil *T -> STOP only (k-mock.go:190-199)
    }
    f = F.enc_next;
  }
  return sz;
}

// ---- byte sink: packs bytes into aligned dwords before writing LDS (or global on the direct path).
// The sink is kept dword-aligned from the start: `head` bytes of the first dword belong to the
// previous record (another lane), so that dword is written byte by byte and every later one whole.
// A put of k bytes stores at most one dword and has no loop, so lanes whose records start at
// different alignments only differ in a predicated store (the old byte-draining loop diverged on
// every field).
typedef __attribute__((address_space(3))) uint8_t LDSB;  // the LDS image (ds_write, not flat stores)

template <class B>
struct SinkT {
  B* base;         // LDS image or global output
  uint64_t off;    // dword-aligned position of the pending bytes
  uint64_t acc;    // pending bytes (including `head` placeholder bytes), first in bits 0..7
  uint32_t n;      // pending bytes (< 4 between puts)
  uint32_t head;   // leading bytes of the first dword not owned by this record (0 once it is written)

  __device__ __forceinline__ SinkT(B* b, uint64_t o)
      : base(b), off(o & ~3ull), acc(0), n((uint32_t)(o & 3)), head((uint32_t)(o & 3)) {}

  __device__ __forceinline__ void emit_dword() {
    const uint32_t v = (uint32_t)acc;
    if (head) {
      for (uint32_t k = head; k < 4; k++) base[off + k] = (uint8_t)(v >> (8 * k));
      head = 0;
    } else {
      *(typename std::conditional<std::is_same<B, LDSB>::value, __attribute__((address_space(3))) uint32_t,
                                  KX_GLOBAL uint32_t>::type*)(base + off) = v;
    }
    off += 4; acc >>= 32; n -= 4;
  }
  // append k (1..4) bytes, first byte in bits 0..7 of v
  __device__ __forceinline__ void put(uint32_t v, uint32_t k) {
    acc |= (uint64_t)(k == 4 ? v : (v & ((1u << (8 * k)) - 1))) << (8 * n);
    n += k;
    if (n >= 4) emit_dword();
  }
  __device__ __forceinline__ void flush() {
    for (uint32_t k = head; k < n; k++) base[off + k] = (uint8_t)(acc >> (8 * k));
    off += n; acc = 0; n = 0; head = 0;
  }
  // the position of the next byte
  __device__ __forceinline__ uint64_t pos() const { return off + n; }
};
typedef KX_GLOBAL uint8_t GB;   // global output (global_store, not flat)
using Sink = SinkT<GB>;        // global (the direct path)
using LSink = SinkT<LDSB>;     // the LDS image

template <class SK>
__device__ __forceinline__ void put_be(SK& s, uint64_t v, uint32_t w) {
  switch (w) {
    case 1: s.put((uint32_t)v, 1); break;
    case 2: s.put(((uint32_t)v >> 8 & 0xff) | (((uint32_t)v & 0xff) << 8), 2); break;
    case 4: s.put(__builtin_bswap32((uint32_t)v), 4); break;
    default: {
      s.put(__builtin_bswap32((uint32_t)(v >> 32)), 4);
      s.put(__builtin_bswap32((uint32_t)v), 4);
    }
  }
}

__device__ __forceinline__ uint64_t load_fixed(const void* base, uint32_t w, uint64_t i) {
  switch (w) {
    case 1: return kx_ld((const uint8_t*)base + i);
    case 2: return kx_ld((const uint16_t*)base + i);
    case 4: return kx_ld((const uint32_t*)base + i);
    default: return kx_ld((const uint64_t*)base + i);
  }
}

// raw bytes into the sink: blocks of up to 64 bytes whose dword loads are all issued before the first
// is used (one memory round trip per block instead of one per 4 bytes: the encoder's write pass was
// latency-bound on these loads)
template <class SK>
__device__ __forceinline__ void put_bytes(SK& s, const uint8_t* src, uint32_t len) {
  const uint64_t sa = (uint64_t)src, se = sa + len;
  const uint32_t sh = (uint32_t)(sa & 3);
  uint64_t A = sa & ~3ull;  // aligned dwords that hold string bytes only
  uint32_t done = 0;
  while (done + 4 <= len) {
    const uint32_t units = min((len - done) >> 2, 16u);
    uint32_t W[17];
#pragma unroll
    for (int j = 0; j < 17; j++) W[j] = ((uint32_t)j <= units && A + 4 * j < se) ? kx_ld((const uint32_t*)(A + 4 * j)) : 0u;
#pragma unroll
    for (int u = 0; u < 16; u++)
      if ((uint32_t)u < units) s.put(sh ? __builtin_amdgcn_alignbyte(W[u + 1], W[u], sh) : W[u], 4);
    A += 4 * units;
    done += 4 * units;
  }
  for (; done < len; done++) s.put(src[done], 1);
}

// ---- wave-cooperative payload copies (the direct write path) ----
// A lane writing its record straight to HBM leaves the bulk of it -- list elements and long strings --
// to its whole wave: it flushes its sink before the payload, queues (destination, source, count, element
// width) in the wave's LDS queue and restarts the sink after it. The wave then copies every queued payload
// with all 64 lanes: lane k assembles aligned output dword k of the payload's big-endian byte stream from
// the (coalesced) source elements and stores it, so each store instruction writes 256 contiguous bytes
// instead of one dword in each of 64 records. Edge dwords shared with the record's own bytes are written
// byte by byte, so no store ever covers a byte another store writes.
constexpr int QCAP = 128;            // queued payloads per wave (a full queue: the lane copies inline)
constexpr uint32_t DEFER_MIN = 32;   // strings shorter than this stay in the lane's sink

struct PayItem {
  uint64_t dst;      // output position (absolute address)
  uint64_t src;      // source elements (absolute address)
  uint32_t n;        // elements
  uint32_t w;        // element width (1: raw bytes, 2 / 4 / 8: big-endian scalars)
};

struct PayQueue {
  PayItem* q;        // this wave's LDS queue (QCAP items)
  uint32_t* cnt;     // LDS counter
};

// the aligned source dword i of a payload's big-endian byte stream (i < ceil(n * w / 4))
__device__ __forceinline__ uint32_t be_stream_dword(const PayItem& it, uint64_t i) {
  const uint64_t total = (uint64_t)it.n * it.w;
  const uint64_t b = 4 * i;
  if (b >= total) return 0u;
  if (it.w == 8) {
    const uint64_t v = kx_ld<uint64_t>(it.src + 8 * (i >> 1));
    return __builtin_bswap32((i & 1) ? (uint32_t)v : (uint32_t)(v >> 32));
  }
  if (it.w == 4) return __builtin_bswap32(kx_ld<uint32_t>(it.src + 4 * i));
  if (it.w == 2) {
    const uint32_t lo = kx_ld<uint16_t>(it.src + 4 * i);
    const uint32_t hi = b + 2 < total ? kx_ld<uint16_t>(it.src + 4 * i + 2) : 0u;
    return ((lo >> 8) | ((lo & 0xff) << 8)) | (((hi >> 8) | ((hi & 0xff) << 8)) << 16);
  }
  // raw bytes: the source may be unaligned; never read past its last byte's dword
  const uint64_t a = it.src + b;
  const uint64_t A = a & ~3ull, end = it.src + total;
  const uint32_t x0 = kx_ld<uint32_t>(A);
  const uint32_t x1 = A + 4 < end ? kx_ld<uint32_t>(A + 4) : 0u;
  return __builtin_amdgcn_alignbyte(x1, x0, (uint32_t)(a & 3));
}

__device__ __forceinline__ void wave_copy(const PayItem& it, int lane) {
  const uint64_t total = (uint64_t)it.n * it.w;
  if (!total) return;
  const uint64_t d0 = it.dst, d1 = it.dst + total;
  const uint64_t A0 = d0 & ~3ull;
  const uint64_t nd = (((d1 + 3) & ~3ull) - A0) >> 2;          // output dwords touched
  const uint32_t sh = (uint32_t)(d0 & 3);                       // stream byte p sits at output A0 + sh + p
  for (uint64_t k = (uint64_t)lane; k < nd; k += 64) {
    // output dword k = stream bytes [4k - sh, 4k - sh + 4)
    uint32_t v;
    if (sh == 0) {
      v = be_stream_dword(it, k);
    } else {
      const uint32_t lo = k ? be_stream_dword(it, k - 1) : 0u;
      const uint32_t hi = be_stream_dword(it, k);
      v = __builtin_amdgcn_alignbyte(hi, lo, 4 - sh);
    }
    const uint64_t a = A0 + 4 * k;
    if (a >= d0 && a + 4 <= d1) {
      kx_st<uint32_t>(a, v);
    } else {
      for (int j = 0; j < 4; j++)
        if (a + j >= d0 && a + j < d1) kx_st<uint8_t>(a + j, (uint8_t)(v >> (8 * j)));
    }
  }
}

// output dwords a payload touches
__device__ __forceinline__ uint64_t item_dwords(const PayItem& it) {
  const uint64_t total = (uint64_t)it.n * it.w;
  if (!total) return 0;
  const uint64_t d0 = it.dst, d1 = it.dst + total;
  return (((d1 + 3) & ~3ull) - (d0 & ~3ull)) >> 2;
}

// every queued payload of the wave as one stream of output dwords (the payloads one after another):
// lane l takes dwords base + 64u + l, u < U, all U loads issued before the first store, so a wave has U
// (2U when unaligned) loads in flight instead of one per payload (wave_copy's loop waits on each load
// before its store: a chain of about 2 memory round trips per list). pre: this wave's LDS array of
// QCAP + 1 payload starts (in dwords).
template <int U>
__device__ __forceinline__ void wave_copy_queue(const PayItem* q, uint32_t nq, int lane, uint64_t* pre) {
  const uint64_t n0 = (uint32_t)lane < nq ? item_dwords(q[lane]) : 0;
  const uint64_t n1 = (uint32_t)lane + 64 < nq ? item_dwords(q[lane + 64]) : 0;
  uint64_t i0 = n0, i1 = n1;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t o0 = __shfl_up(i0, d, 64), o1 = __shfl_up(i1, d, 64);
    if (lane >= d) { i0 += o0; i1 += o1; }
  }
  const uint64_t t0 = __shfl(i0, 63, 64);
  i1 += t0;
  const uint64_t total = __shfl(i1, 63, 64);
  if (lane == 0) pre[0] = 0;
  pre[lane + 1] = i0;
  pre[lane + 65] = i1;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  // Each output dword is two aligned source dwords, loaded unconditionally (addresses clamped into the
  // payload) after the address arithmetic, and assembled only after all 2U loads are out: a load inside
  // a data-dependent branch (be_stream_dword's width switch) is waited for inside that branch, which left
  // one load in flight. i64 / i32 payloads: stream dword s is source dword s ^ 1 / s, byte-swapped;
  // bytes: two aligned dwords around the stream position. i16 payloads (rare) are copied per payload
  // after the stream.
  uint32_t it = 0;
  for (uint64_t base = 0; base < total; base += 64 * U) {
    uint32_t d0[U], d1[U], m[U], mode[U];
    int32_t r[U];
    uint64_t a[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = base + 64 * u + (uint64_t)lane;
      const uint64_t jj = j < total ? j : total - 1;
      while (pre[it + 1] <= jj) it++;
      const PayItem im = q[it];
      const uint64_t k = jj - pre[it];
      const uint64_t tb = (uint64_t)im.n * im.w;              // >= 1: an empty payload owns no dword
      const uint64_t o0 = im.dst, o1 = o0 + tb;
      const int64_t qs = (int64_t)(4 * k) - (int64_t)(o0 & 3);  // stream byte under output byte 0
      uint64_t x0, x1;
      if (im.w <= 2) {
        const uint64_t sp = im.src + (uint64_t)(qs > 0 ? qs : 0);
        const uint64_t last = (im.src + tb - 1) & ~3ull;
        x0 = sp & ~3ull;
        x1 = x0 + 4 <= last ? x0 + 4 : last;
        r[u] = (int32_t)((int64_t)(im.src + (uint64_t)qs) - (int64_t)x0);  // < 0 only at k = 0
        mode[u] = 1;
      } else {
        const int64_t s0 = qs >= 0 ? qs >> 2 : -1;              // stream dwords s0, s0 + 1
        const uint64_t nd = tb >> 2;                             // source dwords (tb % 4 == 0)
        const uint64_t c0 = s0 < 0 ? 0 : (uint64_t)s0 < nd ? (uint64_t)s0 : nd - 1;
        const uint64_t c1 = (uint64_t)(s0 + 1) < nd ? (uint64_t)(s0 + 1) : nd - 1;
        const uint64_t f = im.w == 8 ? 1u : 0u;
        x0 = im.src + 4 * (c0 ^ f);
        x1 = im.src + 4 * (c1 ^ f);
        r[u] = (int32_t)(qs - 4 * s0);
        mode[u] = s0 < 0 ? 2u : 0u;                              // 2: stream dword s0 precedes the payload
      }
      a[u] = (o0 & ~3ull) + 4 * k;
      uint32_t mm = 0;
#pragma unroll
      for (int b = 0; b < 4; b++) mm |= (a[u] + b >= o0 && a[u] + b < o1) ? 1u << b : 0u;
      m[u] = (j < total && im.w != 2) ? mm : 0u;
      d0[u] = kx_ld<uint32_t>(x0);
      d1[u] = kx_ld<uint32_t>(x1);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      uint32_t v;
      if (mode[u] == 1) {
        const uint64_t W = (uint64_t)d0[u] | ((uint64_t)d1[u] << 32);
        v = r[u] < 0 ? (uint32_t)(W << (-8 * r[u])) : (uint32_t)(W >> (8 * r[u]));
      } else {
        const uint64_t W = (uint64_t)(mode[u] == 2 ? 0u : __builtin_bswap32(d0[u])) |
                           ((uint64_t)__builtin_bswap32(d1[u]) << 32);
        v = (uint32_t)(W >> (8 * r[u]));
      }
      if (m[u] == 15u) {
        kx_st<uint32_t>(a[u], v);
      } else if (m[u]) {
        for (int b = 0; b < 4; b++)
          if ((m[u] >> b) & 1) kx_st<uint8_t>(a[u] + b, (uint8_t)(v >> (8 * b)));
      }
    }
  }
  for (uint32_t i = 0; i < nq; i++)
    if (q[i].w == 2) wave_copy(q[i], lane);
}

// 16-byte aligned output chunks a payload touches
__device__ __forceinline__ uint64_t item_chunks(const PayItem& it) {
  const uint64_t total = (uint64_t)it.n * it.w;
  if (!total) return 0;
  const uint64_t d0 = it.dst, d1 = it.dst + total;
  return (((d1 + 15) & ~15ull) - (d0 & ~15ull)) >> 4;
}

// wave_copy_queue with 16-byte output units: lane l takes aligned chunks base + 64u + l, each assembled
// from 5 aligned source dwords (i64 / i32: stream dword s = source dword s ^ 1 / s, byte-swapped; bytes:
// the dwords around the chunk's first source byte) and stored with one 16-byte store when the chunk is
// inside the payload (the chunks at a payload's two ends are stored dword / byte by byte).
template <int U>
__device__ __forceinline__ void wave_copy_queue16(const PayItem* q, uint32_t nq, int lane, uint64_t* pre) {
  const uint64_t n0 = (uint32_t)lane < nq ? item_chunks(q[lane]) : 0;
  const uint64_t n1 = (uint32_t)lane + 64 < nq ? item_chunks(q[lane + 64]) : 0;
  uint64_t i0 = n0, i1 = n1;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t o0 = __shfl_up(i0, d, 64), o1 = __shfl_up(i1, d, 64);
    if (lane >= d) { i0 += o0; i1 += o1; }
  }
  const uint64_t t0 = __shfl(i0, 63, 64);
  i1 += t0;
  const uint64_t total = __shfl(i1, 63, 64);
  if (lane == 0) pre[0] = 0;
  pre[lane + 1] = i0;
  pre[lane + 65] = i1;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  uint32_t it = 0;
  for (uint64_t base = 0; base < total; base += 64 * U) {
    uint32_t x[U][5], bsw[U], r[U], lo[U], hi[U];
    uint64_t a[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t j = base + 64 * u + (uint64_t)lane;
      const uint64_t jj = j < total ? j : total - 1;
      while (pre[it + 1] <= jj) it++;
      const PayItem im = q[it];
      const uint64_t k = jj - pre[it];
      const uint64_t tb = (uint64_t)im.n * im.w;
      const uint64_t o0 = im.dst, o1 = o0 + tb;
      a[u] = (o0 & ~15ull) + 16 * k;
      const int64_t qs = (int64_t)(a[u] - o0);                 // stream byte under the chunk's byte 0
      // chunk bytes [lo, hi) belong to the payload
      lo[u] = qs < 0 ? (uint32_t)(-qs) : 0u;
      const uint64_t endb = o1 - a[u];
      hi[u] = (j < total && im.w != 2) ? (endb < 16 ? (uint32_t)endb : 16u) : 0u;
      uint64_t ad[5];
      if (im.w <= 2) {
        const uint64_t sb = im.src + (uint64_t)qs;               // source byte under chunk byte 0
        const uint64_t d0 = sb & ~3ull, first = im.src & ~3ull, last = (im.src + tb - 1) & ~3ull;
#pragma unroll
        for (int i = 0; i < 5; i++) {
          const uint64_t d = d0 + 4 * (uint64_t)i;
          ad[i] = (int64_t)(d - first) < 0 ? first : d > last ? last : d;
        }
        r[u] = (uint32_t)(sb & 3);
        bsw[u] = 0;
      } else {
        const int64_t s0 = qs >= 0 ? qs >> 2 : -((-qs + 3) >> 2);  // floor(qs / 4)
        const int64_t nd = (int64_t)(tb >> 2);
        const uint64_t f = im.w == 8 ? 1u : 0u;
#pragma unroll
        for (int i = 0; i < 5; i++) {
          const int64_t si = s0 + i;
          const uint64_t c = si < 0 ? 0 : si >= nd ? (uint64_t)(nd - 1) : (uint64_t)si;
          ad[i] = im.src + 4 * (c ^ f);
        }
        r[u] = (uint32_t)(qs - 4 * s0);
        bsw[u] = 1;
      }
#pragma unroll
      for (int i = 0; i < 5; i++) x[u][i] = kx_ld<uint32_t>(ad[i]);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (lo[u] >= hi[u]) continue;
      uint32_t y[5];
#pragma unroll
      for (int i = 0; i < 5; i++) y[i] = bsw[u] ? __builtin_bswap32(x[u][i]) : x[u][i];
      uint32_t v[4];
#pragma unroll
      for (int i = 0; i < 4; i++) v[i] = __builtin_amdgcn_alignbyte(y[i + 1], y[i], r[u]);
      if (lo[u] == 0 && hi[u] == 16) {
        kx_st16(a[u], make_uint4(v[0], v[1], v[2], v[3]));
      } else {
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const uint32_t b0 = 4 * i;
          if (b0 >= lo[u] && b0 + 4 <= hi[u]) {
            kx_st<uint32_t>(a[u] + b0, v[i]);
          } else {
            for (uint32_t b = 0; b < 4; b++)
              if (b0 + b >= lo[u] && b0 + b < hi[u]) kx_st<uint8_t>(a[u] + b0 + b, (uint8_t)(v[i] >> (8 * b)));
          }
        }
      }
    }
  }
  for (uint32_t i = 0; i < nq; i++)
    if (q[i].w == 2) wave_copy(q[i], lane);
}

// queue a payload (false: the queue is full, the caller copies inline)
__device__ __forceinline__ bool defer(const PayQueue& pq, uint64_t dst, const void* src, uint32_t n, uint32_t w) {
  if (!pq.q) return false;
  const uint32_t slot = atomicAdd(pq.cnt, 1u);
  if (slot >= QCAP) return false;
  pq.q[slot] = PayItem{dst, (uint64_t)src, n, w};
  return true;
}

// FastWriteNocopy for one record into the sink
template <bool LS, class SK>
__device__ __forceinline__ void write_record(const KxProgram& P, const KxLaunchCols& C, uint64_t r, SK& s,
                                             const PayQueue& pq) {
  constexpr bool GL = std::is_same<SK, Sink>::value;   // payload queueing: the global (direct) path only
  uint64_t pres = C.presence ? kx_ld(C.presence + r) : 0;
  int inst = 0;
  int f = P.inst[0].enc_first;
  for (;;) {
    if (f < 0) {
      s.put(KX_T_STOP, 1);
      if (inst == 0) break;
      f = P.inst[inst].ret_pred;
      inst = P.inst[inst].parent;
      continue;
    }
    const KxpField F = P.f[f];
    if (F.req == KX_REQ_OPTIONAL && !((pres >> F.pbit) & 1)) { f = F.enc_next; continue; }
    // WriteFieldBegin: type, id (big-endian)
    uint32_t id = (uint16_t)F.id;
    s.put((uint32_t)F.ttype | ((id >> 8) << 8) | ((id & 0xff) << 16), 3);
    if (F.kind == KXP_K_FIXED) {
      uint64_t v = load_fixed(C.data[F.col], F.width, r);
      if (F.ttype == KX_T_BOOL) v = (v & 0xff) ? 1 : 0;
      put_be(s, v, F.width);
    } else if (F.kind == KXP_K_BYTES) {
      uint64_t o = off_at(C, F.col, r);
      uint32_t len = (uint32_t)var_len(C, F.col, r);
      put_be(s, len, 4);
      const uint8_t* src = (const uint8_t*)C.data[F.col] + o;
      if constexpr (GL) {
        if (len >= DEFER_MIN && pq.q) {
          const uint64_t at = s.pos();
          if (defer(pq, (uint64_t)s.base + at, src, len, 1)) {
            s.flush();
            s = Sink(s.base, at + len);
            f = F.enc_next;
            continue;
          }
        }
      }
      put_bytes(s, src, len);
    } else if (F.kind == KXP_K_LIST) {
      uint64_t o = off_at(C, F.col, r);
      uint32_t cnt = (uint32_t)var_len(C, F.col, r);
      s.put(F.elem, 1);
      put_be(s, cnt, 4);
      const void* src = C.data[F.col];
      if constexpr (GL) {
        if (cnt && pq.q && F.elem != KX_T_BOOL && F.width > 1) {
          const uint64_t at = s.pos();
          if (defer(pq, (uint64_t)s.base + at, (const uint8_t*)src + o * F.width, cnt, F.width)) {
            s.flush();
            s = Sink(s.base, at + (uint64_t)cnt * F.width);
            f = F.enc_next;
            continue;
          }
        }
      }
#if KX_ENC_LISTPF
      // blocks of 4 elements whose loads are all issued before the first is written (one memory round
      // trip per block instead of one per element, as put_bytes does for strings)
      for (uint32_t i0 = 0; i0 < cnt; i0 += 4) {
        uint64_t V[4];
#pragma unroll
        for (int u = 0; u < 4; u++) V[u] = i0 + u < cnt ? load_fixed(src, F.width, o + i0 + u) : 0;
#pragma unroll
        for (int u = 0; u < 4; u++) {
          if (i0 + u >= cnt) break;
          uint64_t v = V[u];
          if (F.elem == KX_T_BOOL) v = (v & 0xff) ? 1 : 0;
          put_be(s, v, F.width);
        }
      }
#else
      for (uint32_t i = 0; i < cnt; i++) {
        uint64_t v = load_fixed(src, F.width, o + i);
        if (F.elem == KX_T_BOOL) v = (v & 0xff) ? 1 : 0;
        put_be(s, v, F.width);
      }
#endif
    } else if (LS && F.kind == KXP_K_LSTRUCT) {
      // FieldFastWriteList of S (struct_tpl.go:1011-1036): S.FastWriteNocopy per element, every field of
      // S in IDL order (all fixed-length: the encoder reorder keeps it), then STOP
      const uint32_t cnt = (uint32_t)var_len(C, F.col, r);
      s.put(KX_T_STRUCT, 1);
      put_be(s, cnt, 4);
      for (uint32_t j = 0; j < cnt; j++) {
        for (int c = F.col; c < F.col + F.width; c++) {
          const KxpCol& K = P.col[c];
          const uint32_t sid = (uint16_t)P.sel_id[c];
          s.put((uint32_t)K.elem | ((sid >> 8) << 8) | ((sid & 0xff) << 16), 3);
          uint64_t v = load_fixed(C.data[c], K.width, off_at(C, c, r) + j);
          if (K.elem == KX_T_BOOL) v = (v & 0xff) ? 1 : 0;
          put_be(s, v, K.width);
        }
        s.put(KX_T_STOP, 1);
      }
    } else if (F.kind == KXP_K_LISTB || F.kind == KXP_K_MAP) {
      // FieldFastWriteList of strings / FieldFastWriteMap (struct_tpl.go:875-912, 1011-1036); a map
      // in column order (Go iterates its maps in random order)
      const bool map = F.kind == KXP_K_MAP;
      const uint64_t cnt = var_len(C, F.col, r);
      if (map) {
        s.put(F.elem & 15u, 1);
        s.put(F.elem >> 4, 1);
      } else {
        s.put(KX_T_STRING, 1);
      }
      put_be(s, cnt, 4);
      const int nside = map ? 2 : 1;
      uint64_t E[2] = {off_at(C, F.col, r), map ? off_at(C, F.col + 1, r) : 0};
      for (uint64_t j = 0; j < cnt; j++)
        for (int side = 0; side < nside; side++) {
          const int col = F.col + side;
          const KxpCol& K = P.col[col];
          if (K.kind == KXP_K_LISTB) {
            const uint64_t a = eoff_at(C, col, E[side] + j), len = eoff_at(C, col, E[side] + j + 1) - a;
            put_be(s, len, 4);
            put_bytes(s, (const uint8_t*)C.data[col] + a, (uint32_t)len);
          } else {
            uint64_t v = load_fixed(C.data[col], K.width, E[side] + j);
            if (K.elem == KX_T_BOOL) v = (v & 0xff) ? 1 : 0;
            put_be(s, v, K.width);
          }
        }
    } else {
      if ((pres >> F.pbit) & 1) { inst = F.child; f = P.inst[inst].enc_first; continue; }
      s.put(KX_T_STOP, 1);
    }
    f = F.enc_next;
  }
  s.flush();
}

// ---- Kitex-Protobuf records: `0x0A uvarint(len) body` per record (the Batch message's repeated
//      field 1), body = proto.Marshal of a flat proto3 message: fields in field-number order, zero
//      values of implicit-presence fields omitted, optional fields when set (protobuf.go:64-134) ----
__device__ __forceinline__ uint32_t uvarint_len(uint64_t v) {
  const int bits = v ? 64 - __clzll((long long)v) : 1;
  return (uint32_t)((bits + 6) / 7);
}

template <class SK>
__device__ __forceinline__ void put_uvarint(SK& s, uint64_t v) {
  while (v >= 0x80) {
    s.put((uint32_t)(v & 0x7f) | 0x80u, 1);
    v >>= 7;
  }
  s.put((uint32_t)v, 1);
}

// scalar as the proto wire value: int32/int16/int8 sign-extend to 64 bits, bool -> 0/1
__device__ __forceinline__ uint64_t pb_value(const KxpField& F, const KxLaunchCols& C, uint64_t r) {
  uint64_t v = load_fixed(C.data[F.col], F.width, r);
  if (F.pb_wt == 0) {
    if (F.width == 4) v = (uint64_t)(int64_t)(int32_t)(uint32_t)v;
    else if (F.width == 2) v = (uint64_t)(int64_t)(int16_t)(uint16_t)v;
    else if (F.width == 1) v = F.ttype == KX_T_BOOL ? ((v & 0xff) ? 1 : 0) : (uint64_t)(int64_t)(int8_t)(uint8_t)v;
  }
  return v;
}

__device__ __forceinline__ uint64_t pb_body_size(const KxProgram& P, const KxLaunchCols& C, uint64_t r) {
  const uint64_t pres = C.presence ? kx_ld(C.presence + r) : 0;
  uint64_t sz = 0;
  for (int f = P.pb_first; f >= 0; f = P.f[f].pb_next) {
    const KxpField F = P.f[f];
    const bool expl = F.req == KX_REQ_OPTIONAL;
    if (expl && !((pres >> F.pbit) & 1)) continue;
    const uint32_t tl = uvarint_len(((uint64_t)(uint16_t)F.id << 3) | F.pb_wt);
    if (F.pb_wt == 2) {
      const uint64_t n = var_len(C, F.col, r);
      if (n == 0 && !expl) continue;
      sz += tl + uvarint_len(n) + n;
    } else {
      const uint64_t v = pb_value(F, C, r);
      if (v == 0 && !expl) continue;
      sz += tl + (F.pb_wt == 0 ? uvarint_len(v) : 8u);
    }
  }
  return sz;
}

__device__ __forceinline__ uint64_t pb_record_size(const KxProgram& P, const KxLaunchCols& C, uint64_t r) {
  const uint64_t b = pb_body_size(P, C, r);
  return 1 + uvarint_len(b) + b;
}

template <class SK>
__device__ __forceinline__ void pb_write_record(const KxProgram& P, const KxLaunchCols& C, uint64_t r, SK& s) {
  s.put(0x0Au, 1);
  put_uvarint(s, pb_body_size(P, C, r));
  const uint64_t pres = C.presence ? kx_ld(C.presence + r) : 0;
  for (int f = P.pb_first; f >= 0; f = P.f[f].pb_next) {
    const KxpField F = P.f[f];
    const bool expl = F.req == KX_REQ_OPTIONAL;
    if (expl && !((pres >> F.pbit) & 1)) continue;
    const uint64_t tag = ((uint64_t)(uint16_t)F.id << 3) | F.pb_wt;
    if (F.pb_wt == 2) {
      const uint64_t n = var_len(C, F.col, r);
      if (n == 0 && !expl) continue;
      put_uvarint(s, tag);
      put_uvarint(s, n);
      put_bytes(s, (const uint8_t*)C.data[F.col] + off_at(C, F.col, r), (uint32_t)n);
    } else {
      const uint64_t v = pb_value(F, C, r);
      if (v == 0 && !expl) continue;
      put_uvarint(s, tag);
      if (F.pb_wt == 0) {
        put_uvarint(s, v);
      } else {  // fixed64, little-endian
        s.put((uint32_t)v, 4);
        s.put((uint32_t)(v >> 32), 4);
      }
    }
  }
  s.flush();
}

// BLength of a canonical record (every field present, structs non-nil): the plan's fixed bytes plus the
// payloads of its var steps
__device__ __forceinline__ uint64_t canon_size(const KxProgram& P, const KxLaunchCols& C, uint64_t r) {
  uint64_t sz = P.canon_fixed;
  for (uint32_t k = 0; k < P.nsteps; k++) {
    const KxpStep st = P.steps[k];
    if (st.kind == KXP_S_BYTES || st.kind == KXP_S_LIST)
      sz += var_len(C, st.col, r) * (st.kind == KXP_S_LIST ? st.width : 1u);
  }
  return sz;
}

__device__ __forceinline__ bool is_canon(const KxProgram& P, const KxLaunchCols& C, uint64_t r) {
  return !C.presence || (kx_ld(C.presence + r) & P.canon_pres) == P.canon_pres;
}

template <bool LS, bool CANON = false>
__device__ __forceinline__ uint64_t any_size(const EncParams& ep, const KxProgram& P, uint64_t r) {
  if (CANON && is_canon(P, ep.cols, r)) return canon_size(P, ep.cols, r);
  return ep.pb ? pb_record_size(P, ep.cols, r) : record_size<LS>(P, ep.cols, r);
}

template <bool LS, class SK>
__device__ __forceinline__ void any_write(const EncParams& ep, const KxProgram& P, uint64_t r, SK& s,
                                          const PayQueue& pq = PayQueue{nullptr, nullptr}) {
  if (ep.pb) pb_write_record(P, ep.cols, r, s);
  else write_record<LS>(P, ep.cols, r, s, pq);
}

// FastWriteNocopy of a record with the canonical plan (kx_program.h: encoder order, every field present,
// nil-free structs): a run of fixed-width fields loads all its values before the first is written (one
// memory round trip per run), strings and lists follow their headers. Same bytes as write_record.
template <class SK>
__device__ __forceinline__ void write_canon(const KxProgram& P, const KxLaunchCols& C, uint64_t r, SK& s) {
  const uint32_t ns = P.nsteps;
  for (uint32_t k = 0; k < ns;) {
    const KxpStep st = P.steps[k];
    if (st.kind == KXP_S_FIXED) {
      const uint32_t m = min(st.hdr >> 24, 8u);
      uint64_t v[8];
#pragma unroll
      for (uint32_t j = 0; j < 8; j++) {
        const KxpStep sj = P.steps[k + (j < m ? j : 0)];
        v[j] = j < m ? load_fixed(C.data[sj.col], sj.width, r) : 0;
      }
#pragma unroll
      for (uint32_t j = 0; j < 8; j++) {
        if (j >= m) break;
        const KxpStep sj = P.steps[k + j];
        s.put(sj.hdr & 0xffffffu, 3);
        uint64_t x = v[j];
        if ((sj.hdr & 0xffu) == KX_T_BOOL) x = (x & 0xff) ? 1 : 0;
        put_be(s, x, sj.width);
      }
      k += m;
      continue;
    }
    k++;
    if (st.kind == KXP_S_END) { s.put(KX_T_STOP, 1); continue; }
    s.put(st.hdr & 0xffffffu, 3);
    if (st.kind == KXP_S_STRUCT) continue;
    const uint64_t o = off_at(C, st.col, r);
    const uint32_t len = (uint32_t)(off_at(C, st.col, r + 1) - o);
    if (st.kind == KXP_S_BYTES) {
      put_be(s, len, 4);
      put_bytes(s, (const uint8_t*)C.data[st.col] + o, len);
      continue;
    }
    const KxpCol& K = P.col[st.col];   // KXP_S_LIST: list<scalar>
    s.put(K.elem, 1);
    put_be(s, len, 4);
    const void* src = C.data[st.col];
    for (uint32_t i0 = 0; i0 < len; i0 += KX_ENC_LISTB) {
      uint64_t V[KX_ENC_LISTB];
#pragma unroll
      for (int u = 0; u < KX_ENC_LISTB; u++) V[u] = i0 + u < len ? load_fixed(src, K.width, o + i0 + u) : 0;
#pragma unroll
      for (int u = 0; u < KX_ENC_LISTB; u++) {
        if (i0 + u >= len) break;
        uint64_t x = V[u];
        if (K.elem == KX_T_BOOL) x = (x & 0xff) ? 1 : 0;
        put_be(s, x, K.width);
      }
    }
  }
  s.flush();
}

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

__device__ uint64_t block_excl_scan(uint64_t v, uint64_t* tot, uint64_t* scratch) {
  int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t inc = wave_incl_scan(v, lane);
  __syncthreads();
  if (lane == 63) scratch[wv] = inc;
  __syncthreads();
  uint64_t base = 0, t = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); i++) {
    uint64_t s = scratch[i];
    if (i < wv) base += s;
    t += s;
  }
  *tot = t;
  return base + inc - v;
}

template <bool LS, bool CANON>
__global__ void __launch_bounds__(NT) size_kernel(EncParams ep) {
  __shared__ uint64_t scratch[NT / 64];
  __shared__ uint32_t progw[sizeof(KxProgram) / 4];
  for (int i = threadIdx.x; i < (int)(sizeof(KxProgram) / 4); i += NT) progw[i] = ((const uint32_t*)ep.prog)[i];
  __syncthreads();
  const KxProgram& P = *reinterpret_cast<const KxProgram*>(progw);
  uint64_t b = blockIdx.x;
  uint64_t acc = 0;
  for (int k = 0; k < RB / NT; k++) {
    uint64_t r = b * RB + k * NT + threadIdx.x;
    uint64_t sz = 0;
    if (r < ep.n) {
      sz = any_size<LS, CANON>(ep, P, r);
      if (ep.sizes_out) ep.sizes_out[r] = sz;
    }
    acc += sz;
  }
  uint64_t tot;
  block_excl_scan(acc, &tot, scratch);
  if (threadIdx.x == 0 && ep.block_tot) ep.block_tot[b] = tot;
}

__global__ void __launch_bounds__(1024) scan_kernel(EncParams ep) {
  __shared__ uint64_t scratch[16];
  uint64_t nb = ep.nblocks;
  uint64_t per = (nb + 1023) / 1024;
  uint64_t lo = threadIdx.x * per, hi = kmin64(lo + per, nb);
  uint64_t s = 0;
  for (uint64_t i = lo; i < hi; i++) s += ep.block_tot[i];
  uint64_t tot;
  const uint64_t b0 = ep.out_base ? *ep.out_base : 0;
  uint64_t run = b0 + block_excl_scan(s, &tot, scratch);
  for (uint64_t i = lo; i < hi; i++) {
    uint64_t v = ep.block_tot[i];
    ep.block_tot[i] = run;
    run += v;
  }
  if (threadIdx.x == 0) {
    kx_status* st = ep.status;
    st->n_records = ep.n;
    st->consumed = b0 + tot;
    st->code = b0 + tot > ep.out_cap ? KX_ERR_SIZE_LIMIT : 0;
    if (ep.offsets_out && b0 + tot <= ep.out_cap) ep.offsets_out[ep.n] = b0 + tot;
  }
}

#ifndef KX_ENC_LB
#define KX_ENC_LB 1
#endif
// CANON: the schema has a canonical plan (flat Thrift, no optional field): records whose structs are all
// present are written by write_canon into the LDS image (its own instantiation)
template <bool LS, bool CANON>
__global__ void __launch_bounds__(WT, KX_ENC_LB) write_kernel(EncParams ep) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  uint8_t* img = (uint8_t*)smem_raw;                        // OUTB + 32
  uint32_t* progw = (uint32_t*)(smem_raw + OUTB + 32);
  uint64_t* scratch = (uint64_t*)(smem_raw + OUTB + 32 + sizeof(KxProgram));
  __shared__ uint64_t s_take, s_round_bytes;
  __shared__ uint32_t qcnt[WT / 64];
  // the direct path's payload queues live in the (then unused) LDS image
  PayItem* qbase = (PayItem*)smem_raw;
  static_assert((WT / 64) * (QCAP * sizeof(PayItem) + (QCAP + 1) * 8) <= OUTB, "payload queues fit the image");
  if (ep.status->code != 0) return;                         // size limit: write nothing
  for (int i = threadIdx.x; i < (int)(sizeof(KxProgram) / 4); i += WT) progw[i] = ((const uint32_t*)ep.prog)[i];
  __syncthreads();
  const KxProgram& P = *reinterpret_cast<const KxProgram*>(progw);
  const uint64_t b = blockIdx.x;
  uint64_t r = b * RB;
  const uint64_t rend = kmin64(r + RB, ep.n);
  uint64_t gpos = ep.block_tot[b];
  while (r < rend) {
    uint64_t my = r + threadIdx.x;
    uint64_t sz = my < rend ? any_size<LS, CANON>(ep, P, my) : 0;
    uint64_t tot;
    uint64_t pre = block_excl_scan(sz, &tot, scratch);
    const uint32_t skew = (uint32_t)(((uint64_t)ep.out + gpos) & 15);
    // records that fit entirely into this round's image (at least one)
    bool fits = my < rend && skew + pre + sz <= OUTB;
    if (threadIdx.x == 0) { s_take = 0; s_round_bytes = 0; }
    __syncthreads();
    if (fits) {
      atomicMax((unsigned long long*)&s_take, (unsigned long long)(threadIdx.x + 1));
      atomicMax((unsigned long long*)&s_round_bytes, (unsigned long long)(pre + sz));
    }
    __syncthreads();
    uint64_t take = s_take;
    const uint64_t cnt = kmin64((uint64_t)WT, rend - r);
    if (take < (cnt >> KX_ENC_MINTAKE) || take == 0 || ep.direct) {
      // large records (fewer than half of the round fit the image, or one larger than the whole image):
      // every lane writes its record straight to HBM, leaving list elements and long strings to its wave
      // (wave_copy: coalesced loads, 256 contiguous bytes per store instruction)
      const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
      if (lane == 0) qcnt[wv] = 0;
      __builtin_amdgcn_wave_barrier();
      const PayQueue pq{qbase + wv * QCAP, &qcnt[wv]};
      if (my < rend) {
        Sink s((GB*)ep.out, gpos + pre);
        any_write<LS>(ep, P, my, s, ep.pb ? PayQueue{nullptr, nullptr} : pq);
        if (ep.offsets_out) ep.offsets_out[my] = gpos + pre;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      const uint32_t nq = min(qcnt[wv], (uint32_t)QCAP);
      uint64_t* pre = (uint64_t*)(smem_raw + (WT / 64) * QCAP * sizeof(PayItem)) + wv * (QCAP + 1);
      if (ep.wcu == 0) {}  // diagnostics only (output incomplete): no payload copy
      else if (ep.wcu == 16) wave_copy_queue16<KX_ENC_WCU16>(qbase + wv * QCAP, nq, lane, pre);
      else if (ep.wcu >= 4) wave_copy_queue<KX_ENC_WCU>(qbase + wv * QCAP, nq, lane, pre);
      else for (uint32_t i = 0; i < nq; i++) wave_copy(qbase[wv * QCAP + i], lane);
      __syncthreads();
      gpos += tot;
      r += cnt;
      continue;
    }
    if (threadIdx.x < take) {
      LSink s((LDSB*)img, skew + pre);
      if (CANON && is_canon(P, ep.cols, my))
        write_canon(P, ep.cols, my, s);
      else
        any_write<LS>(ep, P, my, s);
      if (ep.offsets_out) ep.offsets_out[my] = gpos + pre;
    }
    __syncthreads();
    // stream the image [skew, skew + bytes) to out[gpos ...): the image is congruent mod 16
    const uint64_t bytes = s_round_bytes;
    const uint64_t gstart = (uint64_t)ep.out + gpos;
    const uint64_t a0 = gstart & ~15ull;                     // image byte 0 <-> a0
    const uint64_t gend = gstart + bytes;
    const uint64_t nch = (gend - a0 + 15) >> 4;
    for (uint64_t c = threadIdx.x; c < nch; c += WT) {
      uint64_t ca = a0 + c * 16;
      if (ca >= gstart && ca + 16 <= gend) {
        kx_st16(ca, *(const uint4*)(img + c * 16));
      } else {
        for (int k = 0; k < 16; k++) {
          uint64_t x = ca + k;
          if (x >= gstart && x < gend) kx_st<uint8_t>(x, img[c * 16 + k]);
        }
      }
    }
    __syncthreads();
    gpos += bytes;
    r += take;
  }
}

}  // namespace

size_t kx_encode_ws_bytes(uint64_t n) { return ((n + RB - 1) / RB) * 8 + 256; }

int kx_launch_encode(const KxProgram* dprog, const KxProgram& hprog, const KxLaunchCols& cols, uint64_t n,
                     uint8_t* out, uint64_t out_cap, uint64_t* sizes_out, uint64_t* offsets_out,
                     kx_status* status, void* ws, size_t ws_size, hipStream_t stream, bool sizes_only,
                     bool pb, const uint64_t* out_base) {
  (void)hprog;
  EncParams ep{};
  ep.pb = pb;
  ep.out_base = out_base;
  ep.prog = dprog; ep.cols = cols; ep.n = n; ep.out = out; ep.out_cap = out_cap;
  ep.sizes_out = sizes_out; ep.offsets_out = offsets_out; ep.status = status;
  ep.nblocks = (n + RB - 1) / RB;
  ep.direct = kx_knob(KXK_ENC_DIRECT);
  ep.wcu = kx_knob(KXK_ENC_WCU);
  if (ws_size < kx_encode_ws_bytes(n)) return KX_ERR_INVALID_ARG;
  ep.block_tot = (uint64_t*)ws;
  if (status) KX_HIP_CHECK(hipMemsetAsync(status, 0, sizeof(kx_status), stream));
  bool ls = false;
  for (uint32_t f = 0; f < hprog.nfields; f++) ls |= hprog.f[f].kind == KXP_K_LSTRUCT;
  // KX_ENC_CANON=0: the generic sizes and writer for every record (A/B)
  const bool canon = kx_knob(KXK_ENC_CANON) && !pb && !ls && hprog.nsteps > 0;
  if (ls) hipLaunchKernelGGL((size_kernel<true, false>), dim3((unsigned)ep.nblocks), dim3(NT), 0, stream, ep);
  else if (canon) hipLaunchKernelGGL((size_kernel<false, true>), dim3((unsigned)ep.nblocks), dim3(NT), 0, stream, ep);
  else hipLaunchKernelGGL((size_kernel<false, false>), dim3((unsigned)ep.nblocks), dim3(NT), 0, stream, ep);
  KX_HIP_CHECK(hipGetLastError());
  if (sizes_only) return KX_OK;
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, stream, ep);
  KX_HIP_CHECK(hipGetLastError());
  size_t shmem = OUTB + 32 + sizeof(KxProgram) + 8 * (WT / 64);
  if (ls) hipLaunchKernelGGL((write_kernel<true, false>), dim3((unsigned)ep.nblocks), dim3(WT), shmem, stream, ep);
  else if (canon) hipLaunchKernelGGL((write_kernel<false, true>), dim3((unsigned)ep.nblocks), dim3(WT), shmem, stream, ep);
  else hipLaunchKernelGGL((write_kernel<false, false>), dim3((unsigned)ep.nblocks), dim3(WT), shmem, stream, ep);
  KX_HIP_CHECK(hipGetLastError());
  return KX_OK;
}
