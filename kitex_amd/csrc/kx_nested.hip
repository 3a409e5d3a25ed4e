// kx_nested.hip — nested schemas on the device: the record walker of kx_nested.h, lane = record.
//
// Decode (records' extents from the caller's offsets / ends, or from the skip pass for concatenated
// records, pkg/remote/codec/thrift/codec_apache.go:166-172):
//   1. measure: each lane walks its record counting cursor advances (kx_nested.h, W = false) and writes
//      them per cursor (u32, cursor-major: lanes store adjacent words) with its record's code;
//   2. block sums per (1024-record block, cursor), then one workgroup per cursor scans the block sums
//      into block bases and the cursor's total; a one-thread check compares the totals with the
//      columns' capacities (SIZE_LIMIT: nothing is written);
//   3. write: each lane reads its record's cursor bases (block base + the in-block prefix the block-sum
//      pass left in place of the counts) and re-walks the record writing values, offsets and presence;
//   4. finalize: the last entry of every offsets array, the call status.
// Encode: size pass (lane = record, BLength) -> block scan -> write pass (FastWriteNocopy at the
// record's offset); struct_tpl.go:225-391.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "kx_internal.h"
#include "kx_nested.h"

namespace {

constexpr int NT = 256;       // threads per workgroup
constexpr int RB = 1024;      // records per block
constexpr int SNAP = KXN_MAX_SNAP;  // snapshot slots per lane (kx_schema_create refuses schemas needing more)
constexpr int CUR = KXN_MAX_CUR;    // cursors per lane

struct NParams {
  const KxnProgram* P;
  const KxnCols* C;
  const uint8_t* in;
  uint64_t in_len;
  const uint64_t* offsets;    // known offsets (n + 1), or the skip pass's starts (concat)
  const uint64_t* ends;       // explicit ends (optional)
  uint64_t n;
  bool concat;
  const kx_status* skip_st;   // concat: the skip pass's status (records delimited)
  const uint64_t* bstart;     // concat, Kitex-PB: the Batch frames' body extents (the frame pass)
  const uint64_t* bend;
  uint32_t* counts;           // [ncur][n]
  uint64_t* bsum;             // [ncur][nblk]
  uint64_t* totals;           // [ncur]
  uint8_t* rcode;             // [n] record codes of the measure pass
  unsigned long long* errkey; // (record << 8) | code, min
  uint32_t* flag;             // size limit: write nothing
  uint8_t* record_status;     // caller's (optional)
  kx_status* status;
  uint64_t nblk;
  uint32_t ncur;
  bool sizes_only;            // kx_thrift_decode_sizes: no column is written
  const uint64_t* cur_base;   // (optional) every cursor starts here: a record-range chunk of a larger batch
                              // continues the previous chunk's arenas (kx_host_* pipelines)
  uint64_t* totals_out;       // (optional) the absolute cursor totals at the end of the call
};

// record r's extent; false when the record is not decoded at all (concat: past the failing one)
__device__ __forceinline__ int extent(const NParams& p, uint64_t r, uint64_t* a, uint64_t* b) {
  if (p.concat) {
    const uint64_t ok = p.skip_st->code ? p.skip_st->n_records : p.n;
    if (r > ok || (r == ok && !p.skip_st->code)) return -1;
    if (p.bstart) {   // Kitex-PB: the body of frame r; a frame that could not be delimited reads as empty
      *a = r < ok ? p.bstart[r] : 0;
      *b = r < ok ? p.bend[r] : 0;
      return 0;
    }
    *a = p.offsets[r];
    *b = r < ok ? p.offsets[r + 1] : p.in_len;   // the failing record: FastRead finds its error
    return 0;
  }
  *a = p.offsets[r];
  *b = p.ends ? p.ends[r] : p.offsets[r + 1];
  return (*a > *b || *b > p.in_len) ? KX_ERR_INVALID_ARG : 0;
}

// rcode[r]: the record's code, | RC_CAREFUL when it repeats a field (its walks need snapshots, and the write
// walk clipping at its extents); RC_NONE: not decoded (concatenated, past the failing record)
constexpr uint8_t RC_CAREFUL = 0x40, RC_NONE = 0xff;

// The cursors of a workgroup's lanes in LDS, cursor k of lane t at [k * NTD + t] (a wave's accesses to one
// cursor are 64 adjacent dwords): u32 values relative to a per-cursor base the workgroup shares (0 in the
// measure pass; the 1024-record block's base in the write pass, whose in-block prefixes are u32 already,
// bsum_kernel). In scratch, with 1 M lanes' walks in flight, every cursor access missed the caches: the
// measure and write passes fetched 11 and 18 GB per call for 0.76 GB of input (round 5 PMC).
#define KXN_LDS __attribute__((address_space(3)))
constexpr int NTD = 512;   // threads per workgroup of the walker's passes
struct KxnCurL {
  KXN_LDS uint32_t* p;             // this lane's cursor 0
  const KXN_LDS uint64_t* base;    // per cursor
  __device__ uint64_t operator[](int k) const { return base[k] + p[k * NTD]; }
  __device__ void set(int k, uint64_t v) const { p[k * NTD] = (uint32_t)(v - base[k]); }
  __device__ void add(int k, uint64_t d) const { p[k * NTD] += (uint32_t)d; }
  __device__ uint64_t post_inc(int k) const {
    const uint32_t x = p[k * NTD];
    p[k * NTD] = x + 1;
    return base[k] + x;
  }
};

// the walk of record [a, b) (a per-lane LDS window over the record's bytes, refilled 32 bytes at a time,
// measured slower: 7.8 / 21.0 ms for the measure / write passes against 7.2 / 15.6 ms).
// snap == nullptr: the fast walk (KXN_REPEAT at a repeated field). PB: the program is Kitex-Protobuf's (every
// walker kernel is built once per wire format, so that neither walker's registers bound the other's occupancy)
template <bool W, bool PB, class CU>
__device__ __forceinline__ int walk(const NParams& p, const KxnProgram& P, const KxnCols& C, uint64_t a, uint64_t b,
                                   uint64_t r, CU cur, uint64_t* snap, uint64_t* lim) {
  uint64_t used = 0;
  if constexpr (PB) return kxn_pb_read_record<W>(P, C, p.in + a, b - a, r, cur, snap, &used, lim);
  else return kxn_read_record<W>(P, C, p.in + a, b - a, r, cur, snap, &used, lim);
}

template <bool PB, class CU>
__device__ __forceinline__ void measure_record(const NParams& p, const KxnProgram& P, uint64_t r, CU cur,
                                               uint64_t* snap) {
  for (uint32_t k = 0; k < p.ncur; k++) cur.set(k, 0);
  uint64_t a = 0, b = 0;
  int rc = extent(p, r, &a, &b);
  if (rc < 0) {
    rc = 0;  // not decoded: empty
    p.rcode[r] = RC_NONE;
  } else {
    // (a per-lane 16-byte read-ahead block in registers measured slower: 55.7 vs 41.7 ms for 1 M Nesting
    // records, divergent refills and 164 VGPRs in the write pass)
    uint8_t careful = 0;
    if (!rc) {
      rc = walk<false, PB>(p, P, *p.C, a, b, r, cur, nullptr, nullptr);   // no snapshot stores: the common record
      if (rc == KXN_REPEAT) {                                   // a repeated field: again, with snapshots
        for (uint32_t k = 0; k < p.ncur; k++) cur.set(k, 0);
        rc = walk<false, PB>(p, P, *p.C, a, b, r, cur, snap, nullptr);
        careful = RC_CAREFUL;
      }
    }
    if (!rc && p.concat && r < p.n && p.skip_st->code && r == p.skip_st->n_records) rc = p.skip_st->code;
    p.rcode[r] = (uint8_t)rc | careful;
    if (rc) atomicMin(p.errkey, (unsigned long long)((r << 8) | (uint64_t)(rc & 0xff)));
  }
  for (uint32_t k = 0; k < p.ncur; k++) p.counts[(uint64_t)k * p.n + r] = rc ? 0u : (uint32_t)cur[k];
}

// cursors and snapshots in per-lane private (scratch) arrays (an LDS-resident variant, one wave per
// workgroup, measured slower on the MI355X: 62.8 vs 43.7 ms for 1 M Nesting records)
// The program in LDS: the walk's table reads (nodes, fields, structs, roots, entries, defaults: a dozen
// dependent reads per field) at LDS latency instead of through the vector L1 / L2. One copy per 512-thread
// workgroup (31 KB).
__device__ __forceinline__ const KxnProgram& lds_program(const KxnProgram* g, KxnProgram* s) {
  static_assert(sizeof(KxnProgram) % 4 == 0, "dword copy");
  const uint32_t* src = (const uint32_t*)g;
  uint32_t* dst = (uint32_t*)s;
  for (uint32_t i = threadIdx.x; i < sizeof(KxnProgram) / 4; i += blockDim.x) dst[i] = src[i];
  __syncthreads();
  return *s;
}
// the call's column table in LDS too (4 KB), for the passes that store: every store's column pointer, width
// and offset size is then an LDS read instead of a dependent global load (publish with lds_program's barrier)
__device__ __forceinline__ void lds_cols(const KxnCols* g, KxnCols* s) {
  static_assert(sizeof(KxnCols) % 4 == 0, "dword copy");
  const uint32_t* src = (const uint32_t*)g;
  uint32_t* dst = (uint32_t*)s;
  for (uint32_t i = threadIdx.x; i < sizeof(KxnCols) / 4; i += blockDim.x) dst[i] = src[i];
}

// LC: the cursors in LDS (dynamic shared memory: ncur bases, then ncur x NTD u32), else in scratch
template <bool LC, bool PB>
__global__ void __launch_bounds__(NTD) measure_kernel(NParams p) {
  __shared__ KxnProgram sP;
  extern __shared__ uint64_t dyn[];
  if (LC)
    for (uint32_t k = threadIdx.x; k < p.ncur; k += NTD) dyn[k] = 0;
  const KxnProgram& P = lds_program(p.P, &sP);   // (its barrier also publishes the bases)
  const uint64_t r = (uint64_t)blockIdx.x * NTD + threadIdx.x;
  if (r >= p.n) return;
  uint64_t snap[SNAP];
  if constexpr (LC) {
    measure_record<PB>(p, P, r, KxnCurL{(KXN_LDS uint32_t*)(dyn + p.ncur) + threadIdx.x, (const KXN_LDS uint64_t*)dyn},
                   snap);
  } else {
    uint64_t cur[CUR];
    measure_record<PB>(p, P, r, KxnCurP{cur}, snap);
  }
}


__device__ __forceinline__ uint64_t wave_incl(uint64_t v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

// exclusive scan over the workgroup (NT threads); *tot = the sum
__device__ uint64_t wg_excl(uint64_t v, uint64_t* tot, uint64_t* sh) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t inc = wave_incl(v, lane);
  __syncthreads();
  if (lane == 63) sh[wv] = inc;
  __syncthreads();
  uint64_t base = 0, t = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); i++) {
    const uint64_t s = sh[i];
    if (i < wv) base += s;
    t += s;
  }
  *tot = t;
  return base + inc - v;
}

// grid (nblk, ncur): block sums, and each count replaced by its exclusive prefix inside the block (u32:
// a block's units of one cursor stay below 2^32, kx_launch_nested_decode), so that the write pass reads
// every record's cursor bases instead of scanning for them. Thread t owns RB / NT consecutive records.
constexpr int RPT = RB / NT;
__global__ void __launch_bounds__(NT) bsum_kernel(NParams p) {
  __shared__ uint64_t sh[NT / 64];
  const uint64_t b = blockIdx.x, k = blockIdx.y;
  const uint64_t r0 = b * RB + (uint64_t)threadIdx.x * RPT;
  uint32_t* c = p.counts + k * p.n;
  uint32_t x[RPT];
  uint64_t acc = 0;
#pragma unroll
  for (int j = 0; j < RPT; j++) {
    x[j] = r0 + j < p.n ? c[r0 + j] : 0u;
    acc += x[j];
  }
  uint64_t tot;
  uint64_t pre = wg_excl(acc, &tot, sh);
  if (!p.sizes_only) {
#pragma unroll
    for (int j = 0; j < RPT; j++) {
      if (r0 + j < p.n) c[r0 + j] = (uint32_t)pre;
      pre += x[j];
    }
  }
  if (threadIdx.x == 0) p.bsum[k * p.nblk + b] = tot;
}

// one workgroup per cursor: block sums -> block bases, the cursor's total
__global__ void __launch_bounds__(1024) bscan_kernel(NParams p) {
  __shared__ uint64_t sh[16];
  const uint64_t k = blockIdx.x, nb = p.nblk;
  uint64_t* s = p.bsum + k * nb;
  const uint64_t per = (nb + 1023) / 1024;
  const uint64_t lo = threadIdx.x * per, hi = kmin64(lo + per, nb);
  uint64_t acc = 0;
  bool big = false;   // a block holding 2^32 units of one cursor: its u32 in-block prefixes would wrap
  for (uint64_t i = lo; i < hi; i++) {
    acc += s[i];
    big |= s[i] >> 32 != 0;
  }
  if (big) atomicOr(p.flag, 1u);   // SIZE_LIMIT: nothing is written
  uint64_t tot;
  const uint64_t base = p.cur_base ? p.cur_base[k] : 0;
  uint64_t run = base + wg_excl(acc, &tot, sh);
  for (uint64_t i = lo; i < hi; i++) {
    const uint64_t v = s[i];
    s[i] = run;
    run += v;
  }
  if (threadIdx.x == 0) p.totals[k] = base + tot;
}

// the parent domain size of column c's offsets array k
__device__ __forceinline__ uint64_t parent_size(const NParams& p, const KxnCol& K, int k) {
  return k == 0 ? p.n : p.totals[K.acur[k - 1]];
}

// capacities vs totals (one thread); status of a sizes-only call
__global__ void check_kernel(NParams p) {
  if (threadIdx.x != 0) return;
  const KxnProgram& P = *p.P;
  bool over = false;
  for (uint32_t c = 0; c < P.ncols; c++) {
    const KxnCol& K = P.col[c];
    if (K.dcur >= 0 && p.totals[K.dcur] > p.C->cap[c][0]) over = true;
    for (int k = 1; k < K.narr; k++)
      if (parent_size(p, K, k) > p.C->cap[c][1 + k]) over = true;
  }
  if (over) *p.flag = 1u;
}

// record r (of block b), lane = record; cur holds the record's cursor bases: the block base + the in-block
// prefix (bsum_kernel)
template <bool PB, class CU>
__device__ __forceinline__ void write_record(const NParams& p, const KxnProgram& P, const KxnCols& C, uint64_t b,
                                             uint64_t r, CU cur, uint64_t* lim, uint64_t* snap) {
  const uint8_t raw = p.rcode[r];
  const uint8_t rc = raw == RC_NONE ? RC_NONE : (uint8_t)(raw & ~RC_CAREFUL);
  uint64_t a = 0, e = 0;
  if (rc == 0 && extent(p, r, &a, &e) == 0) {
    if (raw & RC_CAREFUL) {
      // a record that repeats a field: its extents end at the next record's prefix, or at the next block's
      // base, and every write is clipped to them (what a replaced occurrence wrote past them is the next
      // record's)
      const uint64_t rb1 = kmin64((b + 1) * RB, p.n);   // the block's end
      for (uint32_t k = 0; k < p.ncur; k++) {
        const uint64_t base = p.bsum[(uint64_t)k * p.nblk + b];
        lim[k] = r + 1 < rb1 ? base + p.counts[(uint64_t)k * p.n + r + 1]
                             : (b + 1 < p.nblk ? p.bsum[(uint64_t)k * p.nblk + b + 1] : p.totals[k]);
      }
      (void)walk<true, PB>(p, P, C, a, e, r, cur, snap, lim);
    } else {   // the fast walk writes only inside the record's extents
      (void)walk<true, PB>(p, P, C, a, e, r, cur, nullptr, nullptr);
    }
  } else {
    kxn_failed_record(P, C, r, cur);
  }
  if (p.record_status && !p.concat) p.record_status[r] = rc == RC_NONE ? 0 : rc;
}

// one record per thread: workgroup w holds records [w·NTD, (w + 1)·NTD) of block w / (RB / NTD) (a workgroup
// per block looping over its quarters left 4 waves per SIMD: DESIGN §3.10)
// CL: the walker's part of the column table (KXN_COLS_HEAD bytes) in LDS after the cursors, when two workgroups
// per CU still fit (the whole 4 KB table measured slower, 10.3 vs 9.0 ms for 1 M Nesting records: one
// workgroup per CU)
template <bool LC, bool PB, bool CL>
__global__ void __launch_bounds__(NTD) write_kernel(NParams p) {
  if (*p.flag) return;
  __shared__ KxnProgram sP;
  extern __shared__ uint64_t dyn[];
  const uint64_t b = blockIdx.x / (RB / NTD);
  if (LC)   // the block's base per cursor, shared by the workgroup's lanes
    for (uint32_t k = threadIdx.x; k < p.ncur; k += NTD) dyn[k] = p.bsum[(uint64_t)k * p.nblk + b];
  KxnCols* sc = (KxnCols*)(dyn + (size_t)p.ncur * (1 + NTD / 2));
  if (CL) {   // (published by lds_program's barrier)
    static_assert(KXN_COLS_HEAD % 4 == 0, "dword copy");
    for (uint32_t i = threadIdx.x; i < KXN_COLS_HEAD / 4; i += NTD) ((uint32_t*)sc)[i] = ((const uint32_t*)p.C)[i];
  }
  const KxnProgram& P = lds_program(p.P, &sP);
  const KxnCols& C = CL ? *sc : *p.C;
  const uint64_t r = (uint64_t)blockIdx.x * NTD + threadIdx.x;
  if (r >= p.n) return;
  uint64_t lim[CUR], snap[SNAP];
  if constexpr (LC) {
    KXN_LDS uint32_t* c = (KXN_LDS uint32_t*)(dyn + p.ncur) + threadIdx.x;
    for (uint32_t k = 0; k < p.ncur; k++) c[k * NTD] = p.counts[(uint64_t)k * p.n + r];   // in-block prefixes
    write_record<PB>(p, P, C, b, r, KxnCurL{c, (const KXN_LDS uint64_t*)dyn}, lim, snap);
  } else {
    uint64_t cur[CUR];
    for (uint32_t k = 0; k < p.ncur; k++) cur[k] = p.bsum[(uint64_t)k * p.nblk + b] + p.counts[(uint64_t)k * p.n + r];
    write_record<PB>(p, P, C, b, r, KxnCurP{cur}, lim, snap);
  }
}


__global__ void finalize_kernel(NParams p) {
  const KxnProgram& P = *p.P;
  if (*p.flag && !p.sizes_only) {
    if (threadIdx.x == 0) {
      p.status->code = KX_ERR_SIZE_LIMIT;
      p.status->n_records = 0;
      for (int v = 0; v < 16; v++) p.status->var_total[v] = v < (int)p.ncur ? p.totals[v] : 0;
      if (p.totals_out)   // the required sizes: a later chunk based on them fails too
        for (uint32_t v = 0; v < p.ncur; v++) p.totals_out[v] = p.totals[v];
      *p.errkey = ~0ull;
    }
    return;
  }
  for (uint32_t c = threadIdx.x; c < P.ncols && !p.sizes_only; c += blockDim.x) {
    const KxnCol& K = P.col[c];
    for (int k = 0; k < K.narr; k++) kxn_put_arr(*p.C, (int)c, k, parent_size(p, K, k), p.totals[K.acur[k]]);
  }
  if (threadIdx.x != 0) return;
  kx_status* st = p.status;
  const unsigned long long key = *p.errkey;
  st->n_records = p.n;
  st->consumed = p.concat ? p.offsets[p.n] : (p.n ? (p.ends ? p.ends[p.n - 1] : p.offsets[p.n]) : 0);
  if (key != ~0ull) {
    const uint64_t r = key >> 8;
    st->code = (int32_t)(key & 0xff);
    st->record = r;
    st->offset = p.offsets[r];
    if (p.concat) {
      st->n_records = r;
      st->consumed = p.offsets[r];
    }
  }
  for (int v = 0; v < 16; v++) st->var_total[v] = v < (int)p.ncur ? p.totals[v] : 0;
  if (p.totals_out)
    for (uint32_t v = 0; v < p.ncur; v++) p.totals_out[v] = p.totals[v];
  *p.errkey = ~0ull;
}

// ---- encode ----
struct EParams {
  const KxnProgram* P;
  const KxnCols* C;
  uint64_t n;
  uint8_t* out;
  uint64_t out_cap;
  uint64_t* sizes;       // [n] (caller's or workspace)
  uint64_t* bsum;        // [nblk]
  uint64_t* offsets_out; // optional
  kx_status* status;
  uint64_t nblk;
  const uint64_t* out_base;  // (optional, device) the records start here: a chunk continues the previous
                             // chunk's output (kx_host_encode_batch pipeline, its status->consumed)
};

// encode blocks: ERB = NT records, one per thread (a workgroup per 1024 records looping over its quarters
// left 4 waves per SIMD)
constexpr int ERB = NT;
template <bool PB>
__global__ void __launch_bounds__(NT) esize_kernel(EParams p) {
  __shared__ uint64_t sh[NT / 64];
  __shared__ KxnProgram sP;
  __shared__ KxnCols sC;
  lds_cols(p.C, &sC);
  const KxnProgram& P = lds_program(p.P, &sP);   // the walk's table reads at LDS latency (as decode)
  const KxnCols& C = sC;
  const uint64_t r = (uint64_t)blockIdx.x * ERB + threadIdx.x;
  uint64_t sz = 0;
  if (r < p.n) {   // Kitex-PB: the record's Batch frame (0x0A, uvarint body length, body)
    if constexpr (PB) sz = kxn_pb_frame_size(P, C, r);
    else sz = kxn_write_record<false>(P, C, r, nullptr, 0);
    p.sizes[r] = sz;
  }
  uint64_t tot;
  (void)wg_excl(sz, &tot, sh);
  if (threadIdx.x == 0 && p.bsum) p.bsum[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(1024) escan_kernel(EParams p) {
  __shared__ uint64_t sh[16];
  const uint64_t nb = p.nblk;
  const uint64_t per = (nb + 1023) / 1024;
  const uint64_t lo = threadIdx.x * per, hi = kmin64(lo + per, nb);
  uint64_t acc = 0;
  for (uint64_t i = lo; i < hi; i++) acc += p.bsum[i];
  uint64_t tot;
  const uint64_t base = p.out_base ? *p.out_base : 0;
  uint64_t run = base + wg_excl(acc, &tot, sh);
  for (uint64_t i = lo; i < hi; i++) {
    const uint64_t v = p.bsum[i];
    p.bsum[i] = run;
    run += v;
  }
  if (threadIdx.x == 0) {
    kx_status* st = p.status;
    const uint64_t end = base + tot;
    st->n_records = p.n;
    st->consumed = end;
    st->code = end > p.out_cap ? KX_ERR_SIZE_LIMIT : 0;
    if (p.offsets_out && end <= p.out_cap) p.offsets_out[p.n] = end;
  }
}

template <bool PB>
__global__ void __launch_bounds__(NT) ewrite_kernel(EParams p) {
  __shared__ uint64_t sh[NT / 64];
  __shared__ KxnProgram sP;
  if (p.status->code != 0) return;
  __shared__ KxnCols sC;
  lds_cols(p.C, &sC);
  const KxnProgram& P = lds_program(p.P, &sP);
  const KxnCols& C = sC;
  const uint64_t r = (uint64_t)blockIdx.x * ERB + threadIdx.x;
  const uint64_t sz = r < p.n ? p.sizes[r] : 0;
  uint64_t tot;
  const uint64_t at = p.bsum[blockIdx.x] + wg_excl(sz, &tot, sh);
  if (r < p.n) {
    if constexpr (PB) kxn_pb_write_frame(P, C, r, p.out, at, sz);
    else (void)kxn_write_record<true>(P, C, r, p.out, at);
    if (p.offsets_out) p.offsets_out[r] = at;
  }
}

}  // namespace

// workspace: [0] errkey u64, [8] flag u32, [64] rcode[n], counts [ncur][n] u32, bsum [ncur][nblk],
// totals [ncur], then (concat) the skip pass's starts (n + 1) and its status
size_t kx_nested_ws_bytes(const KxnProgram& P, uint64_t n, bool concat) {
  const uint64_t nblk = (n + RB - 1) / RB;
  size_t s = 64 + ((n + 63) & ~63ull) + (size_t)P.ncur * n * 4 + 64 + (size_t)P.ncur * nblk * 8 + P.ncur * 8 + 64;
  if (concat) s += (n + 1) * 8 + 64 + sizeof(kx_status) + 64;
  if (concat && P.pb) s += 2 * ((n * 8 + 63) & ~63ull);   // Batch frame body extents
  return s + 4096;
}

namespace {
struct NwsLayout {
  unsigned long long* errkey;
  uint32_t* flag;
  uint8_t* rcode;
  uint32_t* counts;
  uint64_t* bsum;
  uint64_t* totals;
  uint64_t* starts;
  kx_status* skip_st;
  uint64_t* bstart;
  uint64_t* bend;
};
NwsLayout layout(void* ws, const KxnProgram& P, uint64_t n) {
  NwsLayout L;
  char* p = (char*)ws;
  const uint64_t nblk = (n + RB - 1) / RB;
  L.errkey = (unsigned long long*)p;
  L.flag = (uint32_t*)(p + 8);
  p += 64;
  L.rcode = (uint8_t*)p;
  p += (n + 63) & ~63ull;
  L.counts = (uint32_t*)p;
  p += ((size_t)P.ncur * n * 4 + 63) & ~63ull;
  L.bsum = (uint64_t*)p;
  p += (size_t)P.ncur * nblk * 8;
  L.totals = (uint64_t*)p;
  p += ((size_t)P.ncur * 8 + 63) & ~63ull;
  L.starts = (uint64_t*)p;
  p += ((n + 1) * 8 + 63) & ~63ull;
  L.skip_st = (kx_status*)p;
  p += (sizeof(kx_status) + 63) & ~(size_t)63;
  L.bstart = (uint64_t*)p;
  p += (n * 8 + 63) & ~63ull;
  L.bend = (uint64_t*)p;
  return L;
}
}  // namespace

// decode (totals_out != null: sizes only, the cursor totals are copied there and the status is final
// when the stream reaches this point)
int kx_launch_nested_decode(const KxnProgram* dprog, const KxnProgram& hprog, const uint8_t* in, uint64_t in_len,
                            const uint64_t* offsets, const uint64_t* ends, uint64_t n, const KxnCols* dcols,
                            uint8_t* record_status, kx_status* status, void* ws, size_t ws_size,
                            void* skip_ws, size_t skip_ws_size, uint64_t skip_epoch, hipStream_t stream,
                            uint64_t* totals_out, const uint64_t* cur_base_dev, uint64_t* totals_dev) {
  if (hprog.nsnap > SNAP || hprog.ncur > CUR || hprog.ncur == 0) return KX_ERR_NOT_IMPLEMENTED;
  const bool concat = offsets == nullptr;
  if (ws_size < kx_nested_ws_bytes(hprog, n, concat)) return KX_ERR_INVALID_ARG;
  NwsLayout L = layout(ws, hprog, n);
  NParams p{};
  p.P = dprog;
  p.C = dcols;
  p.in = in;
  p.in_len = in_len;
  p.n = n;
  p.concat = concat;
  p.ends = ends;
  p.counts = L.counts;
  p.bsum = L.bsum;
  p.totals = L.totals;
  p.rcode = L.rcode;
  p.errkey = L.errkey;
  p.flag = L.flag;
  p.record_status = record_status;
  p.status = status;
  p.nblk = (n + RB - 1) / RB;
  p.ncur = hprog.ncur;
  p.sizes_only = totals_out != nullptr;
  p.cur_base = cur_base_dev;
  p.totals_out = totals_dev;
  KX_HIP_CHECK(hipMemsetAsync(status, 0, sizeof(kx_status), stream));
  KX_HIP_CHECK(hipMemsetAsync(L.errkey, 0xff, 8, stream));
  KX_HIP_CHECK(hipMemsetAsync(L.flag, 0, 4, stream));
  if (concat && hprog.pb) {
    // Kitex-PB Batch body: the frames (0x0A, uvarint length) on the frame pipeline of kx_decode.hip
    int rc = kx_launch_pb_frames(in, in_len, n, L.starts, L.bstart, L.bend, L.skip_st, skip_ws, skip_ws_size,
                                 skip_epoch, stream);
    if (rc) return rc;
    p.offsets = L.starts;
    p.skip_st = L.skip_st;
    p.bstart = L.bstart;
    p.bend = L.bend;
  } else if (concat) {
    // record boundaries: the skip decoder (codec_apache.go:166-172) on the pipeline of kx_decode.hip
    int rc = kx_launch_skip(in, in_len, n, L.starts, L.skip_st, skip_ws, skip_ws_size, skip_epoch, stream);
    if (rc) return rc;
    p.offsets = L.starts;
    p.skip_st = L.skip_st;
  } else {
    p.offsets = offsets;
  }
  // the cursors in LDS when they fit beside the program at two workgroups per CU (KX_NESTED_LDS=0: scratch)
  const size_t curl = (size_t)hprog.ncur * (8 + 4 * NTD);
  const bool lc = kx_knob(KXK_NESTED_LDS) && sizeof(KxnProgram) + curl <= 160 * 1024;
  const dim3 gw((unsigned)((n + NTD - 1) / NTD));
  auto mk = hprog.pb ? (lc ? measure_kernel<true, true> : measure_kernel<false, true>)
                     : (lc ? measure_kernel<true, false> : measure_kernel<false, false>);
  hipLaunchKernelGGL(mk, gw, dim3(NTD), lc ? curl : 0, stream, p);
  KX_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(bsum_kernel, dim3((unsigned)p.nblk, hprog.ncur), dim3(NT), 0, stream, p);
  KX_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(bscan_kernel, dim3(hprog.ncur), dim3(1024), 0, stream, p);
  KX_HIP_CHECK(hipGetLastError());
  if (totals_out) {
    KX_HIP_CHECK(hipMemcpyAsync(totals_out, L.totals, hprog.ncur * 8, hipMemcpyDeviceToHost, stream));
    // the status of the measure pass: the first failing record
    hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(64), 0, stream, p);
    KX_HIP_CHECK(hipGetLastError());
    return KX_OK;
  }
  hipLaunchKernelGGL(check_kernel, dim3(1), dim3(64), 0, stream, p);
  KX_HIP_CHECK(hipGetLastError());
  const bool cl = lc && 2 * (sizeof(KxnProgram) + curl + KXN_COLS_HEAD) <= 160 * 1024;
  auto wk = hprog.pb ? (cl ? write_kernel<true, true, true> : lc ? write_kernel<true, true, false> : write_kernel<false, true, false>)
                     : (cl ? write_kernel<true, false, true> : lc ? write_kernel<true, false, false> : write_kernel<false, false, false>);
  hipLaunchKernelGGL(wk, gw, dim3(NTD), cl ? curl + KXN_COLS_HEAD : lc ? curl : 0, stream, p);
  KX_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(64), 0, stream, p);
  KX_HIP_CHECK(hipGetLastError());
  return KX_OK;
}

size_t kx_nested_enc_ws_bytes(uint64_t n) { return (n + 64) * 8 + ((n + ERB - 1) / ERB) * 8 + 256; }

int kx_launch_nested_encode(const KxnProgram* dprog, const KxnProgram& hprog, const KxnCols* dcols, uint64_t n,
                            uint8_t* out, uint64_t out_cap, uint64_t* sizes_out, uint64_t* offsets_out,
                            kx_status* status, void* ws, size_t ws_size, hipStream_t stream, bool sizes_only,
                            const uint64_t* out_base) {
  if (ws_size < kx_nested_enc_ws_bytes(n)) return KX_ERR_INVALID_ARG;
  EParams p{};
  p.P = dprog;
  p.C = dcols;
  p.n = n;
  p.out = out;
  p.out_cap = out_cap;
  p.nblk = (n + ERB - 1) / ERB;
  p.bsum = (uint64_t*)ws;
  p.sizes = sizes_out ? sizes_out : (uint64_t*)ws + ((p.nblk + 63) & ~63ull);
  p.offsets_out = offsets_out;
  p.status = status;
  p.out_base = out_base;
  if (status) KX_HIP_CHECK(hipMemsetAsync(status, 0, sizeof(kx_status), stream));
  hipLaunchKernelGGL(hprog.pb ? esize_kernel<true> : esize_kernel<false>, dim3((unsigned)p.nblk), dim3(NT), 0, stream, p);
  KX_HIP_CHECK(hipGetLastError());
  if (sizes_only) return KX_OK;
  hipLaunchKernelGGL(escan_kernel, dim3(1), dim3(1024), 0, stream, p);
  KX_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(hprog.pb ? ewrite_kernel<true> : ewrite_kernel<false>, dim3((unsigned)p.nblk), dim3(NT), 0, stream, p);
  KX_HIP_CHECK(hipGetLastError());
  return KX_OK;
}
