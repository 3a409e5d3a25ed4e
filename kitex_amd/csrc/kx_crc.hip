// kx_crc.hip — CRC32C payload checksums of an RPC batch on CDNA4 / gfx950.
//
// Reference: crcPayloadValidator (pkg/remote/codec/validate.go:168-217). Generate = getCRC32C
// (:208-217): crc32.Update(0, Castagnoli table, payload), i.e. the standard CRC-32C (reflected
// polynomial 0x82F63B78, init and final xor ~0), big-endian hex. Validate (:190-201): an empty expected
// value passes; otherwise the hex of the payload's CRC must equal it (string compare), else
// perrors.InvalidData wrapped in kerrors.ErrPayloadValidation (KX_ERR_PAYLOAD_VALIDATION here).
// payloadChecksumValidate (:91-127) runs in DecodeMeta after the TTHeader is read (default_codec.go:
// 205-209): the expected value is the TTHeader string-KV info under "crc32c" (transmeta.HeaderCRC32C,
// transmeta/metakey.go:67) and the payload is everything after the TTHeader (PayloadLen, including the
// Framed length prefix of TTHeaderFramed: encodeMetaAndPayloadWithPayloadValidator, :263-300).
//
// One kernel, lane = range (payload). Byte work is table-driven (slicing-by-k, tables in LDS):
// * a range of <= LARGE bytes is folded by its own lane: 16-byte aligned granules in blocks of 8 (the
//   block's loads back to back, the next block in flight), each granule folded as two slicing-by-k steps
//   (k table lookups for k bytes, no per-byte chain);
// * longer ranges are taken by the whole wave, one after another: lane l folds the l-th 4 KiB chunk
//   (aligned to absolute 4 KiB boundaries) of a 256 KiB stretch, and the 64 chunk CRCs are combined in
//   order with crc(A||B) = x^(8|B|) * crc(A) + crc(B) mod P (zlib's crc32_combine): a whole chunk is a
//   multiplication by the constant x^(8*4096), applied with four 256-entry LDS tables; a partial chunk
//   (the range's last) uses the generic carry-less multiply.
// Bound: HBM read of the payload bytes (the LDS lookups are ~1 per byte per lane, well under the LDS
// issue rate); ranges are read once. The persistent grid is sized to what is resident at once.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <atomic>

#include "kx_internal.h"
#include "kx_crc.h"
#include "kx_mem.h"

namespace {

constexpr int CT = 256;                  // threads per workgroup
constexpr uint64_t CHUNK = 4096;         // per-lane chunk of a wave-cooperative range
constexpr uint64_t LARGE = 2048;         // longer ranges are folded by the whole wave
constexpr uint64_t MAX_WG = 2048;        // persistent grid when the occupancy query fails

struct CrcParams {
  const uint8_t* in;
  uint64_t in_len;
  const uint64_t* offs;      // GEN: range i = [offs[i], offs[i+1]); VAL: frame i starts at offs[i]
  uint64_t n;
  int val;                   // 1: validate TTHeader frames, 0: generate over ranges
  const kx_status* pre;      // VAL: framing-scan status: frames from its failing frame on are skipped
  uint32_t* crc_out;         // optional (VAL) / required (GEN)
  uint8_t* rs;               // VAL: per-frame code (optional)
  unsigned long long* errkey;
};

struct Tabs {
  uint32_t t[8][256];   // slicing-by-8
  uint32_t s[4][256];   // multiplication by x^(8 * CHUNK), byte-sliced
  uint32_t x2n[32];     // x^(2^k) mod P
};

// a * b mod P (reflected; zlib multmodp). a must be non-zero.
__device__ __forceinline__ uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = b & 1 ? (b >> 1) ^ KX_CRC_POLY : b >> 1;
  }
  return p;
}

// x^(n * 2^k) mod P
__device__ __forceinline__ uint32_t x2nmodp(const Tabs& T, uint64_t n, unsigned k) {
  uint32_t p = 1u << 31;  // x^0
  while (n) {
    if (n & 1) p = multmodp(T.x2n[k & 31], p);
    n >>= 1;
    k++;
  }
  return p;
}

__device__ void build_tabs(Tabs& T) {
  const int t = threadIdx.x;
  uint32_t c = (uint32_t)t;
  for (int k = 0; k < 8; k++) c = c & 1 ? (c >> 1) ^ KX_CRC_POLY : c >> 1;
  T.t[0][t] = c;
  if (t == 0) {
    uint32_t p = 1u << 30;  // x^1
    T.x2n[0] = p;
    for (int k = 1; k < 32; k++) T.x2n[k] = p = multmodp(p, p);
  }
  __syncthreads();
  for (int k = 1; k < 8; k++) {
    c = (c >> 8) ^ T.t[0][c & 0xff];
    T.t[k][t] = c;
  }
  const uint32_t K = x2nmodp(T, CHUNK, 3);
  for (int j = 0; j < 4; j++) T.s[j][t] = multmodp(K, (uint32_t)t << (8 * j));
  __syncthreads();
}

__device__ __forceinline__ uint64_t low_bytes(uint64_t v, uint32_t k) { return k >= 8 ? v : v & ((1ull << (8 * k)) - 1); }

// the 16-byte aligned granule at p: it holds a byte of the range, so it lies inside mapped memory
__device__ __forceinline__ uint4 ld_granule(const uint8_t* p) { return kx_ld16(p); }

// standard CRC-32C of in[a, b): 16-byte aligned granules (absolute addresses), two loads in flight
// ahead of the fold; the bytes of a granule outside [a, b) are shifted / masked away, so every granule
// (whole or partial) is the same two upd_k steps and lanes at different alignments never diverge
__device__ __forceinline__ uint32_t crc_run(const Tabs& T, const uint8_t* in, uint64_t a, uint64_t b) {
  if (a >= b) return 0u;
  const uint8_t* pa = in + a;
  const uint8_t* pb = in + b;
  const uint8_t* g = (const uint8_t*)((uintptr_t)pa & ~(uintptr_t)15);
  uint32_t c = 0xffffffffu;
  uint4 v0 = ld_granule(g);
  uint4 v1 = g + 16 < pb ? ld_granule(g + 16) : v0;
  for (;;) {
    const uint4 v2 = g + 32 < pb ? ld_granule(g + 32) : v1;
    const uint32_t lo = pa > g ? (uint32_t)(pa - g) : 0u;
    const uint32_t hi = pb - g < 16 ? (uint32_t)(pb - g) : 16u;
    uint64_t q0 = (uint64_t)v0.x | ((uint64_t)v0.y << 32), q1 = (uint64_t)v0.z | ((uint64_t)v0.w << 32);
    const uint32_t s = 8 * lo;
    if (s >= 64) { q0 = q1 >> (s - 64); q1 = 0; }
    else if (s) { q0 = (q0 >> s) | (q1 << (64 - s)); q1 >>= s; }
    const uint32_t k = hi - lo, k1 = k < 8 ? k : 8u, k2 = k - k1;
    c = kx_crc_upd_k(T.t, c, low_bytes(q0, k1), k1);
    c = kx_crc_upd_k(T.t, c, low_bytes(q1, k2), k2);
    g += 16;
    if (g >= pb) break;
    v0 = v1;
    v1 = v2;
  }
  return ~c;
}

// a granule (16 bytes, q0 | q1 << 64) of which bytes [lo, hi) belong to the range
__device__ __forceinline__ uint32_t fold_masked(const Tabs& T, uint32_t c, uint64_t q0, uint64_t q1, uint32_t lo,
                                                uint32_t hi) {
  const uint32_t k = hi - lo, k1 = k < 8 ? k : 8u, k2 = k - k1;
  const uint32_t s = 8 * lo;
  if (s >= 64) { q0 = q1 >> (s - 64); q1 = 0; }
  else if (s) { q0 = (q0 >> s) | (q1 << (64 - s)); q1 >>= s; }
  c = kx_crc_upd_k(T.t, c, low_bytes(q0, k1), k1);
  return kx_crc_upd_k(T.t, c, low_bytes(q1, k2), k2);
}

// the same in blocks of G granules from the range's first granule: the block's G loads go out back to
// back, so the lines they share are read while still in the L1 (the single-granule walk above re-reads
// each 128-byte line from the L2 up to 8 times when 64 lanes walk 64 records), and the next block is in
// flight while this one is folded (2G loads outstanding). Only the first and the last granule are
// masked; the ones between are two plain slicing-by-8 steps. Measured on the MI355X (CRC of each of 16 M
// R2 records, 5.08 GB, grid sized to residency): the single-granule walk 2.91 ms, G = 2 1.45, G = 4 1.30,
// G = 8 1.09 (4.7 TB/s, 133 VGPRs); G = 8, 12 or 16 without the next block in flight 1.16 / 1.16 / 1.10
// (16 spills). KX_CRC_BLK = 1 / 4 / 8 (default) picks the form, for A/B runs.
template <int G>
__device__ __forceinline__ uint32_t crc_run_blk(const Tabs& T, const uint8_t* in, uint64_t a, uint64_t b) {
  if (a >= b) return 0u;
  const uint8_t* pa = in + a;
  const uint8_t* pb = in + b;
  const uint8_t* g = (const uint8_t*)((uintptr_t)pa & ~(uintptr_t)15);
  const uint32_t lo0 = (uint32_t)(pa - g);
  const uint32_t ng = (uint32_t)((pb - g + 15) >> 4);            // granules holding range bytes
  const uint32_t hil = (uint32_t)(pb - (g + 16 * (uint64_t)(ng - 1)));  // bytes of the last one (1..16)
  uint32_t c = 0xffffffffu;
  uint4 cur[G], nxt[G];
#pragma unroll
  for (int j = 0; j < G; j++) cur[j] = (uint32_t)j < ng ? ld_granule(g + 16 * j) : make_uint4(0, 0, 0, 0);
  for (uint32_t i0 = 0;; i0 += G) {
#pragma unroll
    for (int j = 0; j < G; j++)
      nxt[j] = i0 + G + j < ng ? ld_granule(g + 16 * (uint64_t)(i0 + G + j)) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < G; j++) {
      const uint32_t i = i0 + j;
      const uint64_t q0 = (uint64_t)cur[j].x | ((uint64_t)cur[j].y << 32), q1 = (uint64_t)cur[j].z | ((uint64_t)cur[j].w << 32);
      if (i == 0 || i + 1 == ng) {
        if (i < ng) c = fold_masked(T, c, q0, q1, i == 0 ? lo0 : 0u, i + 1 == ng ? hil : 16u);
      } else if (i < ng) {
        c = kx_crc_upd_k(T.t, c, q0, 8);
        c = kx_crc_upd_k(T.t, c, q1, 8);
      }
    }
    if (i0 + G >= ng) break;
#pragma unroll
    for (int j = 0; j < G; j++) cur[j] = nxt[j];
  }
  return ~c;
}

__device__ __forceinline__ uint32_t shift_chunk(const Tabs& T, uint32_t c) {
  return T.s[0][c & 0xff] ^ T.s[1][(c >> 8) & 0xff] ^ T.s[2][(c >> 16) & 0xff] ^ T.s[3][c >> 24];
}

// the frame's bytes straight from global memory
struct GlobalBytes {
  const uint8_t* in;
  __device__ __forceinline__ uint32_t operator()(uint64_t p) const { return in[p]; }
};

template <int G>
__device__ __forceinline__ void crc_block(const CrcParams& cp, const Tabs& T, uint64_t i);

// persistent: the tables are built once per workgroup, which then takes blocks of CT ranges
template <int G>
__global__ void __launch_bounds__(CT) crc_kernel(CrcParams cp) {
  __shared__ Tabs T;
  build_tabs(T);
  const uint64_t nblk = (cp.n + CT - 1) / CT;
  for (uint64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) crc_block<G>(cp, T, blk * CT + threadIdx.x);
}

// one range per lane (i); the long ones of the wave folded by the whole wave
template <int G>
__device__ __forceinline__ void crc_block(const CrcParams& cp, const Tabs& T, uint64_t i) {
  const int lane = threadIdx.x & 63;
  int rc = KX_OK, want = 0;
  uint32_t exp = 0;
  uint64_t a = 0, b = 0;
  bool live = i < cp.n;
  if (live && cp.val && cp.pre && cp.pre->code && i >= (uint64_t)cp.pre->record) live = false;  // not delimited
  if (live) {
    if (cp.val) {
      rc = kx_frame_expect(GlobalBytes{cp.in}, cp.in_len, cp.offs[i], &a, &b, &want, &exp);
      if (rc) a = b = 0;
    } else {
      a = cp.offs[i];
      b = cp.offs[i + 1];
      if (a > b || b > cp.in_len) { rc = KX_ERR_INVALID_ARG; a = b = 0; }
    }
  }
  const bool large = b - a > LARGE;
  uint32_t crc = large ? 0u : G == 1 ? crc_run(T, cp.in, a, b) : crc_run_blk<G>(T, cp.in, a, b);
  // long ranges: the whole wave, one range at a time
  uint64_t big = __ballot(large);
  while (big) {
    const int l = __ffsll((unsigned long long)big) - 1;
    big &= big - 1;
    const uint64_t ra = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(a >> 32), l) << 32) |
                        __builtin_amdgcn_readlane((uint32_t)a, l);
    const uint64_t rb = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(b >> 32), l) << 32) |
                        __builtin_amdgcn_readlane((uint32_t)b, l);
    uint32_t acc = 0;
    for (uint64_t base = ra & ~(CHUNK - 1); base < rb; base += 64 * CHUNK) {
      const uint64_t s = kmax64(base + (uint64_t)lane * CHUNK, ra), e = kmin64(base + (uint64_t)(lane + 1) * CHUNK, rb);
      const uint32_t cr = s >= e ? 0u : G == 1 ? crc_run(T, cp.in, s, e) : crc_run_blk<G>(T, cp.in, s, e);
      const uint32_t ln = s < e ? (uint32_t)(e - s) : 0u;
      for (int k = 0; k < 64; k++) {  // combine in lane order (uniform: every lane keeps acc)
        const uint32_t lk = __builtin_amdgcn_readlane(ln, k);
        if (lk == 0) break;
        const uint32_t ck = __builtin_amdgcn_readlane(cr, k);
        if (lk == CHUNK) acc = shift_chunk(T, acc);
        else if (acc) acc = multmodp(x2nmodp(T, lk, 3), acc);
        acc ^= ck;
      }
    }
    if (lane == l) crc = acc;
  }
  if (!live) return;
  if (!cp.val) {
    cp.crc_out[i] = rc ? 0u : crc;
  } else {
    if (!rc && ((want == 1 && crc != exp) || want == 2)) rc = KX_ERR_PAYLOAD_VALIDATION;
    if (cp.crc_out) cp.crc_out[i] = b > a ? crc : 0u;
    if (cp.rs) cp.rs[i] = (uint8_t)rc;
  }
  if (rc) atomicMin(cp.errkey, (unsigned long long)((i << 8) | (uint64_t)(rc & 0xff)));
}

__global__ void crc_final_kernel(kx_status* st, const uint64_t* offs, uint64_t n, int val,
                                 unsigned long long* errkey, const kx_status* pre) {
  if (threadIdx.x != 0) return;
  const unsigned long long k = *errkey;
  *errkey = ~0ull;
  for (int j = 0; j < 3; j++) st->diag[j] = 0;
  for (int j = 0; j < 16; j++) st->var_total[j] = 0;
  if (k != ~0ull) {
    st->code = (int32_t)(k & 0xff);
    st->record = k >> 8;
    st->offset = offs[k >> 8];
  } else {
    st->code = 0;
    st->record = 0;
    st->offset = 0;
  }
  st->reserved0 = 0;
  st->n_records = val && pre && pre->code ? pre->record : n;
  st->consumed = val && pre && pre->code ? pre->offset : offs[n];
}

// the persistent grid is what fits on the device at once (a grid larger than that leaves a second,
// partly occupied round of workgroups behind the first)
template <int G>
void launch_crc(const CrcParams& cp, uint64_t nblk, hipStream_t stream) {
  static std::atomic<int> resident_dev[64];   // per device ordinal (0: not yet asked): devices may differ
  int dev = 0, resident = (int)MAX_WG;
  if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64) {
    resident = resident_dev[dev].load(std::memory_order_relaxed);
    if (!resident) {
      int ncu = 0, per = 0;
      resident = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                         hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, crc_kernel<G>, CT, 0) == hipSuccess &&
                         ncu > 0 && per > 0
                     ? ncu * per
                     : (int)MAX_WG;
      resident_dev[dev].store(resident, std::memory_order_relaxed);
    }
  }
  const unsigned grid = (unsigned)kmin64(nblk, (uint64_t)resident);
  hipLaunchKernelGGL(crc_kernel<G>, dim3(grid), dim3(CT), 0, stream, cp);
}

}  // namespace

int kx_launch_crc32c(const uint8_t* in, uint64_t in_len, const uint64_t* offs, uint64_t n, bool val,
                     const kx_status* pre, uint32_t* crc_out, uint8_t* rs, kx_status* status, void* scratch,
                     hipStream_t stream) {
  CrcParams cp{};
  cp.in = in; cp.in_len = in_len; cp.offs = offs; cp.n = n; cp.val = val ? 1 : 0; cp.pre = pre;
  cp.crc_out = crc_out; cp.rs = rs;
  cp.errkey = (unsigned long long*)scratch;
  const uint64_t nblk = (n + CT - 1) / CT;
  if (nblk) {
    const int blk = kx_knob(KXK_CRC_BLK);
    if (blk == 4) launch_crc<4>(cp, nblk, stream);
    else if (blk == 1) launch_crc<1>(cp, nblk, stream);
    else launch_crc<8>(cp, nblk, stream);
    KX_HIP_CHECK(hipGetLastError());
  }
  if (status) {
    hipLaunchKernelGGL(crc_final_kernel, dim3(1), dim3(64), 0, stream, status, offs, n, cp.val, cp.errkey, pre);
    KX_HIP_CHECK(hipGetLastError());
  }
  return KX_OK;
}
