// kx_crc.h — the CRC-32C pieces shared by the checksum kernel (kx_crc.hip) and the frame pipeline's emit
// pass (kx_decode.hip, CRC32Check fused into the frame walk): the slicing-by-k update and the TTHeader
// "crc32c" lookup of crcPayloadValidator (pkg/remote/codec/validate.go:168-217), over any byte source.
#pragma once
#include <stdint.h>

#include "../../include/kxcodec.h"

#define KX_CRC_POLY 0x82F63B78u  // Castagnoli, reflected

// Slicing tables t[k][b] = CRC of byte b followed by k zero bytes, built by a workgroup: thread `tid` of
// `nt` (nt >= 256) fills column tid; the caller puts a barrier between the two halves (t[0] first).
template <class TAB>
__device__ __forceinline__ uint32_t kx_crc_t0(TAB t, int tid) {
  uint32_t c = (uint32_t)tid;
  for (int k = 0; k < 8; k++) c = c & 1 ? (c >> 1) ^ KX_CRC_POLY : c >> 1;
  t[0][tid] = c;
  return c;
}
template <class TAB>
__device__ __forceinline__ void kx_crc_tk(TAB t, int tid, uint32_t c) {
  for (int k = 1; k < 8; k++) {
    c = (c >> 8) ^ t[0][c & 0xff];
    t[k][tid] = c;
  }
}

// c after feeding the k (0..8) low bytes of d (little-endian; bytes >= k of d must be zero): the
// slicing-by-k form of the byte-at-a-time update, k table lookups, no dependent chain between them
template <class TAB>
__device__ __forceinline__ uint32_t kx_crc_upd_k(TAB t, uint32_t c, uint64_t d, uint32_t k) {
  const uint32_t xl = c ^ (uint32_t)d, xh = (uint32_t)(d >> 32);
  uint32_t r = k == 0 ? c : k < 4 ? xl >> (8 * k) : 0u;
#pragma unroll
  for (uint32_t j = 0; j < 4; j++)
    if (j < k) r ^= t[k - 1 - j][(xl >> (8 * j)) & 0xff];
#pragma unroll
  for (uint32_t j = 0; j < 4; j++)
    if (j + 4 < k) r ^= t[k - 5 - j][(xh >> (8 * j)) & 0xff];
  return r;
}

__device__ __forceinline__ int kx_hexval(uint32_t ch) {
  return ch >= '0' && ch <= '9' ? (int)(ch - '0') : ch >= 'a' && ch <= 'f' ? (int)(ch - 'a' + 10) : -1;
}

// Expected value of frame f (TTHeader at [f, in_len)); rd(p) = input byte p. want = 0 no check (not a
// TTHeader frame, no "crc32c" key, or an empty value), 1 compare with exp, 2 a value that no lowercase
// 8-digit hex CRC can equal (always fails). Payload range [*a, *b) (payloadChecksumValidate,
// validate.go:91-127: everything after the TTHeader). Header layout as kx_decode.hip frame_one / the oracle.
template <class RD>
__device__ int kx_frame_expect(const RD& rd, uint64_t in_len, uint64_t f, uint64_t* a, uint64_t* b, int* want,
                               uint32_t* exp) {
  auto be16 = [&](uint64_t p) { return (rd(p) << 8) | rd(p + 1); };
  auto be32 = [&](uint64_t p) { return (be16(p) << 16) | be16(p + 2); };
  *want = 0;
  *a = *b = f;
  if (f > in_len || in_len - f < 14) return KX_OK;  // too short for a TTHeader: not one (the scan decides)
  if ((be32(f + 4) >> 16) != 0x1000u) return KX_OK;  // IsTTHeader
  const uint64_t len = (uint64_t)be32(f) + 4, hs = (uint64_t)be16(f + 12) * 4;
  if (hs < 2 || 14 + hs > len || len > in_len - f) return KX_ERR_UNKNOWN_PROTOCOL;
  *a = f + 14 + hs;
  *b = f + len;
  const uint64_t info = f + 14;
  uint64_t i = 2 + (uint64_t)rd(info + 1);
  if (i > hs) return KX_ERR_UNKNOWN_PROTOCOL;
  while (i < hs) {
    const uint32_t id = rd(info + i++);
    if (id == 0x00) continue;
    if (id == 0x01) {  // string KVs: the last "crc32c" wins (a map assignment per pair)
      if (i + 2 > hs) return KX_ERR_UNKNOWN_PROTOCOL;
      const uint32_t k = be16(info + i);
      i += 2;
      for (uint32_t j = 0; j < k; j++) {
        if (i + 2 > hs) return KX_ERR_UNKNOWN_PROTOCOL;
        const uint64_t kl = be16(info + i);
        if (i + 2 + kl + 2 > hs) return KX_ERR_UNKNOWN_PROTOCOL;
        const uint64_t key = info + i + 2;
        i += 2 + kl;
        const uint64_t vl = be16(info + i);
        if (i + 2 + vl > hs) return KX_ERR_UNKNOWN_PROTOCOL;
        const uint64_t v = info + i + 2;
        i += 2 + vl;
        if (kl == 6 && rd(key) == 'c' && rd(key + 1) == 'r' && rd(key + 2) == 'c' && rd(key + 3) == '3' &&
            rd(key + 4) == '2' && rd(key + 5) == 'c') {
          if (vl == 0) {
            *want = 0;
          } else {
            uint32_t x = 0;
            bool ok = vl == 8;
            for (int q = 0; ok && q < 8; q++) {
              const int d = kx_hexval(rd(v + q));
              ok = d >= 0;
              x = (x << 4) | (uint32_t)(d & 15);
            }
            *want = ok ? 1 : 2;
            *exp = x;
          }
        }
      }
    } else if (id == 0x10) {  // int KVs: (u16 key, u16-length string)
      if (i + 2 > hs) return KX_ERR_UNKNOWN_PROTOCOL;
      const uint32_t k = be16(info + i);
      i += 2;
      for (uint32_t j = 0; j < k; j++) {
        if (i + 4 > hs) return KX_ERR_UNKNOWN_PROTOCOL;
        const uint64_t l = be16(info + i + 2);
        if (i + 4 + l > hs) return KX_ERR_UNKNOWN_PROTOCOL;
        i += 4 + l;
      }
    } else if (id == 0x11) {  // ACL token
      if (i + 2 > hs) return KX_ERR_UNKNOWN_PROTOCOL;
      const uint64_t l = be16(info + i);
      if (i + 2 + l > hs) return KX_ERR_UNKNOWN_PROTOCOL;
      i += 2 + l;
    } else {
      return KX_ERR_UNKNOWN_PROTOCOL;
    }
  }
  return KX_OK;
}
