// kx_mem.h — global-memory accesses through address-space-1 pointers.
//
// A pointer the compiler cannot prove global (one rebuilt from an integer, read from LDS or from a
// dynamically indexed parameter array) is accessed with flat instructions, and a flat access counts on
// both the vector-memory and the LDS counters: the next wait for an LDS result then also waits for every
// outstanding flat load, so a kernel that mixes LDS lookups with its stream of global loads loses its
// loads in flight (the CRC fold, the encoder's payload copy). These casts make such accesses global_load /
// global_store. Only for pointers that do point at global memory.
#pragma once
#include <hip/hip_runtime.h>

#define KX_GLOBAL __attribute__((address_space(1)))

template <class T>
__device__ __forceinline__ T kx_ld(const T* p) {
  return *(const KX_GLOBAL T*)p;
}
template <class T>
__device__ __forceinline__ T kx_ld(uint64_t addr) {
  return *(const KX_GLOBAL T*)addr;
}
template <class T>
__device__ __forceinline__ void kx_st(T* p, T v) {
  *(KX_GLOBAL T*)p = v;
}
template <class T>
__device__ __forceinline__ void kx_st(uint64_t addr, T v) {
  *(KX_GLOBAL T*)addr = v;
}

// 16-byte accesses: HIP's uint4 class cannot be copied across address spaces, the clang vector can
typedef unsigned int kx_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 kx_ld16(const void* p) {
  const kx_u32x4 v = *(const KX_GLOBAL kx_u32x4*)p;
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void kx_st16(uint64_t addr, uint4 v) {
  kx_u32x4 w;
  w.x = v.x; w.y = v.y; w.z = v.z; w.w = v.w;
  *(KX_GLOBAL kx_u32x4*)addr = w;
}
