// Test infrastructure only: a host-side stand-in for <hip/hip_runtime.h> that lets the decode
// kernel source (kitex_amd/csrc/kx_decode.hip) run on the CPU under a SIMT emulator
// (tests/emu/emu_rt.cpp): one fiber per lane, one OS thread per running workgroup, wave
// intrinsics as lane rendezvous. It exists to exercise the kernel's cross-tile logic
// (look-back, repair, error paths) without a GPU; it is never part of the product library.
#pragma once
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>
#include <utility>

#define __global__
#define __device__
#define __host__
#define __forceinline__ inline
#define __noinline__ __attribute__((noinline))
#define __launch_bounds__(...)
#define __shared__ static thread_local

template <typename A, typename B>
inline typename std::common_type<A, B>::type min(A a, B b) {
  return a < b ? a : b;
}
template <typename A, typename B>
inline typename std::common_type<A, B>::type max(A a, B b) {
  return a < b ? b : a;
}

typedef int hipError_t;
typedef void* hipStream_t;
enum { hipSuccess = 0 };
struct dim3 {
  unsigned x, y, z;
  dim3(unsigned a = 1, unsigned b = 1, unsigned c = 1) : x(a), y(b), z(c) {}
};

// ---- emulator runtime (emu_rt.cpp) ----
struct EmuTid {
  unsigned x, y, z;
};
EmuTid emu_thread_idx();
EmuTid emu_block_idx();
EmuTid emu_grid_dim();
int emu_threads();
int emu_lane();
void emu_yield();
void emu_sync_wg();
uint64_t emu_wave_xchg(uint64_t v, uint64_t* all);  // all lanes' values (64), returns own
void emu_launch(unsigned grid, unsigned block, void (*tramp)(void*), void* arg);
uint64_t emu_clock_ns();

#define threadIdx (emu_thread_idx())
#define blockIdx (emu_block_idx())
#define gridDim (emu_grid_dim())
#define blockDim (EmuTid{256, 1, 1})
inline void __syncthreads() { emu_sync_wg(); }
// an input dword holding the last input bytes: those bytes only (as ASan sees the input allocation), the
// rest 0xA5 (garbage on the device: no caller may depend on it)
inline uint32_t emu_gdword(uint64_t A, uint64_t end) {
  uint32_t x = 0xA5A5A5A5u;
  memcpy(&x, (const void*)A, end - A < 4 ? (size_t)(end - A) : 4);
  return x;
}
inline void __builtin_amdgcn_fence(int, const char*) {}

inline uint64_t __ballot(int pred) {
  uint64_t all[64];
  emu_wave_xchg(pred ? 1 : 0, all);
  uint64_t m = 0;
  for (int i = 0; i < 64; i++) m |= (all[i] & 1ull) << i;
  return m;
}
template <typename T>
inline uint64_t emu_bits(T v) {
  uint64_t b = 0;
  memcpy(&b, &v, sizeof(T));
  return b;
}
template <typename T>
inline T emu_from(uint64_t b) {
  T v;
  memcpy(&v, &b, sizeof(T));
  return v;
}
template <typename T>
inline T __shfl(T v, int src, int width = 64) {
  uint64_t all[64];
  emu_wave_xchg(emu_bits(v), all);
  return emu_from<T>(all[((unsigned)src) & 63]);
}
template <typename T>
inline T __shfl_up(T v, unsigned d, int width = 64) {
  uint64_t all[64];
  emu_wave_xchg(emu_bits(v), all);
  int l = emu_lane();
  return l >= (int)d ? emu_from<T>(all[l - d]) : v;
}
template <typename T>
inline T __shfl_xor(T v, int m, int width = 64) {
  uint64_t all[64];
  emu_wave_xchg(emu_bits(v), all);
  return emu_from<T>(all[(emu_lane() ^ m) & 63]);
}
inline void __builtin_amdgcn_wave_barrier() {
  uint64_t all[64];
  emu_wave_xchg(0, all);
}
// like the real builtins these return int (a sign-extension trap the emulator must reproduce)
inline int __builtin_amdgcn_readlane(int v, int l) {
  uint64_t all[64];
  emu_wave_xchg((uint32_t)v, all);
  return (int)(uint32_t)all[l & 63];
}
// only used where every active lane holds the same value
inline int __builtin_amdgcn_readfirstlane(int v) { return v; }
// src and l are wave-uniform where the kernels use it
inline int emu_writelane(int old, int src, int l) { return emu_lane() == (l & 63) ? src : old; }

// DPP moves the kernels use: row_shr:1..15 (0x111..0x11f), row_bcast:15 (0x142), row_bcast:31 (0x143); a lane of
// a row outside row_mask, or whose source lies outside its row, keeps `old` (bound_ctrl: 0)
inline int __builtin_amdgcn_update_dpp(int old, int src, int ctrl, int row_mask, int bank_mask, bool bound_ctrl) {
  (void)bank_mask;
  uint64_t all[64];
  emu_wave_xchg((uint32_t)src, all);
  const int l = emu_lane(), row = l >> 4;
  if (!((row_mask >> row) & 1)) return old;
  int sl = -1;
  if (ctrl >= 0x111 && ctrl <= 0x11f) {
    const int d = ctrl - 0x110;
    if ((l & 15) >= d) sl = l - d;
  } else if (ctrl == 0x142) {
    if (row >= 1) sl = (l & ~15) - 1;
  } else if (ctrl == 0x143) {
    if (row >= 2) sl = 31;
  } else {
    abort();
  }
  if (sl < 0) return bound_ctrl ? 0 : old;
  return (int)(uint32_t)all[sl];
}
inline uint32_t __builtin_amdgcn_alignbyte(uint32_t hi, uint32_t lo, uint32_t s) {
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> ((s & 3) * 8));
}
inline uint32_t __builtin_amdgcn_perm(uint32_t a, uint32_t b, uint32_t sel) {
  uint64_t c = ((uint64_t)a << 32) | b;
  uint32_t r = 0;
  for (int i = 0; i < 4; i++) {
    uint32_t s = (sel >> (8 * i)) & 0xff, byte;
    if (s < 8) byte = (c >> (8 * s)) & 0xff;
    else if (s == 12) byte = 0;
    else byte = 0xff;
    r |= byte << (8 * i);
  }
  return r;
}
inline uint64_t __builtin_amdgcn_s_memtime() { return emu_clock_ns(); }
inline uint64_t __builtin_amdgcn_s_memrealtime() { return emu_clock_ns() / 10; }
inline void __builtin_amdgcn_s_sleep(int) { emu_yield(); }
inline void emu_wait_vmcnt0() {  // the DMA of every lane of the wave has landed
  uint64_t all[64];
  emu_wave_xchg(0, all);
}
inline void __builtin_amdgcn_global_load_lds(const void* src, void* dst, unsigned size, int, int) {
  memcpy((char*)dst + (size_t)emu_lane() * size, src, size);
}
struct emu_rsrc {
  const char* base;
  int32_t n;
};
typedef emu_rsrc __amdgpu_buffer_rsrc_t;
inline emu_rsrc __builtin_amdgcn_make_buffer_rsrc(void* p, short, int32_t n, int32_t) { return emu_rsrc{(const char*)p, n}; }
inline void __builtin_amdgcn_raw_ptr_buffer_load_lds(emu_rsrc r, void* dst, unsigned size, int voff, int soff, int off,
                                                     int) {
  // the range check turns a chunk past num_records into zeros: the LDS slot is still written
  const int64_t o = (int64_t)voff + soff + off;
  if (o + (int64_t)size <= r.n) memcpy((char*)dst + (size_t)emu_lane() * size, r.base + o, size);
  else memset((char*)dst + (size_t)emu_lane() * size, 0, size);
}
// the inline-assembly LDS DMA of load_window_async: rsrc dwords (base lo, base hi & 0xffff, num_records)
inline void emu_dma_lds16(uint32_t __attribute__((ext_vector_type(4))) rs, void* dst, uint32_t voff, uint32_t soff) {
  const char* base = (const char*)(((uint64_t)rs.y << 32) | rs.x);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(emu_rsrc{base, (int32_t)rs.z}, dst, 16, (int)voff, (int)soff, 0, 0);
}
struct uint4 { uint32_t x, y, z, w; };
inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) { return uint4{x, y, z, w}; }
inline int __ffsll(long long x) { return __builtin_ffsll(x); }
inline int __clzll(long long x) { return x ? __builtin_clzll((unsigned long long)x) : 64; }

#define __HIP_MEMORY_SCOPE_AGENT 0
#define __hip_atomic_load(p, order, scope) __atomic_load_n((p), __ATOMIC_RELAXED)
#define __hip_atomic_store(p, v, order, scope) __atomic_store_n((p), (v), __ATOMIC_RELAXED)

template <typename T, typename U>
inline T atomicAdd(T* p, U v) { return __atomic_fetch_add(p, (T)v, __ATOMIC_SEQ_CST); }
template <typename T, typename U>
inline T atomicOr(T* p, U v) { return __atomic_fetch_or(p, (T)v, __ATOMIC_SEQ_CST); }
template <typename T, typename U>
inline T atomicMin(T* p, U v) {
  T cur = __atomic_load_n(p, __ATOMIC_SEQ_CST);
  while ((T)v < cur && !__atomic_compare_exchange_n(p, &cur, (T)v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {
  }
  return cur;
}
template <typename T, typename U, typename V>
inline T atomicCAS(T* p, U cmp, V val) {
  T c = (T)cmp;
  __atomic_compare_exchange_n(p, &c, (T)val, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);
  return c;
}

template <typename F>
struct EmuThunk {
  F f;
  static void run(void* a) { ((EmuThunk*)a)->f(); }
};
#define hipLaunchKernelGGL(kern, grid, block, shmem, stream, ...)                  \
  do {                                                                            \
    auto emu_fn_ = [=]() { kern(__VA_ARGS__); };                                  \
    EmuThunk<decltype(emu_fn_)> emu_th_{emu_fn_};                                 \
    emu_launch(dim3(grid).x, dim3(block).x, &EmuThunk<decltype(emu_fn_)>::run, &emu_th_); \
  } while (0)
inline hipError_t hipGetLastError() { return hipSuccess; }
enum hipMemcpyKind { hipMemcpyHostToDevice = 1, hipMemcpyDeviceToHost = 2, hipMemcpyDeviceToDevice = 3 };
inline hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t) {
  memcpy(d, s, n);
  return hipSuccess;
}
inline hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
// streams and events: the emulator runs every launch at enqueue time, in enqueue order (a valid
// serialisation of any multi-stream schedule the event waits allow)
typedef void* hipEvent_t;
inline hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
inline hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned) { return hipSuccess; }
inline hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t) {
  memset(p, v, n);
  return hipSuccess;
}
#define HIP_SYMBOL(x) (&(x))
// the persistent decode grid is sized from these: one workgroup per emulator thread, all co-resident
enum hipDeviceAttribute_t { hipDeviceAttributeMultiprocessorCount = 0 };
// (one "device" per emulator thread count: the kernel caches its grid size per device)
inline hipError_t hipGetDevice(int* d) { *d = emu_threads() & 63; return hipSuccess; }
inline hipError_t hipDeviceGetAttribute(int* v, hipDeviceAttribute_t, int) { *v = emu_threads(); return hipSuccess; }
template <typename F>
inline hipError_t hipOccupancyMaxActiveBlocksPerMultiprocessor(int* n, F, int, size_t) { *n = 1; return hipSuccess; }
inline hipError_t hipMemcpyFromSymbol(void* dst, const void* sym, size_t n) {
  memcpy(dst, sym, n);
  return hipSuccess;
}
inline hipError_t hipMalloc(void** p, size_t n) {
  *p = calloc(1, n ? n : 1);
  return *p ? hipSuccess : (hipError_t)1;
}
inline hipError_t hipMemset(void* p, int v, size_t n) {
  memset(p, v, n);
  return hipSuccess;
}
inline hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind) {
  memcpy(d, s, n);
  return hipSuccess;
}
inline hipError_t hipMemcpyToSymbol(const void* sym, const void* src, size_t n) {
  memcpy((void*)sym, src, n);
  return hipSuccess;
}
