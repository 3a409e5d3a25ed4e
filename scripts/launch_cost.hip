// What an empty persistent kernel costs on the MI355X: the redo / emit_redo
// kernels of the decode exit at once when their queue is empty, yet took ~30 us each under rocprofv3.
// Each variant exits after one global load; they differ in what the kernel descriptor asks for:
// LDS (39 KB, as the general decode kernels), scratch (a dynamically indexed private array), both.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/launch_cost scripts/launch_cost.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void __launch_bounds__(256) k_plain(const uint32_t* q, uint32_t* out) {
  if (*(volatile const uint32_t*)q == 12345u) out[threadIdx.x] = 1;
}

__global__ void __launch_bounds__(256) k_lds(const uint32_t* q, uint32_t* out) {
  __shared__ uint32_t win[4][2440];
  if (*(volatile const uint32_t*)q == 12345u) {
    win[threadIdx.x >> 6][threadIdx.x] = 1;
    __syncthreads();
    out[threadIdx.x] = win[0][threadIdx.x ^ 1];
  }
}

__global__ void __launch_bounds__(256) k_scratch(const uint32_t* q, uint32_t* out) {
  volatile uint32_t priv[160];
  const uint32_t n = *(volatile const uint32_t*)q;
  if (n == 12345u) {
    for (int i = 0; i < 160; i++) priv[i] = i * n;
    out[threadIdx.x] = priv[(threadIdx.x * 7 + n) % 160];
  }
}

__global__ void __launch_bounds__(256) k_lds_scratch(const uint32_t* q, uint32_t* out) {
  __shared__ uint32_t win[4][2440];
  volatile uint32_t priv[160];
  const uint32_t n = *(volatile const uint32_t*)q;
  if (n == 12345u) {
    for (int i = 0; i < 160; i++) priv[i] = i * n;
    win[threadIdx.x >> 6][threadIdx.x] = priv[(threadIdx.x * 7 + n) % 160];
    __syncthreads();
    out[threadIdx.x] = win[0][threadIdx.x ^ 1];
  }
}

int main() {
  uint32_t *q, *out;
  CHECK(hipMalloc(&q, 64));
  CHECK(hipMalloc(&out, 4096));
  CHECK(hipMemset(q, 0, 64));
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  auto timeit = [&](const char* name, unsigned grid, auto&& launch) {
    for (int i = 0; i < 20; i++) launch(grid);
    CHECK(hipDeviceSynchronize());
    const int reps = 200;
    CHECK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; i++) launch(grid);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    printf("{\"kernel\": \"%s\", \"grid\": %u, \"us_per_launch\": %.2f}\n", name, grid, ms * 1e3f / reps);
    fflush(stdout);
  };
  for (unsigned grid : {256u, (unsigned)ncu * 4u, 8192u}) {
    timeit("plain", grid, [&](unsigned g) { k_plain<<<g, 256>>>(q, out); });
    timeit("lds39k", grid, [&](unsigned g) { k_lds<<<g, 256>>>(q, out); });
    timeit("scratch640", grid, [&](unsigned g) { k_scratch<<<g, 256>>>(q, out); });
    timeit("lds39k_scratch640", grid, [&](unsigned g) { k_lds_scratch<<<g, 256>>>(q, out); });
  }
  return 0;
}
