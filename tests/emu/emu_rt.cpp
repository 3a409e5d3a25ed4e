// Test infrastructure only: SIMT emulator runtime for running kx_decode.hip on the CPU.
// One OS thread runs one workgroup at a time; every lane is a ucontext fiber; wave intrinsics
// and __syncthreads are rendezvous points; workgroups on different OS threads run truly
// concurrently, so the cross-tile look-back sees real interleavings.
#include <sched.h>
#include <ucontext.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "hip/hip_runtime.h"

namespace {

constexpr size_t STACK = 256 << 10;

struct Fiber {
  ucontext_t ctx;
  char* stack = nullptr;
  bool done = false;
};

struct Wave {
  int gen = 0, arrived = 0, live = 0;
  uint64_t slot[64], snap[64];
};
static_assert(sizeof(uint64_t) == 8, "");

struct WG {
  std::vector<Fiber> f;
  int cur = 0, nthreads = 0;
  ucontext_t sched;
  Wave wave[16];
  int bar_gen = 0, bar_arrived = 0, bar_live = 0;
  unsigned block = 0, grid = 0;
  void (*tramp)(void*) = nullptr;
  void* arg = nullptr;
};

thread_local WG* g_wg = nullptr;

void fiber_main(int idx) {
  WG* wg = g_wg;
  wg->tramp(wg->arg);
  wg->f[idx].done = true;
  wg->wave[idx / 64].live--;
  wg->bar_live--;
}

void run_wg(unsigned b, unsigned grid, unsigned block, void (*tramp)(void*), void* arg) {
  WG wg;
  wg.nthreads = (int)block;
  wg.block = b;
  wg.grid = grid;
  wg.tramp = tramp;
  wg.arg = arg;
  wg.f.resize(block);
  for (unsigned i = 0; i < block; i++) wg.wave[i / 64].live++;
  wg.bar_live = (int)block;
  g_wg = &wg;
  for (unsigned i = 0; i < block; i++) {
    Fiber& fb = wg.f[i];
    fb.stack = (char*)malloc(STACK);
    getcontext(&fb.ctx);
    fb.ctx.uc_stack.ss_sp = fb.stack;
    fb.ctx.uc_stack.ss_size = STACK;
    fb.ctx.uc_link = &wg.sched;
    makecontext(&fb.ctx, (void (*)())fiber_main, 1, (int)i);
  }
  int remaining = (int)block;
  while (remaining > 0) {
    for (unsigned i = 0; i < block; i++) {
      if (wg.f[i].done) continue;
      wg.cur = (int)i;
      swapcontext(&wg.sched, &wg.f[i].ctx);
      if (wg.f[i].done) remaining--;
    }
    sched_yield();
  }
  for (auto& fb : wg.f) free(fb.stack);
  g_wg = nullptr;
}

}  // namespace

EmuTid emu_thread_idx() { return EmuTid{(unsigned)g_wg->cur, 0, 0}; }
EmuTid emu_block_idx() { return EmuTid{g_wg->block, 0, 0}; }
EmuTid emu_grid_dim() { return EmuTid{g_wg->grid, 1, 1}; }
int emu_threads() {
  const char* e = getenv("KX_EMU_THREADS");
  int nt = e ? atoi(e) : 8;
  return nt < 1 ? 1 : nt;
}
int emu_lane() { return g_wg->cur & 63; }

void emu_yield() {
  WG* wg = g_wg;
  swapcontext(&wg->f[wg->cur].ctx, &wg->sched);
}

uint64_t emu_wave_xchg(uint64_t v, uint64_t* all) {
  WG* wg = g_wg;
  Wave& w = wg->wave[wg->cur / 64];
  const int lane = wg->cur & 63;
  const int my = w.gen;
  w.slot[lane] = v;
  if (++w.arrived == w.live) {
    memcpy(w.snap, w.slot, sizeof w.snap);
    w.arrived = 0;
    w.gen++;
  } else {
    while (w.gen == my) emu_yield();
  }
  memcpy(all, w.snap, sizeof w.snap);
  return v;
}

void emu_sync_wg() {
  WG* wg = g_wg;
  const int my = wg->bar_gen;
  if (++wg->bar_arrived == wg->bar_live) {
    wg->bar_arrived = 0;
    wg->bar_gen++;
  } else {
    while (wg->bar_gen == my) emu_yield();
  }
}

uint64_t emu_clock_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void emu_launch(unsigned grid, unsigned block, void (*tramp)(void*), void* arg) {
  const int nt = emu_threads();
  std::atomic<unsigned> next{0};
  std::vector<std::thread> th;
  for (int i = 0; i < nt; i++)
    th.emplace_back([&] {
      for (;;) {
        unsigned b = next.fetch_add(1);
        if (b >= grid) break;
        run_wg(b, grid, block, tramp, arg);
      }
    });
  for (auto& t : th) t.join();
}
