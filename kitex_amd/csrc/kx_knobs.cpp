// kx_knobs.cpp — the tuning switches of kx_knobs.h, read from the environment once per process, and the
// per-device compute-unit count, cached race-free.
#include "kx_knobs.h"

#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>

namespace {

struct KnobDef {
  const char* env;
  int def;
};
const KnobDef kDefs[KXK_N] = {
    {"KX_CHAIN_FAST", 1}, {"KX_EMIT_FAST", 1}, {"KX_FAST_NARROW", 1}, {"KX_FAST_SPLIT", 1}, {"KX_REDO_WG", 4},
    {"KX_FAST", 1},       {"KX_FASTPLAN", 1},  {"KX_SLOTCAP", 0},     {"KX_NOLDS", 0},      {"KX_DIAG", 0},
    {"KX_CRC_FUSED", 1},  {"KX_CRC_BLK", 8},   {"KX_ENC_DIRECT", 0},  {"KX_ENC_WCU", 16},   {"KX_ENC_CANON", 1},
    {"KX_CHUNK_MB", 0},   {"KX_CHUNK_AHEAD", 1}, {"KX_NESTED_LDS", 1}};

std::atomic<int> g_knob[KXK_N];
std::once_flag g_once;

void load() {
  std::call_once(g_once, [] {
    for (int k = 0; k < KXK_N; k++) {
      const char* e = getenv(kDefs[k].env);
      g_knob[k].store(e ? atoi(e) : kDefs[k].def, std::memory_order_relaxed);
    }
  });
}

std::atomic<int> g_cus[64];   // compute units + 1 per device ordinal (0: not yet asked)

}  // namespace

int kx_knob(KxKnob k) {
  load();
  return g_knob[k].load(std::memory_order_relaxed);
}

int kx_device_cus(int dev) {
  if (dev < 0 || dev >= 64) return 0;
  int v = g_cus[dev].load(std::memory_order_relaxed);
  if (!v) {
    int n = 0;
    v = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n + 1 : 1;
    g_cus[dev].store(v, std::memory_order_relaxed);
  }
  return v - 1;
}

// test infrastructure (not in include/kxcodec.h): set a switch by its environment name for this process;
// returns 0, or -1 for an unknown name
extern "C" int kx_debug_set_knob(const char* name, int value) {
  load();
  for (int k = 0; k < KXK_N; k++)
    if (name && !strcmp(name, kDefs[k].env)) {
      g_knob[k].store(value, std::memory_order_relaxed);
      return 0;
    }
  return -1;
}
