// kx_knobs.h — the library's tuning switches and per-device facts, shared by the
// translation units.
//
// Every switch is read from the environment once per process (std::call_once) into an atomic: no launch
// calls getenv (not safe against a setenv on another thread), and the caches are race-free when several
// threads drive different contexts. kx_debug_set_knob (test infrastructure, not in include/kxcodec.h) sets
// one by its environment name, for the tests that run both forms of a switch in one process.
#pragma once

enum KxKnob {
  KXK_CHAIN_FAST,   // KX_CHAIN_FAST (1): the 1024-thread chain fast kernel ahead of the gated general one
  KXK_EMIT_FAST,    // KX_EMIT_FAST (1): the fast emit kernel for T_CANON tiles + the emit redo kernel
  KXK_FAST_NARROW,  // KX_FAST_NARROW (1): the fast kernels in 2-wave workgroups when the window fits
  KXK_FAST_SPLIT,   // KX_FAST_SPLIT (1): the fast index path in its own kernel + the redo kernel
  KXK_REDO_WG,      // KX_REDO_WG (4): workgroups per CU of the resident redo grids
  KXK_FAST,         // KX_FAST (1): canonical-plan fast paths of the index pass
  KXK_FASTPLAN,     // KX_FASTPLAN (1): the segment form of the plan in the fast record walk
  KXK_SLOTCAP,      // KX_SLOTCAP (0 = derived): record-start slots per tile (tests force 64)
  KXK_NOLDS,        // KX_NOLDS (0): diagnostics, every byte from global memory
  KXK_DIAG,         // KX_DIAG (0): diagnostics, timing experiments (output is wrong)
  KXK_CRC_FUSED,    // KX_CRC_FUSED (1): CRC32Check inside the frame scan's emit pass
  KXK_CRC_BLK,      // KX_CRC_BLK (8): CRC32C granules per lane block
  KXK_ENC_DIRECT,   // KX_ENC_DIRECT (0): encoder rounds straight to HBM
  KXK_ENC_WCU,      // KX_ENC_WCU (16): the encoder's payload stream copy unit
  KXK_ENC_CANON,    // KX_ENC_CANON (1): canonical-plan sizes and writer
  KXK_CHUNK_MB,     // KX_CHUNK_MB (0): chunked two-stream decode pipeline
  KXK_CHUNK_AHEAD,  // KX_CHUNK_AHEAD (1)
  KXK_NESTED_LDS,   // KX_NESTED_LDS (1): the nested walker's cursors in LDS (0: in scratch)
  KXK_N
};

int kx_knob(KxKnob k);
// compute units of a device ordinal (cached per device; 0 when the runtime cannot tell)
int kx_device_cus(int dev);
