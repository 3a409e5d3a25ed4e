// Test infrastructure only: C entry point that runs the decode kernel source under the SIMT
// emulator with host buffers (see tests/test_emu_decode.py).
#include "hip/hip_runtime.h"
#include "kx_internal.h"

// mode: 0 = Thrift decode, 1 = skip decoder, 2 = Kitex-Protobuf decode
extern "C" int emu_decode(const kx_struct_desc* structs, uint32_t nstructs, const uint8_t* in, uint64_t in_len,
                          const uint64_t* offsets, uint64_t n, const kx_columns* out, uint8_t* record_status,
                          kx_status* status, int mode, uint64_t* skip_out) {
  static kx_schema s;  // the emulator is single-call-at-a-time
  const bool skip = mode == 1;
  int rc = skip ? KX_OK : kx_build_program(structs, nstructs, &s);
  if (rc) return rc;
  KxLaunchCols lc;
  memset(&lc, 0, sizeof lc);
  if (!skip) {
    for (uint32_t c = 0; c < s.ncols; c++) {
      lc.data[c] = out->cols[c].data;
      lc.offs[c] = out->cols[c].offsets;
      lc.cap[c] = out->cols[c].capacity;
      lc.eoffs[c] = out->cols[c].elem_offsets;
      lc.ecap[c] = out->cols[c].elem_capacity;
      if (out->cols[c].offset_bytes == 8) lc.owide |= 1u << c;
      if (out->cols[c].flags & KX_COLF_VIEW) lc.view |= 1u << c;
    }
    lc.presence = out->presence;
  }
  size_t ws_size = skip ? kx_skip_ws_bytes(in_len, n) : kx_decode_ws_bytes(s.prog, in_len, offsets, n);
  // one workspace reused across calls with a fresh epoch each time, exactly like a kx_ctx
  // (kx_capi.cpp ensure_ws): stale words / counters of earlier calls must never leak into a call
  static char* ws = nullptr;
  static size_t ws_cap = 0;
  static uint64_t epoch = 0xffff;
  if (ws_cap < ws_size) {
    free(ws);
    ws_cap = ws_size + ws_size / 4;
    ws = (char*)malloc(ws_cap);
    epoch = 0xffff;
  }
  if (++epoch > 0xffff) {
    memset(ws, 0, ws_cap);
    memset(ws + 8, 0xff, 8);
    epoch = 1;
  }
  status->diag[0] = status->diag[1] = status->diag[2] = 0;
  if (skip)
    rc = kx_launch_skip(in, in_len, n, skip_out, status, ws, ws_cap, epoch, nullptr);
  else
  {
    // KX_EMU_CHUNK = tiles per chunk (a multiple of 64): the chunked two-stream pipeline of launch_t
    static KxPipe pipe;
    const char* e = getenv("KX_EMU_CHUNK");
    pipe.chunk_tiles = e ? strtoull(e, nullptr, 10) : 0;
    const char* a = getenv("KX_EMU_AHEAD");
    pipe.ahead = a ? atoi(a) : 1;
    pipe.aux = (hipStream_t)&pipe;  // any non-null handle
    rc = kx_launch_decode(&s.prog, s.prog, in, in_len, offsets, n, lc, record_status, status, ws, ws_cap, epoch,
                          nullptr, mode == 2, nullptr, nullptr, &pipe);
  }
  return rc;
}

// split points (kx_launch_split) under the emulator: skip = 1 uses the schema-free skip walker
extern "C" int emu_split(const kx_struct_desc* structs, uint32_t nstructs, const uint8_t* in, uint64_t in_len,
                         uint64_t n, uint32_t parts, uint64_t* points, kx_status* status, int skip) {
  static kx_schema s;
  int rc = skip ? KX_OK : kx_build_program(structs, nstructs, &s);
  if (rc) return rc;
  const size_t ws_size = kx_skip_ws_bytes(in_len, n);
  static char* ws = nullptr;
  static size_t ws_cap = 0;
  static uint64_t epoch = 0xffff;
  if (ws_cap < ws_size) {
    free(ws);
    ws_cap = ws_size + ws_size / 4;
    ws = (char*)malloc(ws_cap);
    epoch = 0xffff;
  }
  if (++epoch > 0xffff) {
    memset(ws, 0, ws_cap);
    memset(ws + 8, 0xff, 8);
    epoch = 1;
  }
  memset(status, 0, sizeof *status);
  return kx_launch_split(skip ? nullptr : &s.prog, skip ? nullptr : &s.prog, in, in_len, n, parts, points, status, ws,
                         ws_cap, epoch, nullptr);
}

// framing sniff (kx_launch_frames) under the emulator, workspace shared with emu_decode's
extern "C" int emu_frames(const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t max_payload, uint64_t* fo,
                          uint64_t* ps, uint64_t* pe, uint8_t* kinds, kx_status* status, int grpc, uint8_t* crc_codes) {
  const size_t ws_size = kx_skip_ws_bytes(in_len, n);
  static char* ws = nullptr;
  static size_t ws_cap = 0;
  static uint64_t epoch = 0xffff;
  if (ws_cap < ws_size) {
    free(ws);
    ws_cap = ws_size + ws_size / 4;
    ws = (char*)malloc(ws_cap);
    epoch = 0xffff;
  }
  if (++epoch > 0xffff) {
    memset(ws, 0, ws_cap);
    memset(ws + 8, 0xff, 8);
    epoch = 1;
  }
  status->diag[0] = status->diag[1] = 0;
  return kx_launch_frames(in, in_len, n, max_payload, fo, ps, pe, kinds, status, ws, ws_cap, epoch, nullptr, grpc != 0,
                          nullptr, nullptr, nullptr, nullptr, crc_codes);
}

// Kitex-PB Batch frames (kx_launch_pb_frames: the nested proto path's record delimiter) under the emulator
extern "C" int emu_pb_frames(const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t* fo, uint64_t* bs, uint64_t* be,
                             kx_status* status) {
  const size_t ws_size = kx_skip_ws_bytes(in_len, n);
  static char* ws = nullptr;
  static size_t ws_cap = 0;
  static uint64_t epoch = 0xffff;
  if (ws_cap < ws_size) {
    free(ws);
    ws_cap = ws_size + ws_size / 4;
    ws = (char*)malloc(ws_cap);
    epoch = 0xffff;
  }
  if (++epoch > 0xffff) {
    memset(ws, 0, ws_cap);
    memset(ws + 8, 0xff, 8);
    epoch = 1;
  }
  status->diag[0] = status->diag[1] = status->diag[2] = 0;
  return kx_launch_pb_frames(in, in_len, n, fo, bs, be, status, ws, ws_cap, epoch, nullptr);
}

// ttstream frame scan (kx_launch_frames with keys) under the emulator
extern "C" int emu_tts_frames(const uint8_t* in, uint64_t in_len, uint64_t n, const kx_ttstream_keys* keys,
                              uint64_t* fo, uint64_t* ps, uint64_t* pe, uint8_t* ft, int32_t* sid, uint64_t* mp,
                              uint32_t* ml, kx_status* status) {
  const size_t ws_size = kx_skip_ws_bytes(in_len, n);
  static char* ws = nullptr;
  static size_t ws_cap = 0;
  static uint64_t epoch = 0xffff;
  if (ws_cap < ws_size) {
    free(ws);
    ws_cap = ws_size + ws_size / 4;
    ws = (char*)malloc(ws_cap);
    epoch = 0xffff;
  }
  if (++epoch > 0xffff) {
    memset(ws, 0, ws_cap);
    memset(ws + 8, 0xff, 8);
    epoch = 1;
  }
  status->diag[0] = status->diag[1] = 0;
  return kx_launch_frames(in, in_len, n, 0, fo, ps, pe, ft, status, ws, ws_cap, epoch, nullptr, false, keys, sid, mp,
                          ml);
}

// CRC32C kernel source (kx_crc.hip): val = 0 ranges [offs[i], offs[i+1]), 1 TTHeader frames at offs[i]
extern "C" int emu_crc(const uint8_t* in, uint64_t in_len, const uint64_t* offs, uint64_t n, int val,
                       uint32_t* crc_out, uint8_t* rs, kx_status* status) {
  static unsigned long long errkey = ~0ull;
  return kx_launch_crc32c(in, in_len, offs, n, val != 0, nullptr, crc_out, rs, status, &errkey, nullptr);
}
