// kx_internal.h — host-side internals shared by the C-ABI translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <vector>

#include "../../include/kxcodec.h"
#include "kx_program.h"
#include "kx_knobs.h"

// 64-bit min/max (HIP's min()/max() on mixed unsigned long / unsigned long long picks a double overload)
__host__ __device__ __forceinline__ uint64_t kmin64(uint64_t a, uint64_t b) { return a < b ? a : b; }
__host__ __device__ __forceinline__ uint64_t kmax64(uint64_t a, uint64_t b) { return a > b ? a : b; }

struct kx_schema {
  KxProgram prog;                      // host copy of the compiled schema
  kx_column_info info[KX_MAX_COLUMNS];
  uint32_t ncols = 0;
  uint32_t npres = 0;
  std::vector<kx_field_desc> fields;   // owned copy of the IDL
  std::vector<uint32_t> struct_first, struct_n;
  // device copies, one per device, uploaded lazily by a ctx
  std::mutex mu;
  void* dev_prog[64] = {nullptr};
  // nested schemas (kx_nested_schema.cpp): the walker's program, nullptr for flat schemas
  struct KxnProgram* nprog = nullptr;
  void* dev_nprog[64] = {nullptr};
  ~kx_schema();
};

// Chunked decode pipeline (kx_decode.hip launch_t): index + group of chunk k run on `aux` while chain +
// emit of chunk k - 1 run on the caller's stream, so emit re-reads a chunk the index pass has just
// pulled through the Infinity Cache. Events order the two streams (rings of KX_PIPE_EV).
#define KX_PIPE_EV 8
struct KxPipe {
  hipStream_t aux = nullptr;
  hipEvent_t fork = nullptr;
  hipEvent_t ev_idx[KX_PIPE_EV] = {};   // chunk k indexed (aux) -> chain(k) may start
  hipEvent_t ev_emit[KX_PIPE_EV] = {};  // chunk k emitted (caller's stream) -> throttles aux
  uint64_t chunk_tiles = 0;             // tiles per chunk (a multiple of 64), 0 = one chunk
  int ahead = 1;                        // chunks the index pass may run ahead of emit
};

#define KX_HOST_CH 16   // record-range chunks of the kx_host_* pipelines

struct kx_ctx {
  int device = 0;
  KxPipe pipe;                         // created lazily (ensure_pipe)
  hipStream_t own_stream = nullptr;
  hipStream_t h2d_stream = nullptr, d2h_stream = nullptr;  // kx_host_decode_batch copy engines
  // grow-only decode workspace: tile counter, error key, overflow flag, epoch-tagged tile
  // descriptors. Zeroed once at allocation; every call leaves it re-armed (finalize kernel).
  void* ws = nullptr;
  size_t ws_size = 0;
  uint64_t epoch = 0;                  // call epoch tagging descriptor words (1..65535)
  // grow-only message-header workspace (kx_*_decode_messages)
  void* mws = nullptr;
  size_t mws_size = 0;
  // grow-only framing-scan scratch (kx_*_decode_frames): frame offsets, payload extents, scan status
  void* fws = nullptr;
  size_t fws_size = 0;
  // CRC32C: 256 B scratch (error key), armed at allocation; CRC32Check for kx_*_decode_frames
  void* cws = nullptr;
  bool crc32c_check = false;
  // grow-only message-encode scratch: record offsets (n + 1) and the method name
  void* xws = nullptr;
  size_t xws_size = 0;
  // nested schemas: grow-only walker workspace, the per-call column table (device) and its staging
  void* nws = nullptr;
  size_t nws_size = 0;
  void* ncols_dev = nullptr;        // KxnCols
  void* ncols_host = nullptr;       // pinned KxnCols staging
  hipEvent_t ncols_ev = nullptr;    // the last upload from the staging buffer has been consumed
  // grow-only encode scratch (per-block sizes)
  void* ews = nullptr;
  size_t ews_size = 0;
  // pinned staging for kx_host_*
  void* pin = nullptr;
  size_t pin_size = 0;
  // grow-only device staging for kx_host_decode_batch (input, offsets, columns, status)
  void* dstage = nullptr;
  size_t dstage_size = 0;
  // kx_host_* pipelines: per chunk, input landed / kernel done / status copied out; pinned status staging
  hipEvent_t hev_in[KX_HOST_CH] = {}, hev_run[KX_HOST_CH] = {}, hev_st[KX_HOST_CH] = {};
  kx_status* hst = nullptr;
  uint64_t* htot = nullptr;         // per chunk: the running unit totals (nested: cursor totals), pinned
  void* hcols = nullptr;            // per chunk: the nested walker's column table (KxnCols), pinned
};

// kx_schema.cpp / kx_nested_schema.cpp
int kx_build_program(const kx_struct_desc* structs, uint32_t nstructs, kx_schema* s);
int kx_build_nested(const kx_struct_desc* structs, uint32_t nstructs, kx_schema* s);

// kx_nested.hip: the nested walker's launches (decode: sizes only when units != null)
struct KxnCols;
size_t kx_nested_ws_bytes(const struct KxnProgram& P, uint64_t n, bool concat);
int kx_launch_nested_decode(const struct KxnProgram* dprog, const struct KxnProgram& hprog, const uint8_t* in,
                            uint64_t in_len, const uint64_t* offsets, const uint64_t* ends, uint64_t n,
                            const KxnCols* dcols, uint8_t* record_status, kx_status* status, void* ws,
                            size_t ws_size, void* skip_ws, size_t skip_ws_size, uint64_t skip_epoch,
                            hipStream_t stream, uint64_t* totals_out, const uint64_t* cur_base_dev = nullptr,
                            uint64_t* totals_dev = nullptr);
size_t kx_nested_enc_ws_bytes(uint64_t n);
int kx_launch_nested_encode(const struct KxnProgram* dprog, const struct KxnProgram& hprog, const KxnCols* dcols,
                            uint64_t n, uint8_t* out, uint64_t out_cap, uint64_t* sizes_out, uint64_t* offsets_out,
                            kx_status* status, void* ws, size_t ws_size, hipStream_t stream, bool sizes_only,
                            const uint64_t* out_base = nullptr);

// device launchers (kx_decode.hip / kx_encode.hip)
struct KxLaunchCols {            // flat schemas (<= KXP_MAX_COLS columns)
  void* data[KXP_MAX_COLS];
  void* offs[KXP_MAX_COLS];      // record offsets (u32 or u64, see owide)
  uint64_t cap[KXP_MAX_COLS];
  void* eoffs[KXP_MAX_COLS];     // LIST_BYTES: element byte offsets
  uint64_t ecap[KXP_MAX_COLS];
  uint32_t owide;                // bit c: column c has 8-byte offsets
  uint32_t view;                 // bit c: BYTES column c receives (offset, length) views (KX_COLF_VIEW)
  uint64_t* presence;
  uint64_t nrec;                 // records of the call (device-side guard of every column store)
  unsigned long long* guard;     // where a refused out-of-range access is reported (kx_status.diag[2])
};

int kx_launch_decode(const KxProgram* dprog, const KxProgram& hprog, const uint8_t* in,
                     uint64_t in_len, const uint64_t* offsets, uint64_t n,
                     const KxLaunchCols& cols, uint8_t* record_status, kx_status* status,
                     void* ws, size_t ws_size, uint64_t epoch, hipStream_t stream, bool pb,
                     const uint64_t* ends = nullptr, const uint64_t* var_base = nullptr,
                     const KxPipe* pipe = nullptr, const uint64_t* var_base_dev = nullptr);
size_t kx_decode_ws_bytes(const KxProgram& hprog, uint64_t in_len, const uint64_t* offsets, uint64_t n);

int kx_launch_skip(const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t* offsets_out,
                   kx_status* status, void* ws, size_t ws_size, uint64_t epoch, hipStream_t stream);
size_t kx_skip_ws_bytes(uint64_t in_len, uint64_t n);
// split points of n concatenated records for `parts` shards (parts + 1 starts; dprog null: skip walker)
int kx_launch_split(const KxProgram* dprog, const KxProgram* hprog, const uint8_t* in, uint64_t in_len, uint64_t n,
                    uint32_t parts, uint64_t* points, kx_status* status, void* ws, size_t ws_size, uint64_t epoch,
                    hipStream_t stream);
// Kitex-PB Batch frames (0x0A, uvarint length, body): frame starts (n + 1) and body extents
int kx_launch_pb_frames(const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t* frame_offsets, uint64_t* body_start,
                        uint64_t* body_end, kx_status* status, void* ws, size_t ws_size, uint64_t epoch,
                        hipStream_t stream);
int kx_launch_frames(const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t max_payload, uint64_t* frame_offsets,
                     uint64_t* pay_start, uint64_t* pay_end, uint8_t* kinds, kx_status* status, void* ws,
                     size_t ws_size, uint64_t epoch, hipStream_t stream, bool grpc = false,
                     const kx_ttstream_keys* tts = nullptr, int32_t* sids = nullptr, uint64_t* mpos = nullptr,
                     uint32_t* mlen = nullptr, uint8_t* crc_codes = nullptr);

int kx_launch_encode(const KxProgram* dprog, const KxProgram& hprog, const KxLaunchCols& cols,
                     uint64_t n, uint8_t* out, uint64_t out_cap, uint64_t* sizes_out,
                     uint64_t* offsets_out, kx_status* status, void* ws, size_t ws_size,
                     hipStream_t stream, bool sizes_only, bool pb = false, const uint64_t* out_base = nullptr);
size_t kx_encode_ws_bytes(uint64_t n);

// kx_message.hip: MessageBegin + Args{1: Req} headers of n framed messages (lane = message)
struct KxMsgOut {
  int32_t* msg_type;            // per message (may be null)
  int32_t* seqid;               // per message (may be null)
  void* name_offs;              // method names: offsets (4 or 8 bytes, name_owide) + arena
  uint8_t* name_data;
  uint64_t name_cap;
  uint32_t name_owide;
};
size_t kx_message_ws_bytes(uint64_t n);
int kx_launch_message_headers(const uint8_t* in, uint64_t in_len, const uint64_t* offsets, uint64_t n,
                              int32_t body_field, bool pb, const KxMsgOut& mo, void* mws,
                              uint64_t** req_start, uint64_t** req_end,
                              uint8_t** hdr_rc, uint8_t** body_rc, hipStream_t stream,
                              const uint64_t* ends = nullptr, const kx_status* pre = nullptr,
                              const uint8_t* pre_rc = nullptr, const uint8_t* raw_flags = nullptr,
                              int raw = 0);
int kx_launch_set_seqids(uint8_t* in, uint64_t in_len, const uint64_t* offsets, uint64_t n, const int32_t* seqids,
                         uint8_t* record_status, kx_status* status, void* mws, hipStream_t stream);
int kx_launch_message_encode(const uint8_t* bodies, const uint64_t* body_off, uint64_t scratch_cap, uint64_t n,
                             const uint8_t* name,
                             uint32_t name_len, int32_t msg_type, const int32_t* seqids, int32_t body_field,
                             uint8_t* out, uint64_t out_cap, uint64_t* offsets_out, kx_status* status,
                             hipStream_t stream);
int kx_launch_message_merge(const uint64_t* offsets, uint64_t n, const uint8_t* hdr_rc, const uint8_t* body_rc,
                            uint8_t* record_status, kx_status* status, void* mws, hipStream_t stream,
                            const kx_status* pre = nullptr);

// kx_crc.hip: CRC-32C of n ranges (val = false: [offs[i], offs[i+1])) or of n TTHeader frames' payloads
// checked against their "crc32c" header (val = true); scratch = 8-byte error key armed to ~0
int kx_launch_crc32c(const uint8_t* in, uint64_t in_len, const uint64_t* offs, uint64_t n, bool val,
                     const kx_status* pre, uint32_t* crc_out, uint8_t* rs, kx_status* status, void* scratch,
                     hipStream_t stream);

#define KX_HIP_CHECK(x)                       \
  do {                                        \
    hipError_t e_ = (x);                      \
    if (e_ != hipSuccess) return KX_ERR_HIP;  \
  } while (0)
