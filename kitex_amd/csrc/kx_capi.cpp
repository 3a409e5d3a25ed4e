// kx_capi.cpp — the C-ABI of libkxcodec.so (include/kxcodec.h).
//
// Thin, allocation-light host layer: argument checks, per-device upload of the compiled schema,
// a grow-only workspace per context, and kernel launches on the caller's stream. No torch types,
// no exceptions cross the boundary.
#include <stdlib.h>
#include <string.h>

#include <new>

#include "kx_internal.h"
#include "kx_nested.h"

namespace {

int prog_on_device(kx_schema* s, int dev, KxProgram** out) {
  if (dev < 0 || dev >= 64) return KX_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(s->mu);
  if (!s->dev_prog[dev]) {
    void* p = nullptr;
    KX_HIP_CHECK(hipMalloc(&p, sizeof(KxProgram)));
    if (hipMemcpy(p, &s->prog, sizeof(KxProgram), hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipFree(p);
      return KX_ERR_HIP;
    }
    s->dev_prog[dev] = p;
  }
  *out = (KxProgram*)s->dev_prog[dev];
  return KX_OK;
}

// Decode workspace: grown on demand, zeroed at allocation (tile counter 0, overflow 0, no
// descriptor word carries a live epoch) with the error key at ~0. Returns the epoch for this call.
int ensure_ws(kx_ctx* c, size_t bytes, hipStream_t stream, uint64_t* epoch) {
  if (c->ws_size < bytes) {
    if (c->ws) {
      KX_HIP_CHECK(hipStreamSynchronize(stream));  // the old workspace may still be in use
      if (c->pipe.aux) KX_HIP_CHECK(hipStreamSynchronize(c->pipe.aux));
      KX_HIP_CHECK(hipFree(c->ws));
      c->ws = nullptr;
      c->ws_size = 0;
    }
    size_t sz = bytes < (1u << 20) ? (1u << 20) : bytes + bytes / 4;
    KX_HIP_CHECK(hipMalloc(&c->ws, sz));
    c->ws_size = sz;
    c->epoch = 0xffff;  // forces the re-initialisation below
  }
  if (++c->epoch > 0xffff) {
    // first use or epoch wrap: clear every descriptor word so no stale tag can match
    KX_HIP_CHECK(hipMemsetAsync(c->ws, 0, c->ws_size, stream));
    KX_HIP_CHECK(hipMemsetAsync((char*)c->ws + 8, 0xff, 8, stream));
    c->epoch = 1;
  }
  *epoch = c->epoch;
  return KX_OK;
}

// The chunked decode pipeline's second stream and events (KxPipe). Chunk size: KX_CHUNK_MB MiB of
// 8 KiB tiles (0 = one chunk; measured slower at every size), KX_CHUNK_AHEAD chunks of
// index-pass lead.
static int ensure_pipe(kx_ctx* c) {
  KxPipe& p = c->pipe;
  if (p.aux) return KX_OK;
  const uint64_t mb = (uint64_t)kx_knob(KXK_CHUNK_MB);
  p.ahead = kx_knob(KXK_CHUNK_AHEAD);
  p.chunk_tiles = (mb * 128 + 63) & ~63ull;  // 128 tiles of 8 KiB per MiB, whole groups of 64 tiles
  KX_HIP_CHECK(hipEventCreateWithFlags(&p.fork, hipEventDisableTiming));
  for (int k = 0; k < KX_PIPE_EV; k++) {
    KX_HIP_CHECK(hipEventCreateWithFlags(&p.ev_idx[k], hipEventDisableTiming));
    KX_HIP_CHECK(hipEventCreateWithFlags(&p.ev_emit[k], hipEventDisableTiming));
  }
  KX_HIP_CHECK(hipStreamCreateWithFlags(&p.aux, hipStreamNonBlocking));
  return KX_OK;
}

int ensure_ews(kx_ctx* c, size_t bytes, hipStream_t stream) {
  if (c->ews_size >= bytes) return KX_OK;
  if (c->ews) {
    KX_HIP_CHECK(hipStreamSynchronize(stream));
    KX_HIP_CHECK(hipFree(c->ews));
    c->ews = nullptr;
    c->ews_size = 0;
  }
  size_t sz = bytes < (1u << 20) ? (1u << 20) : bytes + bytes / 4;
  KX_HIP_CHECK(hipMalloc(&c->ews, sz));
  c->ews_size = sz;
  return KX_OK;
}

int ensure_mws(kx_ctx* c, size_t bytes, hipStream_t stream) {
  if (c->mws_size >= bytes) return KX_OK;
  if (c->mws) {
    KX_HIP_CHECK(hipStreamSynchronize(stream));
    KX_HIP_CHECK(hipFree(c->mws));
    c->mws = nullptr;
    c->mws_size = 0;
  }
  size_t sz = bytes < (1u << 20) ? (1u << 20) : bytes + bytes / 4;
  KX_HIP_CHECK(hipMalloc(&c->mws, sz));
  c->mws_size = sz;
  KX_HIP_CHECK(hipMemsetAsync(c->mws, 0, 256, stream));
  KX_HIP_CHECK(hipMemsetAsync(c->mws, 0xff, 8, stream));  // error key: none
  return KX_OK;
}

int offset_width(const kx_column& k) {
  return k.offset_bytes == 0 || k.offset_bytes == 4 ? 4 : k.offset_bytes == 8 ? 8 : 0;
}

// allow_view: decode calls whose input stays in HBM (KX_COLF_VIEW on BYTES columns); in_len then
// bounds 4-byte views
int to_launch_cols(const kx_schema* s, const kx_columns* out, KxLaunchCols* lc, bool allow_view = false,
                   uint64_t in_len = 0) {
  if (!out) return KX_ERR_INVALID_ARG;
  if (s->nprog) return KX_ERR_NOT_IMPLEMENTED;  // nested schemas: the entry points of nested_* below
  if (out->ncols != s->ncols || s->ncols > KXP_MAX_COLS) return KX_ERR_INVALID_ARG;
  if (s->npres && !out->presence) return KX_ERR_INVALID_ARG;
  memset(lc, 0, sizeof *lc);
  for (uint32_t c = 0; c < s->ncols; c++) {
    const kx_column& k = out->cols[c];
    const uint32_t kind = s->info[c].kind;
    if (k.flags & ~KX_COLF_VIEW) return KX_ERR_INVALID_ARG;
    if (k.flags & KX_COLF_VIEW) {
      if (!allow_view || kind != KX_COL_BYTES || !k.offsets) return KX_ERR_INVALID_ARG;
      const int ow = offset_width(k);
      if (!ow) return KX_ERR_INVALID_ARG;
      if (ow == 4 && in_len > 0xffffffffull) return KX_ERR_SIZE_LIMIT;
      if (ow == 8) lc->owide |= 1u << c;
      lc->view |= 1u << c;
      lc->offs[c] = k.offsets;
      continue;
    }
    if (kind == KX_COL_FIXED) {
      if (!k.data) return KX_ERR_INVALID_ARG;
    } else {
      const int ow = offset_width(k);
      if (!ow || !k.offsets) return KX_ERR_INVALID_ARG;
      if (!k.data && k.capacity) return KX_ERR_INVALID_ARG;
      if (kind == KX_COL_LIST_BYTES && (!k.elem_offsets || (!k.data && k.capacity))) return KX_ERR_INVALID_ARG;
      if (ow == 8) lc->owide |= 1u << c;
    }
    lc->data[c] = k.data;
    lc->offs[c] = k.offsets;
    lc->cap[c] = k.capacity;
    lc->eoffs[c] = k.elem_offsets;
    lc->ecap[c] = k.elem_capacity;
  }
  lc->presence = out->presence;
  return KX_OK;
}

int set_device(kx_ctx* c) {
  KX_HIP_CHECK(hipSetDevice(c->device));
  return KX_OK;
}

// ---- nested schemas ----
int nprog_on_device(kx_schema* s, int dev, KxnProgram** out) {
  if (dev < 0 || dev >= 64) return KX_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> g(s->mu);
  if (!s->dev_nprog[dev]) {
    void* p = nullptr;
    KX_HIP_CHECK(hipMalloc(&p, sizeof(KxnProgram)));
    if (hipMemcpy(p, s->nprog, sizeof(KxnProgram), hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipFree(p);
      return KX_ERR_HIP;
    }
    s->dev_nprog[dev] = p;
  }
  *out = (KxnProgram*)s->dev_nprog[dev];
  return KX_OK;
}

int ensure_nws(kx_ctx* c, size_t bytes, hipStream_t stream) {
  if (c->nws_size >= bytes) return KX_OK;
  if (c->nws) {
    KX_HIP_CHECK(hipStreamSynchronize(stream));
    KX_HIP_CHECK(hipFree(c->nws));
    c->nws = nullptr;
    c->nws_size = 0;
  }
  size_t sz = bytes < (1u << 20) ? (1u << 20) : bytes + bytes / 4;
  KX_HIP_CHECK(hipMalloc(&c->nws, sz));
  c->nws_size = sz;
  return KX_OK;
}

// the call's column table (checked on the host) in the walker's form
int fill_ncols(const kx_schema* s, const kx_columns* cols, bool decode, KxnCols& K) {
  if (!cols || cols->ncols != s->ncols) return KX_ERR_INVALID_ARG;
  if (s->npres && !cols->presence) return KX_ERR_INVALID_ARG;
  memset(&K, 0, sizeof K);
  const KxnProgram& P = *s->nprog;
  for (uint32_t i = 0; i < s->ncols; i++) {
    const kx_column& k = cols->cols[i];
    const KxnCol& C = P.col[i];
    if (k.flags) return KX_ERR_INVALID_ARG;  // no zero-copy views on nested schemas
    if (C.kind == KX_COL_FIXED) {
      if (!k.data) return KX_ERR_INVALID_ARG;
    } else {
      const int ow = offset_width(k);
      if (!ow) return KX_ERR_INVALID_ARG;
      if (ow == 8) K.owide |= 1ull << i;
      void* arrs[3] = {k.offsets, k.elem_offsets, k.sub_offsets};
      for (int a = 0; a < C.narr; a++)
        if (!arrs[a]) return KX_ERR_INVALID_ARG;
      if (!k.data && k.capacity) return KX_ERR_INVALID_ARG;
      for (int a = 0; a < 3; a++) K.arr[i][a] = arrs[a];
      K.cap[i][0] = k.capacity;
      K.cap[i][2] = k.elem_capacity;
      K.cap[i][3] = k.sub_capacity;
      if (ow == 4 && decode) {  // 4-byte offsets never wrap: capacities beyond them are refused
        for (int a = 0; a < 4; a++)
          if (K.cap[i][a] > 0xffffffffull) K.cap[i][a] = 0xffffffffull;
      }
    }
    K.data[i] = k.data;
  }
  K.presence = cols->presence;
  return KX_OK;
}

// the call's column table: checked on the host, staged in pinned memory, copied on the stream (the
// staging buffer is reused once the previous copy has executed)
int nested_cols(kx_ctx* c, const kx_schema* s, const kx_columns* cols, bool decode, hipStream_t st, KxnCols** out) {
  if (!cols || cols->ncols != s->ncols) return KX_ERR_INVALID_ARG;
  if (!c->ncols_dev) {
    KX_HIP_CHECK(hipMalloc(&c->ncols_dev, sizeof(KxnCols)));
    KX_HIP_CHECK(hipHostMalloc(&c->ncols_host, sizeof(KxnCols), hipHostMallocDefault));
    KX_HIP_CHECK(hipEventCreateWithFlags(&c->ncols_ev, hipEventDisableTiming));
  } else {
    KX_HIP_CHECK(hipEventSynchronize(c->ncols_ev));
  }
  KxnCols& K = *(KxnCols*)c->ncols_host;
  int rc = fill_ncols(s, cols, decode, K);
  if (rc) return rc;
  KX_HIP_CHECK(hipMemcpyAsync(c->ncols_dev, &K, sizeof K, hipMemcpyHostToDevice, st));
  KX_HIP_CHECK(hipEventRecord(c->ncols_ev, st));
  *out = (KxnCols*)c->ncols_dev;
  return KX_OK;
}

// decode of a nested schema (offsets / ends as kx_launch_decode; offsets == NULL: concatenated).
// totals: sizes only (host, ncur entries; synchronous). dcols_in: a column table already on the device
// (the host pipelines upload one per chunk); cur_base / totals_dev: a record-range chunk continues the
// arenas of the previous one (device, ncur entries each)
int nested_decode(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len, const uint64_t* offsets,
                  const uint64_t* ends, uint64_t n, const kx_columns* out, uint8_t* record_status, kx_status* status,
                  hipStream_t st, uint64_t* totals, const KxnCols* dcols_in = nullptr,
                  const uint64_t* cur_base = nullptr, uint64_t* totals_dev = nullptr) {
  int rc;
  KxnCols* dcols = nullptr;
  if (n == 0) {  // no record: empty offsets arrays (a single 0 entry each)
    KX_HIP_CHECK(hipMemsetAsync(status, 0, sizeof(kx_status), st));
    if (totals || !out) return totals ? KX_OK : KX_ERR_INVALID_ARG;
    if (out->ncols != s->ncols) return KX_ERR_INVALID_ARG;
    for (uint32_t i = 0; i < s->ncols; i++) {
      const kx_column& k = out->cols[i];
      void* arrs[3] = {k.offsets, k.elem_offsets, k.sub_offsets};
      for (int a = 0; a < s->nprog->col[i].narr; a++) {
        if (!arrs[a]) return KX_ERR_INVALID_ARG;
        KX_HIP_CHECK(hipMemsetAsync(arrs[a], 0, offset_width(k) == 8 ? 8 : 4, st));
      }
    }
    return KX_OK;
  }
  if (totals) {
    if (!c->ncols_dev) {  // the sizes pass reads no column: an empty table
      KX_HIP_CHECK(hipMalloc(&c->ncols_dev, sizeof(KxnCols)));
      KX_HIP_CHECK(hipHostMalloc(&c->ncols_host, sizeof(KxnCols), hipHostMallocDefault));
      KX_HIP_CHECK(hipEventCreateWithFlags(&c->ncols_ev, hipEventDisableTiming));
      KX_HIP_CHECK(hipMemsetAsync(c->ncols_dev, 0, sizeof(KxnCols), st));
    }
    dcols = (KxnCols*)c->ncols_dev;
  } else if (dcols_in) {
    dcols = const_cast<KxnCols*>(dcols_in);
  } else if ((rc = nested_cols(c, s, out, true, st, &dcols))) {
    return rc;
  }
  KxnProgram* dp = nullptr;
  if ((rc = nprog_on_device(const_cast<kx_schema*>(s), c->device, &dp))) return rc;
  if ((rc = ensure_nws(c, kx_nested_ws_bytes(*s->nprog, n, offsets == nullptr), st))) return rc;
  uint64_t epoch = 0;
  if (!offsets && (rc = ensure_ws(c, kx_skip_ws_bytes(in_len, n), st, &epoch))) return rc;
  return kx_launch_nested_decode(dp, *s->nprog, in, in_len, offsets, ends, n, dcols, record_status, status, c->nws,
                                 c->nws_size, c->ws, c->ws_size, epoch, st, totals, cur_base, totals_dev);
}

int nested_encode(kx_ctx* c, const kx_schema* s, const kx_columns* in, uint64_t n, uint8_t* out, uint64_t out_cap,
                  uint64_t* sizes_out, uint64_t* offsets_out, kx_status* status, hipStream_t st, bool sizes_only,
                  const KxnCols* dcols_in = nullptr, const uint64_t* out_base = nullptr) {
  int rc;
  KxnCols* dcols = const_cast<KxnCols*>(dcols_in);
  if (!dcols && (rc = nested_cols(c, s, in, false, st, &dcols))) return rc;
  if (n == 0) return KX_OK;
  KxnProgram* dp = nullptr;
  if ((rc = nprog_on_device(const_cast<kx_schema*>(s), c->device, &dp))) return rc;
  if ((rc = ensure_ews(c, kx_nested_enc_ws_bytes(n), st))) return rc;
  return kx_launch_nested_encode(dp, *s->nprog, dcols, n, out, out_cap, sizes_out, offsets_out, status, c->ews,
                                 c->ews_size, st, sizes_only, out_base);
}

}  // namespace

extern "C" {

int kx_abi_version(void) { return KX_ABI_VERSION; }

const char* kx_strerror(int code) {
  switch (code) {
    case KX_OK: return "ok";
    case KX_ERR_INVALID_DATA: return "invalid data";
    case KX_ERR_NEGATIVE_SIZE: return "negative size";
    case KX_ERR_SIZE_LIMIT: return "size limit";
    case KX_ERR_BAD_VERSION: return "bad version";
    case KX_ERR_NOT_IMPLEMENTED: return "not implemented";
    case KX_ERR_DEPTH_LIMIT: return "depth limit exceeded";
    case KX_ERR_EOF: return "unexpected EOF";
    case KX_ERR_APPLICATION_EXCEPTION: return "application exception message";
    case KX_ERR_UNKNOWN_PROTOCOL: return "unknown protocol (framing sniff)";
    case KX_ERR_PAYLOAD_VALIDATION: return "payload validation failed (crc32c)";
    case KX_ERR_INVALID_ARG: return "invalid argument";
    case KX_ERR_HIP: return "HIP runtime error";
    case KX_ERR_NO_DEVICE: return "no device";
    case KX_ERR_INTERNAL: return "internal error";
    default: return "unknown error";
  }
}

// A Kitex-Protobuf schema stays on the flat program only as a flat proto3 message the tile pipeline's
// proto walker reads: scalars of the natural kinds (int32 / int64 varint, bool, double) and strings /
// bytes. Everything else (other kinds, messages, repeated, maps) goes to the nested walker.
static bool pb_flat_ok(const kx_struct_desc* structs, uint32_t nstructs) {
  if (!structs || nstructs != 1 || (structs[0].nfields && !structs[0].fields)) return false;
  uint32_t nstr = 0;
  for (uint32_t i = 0; i < structs[0].nfields; i++) {
    const kx_field_desc& f = structs[0].fields[i];
    const bool ok_t = f.ttype == KX_T_BOOL || f.ttype == KX_T_I32 || f.ttype == KX_T_I64 ||
                      f.ttype == KX_T_DOUBLE || f.ttype == KX_T_STRING;
    if (!ok_t || (f.default_bits & 0xffff) != 0 || f.req == KX_REQ_REQUIRED) return false;
    nstr += f.ttype == KX_T_STRING;
  }
  return nstr <= 8;   // the flat proto walker's instantiations stop at 8 var slots (kx_decode.hip launch_nv)
}

int kx_schema_create(const kx_struct_desc* structs, uint32_t nstructs, kx_schema** out) {
  if (!out) return KX_ERR_INVALID_ARG;
  *out = nullptr;
  kx_schema* s = new (std::nothrow) kx_schema();
  if (!s) return KX_ERR_INTERNAL;
  const bool pb = structs && nstructs && (structs[0].reserved0 & KX_STRUCT_PROTOBUF);
  int rc = pb && !pb_flat_ok(structs, nstructs) ? KX_ERR_NOT_IMPLEMENTED : kx_build_program(structs, nstructs, s);
  if (rc == KX_ERR_NOT_IMPLEMENTED) rc = kx_build_nested(structs, nstructs, s);
  if (rc) {
    delete s;
    return rc;
  }
  if (!s->nprog) s->prog.is_pb = pb ? 1u : 0u;   // the flat program remembers its wire format (split points)
  *out = s;
  return KX_OK;
}

int kx_schema_is_nested(const kx_schema* s) { return s && s->nprog ? 1 : 0; }

void kx_schema_destroy(kx_schema* s) {
  if (!s) return;
  for (int d = 0; d < 64; d++)
    if (s->dev_prog[d] || s->dev_nprog[d]) {
      (void)hipSetDevice(d);
      if (s->dev_prog[d]) (void)hipFree(s->dev_prog[d]);
      if (s->dev_nprog[d]) (void)hipFree(s->dev_nprog[d]);
    }
  delete s;
}

uint32_t kx_schema_num_columns(const kx_schema* s) { return s ? s->ncols : 0; }

int kx_schema_column_info(const kx_schema* s, uint32_t col, kx_column_info* out) {
  if (!s || !out || col >= s->ncols) return KX_ERR_INVALID_ARG;
  *out = s->info[col];
  return KX_OK;
}

uint32_t kx_schema_presence_bits(const kx_schema* s) { return s ? s->npres : 0; }

uint64_t kx_schema_min_record_size(const kx_schema* s) { return s && !s->nprog ? s->prog.fixed_min : s ? 1 : 0; }

// diagnostics (not part of the public ABI): the decode workspace of a ctx and its current epoch
int kx_debug_workspace(kx_ctx* c, void** ptr, size_t* size, uint64_t* epoch) {
  if (!c || !ptr || !size || !epoch) return KX_ERR_INVALID_ARG;
  *ptr = c->ws;
  *size = c->ws_size;
  *epoch = c->epoch;
  return KX_OK;
}

int kx_ctx_create(int device, kx_ctx** out) {
  if (!out) return KX_ERR_INVALID_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return KX_ERR_NO_DEVICE;
  if (device < 0 || device >= n) return KX_ERR_INVALID_ARG;
  kx_ctx* c = new (std::nothrow) kx_ctx();
  if (!c) return KX_ERR_INTERNAL;
  c->device = device;
  *out = c;
  return KX_OK;
}

void kx_ctx_destroy(kx_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->ws) (void)hipFree(c->ws);
  if (c->ews) (void)hipFree(c->ews);
  if (c->mws) (void)hipFree(c->mws);
  if (c->fws) (void)hipFree(c->fws);
  if (c->cws) (void)hipFree(c->cws);
  if (c->pin) (void)hipHostFree(c->pin);
  if (c->dstage) (void)hipFree(c->dstage);
  if (c->nws) (void)hipFree(c->nws);
  if (c->ncols_dev) (void)hipFree(c->ncols_dev);
  if (c->ncols_host) (void)hipHostFree(c->ncols_host);
  if (c->ncols_ev) (void)hipEventDestroy(c->ncols_ev);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  if (c->pipe.aux) {
    (void)hipStreamSynchronize(c->pipe.aux);
    (void)hipStreamDestroy(c->pipe.aux);
    (void)hipEventDestroy(c->pipe.fork);
    for (int k = 0; k < KX_PIPE_EV; k++) {
      (void)hipEventDestroy(c->pipe.ev_idx[k]);
      (void)hipEventDestroy(c->pipe.ev_emit[k]);
    }
  }
  if (c->h2d_stream) (void)hipStreamDestroy(c->h2d_stream);
  if (c->d2h_stream) (void)hipStreamDestroy(c->d2h_stream);
  for (int k = 0; k < KX_HOST_CH; k++) {
    if (c->hev_in[k]) (void)hipEventDestroy(c->hev_in[k]);
    if (c->hev_run[k]) (void)hipEventDestroy(c->hev_run[k]);
    if (c->hev_st[k]) (void)hipEventDestroy(c->hev_st[k]);
  }
  if (c->hst) (void)hipHostFree(c->hst);
  if (c->htot) (void)hipHostFree(c->htot);
  if (c->hcols) (void)hipHostFree(c->hcols);
  delete c;
}

int kx_ctx_set_pipeline(kx_ctx* c, uint64_t chunk_bytes, int ahead) {
  if (!c || ahead < 0 || ahead > KX_PIPE_EV - 2) return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  if ((rc = ensure_pipe(c))) return rc;
  const uint64_t tiles = (chunk_bytes + 8191) / 8192;
  c->pipe.chunk_tiles = (tiles + 63) & ~63ull;
  c->pipe.ahead = ahead;
  return KX_OK;
}

int kx_thrift_decode_batch(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                           const uint64_t* offsets, uint64_t n, const kx_columns* out,
                           uint8_t* record_status, kx_status* status, void* stream) {
  if (!c || !s || !status || (!in && in_len)) return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (s->nprog) {
    if (s->nprog->pb) return KX_ERR_NOT_IMPLEMENTED;   // a Kitex-Protobuf schema: kx_pb_decode_batch
    return nested_decode(c, s, in, in_len, offsets, nullptr, n, out, record_status, status, st, nullptr);
  }
  KxLaunchCols lc;
  if ((rc = to_launch_cols(s, out, &lc, true, in_len))) return rc;
  if (n == 0) {
    KX_HIP_CHECK(hipMemsetAsync(status, 0, sizeof(kx_status), st));
    for (uint32_t k = 0; k < s->ncols; k++)
      if (lc.offs[k] && !((lc.view >> k) & 1))
        KX_HIP_CHECK(hipMemsetAsync(lc.offs[k], 0, ((lc.owide >> k) & 1) ? 8 : 4, st));
    return KX_OK;
  }
  KxProgram* dp = nullptr;
  if ((rc = prog_on_device(const_cast<kx_schema*>(s), c->device, &dp))) return rc;
  size_t ws = kx_decode_ws_bytes(s->prog, in_len, offsets, n);
  uint64_t epoch = 0;
  if ((rc = ensure_ws(c, ws, st, &epoch))) return rc;
  if ((rc = ensure_pipe(c))) return rc;
  return kx_launch_decode(dp, s->prog, in, in_len, offsets, n, lc, record_status, status, c->ws, c->ws_size,
                          epoch, st, false, nullptr, nullptr, &c->pipe);
}

uint64_t kx_decode_workspace_bytes(const kx_schema* s, uint64_t in_len, int known_offsets, uint64_t n) {
  if (!s) return 0;
  const uint64_t* offs = known_offsets ? (const uint64_t*)(uintptr_t)1 : nullptr;  // only its presence is read
  if (s->nprog) return kx_nested_ws_bytes(*s->nprog, n, !known_offsets) + (known_offsets ? 0 : kx_skip_ws_bytes(in_len, n));
  return kx_decode_ws_bytes(s->prog, in_len, offs, n);
}

static int decode_sizes(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len, const uint64_t* offsets,
                        const uint64_t* ends, uint64_t n, uint64_t* units, kx_status* status, void* stream) {
  if (!c || !s || !status || !units || (!in && in_len) || (ends && !offsets)) return KX_ERR_INVALID_ARG;
  if (!s->nprog) return KX_ERR_NOT_IMPLEMENTED;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  const KxnProgram& P = *s->nprog;
  memset(status, 0, sizeof *status);
  uint64_t tot[KXN_MAX_CUR] = {0};
  if (n) {
    kx_status* dst = nullptr;
    KX_HIP_CHECK(hipMalloc(&dst, sizeof(kx_status)));
    rc = nested_decode(c, s, in, in_len, offsets, ends, n, nullptr, nullptr, dst, st, tot);
    if (!rc && hipMemcpyAsync(status, dst, sizeof(kx_status), hipMemcpyDeviceToHost, st) != hipSuccess) rc = KX_ERR_HIP;
    if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = KX_ERR_HIP;
    (void)hipFree(dst);
    if (rc) return rc;
  }
  for (uint32_t i = 0; i < s->ncols; i++) {
    const KxnCol& K = P.col[i];
    units[3 * i] = K.dcur >= 0 ? tot[K.dcur] : n;
    units[3 * i + 1] = K.narr >= 2 ? tot[K.acur[0]] : 0;
    units[3 * i + 2] = K.narr >= 3 ? tot[K.acur[1]] : 0;
  }
  return KX_OK;
}

int kx_thrift_decode_sizes(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                           const uint64_t* offsets, uint64_t n, uint64_t* units, kx_status* status, void* stream) {
  return decode_sizes(c, s, in, in_len, offsets, nullptr, n, units, status, stream);
}

int kx_thrift_decode_sizes_extents(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                                   const uint64_t* starts, const uint64_t* ends, uint64_t n, uint64_t* units,
                                   kx_status* status, void* stream) {
  if (!starts || !ends) return KX_ERR_INVALID_ARG;
  return decode_sizes(c, s, in, in_len, starts, ends, n, units, status, stream);
}

int kx_thrift_skip_batch(kx_ctx* c, const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t* offsets_out,
                         kx_status* status, void* stream) {
  if (!c || !status || !offsets_out || (!in && in_len)) return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    KX_HIP_CHECK(hipMemsetAsync(status, 0, sizeof(kx_status), st));
    KX_HIP_CHECK(hipMemsetAsync(offsets_out, 0, 8, st));
    return KX_OK;
  }
  uint64_t epoch = 0;
  if ((rc = ensure_ws(c, kx_skip_ws_bytes(in_len, n), st, &epoch))) return rc;
  return kx_launch_skip(in, in_len, n, offsets_out, status, c->ws, c->ws_size, epoch, st);
}

int kx_thrift_split_points(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len, uint64_t n,
                           uint32_t parts, uint64_t* points_out, kx_status* status, void* stream) {
  if (!c || !s || !status || !points_out || (!in && in_len) || parts == 0 || parts > 65536)
    return KX_ERR_INVALID_ARG;
  // Kitex-Protobuf (nested or flat): Batch frames, not Thrift records
  if ((s->nprog && s->nprog->pb) || (!s->nprog && s->prog.is_pb)) return KX_ERR_NOT_IMPLEMENTED;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    KX_HIP_CHECK(hipMemsetAsync(status, 0, sizeof(kx_status), st));
    KX_HIP_CHECK(hipMemsetAsync(points_out, 0, 8ull * (parts + 1), st));
    return KX_OK;
  }
  KxProgram* dp = nullptr;
  if (!s->nprog && (rc = prog_on_device(const_cast<kx_schema*>(s), c->device, &dp))) return rc;
  uint64_t epoch = 0;
  if ((rc = ensure_ws(c, kx_skip_ws_bytes(in_len, n), st, &epoch))) return rc;
  return kx_launch_split(dp, s->nprog ? nullptr : &s->prog, in, in_len, n, parts, points_out, status, c->ws,
                         c->ws_size, epoch, st);
}

int kx_thrift_encoded_size_batch(kx_ctx* c, const kx_schema* s, const kx_columns* in, uint64_t n,
                                 uint64_t* sizes_out, void* stream) {
  if (!c || !s || !sizes_out) return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (s->nprog) {
    if (s->nprog->pb) return KX_ERR_NOT_IMPLEMENTED;   // a Kitex-Protobuf schema: kx_pb_encoded_size_batch
    return nested_encode(c, s, in, n, nullptr, 0, sizes_out, nullptr, nullptr, st, true);
  }
  KxLaunchCols lc;
  if ((rc = to_launch_cols(s, in, &lc))) return rc;
  if (n == 0) return KX_OK;
  KxProgram* dp = nullptr;
  if ((rc = prog_on_device(const_cast<kx_schema*>(s), c->device, &dp))) return rc;
  if ((rc = ensure_ews(c, kx_encode_ws_bytes(n), st))) return rc;
  return kx_launch_encode(dp, s->prog, lc, n, nullptr, 0, sizes_out, nullptr, nullptr, c->ews, c->ews_size, st,
                          true);
}

int kx_thrift_encode_batch(kx_ctx* c, const kx_schema* s, const kx_columns* in, uint64_t n, uint8_t* out,
                           uint64_t out_cap, uint64_t* offsets_out, kx_status* status, void* stream) {
  if (!c || !s || !status || (!out && out_cap)) return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (s->nprog && s->nprog->pb) return KX_ERR_NOT_IMPLEMENTED;   // a Kitex-Protobuf schema: kx_pb_encode_batch
  if (s->nprog && n) return nested_encode(c, s, in, n, out, out_cap, nullptr, offsets_out, status, st, false);
  KxLaunchCols lc;
  if (!s->nprog && (rc = to_launch_cols(s, in, &lc))) return rc;
  if (n == 0) {
    KX_HIP_CHECK(hipMemsetAsync(status, 0, sizeof(kx_status), st));
    if (offsets_out) KX_HIP_CHECK(hipMemsetAsync(offsets_out, 0, 8, st));
    return KX_OK;
  }
  KxProgram* dp = nullptr;
  if ((rc = prog_on_device(const_cast<kx_schema*>(s), c->device, &dp))) return rc;
  if ((rc = ensure_ews(c, kx_encode_ws_bytes(n), st))) return rc;
  return kx_launch_encode(dp, s->prog, lc, n, out, out_cap, nullptr, offsets_out, status, c->ews, c->ews_size,
                          st, false);
}

int kx_thrift_encode_messages(kx_ctx* c, const kx_schema* s, const kx_columns* in, uint64_t n, const char* name,
                              uint32_t name_len, int32_t msg_type, const int32_t* seqids, int32_t body_field,
                              uint8_t* body_scratch, uint64_t scratch_cap, uint8_t* out, uint64_t out_cap,
                              uint64_t* offsets_out, kx_status* status, void* stream) {
  if (!c || !s || !status || (!out && out_cap) || (!body_scratch && scratch_cap) || (n && !seqids) ||
      (name_len && !name) || body_field < 0 || body_field > 32767 || msg_type < 1 || msg_type > 4)
    return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  KxLaunchCols lc;
  if ((rc = to_launch_cols(s, in, &lc))) return rc;
  // scratch: record offsets (n + 1), then the name
  const size_t need = (n + 1) * 8 + name_len + 8;
  if (c->xws_size < need) {
    if (c->xws) {
      KX_HIP_CHECK(hipStreamSynchronize(st));
      KX_HIP_CHECK(hipFree(c->xws));
      c->xws = nullptr;
      c->xws_size = 0;
    }
    const size_t sz = need < (1u << 20) ? (1u << 20) : need + need / 4;
    KX_HIP_CHECK(hipMalloc(&c->xws, sz));
    c->xws_size = sz;
  }
  uint64_t* boff = (uint64_t*)c->xws;
  uint8_t* dname = (uint8_t*)c->xws + (n + 1) * 8;
  if (name_len) KX_HIP_CHECK(hipMemcpyAsync(dname, name, name_len, hipMemcpyHostToDevice, st));
  if (n == 0) {
    KX_HIP_CHECK(hipMemsetAsync(boff, 0, 8, st));
    KX_HIP_CHECK(hipMemsetAsync(status, 0, sizeof(kx_status), st));
  } else {
    KxProgram* dp = nullptr;
    if ((rc = prog_on_device(const_cast<kx_schema*>(s), c->device, &dp))) return rc;
    if ((rc = ensure_ews(c, kx_encode_ws_bytes(n), st))) return rc;
    // the records back to back (FastWriteNocopy), then each wrapped into its message
    if ((rc = kx_launch_encode(dp, s->prog, lc, n, body_scratch, scratch_cap, nullptr, boff, status, c->ews,
                               c->ews_size, st, false)))
      return rc;
  }
  // the status keeps the record encoder's code (SIZE_LIMIT: the scratch is too small); the message pass
  // sets consumed / n_records and SIZE_LIMIT when `out` is too small
  return kx_launch_message_encode(body_scratch, boff, scratch_cap, n, dname, name_len, msg_type, seqids, body_field, out,
                                  out_cap, offsets_out, status, st);
}

static int pb_schema_ok(const kx_schema* s) {
  for (uint32_t f = 0; f < s->prog.nfields; f++)
    if (s->prog.f[f].pb_wt == 7 || s->prog.ninst != 1) return KX_ERR_NOT_IMPLEMENTED;
  return KX_OK;
}

int kx_pb_decode_batch(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                       const uint64_t* offsets, uint64_t n, const kx_columns* out, uint8_t* record_status,
                       kx_status* status, void* stream) {
  if (!c || !s || !status || (!in && in_len)) return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (s->nprog) {   // nested proto3 messages (KX_STRUCT_PROTOBUF): the nested walker in proto mode
    if (!s->nprog->pb) return KX_ERR_NOT_IMPLEMENTED;
    return nested_decode(c, s, in, in_len, offsets, nullptr, n, out, record_status, status, st, nullptr);
  }
  KxLaunchCols lc;
  if ((rc = to_launch_cols(s, out, &lc, true, in_len))) return rc;
  if ((rc = pb_schema_ok(s))) return rc;
  if (n == 0) {
    KX_HIP_CHECK(hipMemsetAsync(status, 0, sizeof(kx_status), st));
    for (uint32_t k = 0; k < s->ncols; k++)
      if (lc.offs[k] && !((lc.view >> k) & 1))
        KX_HIP_CHECK(hipMemsetAsync(lc.offs[k], 0, ((lc.owide >> k) & 1) ? 8 : 4, st));
    return KX_OK;
  }
  KxProgram* dp = nullptr;
  if ((rc = prog_on_device(const_cast<kx_schema*>(s), c->device, &dp))) return rc;
  size_t ws = kx_decode_ws_bytes(s->prog, in_len, offsets, n);
  uint64_t epoch = 0;
  if ((rc = ensure_ws(c, ws, st, &epoch))) return rc;
  if ((rc = ensure_pipe(c))) return rc;
  return kx_launch_decode(dp, s->prog, in, in_len, offsets, n, lc, record_status, status, c->ws, c->ws_size,
                          epoch, st, true, nullptr, nullptr, &c->pipe);
}

// N framed messages: headers on the device (kx_message.hip), then the record bodies through the
// known-offsets decode with explicit ends, then the per-message codes merged (header code first)
// (framed payloads: message i = in[offsets[i] .. ends[i]), rep = the n + 1 frame offsets reported in
// the status, pre = the framing scan's status)
static int decode_messages(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                           const uint64_t* offsets, uint64_t n, int32_t body_field, bool pb,
                           const kx_column* msg_cols, const kx_columns* out, uint8_t* record_status,
                           kx_status* status, void* stream, const uint64_t* ends = nullptr,
                           const uint64_t* rep = nullptr, const kx_status* pre = nullptr,
                           const uint8_t* pre_rc = nullptr, const uint8_t* raw_flags = nullptr,
                           bool raw = false) {
  if (!c || !s || !status || !offsets || (!in && in_len)) return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  KxLaunchCols lc;
  if ((rc = to_launch_cols(s, out, &lc, true, in_len))) return rc;
  if (pb && (rc = pb_schema_ok(s))) return rc;
  KxMsgOut mo{};
  if (msg_cols) {
    const kx_column& nm = msg_cols[0];
    const int w = offset_width(nm);
    if (!w) return KX_ERR_INVALID_ARG;
    mo.name_offs = nm.offsets;
    mo.name_data = (uint8_t*)nm.data;
    mo.name_cap = nm.data ? nm.capacity : 0;
    mo.name_owide = w == 8;
    mo.msg_type = (int32_t*)msg_cols[1].data;
    mo.seqid = (int32_t*)msg_cols[2].data;
  }
  if (n == 0) {
    KX_HIP_CHECK(hipMemsetAsync(status, 0, sizeof(kx_status), st));
    for (uint32_t k = 0; k < s->ncols; k++)
      if (lc.offs[k] && !((lc.view >> k) & 1))
        KX_HIP_CHECK(hipMemsetAsync(lc.offs[k], 0, ((lc.owide >> k) & 1) ? 8 : 4, st));
    if (mo.name_offs) KX_HIP_CHECK(hipMemsetAsync(mo.name_offs, 0, mo.name_owide ? 8 : 4, st));
    return KX_OK;
  }
  if ((rc = ensure_mws(c, kx_message_ws_bytes(n), st))) return rc;
  uint64_t *rs = nullptr, *re = nullptr;
  uint8_t *hrc = nullptr, *brc = nullptr;
  if ((rc = kx_launch_message_headers(in, in_len, offsets, n, body_field, pb, mo, c->mws, &rs, &re, &hrc, &brc,
                                      st, ends, pre, pre_rc, raw_flags, raw)))
    return rc;
  KxProgram* dp = nullptr;
  if ((rc = prog_on_device(const_cast<kx_schema*>(s), c->device, &dp))) return rc;
  uint64_t epoch = 0;
  if ((rc = ensure_ws(c, kx_decode_ws_bytes(s->prog, in_len, rs, n), st, &epoch))) return rc;
  if ((rc = ensure_pipe(c))) return rc;
  if ((rc = kx_launch_decode(dp, s->prog, in, in_len, rs, n, lc, brc, status, c->ws, c->ws_size, epoch, st, pb,
                             re, nullptr, &c->pipe)))
    return rc;
  return kx_launch_message_merge(rep ? rep : offsets, n, hrc, brc, record_status, status, c->mws, st, pre);
}

static int ensure_fws(kx_ctx* c, size_t bytes, hipStream_t stream) {
  if (c->fws_size >= bytes) return KX_OK;
  if (c->fws) {
    KX_HIP_CHECK(hipStreamSynchronize(stream));
    KX_HIP_CHECK(hipFree(c->fws));
    c->fws = nullptr;
    c->fws_size = 0;
  }
  size_t sz = bytes < (1u << 20) ? (1u << 20) : bytes + bytes / 4;
  KX_HIP_CHECK(hipMalloc(&c->fws, sz));
  c->fws_size = sz;
  return KX_OK;
}

static int frame_scan(kx_ctx* c, const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t max_payload,
                      uint64_t* frame_offsets, uint64_t* payload_start, uint64_t* payload_end, uint8_t* kinds,
                      kx_status* status, void* stream, uint8_t* crc_codes) {
  if (!c || !status || !frame_offsets || (n && (!payload_start || !payload_end)) || (!in && in_len))
    return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    KX_HIP_CHECK(hipMemsetAsync(status, 0, sizeof(kx_status), st));
    KX_HIP_CHECK(hipMemsetAsync(frame_offsets, 0, 8, st));
    return KX_OK;
  }
  uint64_t epoch = 0;
  if ((rc = ensure_ws(c, kx_skip_ws_bytes(in_len, n), st, &epoch))) return rc;
  return kx_launch_frames(in, in_len, n, max_payload, frame_offsets, payload_start, payload_end, kinds, status, c->ws,
                          c->ws_size, epoch, st, false, nullptr, nullptr, nullptr, nullptr, crc_codes);
}

int kx_frame_scan(kx_ctx* c, const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t max_payload,
                  uint64_t* frame_offsets, uint64_t* payload_start, uint64_t* payload_end, uint8_t* kinds,
                  kx_status* status, void* stream) {
  return frame_scan(c, in, in_len, n, max_payload, frame_offsets, payload_start, payload_end, kinds, status, stream,
                    nullptr);
}

// CRC32C scratch: the launcher's error key (8 bytes, ~0 = none; its final kernel re-arms it)
static int ensure_cws(kx_ctx* c, hipStream_t stream) {
  if (c->cws) return KX_OK;
  KX_HIP_CHECK(hipMalloc(&c->cws, 256));
  KX_HIP_CHECK(hipMemsetAsync(c->cws, 0xff, 8, stream));
  return KX_OK;
}

int kx_crc32c_batch(kx_ctx* c, const uint8_t* in, uint64_t in_len, const uint64_t* offsets, uint64_t n,
                    uint32_t* crc_out, kx_status* status, void* stream) {
  if (!c || !status || !offsets || (n && !crc_out) || (!in && in_len)) return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if ((rc = ensure_cws(c, st))) return rc;
  return kx_launch_crc32c(in, in_len, offsets, n, false, nullptr, crc_out, nullptr, status, c->cws, st);
}

int kx_frame_crc32c_validate(kx_ctx* c, const uint8_t* in, uint64_t in_len, const uint64_t* frame_offsets,
                             uint64_t n, uint32_t* crc_out, uint8_t* record_status, kx_status* status,
                             void* stream) {
  if (!c || !status || !frame_offsets || (!in && in_len)) return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if ((rc = ensure_cws(c, st))) return rc;
  return kx_launch_crc32c(in, in_len, frame_offsets, n, true, nullptr, crc_out, record_status, status, c->cws, st);
}

int kx_ctx_set_crc32c_check(kx_ctx* c, int enable) {
  if (!c) return KX_ERR_INVALID_ARG;
  c->crc32c_check = enable != 0;
  return KX_OK;
}

// a kx_status inside a scratch layout takes a slot of this many bytes (the status grew to 192 B
// and the CRC status used to overlap the frame offsets)
#define KX_STATUS_SLOT 256
static_assert(sizeof(kx_status) <= KX_STATUS_SLOT, "scratch status slot");

// a socket buffer of n frames -> frame scan -> message headers -> record bodies
static int decode_frames(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len, uint64_t n,
                         int32_t body_field, bool pb, uint64_t max_payload, uint64_t* frame_offsets, uint8_t* kinds,
                         const kx_column* msg_cols, const kx_columns* out, uint8_t* record_status, kx_status* status,
                         void* stream) {
  if (!c || !s || !status || (!in && in_len)) return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    if (frame_offsets) KX_HIP_CHECK(hipMemsetAsync(frame_offsets, 0, 8, st));
    uint64_t z = 0;
    return decode_messages(c, s, in, in_len, &z, 0, body_field, pb, msg_cols, out, record_status, status, stream);
  }
  // scratch: [scan status][crc status][frame offsets n + 1][payload starts n + 1][payload ends n][crc codes n],
  // each status in its own KX_STATUS_SLOT-byte slot
  const size_t cs_at = KX_STATUS_SLOT, fo_at = 2 * KX_STATUS_SLOT, ps_at = fo_at + (n + 1) * 8,
               pe_at = ps_at + (n + 1) * 8, vr_at = pe_at + n * 8;
  if ((rc = ensure_fws(c, vr_at + n, st))) return rc;
  char* f = (char*)c->fws;
  kx_status* pre = (kx_status*)f;
  uint64_t* fo = frame_offsets ? frame_offsets : (uint64_t*)(f + fo_at);
  uint64_t* ps = (uint64_t*)(f + ps_at);
  uint64_t* pe = (uint64_t*)(f + pe_at);
  // DecodeMeta's payloadChecksumValidate (default_codec.go:205-209): fused into the frame scan's emit pass
  // (the payload is checked from the LDS window the scan already holds); KX_CRC_FUSED=0 runs the separate
  // checksum kernel after the scan instead
  uint8_t* vrc = c->crc32c_check ? (uint8_t*)(f + vr_at) : nullptr;
  const bool fused = vrc && kx_knob(KXK_CRC_FUSED);
  if ((rc = frame_scan(c, in, in_len, n, max_payload, fo, ps, pe, kinds, pre, stream, fused ? vrc : nullptr)))
    return rc;
  if (vrc && !fused) {
    if ((rc = ensure_cws(c, st))) return rc;
    if ((rc = kx_launch_crc32c(in, in_len, fo, n, true, pre, nullptr, vrc, (kx_status*)(f + cs_at), c->cws, st)))
      return rc;
  }
  return decode_messages(c, s, in, in_len, ps, n, body_field, pb, msg_cols, out, record_status, status, stream, pe,
                         fo, pre, vrc);
}

int kx_grpc_frame_scan(kx_ctx* c, const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t max_payload,
                       uint64_t* frame_offsets, uint64_t* payload_start, uint64_t* payload_end, uint8_t* flags,
                       kx_status* status, void* stream) {
  if (!c || !status || !frame_offsets || (n && (!payload_start || !payload_end)) || (!in && in_len))
    return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    KX_HIP_CHECK(hipMemsetAsync(status, 0, sizeof(kx_status), st));
    KX_HIP_CHECK(hipMemsetAsync(frame_offsets, 0, 8, st));
    return KX_OK;
  }
  uint64_t epoch = 0;
  if ((rc = ensure_ws(c, kx_skip_ws_bytes(in_len, n), st, &epoch))) return rc;
  return kx_launch_frames(in, in_len, n, max_payload, frame_offsets, payload_start, payload_end, flags, status, c->ws,
                          c->ws_size, epoch, st, true);
}

// n gRPC messages -> framing scan -> bodies (no message header: the payload is the record)
static int decode_grpc(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len, uint64_t n, bool pb,
                       uint64_t max_payload, uint64_t* frame_offsets, const kx_columns* out, uint8_t* record_status,
                       kx_status* status, void* stream) {
  if (!c || !s || !status || (!in && in_len)) return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    if (frame_offsets) KX_HIP_CHECK(hipMemsetAsync(frame_offsets, 0, 8, st));
    uint64_t z = 0;
    return decode_messages(c, s, in, in_len, &z, 0, 0, pb, nullptr, out, record_status, status, stream);
  }
  // scratch: [scan status][frame offsets n + 1][payload starts n + 1][payload ends n][flags n]
  const size_t fo_at = KX_STATUS_SLOT, ps_at = fo_at + (n + 1) * 8, pe_at = ps_at + (n + 1) * 8, fl_at = pe_at + n * 8;
  if ((rc = ensure_fws(c, fl_at + n, st))) return rc;
  char* f = (char*)c->fws;
  kx_status* pre = (kx_status*)f;
  uint64_t* fo = frame_offsets ? frame_offsets : (uint64_t*)(f + fo_at);
  uint64_t* ps = (uint64_t*)(f + ps_at);
  uint64_t* pe = (uint64_t*)(f + pe_at);
  uint8_t* fl = (uint8_t*)(f + fl_at);
  if ((rc = kx_grpc_frame_scan(c, in, in_len, n, max_payload, fo, ps, pe, fl, pre, stream))) return rc;
  return decode_messages(c, s, in, in_len, ps, n, 0, pb, nullptr, out, record_status, status, stream, pe, fo, pre,
                         nullptr, fl, true);
}

int kx_thrift_decode_grpc(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len, uint64_t n,
                          uint64_t max_payload, uint64_t* frame_offsets, const kx_columns* out,
                          uint8_t* record_status, kx_status* status, void* stream) {
  return decode_grpc(c, s, in, in_len, n, false, max_payload, frame_offsets, out, record_status, status, stream);
}

int kx_pb_decode_grpc(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len, uint64_t n,
                      uint64_t max_payload, uint64_t* frame_offsets, const kx_columns* out, uint8_t* record_status,
                      kx_status* status, void* stream) {
  return decode_grpc(c, s, in, in_len, n, true, max_payload, frame_offsets, out, record_status, status, stream);
}

// the values this library assumes for the un-vendored gopkg ttheader streaming constants (parity
// unpinned: DESIGN.md §3.6); ToMethod is transmeta.ToMethod (pkg/remote/transmeta/metakey.go:33)
void kx_ttstream_default_keys(kx_ttstream_keys* k) {
  if (!k) return;
  memset(k, 0, sizeof *k);
  k->frame_type_key = 27;   // ttheader.FrameType
  k->to_method_key = 9;     // ttheader.ToMethod = transmeta.ToMethod
  k->streaming_flag = 0x2;  // ttheader.HeaderFlagsStreaming
  const char* names[5] = {"1", "2", "3", "4", "5"};  // ttheader.FrameTypeMeta .. FrameTypeRst
  for (int i = 0; i < 5; i++) strncpy(k->type_names[i], names[i], 8);
}

int kx_ttstream_frame_scan(kx_ctx* c, const uint8_t* in, uint64_t in_len, uint64_t n, const kx_ttstream_keys* keys,
                           uint64_t* frame_offsets, uint64_t* payload_start, uint64_t* payload_end,
                           uint8_t* frame_types, int32_t* stream_ids, uint64_t* method_pos, uint32_t* method_len,
                           kx_status* status, void* stream) {
  if (!c || !status || !keys || !frame_offsets || (n && (!payload_start || !payload_end)) || (!in && in_len))
    return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    KX_HIP_CHECK(hipMemsetAsync(status, 0, sizeof(kx_status), st));
    KX_HIP_CHECK(hipMemsetAsync(frame_offsets, 0, 8, st));
    return KX_OK;
  }
  uint64_t epoch = 0;
  if ((rc = ensure_ws(c, kx_skip_ws_bytes(in_len, n), st, &epoch))) return rc;
  return kx_launch_frames(in, in_len, n, 0, frame_offsets, payload_start, payload_end, frame_types, status, c->ws,
                          c->ws_size, epoch, st, false, keys, stream_ids, method_pos, method_len);
}

static int decode_extents(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len, const uint64_t* starts,
                          const uint64_t* ends, uint64_t n, bool pb, const kx_columns* out, uint8_t* record_status,
                          kx_status* status, void* stream) {
  if (!c || !s || !status || (!in && in_len) || (n && (!starts || !ends))) return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (s->nprog && n) {   // nested schemas: the walker of the call's wire format
    if ((s->nprog->pb != 0) != pb) return KX_ERR_NOT_IMPLEMENTED;
    return nested_decode(c, s, in, in_len, starts, ends, n, out, record_status, status, st, nullptr);
  }
  KxLaunchCols lc;
  if ((rc = to_launch_cols(s, out, &lc, true, in_len))) return rc;
  if (n == 0) {
    KX_HIP_CHECK(hipMemsetAsync(status, 0, sizeof(kx_status), st));
    for (uint32_t k = 0; k < s->ncols; k++)
      if (lc.offs[k] && !((lc.view >> k) & 1))
        KX_HIP_CHECK(hipMemsetAsync(lc.offs[k], 0, ((lc.owide >> k) & 1) ? 8 : 4, st));
    return KX_OK;
  }
  KxProgram* dp = nullptr;
  if ((rc = prog_on_device(const_cast<kx_schema*>(s), c->device, &dp))) return rc;
  size_t ws = kx_decode_ws_bytes(s->prog, in_len, starts, n);
  uint64_t epoch = 0;
  if ((rc = ensure_ws(c, ws, st, &epoch))) return rc;
  return kx_launch_decode(dp, s->prog, in, in_len, starts, n, lc, record_status, status, c->ws, c->ws_size, epoch, st,
                          pb, ends, nullptr, nullptr);
}

int kx_thrift_decode_extents(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                             const uint64_t* starts, const uint64_t* ends, uint64_t n, const kx_columns* out,
                             uint8_t* record_status, kx_status* status, void* stream) {
  return decode_extents(c, s, in, in_len, starts, ends, n, false, out, record_status, status, stream);
}

int kx_pb_decode_extents(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                         const uint64_t* starts, const uint64_t* ends, uint64_t n, const kx_columns* out,
                         uint8_t* record_status, kx_status* status, void* stream) {
  return decode_extents(c, s, in, in_len, starts, ends, n, true, out, record_status, status, stream);
}

int kx_thrift_raw_messages(kx_ctx* c, const uint8_t* in, uint64_t in_len, const uint64_t* offsets, uint64_t n,
                           const kx_column* msg_cols, uint8_t* record_status, kx_status* status, void* stream) {
  if (!c || !status || !offsets || (!in && in_len)) return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  KxMsgOut mo{};
  if (msg_cols) {
    const kx_column& nm = msg_cols[0];
    const int w = offset_width(nm);
    if (!w) return KX_ERR_INVALID_ARG;
    mo.name_offs = nm.offsets;
    mo.name_data = (uint8_t*)nm.data;
    mo.name_cap = nm.data ? nm.capacity : 0;
    mo.name_owide = w == 8;
    mo.msg_type = (int32_t*)msg_cols[1].data;
    mo.seqid = (int32_t*)msg_cols[2].data;
  }
  KX_HIP_CHECK(hipMemsetAsync(status, 0, sizeof(kx_status), st));
  if (n == 0) {
    if (mo.name_offs) KX_HIP_CHECK(hipMemsetAsync(mo.name_offs, 0, mo.name_owide ? 8 : 4, st));
    return KX_OK;
  }
  if ((rc = ensure_mws(c, kx_message_ws_bytes(n), st))) return rc;
  uint64_t *rs = nullptr, *re = nullptr;
  uint8_t *hrc = nullptr, *brc = nullptr;
  if ((rc = kx_launch_message_headers(in, in_len, offsets, n, 0, false, mo, c->mws, &rs, &re, &hrc, &brc, st,
                                      nullptr, nullptr, nullptr, nullptr, 2)))
    return rc;
  KX_HIP_CHECK(hipMemsetAsync(brc, 0, n, st));  // no body is decoded: the request stays raw
  return kx_launch_message_merge(offsets, n, hrc, brc, record_status, status, c->mws, st, nullptr);
}

int kx_thrift_set_seqids(kx_ctx* c, uint8_t* in, uint64_t in_len, const uint64_t* offsets, uint64_t n,
                         const int32_t* seqids, uint8_t* record_status, kx_status* status, void* stream) {
  if (!c || !status || !offsets || (n && !seqids) || (!in && in_len)) return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if ((rc = ensure_mws(c, kx_message_ws_bytes(n), st))) return rc;
  return kx_launch_set_seqids(in, in_len, offsets, n, seqids, record_status, status, c->mws, st);
}

int kx_thrift_decode_frames(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len, uint64_t n,
                            int32_t body_field, uint64_t max_payload, uint64_t* frame_offsets, uint8_t* kinds,
                            const kx_column* msg_cols, const kx_columns* out, uint8_t* record_status,
                            kx_status* status, void* stream) {
  return decode_frames(c, s, in, in_len, n, body_field, false, max_payload, frame_offsets, kinds, msg_cols, out,
                       record_status, status, stream);
}

int kx_pb_decode_frames(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len, uint64_t n,
                        uint64_t max_payload, uint64_t* frame_offsets, uint8_t* kinds, const kx_column* msg_cols,
                        const kx_columns* out, uint8_t* record_status, kx_status* status, void* stream) {
  return decode_frames(c, s, in, in_len, n, 1, true, max_payload, frame_offsets, kinds, msg_cols, out,
                       record_status, status, stream);
}

int kx_thrift_decode_messages(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                              const uint64_t* offsets, uint64_t n, int32_t body_field,
                              const kx_column* msg_cols, const kx_columns* out, uint8_t* record_status,
                              kx_status* status, void* stream) {
  return decode_messages(c, s, in, in_len, offsets, n, body_field, false, msg_cols, out, record_status, status,
                         stream);
}

int kx_pb_decode_messages(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                          const uint64_t* offsets, uint64_t n, const kx_column* msg_cols,
                          const kx_columns* out, uint8_t* record_status, kx_status* status, void* stream) {
  return decode_messages(c, s, in, in_len, offsets, n, 0, true, msg_cols, out, record_status, status, stream);
}

int kx_pb_encoded_size_batch(kx_ctx* c, const kx_schema* s, const kx_columns* in, uint64_t n,
                             uint64_t* sizes_out, void* stream) {
  if (!c || !s || !sizes_out) return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (s->nprog) {
    if (!s->nprog->pb) return KX_ERR_NOT_IMPLEMENTED;
    return nested_encode(c, s, in, n, nullptr, 0, sizes_out, nullptr, nullptr, st, true);
  }
  if ((rc = pb_schema_ok(s))) return rc;
  KxLaunchCols lc;
  if ((rc = to_launch_cols(s, in, &lc))) return rc;
  if (n == 0) return KX_OK;
  KxProgram* dp = nullptr;
  if ((rc = prog_on_device(const_cast<kx_schema*>(s), c->device, &dp))) return rc;
  if ((rc = ensure_ews(c, kx_encode_ws_bytes(n), st))) return rc;
  return kx_launch_encode(dp, s->prog, lc, n, nullptr, 0, sizes_out, nullptr, nullptr, c->ews, c->ews_size, st,
                          true, true);
}

int kx_pb_encode_batch(kx_ctx* c, const kx_schema* s, const kx_columns* in, uint64_t n, uint8_t* out,
                       uint64_t out_cap, uint64_t* offsets_out, kx_status* status, void* stream) {
  if (!c || !s || !status || (!out && out_cap)) return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (s->nprog) {
    if (!s->nprog->pb) return KX_ERR_NOT_IMPLEMENTED;
    if (n == 0) {
      KX_HIP_CHECK(hipMemsetAsync(status, 0, sizeof(kx_status), st));
      if (offsets_out) KX_HIP_CHECK(hipMemsetAsync(offsets_out, 0, 8, st));
      return KX_OK;
    }
    return nested_encode(c, s, in, n, out, out_cap, nullptr, offsets_out, status, st, false);
  }
  if ((rc = pb_schema_ok(s))) return rc;
  KxLaunchCols lc;
  if ((rc = to_launch_cols(s, in, &lc))) return rc;
  if (n == 0) {
    KX_HIP_CHECK(hipMemsetAsync(status, 0, sizeof(kx_status), st));
    if (offsets_out) KX_HIP_CHECK(hipMemsetAsync(offsets_out, 0, 8, st));
    return KX_OK;
  }
  KxProgram* dp = nullptr;
  if ((rc = prog_on_device(const_cast<kx_schema*>(s), c->device, &dp))) return rc;
  if ((rc = ensure_ews(c, kx_encode_ws_bytes(n), st))) return rc;
  return kx_launch_encode(dp, s->prog, lc, n, out, out_cap, nullptr, offsets_out, status, c->ews, c->ews_size,
                          st, false, true);
}

// device decode of one batch (thrift or protobuf body, flat schema), arena positions starting at var_base
static int decode_device(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len, const uint64_t* offsets,
                         uint64_t n, const kx_columns* out, uint8_t* record_status, kx_status* status, hipStream_t st,
                         bool pb, const uint64_t* var_base_dev) {
  KxLaunchCols lc;
  int rc = to_launch_cols(s, out, &lc);
  if (rc) return rc;
  if (pb && (rc = pb_schema_ok(s))) return rc;
  KxProgram* dp = nullptr;
  if ((rc = prog_on_device(const_cast<kx_schema*>(s), c->device, &dp))) return rc;
  uint64_t epoch = 0;
  if ((rc = ensure_ws(c, kx_decode_ws_bytes(s->prog, in_len, offsets, n), st, &epoch))) return rc;
  if ((rc = ensure_pipe(c))) return rc;
  return kx_launch_decode(dp, s->prog, in, in_len, offsets, n, lc, record_status, status, c->ws, c->ws_size, epoch, st,
                          pb, nullptr, nullptr, &c->pipe, var_base_dev);
}

// the host pipelines' streams, events (a ring of KX_HOST_CH per kind) and pinned staging (per-chunk status,
// per-chunk unit totals, per-chunk nested column tables), created once per ctx
static int ensure_host(kx_ctx* c) {
  if (!c->own_stream) KX_HIP_CHECK(hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking));
  if (!c->h2d_stream) KX_HIP_CHECK(hipStreamCreateWithFlags(&c->h2d_stream, hipStreamNonBlocking));
  if (!c->d2h_stream) KX_HIP_CHECK(hipStreamCreateWithFlags(&c->d2h_stream, hipStreamNonBlocking));
  if (c->hst) return KX_OK;
  for (int k = 0; k < KX_HOST_CH; k++) {
    KX_HIP_CHECK(hipEventCreateWithFlags(&c->hev_in[k], hipEventDisableTiming));
    KX_HIP_CHECK(hipEventCreateWithFlags(&c->hev_run[k], hipEventDisableTiming));
    KX_HIP_CHECK(hipEventCreateWithFlags(&c->hev_st[k], hipEventDisableTiming));
  }
  KX_HIP_CHECK(hipHostMalloc((void**)&c->htot, KX_HOST_CH * KXN_MAX_CUR * sizeof(uint64_t), hipHostMallocDefault));
  KX_HIP_CHECK(hipHostMalloc((void**)&c->hcols, KX_HOST_CH * sizeof(KxnCols), hipHostMallocDefault));
  KX_HIP_CHECK(hipHostMalloc((void**)&c->hst, KX_HOST_CH * sizeof(kx_status), hipHostMallocDefault));
  return KX_OK;
}

// entry i of a host offsets array (4 or 8 bytes)
static inline uint64_t host_off(const void* p, uint32_t ob, uint64_t i) {
  return ob == 8 ? ((const uint64_t*)p)[i] : ((const uint32_t*)p)[i];
}

// What the host pipelines copy of one column: its offsets arrays (array 0 = record offsets, n + 1
// entries; array j >= 1 indexed by the element domain array j - 1 points into) and its data units. key[j]
// names the running total (a flat schema's var slot, a nested schema's cursor) that counts array j's
// entries past the first, dkey the one that counts data units (-1: one value per record).
struct HostCol {
  uint32_t narr;   // offsets arrays (0: FIXED)
  uint32_t unit;   // bytes per data unit
  int key[3];
  int dkey;
};

static void host_plan(const kx_schema* s, HostCol* hc) {
  for (uint32_t c = 0; c < s->ncols; c++) {
    HostCol& h = hc[c];
    h.key[0] = h.key[1] = h.key[2] = -1;
    if (s->nprog) {
      const KxnCol& K = s->nprog->col[c];
      h.narr = K.narr;
      h.unit = K.width ? K.width : 1;
      for (int j = 1; j < K.narr && j < 3; j++) h.key[j] = K.acur[j - 1];
      h.dkey = K.dcur;
      continue;
    }
    const KxpCol& K = s->prog.col[c];
    const uint32_t kind = s->info[c].kind;
    h.unit = kind == KX_COL_BYTES || kind == KX_COL_LIST_BYTES ? 1u : s->info[c].width;
    h.narr = kind == KX_COL_FIXED ? 0u : kind == KX_COL_LIST_BYTES ? 2u : 1u;
    h.dkey = kind == KX_COL_FIXED ? -1 : kind == KX_COL_LIST_BYTES ? (int)K.vslot2 : (int)K.vslot;
    if (kind == KX_COL_LIST_BYTES) h.key[1] = K.vslot;
  }
}

static inline void* host_arr(const kx_column& k, int j) {
  return j == 0 ? k.offsets : j == 1 ? k.elem_offsets : k.sub_offsets;
}
static inline uint64_t host_arr_cap(const kx_column& k, int j, uint64_t n) {   // entries - 1
  return j == 0 ? n : j == 1 ? k.elem_capacity : k.sub_capacity;
}
static inline void set_arr(kx_column& k, int j, void* p, uint64_t cap) {
  if (j == 0) k.offsets = p;
  else if (j == 1) { k.elem_offsets = p; k.elem_capacity = cap; }
  else { k.sub_offsets = p; k.sub_capacity = cap; }
}

// the host columns of a host pipeline: no views, every array its column kind needs
static int check_host_cols(const kx_schema* s, const HostCol* hc, const kx_columns* cols) {
  if (cols->ncols != s->ncols || (s->npres && !cols->presence)) return KX_ERR_INVALID_ARG;
  for (uint32_t k = 0; k < s->ncols; k++) {
    const kx_column& col = cols->cols[k];
    if (col.flags) return KX_ERR_INVALID_ARG;   // views: device-resident inputs only
    if (!hc[k].narr) {
      if (!col.data) return KX_ERR_INVALID_ARG;
      continue;
    }
    if (!offset_width(col) || (!col.data && col.capacity)) return KX_ERR_INVALID_ARG;
    for (uint32_t j = 0; j < hc[k].narr; j++)
      if (!host_arr(col, (int)j)) return KX_ERR_INVALID_ARG;
  }
  return KX_OK;
}

// Column staging in the device area at p (advanced): the same shape as the host columns, arrays sized
// to their capacities (decode) or to the units the host columns hold (encode: units[k][j], data at j = narr)
static void stage_cols(const kx_schema* s, const HostCol* hc, const kx_columns* host, uint64_t n,
                       const uint64_t (*units)[4], char** p, kx_columns* dc) {
  auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
  memset(dc, 0, sizeof *dc);
  dc->ncols = s->ncols;
  for (uint32_t k = 0; k < s->ncols; k++) {
    const kx_column& col = host->cols[k];
    kx_column& d = dc->cols[k];
    if (!hc[k].narr) {
      d.data = *p;
      *p += al(n * hc[k].unit);
      continue;
    }
    const uint32_t ob = (uint32_t)offset_width(col);
    d.offset_bytes = ob;
    for (uint32_t j = 0; j < hc[k].narr; j++) {
      const uint64_t cap = units ? units[k][j] : host_arr_cap(col, (int)j, n);
      set_arr(d, (int)j, *p, cap);
      *p += al((cap + 1) * ob);
    }
    d.capacity = units ? units[k][hc[k].narr] : col.capacity;
    d.data = *p;
    *p += al(d.capacity * hc[k].unit);
  }
  if (s->npres) {
    dc->presence = (uint64_t*)*p;
    *p += al(n * 8);
  }
}

static uint64_t stage_bytes(const kx_schema* s, const HostCol* hc, const kx_columns* host, uint64_t n,
                            const uint64_t (*units)[4]) {
  char* p = nullptr;
  kx_columns dc;
  stage_cols(s, hc, host, n, units, &p, &dc);
  return (uint64_t)(uintptr_t)p;
}

// record rows [r0, r0 + nk) of staged columns: the window a chunk's kernels see (record-indexed arrays and
// fixed values shifted, element arrays and arenas absolute)
static kx_columns chunk_window(const kx_schema* s, const HostCol* hc, const kx_columns& dc, uint64_t r0) {
  kx_columns ck = dc;
  for (uint32_t j = 0; j < s->ncols; j++) {
    if (!hc[j].narr) ck.cols[j].data = (char*)dc.cols[j].data + r0 * hc[j].unit;
    else ck.cols[j].offsets = (char*)dc.cols[j].offsets + r0 * dc.cols[j].offset_bytes;
  }
  if (dc.presence) ck.presence = dc.presence + r0;
  return ck;
}

static int grow_dstage(kx_ctx* c, uint64_t need) {
  if (c->dstage_size >= need) return KX_OK;
  if (c->dstage) KX_HIP_CHECK(hipFree(c->dstage));
  c->dstage = nullptr;
  c->dstage_size = 0;
  KX_HIP_CHECK(hipMalloc(&c->dstage, need));
  c->dstage_size = need;
  return KX_OK;
}

// fastUnmarshal end to end from host (netpoll) memory, for every schema the device entry points take
// (flat columns of every kind, nested Thrift and Kitex-PB schemas). With message offsets (the RPC case:
// framing gives every message's length) and n >= 64 Ki the batch runs as a pipeline of KX_HOST_CH
// record-range chunks over three streams: the H2D of every chunk is queued at once (each chunk's input at
// its own offsets, so the caller's offsets work unchanged on the device); decode k waits for its chunk's
// input and continues the arenas where chunk k - 1 ended, reading chunk k - 1's totals ON THE DEVICE (a
// flat schema's var_total, a nested schema's cursor totals), so decode k + 1 is queued before the host
// reads chunk k's totals; the host reads them (pinned, behind the decode on the decode stream) only to size
// the D2H of chunk k's element and arena ranges. Without offsets: one chunk (the boundaries are found by
// the decode). record_status (host, n bytes, optional): each record's code (known offsets: records fail
// independently, codec_fast.go:62-71; concatenated: records from the failing one on carry its code).
static int host_decode(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len, const uint64_t* offsets,
                       uint64_t n, const kx_columns* out, uint8_t* record_status, kx_status* status, bool pb) {
  if (!c || !s || !status || !out || (!in && in_len)) return KX_ERR_INVALID_ARG;
  const bool nested = s->nprog != nullptr;
  if (nested && (s->nprog->pb != 0) != pb) return KX_ERR_NOT_IMPLEMENTED;
  int rc;
  if (!nested && pb && (rc = pb_schema_ok(s))) return rc;
  HostCol hc[KX_MAX_COLUMNS];
  host_plan(s, hc);
  if ((rc = check_host_cols(s, hc, out))) return rc;
  const uint32_t K = offsets && n >= (1u << 16) ? (uint32_t)KX_HOST_CH : 1u;  // chunks
  uint64_t r[KX_HOST_CH + 1];
  for (uint32_t k = 0; k <= K; k++) r[k] = n * k / K;
  if (offsets) {   // every chunk's input range, checked before anything is queued
    if (offsets[n] > in_len || offsets[0] > offsets[n]) return KX_ERR_INVALID_ARG;
    for (uint32_t k = 0; k < K; k++)
      if (offsets[r[k + 1]] < offsets[r[k]]) return KX_ERR_INVALID_ARG;
  }
  if ((rc = set_device(c))) return rc;
  if ((rc = ensure_host(c))) return rc;
  hipStream_t st = c->own_stream, sh = c->h2d_stream, sd = c->d2h_stream;
  if (n == 0) {
    memset(status, 0, sizeof *status);
    for (uint32_t k = 0; k < s->ncols; k++)
      for (uint32_t j = 0; j < hc[k].narr; j++)
        memset(host_arr(out->cols[k], (int)j), 0, (size_t)offset_width(out->cols[k]));
    return KX_OK;
  }
  const uint32_t nt = nested ? s->nprog->ncur : KXP_NV_MAX;   // running totals per chunk
  auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
  // staging: K statuses | K totals | K column tables | input | offsets | record codes | columns | presence
  const uint64_t cols_at = al(K * sizeof(kx_status)) + al(K * KXN_MAX_CUR * 8) + (nested ? al(K * sizeof(KxnCols)) : 0);
  const uint64_t in_at = cols_at, off_at = in_at + al(in_len), rs_at = off_at + (offsets ? al((n + 1) * 8) : 0),
                 col_at = rs_at + al(n);
  if ((rc = grow_dstage(c, col_at + stage_bytes(s, hc, out, n, nullptr)))) return rc;
  char* base = (char*)c->dstage;
  kx_status* d_st = (kx_status*)base;
  uint64_t* d_tot = (uint64_t*)(base + al(K * sizeof(kx_status)));
  KxnCols* d_cols = (KxnCols*)(base + al(K * sizeof(kx_status)) + al(K * KXN_MAX_CUR * 8));
  uint8_t* d_in = (uint8_t*)(base + in_at);
  uint64_t* d_off = offsets ? (uint64_t*)(base + off_at) : nullptr;
  uint8_t* d_rs = (uint8_t*)(base + rs_at);
  char* p = base + col_at;
  kx_columns dc;
  stage_cols(s, hc, out, n, nullptr, &p, &dc);
  // a failure after copies are queued: drain every stream before returning (the caller may free its
  // buffers as soon as this synchronous call returns)
  auto fail = [&](int e) {
    (void)hipStreamSynchronize(sh);
    (void)hipStreamSynchronize(st);
    (void)hipStreamSynchronize(sd);
    return e;
  };
  if (nested) {   // one column table per chunk, uploaded with the input (the walker's pinned staging is per ctx)
    KxnCols* hcols = (KxnCols*)c->hcols;
    for (uint32_t k = 0; k < K; k++) {
      const kx_columns ck = chunk_window(s, hc, dc, r[k]);
      if ((rc = fill_ncols(s, &ck, true, hcols[k]))) return rc;
    }
    KX_HIP_CHECK(hipMemcpyAsync(d_cols, hcols, K * sizeof(KxnCols), hipMemcpyHostToDevice, sh));
    if ((rc = ensure_nws(c, kx_nested_ws_bytes(*s->nprog, n / K + 1, offsets == nullptr), st))) return fail(rc);
  }
  if (offsets) {
    KX_HIP_CHECK(hipMemcpyAsync(d_off, offsets, (n + 1) * 8, hipMemcpyHostToDevice, sh));
    for (uint32_t k = 0; k < K; k++) {
      const uint64_t a = offsets[r[k]], b = offsets[r[k + 1]];
      if (b > a && hipMemcpyAsync(d_in + a, in + a, b - a, hipMemcpyHostToDevice, sh) != hipSuccess)
        return fail(KX_ERR_HIP);
      if (hipEventRecord(c->hev_in[k], sh) != hipSuccess) return fail(KX_ERR_HIP);
    }
  } else {
    if (in_len) KX_HIP_CHECK(hipMemcpyAsync(d_in, in, in_len, hipMemcpyHostToDevice, sh));
    KX_HIP_CHECK(hipEventRecord(c->hev_in[0], sh));
  }
  auto launch_chunk = [&](uint32_t k) -> int {
    const uint64_t r0 = r[k], nk = r[k + 1] - r[k];
    KX_HIP_CHECK(hipStreamWaitEvent(st, c->hev_in[k], 0));
    const uint64_t* ob = offsets ? d_off + r0 : nullptr;
    int e;
    if (nested) {
      e = nested_decode(c, s, d_in, in_len, ob, nullptr, nk, nullptr, d_rs + r0, d_st + k, st, nullptr, d_cols + k,
                        k ? d_tot + (uint64_t)(k - 1) * KXN_MAX_CUR : nullptr, d_tot + (uint64_t)k * KXN_MAX_CUR);
    } else {
      const kx_columns ck = chunk_window(s, hc, dc, r0);
      e = decode_device(c, s, d_in, in_len, ob, nk, &ck, offsets ? d_rs + r0 : nullptr, d_st + k, st, pb,
                        k ? d_st[k - 1].var_total : nullptr);
    }
    if (e) return e;
    // the status and the totals (pinned) right behind the decode, on the decode stream: nothing is queued on
    // the copy-out stream before it can run (streams share hardware queues: a queued wait would hold back
    // what follows)
    KX_HIP_CHECK(hipMemcpyAsync(&c->hst[k], d_st + k, sizeof(kx_status), hipMemcpyDeviceToHost, st));
    if (nested)
      KX_HIP_CHECK(hipMemcpyAsync(c->htot + (uint64_t)k * KXN_MAX_CUR, d_tot + (uint64_t)k * KXN_MAX_CUR, nt * 8,
                                  hipMemcpyDeviceToHost, st));
    KX_HIP_CHECK(hipEventRecord(c->hev_st[k], st));
    return KX_OK;
  };
  static const uint64_t zeros[KXN_MAX_CUR] = {0};
  auto totals_of = [&](uint32_t k) -> const uint64_t* {
    return nested ? c->htot + (uint64_t)k * KXN_MAX_CUR : c->hst[k].var_total;
  };
  // chunk k has been decoded: its rows of the fixed columns, record offsets, presence and record codes,
  // and the element / arena ranges its totals span past chunk k - 1's
  auto copy_out = [&](uint32_t k) -> int {
    const uint64_t r0 = r[k], nk = r[k + 1] - r[k];
    const uint64_t* t0 = k ? totals_of(k - 1) : zeros;
    const uint64_t* t1 = totals_of(k);
    auto d2h = [&](void* h, const void* d, uint64_t bytes) -> int {
      if (bytes) KX_HIP_CHECK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, sd));
      return KX_OK;
    };
    for (uint32_t j = 0; j < s->ncols; j++) {
      const HostCol& h = hc[j];
      const kx_column& o = out->cols[j];
      const kx_column& d = dc.cols[j];
      int e;
      if (!h.narr) {
        if ((e = d2h((char*)o.data + r0 * h.unit, (const char*)d.data + r0 * h.unit, nk * h.unit))) return e;
        continue;
      }
      const uint32_t ob = d.offset_bytes;
      for (uint32_t a = 0; a < h.narr; a++) {   // entries [lo, hi] of array a (its closing entry included)
        uint64_t lo = r0, hi = r0 + nk;
        if (a) {
          const uint64_t cap = host_arr_cap(o, (int)a, n);
          lo = kmin64(t0[h.key[a]], cap);
          hi = kmin64(t1[h.key[a]], cap);
          if (hi < lo) continue;
        }
        if ((e = d2h((char*)host_arr(o, (int)a) + lo * ob, (const char*)host_arr(d, (int)a) + lo * ob,
                     (hi - lo + 1) * ob)))
          return e;
      }
      const uint64_t lo = kmin64(t0[h.dkey], o.capacity), hi = kmin64(t1[h.dkey], o.capacity);
      if (hi > lo && (e = d2h((char*)o.data + lo * h.unit, (const char*)d.data + lo * h.unit, (hi - lo) * h.unit)))
        return e;
    }
    if (s->npres) KX_HIP_CHECK(hipMemcpyAsync(out->presence + r0, dc.presence + r0, nk * 8, hipMemcpyDeviceToHost, sd));
    if (record_status && offsets)
      KX_HIP_CHECK(hipMemcpyAsync(record_status + r0, d_rs + r0, nk, hipMemcpyDeviceToHost, sd));
    return KX_OK;
  };
  kx_status first{};
  bool failed = false;
  uint32_t fail_chunk = K;
  if ((rc = launch_chunk(0))) return fail(rc);
  for (uint32_t k = 0; k < K; k++) {
    if (k + 1 < K && (rc = launch_chunk(k + 1))) return fail(rc);   // queued before chunk k's status is read
    if (hipEventSynchronize(c->hev_st[k]) != hipSuccess) return fail(KX_ERR_HIP);
    if ((rc = copy_out(k))) return fail(rc);
    const kx_status sk = c->hst[k];
    if (sk.code && !failed) {
      failed = true;
      first = sk;
      first.record += r[k];
    }
    if (sk.code == KX_ERR_SIZE_LIMIT && fail_chunk == K) fail_chunk = k;
  }
  if (hipStreamSynchronize(sd) != hipSuccess) return fail(KX_ERR_HIP);
  const kx_status last = c->hst[K - 1];
  *status = failed ? first : last;
  if (offsets) {
    status->n_records = n;
    status->consumed = offsets[n];
  }
  for (uint32_t v = 0; v < 16; v++) status->var_total[v] = last.var_total[v];
  if (record_status) {
    if (!offsets) {   // concatenated: the records before the failing one decoded, the rest carry its code
      const uint64_t ok = failed ? kmin64(first.record, n) : n;
      memset(record_status, 0, ok);
      if (ok < n) memset(record_status + ok, first.code, n - ok);
    } else if (fail_chunk < K) {   // an arena too small: nothing of that chunk or a later one was written
      memset(record_status + r[fail_chunk], KX_ERR_SIZE_LIMIT, n - r[fail_chunk]);
    }
  }
  return KX_OK;
}

// fastMarshal from host (netpoll-bound) memory: the columns go up, the wire comes back, for flat and
// nested schemas. The records are cut into KX_HOST_CH chunks (n >= 64 Ki): H2D of every chunk's column
// slices is queued at once (fixed rows, record offsets rows, and the element / arena ranges those offsets
// span level by level, all at their own positions, so the caller's offsets work unchanged on the device);
// encode k waits for its slices and starts writing where chunk k - 1 ended, which it reads from chunk k - 1's
// status on the device (out_base), so it is queued before the host learns chunk k - 1's size; the host reads
// each chunk's status (pinned, behind its encode) to copy that chunk's wire bytes out while the next chunk
// encodes. Every range is checked before the first copy is queued.
static int host_encode(kx_ctx* c, const kx_schema* s, const kx_columns* in, uint64_t n, uint8_t* out,
                       uint64_t out_cap, uint64_t* offsets_out, uint8_t* record_status, kx_status* status, bool pb) {
  if (!c || !s || !in || !status || (!out && out_cap)) return KX_ERR_INVALID_ARG;
  const bool nested = s->nprog != nullptr;
  if (nested && (s->nprog->pb != 0) != pb) return KX_ERR_NOT_IMPLEMENTED;
  int rc;
  if (!nested && pb && (rc = pb_schema_ok(s))) return rc;
  HostCol hc[KX_MAX_COLUMNS];
  host_plan(s, hc);
  if ((rc = check_host_cols(s, hc, in))) return rc;
  if (n == 0) {
    memset(status, 0, sizeof *status);
    if (offsets_out) offsets_out[0] = 0;
    return KX_OK;
  }
  const uint32_t K = n >= (1u << 16) ? (uint32_t)KX_HOST_CH : 1u;
  uint64_t r[KX_HOST_CH + 1];
  for (uint32_t k = 0; k <= K; k++) r[k] = n * k / K;
  // pos[k][c][j]: where chunk boundary k falls in array j of column c (j = narr: the data units); checked
  // monotonic and inside the arrays the host columns hold
  static thread_local uint64_t pos[KX_HOST_CH + 1][KX_MAX_COLUMNS][4];
  uint64_t units[KX_MAX_COLUMNS][4] = {{0}};
  for (uint32_t j = 0; j < s->ncols; j++) {
    const HostCol& h = hc[j];
    const kx_column& col = in->cols[j];
    if (!h.narr) continue;
    const uint32_t ob = (uint32_t)offset_width(col);
    for (uint32_t k = 0; k <= K; k++) {
      uint64_t x = r[k];
      pos[k][j][0] = x;
      for (uint32_t a = 0; a < h.narr; a++) {
        x = host_off(host_arr(col, (int)a), ob, x);
        pos[k][j][a + 1] = x;
        const uint64_t lim = a + 1 < h.narr ? host_arr_cap(col, (int)a + 1, n) : col.capacity;
        if (x > lim || (k && x < pos[k - 1][j][a + 1])) return KX_ERR_INVALID_ARG;
      }
    }
    units[j][0] = n;
    for (uint32_t a = 1; a <= h.narr; a++) units[j][a] = pos[K][j][a];
  }
  if ((rc = set_device(c))) return rc;
  if ((rc = ensure_host(c))) return rc;
  hipStream_t st = c->own_stream, sh = c->h2d_stream, sd = c->d2h_stream;
  auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
  // staging: K statuses | K column tables | out | offsets_out (n + 1) | columns | presence
  const uint64_t tab_at = al(K * sizeof(kx_status)), out_at = tab_at + (nested ? al(K * sizeof(KxnCols)) : 0),
                 offs_at = out_at + al(out_cap), col_at = offs_at + al((n + 1) * 8);
  if ((rc = grow_dstage(c, col_at + stage_bytes(s, hc, in, n, units)))) return rc;
  char* base = (char*)c->dstage;
  kx_status* d_st = (kx_status*)base;
  KxnCols* d_cols = (KxnCols*)(base + tab_at);
  uint8_t* d_out = (uint8_t*)(base + out_at);
  uint64_t* d_offs = (uint64_t*)(base + offs_at);
  char* p = base + col_at;
  kx_columns dc;
  stage_cols(s, hc, in, n, units, &p, &dc);
  auto fail = [&](int e) {
    (void)hipStreamSynchronize(sh);
    (void)hipStreamSynchronize(st);
    (void)hipStreamSynchronize(sd);
    return e;
  };
  KxProgram* dprog = nullptr;
  if (!nested && (rc = prog_on_device(const_cast<kx_schema*>(s), c->device, &dprog))) return rc;
  if (nested) {
    KxnCols* hcols = (KxnCols*)c->hcols;
    for (uint32_t k = 0; k < K; k++) {
      const kx_columns ck = chunk_window(s, hc, dc, r[k]);
      if ((rc = fill_ncols(s, &ck, false, hcols[k]))) return rc;
    }
    KX_HIP_CHECK(hipMemcpyAsync(d_cols, hcols, K * sizeof(KxnCols), hipMemcpyHostToDevice, sh));
  }
  const uint64_t chunk_max = r[1] - r[0] + 1;
  if ((rc = ensure_ews(c, nested ? kx_nested_enc_ws_bytes(chunk_max) : kx_encode_ws_bytes(chunk_max), st)))
    return fail(rc);
  // H2D of every chunk's slices, queued at once
  for (uint32_t k = 0; k < K; k++) {
    const uint64_t r0 = r[k], r1 = r[k + 1];
    auto h2d = [&](void* d, const void* h, uint64_t bytes) -> int {
      if (bytes) KX_HIP_CHECK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, sh));
      return KX_OK;
    };
    for (uint32_t j = 0; j < s->ncols; j++) {
      const HostCol& h = hc[j];
      const kx_column& col = in->cols[j];
      const kx_column& d = dc.cols[j];
      if (!h.narr) {
        if ((rc = h2d((char*)d.data + r0 * h.unit, (const char*)col.data + r0 * h.unit, (r1 - r0) * h.unit)))
          return fail(rc);
        continue;
      }
      const uint32_t ob = d.offset_bytes;
      for (uint32_t a = 0; a < h.narr; a++) {   // entries [pos_k, pos_k+1] of array a
        const uint64_t lo = pos[k][j][a], hi = pos[k + 1][j][a];
        if ((rc = h2d((char*)host_arr(d, (int)a) + lo * ob, (const char*)host_arr(col, (int)a) + lo * ob,
                      (hi - lo + 1) * ob)))
          return fail(rc);
      }
      const uint64_t lo = pos[k][j][h.narr], hi = pos[k + 1][j][h.narr];
      if ((rc = h2d((char*)d.data + lo * h.unit, (const char*)col.data + lo * h.unit, (hi - lo) * h.unit)))
        return fail(rc);
    }
    if (s->npres && (rc = h2d(dc.presence + r0, in->presence + r0, (r1 - r0) * 8))) return fail(rc);
    if (hipEventRecord(c->hev_in[k], sh) != hipSuccess) return fail(KX_ERR_HIP);
  }
  auto launch_chunk = [&](uint32_t k) -> int {
    const uint64_t r0 = r[k], nk = r[k + 1] - r[k];
    const uint64_t* ob = k ? &d_st[k - 1].consumed : nullptr;
    KX_HIP_CHECK(hipStreamWaitEvent(st, c->hev_in[k], 0));
    int e;
    if (nested) {
      e = nested_encode(c, s, nullptr, nk, d_out, out_cap, nullptr, d_offs + r0, d_st + k, st, false, d_cols + k, ob);
    } else {
      const kx_columns ck = chunk_window(s, hc, dc, r0);
      KxLaunchCols lc;
      if ((e = to_launch_cols(s, &ck, &lc))) return e;
      e = kx_launch_encode(dprog, s->prog, lc, nk, d_out, out_cap, nullptr, d_offs + r0, d_st + k, c->ews, c->ews_size,
                           st, false, pb, ob);
    }
    if (e) return e;
    // the status (pinned) right behind the encode on its stream (see host_decode)
    KX_HIP_CHECK(hipMemcpyAsync(&c->hst[k], d_st + k, sizeof(kx_status), hipMemcpyDeviceToHost, st));
    KX_HIP_CHECK(hipEventRecord(c->hev_st[k], st));
    return KX_OK;
  };
  if ((rc = launch_chunk(0))) return fail(rc);
  uint64_t pos_out = 0;
  kx_status first{};
  bool failed = false;
  uint32_t fail_chunk = K;
  for (uint32_t k = 0; k < K; k++) {
    if (k + 1 < K && (rc = launch_chunk(k + 1))) return fail(rc);   // queued before chunk k's size is known
    if (hipEventSynchronize(c->hev_st[k]) != hipSuccess) return fail(KX_ERR_HIP);
    const kx_status sk = c->hst[k];
    if (sk.code && !failed) {
      failed = true;
      first = sk;
      fail_chunk = k;
    }
    if (!failed) {
      const uint64_t r0 = r[k], nk = r[k + 1] - r[k];
      if (offsets_out && hipMemcpyAsync(offsets_out + r0, d_offs + r0, (nk + (k == K - 1 ? 1 : 0)) * 8,
                                        hipMemcpyDeviceToHost, sd) != hipSuccess)
        return fail(KX_ERR_HIP);
      if (sk.consumed > pos_out) {
        if (hipMemcpyAsync(out + pos_out, d_out + pos_out, sk.consumed - pos_out, hipMemcpyDeviceToHost, sd) !=
            hipSuccess)
          return fail(KX_ERR_HIP);
        pos_out = sk.consumed;
      }
    }
  }
  if (hipStreamSynchronize(sd) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) return fail(KX_ERR_HIP);
  memset(status, 0, sizeof *status);
  status->n_records = n;
  if (failed) {
    // the first failing chunk's code; consumed = the size the whole batch needs (chunk bases chain on the
    // device, so the last chunk's end is the total even past the failure), a caller retries with that
    status->code = first.code;
    status->record = r[fail_chunk];
    status->offset = pos_out;
    status->consumed = c->hst[K - 1].consumed;
  } else {
    status->consumed = pos_out;
  }
  if (record_status) {   // the records whose bytes are in `out`: 0; the rest: the failing chunk's code
    const uint64_t ok = failed ? r[fail_chunk] : n;
    memset(record_status, 0, ok);
    if (ok < n) memset(record_status + ok, first.code, n - ok);
  }
  return KX_OK;
}

int kx_host_encode_batch(kx_ctx* c, const kx_schema* s, const kx_columns* in, uint64_t n, uint8_t* out,
                         uint64_t out_cap, uint64_t* offsets_out, uint8_t* record_status, kx_status* status) {
  return host_encode(c, s, in, n, out, out_cap, offsets_out, record_status, status, false);
}

int kx_host_pb_encode_batch(kx_ctx* c, const kx_schema* s, const kx_columns* in, uint64_t n, uint8_t* out,
                            uint64_t out_cap, uint64_t* offsets_out, uint8_t* record_status, kx_status* status) {
  return host_encode(c, s, in, n, out, out_cap, offsets_out, record_status, status, true);
}

int kx_host_decode_batch(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                         const uint64_t* offsets, uint64_t n, const kx_columns* out, uint8_t* record_status,
                         kx_status* status) {
  return host_decode(c, s, in, in_len, offsets, n, out, record_status, status, false);
}

int kx_host_pb_decode_batch(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                            const uint64_t* offsets, uint64_t n, const kx_columns* out, uint8_t* record_status,
                            kx_status* status) {
  return host_decode(c, s, in, in_len, offsets, n, out, record_status, status, true);
}

uint64_t kx_thrift_message_begin_length(uint32_t name_len) { return 12ull + name_len; }

int kx_thrift_write_message_begin(uint8_t* buf, uint64_t cap, const char* name, uint32_t name_len,
                                  int32_t msg_type, int32_t seqid, uint64_t* written) {
  if (!buf || (!name && name_len) || !written) return KX_ERR_INVALID_ARG;
  uint64_t need = 12ull + name_len;
  if (cap < need) return KX_ERR_SIZE_LIMIT;
  uint32_t v = 0x80010000u | ((uint32_t)msg_type & 0xffu);
  uint8_t* p = buf;
  p[0] = v >> 24; p[1] = v >> 16; p[2] = v >> 8; p[3] = (uint8_t)v;
  p[4] = name_len >> 24; p[5] = name_len >> 16; p[6] = name_len >> 8; p[7] = (uint8_t)name_len;
  if (name_len) memcpy(p + 8, name, name_len);
  uint32_t sq = (uint32_t)seqid;
  p += 8 + name_len;
  p[0] = sq >> 24; p[1] = sq >> 16; p[2] = sq >> 8; p[3] = (uint8_t)sq;
  *written = need;
  return KX_OK;
}

int kx_thrift_read_message_begin(const uint8_t* buf, uint64_t len, const char** name, uint32_t* name_len,
                                 int32_t* msg_type, int32_t* seqid, uint64_t* consumed) {
  if (!buf || !name || !name_len || !msg_type || !seqid || !consumed) return KX_ERR_INVALID_ARG;
  auto be = [](const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
  };
  if (len < 4) return KX_ERR_EOF;
  uint32_t v = be(buf);
  if ((v & 0xffff0000u) != 0x80010000u) return KX_ERR_BAD_VERSION;
  if (len < 8) return KX_ERR_EOF;
  int32_t n = (int32_t)be(buf + 4);
  if (n < 0) return KX_ERR_NEGATIVE_SIZE;
  if (len < 12ull + (uint64_t)n) return KX_ERR_EOF;
  *name = (const char*)buf + 8;
  *name_len = (uint32_t)n;
  *msg_type = (int32_t)(v & 0xffu);
  *seqid = (int32_t)be(buf + 8 + n);
  *consumed = 12ull + (uint64_t)n;
  return KX_OK;
}

uint64_t kx_pb_meta_length(uint32_t name_len) { return 12ull + name_len; }

// codec.WriteUint32(ProtobufV1Magic + msgType), codec.WriteString(method), codec.WriteUint32(seqID)
// (protobuf.go:77-90)
int kx_pb_write_meta(uint8_t* buf, uint64_t cap, const char* name, uint32_t name_len, int32_t msg_type,
                     int32_t seqid, uint64_t* written) {
  if (!buf || (!name && name_len) || !written) return KX_ERR_INVALID_ARG;
  const uint64_t need = 12ull + name_len;
  if (cap < need) return KX_ERR_SIZE_LIMIT;
  auto put = [](uint8_t* p, uint32_t v) { p[0] = v >> 24; p[1] = v >> 16; p[2] = v >> 8; p[3] = (uint8_t)v; };
  put(buf, 0x90010000u + ((uint32_t)msg_type & 0xffffu));
  put(buf + 4, name_len);
  if (name_len) memcpy(buf + 8, name, name_len);
  put(buf + 8 + name_len, (uint32_t)seqid);
  *written = need;
  return KX_OK;
}

// protobufCodec.Unmarshal's meta read (protobuf.go:136-160): magic check, type, method, seqID
int kx_pb_read_meta(const uint8_t* buf, uint64_t len, const char** name, uint32_t* name_len, int32_t* msg_type,
                    int32_t* seqid, uint64_t* consumed) {
  if (!buf || !name || !name_len || !msg_type || !seqid || !consumed) return KX_ERR_INVALID_ARG;
  auto be = [](const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
  };
  if (len < 4) return KX_ERR_EOF;
  const uint32_t v = be(buf);
  if ((v & 0xffff0000u) != 0x90010000u) return KX_ERR_BAD_VERSION;
  if (len < 8) return KX_ERR_EOF;
  const int32_t n = (int32_t)be(buf + 4);
  if (n < 0) return KX_ERR_NEGATIVE_SIZE;
  if (len < 12ull + (uint64_t)n) return KX_ERR_EOF;
  *name = (const char*)buf + 8;
  *name_len = (uint32_t)n;
  *msg_type = (int32_t)(v & 0xffffu);
  *seqid = (int32_t)be(buf + 8 + n);
  *consumed = 12ull + (uint64_t)n;
  return KX_OK;
}

}  // extern "C"
