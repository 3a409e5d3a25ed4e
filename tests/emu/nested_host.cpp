// Test infrastructure only: the nested record walker (kitex_amd/csrc/kx_nested.h) run on the host with
// the device pipeline's steps in sequence (skip-delimited records, measure, per-cursor prefix sums,
// capacity check, write, closing entries), so CPU tests can compare it with the oracle.
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "hip/hip_runtime.h"
#include "kx_internal.h"
#include "kx_nested.h"

static int build(const kx_struct_desc* structs, uint32_t ns, kx_schema* s) {
  if (ns && (structs[0].reserved0 & KX_STRUCT_PROTOBUF)) return kx_build_nested(structs, ns, s);  // proto mode
  int rc = kx_build_program(structs, ns, s);
  if (rc == KX_OK) return KX_ERR_INVALID_ARG;  // a flat schema: not this path
  if (rc != KX_ERR_NOT_IMPLEMENTED) return rc;
  return kx_build_nested(structs, ns, s);
}

static void cols_of(const kx_schema& s, const kx_columns* out, KxnCols* C) {
  memset(C, 0, sizeof *C);
  for (uint32_t i = 0; i < s.ncols; i++) {
    const kx_column& k = out->cols[i];
    C->data[i] = k.data;
    C->arr[i][0] = k.offsets;
    C->arr[i][1] = k.elem_offsets;
    C->arr[i][2] = k.sub_offsets;
    C->cap[i][0] = k.capacity;
    C->cap[i][2] = k.elem_capacity;
    C->cap[i][3] = k.sub_capacity;
    if (k.offset_bytes == 8) C->owide |= 1ull << i;
  }
  C->presence = out->presence;
}

extern "C" int emu_nested_decode(const kx_struct_desc* structs, uint32_t ns, const uint8_t* in, uint64_t in_len,
                                 const uint64_t* offsets, uint64_t n, const kx_columns* out, uint8_t* rstat,
                                 kx_status* st) {
  kx_schema s;
  int rc = build(structs, ns, &s);
  if (rc) return rc;
  const KxnProgram& P = *s.nprog;
  KxnCols C;
  cols_of(s, out, &C);
  memset(st, 0, sizeof *st);
  // extents: the caller's, or the skip decoder's (codec_apache.go:166-172) for concatenated records
  std::vector<uint64_t> a(n), b(n);
  uint64_t nok = n;
  int skip_rc = 0;
  std::vector<uint64_t> fstart(n + 1, 0);   // proto: Batch frame starts (status offsets)
  if (offsets) {
    for (uint64_t r = 0; r < n; r++) { a[r] = offsets[r]; b[r] = offsets[r + 1]; }
  } else if (P.pb) {   // Kitex-PB Batch frames: 0x0A, uvarint length, body
    uint64_t pos = 0;
    for (uint64_t r = 0; r < n; r++) {
      fstart[r] = pos;
      uint64_t q = pos + 1, l = 0;
      skip_rc = pos >= in_len ? KX_ERR_EOF : in[pos] != 0x0A ? KX_ERR_INVALID_DATA : kxn_uvarint(in, in_len, &q, &l);
      if (!skip_rc && l > in_len - q) skip_rc = KX_ERR_EOF;
      if (skip_rc) { nok = r; a[r] = b[r] = 0; break; }
      a[r] = q;
      b[r] = q + l;
      pos = q + l;
    }
    fstart[nok < n ? nok : n] = pos;
  } else {
    uint64_t pos = 0;
    for (uint64_t r = 0; r < n; r++) {
      uint64_t q = pos;
      a[r] = pos;
      skip_rc = kxn_skip(in, in_len, &q, KX_T_STRUCT, KXN_SKIP_DEPTH);
      if (skip_rc) { nok = r; b[r] = in_len; break; }
      b[r] = q;
      pos = q;
    }
  }
  // measure
  std::vector<uint64_t> cnt((size_t)P.ncur * n, 0);
  std::vector<uint8_t> code(n, 0), careful(n, 0);
  std::vector<uint64_t> cur(KXN_MAX_CUR), lim(KXN_MAX_CUR), snap(KXN_MAX_SNAP);
  uint64_t first = n;
  for (uint64_t r = 0; r < n; r++) {
    if (!offsets && (r > nok || (r == nok && !skip_rc))) { code[r] = 0xff; continue; }
    for (uint32_t k = 0; k < P.ncur; k++) cur[k] = 0;
    uint64_t used = 0;
    // as the device: the fast walk (no snapshots), and for a record that repeats a field the careful walk
    auto walk = [&](uint64_t* sn) {
      return P.pb ? kxn_pb_read_record<false>(P, C, in + a[r], b[r] - a[r], r, KxnCurP{cur.data()}, sn, &used)
                  : kxn_read_record<false>(P, C, in + a[r], b[r] - a[r], r, KxnCurP{cur.data()}, sn, &used);
    };
    int e = (a[r] > b[r] || b[r] > in_len) ? KX_ERR_INVALID_ARG : walk(nullptr);
    if (e == KXN_REPEAT) {
      for (uint32_t k = 0; k < P.ncur; k++) cur[k] = 0;
      e = walk(snap.data());
      careful[r] = 1;
    }
    if (!e && !offsets && skip_rc && r == nok) e = skip_rc;
    code[r] = (uint8_t)e;
    if (e) { if (r < first) first = r; continue; }
    for (uint32_t k = 0; k < P.ncur; k++) cnt[(size_t)k * n + r] = cur[k];
  }
  // bases and totals
  std::vector<uint64_t> base((size_t)P.ncur * n), tot(P.ncur, 0);
  for (uint32_t k = 0; k < P.ncur; k++)
    for (uint64_t r = 0; r < n; r++) { base[(size_t)k * n + r] = tot[k]; tot[k] += cnt[(size_t)k * n + r]; }
  // capacities
  for (uint32_t c = 0; c < P.ncols; c++) {
    const KxnCol& K = P.col[c];
    bool over = K.dcur >= 0 && tot[K.dcur] > C.cap[c][0];
    for (int k = 1; k < K.narr; k++) over |= tot[K.acur[k - 1]] > C.cap[c][1 + k];
    if (over) { st->code = KX_ERR_SIZE_LIMIT; return KX_ERR_SIZE_LIMIT; }
  }
  // write (records in reverse order: what a replaced occurrence writes past its record's extent would
  // corrupt the next record if it were not clipped, as on the device where records run in parallel)
  for (uint64_t rr = n; rr-- > 0;) {
    const uint64_t r = rr;
    for (uint32_t k = 0; k < P.ncur; k++) {
      cur[k] = base[(size_t)k * n + r];
      lim[k] = cur[k] + cnt[(size_t)k * n + r];
    }
    uint64_t used = 0;
    uint64_t* sn = careful[r] ? snap.data() : nullptr;   // the fast walk stays inside the record's extents
    const uint64_t* li = careful[r] ? lim.data() : nullptr;
    if (code[r] == 0 && P.pb)
      (void)kxn_pb_read_record<true>(P, C, in + a[r], b[r] - a[r], r, KxnCurP{cur.data()}, sn, &used, li);
    else if (code[r] == 0)
      (void)kxn_read_record<true>(P, C, in + a[r], b[r] - a[r], r, KxnCurP{cur.data()}, sn, &used, li);
    else kxn_failed_record(P, C, r, KxnCurP{cur.data()});
    if (rstat && offsets) rstat[r] = code[r] == 0xff ? 0 : code[r];
  }
  for (uint32_t c = 0; c < P.ncols; c++) {
    const KxnCol& K = P.col[c];
    for (int k = 0; k < K.narr; k++) kxn_put_arr(C, (int)c, k, k == 0 ? n : tot[K.acur[k - 1]], tot[K.acur[k]]);
  }
  st->n_records = n;
  st->consumed = n ? b[n - 1] : 0;
  if (!offsets && P.pb) st->consumed = n ? b[n - 1] : 0;
  if (first < n) {
    st->code = code[first];
    st->record = first;
    st->offset = !offsets && P.pb ? fstart[first] : a[first];
    if (!offsets) { st->n_records = first; st->consumed = st->offset; }
  }
  return st->code;
}

extern "C" int emu_nested_encode(const kx_struct_desc* structs, uint32_t ns, const kx_columns* in, uint64_t n,
                                 uint8_t* out, uint64_t cap, uint64_t* offsets_out, uint64_t* total) {
  kx_schema s;
  int rc = build(structs, ns, &s);
  if (rc) return rc;
  KxnCols C;
  cols_of(s, in, &C);
  uint64_t pos = 0;
  const KxnProgram& P = *s.nprog;
  for (uint64_t r = 0; r < n; r++) pos += P.pb ? kxn_pb_frame_size(P, C, r) : kxn_write_record<false>(P, C, r, nullptr, 0);
  *total = pos;
  if (pos > cap) return KX_ERR_SIZE_LIMIT;
  pos = 0;
  for (uint64_t r = 0; r < n; r++) {
    if (offsets_out) offsets_out[r] = pos;
    if (P.pb) {
      const uint64_t fs = kxn_pb_frame_size(P, C, r);
      kxn_pb_write_frame(P, C, r, out, pos, fs);
      pos += fs;
    } else {
      pos += kxn_write_record<true>(P, C, r, out, pos);
    }
  }
  if (offsets_out) offsets_out[n] = pos;
  return KX_OK;
}
