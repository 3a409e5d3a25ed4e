// kx_nested.h — the nested record walker: generated FastRead / FastWriteNocopy for schemas beyond the
// flat model (list<S> / map<K, S> with strings, optional and nested fields; containers of containers;
// more than 8 var-length slots or 32 columns; string defaults; recursive structs kept as bytes).
//
// Reference semantics (tool/internal_pkg/pluginmode/thriftgo/struct_tpl.go): the field loop :41-149
// (unknown ids / wrong wire types skipped, the last occurrence of a field wins, required fields
// checked at STOP), base types :425-450, struct fields :405-422 (a fresh NewX() per occurrence),
// maps :466-533, sets :537-579, lists :583-625 (element / key / value type bytes are not validated),
// FastWriteNocopy :225-264 with the encoder order of patcher.go:503-522 (fixed-length fields first),
// and the skip decoder pkg/remote/codec/thrift/codec_apache.go:191-293 for everything skipped.
//
// Column model (include/kxcodec.h, "Nested schemas"): every container opens an element domain one
// level down; a leaf at level L has L offsets arrays (record -> D1, D1 -> D2) plus a byte-offsets
// array when it is a string. The walker keeps one cursor per domain and per string leaf: decoding a
// record advances cursors; an instance (the record, or one element of a container) writes, when it
// starts, every offsets entry of the columns below it (the cursor value at that moment), and the
// scalar defaults of its fields, which present fields then overwrite. A field seen a second time in
// the same instance rewinds the cursors of its subtree to the snapshot taken at its first occurrence
// (so only the last occurrence's elements / bytes remain: Go's `p.F = _field`).
//
// The same code runs on the device (lane = record; kx_nested.hip: a measure pass counts each record's
// cursor advances, a block scan turns them into bases, a write pass re-walks with cursors at the
// bases) and on the host (test harness), so it is plain C++ with host/device qualifiers.
#pragma once
#include <stdint.h>

#include "../../include/kxcodec.h"

#if defined(__HIPCC__)
#define KXN_HD __host__ __device__ __forceinline__
#else
#define KXN_HD static inline
#endif

#define KXN_MAX_NODES 256
#define KXN_MAX_FIELDS 192
#define KXN_MAX_STRUCTS 64
#define KXN_MAX_ROOTS 32
#define KXN_MAX_CUR 64          // = the device walker's per-lane cursor array (kx_nested.hip)
#define KXN_MAX_ENT 384
#define KXN_MAX_DFL 256
#define KXN_MAX_SDF 64
#define KXN_MAX_SNAP 128        // = the device walker's per-lane snapshot slots: a schema needing more is
                                // refused at kx_schema_create, not at its first decode
#define KXN_MAX_DEFB 4096
#define KXN_STACK 32          // walker frames (struct nesting + containers)
#define KXN_SKIP_DEPTH 64     // codec_apache.go:167

enum : uint8_t { KN_SCALAR = 1, KN_STRING = 2, KN_RAW = 3, KN_STRUCT = 4, KN_LIST = 5, KN_MAP = 6 };

struct KxnNode {        // a value position: a field's value, a container's element / key / value (24 B)
  uint8_t kind;         // KN_*
  uint8_t ttype;        // its wire type (SET stays SET)
  uint8_t width;        // scalar width
  uint8_t level;        // containers above it (0: one per record)
  int16_t col;          // SCALAR / STRING / RAW: leaf column
  int16_t cur;          // STRING / RAW: byte cursor; LIST / MAP: its element-domain cursor
  int16_t a;            // LIST: element node; MAP: key node; STRUCT: struct instance
  int16_t b;            // MAP: value node
  int16_t root;         // LIST / MAP: the instance root of its elements (entries)
  int16_t rep_col;      // LIST / MAP: a column whose array `level` counts its elements (encode)
  uint8_t etype, vtype; // LIST: element wire type; MAP: key, value wire types (encode headers)
  uint16_t cur_lo, cur_hi;  // cursors of this value's subtree
};

struct KxnField {       // 32 B
  int16_t id;
  uint8_t ttype;        // expected wire type
  uint8_t req;          // KX_REQ_*
  int16_t node;
  int16_t snap;         // snapshot slots of its subtree cursors (var fields), -1
  int8_t pbit;          // presence bit in its instance's word, -1
  uint8_t sbit;         // seen bit in its instance's mask
  int16_t enc_next;     // next field of its struct in encoder order, -1
  uint32_t def_off, def_len;  // string default bytes (P.defb)
  int64_t defv;         // scalar default
};

struct KxnStruct {      // a struct occurrence (instances are per position: columns differ) (40 B)
  int16_t first, nfields;
  int16_t enc_first;    // first field in encoder order, -1
  uint16_t dfl_lo, dfl_hi;  // scalar defaults of its inline subtree (P.dfl)
  uint8_t level;        // level of its fields
  uint8_t pad;
  int16_t root;         // its instance root
  int16_t pad2;
  uint64_t req_mask;    // seen bits of its required fields
  uint64_t sub_mask;    // seen bits of its fields and its inline structs' fields
  uint64_t pres_mask;   // presence bits inside its inline subtree
};

struct KxnRoot {        // an instance root: the record, or one element / entry of a container (16 B)
  uint8_t level;
  uint8_t pad;
  int16_t pres_col;     // level >= 1: column of its presence words, -1 (level 0: kx_columns.presence)
  int16_t dcur;         // level >= 1: the cursor of its element domain (-1 for the record)
  int16_t pad2;
  uint16_t ent_lo, ent_hi;  // offsets entries written when an instance starts (P.ent)
  uint16_t dfl_lo, dfl_hi;  // scalar defaults written when it starts (P.dfl)
  uint16_t sdf_lo, sdf_hi;  // string defaults written at its end when the field was not seen (P.sdf)
};

struct KxnEntry {       // array `arr` of column `col` at the instance index = cursor `cur` (8 B)
  int16_t col;
  uint8_t arr;
  uint8_t pad;
  int16_t cur;
  int16_t pad2;
};

struct KxnDflt {        // data(col)[e] = v (16 B)
  int16_t col;
  uint8_t width;
  uint8_t pad[5];
  int64_t v;
};

struct KxnSdef {        // string default of field `field` (16 B)
  int16_t col;
  int16_t cur;
  uint8_t sbit;
  uint8_t pad[3];
  uint32_t off, len;
};

struct KxnCol {         // per column (16 B)
  uint8_t kind;         // KX_COL_*
  uint8_t width;        // value width (strings: 1)
  uint8_t level;
  uint8_t narr;         // offsets arrays: level (+1 for strings)
  int16_t acur[3];      // cursor whose values array k stores
  int16_t dcur;         // cursor counting its data units (-1: one value per record)
  uint8_t elem;         // value wire type (BOOL normalisation)
  uint8_t pad[5];
};

struct KxnProgram {
  uint32_t nnodes, nfields, nstructs, nroots, ncur, nent, ndfl, nsdf, nsnap, ncols, npres, ndefb;
  int16_t rec_node;     // the record's STRUCT node
  int16_t pad[3];
  KxnNode node[KXN_MAX_NODES];
  KxnField f[KXN_MAX_FIELDS];
  KxnStruct st[KXN_MAX_STRUCTS];
  KxnRoot root[KXN_MAX_ROOTS];
  KxnEntry ent[KXN_MAX_ENT];
  KxnDflt dfl[KXN_MAX_DFL];
  KxnSdef sdf[KXN_MAX_SDF];
  KxnCol col[KX_MAX_COLUMNS];
  uint8_t defb[KXN_MAX_DEFB];
};

// the column buffers of one call (device memory, uploaded per call)
struct KxnCols {
  void* data[KX_MAX_COLUMNS];
  void* arr[KX_MAX_COLUMNS][3];   // offsets, elem_offsets, sub_offsets
  uint64_t cap[KX_MAX_COLUMNS][4];  // units of data, arr0 (n), arr1, arr2 (entries - 1)
  uint64_t owide;                 // bit c: 8-byte offsets
  uint64_t* presence;
};

// ---------------------------------------------------------------------------------------------
// byte reads (big-endian wire)
KXN_HD uint32_t kxn_be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
KXN_HD uint32_t kxn_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
KXN_HD uint64_t kxn_be64(const uint8_t* p) { return ((uint64_t)kxn_be32(p) << 32) | kxn_be32(p + 4); }

KXN_HD int kxn_tsize(uint32_t t) {
  switch (t) {
    case KX_T_BOOL: case KX_T_BYTE: return 1;
    case KX_T_I16: return 2;
    case KX_T_I32: return 4;
    case KX_T_I64: case KX_T_DOUBLE: return 8;
    default: return 0;
  }
}

// ---------------------------------------------------------------------------------------------
// Skip decoder (codec_apache.go:191-293), iterative: a frame per open struct / list / map
struct KxnSkipFrame {
  uint8_t kind;   // 1 struct, 2 list, 3 map
  uint8_t et, kt, phase;
  int32_t depth;  // the maxdepth the container was visited with
  int64_t rem;
};

// visit one value of type t with depth d at b[*n]: skip it or push its frame
KXN_HD int kxn_skip_visit(const uint8_t* b, uint64_t len, uint64_t* n, uint32_t t, int d, KxnSkipFrame* st,
                          int* sp) {
  if (d == 0) return KX_ERR_DEPTH_LIMIT;                     // :192-194
  const int sz = kxn_tsize(t);
  if (sz > 0) {                                              // :195-197
    if (*n + (uint64_t)sz > len) return KX_ERR_EOF;
    *n += (uint64_t)sz;
    return KX_OK;
  }
  switch (t) {
    case KX_T_STRING: {                                      // :199-209
      if (*n + 4 > len) return KX_ERR_EOF;
      const int32_t l = (int32_t)kxn_be32(b + *n);
      *n += 4;
      if (l < 0) return KX_ERR_INVALID_DATA;
      if (*n + (uint64_t)l > len) return KX_ERR_EOF;
      *n += (uint64_t)l;
      return KX_OK;
    }
    case KX_T_STRUCT:                                        // :210-234
      st[*sp] = KxnSkipFrame{1, 0, 0, 0, d, 0};
      (*sp)++;
      return KX_OK;
    case KX_T_MAP: {                                         // :235-268
      if (*n + 6 > len) return KX_ERR_EOF;
      const uint32_t kt = b[*n], vt = b[*n + 1];
      const int32_t c = (int32_t)kxn_be32(b + *n + 2);
      *n += 6;
      if (c < 0) return KX_ERR_INVALID_DATA;
      const int ks = kxn_tsize(kt), vs = kxn_tsize(vt);
      if (ks > 0 && vs > 0) {
        const uint64_t k = (uint64_t)c * (uint64_t)(ks + vs);
        if (*n + k > len) return KX_ERR_EOF;
        *n += k;
        return KX_OK;
      }
      st[*sp] = KxnSkipFrame{3, (uint8_t)vt, (uint8_t)kt, 0, d, (int64_t)c};
      (*sp)++;
      return KX_OK;
    }
    case KX_T_SET: case KX_T_LIST: {                         // :269-286
      if (*n + 5 > len) return KX_ERR_EOF;
      const uint32_t vt = b[*n];
      const int32_t c = (int32_t)kxn_be32(b + *n + 1);
      *n += 5;
      if (c < 0) return KX_ERR_INVALID_DATA;
      const int vs = kxn_tsize(vt);
      if (vs > 0) {
        const uint64_t k = (uint64_t)c * (uint64_t)vs;
        if (*n + k > len) return KX_ERR_EOF;
        *n += k;
        return KX_OK;
      }
      st[*sp] = KxnSkipFrame{2, (uint8_t)vt, 0, 0, d, (int64_t)c};
      (*sp)++;
      return KX_OK;
    }
    default:                                                 // :287-290 unknown data type
      return KX_ERR_INVALID_DATA;
  }
}

// skip one value of wire type t at b[*n] (len: the readable extent)
KXN_HD int kxn_skip(const uint8_t* b, uint64_t len, uint64_t* n, uint32_t t, int maxdepth) {
  KxnSkipFrame st[KXN_SKIP_DEPTH + 1];
  int sp = 0;
  int rc = kxn_skip_visit(b, len, n, t, maxdepth, st, &sp);
  while (!rc && sp > 0) {
    KxnSkipFrame& F = st[sp - 1];
    if (F.kind == 1) {
      if (*n + 1 > len) return KX_ERR_EOF;
      const uint32_t tp = b[*n];
      *n += 1;
      if (tp == KX_T_STOP) { sp--; continue; }
      const int fsz = kxn_tsize(tp);
      if (fsz > 0) {
        if (*n + 2 + (uint64_t)fsz > len) return KX_ERR_EOF;
        *n += 2 + (uint64_t)fsz;
        continue;
      }
      if (*n + 2 > len) return KX_ERR_EOF;
      *n += 2;
      rc = kxn_skip_visit(b, len, n, tp, F.depth - 1, st, &sp);
    } else if (F.kind == 2) {
      if (F.rem == 0) { sp--; continue; }
      F.rem--;
      rc = kxn_skip_visit(b, len, n, F.et, F.depth - 1, st, &sp);
    } else {
      if (F.rem == 0) { sp--; continue; }
      const int d = F.depth - 1;
      if (F.phase == 0) {
        F.phase = 1;
        const int ks = kxn_tsize(F.kt);
        if (ks > 0) {
          if (*n + (uint64_t)ks > len) return KX_ERR_EOF;
          *n += (uint64_t)ks;
        } else {
          rc = kxn_skip_visit(b, len, n, F.kt, d, st, &sp);
        }
      } else {
        F.phase = 0;
        F.rem--;
        const uint32_t vt = F.et;
        const int vs = kxn_tsize(vt);
        if (vs > 0) {
          if (*n + (uint64_t)vs > len) return KX_ERR_EOF;
          *n += (uint64_t)vs;
        } else {
          rc = kxn_skip_visit(b, len, n, vt, d, st, &sp);
        }
      }
    }
  }
  return rc;
}

// ---------------------------------------------------------------------------------------------
// column stores
KXN_HD void kxn_put_arr(const KxnCols& C, int c, int k, uint64_t i, uint64_t v) {
  if ((C.owide >> c) & 1) ((uint64_t*)C.arr[c][k])[i] = v;
  else ((uint32_t*)C.arr[c][k])[i] = (uint32_t)v;
}
KXN_HD uint64_t kxn_get_arr(const KxnCols& C, int c, int k, uint64_t i) {
  return ((C.owide >> c) & 1) ? ((const uint64_t*)C.arr[c][k])[i] : (uint64_t)((const uint32_t*)C.arr[c][k])[i];
}
KXN_HD void kxn_put_val(const KxnCols& C, int c, uint32_t w, uint64_t i, uint64_t v) {
  switch (w) {
    case 1: ((uint8_t*)C.data[c])[i] = (uint8_t)v; break;
    case 2: ((uint16_t*)C.data[c])[i] = (uint16_t)v; break;
    case 4: ((uint32_t*)C.data[c])[i] = (uint32_t)v; break;
    default: ((uint64_t*)C.data[c])[i] = v; break;
  }
}
KXN_HD uint64_t kxn_get_val(const KxnCols& C, int c, uint32_t w, uint64_t i) {
  switch (w) {
    case 1: return ((const uint8_t*)C.data[c])[i];
    case 2: return ((const uint16_t*)C.data[c])[i];
    case 4: return ((const uint32_t*)C.data[c])[i];
    default: return ((const uint64_t*)C.data[c])[i];
  }
}

KXN_HD uint64_t kxn_scalar(uint32_t t, const uint8_t* p) {  // host order; BOOL is `b == 1` (parity unpinned)
  switch (t) {
    case KX_T_BOOL: return p[0] == 1;
    case KX_T_BYTE: return p[0];
    case KX_T_I16: return kxn_be16(p);
    case KX_T_I32: return kxn_be32(p);
    default: return kxn_be64(p);
  }
}

// ---------------------------------------------------------------------------------------------
// decode walker
struct KxnFrame {
  uint8_t kind;     // KN_STRUCT / KN_LIST / KN_MAP
  uint8_t open;     // LIST / MAP: an element instance is open
  uint8_t phase;    // MAP: 0 key next, 1 value next
  uint8_t pad;
  int16_t id;       // STRUCT: struct instance; LIST / MAP: container node
  int16_t pad2;
  int64_t rem;      // LIST / MAP: elements left
};

// Writes are clipped to the record's own extent of every cursor ([base, lim) from the measure pass):
// an occurrence that a later one of the same field replaces may have been longer, and what it wrote
// past the record's final extent belongs to the next record (another lane). Inside the extent every
// byte / element is written again by a later, final occurrence.
struct KxnState {
  uint64_t idx[3];    // index of the open instance per level
  uint64_t seen[3];   // seen masks per level
  uint64_t pres[3];   // presence words per level
  bool live[3];       // the open instance lies inside the record's extent of its domain (writes allowed)
  const uint64_t* lim;  // W: per cursor, the end of the record's extent
};

// an instance of root R at index e starts: offsets entries, scalar defaults
template <bool W>
KXN_HD void kxn_inst_start(const KxnProgram& P, const KxnCols& C, int R, uint64_t e, const uint64_t* cur,
                           KxnState& S) {
  const KxnRoot& RT = P.root[R];
  S.idx[RT.level] = e;
  S.seen[RT.level] = 0;
  S.pres[RT.level] = 0;
  if (!W) return;
  S.live[RT.level] = RT.level == 0 || e < S.lim[RT.dcur];
  if (!S.live[RT.level]) return;
  for (int k = RT.ent_lo; k < RT.ent_hi; k++) {
    const KxnEntry& E = P.ent[k];
    kxn_put_arr(C, E.col, E.arr, e, cur[E.cur]);
  }
  for (int k = RT.dfl_lo; k < RT.dfl_hi; k++) kxn_put_val(C, P.dfl[k].col, P.dfl[k].width, e, (uint64_t)P.dfl[k].v);
}

// the instance ends: absent string fields take their defaults, the presence word is stored
template <bool W>
KXN_HD void kxn_inst_end(const KxnProgram& P, const KxnCols& C, int R, uint64_t* cur, KxnState& S) {
  const KxnRoot& RT = P.root[R];
  const int L = RT.level;
  for (int k = RT.sdf_lo; k < RT.sdf_hi; k++) {
    const KxnSdef& D = P.sdf[k];
    if ((S.seen[L] >> D.sbit) & 1) continue;
    if (W)
      for (uint32_t j = 0; j < D.len; j++)
        if (cur[D.cur] + j < S.lim[D.cur]) ((uint8_t*)C.data[D.col])[cur[D.cur] + j] = P.defb[D.off + j];
    cur[D.cur] += D.len;
  }
  if (!W || !S.live[L]) return;
  if (L == 0) {
    if (C.presence) C.presence[S.idx[0]] = S.pres[0];
  } else if (RT.pres_col >= 0) {
    ((uint64_t*)C.data[RT.pres_col])[S.idx[L]] = S.pres[L];
  }
}

// read one value of node X at b[*q] (scalars, strings, raw structs directly; structs / containers push a
// frame). Element instances of containers are opened by the caller.
template <bool W>
KXN_HD int kxn_value(const KxnProgram& P, const KxnCols& C, const uint8_t* b, uint64_t len, uint64_t* q, int X,
                     uint64_t* cur, KxnState& S, KxnFrame* stk, int* sp) {
  const KxnNode& N = P.node[X];
  switch (N.kind) {
    case KN_SCALAR: {
      if (*q + N.width > len) return KX_ERR_EOF;
      if (W && S.live[N.level]) kxn_put_val(C, N.col, N.width, S.idx[N.level], kxn_scalar(N.ttype, b + *q));
      *q += N.width;
      return KX_OK;
    }
    case KN_STRING: {                                        // ReadString: a copy
      if (*q + 4 > len) return KX_ERR_EOF;
      const int32_t l = (int32_t)kxn_be32(b + *q);
      if (l < 0) return KX_ERR_NEGATIVE_SIZE;
      if (*q + 4 + (uint64_t)l > len) return KX_ERR_EOF;
      if (W) {
        uint8_t* dst = (uint8_t*)C.data[N.col] + cur[N.cur];
        const uint64_t room = S.lim[N.cur] > cur[N.cur] ? S.lim[N.cur] - cur[N.cur] : 0;
        const uint64_t m = (uint64_t)l < room ? (uint64_t)l : room;
        for (uint64_t j = 0; j < m; j++) dst[j] = b[*q + 4 + j];
      }
      cur[N.cur] += (uint64_t)l;
      *q += 4 + (uint64_t)l;
      return KX_OK;
    }
    case KN_RAW: {                                           // a recursive struct: its encoded bytes
      uint64_t e = *q;
      const int rc = kxn_skip(b, len, &e, KX_T_STRUCT, KXN_SKIP_DEPTH);
      if (rc) return rc;
      if (W) {
        uint8_t* dst = (uint8_t*)C.data[N.col] + cur[N.cur];
        const uint64_t room = S.lim[N.cur] > cur[N.cur] ? S.lim[N.cur] - cur[N.cur] : 0;
        const uint64_t m = e - *q < room ? e - *q : room;
        for (uint64_t j = 0; j < m; j++) dst[j] = b[*q + j];
      }
      cur[N.cur] += e - *q;
      *q = e;
      return KX_OK;
    }
    case KN_STRUCT:
      if (*sp >= KXN_STACK) return KX_ERR_DEPTH_LIMIT;
      stk[*sp] = KxnFrame{KN_STRUCT, 0, 0, 0, N.a, 0, 0};
      (*sp)++;
      return KX_OK;
    case KN_LIST: {                                          // ReadListBegin / ReadSetBegin (:537-625)
      if (*q + 5 > len) return KX_ERR_EOF;
      const int32_t c = (int32_t)kxn_be32(b + *q + 1);
      if (c < 0) return KX_ERR_NEGATIVE_SIZE;
      *q += 5;
      if (*sp >= KXN_STACK) return KX_ERR_DEPTH_LIMIT;
      stk[*sp] = KxnFrame{KN_LIST, 0, 0, 0, (int16_t)X, 0, (int64_t)c};
      (*sp)++;
      return KX_OK;
    }
    default: {                                               // ReadMapBegin (:466-533)
      if (*q + 6 > len) return KX_ERR_EOF;
      const int32_t c = (int32_t)kxn_be32(b + *q + 2);
      if (c < 0) return KX_ERR_NEGATIVE_SIZE;
      *q += 6;
      if (*sp >= KXN_STACK) return KX_ERR_DEPTH_LIMIT;
      stk[*sp] = KxnFrame{KN_MAP, 0, 0, 0, (int16_t)X, 0, (int64_t)c};
      (*sp)++;
      return KX_OK;
    }
  }
}

// FastRead of record r = b[0 .. len). cur: cursors (measure: from 0, write: at the record's bases);
// lim (write): the ends of the record's extents; snap: KXN_MAX_SNAP slots. *used = bytes of the struct.
template <bool W>
KXN_HD int kxn_read_record(const KxnProgram& P, const KxnCols& C, const uint8_t* b, uint64_t len, uint64_t r,
                           uint64_t* cur, uint64_t* snap, uint64_t* used, const uint64_t* lim = nullptr) {
  KxnFrame stk[KXN_STACK];
  KxnState S;
  S.lim = lim;
  S.live[0] = S.live[1] = S.live[2] = true;
  S.idx[0] = S.idx[1] = S.idx[2] = 0;
  S.seen[0] = S.seen[1] = S.seen[2] = 0;
  S.pres[0] = S.pres[1] = S.pres[2] = 0;
  int sp = 0;
  uint64_t q = 0;
  kxn_inst_start<W>(P, C, 0, r, cur, S);
  int rc = kxn_value<W>(P, C, b, len, &q, P.rec_node, cur, S, stk, &sp);
  while (!rc && sp > 0) {
    KxnFrame& F = stk[sp - 1];
    if (F.kind == KN_STRUCT) {
      const KxnStruct& T = P.st[F.id];
      if (q + 1 > len) { rc = KX_ERR_EOF; break; }             // ReadFieldBegin
      const uint32_t t = b[q];
      const int L = T.level;
      if (t == KX_T_STOP) {
        q += 1;
        if ((S.seen[L] & T.req_mask) != T.req_mask) { rc = KX_ERR_INVALID_DATA; break; }  // :124-145
        sp--;
        continue;
      }
      if (q + 3 > len) { rc = KX_ERR_EOF; break; }
      const int16_t id = (int16_t)kxn_be16(b + q + 1);
      q += 3;
      int fi = -1;
      for (int k = 0; k < T.nfields; k++)
        if (P.f[T.first + k].id == id) { fi = T.first + k; break; }
      if (fi < 0 || P.f[fi].ttype != t) {                       // default: / mismatched type -> Skip
        rc = kxn_skip(b, len, &q, t, KXN_SKIP_DEPTH);
        continue;
      }
      const KxnField& G = P.f[fi];
      const KxnNode& N = P.node[G.node];
      const uint64_t bit = 1ull << G.sbit;
      if (G.snap >= 0) {
        if (S.seen[L] & bit) {                                  // repeated: keep only this occurrence
          for (int k = N.cur_lo; k < N.cur_hi; k++) cur[k] = snap[G.snap + k - N.cur_lo];
          if (N.kind == KN_STRUCT) {                            // a fresh NewX()
            const KxnStruct& U = P.st[N.a];
            if (W && S.live[L])
              for (int k = U.dfl_lo; k < U.dfl_hi; k++)
                kxn_put_val(C, P.dfl[k].col, P.dfl[k].width, S.idx[L], (uint64_t)P.dfl[k].v);
            S.seen[L] &= ~U.sub_mask;
            S.pres[L] &= ~U.pres_mask;
          }
        } else {
          for (int k = N.cur_lo; k < N.cur_hi; k++) snap[G.snap + k - N.cur_lo] = cur[k];
        }
      } else if (N.kind == KN_STRUCT && (S.seen[L] & bit)) {  // repeated struct without var fields
        const KxnStruct& U = P.st[N.a];
        if (W && S.live[L])
          for (int k = U.dfl_lo; k < U.dfl_hi; k++)
            kxn_put_val(C, P.dfl[k].col, P.dfl[k].width, S.idx[L], (uint64_t)P.dfl[k].v);
        S.seen[L] &= ~U.sub_mask;
        S.pres[L] &= ~U.pres_mask;
      }
      S.seen[L] |= bit;
      if (G.pbit >= 0) S.pres[L] |= 1ull << G.pbit;
      rc = kxn_value<W>(P, C, b, len, &q, G.node, cur, S, stk, &sp);
      continue;
    }
    // LIST / MAP: close the open element, then open the next one
    const KxnNode& N = P.node[F.id];
    if (F.open && (N.kind == KN_LIST || F.phase == 0)) {
      kxn_inst_end<W>(P, C, N.root, cur, S);
      F.open = 0;
    }
    if (N.kind == KN_LIST) {
      if (F.rem == 0) { sp--; continue; }
      F.rem--;
      const uint64_t e = cur[N.cur]++;
      kxn_inst_start<W>(P, C, N.root, e, cur, S);
      F.open = 1;
      rc = kxn_value<W>(P, C, b, len, &q, N.a, cur, S, stk, &sp);
    } else if (F.phase == 0) {
      if (F.rem == 0) { sp--; continue; }
      F.rem--;
      const uint64_t e = cur[N.cur]++;
      kxn_inst_start<W>(P, C, N.root, e, cur, S);
      F.open = 1;
      F.phase = 1;
      rc = kxn_value<W>(P, C, b, len, &q, N.a, cur, S, stk, &sp);
    } else {
      F.phase = 0;
      rc = kxn_value<W>(P, C, b, len, &q, N.b, cur, S, stk, &sp);
    }
  }
  if (rc) return rc;
  kxn_inst_end<W>(P, C, 0, cur, S);
  *used = q;
  return KX_OK;
}

// the instance of record r of a record that failed: defaults, empty extents, presence 0
KXN_HD void kxn_failed_record(const KxnProgram& P, const KxnCols& C, uint64_t r, const uint64_t* cur) {
  const KxnRoot& RT = P.root[0];
  for (int k = RT.ent_lo; k < RT.ent_hi; k++) kxn_put_arr(C, P.ent[k].col, P.ent[k].arr, r, cur[P.ent[k].cur]);
  for (int k = RT.dfl_lo; k < RT.dfl_hi; k++) kxn_put_val(C, P.dfl[k].col, P.dfl[k].width, r, (uint64_t)P.dfl[k].v);
  if (C.presence) C.presence[r] = 0;
}

// ---------------------------------------------------------------------------------------------
// encode walker: FastWriteNocopy of record r from the columns (W: write to out + pos, else size only)
struct KxnEFrame {
  uint8_t kind;   // KN_STRUCT (next field f), KN_LIST / KN_MAP (next element i < end)
  uint8_t phase;  // MAP: 0 key next, 1 value next
  int16_t id;     // STRUCT: struct; LIST / MAP: node
  int16_t f;      // STRUCT: next field in encoder order
  int16_t root;   // STRUCT: its instance root (presence word)
  uint64_t i, end;  // LIST / MAP: element index range
  uint64_t e;       // STRUCT: its instance index
};

template <bool W>
KXN_HD void kxn_out(uint8_t* out, uint64_t* pos, uint64_t v, int nbytes) {  // big-endian
  if (W)
    for (int k = 0; k < nbytes; k++) out[*pos + k] = (uint8_t)(v >> (8 * (nbytes - 1 - k)));
  *pos += (uint64_t)nbytes;
}

KXN_HD uint64_t kxn_pres_word(const KxnProgram& P, const KxnCols& C, int R, uint64_t e) {
  const KxnRoot& RT = P.root[R];
  if (RT.level == 0) return C.presence ? C.presence[e] : 0;
  return RT.pres_col >= 0 ? ((const uint64_t*)C.data[RT.pres_col])[e] : 0;
}

// one value of node X at instance index e (level X.level); structs / containers push a frame
template <bool W>
KXN_HD void kxn_wvalue(const KxnProgram& P, const KxnCols& C, int X, uint64_t e, uint8_t* out, uint64_t* pos,
                       KxnEFrame* stk, int* sp) {
  const KxnNode& N = P.node[X];
  switch (N.kind) {
    case KN_SCALAR: {
      uint64_t v = kxn_get_val(C, N.col, N.width, e);
      if (N.ttype == KX_T_BOOL) v = (v & 0xff) ? 1 : 0;
      kxn_out<W>(out, pos, v, N.width);
      return;
    }
    case KN_STRING: case KN_RAW: {
      const uint64_t a = kxn_get_arr(C, N.col, N.level, e), z = kxn_get_arr(C, N.col, N.level, e + 1);
      const uint64_t l = z - a;
      if (N.kind == KN_STRING) kxn_out<W>(out, pos, l, 4);
      else if (l == 0) { kxn_out<W>(out, pos, KX_T_STOP, 1); return; }  // an empty raw struct: STOP
      if (W)
        for (uint64_t j = 0; j < l; j++) out[*pos + j] = ((const uint8_t*)C.data[N.col])[a + j];
      *pos += l;
      return;
    }
    case KN_STRUCT:
      stk[*sp] = KxnEFrame{KN_STRUCT, 0, N.a, P.st[N.a].enc_first, P.st[N.a].root, 0, 0, e};
      (*sp)++;
      return;
    default: {
      const uint64_t a = kxn_get_arr(C, N.rep_col, N.level, e), z = kxn_get_arr(C, N.rep_col, N.level, e + 1);
      if (N.kind == KN_LIST) {
        kxn_out<W>(out, pos, N.etype, 1);
      } else {
        kxn_out<W>(out, pos, N.etype, 1);
        kxn_out<W>(out, pos, N.vtype, 1);
      }
      kxn_out<W>(out, pos, z - a, 4);
      stk[*sp] = KxnEFrame{N.kind, 0, (int16_t)X, 0, 0, a, z, 0};
      (*sp)++;
      return;
    }
  }
}

template <bool W>
KXN_HD uint64_t kxn_write_record(const KxnProgram& P, const KxnCols& C, uint64_t r, uint8_t* out, uint64_t pos0) {
  KxnEFrame stk[KXN_STACK];
  int sp = 0;
  uint64_t pos = pos0;
  kxn_wvalue<W>(P, C, P.rec_node, r, out, &pos, stk, &sp);
  while (sp > 0) {
    KxnEFrame& F = stk[sp - 1];
    if (F.kind == KN_STRUCT) {
      if (F.f < 0) {
        kxn_out<W>(out, &pos, KX_T_STOP, 1);
        sp--;
        continue;
      }
      const KxnField& G = P.f[F.f];
      F.f = G.enc_next;
      const KxnNode& N = P.node[G.node];
      uint64_t pres = 0;
      if (G.pbit >= 0) {
        pres = kxn_pres_word(P, C, F.root, F.e);
        if (G.req == KX_REQ_OPTIONAL && !((pres >> G.pbit) & 1)) continue;  // optional: only when set
      }
      kxn_out<W>(out, &pos, ((uint64_t)G.ttype << 16) | (uint16_t)G.id, 3);  // WriteFieldBegin
      if (N.kind == KN_STRUCT && G.pbit >= 0 && !((pres >> G.pbit) & 1)) {
        kxn_out<W>(out, &pos, KX_T_STOP, 1);                    // nil *T -> STOP only (k-mock.go:190-199)
        continue;
      }
      kxn_wvalue<W>(P, C, G.node, F.e, out, &pos, stk, &sp);
      continue;
    }
    const KxnNode& N = P.node[F.id];
    if (F.i >= F.end) { sp--; continue; }
    const uint64_t e = F.i;
    if (N.kind == KN_LIST) {
      F.i++;
      kxn_wvalue<W>(P, C, N.a, e, out, &pos, stk, &sp);
    } else if (F.phase == 0) {
      F.phase = 1;
      kxn_wvalue<W>(P, C, N.a, e, out, &pos, stk, &sp);
    } else {
      F.phase = 0;
      F.i++;
      kxn_wvalue<W>(P, C, N.b, e, out, &pos, stk, &sp);
    }
  }
  return pos - pos0;
}
