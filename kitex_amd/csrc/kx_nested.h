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
#define KXN_MHD __host__ __device__ __forceinline__   // member functions
#else
#define KXN_HD static inline
#define KXN_MHD inline
#endif
// global memory through address-space-1 pointers on the device pass (column arrays, the input and the
// output are all global): the column pointers come out of the KxnCols struct in device memory, which the
// compiler cannot prove global, and flat accesses also count on the LDS counter (kx_mem.h)
#if defined(__HIP_DEVICE_COMPILE__)
#define KXN_G(T) __attribute__((address_space(1))) T
#else
#define KXN_G(T) T
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
#define KXN_FMAP 32           // field ids 0 .. 31: direct lookup per struct (KxnProgram.fmap)
// A walk without snapshots (snap == nullptr: the common, canonical record) met a field a second time in one
// instance: the record needs the careful walk (snapshots, and in the write pass clipping at the record's
// extents). Internal to the walker's callers, never a status code.
#define KXN_REPEAT 0x7e

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
  uint8_t pbk;          // Kitex-Protobuf: proto scalar kind (KX_PB_*) of a SCALAR / STRING value
  uint8_t pad;
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
  int16_t pb;           // a Kitex-Protobuf schema: proto3 wire format (kxn_pb_*), field-number encoder order
  int16_t pad[2];
  KxnNode node[KXN_MAX_NODES];
  KxnField f[KXN_MAX_FIELDS];
  KxnStruct st[KXN_MAX_STRUCTS];
  KxnRoot root[KXN_MAX_ROOTS];
  KxnEntry ent[KXN_MAX_ENT];
  KxnDflt dfl[KXN_MAX_DFL];
  KxnSdef sdf[KXN_MAX_SDF];
  KxnCol col[KX_MAX_COLUMNS];
  uint8_t defb[KXN_MAX_DEFB];
  uint8_t fmap[KXN_MAX_STRUCTS][KXN_FMAP];   // struct s, field id i < KXN_FMAP: its field's index - st[s].first, 0xff none
};

// the field of struct T (index si) with id `id`, or -1: one table read for ids below KXN_FMAP, else a scan
KXN_HD int kxn_field(const KxnProgram& P, int si, const KxnStruct& T, int64_t id) {
  if (id >= 0 && id < KXN_FMAP) {
    const uint32_t m = P.fmap[si][id];
    return m == 0xff ? -1 : T.first + (int)m;
  }
  for (int k = 0; k < T.nfields; k++)
    if (P.f[T.first + k].id == id) return T.first + k;
  return -1;
}

// the column buffers of one call (device memory, uploaded per call)
struct KxnCols {
  void* data[KX_MAX_COLUMNS];
  void* arr[KX_MAX_COLUMNS][3];   // offsets, elem_offsets, sub_offsets
  uint64_t owide;                 // bit c: 8-byte offsets
  uint64_t* presence;
  uint64_t cap[KX_MAX_COLUMNS][4];  // units of data, arr0 (n), arr1, arr2 (entries - 1): the capacity check only
};
// the part of KxnCols the walkers read (everything before cap): the decode write pass keeps this much in LDS
constexpr unsigned KXN_COLS_HEAD = (unsigned)__builtin_offsetof(KxnCols, cap);

// The walker's cursors, behind a small interface so that they can live where the caller wants them: a
// plain array here (the host harness, the device's scratch fallback); on the device a per-lane column of
// the workgroup's LDS (kx_nested.hip KxnCurL), which keeps them out of scratch.
struct KxnCurP {
  uint64_t* p;
  KXN_MHD uint64_t operator[](int k) const { return p[k]; }
  KXN_MHD void set(int k, uint64_t v) const { p[k] = v; }
  KXN_MHD void add(int k, uint64_t d) const { p[k] += d; }
  KXN_MHD uint64_t post_inc(int k) const { return p[k]++; }
};

// ---------------------------------------------------------------------------------------------
// byte reads (big-endian wire)
template <class B>
KXN_HD uint32_t kxn_be16(B p) { return ((uint32_t)p[0] << 8) | p[1]; }
template <class B>
KXN_HD uint32_t kxn_be32(B p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
template <class B>
KXN_HD uint64_t kxn_be64(B p) { return ((uint64_t)kxn_be32(p) << 32) | kxn_be32(p + 4); }
// the input itself: one unaligned load per value (global_load_dword / dwordx2 at any byte address on the
// device) instead of a load per byte, which left every lane's walk a chain of byte round trips
KXN_HD uint32_t kxn_be16(const uint8_t* p) {
  uint16_t x;
  __builtin_memcpy(&x, p, 2);
  return (uint32_t)(uint16_t)((x << 8) | (x >> 8));
}
KXN_HD uint32_t kxn_be32(const uint8_t* p) {
  uint32_t x;
  __builtin_memcpy(&x, p, 4);
  return __builtin_bswap32(x);
}
KXN_HD uint64_t kxn_be64(const uint8_t* p) {
  uint64_t x;
  __builtin_memcpy(&x, p, 8);
  return __builtin_bswap64(x);
}

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
template <class B>
KXN_HD int kxn_skip_visit(B b, uint64_t len, uint64_t* n, uint32_t t, int d, KxnSkipFrame* st,
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
template <class B>
KXN_HD int kxn_skip(B b, uint64_t len, uint64_t* n, uint32_t t, int maxdepth) {
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
  if ((C.owide >> c) & 1) ((KXN_G(uint64_t)*)C.arr[c][k])[i] = v;
  else ((KXN_G(uint32_t)*)C.arr[c][k])[i] = (uint32_t)v;
}
KXN_HD uint64_t kxn_get_arr(const KxnCols& C, int c, int k, uint64_t i) {
  return ((C.owide >> c) & 1) ? ((const KXN_G(uint64_t)*)C.arr[c][k])[i] : (uint64_t)((const KXN_G(uint32_t)*)C.arr[c][k])[i];
}
KXN_HD void kxn_put_val(const KxnCols& C, int c, uint32_t w, uint64_t i, uint64_t v) {
  switch (w) {
    case 1: ((KXN_G(uint8_t)*)C.data[c])[i] = (uint8_t)v; break;
    case 2: ((KXN_G(uint16_t)*)C.data[c])[i] = (uint16_t)v; break;
    case 4: ((KXN_G(uint32_t)*)C.data[c])[i] = (uint32_t)v; break;
    default: ((KXN_G(uint64_t)*)C.data[c])[i] = v; break;
  }
}
KXN_HD uint64_t kxn_get_val(const KxnCols& C, int c, uint32_t w, uint64_t i) {
  switch (w) {
    case 1: return ((const KXN_G(uint8_t)*)C.data[c])[i];
    case 2: return ((const KXN_G(uint16_t)*)C.data[c])[i];
    case 4: return ((const KXN_G(uint32_t)*)C.data[c])[i];
    default: return ((const KXN_G(uint64_t)*)C.data[c])[i];
  }
}

template <class B>
KXN_HD uint64_t kxn_scalar(uint32_t t, B p) {  // host order; BOOL is `b == 1` (parity unpinned)
  switch (t) {
    case KX_T_BOOL: return p[0] == 1;
    case KX_T_BYTE: return p[0];
    case KX_T_I16: return kxn_be16(p);
    case KX_T_I32: return kxn_be32(p);
    default: return kxn_be64(p);
  }
}
// the same from the value's first 8 bytes in a register (little-endian load of the big-endian value)
KXN_HD uint64_t kxn_scalar_pre(uint32_t t, uint64_t lo) {
  switch (t) {
    case KX_T_BOOL: return (lo & 0xff) == 1;
    case KX_T_BYTE: return lo & 0xff;
    case KX_T_I16: return (uint32_t)__builtin_bswap16((uint16_t)lo);
    case KX_T_I32: return __builtin_bswap32((uint32_t)lo);
    default: return __builtin_bswap64(lo);
  }
}

// byte copy in blocks of 16: a block's loads are all issued before its stores (the compiler may not
// reorder them itself: source and destination could alias), so a lane waits once per 16 bytes rather
// than once per byte
template <class S>
KXN_HD uint8_t kxn_ld8(S s, uint64_t i) { return s[i]; }
KXN_HD uint8_t kxn_ld8(const uint8_t* s, uint64_t i) { return ((const KXN_G(uint8_t)*)s)[i]; }

template <class S>
KXN_HD void kxn_copy(uint8_t* dst_, S src, uint64_t m) {
  KXN_G(uint8_t)* dst = (KXN_G(uint8_t)*)dst_;
  uint64_t j = 0;
  for (; j + 16 <= m; j += 16) {
    uint8_t t[16];
#pragma unroll
    for (int k = 0; k < 16; k++) t[k] = kxn_ld8(src, j + k);
#pragma unroll
    for (int k = 0; k < 16; k++) dst[j + k] = t[k];
  }
  for (; j < m; j++) dst[j] = kxn_ld8(src, j);
}
// from the input: 16-byte unaligned loads and stores
KXN_HD void kxn_copy(uint8_t* dst, const uint8_t* src, uint64_t m) {
  uint64_t j = 0;
  for (; j + 16 <= m; j += 16) {
    uint64_t t[2];
    __builtin_memcpy(t, src + j, 16);
    __builtin_memcpy(dst + j, t, 16);
  }
  for (; j < m; j++) ((KXN_G(uint8_t)*)dst)[j] = ((const KXN_G(uint8_t)*)src)[j];
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
// A value per container level (0 .. 2) as three named members, read and written with selects: an array
// indexed by the level a program node names would live in scratch (device), one memory round trip per use
template <class T>
struct KxnL3 {
  T v0, v1, v2;
  struct Ref {
    KxnL3* s;
    int L;
    KXN_MHD operator T() const { return s->get(L); }
    KXN_MHD Ref& operator=(T x) { s->put(L, x); return *this; }
    KXN_MHD Ref& operator|=(T x) { s->put(L, s->get(L) | x); return *this; }
    KXN_MHD Ref& operator&=(T x) { s->put(L, s->get(L) & x); return *this; }
  };
  KXN_MHD T get(int L) const { return L == 0 ? v0 : L == 1 ? v1 : v2; }
  KXN_MHD void put(int L, T x) {
    v0 = L == 0 ? x : v0;
    v1 = L == 1 ? x : v1;
    v2 = L == 2 ? x : v2;
  }
  KXN_MHD void fill(T x) { v0 = v1 = v2 = x; }
  KXN_MHD Ref operator[](int L) { return Ref{this, L}; }
};

struct KxnState {
  KxnL3<uint64_t> idx;   // index of the open instance per level
  KxnL3<uint64_t> seen;  // seen masks per level
  KxnL3<uint64_t> pres;  // presence words per level
  KxnL3<bool> live;      // the open instance lies inside the record's extent of its domain (writes allowed)
  const uint64_t* lim;  // W, careful walk: per cursor, the end of the record's extent (nullptr: the walk
                        // has no repeated field, so it never leaves the extents the measure pass found)
};

// units of cursor k a write at cursor value c may fill (all of n without clipping)
KXN_HD uint64_t kxn_room(const KxnState& S, int k, uint64_t c, uint64_t n) {
  if (!S.lim) return n;
  const uint64_t room = S.lim[k] > c ? S.lim[k] - c : 0;
  return n < room ? n : room;
}

// an instance of root R at index e starts: offsets entries, scalar defaults
template <bool W, class CU>
KXN_HD void kxn_inst_start(const KxnProgram& P, const KxnCols& C, int R, uint64_t e, CU cur, KxnState& S) {
  const KxnRoot& RT = P.root[R];
  S.idx[RT.level] = e;
  S.seen[RT.level] = 0;
  S.pres[RT.level] = 0;
  if (!W) return;
  S.live[RT.level] = RT.level == 0 || !S.lim || e < S.lim[RT.dcur];
  if (!S.live[RT.level]) return;
  for (int k = RT.ent_lo; k < RT.ent_hi; k++) {
    const KxnEntry& E = P.ent[k];
    kxn_put_arr(C, E.col, E.arr, e, cur[E.cur]);
  }
  for (int k = RT.dfl_lo; k < RT.dfl_hi; k++) kxn_put_val(C, P.dfl[k].col, P.dfl[k].width, e, (uint64_t)P.dfl[k].v);
}

// the instance ends: absent string fields take their defaults, the presence word is stored
template <bool W, class CU>
KXN_HD void kxn_inst_end(const KxnProgram& P, const KxnCols& C, int R, CU cur, KxnState& S) {
  const KxnRoot& RT = P.root[R];
  const int L = RT.level;
  for (int k = RT.sdf_lo; k < RT.sdf_hi; k++) {
    const KxnSdef& D = P.sdf[k];
    if ((S.seen[L] >> D.sbit) & 1) continue;
    if (W)
      for (uint32_t j = 0; j < D.len; j++)
        if (!S.lim || cur[D.cur] + j < S.lim[D.cur]) ((KXN_G(uint8_t)*)C.data[D.col])[cur[D.cur] + j] = P.defb[D.off + j];
    cur.add(D.cur, D.len);
  }
  if (!W || !S.live[L]) return;
  if (L == 0) {
    if (C.presence) C.presence[S.idx[0]] = S.pres[0];
  } else if (RT.pres_col >= 0) {
    ((KXN_G(uint64_t)*)C.data[RT.pres_col])[S.idx[L]] = S.pres[L];
  }
}

// 16 bytes of the input at a Thrift field's header, in registers: the header and the field's value (a scalar, a
// string's length, a container's header) decode without a second dependent load (av: bytes valid; 0 = none).
// (The same for Kitex-PB tags + values measured slower: 14.1 vs 11.0 ms for 1 M PN records, the proto walker's
// registers grew past its occupancy step.)
struct KxnPre {
  uint64_t lo, hi;
  uint32_t av;
};
template <class B>
KXN_HD bool kxn_pre_load(B b, uint64_t q, KxnPre* p) {
  (void)b; (void)q; (void)p;
  return false;
}
KXN_HD bool kxn_pre_load(const uint8_t* b, uint64_t q, KxnPre* p) {
  __builtin_memcpy(&p->lo, b + q, 8);
  __builtin_memcpy(&p->hi, b + q + 8, 8);
  p->av = 16;
  return true;
}
// the window advanced by u (1 .. 10) bytes
KXN_HD void kxn_pre_skip(KxnPre* p, uint32_t u) {
  if (u < 8) {
    p->lo = (p->lo >> (8 * u)) | (p->hi << (64 - 8 * u));
    p->hi >>= 8 * u;
  } else {
    p->lo = p->hi >> (8 * (u - 8));
    p->hi = 0;
  }
  p->av = p->av > u ? p->av - u : 0;
}

// read one leaf value (SCALAR / STRING / RAW) of node X at b[*q]
// (pre: the value's first bytes in registers, Thrift byte order, when av > 0)
template <bool W, class B, class CU>
KXN_HD int kxn_leaf(const KxnProgram& P, const KxnCols& C, B b, uint64_t len, uint64_t* q, int X, CU cur,
                    KxnState& S, const KxnPre* pre = nullptr) {
  const KxnNode& N = P.node[X];
  if (N.kind == KN_RAW) {                                    // a recursive struct: its encoded bytes
    uint64_t e = *q;
    const int rc = kxn_skip(b, len, &e, KX_T_STRUCT, KXN_SKIP_DEPTH);
    if (rc) return rc;
    if (W) kxn_copy((uint8_t*)C.data[N.col] + cur[N.cur], b + *q, kxn_room(S, N.cur, cur[N.cur], e - *q));
    cur.add(N.cur, e - *q);
    *q = e;
    return KX_OK;
  }
  const bool pr = pre && pre->av >= 8;
  if (N.kind == KN_SCALAR) {
    if (*q + N.width > len) return KX_ERR_EOF;
    if (W && S.live[N.level])
      kxn_put_val(C, N.col, N.width, S.idx[N.level], pr ? kxn_scalar_pre(N.ttype, pre->lo) : kxn_scalar(N.ttype, b + *q));
    *q += N.width;
    return KX_OK;
  }
  if (*q + 4 > len) return KX_ERR_EOF;                       // ReadString: a copy
  const int32_t c = (int32_t)(pr ? __builtin_bswap32((uint32_t)pre->lo) : kxn_be32(b + *q));
  if (c < 0) return KX_ERR_NEGATIVE_SIZE;
  const uint64_t l = (uint64_t)c;
  if (*q + 4 + l > len) return KX_ERR_EOF;
  if (W) kxn_copy((uint8_t*)C.data[N.col] + cur[N.cur], b + *q + 4, kxn_room(S, N.cur, cur[N.cur], l));
  cur.add(N.cur, l);
  *q += 4 + l;
  return KX_OK;
}

// read one value of node X at b[*q] (scalars, strings, raw structs directly; structs / containers push a
// frame, except a list / map whose elements are leaves: its elements are read here, the frame loop's order
// of instance starts / ends kept, with no frame stored and updated per element). Element instances of the
// containers that push a frame are opened by the caller.
template <bool W, class B, class CU>
KXN_HD int kxn_value(const KxnProgram& P, const KxnCols& C, B b, uint64_t len, uint64_t* q, int X,
                     CU cur, KxnState& S, KxnFrame* stk, int* sp, const KxnPre& pre) {
  const KxnNode& N = P.node[X];
  const uint32_t kind = N.kind;
  if (kind <= KN_RAW) return kxn_leaf<W>(P, C, b, len, q, X, cur, S, &pre);
  // STRUCT / LIST / SET / MAP: ReadListBegin's type + count, ReadMapBegin's two types + count
  // (struct_tpl.go:425-625)
  const uint32_t hl = kind == KN_LIST ? 5u : kind == KN_MAP ? 6u : 0u;
  if (*q + hl > len) return KX_ERR_EOF;
  const uint32_t ho = kind == KN_LIST ? 1u : 2u;
  const int32_t c = !hl ? 0 : pre.av >= 8 ? (int32_t)__builtin_bswap32((uint32_t)(pre.lo >> (8 * ho)))
                                          : (int32_t)kxn_be32(b + *q + ho);
  if (c < 0) return KX_ERR_NEGATIVE_SIZE;
  if (hl && P.node[N.a].kind <= KN_RAW && (kind == KN_LIST || P.node[N.b].kind <= KN_RAW)) {
    *q += hl;
    for (int32_t i = 0; i < c; i++) {
      const uint64_t e = cur.post_inc(N.cur);
      kxn_inst_start<W>(P, C, N.root, e, cur, S);
      int rc = kxn_leaf<W>(P, C, b, len, q, N.a, cur, S);
      if (!rc && kind == KN_MAP) rc = kxn_leaf<W>(P, C, b, len, q, N.b, cur, S);
      if (rc) return rc;
      kxn_inst_end<W>(P, C, N.root, cur, S);
    }
    return KX_OK;
  }
  if (*sp >= KXN_STACK) return KX_ERR_DEPTH_LIMIT;
  stk[*sp] = KxnFrame{(uint8_t)kind, 0, 0, 0, (int16_t)(kind == KN_STRUCT ? N.a : X), 0, (int64_t)c};
  (*sp)++;
  *q += hl;
  return KX_OK;
}

// FastRead of record r = b[0 .. len). cur: cursors (measure: from 0, write: at the record's bases);
// lim (write, careful walk): the ends of the record's extents; snap: KXN_MAX_SNAP slots, or nullptr for the
// fast walk, which returns KXN_REPEAT at a field's second occurrence in one instance (the caller then walks
// the record again with snapshots, and in the write pass with lim). *used = bytes of the struct.
template <bool W, class B, class CU>
KXN_HD int kxn_read_record(const KxnProgram& P, const KxnCols& C, B b, uint64_t len, uint64_t r,
                           CU cur, uint64_t* snap, uint64_t* used, const uint64_t* lim = nullptr) {
  KxnFrame stk[KXN_STACK];
  KxnState S;
  S.lim = lim;
  S.live.fill(true);
  S.idx.fill(0);
  S.seen.fill(0);
  S.pres.fill(0);
  int sp = 0;
  uint64_t q = 0;
  kxn_inst_start<W>(P, C, 0, r, cur, S);
  // One value read per iteration, at a single call site: the frame logic only chooses the node X to read
  // (a struct's next field, a container's next element / key / value), so lanes of a wave at different
  // frame kinds meet again at the read (lane = record: 3.4x between 4 096 distinct Nesting records and
  // one record tiled, DESIGN §3.10, most of it divergence)
  int rc = KX_OK;
  int X = P.rec_node;
  KxnPre pre{0, 0, 0};   // a field's value bytes, loaded with its header (consumed by the next value read)
  for (;;) {
    if (X >= 0) {
      rc = kxn_value<W>(P, C, b, len, &q, X, cur, S, stk, &sp, pre);
      X = -1;
      pre.av = 0;
      if (rc) break;
    }
    if (sp == 0) break;
    KxnFrame& F = stk[sp - 1];
    if (F.kind == KN_STRUCT) {
      const KxnStruct& T = P.st[F.id];
      if (q + 1 > len) { rc = KX_ERR_EOF; break; }             // ReadFieldBegin
      // header and value from one 16-byte load where the record holds it, else type and id in one load where
      // 4 bytes remain (all but a record's final STOP)
      pre.av = 0;
      const bool h16 = len - q >= 16 && kxn_pre_load(b, q, &pre);
      const bool h4 = h16 || q + 4 <= len;
      const uint32_t hw = h16 ? __builtin_bswap32((uint32_t)pre.lo) : h4 ? kxn_be32(b + q) : 0u;
      const uint32_t t = h4 ? hw >> 24 : (uint32_t)b[q];
      const int L = T.level;
      if (t == KX_T_STOP) {
        q += 1;
        if ((S.seen[L] & T.req_mask) != T.req_mask) { rc = KX_ERR_INVALID_DATA; break; }  // :124-145
        sp--;
        continue;
      }
      if (q + 3 > len) { rc = KX_ERR_EOF; break; }
      const int16_t id = h4 ? (int16_t)(uint16_t)(hw >> 8) : (int16_t)kxn_be16(b + q + 1);
      q += 3;
      kxn_pre_skip(&pre, 3);
      const int fi = kxn_field(P, F.id, T, id);
      if (fi < 0 || P.f[fi].ttype != t) {                       // default: / mismatched type -> Skip
        if ((rc = kxn_skip(b, len, &q, t, KXN_SKIP_DEPTH))) break;
        continue;
      }
      const KxnField& G = P.f[fi];
      const KxnNode& N = P.node[G.node];
      const uint64_t bit = 1ull << G.sbit;
      const bool again = (S.seen[L] & bit) != 0;
      if (G.snap >= 0) {
        if (!snap) {                                            // fast walk: no snapshot was taken
          if (again) { rc = KXN_REPEAT; break; }
        } else if (again) {                                     // repeated: keep only this occurrence
          for (int k = N.cur_lo; k < N.cur_hi; k++) cur.set(k, snap[G.snap + k - N.cur_lo]);
        } else {
          for (int k = N.cur_lo; k < N.cur_hi; k++) snap[G.snap + k - N.cur_lo] = cur[k];
        }
      }
      if (again && N.kind == KN_STRUCT) {                       // a fresh NewX()
        const KxnStruct& U = P.st[N.a];
        if (W && S.live[L])
          for (int k = U.dfl_lo; k < U.dfl_hi; k++)
            kxn_put_val(C, P.dfl[k].col, P.dfl[k].width, S.idx[L], (uint64_t)P.dfl[k].v);
        S.seen[L] &= ~U.sub_mask;
        S.pres[L] &= ~U.pres_mask;
      }
      S.seen[L] |= bit;
      if (G.pbit >= 0) S.pres[L] |= 1ull << G.pbit;
      X = G.node;
      continue;
    }
    // LIST / MAP: close the open element, then open the next one (its value is read from memory)
    pre.av = 0;
    const KxnNode& N = P.node[F.id];
    if (F.open && (N.kind == KN_LIST || F.phase == 0)) {
      kxn_inst_end<W>(P, C, N.root, cur, S);
      F.open = 0;
    }
    if (N.kind == KN_LIST || F.phase == 0) {
      if (F.rem == 0) { sp--; continue; }
      F.rem--;
      const uint64_t e = cur.post_inc(N.cur);
      kxn_inst_start<W>(P, C, N.root, e, cur, S);
      F.open = 1;
      if (N.kind == KN_MAP) F.phase = 1;
      X = N.a;
    } else {
      F.phase = 0;
      X = N.b;
    }
  }
  if (rc) return rc;
  kxn_inst_end<W>(P, C, 0, cur, S);
  *used = q;
  return KX_OK;
}

// the instance of record r of a record that failed: defaults, empty extents, presence 0
template <class CU>
KXN_HD void kxn_failed_record(const KxnProgram& P, const KxnCols& C, uint64_t r, CU cur) {
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
    for (int k = 0; k < nbytes; k++) ((KXN_G(uint8_t)*)out)[*pos + k] = (uint8_t)(v >> (8 * (nbytes - 1 - k)));
  *pos += (uint64_t)nbytes;
}

KXN_HD uint64_t kxn_pres_word(const KxnProgram& P, const KxnCols& C, int R, uint64_t e) {
  const KxnRoot& RT = P.root[R];
  if (RT.level == 0) return C.presence ? C.presence[e] : 0;
  return RT.pres_col >= 0 ? ((const KXN_G(uint64_t)*)C.data[RT.pres_col])[e] : 0;
}

// one leaf value (SCALAR / STRING / RAW) of node X at instance index e
template <bool W>
KXN_HD void kxn_wleaf(const KxnProgram& P, const KxnCols& C, int X, uint64_t e, uint8_t* out, uint64_t* pos) {
  const KxnNode& N = P.node[X];
  if (N.kind == KN_SCALAR) {
    uint64_t v = kxn_get_val(C, N.col, N.width, e);
    if (N.ttype == KX_T_BOOL) v = (v & 0xff) ? 1 : 0;
    kxn_out<W>(out, pos, v, N.width);
    return;
  }
  const uint64_t a = kxn_get_arr(C, N.col, N.level, e), z = kxn_get_arr(C, N.col, N.level, e + 1);
  const uint64_t l = z - a;
  if (N.kind == KN_STRING) kxn_out<W>(out, pos, l, 4);
  else if (l == 0) { kxn_out<W>(out, pos, KX_T_STOP, 1); return; }  // an empty raw struct: STOP
  if (W)
    kxn_copy(out + *pos, (const uint8_t*)C.data[N.col] + a, l);
  *pos += l;
}

// one value of node X at instance index e (level X.level); structs / containers push a frame, except a
// list / map of leaves, whose elements are written here
template <bool W>
KXN_HD void kxn_wvalue(const KxnProgram& P, const KxnCols& C, int X, uint64_t e, uint8_t* out, uint64_t* pos,
                       KxnEFrame* stk, int* sp) {
  const KxnNode& N = P.node[X];
  if (N.kind <= KN_RAW) {
    kxn_wleaf<W>(P, C, X, e, out, pos);
    return;
  }
  if (N.kind == KN_STRUCT) {
    stk[*sp] = KxnEFrame{KN_STRUCT, 0, N.a, P.st[N.a].enc_first, P.st[N.a].root, 0, 0, e};
    (*sp)++;
    return;
  }
  const uint64_t a = kxn_get_arr(C, N.rep_col, N.level, e), z = kxn_get_arr(C, N.rep_col, N.level, e + 1);
  if (N.kind == KN_LIST) {
    kxn_out<W>(out, pos, N.etype, 1);
  } else {
    kxn_out<W>(out, pos, N.etype, 1);
    kxn_out<W>(out, pos, N.vtype, 1);
  }
  kxn_out<W>(out, pos, z - a, 4);
  if (P.node[N.a].kind <= KN_RAW && (N.kind == KN_LIST || P.node[N.b].kind <= KN_RAW)) {
    for (uint64_t i = a; i < z; i++) {
      kxn_wleaf<W>(P, C, N.a, i, out, pos);
      if (N.kind == KN_MAP) kxn_wleaf<W>(P, C, N.b, i, out, pos);
    }
    return;
  }
  stk[*sp] = KxnEFrame{N.kind, 0, (int16_t)X, 0, 0, a, z, 0};
  (*sp)++;
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

// ---------------------------------------------------------------------------------------------
// Kitex-Protobuf (proto3) on the same program and columns (KxnProgram.pb): proto.Unmarshal and
// proto.Marshal as protobuf-go does them (google.golang.org/protobuf: encoding/protowire for the wire
// format, internal/impl for the message semantics; not vendored in the reference, which calls them from
// pkg/remote/codec/protobuf/protobuf.go:64-134,209-216). A singular scalar or string keeps its last
// occurrence (a string rewinds its byte cursor to the first occurrence's snapshot), a message field merges
// its occurrences (no rewind, no reset), a repeated field appends one element per occurrence (scalars also
// as packed runs), a map appends one entry per occurrence (its key and value default to zero); unknown
// numbers and known numbers with another wire type are skipped.

template <class B>
KXN_HD int kxn_uvarint(B b, uint64_t end, uint64_t* q, uint64_t* v) {  // protowire.ConsumeVarint
  uint64_t x = 0;
  for (int i = 0; i < 10; i++) {
    if (*q + (uint64_t)i >= end) return KX_ERR_EOF;
    const uint32_t c = b[*q + (uint64_t)i];
    if (i == 9 && c > 1) return KX_ERR_INVALID_DATA;   // more than 64 bits
    x |= (uint64_t)(c & 0x7f) << (7 * i);
    if (c < 0x80) {
      *v = x;
      *q += (uint64_t)i + 1;
      return KX_OK;
    }
  }
  return KX_ERR_INVALID_DATA;
}

// the input itself (the device's walk over global memory): with 10 bytes left, the whole varint from one
// unaligned 8-byte load and a 2-byte one, branch-free (terminator = the first byte with bit 7 clear, the 7-bit
// groups compacted in three shift / mask steps), instead of a chain of dependent byte loads
KXN_HD int kxn_uvarint(const uint8_t* b, uint64_t end, uint64_t* q, uint64_t* v) {
  if (end - *q < 10) return kxn_uvarint<const uint8_t*>(b, end, q, v);
  uint64_t lo;
  uint16_t hi;
  __builtin_memcpy(&lo, b + *q, 8);
  __builtin_memcpy(&hi, b + *q + 8, 2);
  const uint32_t b8 = hi & 0xffu, b9 = hi >> 8;
  const uint64_t stop = ~lo & 0x8080808080808080ull;
  const uint32_t k = stop ? (uint32_t)__builtin_ctzll(stop) >> 3 : b8 < 0x80 ? 8u : 9u;
  if (k == 9 && b9 > 1) return KX_ERR_INVALID_DATA;   // more than 64 bits (or no terminator in 10 bytes)
  const uint64_t keep = k >= 7 ? ~0ull : (2ull << (8 * k + 7)) - 1;   // bytes 0..k
  uint64_t x = lo & keep & 0x7f7f7f7f7f7f7f7full;
  x = (x & 0x007f007f007f007full) | ((x & 0x7f007f007f007f00ull) >> 1);
  x = (x & 0x00003fff00003fffull) | ((x & 0x3fff00003fff0000ull) >> 2);
  x = (x & 0x000000000fffffffull) | ((x & 0x0fffffff00000000ull) >> 4);
  if (k >= 8) x |= (uint64_t)(b8 & 0x7f) << 56;
  if (k >= 9) x |= (uint64_t)(b9 & 0x01) << 63;
  *v = x;
  *q += k + 1;
  return KX_OK;
}

KXN_HD uint32_t kxn_uvlen(uint64_t v) {
  uint32_t n = 1;
  while (v >= 0x80) { v >>= 7; n++; }
  return n;
}

// wire type of one value of node N (scalars by kind; strings, bytes, messages and map entries: 2)
KXN_HD uint32_t kxn_pb_wt(const KxnNode& N) {
  if (N.kind != KN_SCALAR) return 2;
  if (N.ttype == KX_T_DOUBLE) return 1;
  if (N.pbk == KX_PB_FIXED) return N.ttype == KX_T_I32 ? 5u : 1u;
  return 0;
}

template <class B>
KXN_HD int kxn_pb_skip(B b, uint64_t end, uint64_t* q, uint32_t wt) {
  uint64_t v;
  switch (wt) {
    case 0: return kxn_uvarint(b, end, q, &v);
    case 1: if (end - *q < 8) return KX_ERR_EOF; *q += 8; return KX_OK;
    case 2: {
      const int rc = kxn_uvarint(b, end, q, &v);
      if (rc) return rc;
      if (v > end - *q) return KX_ERR_EOF;
      *q += v;
      return KX_OK;
    }
    case 5: if (end - *q < 4) return KX_ERR_EOF; *q += 4; return KX_OK;
    default: return KX_ERR_INVALID_DATA;   // groups (3, 4) and 6, 7: rejected (as the flat proto path)
  }
}

template <class B>
KXN_HD uint64_t kxn_le(B p, int n) {
  uint64_t v = 0;
  for (int k = n - 1; k >= 0; k--) v = (v << 8) | p[k];
  return v;
}
KXN_HD uint64_t kxn_le(const uint8_t* p, int n) {   // the input itself: one unaligned load
  if (n == 8) {
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
  }
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
}

// one scalar of node N at b[*q] (its wire type already matched), in the column's host form
template <class B>
KXN_HD int kxn_pb_scalar(const KxnNode& N, B b, uint64_t end, uint64_t* q, uint64_t* out) {
  const uint32_t wt = kxn_pb_wt(N);
  uint64_t v;
  if (wt == 0) {
    const int rc = kxn_uvarint(b, end, q, &v);
    if (rc) return rc;
    if (N.ttype == KX_T_BOOL) {
      v = v != 0;
    } else if (N.pbk == KX_PB_SINT) {   // protowire.DecodeZigZag (sint32: of the low 32 bits)
      if (N.ttype == KX_T_I32) {
        const uint32_t u = (uint32_t)v;
        v = (uint64_t)((u >> 1) ^ (0u - (u & 1u)));
      } else {
        v = (v >> 1) ^ (0ull - (v & 1ull));
      }
    }                                   // int32 / uint32 / enum: the column keeps the low 32 bits
  } else {
    const int n = wt == 1 ? 8 : 4;
    if (end - *q < (uint64_t)n) return KX_ERR_EOF;
    v = kxn_le(b + *q, n);
    *q += (uint64_t)n;
  }
  *out = v;
  return KX_OK;
}

// utf8.Valid, as protobuf-go checks proto3 `string` fields; over the input itself 8 bytes per step while they
// are ASCII (one unaligned load each)
template <class B>
KXN_HD uint64_t kxn_ascii_prefix(B s, uint64_t n) { (void)s; (void)n; return 0; }
KXN_HD uint64_t kxn_ascii_prefix(const uint8_t* s, uint64_t n) {
  uint64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t x;
    __builtin_memcpy(&x, s + i, 8);
    if (x & 0x8080808080808080ull) break;
  }
  return i;
}
template <class B>
KXN_HD bool kxn_utf8(B s, uint64_t n, B lo) {
  (void)lo;
  uint64_t i = kxn_ascii_prefix(s, n);
  while (i < n) {
    const uint32_t c = s[i];
    if (c < 0x80) { i++; continue; }
    int k;
    uint32_t cp;
    if ((c & 0xe0) == 0xc0) { k = 1; cp = c & 0x1f; }
    else if ((c & 0xf0) == 0xe0) { k = 2; cp = c & 0x0f; }
    else if ((c & 0xf8) == 0xf0) { k = 3; cp = c & 0x07; }
    else return false;
    if (i + (uint64_t)k >= n) return false;
    for (int j = 1; j <= k; j++) {
      const uint32_t d = s[i + (uint64_t)j];
      if ((d & 0xc0) != 0x80) return false;
      cp = (cp << 6) | (d & 0x3f);
    }
    if ((k == 1 && cp < 0x80) || (k == 2 && cp < 0x800) || (k == 3 && cp < 0x10000)) return false;
    if (cp > 0x10ffff || (cp >= 0xd800 && cp <= 0xdfff)) return false;
    i += (uint64_t)k + 1;
  }
  return true;
}

// the input itself: 8 bytes per load into a register, each word checked with byte masks and no per-byte loop
// (the per-byte sequence check was 1.2 of the 4.3 ms of the measure pass over 1 M PN records, whose strings
// hold 2- and 3-byte characters). Masks hold one flag per byte in its bit 7: continuation (10xxxxxx) and
// lead bytes (110 / 1110 / 11110); the continuations the leads expect (shifted by 1 .. 3 bytes, the ones past
// the word carried into the next) must be exactly the continuation bytes; the lead / next-byte pairs that
// utf8.Valid refuses (C0 C1, E0 < A0, ED >= A0, F0 < 90, F4 >= 90, F5 and up) are flags too. The last < 8
// bytes come from one load ending at the string's end when the record holds 8 bytes there ([lo, s + n) is
// readable); bytes past the string read as 0 (ASCII), so a truncated sequence fails the continuation test.
KXN_HD uint64_t kxn_nzb(uint64_t v) {   // bit 7 of every nonzero byte
  return (((v & 0x7f7f7f7f7f7f7f7full) + 0x7f7f7f7f7f7f7f7full) | v) & 0x8080808080808080ull;
}
KXN_HD bool kxn_utf8(const uint8_t* s, uint64_t n, const uint8_t* lo) {
  constexpr uint64_t H = 0x8080808080808080ull;
  uint64_t i = 0, cin = 0, pend = 0;   // pend: E0 / ED / F0 / F4 lead in the previous word's last byte (bit 7, 15, 23, 31)
  while (i < n) {
    const uint64_t m = n - i < 8 ? n - i : 8;
    uint64_t x = 0;
    if (m == 8) {
      __builtin_memcpy(&x, s + i, 8);
    } else if ((uint64_t)(s + n - lo) >= 8) {
      __builtin_memcpy(&x, s + n - 8, 8);
      x >>= 8 * (8 - m);
    } else {
      for (uint64_t j = 0; j < m; j++) x |= (uint64_t)s[i + j] << (8 * j);
    }
    i += m;
    if ((cin | pend) == 0 && !(x & H)) continue;   // ASCII
    const uint64_t h = x & H, b6 = (x << 1) & H, b5 = (x << 2) & H, b4 = (x << 3) & H, b3 = (x << 4) & H;
    const uint64_t b2 = (x << 5) & H, b1 = (x << 6) & H, b0 = (x << 7) & H;
    const uint64_t cont = h & ~b6, lead = h & b6;
    const uint64_t l2 = lead & ~b5, l3 = lead & b5 & ~b4, l4 = lead & b5 & b4 & ~b3;
    uint64_t bad = lead & b5 & b4 & b3;                                           // F8 .. FF
    bad |= l2 & ~kxn_nzb(x & 0x1e1e1e1e1e1e1e1eull);                             // C0 C1
    bad |= l4 & b2 & (b1 | b0);                                                    // F5 .. F7
    const uint64_t e0 = l3 & ~kxn_nzb(x & 0x0f0f0f0f0f0f0f0full);
    const uint64_t ed = l3 & ~kxn_nzb((x & 0x0f0f0f0f0f0f0f0full) ^ 0x0d0d0d0d0d0d0d0dull);
    const uint64_t f0 = l4 & ~kxn_nzb(x & 0x0707070707070707ull);
    const uint64_t f4 = l4 & ~kxn_nzb((x & 0x0707070707070707ull) ^ 0x0404040404040404ull);
    const uint64_t E0 = (e0 << 8) | ((pend & 0x80) ? 0x80 : 0), ED = (ed << 8) | ((pend & 0x8000) ? 0x80 : 0);
    const uint64_t F0 = (f0 << 8) | ((pend & 0x800000) ? 0x80 : 0), F4 = (f4 << 8) | ((pend & 0x80000000) ? 0x80 : 0);
    bad |= (E0 & ~b5) | (ED & b5) | (F0 & ~(b5 | b4)) | (F4 & (b5 | b4));
    const uint64_t l234 = l2 | l3 | l4, l34 = l3 | l4;
    if (bad || ((l234 << 8) | (l34 << 16) | (l4 << 24) | cin) != cont) return false;
    cin = (l234 >> 56) | (l34 >> 48) | (l4 >> 40);
    pend = (e0 >> 56) | ((ed >> 56) << 8) | ((f0 >> 56) << 16) | ((f4 >> 56) << 24);
  }
  return cin == 0;
}

struct KxnPFrame {      // an open message (its fields) or map entry (fields 1 / 2) (32 B)
  uint8_t kind;         // 0 message, 1 map entry
  uint8_t seen;         // map entry: key / value read (bits 0 / 1)
  int16_t id;           // message: struct instance; entry: the map node
  int16_t close;        // root whose instance ends when the frame does (-1)
  int16_t pad;
  uint64_t end;         // where its bytes end
  uint64_t c0[2];       // map entry: cursor of a string key / value at its first occurrence
};

// one value of node X (wire type matched) into the open instance of its level; a message value pushes a
// frame (close: the root to end with it), a scalar / string value ends `close` at once
template <bool W, class B, class CU>
KXN_HD int kxn_pb_value(const KxnProgram& P, const KxnCols& C, B b, uint64_t end, uint64_t* q, int X,
                        CU cur, KxnState& S, KxnPFrame* stk, int* sp, int close) {
  const KxnNode& N = P.node[X];
  switch (N.kind) {
    case KN_SCALAR: {
      uint64_t v;
      const int rc = kxn_pb_scalar(N, b, end, q, &v);
      if (rc) return rc;
      if (W && S.live[N.level]) kxn_put_val(C, N.col, N.width, S.idx[N.level], v);
      break;
    }
    case KN_STRING: case KN_RAW: {   // string / bytes; a recursive message keeps its bytes (they merge)
      uint64_t l;
      const int rc = kxn_uvarint(b, end, q, &l);
      if (rc) return rc;
      if (l > end - *q) return KX_ERR_EOF;
      // (the write walk reads only records its measure walk validated)
      if (!W && N.kind == KN_STRING && N.pbk != KX_PB_BYTES && !kxn_utf8(b + *q, l, b)) return KX_ERR_INVALID_DATA;
      if (W) kxn_copy((uint8_t*)C.data[N.col] + cur[N.cur], b + *q, kxn_room(S, N.cur, cur[N.cur], l));
      cur.add(N.cur, l);
      *q += l;
      break;
    }
    case KN_STRUCT: {
      uint64_t l;
      const int rc = kxn_uvarint(b, end, q, &l);
      if (rc) return rc;
      if (l > end - *q) return KX_ERR_EOF;
      if (*sp >= KXN_STACK) return KX_ERR_DEPTH_LIMIT;
      stk[*sp] = KxnPFrame{0, 0, N.a, (int16_t)close, 0, *q + l, {0, 0}};
      (*sp)++;
      return KX_OK;
    }
    default:
      return KX_ERR_INTERNAL;   // containers are opened by the field loop
  }
  if (close >= 0) kxn_inst_end<W>(P, C, close, cur, S);
  return KX_OK;
}

// proto.Unmarshal of record r = b[0 .. len): same cursors / snapshots / clipping / fast walk as kxn_read_record
template <bool W, class B, class CU>
KXN_HD int kxn_pb_read_record(const KxnProgram& P, const KxnCols& C, B b, uint64_t len, uint64_t r,
                              CU cur, uint64_t* snap, uint64_t* used, const uint64_t* lim = nullptr) {
  KxnPFrame stk[KXN_STACK];
  KxnState S;
  S.lim = lim;
  S.live.fill(true);
  S.idx.fill(0);
  S.seen.fill(0);
  S.pres.fill(0);
  int sp = 0;
  uint64_t q = 0;
  int rc = KX_OK;
  kxn_inst_start<W>(P, C, 0, r, cur, S);
  stk[sp++] = KxnPFrame{0, 0, P.node[P.rec_node].a, -1, 0, len, {0, 0}};
  // one value read per iteration at a single call site (as kxn_read_record): X, its frame's end and the
  // root its instance closes are chosen by the field logic below
  int X = -1, xclose = -1;
  uint64_t xend = 0;
  for (;;) {
    if (X >= 0) {
      rc = kxn_pb_value<W>(P, C, b, xend, &q, X, cur, S, stk, &sp, xclose);
      X = -1;
      if (rc) break;
    }
    if (sp == 0) break;
    KxnPFrame& F = stk[sp - 1];
    if (q >= F.end) {
      const int cl = F.close;
      sp--;
      if (cl >= 0) kxn_inst_end<W>(P, C, cl, cur, S);
      continue;
    }
    uint64_t tag;
    if ((rc = kxn_uvarint(b, F.end, &q, &tag))) break;
    const uint64_t num = tag >> 3;
    const uint32_t wt = (uint32_t)(tag & 7);
    if (num == 0 || num > 536870911ull) { rc = KX_ERR_INVALID_DATA; break; }   // protowire.MaxValidNumber
    if (F.kind == 1) {                                  // map entry: key = 1, value = 2
      const KxnNode& M = P.node[F.id];
      const int Xm = num == 1 ? M.a : num == 2 ? M.b : -1;
      if (Xm < 0 || wt != kxn_pb_wt(P.node[Xm])) {
        if ((rc = kxn_pb_skip(b, F.end, &q, wt))) break;
        continue;
      }
      const KxnNode& V = P.node[Xm];
      const int k = num == 1 ? 0 : 1;
      if (V.kind == KN_STRING || V.kind == KN_RAW) {    // a repeated key / value string: the last one wins
        if (F.seen & (1 << k)) {
          if (!snap) { rc = KXN_REPEAT; break; }        // fast walk: the careful one clips the first copy
          cur.set(V.cur, F.c0[k]);
        } else {
          F.c0[k] = cur[V.cur];
        }
      }
      F.seen |= (uint8_t)(1 << k);
      xend = F.end;
      xclose = -1;
      X = Xm;
      continue;
    }
    const KxnStruct& T = P.st[F.id];
    const int L = T.level;
    const int fi = kxn_field(P, F.id, T, (int64_t)num);
    if (fi < 0) {                                       // unknown field
      if ((rc = kxn_pb_skip(b, F.end, &q, wt))) break;
      continue;
    }
    const KxnField& G = P.f[fi];
    const KxnNode& N = P.node[G.node];
    const uint64_t bit = 1ull << G.sbit;
    const uint64_t fend = F.end;
    if (N.kind == KN_LIST) {                            // repeated: append
      const KxnNode& E = P.node[N.a];
      const uint32_t ewt = kxn_pb_wt(E);
      if (wt == ewt) {
        S.seen[L] |= bit;
        if (G.pbit >= 0) S.pres[L] |= 1ull << G.pbit;
        const uint64_t e = cur.post_inc(N.cur);
        kxn_inst_start<W>(P, C, N.root, e, cur, S);
        xend = fend;
        xclose = N.root;
        X = N.a;
      } else if (wt == 2 && E.kind == KN_SCALAR) {      // a packed run
        uint64_t l;
        if ((rc = kxn_uvarint(b, fend, &q, &l))) break;
        if (l > fend - q) { rc = KX_ERR_EOF; break; }
        S.seen[L] |= bit;
        if (G.pbit >= 0) S.pres[L] |= 1ull << G.pbit;
        const uint64_t pend = q + l;
        while (q < pend) {
          const uint64_t e = cur.post_inc(N.cur);
          kxn_inst_start<W>(P, C, N.root, e, cur, S);
          uint64_t v;
          if ((rc = kxn_pb_scalar(E, b, pend, &q, &v))) break;
          if (W && S.live[E.level]) kxn_put_val(C, E.col, E.width, S.idx[E.level], v);
          kxn_inst_end<W>(P, C, N.root, cur, S);
        }
        if (rc) break;
      } else if ((rc = kxn_pb_skip(b, fend, &q, wt))) {
        break;
      }
      continue;
    }
    if (N.kind == KN_MAP) {                             // one entry per occurrence
      if (wt != 2) {
        if ((rc = kxn_pb_skip(b, fend, &q, wt))) break;
        continue;
      }
      uint64_t l;
      if ((rc = kxn_uvarint(b, fend, &q, &l))) break;
      if (l > fend - q) { rc = KX_ERR_EOF; break; }
      if (sp >= KXN_STACK) { rc = KX_ERR_DEPTH_LIMIT; break; }
      S.seen[L] |= bit;
      if (G.pbit >= 0) S.pres[L] |= 1ull << G.pbit;
      const uint64_t e = cur.post_inc(N.cur);
      kxn_inst_start<W>(P, C, N.root, e, cur, S);
      stk[sp++] = KxnPFrame{1, 0, G.node, N.root, 0, q + l, {0, 0}};
      continue;
    }
    if (wt != kxn_pb_wt(N)) {                           // another wire type: unknown
      if ((rc = kxn_pb_skip(b, fend, &q, wt))) break;
      continue;
    }
    if (N.kind == KN_STRING && G.snap >= 0) {           // singular string: the last occurrence wins
      if (!snap) {
        if (S.seen[L] & bit) { rc = KXN_REPEAT; break; }
      } else if (S.seen[L] & bit) {
        cur.set(N.cur, snap[G.snap]);
      } else {
        snap[G.snap] = cur[N.cur];
      }
    }
    S.seen[L] |= bit;
    if (G.pbit >= 0) S.pres[L] |= 1ull << G.pbit;
    xend = fend;   // a message merges
    xclose = -1;
    X = G.node;
  }
  if (rc) return rc;
  kxn_inst_end<W>(P, C, 0, cur, S);
  *used = q;
  return KX_OK;
}

// ---- proto.Marshal from the columns ----
template <bool W>
KXN_HD void kxn_pb_put_uv(uint8_t* out, uint64_t* pos, uint64_t v) {
  while (v >= 0x80) {
    if (W) ((KXN_G(uint8_t)*)out)[*pos] = (uint8_t)(v | 0x80);
    (*pos)++;
    v >>= 7;
  }
  if (W) ((KXN_G(uint8_t)*)out)[*pos] = (uint8_t)v;
  (*pos)++;
}

// the scalar of node N at instance e: *wire = its varint value, or its fixed bytes (*fixed = 4 / 8)
KXN_HD uint64_t kxn_pb_wire_scalar_c(const KxnCols& C, const KxnNode& N, uint64_t e, int* fixed, bool* zero) {
  const uint64_t v = kxn_get_val(C, N.col, N.width, e);
  const uint32_t wt = kxn_pb_wt(N);
  *zero = (N.ttype == KX_T_BOOL ? (v & 0xff) : v) == 0;
  if (wt != 0) {
    *fixed = wt == 1 ? 8 : 4;
    return v;
  }
  *fixed = 0;
  if (N.ttype == KX_T_BOOL) return (v & 0xff) ? 1 : 0;
  if (N.ttype == KX_T_I32) {
    const uint32_t x = (uint32_t)v;
    if (N.pbk == KX_PB_SINT) return (uint64_t)((x << 1) ^ (uint32_t)((int32_t)x >> 31));
    if (N.pbk == KX_PB_UINT) return (uint64_t)x;
    return (uint64_t)(int64_t)(int32_t)x;   // int32 / enum: sign-extended
  }
  return N.pbk == KX_PB_SINT ? ((v << 1) ^ (uint64_t)((int64_t)v >> 63)) : v;
}
KXN_HD uint64_t kxn_pb_wire_scalar(const KxnProgram& P, const KxnCols& C, const KxnNode& N, uint64_t e, int* fixed,
                                   bool* zero) {
  (void)P;
  return kxn_pb_wire_scalar_c(C, N, e, fixed, zero);
}

template <bool W>
KXN_HD void kxn_pb_put_scalar(uint8_t* out, uint64_t* pos, uint64_t v, int fixed) {
  if (fixed) {
    if (W)
      for (int k = 0; k < fixed; k++) ((KXN_G(uint8_t)*)out)[*pos + k] = (uint8_t)(v >> (8 * k));
    *pos += (uint64_t)fixed;
  } else {
    kxn_pb_put_uv<W>(out, pos, v);
  }
}

// a map entry's key (field 1) or value (field 2) that is a leaf: its tag + value bytes, and the writer
KXN_HD uint64_t kxn_pb_leaf_size(const KxnCols& C, const KxnNode& V, int fnum, uint64_t e) {
  const uint64_t tag = ((uint64_t)fnum << 3) | kxn_pb_wt(V);
  if (V.kind == KN_SCALAR) {
    int fixed;
    bool zero;
    const uint64_t v = kxn_pb_wire_scalar_c(C, V, e, &fixed, &zero);
    return kxn_uvlen(tag) + (fixed ? (uint64_t)fixed : kxn_uvlen(v));
  }
  const uint64_t l = kxn_get_arr(C, V.col, V.level, e + 1) - kxn_get_arr(C, V.col, V.level, e);
  return kxn_uvlen(tag) + kxn_uvlen(l) + l;
}
template <bool W>
KXN_HD void kxn_pb_put_leaf(const KxnCols& C, const KxnNode& V, int fnum, uint64_t e, uint8_t* out, uint64_t* pos) {
  const uint64_t tag = ((uint64_t)fnum << 3) | kxn_pb_wt(V);
  kxn_pb_put_uv<W>(out, pos, tag);
  if (V.kind == KN_SCALAR) {
    int fixed;
    bool zero;
    const uint64_t v = kxn_pb_wire_scalar_c(C, V, e, &fixed, &zero);
    kxn_pb_put_scalar<W>(out, pos, v, fixed);
    return;
  }
  const uint64_t a = kxn_get_arr(C, V.col, V.level, e), z = kxn_get_arr(C, V.col, V.level, e + 1);
  kxn_pb_put_uv<W>(out, pos, z - a);
  if (W) kxn_copy(out + *pos, (const uint8_t*)C.data[V.col] + a, z - a);
  *pos += z - a;
}

struct KxnPEFrame {     // encode: a message's fields, a repeated message's elements, a map's entries (48 B)
  uint8_t kind;         // 0 message, 1 repeated message elements, 2 map entries, 3 one map entry
  uint8_t phase;        // map entry: 0 key + value, 1 (message value) done
  int16_t id;           // message: struct; elements / entries / entry: the container node
  int16_t f;            // message: next field (field-number order)
  int16_t root;         // message: its instance root (presence word)
  uint32_t tagsz;       // size mode: the tag bytes of this value in its parent (0: not length-delimited)
  uint32_t fnum;        // elements / entries: the field number
  uint64_t e;           // message / entry: its instance index; elements / entries: next index
  uint64_t end;         // elements / entries: end index
  uint64_t acc;         // size mode: bytes so far
};

// Size (W = false: returns the body size of the frame it starts with, post-order over nested messages)
// or write (W = true: message bodies' sizes from the size walk) of a message / entry. start: the first frame.
template <bool W>
KXN_HD uint64_t kxn_pb_walk(const KxnProgram& P, const KxnCols& C, KxnPEFrame start, uint8_t* out, uint64_t pos0);

template <bool W>
KXN_HD uint64_t kxn_pb_walk(const KxnProgram& P, const KxnCols& C, KxnPEFrame start, uint8_t* out, uint64_t pos0) {
  KxnPEFrame stk[KXN_STACK];
  int sp = 0;
  stk[sp++] = start;
  uint64_t pos = pos0;      // W: where the next byte goes
  uint64_t result = 0;
  // a length-delimited child: size mode pushes it (its size returns through acc); write mode writes
  // tag + length (from a size walk of the child) and pushes it
  while (sp > 0) {
    KxnPEFrame& F = stk[sp - 1];
    uint64_t sz = 0;            // size mode: bytes this step adds to F.acc
    if (F.kind == 0) {          // message fields, field-number order
      if (F.f < 0) {            // done
        const KxnPEFrame D = F;
        sp--;
        if (!W) {
          if (sp == 0) result = D.acc;
          else stk[sp - 1].acc += D.tagsz ? D.tagsz + kxn_uvlen(D.acc) + D.acc : D.acc;
        }
        continue;
      }
      const KxnField& G = P.f[F.f];
      F.f = G.enc_next;
      const KxnNode& N = P.node[G.node];
      const uint64_t e = F.e;
      uint64_t pres = 0;
      bool isset = false;
      if (G.pbit >= 0) {
        pres = kxn_pres_word(P, C, F.root, e);
        isset = (pres >> G.pbit) & 1;
      }
      const bool optional = G.req == KX_REQ_OPTIONAL;
      if (N.kind == KN_SCALAR) {
        int fixed;
        bool zero;
        const uint64_t v = kxn_pb_wire_scalar(P, C, N, e, &fixed, &zero);
        if (optional ? !isset : zero) continue;       // proto3: zero omitted; `optional`: when present
        const uint64_t tag = ((uint64_t)(uint16_t)G.id << 3) | kxn_pb_wt(N);
        if (W) {
          kxn_pb_put_uv<W>(out, &pos, tag);
          kxn_pb_put_scalar<W>(out, &pos, v, fixed);
        } else {
          sz = kxn_uvlen(tag) + (fixed ? (uint64_t)fixed : kxn_uvlen(v));
        }
      } else if (N.kind == KN_STRING || N.kind == KN_RAW) {
        const uint64_t a = kxn_get_arr(C, N.col, N.level, e), z = kxn_get_arr(C, N.col, N.level, e + 1);
        const uint64_t l = z - a;
        if (N.kind == KN_RAW ? !isset : (optional ? !isset : l == 0)) continue;
        const uint64_t tag = ((uint64_t)(uint16_t)G.id << 3) | 2u;
        if (W) {
          kxn_pb_put_uv<W>(out, &pos, tag);
          kxn_pb_put_uv<W>(out, &pos, l);
          kxn_copy(out + pos, (const uint8_t*)C.data[N.col] + a, l);
          pos += l;
        } else {
          sz = kxn_uvlen(tag) + kxn_uvlen(l) + l;
        }
      } else if (N.kind == KN_STRUCT) {
        if (!isset) continue;                          // a nil message is not written
        const uint64_t tag = ((uint64_t)(uint16_t)G.id << 3) | 2u;
        if (sp >= KXN_STACK) break;
        const KxnPEFrame Cf{0, 0, N.a, P.st[N.a].enc_first, F.root, (uint32_t)kxn_uvlen(tag), 0, e, 0, 0};
        if (W) {
          kxn_pb_put_uv<W>(out, &pos, tag);
          kxn_pb_put_uv<W>(out, &pos, kxn_pb_walk<false>(P, C, KxnPEFrame{0, 0, N.a, P.st[N.a].enc_first, F.root,
                                                                          0, 0, e, 0, 0}, nullptr, 0));
        }
        stk[sp++] = Cf;
        continue;
      } else {                                         // repeated / map
        const uint64_t a = kxn_get_arr(C, N.rep_col, N.level, e), z = kxn_get_arr(C, N.rep_col, N.level, e + 1);
        if (a == z) continue;
        const KxnNode& E = P.node[N.a];
        if (N.kind == KN_LIST && E.kind == KN_SCALAR) {  // packed
          uint64_t body = 0;
          for (uint64_t j = a; j < z; j++) {
            int fixed;
            bool zero;
            const uint64_t v = kxn_pb_wire_scalar(P, C, E, j, &fixed, &zero);
            body += fixed ? (uint64_t)fixed : kxn_uvlen(v);
          }
          const uint64_t tag = ((uint64_t)(uint16_t)G.id << 3) | 2u;
          if (W) {
            kxn_pb_put_uv<W>(out, &pos, tag);
            kxn_pb_put_uv<W>(out, &pos, body);
            for (uint64_t j = a; j < z; j++) {
              int fixed;
              bool zero;
              const uint64_t v = kxn_pb_wire_scalar(P, C, E, j, &fixed, &zero);
              kxn_pb_put_scalar<W>(out, &pos, v, fixed);
            }
          } else {
            sz = kxn_uvlen(tag) + kxn_uvlen(body) + body;
          }
        } else if (N.kind == KN_LIST && (E.kind == KN_STRING || E.kind == KN_RAW)) {
          const uint64_t tag = ((uint64_t)(uint16_t)G.id << 3) | 2u;
          for (uint64_t j = a; j < z; j++) {
            const uint64_t sa = kxn_get_arr(C, E.col, E.level, j), sb = kxn_get_arr(C, E.col, E.level, j + 1);
            const uint64_t l = sb - sa;
            if (W) {
              kxn_pb_put_uv<W>(out, &pos, tag);
              kxn_pb_put_uv<W>(out, &pos, l);
              for (uint64_t k = 0; k < l; k++) ((KXN_G(uint8_t)*)out)[pos + k] = ((const KXN_G(uint8_t)*)C.data[E.col])[sa + k];
              pos += l;
            } else {
              sz += kxn_uvlen(tag) + kxn_uvlen(l) + l;
            }
          }
        } else if (N.kind == KN_MAP && P.node[N.a].kind <= KN_RAW && P.node[N.b].kind <= KN_RAW) {
          // entries of leaves: each entry's size from its key and value here, no entry frame and no size walk
          const uint64_t tag = ((uint64_t)(uint16_t)G.id << 3) | 2u;
          for (uint64_t j = a; j < z; j++) {
            uint64_t body = 0;
            for (int k = 0; k < 2; k++) body += kxn_pb_leaf_size(C, P.node[k == 0 ? N.a : N.b], k + 1, j);
            if (W) {
              kxn_pb_put_uv<W>(out, &pos, tag);
              kxn_pb_put_uv<W>(out, &pos, body);
              for (int k = 0; k < 2; k++) kxn_pb_put_leaf<W>(C, P.node[k == 0 ? N.a : N.b], k + 1, j, out, &pos);
            } else {
              sz += kxn_uvlen(tag) + kxn_uvlen(body) + body;
            }
          }
        } else {                                       // repeated messages / map entries: a frame
          if (sp >= KXN_STACK) break;
          const uint64_t tag = ((uint64_t)(uint16_t)G.id << 3) | 2u;
          stk[sp++] = KxnPEFrame{(uint8_t)(N.kind == KN_LIST ? 1 : 2), 0, G.node, 0, 0, (uint32_t)kxn_uvlen(tag),
                                 (uint32_t)G.id, a, z, 0};
          continue;
        }
      }
      if (!W) F.acc += sz;
      continue;
    }
    if (F.kind == 1 || F.kind == 2) {   // the next element / entry
      if (F.e >= F.end) {
        const KxnPEFrame D = F;
        sp--;
        if (!W) {
          if (sp == 0) result = D.acc;
          else stk[sp - 1].acc += D.acc;   // each element / entry already carries its own tag + length
        }
        continue;
      }
      const uint64_t j = F.e++;
      const KxnNode& N = P.node[F.id];
      const uint64_t tag = ((uint64_t)F.fnum << 3) | 2u;
      if (sp >= KXN_STACK) break;
      KxnPEFrame Cf;
      if (F.kind == 1) {
        const KxnNode& E = P.node[N.a];
        Cf = KxnPEFrame{0, 0, E.a, P.st[E.a].enc_first, N.root, F.tagsz, 0, j, 0, 0};
      } else {
        Cf = KxnPEFrame{3, 0, F.id, 0, N.root, F.tagsz, 0, j, 0, 0};
      }
      if (W) {
        kxn_pb_put_uv<W>(out, &pos, tag);
        KxnPEFrame Sf = Cf;
        Sf.tagsz = 0;
        kxn_pb_put_uv<W>(out, &pos, kxn_pb_walk<false>(P, C, Sf, nullptr, 0));
      }
      stk[sp++] = Cf;
      continue;
    }
    // one map entry: key (field 1) and value (field 2), both always written
    const KxnNode& M = P.node[F.id];
    if (F.phase == 1) {
      const KxnPEFrame D = F;
      sp--;
      if (!W) {
        if (sp == 0) result = D.acc;
        else stk[sp - 1].acc += D.tagsz ? D.tagsz + kxn_uvlen(D.acc) + D.acc : D.acc;
      }
      continue;
    }
    F.phase = 1;
    for (int k = 0; k < 2; k++) {
      const KxnNode& V = P.node[k == 0 ? M.a : M.b];
      const uint64_t tag = ((uint64_t)(k + 1) << 3) | kxn_pb_wt(V);
      if (V.kind == KN_SCALAR) {
        int fixed;
        bool zero;
        const uint64_t v = kxn_pb_wire_scalar(P, C, V, F.e, &fixed, &zero);
        if (W) {
          kxn_pb_put_uv<W>(out, &pos, tag);
          kxn_pb_put_scalar<W>(out, &pos, v, fixed);
        } else {
          F.acc += kxn_uvlen(tag) + (fixed ? (uint64_t)fixed : kxn_uvlen(v));
        }
      } else if (V.kind == KN_STRING || V.kind == KN_RAW) {
        const uint64_t a = kxn_get_arr(C, V.col, V.level, F.e), z = kxn_get_arr(C, V.col, V.level, F.e + 1);
        const uint64_t l = z - a;
        if (W) {
          kxn_pb_put_uv<W>(out, &pos, tag);
          kxn_pb_put_uv<W>(out, &pos, l);
          kxn_copy(out + pos, (const uint8_t*)C.data[V.col] + a, l);
          pos += l;
        } else {
          F.acc += kxn_uvlen(tag) + kxn_uvlen(l) + l;
        }
      } else {                                          // a message value: a child frame (the entry's instance)
        const KxnPEFrame Cf{0, 0, V.a, P.st[V.a].enc_first, M.root, (uint32_t)kxn_uvlen(tag), 0, F.e, 0, 0};
        if (W) {
          kxn_pb_put_uv<W>(out, &pos, tag);
          KxnPEFrame Sf = Cf;
          Sf.tagsz = 0;
          kxn_pb_put_uv<W>(out, &pos, kxn_pb_walk<false>(P, C, Sf, nullptr, 0));
        }
        if (sp < KXN_STACK) stk[sp++] = Cf;
      }
    }
  }
  return W ? pos - pos0 : result;
}

// record r as a Batch frame: 0x0A, uvarint(body), body
KXN_HD uint64_t kxn_pb_frame_size(const KxnProgram& P, const KxnCols& C, uint64_t r) {
  const int si = P.node[P.rec_node].a;
  const uint64_t body = kxn_pb_walk<false>(P, C, KxnPEFrame{0, 0, (int16_t)si, P.st[si].enc_first, 0, 0, 0, r, 0, 0},
                                           nullptr, 0);
  return 1 + kxn_uvlen(body) + body;
}

KXN_HD void kxn_pb_write_frame(const KxnProgram& P, const KxnCols& C, uint64_t r, uint8_t* out, uint64_t pos,
                               uint64_t frame_size) {
  const int si = P.node[P.rec_node].a;
  // body = frame_size - 1 - uvlen(body): the uvarint length that fits
  uint64_t body = 0;
  for (uint32_t u = 1; u <= 10; u++) {
    if (frame_size < 1 + (uint64_t)u) break;
    body = frame_size - 1 - u;
    if (kxn_uvlen(body) == u) break;
  }
  ((KXN_G(uint8_t)*)out)[pos] = 0x0A;
  uint64_t p = pos + 1;
  kxn_pb_put_uv<true>(out, &p, body);
  (void)kxn_pb_walk<true>(P, C, KxnPEFrame{0, 0, (int16_t)si, P.st[si].enc_first, 0, 0, 0, r, 0, 0}, out, p);
}
