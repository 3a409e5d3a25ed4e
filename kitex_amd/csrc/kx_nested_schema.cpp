// kx_nested_schema.cpp — compile an IDL (kx_struct_desc[]) into the nested walker's program
// (kx_nested.h) and its column layout (include/kxcodec.h, "Nested schemas").
//
// Used for every schema the flat program (kx_schema.cpp) cannot hold. Layout rules (the CPU oracle
// restates them independently, oracle/kx_oracle.c kxo_nflatten):
//  * depth-first in IDL order; struct fields inlined (a struct field at level L puts its fields at L);
//  * a list / set / map opens an element domain at L + 1; a map's key columns come before its value
//    columns; an element domain whose elements have presence bits gets a u64 presence column after
//    its own columns;
//  * presence bits (optional, struct and container fields) and seen bits are numbered per instance
//    root (the record, or a container's element), in depth-first order;
//  * encoder order per struct: fixed-length fields first, IDL order inside each group
//    (reorderStructFields, tool/internal_pkg/pluginmode/thriftgo/patcher.go:503-522);
//  * a struct met again on its own path (a recursive type) is kept as its encoded bytes (KN_RAW).
#include <string.h>

#include <new>
#include <vector>

#include "kx_internal.h"
#include "kx_nested.h"

namespace {

int tsize(uint32_t t) {
  switch (t) {
    case KX_T_BOOL: case KX_T_BYTE: return 1;
    case KX_T_I16: return 2;
    case KX_T_I32: return 4;
    case KX_T_I64: case KX_T_DOUBLE: return 8;
    default: return 0;
  }
}

bool is_container(uint32_t t) { return t == KX_T_LIST || t == KX_T_SET || t == KX_T_MAP; }

struct TypeRef {  // a value type: wire type + the descriptor parts that refine it
  uint8_t ttype;
  uint8_t elem;   // LIST/SET: element type; MAP: key | value << 4
  int16_t child;  // struct index (STRUCT, list<STRUCT>, map<K, STRUCT>) or element-type struct
  uint16_t pbk;   // Kitex-Protobuf: proto kind of the value (elements / key) | map value kind << 8
};

struct RootB {    // an instance root under construction
  int level;
  int nsbit = 0, npbit = 0;
  int c_lo = 0, c_hi = 0;
  std::vector<KxnDflt> dfl;
  std::vector<int> structs;          // struct instances whose dfl ranges are relative to `dfl`
  std::vector<KxnSdef> sdf;
};

struct NB {
  const kx_struct_desc* structs;
  uint32_t nstructs;
  kx_schema* s;
  KxnProgram& P;
  std::vector<RootB> roots;
  std::vector<int> stack;            // struct indices on the current path (recursion)
  int16_t chain[3] = {-1, -1, -1};   // container cursors by level on the current path
  int16_t path[8] = {0};
  int depth = 0;                     // path length - 1
  int16_t top_field_ttype = 0;       // the record field on the current path
  bool pb = false;                   // Kitex-Protobuf: proto3 messages (kinds in default_bits, no defaults)
  int rc = KX_OK;

  int fail(int code) {
    if (!rc) rc = code;
    return -1;
  }

  int new_node() {
    if (P.nnodes >= KXN_MAX_NODES) return fail(KX_ERR_NOT_IMPLEMENTED);
    KxnNode& N = P.node[P.nnodes];
    memset(&N, 0, sizeof N);
    N.col = N.cur = N.a = N.b = N.root = N.rep_col = -1;
    return (int)P.nnodes++;
  }

  int new_cur() {
    if (P.ncur >= KXN_MAX_CUR) return fail(KX_ERR_NOT_IMPLEMENTED);
    return (int)P.ncur++;
  }

  // a leaf column at `level` (string: with its byte cursor bc), value type vt
  int new_col(int level, bool str, int bc, uint8_t vt, uint8_t flags, int16_t fid, int pbit) {
    if (s->ncols >= KX_MAX_COLUMNS) return fail(KX_ERR_NOT_IMPLEMENTED);
    const int c = (int)s->ncols++;
    kx_column_info& ci = s->info[c];
    memset(&ci, 0, sizeof ci);
    static const uint32_t kinds[2][3] = {{KX_COL_FIXED, KX_COL_LIST, KX_COL_LIST2},
                                         {KX_COL_BYTES, KX_COL_LIST_BYTES, KX_COL_LIST2_BYTES}};
    ci.kind = kinds[str ? 1 : 0][level];
    ci.width = str ? 1u : (uint32_t)tsize(vt & 15);
    if (flags & KX_ELEM_PRESENCE) ci.width = 8;
    ci.ttype = (uint8_t)top_field_ttype;
    ci.elem_ttype = (uint8_t)(level == 0 ? 0 : (vt | flags));
    if (level == 0 && vt == KX_T_STRUCT) ci.ttype = KX_T_STRUCT;  // a raw recursive struct at the top
    ci.field_id = fid;
    ci.presence_bit = pbit;
    ci.depth = (uint32_t)(depth < 0 ? 0 : depth);
    for (int d = 0; d <= depth && d < 8; d++) ci.path[d] = path[d];
    ci.level = (uint8_t)level;
    KxnCol& K = P.col[c];
    memset(&K, 0, sizeof K);
    K.kind = (uint8_t)ci.kind;
    K.width = (uint8_t)ci.width;
    K.level = (uint8_t)level;
    K.narr = (uint8_t)(level + (str ? 1 : 0));
    K.acur[0] = K.acur[1] = K.acur[2] = -1;
    for (int k = 0; k < level; k++) K.acur[k] = chain[k];
    if (str) K.acur[level] = (int16_t)bc;
    K.dcur = str ? (int16_t)bc : level > 0 ? chain[level - 1] : (int16_t)-1;
    K.elem = (uint8_t)(vt & 15);
    return c;
  }

  // resolve the element (or map value) type of a container from its descriptor
  bool elem_type(uint8_t t, int16_t child, TypeRef* out) {
    out->ttype = t;
    out->elem = 0;
    out->child = -1;
    if (t == KX_T_STRUCT) {
      if (child < 0 || (uint32_t)child >= nstructs) return false;
      out->child = child;
      return true;
    }
    if (is_container(t)) {  // described by field 0 of the one-field struct `child`
      if (pb) return false;   // proto3 has no containers of containers
      if (child < 0 || (uint32_t)child >= nstructs) return false;
      const kx_struct_desc& d = structs[child];
      if (d.nfields != 1 || !d.fields || d.fields[0].ttype != t) return false;
      out->elem = d.fields[0].elem_ttype;
      out->child = d.fields[0].child;
      return true;
    }
    return tsize(t) > 0 || t == KX_T_STRING;
  }

  // build the node for one value of type T at `level` inside root R. fid / pbit / def: the field (or
  // element) it belongs to. Returns the node index (-1 on failure, rc set).
  int value(const TypeRef& T, int level, int R, int16_t fid, int pbit, const kx_field_desc* fd) {
    if (level > 2) return fail(KX_ERR_NOT_IMPLEMENTED);
    const int X = new_node();
    if (X < 0) return -1;
    {
      KxnNode& N = P.node[X];
      N.ttype = T.ttype;
      N.level = (uint8_t)level;
      N.cur_lo = (uint16_t)P.ncur;
    }
    if (tsize(T.ttype) > 0) {
      if (pb && (T.ttype == KX_T_BYTE || T.ttype == KX_T_I16)) return fail(KX_ERR_NOT_IMPLEMENTED);  // no proto type
      if (pb && (T.pbk & 0xff) > KX_PB_UINT) return fail(KX_ERR_INVALID_ARG);
      const int c = new_col(level, false, -1, T.ttype, elem_flags, fid, pbit);
      if (c < 0) return -1;
      KxnNode& N = P.node[X];
      N.kind = KN_SCALAR;
      N.width = (uint8_t)tsize(T.ttype);
      N.col = (int16_t)c;
      N.pbk = (uint8_t)(T.pbk & 0xff);
      if (fd || (pb && pb_entry)) {  // a field: its default (proto3: zero; a map entry's key / value too)
        RootB& RB = roots[R];
        KxnDflt d;
        memset(&d, 0, sizeof d);
        d.col = (int16_t)c;
        d.width = (uint8_t)tsize(T.ttype);
        d.v = pb ? 0 : fd->default_bits;
        RB.dfl.push_back(d);
      }
    } else if (T.ttype == KX_T_STRING || (T.ttype == KX_T_STRUCT && recursive(T.child))) {
      const bool raw = T.ttype == KX_T_STRUCT;
      const int bc = new_cur();
      if (bc < 0) return -1;
      const int c = new_col(level, true, bc, raw ? KX_T_STRUCT : KX_T_STRING, elem_flags, fid, pbit);
      if (c < 0) return -1;
      KxnNode& N = P.node[X];
      N.kind = raw ? KN_RAW : KN_STRING;
      N.col = (int16_t)c;
      N.cur = (int16_t)bc;
      N.pbk = (uint8_t)(T.pbk & 0xff);
      if (pb && fd && (fd->reserved0 & KX_FIELD_BINARY)) N.pbk = KX_PB_BYTES;
      if (!pb && fd && !raw && (fd->reserved0 & KX_FIELD_STRING_DEFAULT) && fd->default_bits) {
        const char* dv = (const char*)(intptr_t)fd->default_bits;
        const size_t len = strlen(dv);
        if (len) {
          if (P.ndefb + len > KXN_MAX_DEFB) return fail(KX_ERR_NOT_IMPLEMENTED);
          KxnSdef d;
          memset(&d, 0, sizeof d);
          d.col = (int16_t)c;
          d.cur = (int16_t)bc;
          d.sbit = 0;  // set by the caller (the field's seen bit)
          d.off = P.ndefb;
          d.len = (uint32_t)len;
          memcpy(P.defb + P.ndefb, dv, len);
          P.ndefb += (uint32_t)len;
          roots[R].sdf.push_back(d);
          pending_sdef = (int)roots[R].sdf.size() - 1;
        }
      }
    } else if (T.ttype == KX_T_STRUCT) {
      const int si = strct(T.child, level, R);
      if (si < 0) return -1;
      KxnNode& N = P.node[X];
      N.kind = KN_STRUCT;
      N.a = (int16_t)si;
    } else if (T.ttype == KX_T_LIST || T.ttype == KX_T_SET || T.ttype == KX_T_MAP) {
      const bool map = T.ttype == KX_T_MAP;
      const int dc = new_cur();
      if (dc < 0) return -1;
      const int ER = new_root(level + 1);
      if (ER < 0) return -1;
      P.node[X].kind = map ? KN_MAP : KN_LIST;
      P.node[X].cur = (int16_t)dc;
      P.node[X].root = (int16_t)ER;
      P.root[ER].dcur = (int16_t)dc;
      const int16_t save = chain[level];
      chain[level] = (int16_t)dc;
      roots[ER].c_lo = (int)s->ncols;
      TypeRef K, V;
      const uint8_t saved_flags = elem_flags;
      if (map) {
        const uint8_t kt = T.elem & 15, vt = (uint8_t)(T.elem >> 4);
        if (tsize(kt) == 0 && kt != KX_T_STRING) return fail(KX_ERR_NOT_IMPLEMENTED);  // struct / container keys
        K = TypeRef{kt, 0, -1, (uint16_t)(T.pbk & 0xff)};
        if (!elem_type(vt, T.child, &V)) return fail(KX_ERR_NOT_IMPLEMENTED);
        V.pbk = (uint16_t)(T.pbk >> 8);
        if (pb && (kt == KX_T_DOUBLE || (kt == KX_T_STRING && (K.pbk & 0xff) == KX_PB_BYTES)))
          return fail(KX_ERR_INVALID_ARG);   // proto map keys: integral, bool or string
        elem_flags = 0;
        const bool saved_entry = pb_entry;
        pb_entry = true;
        const int kn = value(K, level + 1, ER, fid, pbit, nullptr);
        if (kn < 0) return -1;
        elem_flags = KX_ELEM_MAP_VALUE;
        const int vn = value(V, level + 1, ER, fid, pbit, nullptr);
        pb_entry = saved_entry;
        if (vn < 0) return -1;
        P.node[X].a = (int16_t)kn;
        P.node[X].b = (int16_t)vn;
        P.node[X].etype = kt;
        P.node[X].vtype = vt;
      } else {
        if (!elem_type(T.elem, T.child, &V)) return fail(KX_ERR_NOT_IMPLEMENTED);
        V.pbk = (uint16_t)(T.pbk & 0xff);
        elem_flags = 0;
        const bool saved_entry = pb_entry;
        pb_entry = false;
        const int en = value(V, level + 1, ER, fid, pbit, nullptr);
        pb_entry = saved_entry;
        if (en < 0) return -1;
        P.node[X].a = (int16_t)en;
        P.node[X].etype = T.elem;
      }
      elem_flags = saved_flags;
      if (roots[ER].npbit > 0) {  // presence words of the elements
        const int pc = new_col(level + 1, false, -1, 0, KX_ELEM_PRESENCE, fid, -1);
        if (pc < 0) return -1;
        P.root[ER].pres_col = (int16_t)pc;
      }
      roots[ER].c_hi = (int)s->ncols;
      if (roots[ER].c_hi == roots[ER].c_lo) return fail(KX_ERR_NOT_IMPLEMENTED);  // elements without columns
      P.node[X].rep_col = (int16_t)roots[ER].c_lo;
      chain[level] = save;
      close_root(ER);
      if (rc) return -1;
    } else {
      return fail(KX_ERR_INVALID_ARG);
    }
    P.node[X].cur_hi = (uint16_t)P.ncur;
    return X;
  }

  uint8_t elem_flags = 0;    // flags of the element columns being built (KX_ELEM_MAP_VALUE / STRUCT_FIELD)
  bool pb_entry = false;     // building a map entry's key / value (proto3: zero defaults when absent)
  int pending_sdef = -1;     // a string default just added (its seen bit is set by the field)

  bool recursive(int16_t child) {
    for (int x : stack)
      if (x == child) return true;
    return false;
  }

  int new_root(int level) {
    if (P.nroots >= KXN_MAX_ROOTS) return fail(KX_ERR_NOT_IMPLEMENTED);
    const int R = (int)P.nroots++;
    memset(&P.root[R], 0, sizeof(KxnRoot));
    P.root[R].level = (uint8_t)level;
    P.root[R].pres_col = -1;
    P.root[R].dcur = -1;
    roots.emplace_back();
    roots.back().level = level;
    return R;
  }

  // lay out a finished root's defaults and string defaults; struct ranges become absolute
  void close_root(int R) {
    RootB& RB = roots[R];
    if (P.ndfl + RB.dfl.size() > KXN_MAX_DFL || P.nsdf + RB.sdf.size() > KXN_MAX_SDF) {
      fail(KX_ERR_NOT_IMPLEMENTED);
      return;
    }
    const uint32_t base = P.ndfl;
    for (const KxnDflt& d : RB.dfl) P.dfl[P.ndfl++] = d;
    for (int si : RB.structs) {
      P.st[si].dfl_lo = (uint16_t)(P.st[si].dfl_lo + base);
      P.st[si].dfl_hi = (uint16_t)(P.st[si].dfl_hi + base);
    }
    KxnRoot& RT = P.root[R];
    RT.dfl_lo = (uint16_t)base;
    RT.dfl_hi = (uint16_t)P.ndfl;
    RT.sdf_lo = (uint16_t)P.nsdf;
    for (const KxnSdef& d : RB.sdf) P.sdf[P.nsdf++] = d;
    RT.sdf_hi = (uint16_t)P.nsdf;
  }

  // a struct instance at `level` in root R
  int strct(int16_t sidx, int level, int R) {
    if (sidx < 0 || (uint32_t)sidx >= nstructs) return fail(KX_ERR_INVALID_ARG);
    if (P.nstructs >= KXN_MAX_STRUCTS || depth >= 6) return fail(KX_ERR_NOT_IMPLEMENTED);
    const kx_struct_desc& sd = structs[sidx];
    if (sd.nfields && !sd.fields) return fail(KX_ERR_INVALID_ARG);
    if (P.nfields + sd.nfields > KXN_MAX_FIELDS) return fail(KX_ERR_NOT_IMPLEMENTED);
    const int si = (int)P.nstructs++;
    KxnStruct& S0 = P.st[si];
    memset(&S0, 0, sizeof S0);
    S0.first = (int16_t)P.nfields;
    S0.nfields = (int16_t)sd.nfields;
    S0.level = (uint8_t)level;
    S0.root = (int16_t)R;
    P.nfields += sd.nfields;
    RootB& RB0 = roots[R];
    S0.dfl_lo = (uint16_t)RB0.dfl.size();
    RB0.structs.push_back(si);
    stack.push_back(sidx);
    for (uint32_t i = 0; i < sd.nfields; i++) {
      const kx_field_desc& fd = sd.fields[i];
      for (uint32_t j = 0; j < i; j++)
        if (sd.fields[j].id == fd.id) return fail(KX_ERR_INVALID_ARG);
      if (fd.req > KX_REQ_OPTIONAL) return fail(KX_ERR_INVALID_ARG);
      const int fi = P.st[si].first + (int)i;
      KxnField& F = P.f[fi];
      memset(&F, 0, sizeof F);
      F.id = fd.id;
      F.ttype = fd.ttype;
      F.req = fd.req;
      F.pbit = -1;
      F.snap = -1;
      F.enc_next = -1;
      F.defv = fd.default_bits;
      RootB& RB = roots[R];
      if (RB.nsbit >= 64) return fail(KX_ERR_NOT_IMPLEMENTED);
      F.sbit = (uint8_t)RB.nsbit++;
      const bool nilable = fd.req == KX_REQ_OPTIONAL || fd.ttype == KX_T_STRUCT || is_container(fd.ttype);
      if (nilable) {
        if (RB.npbit >= 64) return fail(KX_ERR_NOT_IMPLEMENTED);
        F.pbit = (int8_t)RB.npbit++;
        P.st[si].pres_mask |= 1ull << F.pbit;
      }
      if (fd.req == KX_REQ_REQUIRED) P.st[si].req_mask |= 1ull << F.sbit;
      P.st[si].sub_mask |= 1ull << F.sbit;
      if (depth + 1 >= 8) return fail(KX_ERR_NOT_IMPLEMENTED);
      depth++;
      path[depth] = fd.id;
      const int16_t saved_top = top_field_ttype;
      if (depth == 0) top_field_ttype = fd.ttype;
      const uint8_t saved_flags = elem_flags;
      if (level > 0) elem_flags = (uint8_t)(elem_flags | KX_ELEM_STRUCT_FIELD);
      TypeRef T{fd.ttype, fd.elem_ttype, fd.child, (uint16_t)(pb ? (fd.default_bits & 0xffff) : 0)};
      if (pb && fd.req == KX_REQ_REQUIRED) return fail(KX_ERR_INVALID_ARG);   // proto3 has no required fields
      if (fd.ttype == KX_T_STRUCT && (fd.child < 0 || (uint32_t)fd.child >= nstructs)) return fail(KX_ERR_INVALID_ARG);
      if ((fd.ttype == KX_T_LIST || fd.ttype == KX_T_SET) && (fd.elem_ttype == KX_T_STRUCT || is_container(fd.elem_ttype)) &&
          (fd.child < 0 || (uint32_t)fd.child >= nstructs))
        return fail(KX_ERR_INVALID_ARG);
      pending_sdef = -1;
      const int X = value(T, level, R, fd.id, F.pbit, &fd);
      elem_flags = saved_flags;
      top_field_ttype = saved_top;
      depth--;
      if (X < 0) return -1;
      KxnField& F2 = P.f[fi];
      F2.node = (int16_t)X;
      if (pending_sdef >= 0) roots[R].sdf[pending_sdef].sbit = F2.sbit;
      pending_sdef = -1;
      const KxnNode& N = P.node[X];
      if (N.cur_hi > N.cur_lo) {
        if (P.nsnap + (N.cur_hi - N.cur_lo) > KXN_MAX_SNAP) return fail(KX_ERR_NOT_IMPLEMENTED);
        F2.snap = (int16_t)P.nsnap;
        P.nsnap += (uint32_t)(N.cur_hi - N.cur_lo);
      }
      if (N.kind == KN_STRUCT) {  // an inline struct's bits belong to this struct's subtree
        P.st[si].sub_mask |= P.st[N.a].sub_mask;
        P.st[si].pres_mask |= P.st[N.a].pres_mask;
      }
    }
    stack.pop_back();
    memset(P.fmap[si], 0xff, KXN_FMAP);
    for (uint32_t i = 0; i < sd.nfields; i++)
      if (sd.fields[i].id >= 0 && sd.fields[i].id < KXN_FMAP) P.fmap[si][sd.fields[i].id] = (uint8_t)i;
    P.st[si].dfl_hi = (uint16_t)roots[R].dfl.size();
    // encoder order: fixed-length fields first (patcher.go:503-522), IDL order inside each group;
    // Kitex-Protobuf: field-number order (proto.Marshal)
    int prev = -1;
    P.st[si].enc_first = -1;
    if (pb) {
      int last = INT32_MIN;
      for (int k = 0; k < P.st[si].nfields; k++) {
        int best = -1;
        for (int j = 0; j < P.st[si].nfields; j++) {
          const int fj = P.st[si].first + j;
          if (P.f[fj].id > last && (best < 0 || P.f[fj].id < P.f[best].id)) best = fj;
        }
        if (best < 0) break;
        last = P.f[best].id;
        if (prev < 0) P.st[si].enc_first = (int16_t)best;
        else P.f[prev].enc_next = (int16_t)best;
        prev = best;
      }
      return si;
    }
    for (int pass = 0; pass < 2; pass++)
      for (int k = 0; k < P.st[si].nfields; k++) {
        const int fi = P.st[si].first + k;
        if ((tsize(P.f[fi].ttype) > 0) != (pass == 0)) continue;
        if (prev < 0) P.st[si].enc_first = (int16_t)fi;
        else P.f[prev].enc_next = (int16_t)fi;
        prev = fi;
      }
    return si;
  }
};

// offsets entries of root R: every column below it with an array at R's level
void entries(KxnProgram& P, const NB& b, int R, int* rc) {
  const int L = P.root[R].level;
  KxnRoot& RT = P.root[R];
  RT.ent_lo = (uint16_t)P.nent;
  for (int c = b.roots[R].c_lo; c < b.roots[R].c_hi; c++) {
    const KxnCol& K = P.col[c];
    if (K.narr <= L) continue;
    if (P.nent >= KXN_MAX_ENT) { *rc = KX_ERR_NOT_IMPLEMENTED; return; }
    KxnEntry& E = P.ent[P.nent++];
    memset(&E, 0, sizeof E);
    E.col = (int16_t)c;
    E.arr = (uint8_t)L;
    E.cur = K.acur[L];
  }
  RT.ent_hi = (uint16_t)P.nent;
}

}  // namespace

kx_schema::~kx_schema() { delete nprog; }

int kx_build_nested(const kx_struct_desc* structs, uint32_t nstructs, kx_schema* s) {
  if (!structs || nstructs == 0 || nstructs > KX_MAX_STRUCTS) return KX_ERR_INVALID_ARG;
  KxnProgram* P = new (std::nothrow) KxnProgram();
  if (!P) return KX_ERR_INTERNAL;
  memset(P, 0, sizeof *P);
  s->ncols = 0;
  s->npres = 0;
  NB b{structs, nstructs, s, *P, {}, {}};
  b.pb = (structs[0].reserved0 & KX_STRUCT_PROTOBUF) != 0;
  P->pb = b.pb ? 1 : 0;
  const int R0 = b.new_root(0);
  b.roots[R0].c_lo = 0;
  b.depth = -1;  // the record's fields are at depth 0
  const int X = b.value(TypeRef{KX_T_STRUCT, 0, 0}, 0, R0, 0, -1, nullptr);
  int rc = b.rc;
  if (!rc && X < 0) rc = KX_ERR_INTERNAL;
  if (!rc) {
    b.roots[R0].c_hi = (int)s->ncols;
    b.close_root(R0);
    rc = b.rc;
  }
  if (!rc && s->ncols == 0) rc = KX_ERR_NOT_IMPLEMENTED;
  if (!rc)
    for (uint32_t R = 0; R < P->nroots && !rc; R++) entries(*P, b, (int)R, &rc);
  if (rc) {
    delete P;
    s->ncols = 0;
    return rc;
  }
  P->rec_node = (int16_t)X;
  P->ncols = s->ncols;
  P->npres = (uint32_t)b.roots[R0].npbit;
  s->npres = P->npres;
  delete s->nprog;
  s->nprog = P;
  return KX_OK;
}
