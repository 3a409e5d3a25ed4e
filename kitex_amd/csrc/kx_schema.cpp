// kx_schema.cpp — flatten an IDL (kx_struct_desc[]) into a KxProgram (see kx_program.h).
//
// Semantics follow the generated FastCodec: fields are matched by id and wire type
// (struct_tpl.go:75-101), fixed-length fields are written before the others in IDL order
// (reorderStructFields, tool/internal_pkg/pluginmode/thriftgo/patcher.go:503-522).
#include <string.h>

#include <algorithm>

#include "kx_internal.h"

namespace {

int type_size(uint8_t t) {
  switch (t) {
    case KX_T_BOOL: case KX_T_BYTE: return 1;
    case KX_T_I16: return 2;
    case KX_T_I32: return 4;
    case KX_T_I64: case KX_T_DOUBLE: return 8;
    default: return 0;
  }
}

int pb_wire_type(uint8_t t) {
  switch (t) {
    case KX_T_BOOL: case KX_T_BYTE: case KX_T_I16: case KX_T_I32: case KX_T_I64: return 0;
    case KX_T_DOUBLE: return 1;
    case KX_T_STRING: return 2;
    default: return 7;  // unsupported in the protobuf path
  }
}

struct PendField {
  const kx_field_desc* d;
  int col;    // leaf column or -1
  int child;  // child instance or -1
  int pbit;
};

struct Builder {
  const kx_struct_desc* structs;
  uint32_t nstructs;
  kx_schema* s;
  std::vector<std::vector<PendField>> inst_fields;
  std::vector<int> inst_parent, inst_self;  // self: index into parent's field list
  int stack[8];
  int64_t sel_def[KXP_MAX_COLS] = {};     // list<struct> element field defaults, per column

  int rec(int sidx, int depth, int parent, int self_idx, int16_t* path, int* out) {
    if (sidx < 0 || (uint32_t)sidx >= nstructs) return KX_ERR_INVALID_ARG;
    if (depth >= 8) return KX_ERR_NOT_IMPLEMENTED;
    for (int i = 0; i < depth; i++)
      if (stack[i] == sidx) return KX_ERR_NOT_IMPLEMENTED;  // recursive type: no flat columns
    if ((int)inst_fields.size() >= KXP_MAX_INST) return KX_ERR_NOT_IMPLEMENTED;
    const kx_struct_desc& sd = structs[sidx];
    if (sd.nfields && !sd.fields) return KX_ERR_INVALID_ARG;
    int me = (int)inst_fields.size();
    inst_fields.emplace_back();
    inst_parent.push_back(parent);
    inst_self.push_back(self_idx);
    stack[depth] = sidx;
    for (uint32_t i = 0; i < sd.nfields; i++) {
      const kx_field_desc* f = &sd.fields[i];
      for (uint32_t j = 0; j < i; j++)
        if (sd.fields[j].id == f->id) return KX_ERR_INVALID_ARG;
      if (f->req > KX_REQ_OPTIONAL) return KX_ERR_INVALID_ARG;
      PendField pf{f, -1, -1, -1};
      bool container = f->ttype == KX_T_STRUCT || f->ttype == KX_T_LIST || f->ttype == KX_T_SET ||
                       f->ttype == KX_T_MAP;
      if (f->req == KX_REQ_OPTIONAL || container) {
        if (s->npres >= 64) return KX_ERR_NOT_IMPLEMENTED;
        pf.pbit = (int)s->npres++;
      }
      path[depth] = f->id;
      kx_column_info ci;
      memset(&ci, 0, sizeof ci);
      ci.ttype = f->ttype;
      ci.field_id = f->id;
      ci.presence_bit = pf.pbit;
      ci.depth = (uint32_t)depth;
      for (int d = 0; d <= depth; d++) ci.path[d] = path[d];
      switch (f->ttype) {
        case KX_T_BOOL: case KX_T_BYTE: case KX_T_I16: case KX_T_I32: case KX_T_I64: case KX_T_DOUBLE:
          ci.kind = KX_COL_FIXED;
          ci.width = (uint32_t)type_size(f->ttype);
          break;
        case KX_T_STRING:
          // a non-empty string default: the nested program (kx_nested_schema.cpp)
          if ((f->reserved0 & KX_FIELD_STRING_DEFAULT) && f->default_bits && *(const char*)(intptr_t)f->default_bits)
            return KX_ERR_NOT_IMPLEMENTED;
          ci.kind = KX_COL_BYTES;
          ci.width = 1;
          break;
        case KX_T_LIST: case KX_T_SET:
          if (f->elem_ttype == KX_T_STRING) {  // list/set<string>: FieldFastReadList (struct_tpl.go:582-625)
            ci.kind = KX_COL_LIST_BYTES;
            ci.width = 1;
            ci.elem_ttype = KX_T_STRING;
            break;
          }
          if (f->elem_ttype == KX_T_STRUCT) {  // list/set<S> of fixed scalars: one LIST column per field of S
            if (f->child < 0 || (uint32_t)f->child >= nstructs || depth + 1 >= 8) return KX_ERR_NOT_IMPLEMENTED;
            const kx_struct_desc& es = structs[f->child];
            if (es.nfields == 0 || es.nfields > 8 || !es.fields || s->ncols + es.nfields > KXP_MAX_COLS)
              return KX_ERR_NOT_IMPLEMENTED;
            for (uint32_t k = 0; k < es.nfields; k++) {
              const kx_field_desc& g = es.fields[k];
              for (uint32_t j = 0; j < k; j++)
                if (es.fields[j].id == g.id) return KX_ERR_INVALID_ARG;
              if (type_size(g.ttype) == 0 || g.req == KX_REQ_OPTIONAL) return KX_ERR_NOT_IMPLEMENTED;
              if (g.req > KX_REQ_OPTIONAL) return KX_ERR_INVALID_ARG;
            }
            pf.col = (int)s->ncols;
            KxProgram& P = s->prog;
            for (uint32_t k = 0; k < es.nfields; k++) {
              const kx_field_desc& g = es.fields[k];
              kx_column_info cs = ci;
              cs.kind = KX_COL_LIST;
              cs.width = (uint32_t)type_size(g.ttype);
              cs.elem_ttype = (uint8_t)(g.ttype | KX_ELEM_STRUCT_FIELD);
              cs.field_id = g.id;
              cs.depth = (uint32_t)depth + 1;
              cs.path[depth + 1] = g.id;
              P.sel_id[s->ncols] = g.id;
              P.sel_req[s->ncols] = g.req == KX_REQ_REQUIRED ? 1 : 0;
              P.sel_first[s->ncols] = (uint8_t)pf.col;
              P.sel_n[s->ncols] = (uint8_t)es.nfields;
              sel_def[s->ncols] = g.default_bits;
              s->info[s->ncols++] = cs;
            }
            inst_fields[me].push_back(pf);
            continue;
          }
          if (type_size(f->elem_ttype) == 0) return KX_ERR_NOT_IMPLEMENTED;  // list<container>
          ci.kind = KX_COL_LIST;
          ci.width = (uint32_t)type_size(f->elem_ttype);
          ci.elem_ttype = f->elem_ttype;
          break;
        case KX_T_STRUCT: {
          int child = -1;
          // the child instance is created before this field is appended: remember the slot
          int slot = (int)inst_fields[me].size();
          inst_fields[me].push_back(pf);
          int rc = rec(f->child, depth + 1, me, slot, path, &child);
          if (rc) return rc;
          inst_fields[me][slot].child = child;
          continue;
        }
        case KX_T_MAP: {  // FieldFastReadMap (struct_tpl.go:466-533): a keys column and a values column
          const uint8_t kt = f->elem_ttype & 15, vt = (uint8_t)(f->elem_ttype >> 4);
          if ((type_size(kt) == 0 && kt != KX_T_STRING) || (type_size(vt) == 0 && vt != KX_T_STRING))
            return KX_ERR_NOT_IMPLEMENTED;  // map<.., struct|container>
          if (s->ncols + 2 > KXP_MAX_COLS) return KX_ERR_NOT_IMPLEMENTED;
          pf.col = (int)s->ncols;
          for (int side = 0; side < 2; side++) {
            const uint8_t t = side ? vt : kt;
            kx_column_info cm = ci;
            cm.kind = t == KX_T_STRING ? KX_COL_LIST_BYTES : KX_COL_LIST;
            cm.width = t == KX_T_STRING ? 1u : (uint32_t)type_size(t);
            cm.elem_ttype = (uint8_t)(t | (side ? KX_ELEM_MAP_VALUE : 0));
            s->info[s->ncols++] = cm;
          }
          inst_fields[me].push_back(pf);
          continue;
        }
        default:
          return KX_ERR_INVALID_ARG;
      }
      if (s->ncols >= KXP_MAX_COLS) return KX_ERR_NOT_IMPLEMENTED;
      pf.col = (int)s->ncols;
      s->info[s->ncols++] = ci;
      inst_fields[me].push_back(pf);
    }
    *out = me;
    return KX_OK;
  }
};

}  // namespace

int kx_build_program(const kx_struct_desc* structs, uint32_t nstructs, kx_schema* s) {
  if (!structs || nstructs == 0 || nstructs > KX_MAX_STRUCTS) return KX_ERR_INVALID_ARG;
  memset(&s->prog, 0, sizeof s->prog);
  s->ncols = 0;
  s->npres = 0;
  Builder b{structs, nstructs, s, {}, {}, {}, {}};
  int16_t path[8];
  int root = -1;
  int rc = b.rec(0, 0, -1, -1, path, &root);
  if (rc) return rc;

  KxProgram& P = s->prog;
  P.ninst = (uint32_t)b.inst_fields.size();
  // flat field indices: instances in creation order, fields contiguous per instance
  std::vector<int> first(P.ninst);
  int nf = 0;
  for (uint32_t i = 0; i < P.ninst; i++) {
    first[i] = nf;
    nf += (int)b.inst_fields[i].size();
  }
  if (nf > KXP_MAX_FIELDS) return KX_ERR_NOT_IMPLEMENTED;
  P.nfields = (uint32_t)nf;
  P.ncols = s->ncols;
  P.npres = s->npres;

  // var slots in column order (LIST_BYTES: the elements slot, then the bytes slot)
  int nvar = 0;
  for (uint32_t c = 0; c < s->ncols; c++) {
    KxpCol& kc = P.col[c];
    const kx_column_info& ci = s->info[c];
    kc.kind = ci.kind == KX_COL_FIXED ? KXP_K_FIXED : ci.kind == KX_COL_BYTES ? KXP_K_BYTES
            : ci.kind == KX_COL_LIST_BYTES ? KXP_K_LISTB : KXP_K_LIST;
    kc.width = (uint8_t)ci.width;
    kc.elem = (uint8_t)(ci.elem_ttype & 15);
    kc.ttype = ci.ttype;
    kc.vslot = 0xff;
    kc.vslot2 = 0xff;
    kc.mside = ci.ttype == KX_T_MAP ? ((ci.elem_ttype & KX_ELEM_MAP_VALUE) ? 2 : 1)
             : (ci.elem_ttype & KX_ELEM_STRUCT_FIELD) ? 3 : 0;
    if (ci.kind != KX_COL_FIXED) {
      if (nvar + (ci.kind == KX_COL_LIST_BYTES ? 2 : 1) > KXP_NV_MAX) return KX_ERR_NOT_IMPLEMENTED;
      kc.vslot = (uint8_t)nvar;
      P.var_col[nvar++] = (uint8_t)c;
      if (ci.kind == KX_COL_LIST_BYTES) {
        kc.vslot2 = (uint8_t)nvar;
        P.var_col[nvar++] = (uint8_t)c;
      }
    }
  }
  P.nvar = (uint32_t)nvar;

  for (uint32_t i = 0; i < P.ninst; i++) {
    KxpInst& I = P.inst[i];
    const auto& fl = b.inst_fields[i];
    I.first = (int8_t)first[i];
    I.nfields = (int8_t)fl.size();
    I.parent = (int8_t)b.inst_parent[i];
    I.self_field = b.inst_parent[i] >= 0 ? (int8_t)(first[b.inst_parent[i]] + b.inst_self[i]) : -1;
    // encoder order: fixed-length first, then the rest, IDL order inside each group
    std::vector<int> order;
    for (int pass = 0; pass < 2; pass++)
      for (int k = 0; k < (int)fl.size(); k++)
        if ((type_size(fl[k].d->ttype) > 0) == (pass == 0)) order.push_back(k);
    I.enc_first = order.empty() ? -1 : (int8_t)(first[i] + order[0]);
    for (int k = 0; k < (int)fl.size(); k++) {
      int ff = first[i] + k;
      KxpField& F = P.f[ff];
      const kx_field_desc* d = fl[k].d;
      F.id = d->id;
      F.ttype = d->ttype;
      F.elem = d->elem_ttype;
      F.col = (int8_t)fl[k].col;
      F.child = (int8_t)fl[k].child;
      F.pbit = (int8_t)fl[k].pbit;
      F.inst = (uint8_t)i;
      F.req = d->req;
      F.flags = d->reserved0;
      F.pb_wt = (uint8_t)pb_wire_type(d->ttype);
      F.enc_next = -1;
      if (fl[k].col >= 0 && P.col[fl[k].col].mside == 3) {  // list<struct>: width = fields of S
        const int c0 = fl[k].col, ns = P.sel_n[c0];
        F.kind = KXP_K_LSTRUCT;
        F.width = (uint8_t)ns;
        F.vslot = P.col[c0].vslot;
        for (int c = c0; c < c0 + ns; c++) {
          P.col[c].field = (int8_t)ff;
          P.col[c].defv = b.sel_def[c];
        }
      } else if (fl[k].col >= 0) {
        const KxpCol& kc = P.col[fl[k].col];
        F.kind = d->ttype == KX_T_MAP ? KXP_K_MAP : kc.kind;
        F.width = kc.width;
        F.vslot = kc.vslot;
        P.col[fl[k].col].field = (int8_t)ff;
        P.col[fl[k].col].defv = d->default_bits;
        if (d->ttype == KX_T_MAP) P.col[fl[k].col + 1].field = (int8_t)ff;
      } else {
        F.kind = KXP_K_STRUCT;
        F.width = 0;
        F.vslot = 0xff;
      }
      if (d->req == KX_REQ_REQUIRED) I.req_mask |= 1ull << ff;
    }
    for (size_t o = 0; o + 1 < order.size(); o++)
      P.f[first[i] + order[o]].enc_next = (int8_t)(first[i] + order[o + 1]);
  }
  // subtree masks (children are created after parents: walk in reverse creation order)
  for (int i = (int)P.ninst - 1; i >= 0; i--) {
    KxpInst& I = P.inst[i];
    uint64_t m = 0, pm = 0;
    uint16_t vm = 0;
    for (int k = 0; k < I.nfields; k++) {
      const KxpField& F = P.f[I.first + k];
      m |= 1ull << (I.first + k);
      if (F.pbit >= 0) pm |= 1ull << F.pbit;
      if (F.col >= 0)  // every var slot of the field's columns (map: both sides; LISTB: both slots)
        for (int cc = F.col; cc <= F.col + (F.kind == KXP_K_MAP ? 1 : F.kind == KXP_K_LSTRUCT ? F.width - 1 : 0); cc++) {
          if (P.col[cc].vslot != 0xff) vm |= (uint16_t)(1u << P.col[cc].vslot);
          if (P.col[cc].vslot2 != 0xff) vm |= (uint16_t)(1u << P.col[cc].vslot2);
        }
      if (F.child >= 0) {
        m |= P.inst[F.child].subtree_mask;
        pm |= P.inst[F.child].pres_mask;
        vm |= P.inst[F.child].vslot_mask;
      }
    }
    I.subtree_mask = m;
    I.pres_mask = pm;
    I.vslot_mask = vm;
  }
  for (uint32_t i = 1; i < P.ninst; i++) {
    KxpInst& I = P.inst[i];
    I.ret_pred = P.f[I.self_field].enc_next;
  }
  P.inst[0].ret_pred = -1;

  // protobuf encode order: root fields by field number (stable), proto.Marshal's deterministic order
  {
    const KxpInst& R0 = P.inst[0];
    std::vector<int> ord;
    for (int k = 0; k < R0.nfields; k++) ord.push_back(R0.first + k);
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return P.f[a].id < P.f[b].id; });
    P.pb_first = ord.empty() ? -1 : ord[0];
    for (size_t o = 0; o < ord.size(); o++) P.f[ord[o]].pb_next = o + 1 < ord.size() ? (int8_t)ord[o + 1] : (int8_t)-1;
    // canonical plan: every root field in number order, each a scalar or string with a tag of <= 2
    // bytes (field numbers < 2048); any other shape decodes through the generic field loop only
    P.npbsteps = 0;
    bool ok = P.ninst == 1 && !ord.empty();
    for (size_t o = 0; ok && o < ord.size(); o++) {
      const KxpField& F = P.f[ord[o]];
      if (F.pb_wt == 7 || F.id <= 0 || F.id >= 2048 || (F.kind != KXP_K_FIXED && F.kind != KXP_K_BYTES)) {
        ok = false;
        break;
      }
      const uint32_t tag = ((uint32_t)F.id << 3) | F.pb_wt;
      KxpStep& T = P.pbsteps[o];
      const uint32_t tb = tag < 0x80 ? tag : ((tag & 0x7f) | 0x80) | ((tag >> 7) << 8);
      T.hdr = tb | ((tag < 0x80 ? 1u : 2u) << 16) | ((F.ttype == KX_T_BOOL ? 1u : 0u) << 24) |
              ((F.flags & 1u) << 25);
      T.kind = F.pb_wt == 0 ? KXP_S_PB_VARINT : F.pb_wt == 1 ? KXP_S_PB_FIXED64 : KXP_S_PB_LEN;
      // the field's presence bit + 1 rides in the byte the step's kind leaves unused (LEN: width;
      // VARINT / FIXED64: vslot), so a present field costs the decoder one descriptor load
      T.width = T.kind == KXP_S_PB_LEN ? (uint8_t)(F.pbit + 1) : F.width;
      T.col = F.col;
      T.vslot = T.kind == KXP_S_PB_LEN ? F.vslot : (uint8_t)(F.pbit + 1);
    }
    if (ok) P.npbsteps = (uint32_t)ord.size();
  }

  // canonical first bytes of a record (speculative boundary signature)
  const KxpInst& R = P.inst[0];
  if (R.enc_first >= 0) {
    const KxpField& F = P.f[R.enc_first];
    P.sig = (uint32_t)F.ttype | ((uint32_t)((uint16_t)F.id >> 8) << 8) | ((uint32_t)(F.id & 0xff) << 16);
    P.sig_len = 3;
    // a nested struct whose encoder-first field has the same header makes every occurrence of that
    // struct a false record candidate (R3: Inner.x and R3.id are both `i64, id 1`)
    P.sig_ambig = 0;
    for (uint32_t i = 1; i < P.ninst; i++) {
      const int ef = P.inst[i].enc_first;
      if (ef < 0) continue;
      const KxpField& G = P.f[ef];
      const uint32_t h = (uint32_t)G.ttype | ((uint32_t)((uint16_t)G.id >> 8) << 8) | ((uint32_t)(G.id & 0xff) << 16);
      if (h == P.sig) P.sig_ambig = 1;
    }
    // a fixed-width, always-written first field puts the second field's header at a fixed offset
    P.sig2_off = 0;
    P.sig2 = 0;
    if (F.kind == KXP_K_FIXED && F.req != KX_REQ_OPTIONAL && F.enc_next >= 0) {
      const KxpField& G = P.f[F.enc_next];
      if (G.req != KX_REQ_OPTIONAL) {
        P.sig2_off = 3u + F.width;
        P.sig2 = (uint32_t)G.ttype | ((uint32_t)((uint16_t)G.id >> 8) << 8) | ((uint32_t)(G.id & 0xff) << 16);
      }
    }
  } else {
    P.sig = 0;
    P.sig_len = 1;
  }
  // minimum encoded size: non-optional fields with empty var data, nil structs = STOP
  uint64_t mn = 1;
  for (int k = 0; k < R.nfields; k++) {
    const KxpField& F = P.f[R.first + k];
    if (F.req == KX_REQ_OPTIONAL) continue;
    mn += 3;
    if (F.kind == KXP_K_FIXED) mn += F.width;
    else if (F.kind == KXP_K_BYTES) mn += 4;
    else if (F.kind == KXP_K_LIST || F.kind == KXP_K_LISTB || F.kind == KXP_K_LSTRUCT) mn += 5;
    else if (F.kind == KXP_K_MAP) mn += 6;
    else mn += 1;
  }
  P.fixed_min = mn;

  // canonical plan: depth-first in encoder order; any optional field disables the fast path
  // (its presence varies per record), as does a plan longer than KXP_MAX_STEPS
  struct PlanB {
    KxProgram& P;
    bool ok = true;
    uint32_t n = 0;
    uint64_t pres = 0;
    void push(const KxpStep& st) {
      if (n >= KXP_MAX_STEPS) { ok = false; return; }
      P.steps[n++] = st;
    }
    void inst(int i) {
      const KxpInst& I = P.inst[i];
      for (int f = I.enc_first; f >= 0; f = P.f[f].enc_next) {
        const KxpField& F = P.f[f];
        if (F.req == KX_REQ_OPTIONAL || F.kind == KXP_K_LISTB || F.kind == KXP_K_MAP || F.kind == KXP_K_LSTRUCT) {
          ok = false;
          return;
        }
        KxpStep st{};
        st.hdr = (uint32_t)F.ttype | ((uint32_t)((uint16_t)F.id >> 8) << 8) | ((uint32_t)(F.id & 0xff) << 16);
        st.col = F.col;
        st.vslot = F.vslot;
        st.width = F.width;
        if (F.pbit >= 0) pres |= 1ull << F.pbit;
        if (F.kind == KXP_K_FIXED) st.kind = KXP_S_FIXED;
        else if (F.kind == KXP_K_BYTES) st.kind = KXP_S_BYTES;
        else if (F.kind == KXP_K_LIST) st.kind = KXP_S_LIST;
        else st.kind = KXP_S_STRUCT;
        push(st);
        if (F.kind == KXP_K_STRUCT) inst(F.child);
        if (!ok) return;
      }
      KxpStep end{};
      end.kind = KXP_S_END;
      push(end);
    }
  } pb{P};
  pb.inst(0);
  P.nsteps = pb.ok ? pb.n : 0;
  // top header byte of a FIXED step = length of the run of consecutive FIXED steps starting there
  for (int k = (int)P.nsteps - 1; k >= 0; k--) {
    if (P.steps[k].kind != KXP_S_FIXED) continue;
    uint32_t run = 1;
    if (k + 1 < (int)P.nsteps && P.steps[k + 1].kind == KXP_S_FIXED) run += P.steps[k + 1].hdr >> 24;
    if (run > 255) run = 255;
    P.steps[k].hdr = (P.steps[k].hdr & 0xffffffu) | (run << 24);
  }
  P.canon_pres = pb.pres;
  P.canon_fixed = 0;
  for (uint32_t k = 0; k < P.nsteps; k++) {
    const KxpStep& st = P.steps[k];
    P.canon_fixed += st.kind == KXP_S_FIXED ? 3u + st.width : st.kind == KXP_S_BYTES ? 7u
                   : st.kind == KXP_S_LIST ? 8u : st.kind == KXP_S_STRUCT ? 3u : 1u;
  }
  s->ncols = P.ncols;
  return KX_OK;
}
