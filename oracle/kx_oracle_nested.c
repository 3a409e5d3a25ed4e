/* kx_oracle_nested.c — TEST INFRASTRUCTURE: CPU restatement of the generated FastRead / FastWriteNocopy
 * for nested schemas (include/kxcodec.h, "Nested schemas"), the parity checker of the device's nested
 * walker (kitex_amd/csrc/kx_nested.h). Never linked into the product.
 *
 * This is written the way the reference's generated code works, not the way the device does: a record
 * is FastRead into a value tree (the Go object: every struct a fresh NewX() with its defaults, a field's
 * value assigned each time it is read, so the last occurrence wins; struct_tpl.go:41-149, 405-450,
 * 466-625), then the tree is flattened into the column layout; encoding walks the schema over the
 * columns as FastWriteNocopy (struct_tpl.go:225-391; fixed-length fields first, patcher.go:503-522).
 * Skipped values use kxo_skip (codec_apache.go:191-293). */
#include <stdlib.h>
#include <string.h>

#include "kx_oracle.h"

enum { NK_SCALAR = 1, NK_STRING, NK_RAW, NK_STRUCT, NK_LIST, NK_MAP };

typedef struct onode onode;
typedef struct {
  const kx_field_desc* d;
  onode* node;
  int pbit;
} ofield;

struct onode {
  int kind, ttype, width, level;
  int col;                   /* SCALAR / STRING / RAW */
  int nfields;               /* STRUCT */
  ofield* fields;
  onode *elem, *key, *val;   /* LIST: elem; MAP: key, val */
  int etype, vtype;          /* LIST: element type; MAP: key / value types (encode headers) */
  int c_lo, c_hi;            /* LIST / MAP: columns of its elements */
  int pres_col;              /* LIST / MAP: presence words of its elements, -1 */
  const char* sdef;          /* STRING field: default */
  int pbk;                   /* Kitex-Protobuf: proto kind (KX_PB_*) of a scalar / string value */
};

#define NMAXN 512
typedef struct {
  const kx_struct_desc* structs;
  uint32_t nstructs;
  onode nodes[NMAXN];
  int nn;
  ofield fpool[512];
  int nf;
  kx_column_info cols[KX_MAX_COLUMNS];
  int ncols;
  int npres0;
  int stack[16], sdepth;
  int16_t path[8];
  int depth;
  int top_ttype;
  int flags;                 /* KX_ELEM_* of the columns being built */
  onode* chain[3];           /* containers by level on the current path */
  onode* cchain[KX_MAX_COLUMNS][3];  /* per column: the containers of its levels */
  int rc;
  onode* rec;
  int pb;                    /* Kitex-Protobuf schema (KX_STRUCT_PROTOBUF): kinds in default_bits */
} nplan;

static int tsz(int t) {
  switch (t) {
    case KX_T_BOOL: case KX_T_BYTE: return 1;
    case KX_T_I16: return 2;
    case KX_T_I32: return 4;
    case KX_T_I64: case KX_T_DOUBLE: return 8;
    default: return 0;
  }
}
static int is_cont(int t) { return t == KX_T_LIST || t == KX_T_SET || t == KX_T_MAP; }

static onode* nnew(nplan* p) {
  if (p->nn >= NMAXN) { p->rc = KX_ERR_NOT_IMPLEMENTED; return NULL; }
  onode* x = &p->nodes[p->nn++];
  memset(x, 0, sizeof *x);
  x->col = -1; x->pres_col = -1;
  return x;
}

static int ncol(nplan* p, int level, int str, int vt, int flags, int fid, int pbit) {
  if (p->ncols >= KX_MAX_COLUMNS) { p->rc = KX_ERR_NOT_IMPLEMENTED; return -1; }
  kx_column_info* ci = &p->cols[p->ncols];
  memset(ci, 0, sizeof *ci);
  static const uint32_t kinds[2][3] = {{KX_COL_FIXED, KX_COL_LIST, KX_COL_LIST2},
                                       {KX_COL_BYTES, KX_COL_LIST_BYTES, KX_COL_LIST2_BYTES}};
  ci->kind = kinds[str][level];
  ci->width = (flags & KX_ELEM_PRESENCE) ? 8u : str ? 1u : (uint32_t)tsz(vt);
  ci->ttype = (uint8_t)p->top_ttype;
  if (level == 0 && vt == KX_T_STRUCT) ci->ttype = KX_T_STRUCT;
  ci->elem_ttype = (uint8_t)(level == 0 ? 0 : (vt | flags));
  ci->field_id = (int16_t)fid;
  ci->presence_bit = pbit;
  ci->depth = (uint32_t)(p->depth < 0 ? 0 : p->depth);
  for (int d = 0; d <= p->depth && d < 8; d++) ci->path[d] = p->path[d];
  ci->level = (uint8_t)level;
  for (int k = 0; k < 3; k++) p->cchain[p->ncols][k] = k < level ? p->chain[k] : NULL;
  return p->ncols++;
}

/* the element (or map value) type of a container: (type, elem, child) */
static int etype_of(nplan* p, int t, int child, int* ot, int* oelem, int* ochild) {
  *ot = t; *oelem = 0; *ochild = -1;
  if (t == KX_T_STRUCT) {
    if (child < 0 || (uint32_t)child >= p->nstructs) return 0;
    *ochild = child;
    return 1;
  }
  if (is_cont(t)) {
    if (child < 0 || (uint32_t)child >= p->nstructs) return 0;
    const kx_struct_desc* d = &p->structs[child];
    if (d->nfields != 1 || !d->fields || d->fields[0].ttype != t) return 0;
    *oelem = d->fields[0].elem_ttype; *ochild = d->fields[0].child;
    return 1;
  }
  return tsz(t) > 0 || t == KX_T_STRING;
}

static onode* build(nplan* p, int t, int elem, int child, int level, int* npbit, int fid, int pbit,
                    const kx_field_desc* fd, int kinds);

static onode* build_struct(nplan* p, int sidx, int level, int* npbit) {
  onode* x = nnew(p);
  if (!x) return NULL;
  const kx_struct_desc* sd = &p->structs[sidx];
  if (sd->nfields && !sd->fields) { p->rc = KX_ERR_INVALID_ARG; return NULL; }
  if (p->nf + (int)sd->nfields > 512 || p->sdepth >= 16) { p->rc = KX_ERR_NOT_IMPLEMENTED; return NULL; }
  x->kind = NK_STRUCT; x->ttype = KX_T_STRUCT; x->level = level;
  x->nfields = (int)sd->nfields;
  x->fields = &p->fpool[p->nf];
  p->nf += (int)sd->nfields;
  p->stack[p->sdepth++] = sidx;
  for (uint32_t i = 0; i < sd->nfields; i++) {
    const kx_field_desc* f = &sd->fields[i];
    for (uint32_t j = 0; j < i; j++) if (sd->fields[j].id == f->id) { p->rc = KX_ERR_INVALID_ARG; return NULL; }
    if (f->req > KX_REQ_OPTIONAL || (p->pb && f->req == KX_REQ_REQUIRED)) { p->rc = KX_ERR_INVALID_ARG; return NULL; }
    ofield* F = &x->fields[i];
    F->d = f; F->pbit = -1;
    if (f->req == KX_REQ_OPTIONAL || f->ttype == KX_T_STRUCT || is_cont(f->ttype)) {
      if (*npbit >= 64) { p->rc = KX_ERR_NOT_IMPLEMENTED; return NULL; }
      F->pbit = (*npbit)++;
    }
    if (p->depth + 1 >= 8) { p->rc = KX_ERR_NOT_IMPLEMENTED; return NULL; }
    p->depth++;
    p->path[p->depth] = f->id;
    const int top = p->top_ttype, fl = p->flags;
    if (p->depth == 0) p->top_ttype = f->ttype;
    if (level > 0) p->flags |= KX_ELEM_STRUCT_FIELD;
    F->node = build(p, f->ttype, f->elem_ttype, f->child, level, npbit, f->id, F->pbit, f,
                    p->pb ? (int)(f->default_bits & 0xffff) : 0);
    p->flags = fl; p->top_ttype = top;
    p->depth--;
    if (!F->node) return NULL;
  }
  p->sdepth--;
  return x;
}

static onode* build(nplan* p, int t, int elem, int child, int level, int* npbit, int fid, int pbit,
                    const kx_field_desc* fd, int kinds) {
  if (level > 2) { p->rc = KX_ERR_NOT_IMPLEMENTED; return NULL; }
  if (tsz(t) > 0) {
    if (p->pb && (t == KX_T_BYTE || t == KX_T_I16)) { p->rc = KX_ERR_NOT_IMPLEMENTED; return NULL; }
    if (p->pb && (kinds & 0xff) > KX_PB_UINT) { p->rc = KX_ERR_INVALID_ARG; return NULL; }
    onode* x = nnew(p);
    if (!x) return NULL;
    x->kind = NK_SCALAR; x->ttype = t; x->width = tsz(t); x->level = level;
    x->pbk = kinds & 0xff;
    x->col = ncol(p, level, 0, t, p->flags, fid, pbit);
    return x->col < 0 ? NULL : x;
  }
  if (t == KX_T_STRUCT) {
    if (child < 0 || (uint32_t)child >= p->nstructs) { p->rc = KX_ERR_INVALID_ARG; return NULL; }
    int rec = 0;
    for (int k = 0; k < p->sdepth; k++) if (p->stack[k] == child) rec = 1;
    if (!rec) return build_struct(p, child, level, npbit);
  }
  if (t == KX_T_STRING || t == KX_T_STRUCT) {   /* a string, or a recursive struct kept as bytes */
    onode* x = nnew(p);
    if (!x) return NULL;
    x->kind = t == KX_T_STRING ? NK_STRING : NK_RAW; x->ttype = t; x->level = level;
    x->pbk = kinds & 0xff;
    if (p->pb && fd && (fd->reserved0 & 1)) x->pbk = KX_PB_BYTES;   /* KX_FIELD_BINARY */
    x->col = ncol(p, level, 1, t, p->flags, fid, pbit);
    if (!p->pb && fd && t == KX_T_STRING && (fd->reserved0 & KX_FIELD_STRING_DEFAULT) && fd->default_bits)
      x->sdef = (const char*)(intptr_t)fd->default_bits;
    return x->col < 0 ? NULL : x;
  }
  if (!is_cont(t)) { p->rc = KX_ERR_INVALID_ARG; return NULL; }
  onode* x = nnew(p);
  if (!x) return NULL;
  x->kind = t == KX_T_MAP ? NK_MAP : NK_LIST; x->ttype = t; x->level = level;
  x->c_lo = p->ncols;
  onode* saved_chain = p->chain[level];
  p->chain[level] = x;
  int epb = 0;                                  /* presence bits of the element instances */
  const int fl = p->flags;
  if (t == KX_T_MAP) {
    const int kt = elem & 15, vt = (elem >> 4) & 15;
    int vt2, ve, vc;
    if ((tsz(kt) == 0 && kt != KX_T_STRING) || !etype_of(p, vt, child, &vt2, &ve, &vc) ||
        (p->pb && is_cont(vt2))) {
      p->rc = KX_ERR_NOT_IMPLEMENTED; return NULL;
    }
    if (p->pb && (kt == KX_T_DOUBLE || (kt == KX_T_STRING && (kinds & 0xff) == KX_PB_BYTES))) {
      p->rc = KX_ERR_INVALID_ARG; return NULL;                    /* proto map keys */
    }
    p->flags = 0;
    x->key = build(p, kt, 0, -1, level + 1, &epb, fid, pbit, NULL, kinds & 0xff);
    if (!x->key) return NULL;
    p->flags = KX_ELEM_MAP_VALUE;
    x->val = build(p, vt2, ve, vc, level + 1, &epb, fid, pbit, NULL, (kinds >> 8) & 0xff);
    if (!x->val) return NULL;
    x->etype = kt; x->vtype = vt;
  } else {
    int et, ee, ec;
    if (!etype_of(p, elem, child, &et, &ee, &ec) || (p->pb && is_cont(et))) {
      p->rc = KX_ERR_NOT_IMPLEMENTED; return NULL;
    }
    p->flags = 0;
    x->elem = build(p, et, ee, ec, level + 1, &epb, fid, pbit, NULL, kinds & 0xff);
    if (!x->elem) return NULL;
    x->etype = elem;
  }
  p->flags = fl;
  if (epb > 0) {
    x->pres_col = ncol(p, level + 1, 0, 0, KX_ELEM_PRESENCE, fid, -1);
    if (x->pres_col < 0) return NULL;
  }
  x->c_hi = p->ncols;
  p->chain[level] = saved_chain;
  if (x->c_hi == x->c_lo) { p->rc = KX_ERR_NOT_IMPLEMENTED; return NULL; }
  return x;
}

static int nplan_build(nplan* p, const kx_struct_desc* structs, uint32_t nstructs) {
  memset(p, 0, sizeof *p);
  if (!structs || nstructs == 0 || nstructs > KX_MAX_STRUCTS) return KX_ERR_INVALID_ARG;
  p->structs = structs; p->nstructs = nstructs;
  p->pb = (structs[0].reserved0 & KX_STRUCT_PROTOBUF) != 0;
  p->depth = -1;
  int np = 0;
  p->rec = build_struct(p, 0, 0, &np);
  if (!p->rec) return p->rc ? p->rc : KX_ERR_INTERNAL;
  if (p->ncols == 0) return KX_ERR_NOT_IMPLEMENTED;
  p->npres0 = np;
  return KX_OK;
}

int kxo_nflatten(const kx_struct_desc* structs, uint32_t nstructs, kx_column_info* cols, uint32_t* ncols,
                 uint32_t* npresence) {
  nplan* p = (nplan*)malloc(sizeof(nplan));
  int rc = nplan_build(p, structs, nstructs);
  if (!rc) {
    memcpy(cols, p->cols, sizeof(kx_column_info) * (size_t)p->ncols);
    *ncols = (uint32_t)p->ncols; *npresence = (uint32_t)p->npres0;
  }
  free(p);
  return rc;
}

/* ---- FastRead into a value tree ---- */
typedef struct oval oval;
struct oval {
  int set;                   /* a field: read at least once */
  uint64_t u;                /* scalar */
  const uint8_t* p;          /* string / raw bytes */
  uint64_t len;
  oval* sub;                 /* STRUCT: its fields; LIST: elements; MAP: key, value pairs */
  uint64_t n;                /* LIST / MAP: elements / entries */
};

typedef struct { char* buf; size_t cap, used; } arena_t;

static void* aalloc(arena_t* a, size_t sz) {
  sz = (sz + 15) & ~(size_t)15;
  if (a->used + sz > a->cap) {   /* blocks are chained through a small header */
    size_t nc = sz + (1u << 20);
    char* b = (char*)malloc(nc + 16);
    if (!b) return NULL;
    *(char**)b = a->buf;
    a->buf = b; a->cap = nc; a->used = 16;
    a->cap += 16;
  }
  void* r = a->buf + a->used;
  a->used += sz;
  memset(r, 0, sz);
  return r;
}
static void areset(arena_t* a) {  /* keep the newest block, release the others */
  if (!a->buf) return;
  char* nx = *(char**)a->buf;
  while (nx) { char* t = *(char**)nx; free(nx); nx = t; }
  *(char**)a->buf = NULL;
  a->used = 16;
}
static void afree(arena_t* a) {
  while (a->buf) { char* nx = *(char**)a->buf; free(a->buf); a->buf = nx; }
  a->cap = a->used = 0;
}

static uint64_t rd_scalar(int t, const uint8_t* b) {
  switch (t) {
    case KX_T_BOOL: return b[0] == 1;           /* parity unpinned (bool bytes other than 0 / 1) */
    case KX_T_BYTE: return b[0];
    case KX_T_I16: return ((uint32_t)b[0] << 8) | b[1];
    case KX_T_I32: return ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
    default: {
      uint64_t v = 0;
      for (int k = 0; k < 8; k++) v = (v << 8) | b[k];
      return v;
    }
  }
}
static int32_t rd32(const uint8_t* b) { return (int32_t)rd_scalar(KX_T_I32, b); }

static int read_value(arena_t* A, const onode* x, const uint8_t* b, size_t len, size_t* off, oval* v);

/* StructLikeFastRead (struct_tpl.go:41-149) */
static int read_struct(arena_t* A, const onode* x, const uint8_t* b, size_t len, size_t* off, oval* v) {
  v->sub = (oval*)aalloc(A, sizeof(oval) * (size_t)(x->nfields ? x->nfields : 1));   /* NewX() */
  if (!v->sub) return KX_ERR_INTERNAL;
  for (;;) {
    if (len - *off < 1) return KX_ERR_EOF;
    const int t = b[*off];
    if (t == KX_T_STOP) { *off += 1; break; }
    if (len - *off < 3) return KX_ERR_EOF;
    const int16_t id = (int16_t)rd_scalar(KX_T_I16, b + *off + 1);
    *off += 3;
    int fi = -1;
    for (int k = 0; k < x->nfields; k++) if (x->fields[k].d->id == id) { fi = k; break; }
    if (fi < 0 || x->fields[fi].d->ttype != t) {       /* unknown / mismatched -> Skip */
      size_t u = 0;
      const int rc = kxo_skip(b + *off, len - *off, (uint8_t)t, 64, &u);
      if (rc) return rc;
      *off += u;
      continue;
    }
    oval nv;
    memset(&nv, 0, sizeof nv);
    const int rc = read_value(A, x->fields[fi].node, b, len, off, &nv);
    if (rc) return rc;
    nv.set = 1;
    v->sub[fi] = nv;                                    /* p.F = _field: the last occurrence wins */
  }
  for (int k = 0; k < x->nfields; k++)                  /* RequiredFieldNotSetError (:124-145) */
    if (x->fields[k].d->req == KX_REQ_REQUIRED && !v->sub[k].set) return KX_ERR_INVALID_DATA;
  return KX_OK;
}

static int read_value(arena_t* A, const onode* x, const uint8_t* b, size_t len, size_t* off, oval* v) {
  const size_t rem = len - *off;
  switch (x->kind) {
    case NK_SCALAR:
      if (rem < (size_t)x->width) return KX_ERR_EOF;
      v->u = rd_scalar(x->ttype, b + *off);
      *off += (size_t)x->width;
      return KX_OK;
    case NK_STRING: {                                   /* ReadString: a copy */
      if (rem < 4) return KX_ERR_EOF;
      const int32_t l = rd32(b + *off);
      if (l < 0) return KX_ERR_NEGATIVE_SIZE;
      if ((uint64_t)rem < 4 + (uint64_t)l) return KX_ERR_EOF;
      v->p = b + *off + 4; v->len = (uint64_t)l;
      *off += 4 + (size_t)l;
      return KX_OK;
    }
    case NK_RAW: {                                      /* a recursive struct: its bytes */
      size_t u = 0;
      const int rc = kxo_skip(b + *off, rem, KX_T_STRUCT, 64, &u);
      if (rc) return rc;
      v->p = b + *off; v->len = u;
      *off += u;
      return KX_OK;
    }
    case NK_STRUCT:                                     /* NewX() + FastRead (:405-422) */
      return read_struct(A, x, b, len, off, v);
    case NK_LIST: {                                     /* ReadListBegin: element type ignored (:587) */
      if (rem < 5) return KX_ERR_EOF;
      const int32_t n = rd32(b + *off + 1);
      if (n < 0) return KX_ERR_NEGATIVE_SIZE;
      *off += 5;
      const uint64_t cap = (uint64_t)n < len - *off + 1 ? (uint64_t)n : len - *off + 1;
      v->sub = (oval*)aalloc(A, sizeof(oval) * (size_t)(cap ? cap : 1));
      if (!v->sub) return KX_ERR_INTERNAL;
      for (int32_t j = 0; j < n; j++) {
        if ((uint64_t)j >= cap) return KX_ERR_EOF;      /* every element takes at least one byte */
        const int rc = read_value(A, x->elem, b, len, off, &v->sub[j]);
        if (rc) return rc;
      }
      v->n = (uint64_t)n;
      return KX_OK;
    }
    default: {                                          /* ReadMapBegin: key / value types ignored */
      if (rem < 6) return KX_ERR_EOF;
      const int32_t n = rd32(b + *off + 2);
      if (n < 0) return KX_ERR_NEGATIVE_SIZE;
      *off += 6;
      const uint64_t cap = (uint64_t)n < len - *off + 1 ? (uint64_t)n : len - *off + 1;
      v->sub = (oval*)aalloc(A, sizeof(oval) * 2 * (size_t)(cap ? cap : 1));
      if (!v->sub) return KX_ERR_INTERNAL;
      for (int32_t j = 0; j < n; j++) {
        if ((uint64_t)j >= cap) return KX_ERR_EOF;
        int rc = read_value(A, x->key, b, len, off, &v->sub[2 * j]);
        if (rc) return rc;
        rc = read_value(A, x->val, b, len, off, &v->sub[2 * j + 1]);
        if (rc) return rc;
      }
      v->n = (uint64_t)n;
      return KX_OK;
    }
  }
}

/* ---- the value tree -> columns: running counters per container domain and per string column ---- */
typedef struct {
  const nplan* p;
  const kx_columns* out;
  uint64_t dom[NMAXN];               /* per container node: elements so far */
  uint64_t bytes[KX_MAX_COLUMNS];    /* per string / raw column: bytes so far */
  int overflow;
  int failed;                        /* flattening a failed record: no string defaults */
} flat_t;

static int owide(const kx_column* c) { return c->offset_bytes == 8; }
static void* arr_ptr(const kx_column* c, int k) { return k == 0 ? c->offsets : k == 1 ? c->elem_offsets : c->sub_offsets; }
static void arr_set(flat_t* F, int c, int k, uint64_t i, uint64_t v) {
  const kx_column* col = &F->out->cols[c];
  void* a = arr_ptr(col, k);
  const uint64_t lim = k == 0 ? ~0ull : k == 1 ? col->elem_capacity : col->sub_capacity;
  if (!a || (k > 0 && i > lim)) { F->overflow = 1; return; }
  if (owide(col)) ((uint64_t*)a)[i] = v; else ((uint32_t*)a)[i] = (uint32_t)v;
}
static uint64_t arr_get(const kx_column* c, int k, uint64_t i) {
  const void* a = arr_ptr(c, k);
  return owide(c) ? ((const uint64_t*)a)[i] : ((const uint32_t*)a)[i];
}
static void val_set(flat_t* F, int c, uint64_t i, uint64_t v) {
  const kx_column* col = &F->out->cols[c];
  const uint32_t w = F->p->cols[c].width;
  if (F->p->cols[c].kind != KX_COL_FIXED && i >= col->capacity) { F->overflow = 1; return; }
  memcpy((uint8_t*)col->data + i * w, &v, w);   /* host little-endian */
}
static int n_arrays(const kx_column_info* ci) {
  const int str = ci->kind == KX_COL_BYTES || ci->kind == KX_COL_LIST_BYTES || ci->kind == KX_COL_LIST2_BYTES;
  return ci->level + str;
}

static void flat_value(flat_t* F, const onode* x, const oval* v, uint64_t e, uint64_t* pres);

/* instance e of struct x (absent fields: their defaults; v == NULL: a nil struct) */
static void flat_struct(flat_t* F, const onode* x, const oval* v, uint64_t e, uint64_t* pres) {
  for (int k = 0; k < x->nfields; k++) {
    const ofield* G = &x->fields[k];
    const oval* fv = v && v->sub && v->sub[k].set ? &v->sub[k] : NULL;
    if (fv) {
      if (G->pbit >= 0) *pres |= 1ull << G->pbit;
      flat_value(F, G->node, fv, e, pres);
      continue;
    }
    if (G->node->kind == NK_STRUCT) { flat_struct(F, G->node, NULL, e, pres); continue; }
    oval d;
    memset(&d, 0, sizeof d);
    if (G->node->kind == NK_SCALAR && !F->p->pb) d.u = (uint64_t)G->d->default_bits;   /* proto3: zero */
    if (G->node->kind == NK_STRING && G->node->sdef && !F->failed) {
      d.p = (const uint8_t*)G->node->sdef;
      d.len = strlen(G->node->sdef);
    }
    flat_value(F, G->node, &d, e, pres);
  }
}

/* element j of container x: an instance at level x->level + 1 */
static void flat_elem(flat_t* F, const onode* x, const onode* y, const oval* v, uint64_t e, uint64_t* epres) {
  if (y->kind == NK_STRUCT) flat_struct(F, y, v, e, epres);
  else flat_value(F, y, v, e, epres);
}

static void flat_value(flat_t* F, const onode* x, const oval* v, uint64_t e, uint64_t* pres) {
  const int L = x->level;
  switch (x->kind) {
    case NK_SCALAR:
      val_set(F, x->col, e, v->u);
      return;
    case NK_STRING: case NK_RAW: {
      const kx_column* col = &F->out->cols[x->col];
      const uint64_t at = F->bytes[x->col];
      arr_set(F, x->col, L, e, at);
      if (at + v->len > col->capacity) { F->overflow = 1; F->bytes[x->col] = at + v->len; return; }
      if (v->len) memcpy((uint8_t*)col->data + at, v->p, (size_t)v->len);
      F->bytes[x->col] = at + v->len;
      return;
    }
    case NK_STRUCT:
      flat_struct(F, x, v, e, pres);
      return;
    default: {
      const int xi = (int)(x - F->p->nodes);
      for (int c = x->c_lo; c < x->c_hi; c++) arr_set(F, c, L, e, F->dom[xi]);
      for (uint64_t j = 0; j < v->n; j++) {
        const uint64_t ej = F->dom[xi]++;
        uint64_t ep = 0;
        if (x->kind == NK_LIST) {
          flat_elem(F, x, x->elem, &v->sub[j], ej, &ep);
        } else {
          flat_elem(F, x, x->key, &v->sub[2 * j], ej, &ep);
          flat_elem(F, x, x->val, &v->sub[2 * j + 1], ej, &ep);
        }
        if (x->pres_col >= 0) val_set(F, x->pres_col, ej, ep);
      }
      return;
    }
  }
}

/* the closing entry of every offsets array */
static void flat_close(flat_t* F, uint64_t nrec) {
  const nplan* p = F->p;
  for (int c = 0; c < p->ncols; c++) {
    const kx_column_info* ci = &p->cols[c];
    const int na = n_arrays(ci);
    for (int k = 0; k < na; k++) {
      const uint64_t parent = k == 0 ? nrec : F->dom[p->cchain[c][k - 1] - p->nodes];
      const uint64_t target = k < ci->level ? F->dom[p->cchain[c][k] - p->nodes] : F->bytes[c];
      arr_set(F, c, k, parent, target);
    }
  }
}

static int ncheck_out(const nplan* p, const kx_columns* out) {
  if (!out || out->ncols != (uint32_t)p->ncols) return KX_ERR_INVALID_ARG;
  if (p->npres0 && !out->presence) return KX_ERR_INVALID_ARG;
  for (int c = 0; c < p->ncols; c++) {
    const kx_column* k = &out->cols[c];
    if (p->cols[c].kind == KX_COL_FIXED) { if (!k->data) return KX_ERR_INVALID_ARG; continue; }
    for (int a = 0; a < n_arrays(&p->cols[c]); a++) if (!arr_ptr(k, a)) return KX_ERR_INVALID_ARG;
  }
  return KX_OK;
}

/* decode (offsets mode: every record independently; concatenated: until the first failing record) */
int kxo_nthrift_decode(const kx_struct_desc* structs, uint32_t nstructs, const uint8_t* in, uint64_t in_len,
                       const uint64_t* offsets, uint64_t n, const kx_columns* out, uint8_t* record_status,
                       kx_status* st) {
  nplan* p = (nplan*)malloc(sizeof(nplan));
  int rc = nplan_build(p, structs, nstructs);
  if (!rc) rc = ncheck_out(p, out);
  if (rc) { free(p); return rc; }
  flat_t* F = (flat_t*)calloc(1, sizeof(flat_t));
  F->p = p; F->out = out;
  memset(st, 0, sizeof *st);
  arena_t A = {0};
  uint64_t pos = 0, r = 0;
  for (; r < n; r++) {
    const uint8_t* b;
    size_t len;
    if (offsets) {
      if (offsets[r] > offsets[r + 1] || offsets[r + 1] > in_len) { rc = KX_ERR_INVALID_ARG; goto fail_rec; }
      b = in + offsets[r]; len = (size_t)(offsets[r + 1] - offsets[r]);
    } else {
      b = in + pos; len = (size_t)(in_len - pos);
    }
    {
      oval v;
      memset(&v, 0, sizeof v);
      size_t off = 0;
      areset(&A);
      rc = read_struct(&A, p->rec, b, len, &off, &v);
      if (!rc) {
        uint64_t pres = 0;
        flat_struct(F, p->rec, &v, r, &pres);
        if (out->presence) out->presence[r] = pres;
        if (record_status) record_status[r] = 0;
        pos += off;
        continue;
      }
    }
  fail_rec:
    /* a failing record reads as all defaults with empty extents (its strings' defaults included) */
    if (record_status) record_status[r] = (uint8_t)rc;
    if (st->code == 0) { st->code = rc; st->record = r; st->offset = offsets ? offsets[r] : pos; }
    {
      uint64_t pres = 0;
      F->failed = 1;
      flat_struct(F, p->rec, NULL, r, &pres);
      F->failed = 0;
      if (out->presence) out->presence[r] = 0;
    }
    if (!offsets) break;
  }
  afree(&A);
  const uint64_t nrec = offsets ? n : r;
  st->n_records = nrec;
  st->consumed = offsets ? (n ? offsets[n] : 0) : pos;
  flat_close(F, offsets ? n : r);
  if (F->overflow && st->code == 0) st->code = KX_ERR_SIZE_LIMIT;
  for (int k = 0; k < 16; k++) st->var_total[k] = 0;
  rc = st->code;
  free(F);
  free(p);
  return rc;
}

/* ---- FastWriteNocopy from the columns ---- */
typedef struct {
  const nplan* p;
  const kx_columns* in;
  uint8_t* out;    /* NULL: size only */
  uint64_t pos;
} enc_t;

static void put(enc_t* E, uint64_t v, int nb) {
  if (E->out) for (int k = 0; k < nb; k++) E->out[E->pos + k] = (uint8_t)(v >> (8 * (nb - 1 - k)));
  E->pos += (uint64_t)nb;
}
static void put_bytes(enc_t* E, const uint8_t* s, uint64_t n) {
  if (E->out && n) memcpy(E->out + E->pos, s, (size_t)n);
  E->pos += n;
}
static uint64_t val_get(const enc_t* E, int c, uint64_t i) {
  const uint32_t w = E->p->cols[c].width;
  uint64_t v = 0;
  memcpy(&v, (const uint8_t*)E->in->cols[c].data + i * w, w);
  return v;
}

static void enc_value(enc_t* E, const onode* x, uint64_t e, uint64_t pres);

static void enc_struct(enc_t* E, const onode* x, uint64_t e, uint64_t pres) {
  /* encoder order: fixed-length fields first, IDL order inside each group (patcher.go:503-522) */
  for (int pass = 0; pass < 2; pass++)
    for (int k = 0; k < x->nfields; k++) {
      const ofield* G = &x->fields[k];
      if ((tsz(G->d->ttype) > 0) != (pass == 0)) continue;
      const int isset = G->pbit >= 0 && ((pres >> G->pbit) & 1);
      if (G->d->req == KX_REQ_OPTIONAL && !isset) continue;   /* optional: only when set */
      put(E, G->d->ttype, 1);                                  /* WriteFieldBegin */
      put(E, (uint16_t)G->d->id, 2);
      if (G->node->kind == NK_STRUCT && !isset) { put(E, KX_T_STOP, 1); continue; }  /* nil *T */
      enc_value(E, G->node, e, pres);
    }
  put(E, KX_T_STOP, 1);
}

static void enc_value(enc_t* E, const onode* x, uint64_t e, uint64_t pres) {
  const int L = x->level;
  const kx_columns* in = E->in;
  switch (x->kind) {
    case NK_SCALAR: {
      uint64_t v = val_get(E, x->col, e);
      if (x->ttype == KX_T_BOOL) v = (v & 0xff) ? 1 : 0;
      put(E, v, x->width);
      return;
    }
    case NK_STRING: case NK_RAW: {
      const kx_column* c = &in->cols[x->col];
      const uint64_t a = arr_get(c, L, e), z = arr_get(c, L, e + 1);
      if (x->kind == NK_STRING) put(E, z - a, 4);
      else if (z == a) { put(E, KX_T_STOP, 1); return; }
      put_bytes(E, (const uint8_t*)c->data + a, z - a);
      return;
    }
    case NK_STRUCT:
      enc_struct(E, x, e, pres);
      return;
    default: {
      const kx_column* rc = &in->cols[x->c_lo];
      const uint64_t a = arr_get(rc, L, e), z = arr_get(rc, L, e + 1);
      put(E, x->etype, 1);
      if (x->kind == NK_MAP) put(E, x->vtype, 1);
      put(E, z - a, 4);
      for (uint64_t j = a; j < z; j++) {
        const uint64_t ep = x->pres_col >= 0 ? val_get(E, x->pres_col, j) : 0;
        if (x->kind == NK_LIST) {
          enc_value(E, x->elem, j, ep);
        } else {
          enc_value(E, x->key, j, ep);
          enc_value(E, x->val, j, ep);
        }
      }
      return;
    }
  }
}

int kxo_nthrift_encode(const kx_struct_desc* structs, uint32_t nstructs, const kx_columns* in, uint64_t n,
                       uint8_t* out, uint64_t cap, uint64_t* sizes, uint64_t* offsets_out, uint64_t* total) {
  nplan* p = (nplan*)malloc(sizeof(nplan));
  int rc = nplan_build(p, structs, nstructs);
  if (!rc) rc = ncheck_out(p, in);
  if (rc) { free(p); return rc; }
  enc_t E = {p, in, NULL, 0};
  for (uint64_t r = 0; r < n; r++) {
    const uint64_t s0 = E.pos;
    enc_struct(&E, p->rec, r, in->presence ? in->presence[r] : 0);
    if (sizes) sizes[r] = E.pos - s0;
  }
  *total = E.pos;
  if (!out) { free(p); return KX_OK; }
  if (E.pos > cap) { free(p); return KX_ERR_SIZE_LIMIT; }
  E.out = out;
  E.pos = 0;
  for (uint64_t r = 0; r < n; r++) {
    if (offsets_out) offsets_out[r] = E.pos;
    enc_struct(&E, p->rec, r, in->presence ? in->presence[r] : 0);
  }
  if (offsets_out) offsets_out[n] = E.pos;
  free(p);
  return KX_OK;
}

/* ================================================================================================
 * Kitex-Protobuf (KX_STRUCT_PROTOBUF) nested messages: proto.Unmarshal into the same value tree, then the
 * same flattening; proto.Marshal from the columns. Restated from the published proto3 wire format and
 * message semantics as protobuf-go implements them (google.golang.org/protobuf encoding/protowire and
 * internal/impl; third-party, not vendored in the reference, which calls proto.Unmarshal / proto.Marshal
 * from pkg/remote/codec/protobuf/protobuf.go:64-134,209-216): a singular scalar or string is assigned
 * (last wins), a message merges (the same Go struct is read into again), a repeated field appends (packed
 * runs too), a map entry is inserted (kept in wire order here, key / value zero when absent), unknown
 * numbers and mismatched wire types are skipped, `string` must be UTF-8.
 * ================================================================================================ */
static int pb_wt_of(const onode* x) {
  if (x->kind != NK_SCALAR) return 2;
  if (x->ttype == KX_T_DOUBLE) return 1;
  if (x->pbk == KX_PB_FIXED) return x->ttype == KX_T_I32 ? 5 : 1;
  return 0;
}

static int pb_utf8(const uint8_t* s, uint64_t n) {   /* utf8.Valid */
  uint64_t i = 0;
  while (i < n) {
    uint8_t c = s[i];
    if (c < 0x80) { i++; continue; }
    int k; uint32_t cp;
    if ((c & 0xe0) == 0xc0) { k = 1; cp = c & 0x1f; }
    else if ((c & 0xf0) == 0xe0) { k = 2; cp = c & 0x0f; }
    else if ((c & 0xf8) == 0xf0) { k = 3; cp = c & 0x07; }
    else return 0;
    if (i + (uint64_t)k >= n) return 0;
    for (int j = 1; j <= k; j++) {
      uint8_t d = s[i + (uint64_t)j];
      if ((d & 0xc0) != 0x80) return 0;
      cp = (cp << 6) | (d & 0x3f);
    }
    if ((k == 1 && cp < 0x80) || (k == 2 && cp < 0x800) || (k == 3 && cp < 0x10000)) return 0;
    if (cp > 0x10ffff || (cp >= 0xd800 && cp <= 0xdfff)) return 0;
    i += (uint64_t)k + 1;
  }
  return 1;
}

static int pb_skip_val(int wt, const uint8_t* b, size_t len, size_t* off) {
  uint64_t v; size_t u;
  int rc;
  switch (wt) {
    case 0: rc = kxo_get_uvarint(b + *off, len - *off, &v, &u); if (rc) return rc; *off += u; return KX_OK;
    case 1: if (len - *off < 8) return KX_ERR_EOF; *off += 8; return KX_OK;
    case 2:
      rc = kxo_get_uvarint(b + *off, len - *off, &v, &u); if (rc) return rc;
      if (v > (uint64_t)(len - *off - u)) return KX_ERR_EOF;
      *off += u + (size_t)v; return KX_OK;
    case 5: if (len - *off < 4) return KX_ERR_EOF; *off += 4; return KX_OK;
    default: return KX_ERR_INVALID_DATA;
  }
}

/* one scalar (wire type matched): protowire.ConsumeVarint / ConsumeFixed32 / ConsumeFixed64, DecodeZigZag */
static int pb_scalar(const onode* x, const uint8_t* b, size_t len, size_t* off, uint64_t* out) {
  const int wt = pb_wt_of(x);
  uint64_t v = 0;
  if (wt == 0) {
    size_t u;
    int rc = kxo_get_uvarint(b + *off, len - *off, &v, &u);
    if (rc) return rc;
    *off += u;
    if (x->ttype == KX_T_BOOL) v = v != 0;
    else if (x->pbk == KX_PB_SINT && x->ttype == KX_T_I32) {
      int32_t d = (int32_t)(((uint32_t)v) >> 1) ^ -(int32_t)(((uint32_t)v) & 1);
      v = (uint64_t)(uint32_t)d;
    } else if (x->pbk == KX_PB_SINT) {
      v = (v >> 1) ^ (uint64_t)(-(int64_t)(v & 1));
    } else if (x->ttype == KX_T_I32) {
      v = (uint32_t)v;                                /* int32 / uint32 / enum: 32 bits */
    }
  } else {
    const size_t n = wt == 1 ? 8 : 4;
    if (len - *off < n) return KX_ERR_EOF;
    memcpy(&v, b + *off, n);                          /* little-endian host */
    *off += n;
  }
  *out = v;
  return KX_OK;
}

/* append one slot to a growable list of ovals (n used, cap in ->u of the list's holder) */
static oval* pb_push(arena_t* A, oval* list, int pair) {
  const uint64_t per = pair ? 2 : 1;
  if (list->n >= list->u) {
    const uint64_t nc = list->u ? list->u * 2 : 4;
    oval* ns = (oval*)aalloc(A, sizeof(oval) * (size_t)(nc * per));
    if (!ns) return NULL;
    if (list->n) memcpy(ns, list->sub, sizeof(oval) * (size_t)(list->n * per));
    list->sub = ns;
    list->u = nc;
  }
  oval* e = &list->sub[list->n * per];
  list->n++;
  return e;
}

static int pb_read_msg(arena_t* A, const onode* x, const uint8_t* b, size_t len, oval* v);

/* one value of node y (wire type matched): scalar / string assigned, message merged, raw bytes appended */
static int pb_read_value(arena_t* A, const onode* y, const uint8_t* b, size_t len, size_t* off, oval* v) {
  if (y->kind == NK_SCALAR) return pb_scalar(y, b, len, off, &v->u);
  uint64_t l; size_t u;
  int rc = kxo_get_uvarint(b + *off, len - *off, &l, &u);
  if (rc) return rc;
  *off += u;
  if (l > (uint64_t)(len - *off)) return KX_ERR_EOF;
  const uint8_t* s = b + *off;
  *off += (size_t)l;
  if (y->kind == NK_STRING) {
    if (y->pbk != KX_PB_BYTES && !pb_utf8(s, l)) return KX_ERR_INVALID_DATA;
    v->p = s; v->len = l;
    return KX_OK;
  }
  if (y->kind == NK_RAW) {                            /* a recursive message: its bytes, merged = concatenated */
    if (v->len && l) {
      uint8_t* nb = (uint8_t*)aalloc(A, (size_t)(v->len + l));
      if (!nb) return KX_ERR_INTERNAL;
      memcpy(nb, v->p, (size_t)v->len);
      memcpy(nb + v->len, s, (size_t)l);
      v->p = nb; v->len += l;
    } else if (l) {
      v->p = s; v->len = l;
    }
    return KX_OK;
  }
  return pb_read_msg(A, y, s, (size_t)l, v);          /* NK_STRUCT: merge into v */
}

/* proto.Unmarshal of one message body into v (merging with what v already holds) */
static int pb_read_msg(arena_t* A, const onode* x, const uint8_t* b, size_t len, oval* v) {
  if (!v->sub) {
    v->sub = (oval*)aalloc(A, sizeof(oval) * (size_t)(x->nfields ? x->nfields : 1));
    if (!v->sub) return KX_ERR_INTERNAL;
  }
  size_t off = 0;
  while (off < len) {
    uint64_t tag; size_t u;
    int rc = kxo_get_uvarint(b + off, len - off, &tag, &u);
    if (rc) return rc;
    off += u;
    const uint64_t num = tag >> 3;
    const int wt = (int)(tag & 7);
    if (num == 0 || num > 536870911ull) return KX_ERR_INVALID_DATA;
    int fi = -1;
    for (int k = 0; k < x->nfields; k++) if ((uint64_t)(int64_t)x->fields[k].d->id == num) { fi = k; break; }
    if (fi < 0) { rc = pb_skip_val(wt, b, len, &off); if (rc) return rc; continue; }
    const onode* y = x->fields[fi].node;
    oval* fv = &v->sub[fi];
    if (y->kind == NK_LIST) {
      const onode* e = y->elem;
      const int ewt = pb_wt_of(e);
      if (wt == ewt) {
        oval* ev = pb_push(A, fv, 0);
        if (!ev) return KX_ERR_INTERNAL;
        rc = pb_read_value(A, e, b, len, &off, ev);
        if (rc) return rc;
      } else if (wt == 2 && e->kind == NK_SCALAR) {   /* packed */
        uint64_t l;
        rc = kxo_get_uvarint(b + off, len - off, &l, &u);
        if (rc) return rc;
        off += u;
        if (l > (uint64_t)(len - off)) return KX_ERR_EOF;
        const size_t pend = off + (size_t)l;
        while (off < pend) {
          oval* ev = pb_push(A, fv, 0);
          if (!ev) return KX_ERR_INTERNAL;
          rc = pb_scalar(e, b, pend, &off, &ev->u);
          if (rc) return rc;
        }
      } else {
        rc = pb_skip_val(wt, b, len, &off);
        if (rc) return rc;
        continue;
      }
      fv->set = 1;
      continue;
    }
    if (y->kind == NK_MAP) {
      if (wt != 2) { rc = pb_skip_val(wt, b, len, &off); if (rc) return rc; continue; }
      uint64_t l;
      rc = kxo_get_uvarint(b + off, len - off, &l, &u);
      if (rc) return rc;
      off += u;
      if (l > (uint64_t)(len - off)) return KX_ERR_EOF;
      const uint8_t* eb = b + off;
      const size_t el = (size_t)l;
      off += el;
      oval* kv = pb_push(A, fv, 1);                   /* entry: key, value (zero when absent) */
      if (!kv) return KX_ERR_INTERNAL;
      size_t eo = 0;
      while (eo < el) {
        uint64_t et; size_t eu;
        rc = kxo_get_uvarint(eb + eo, el - eo, &et, &eu);
        if (rc) return rc;
        eo += eu;
        const uint64_t en = et >> 3;
        const int ew = (int)(et & 7);
        if (en == 0 || en > 536870911ull) return KX_ERR_INVALID_DATA;
        const onode* t = en == 1 ? y->key : en == 2 ? y->val : NULL;
        if (!t || ew != pb_wt_of(t)) { rc = pb_skip_val(ew, eb, el, &eo); if (rc) return rc; continue; }
        oval* tv = &kv[en == 1 ? 0 : 1];
        if (t->kind == NK_STRING) { tv->p = NULL; tv->len = 0; }   /* a repeated key / value: the last one */
        rc = pb_read_value(A, t, eb, el, &eo, tv);
        if (rc) return rc;
        tv->set = 1;
      }
      fv->set = 1;
      continue;
    }
    if (wt != pb_wt_of(y)) { rc = pb_skip_val(wt, b, len, &off); if (rc) return rc; continue; }
    rc = pb_read_value(A, y, b, len, &off, fv);
    if (rc) return rc;
    fv->set = 1;
  }
  return KX_OK;
}

/* record bodies: offsets mode (every record independently), or the Batch frames (0x0A, uvarint, body)
 * until the first record that fails */
int kxo_npb_decode(const kx_struct_desc* structs, uint32_t nstructs, const uint8_t* in, uint64_t in_len,
                   const uint64_t* offsets, uint64_t n, const kx_columns* out, uint8_t* record_status,
                   kx_status* st) {
  nplan* p = (nplan*)malloc(sizeof(nplan));
  int rc = nplan_build(p, structs, nstructs);
  if (!rc && !p->pb) rc = KX_ERR_INVALID_ARG;
  if (!rc) rc = ncheck_out(p, out);
  if (rc) { free(p); return rc; }
  flat_t* F = (flat_t*)calloc(1, sizeof(flat_t));
  F->p = p; F->out = out;
  memset(st, 0, sizeof *st);
  arena_t A = {0};
  uint64_t pos = 0, r = 0;
  for (; r < n; r++) {
    const uint8_t* b;
    size_t len;
    uint64_t fstart = pos;
    if (offsets) {
      if (offsets[r] > offsets[r + 1] || offsets[r + 1] > in_len) { rc = KX_ERR_INVALID_ARG; goto fail_rec; }
      b = in + offsets[r]; len = (size_t)(offsets[r + 1] - offsets[r]);
    } else {
      if (pos >= in_len) { rc = KX_ERR_EOF; goto fail_rec; }
      if (in[pos] != 0x0A) { rc = KX_ERR_INVALID_DATA; goto fail_rec; }
      uint64_t l; size_t u;
      rc = kxo_get_uvarint(in + pos + 1, (size_t)(in_len - pos - 1), &l, &u);
      if (!rc && l > in_len - pos - 1 - u) rc = KX_ERR_EOF;
      if (rc) goto fail_rec;
      b = in + pos + 1 + u; len = (size_t)l;
      pos += 1 + u + l;
    }
    {
      oval v;
      memset(&v, 0, sizeof v);
      areset(&A);
      rc = pb_read_msg(&A, p->rec, b, len, &v);
      if (!rc) {
        uint64_t pres = 0;
        flat_struct(F, p->rec, &v, r, &pres);
        if (out->presence) out->presence[r] = pres;
        if (record_status) record_status[r] = 0;
        continue;
      }
    }
  fail_rec:
    if (record_status) record_status[r] = (uint8_t)rc;
    if (st->code == 0) { st->code = rc; st->record = r; st->offset = offsets ? offsets[r] : fstart; }
    {
      uint64_t pres = 0;
      F->failed = 1;
      flat_struct(F, p->rec, NULL, r, &pres);
      F->failed = 0;
      if (out->presence) out->presence[r] = 0;
    }
    if (!offsets) { pos = fstart; break; }
  }
  afree(&A);
  st->n_records = offsets ? n : r;
  st->consumed = offsets ? (n ? offsets[n] : 0) : pos;
  flat_close(F, offsets ? n : r);
  if (F->overflow && st->code == 0) st->code = KX_ERR_SIZE_LIMIT;
  rc = st->code;
  free(F);
  free(p);
  return rc;
}

/* ---- proto.Marshal: field-number order, proto3 zero omission, packed repeated scalars, map entries
 * with key and value always written (columns' order); a message body's length from a size-only pass ---- */
static void pb_put_uv(enc_t* E, uint64_t v) {
  uint8_t t[10];
  const size_t u = kxo_put_uvarint(t, v);
  put_bytes(E, t, u);
}

/* the wire form of scalar node x at index e: returns the varint value, or sets *fixed (4 / 8) */
static uint64_t pb_wire(const enc_t* E, const onode* x, uint64_t e, int* fixed, int* zero) {
  const uint64_t v = val_get(E, x->col, e);
  const int wt = pb_wt_of(x);
  *zero = (x->ttype == KX_T_BOOL ? (v & 0xff) : v) == 0;
  *fixed = wt == 1 ? 8 : wt == 5 ? 4 : 0;
  if (*fixed) return v;
  if (x->ttype == KX_T_BOOL) return (v & 0xff) ? 1 : 0;
  if (x->ttype == KX_T_I32) {
    const int32_t s = (int32_t)(uint32_t)v;
    if (x->pbk == KX_PB_SINT) return (uint32_t)(((uint32_t)s << 1) ^ (uint32_t)(s >> 31));   /* EncodeZigZag */
    if (x->pbk == KX_PB_UINT) return (uint32_t)v;
    return (uint64_t)(int64_t)s;
  }
  if (x->pbk == KX_PB_SINT) return (v << 1) ^ (uint64_t)((int64_t)v >> 63);
  return v;
}

static void pb_put_scalar(enc_t* E, uint64_t v, int fixed) {
  if (fixed) { uint8_t t[8]; memcpy(t, &v, 8); put_bytes(E, t, (uint64_t)fixed); }
  else pb_put_uv(E, v);
}

static void pb_enc_msg(enc_t* E, const onode* x, uint64_t e, uint64_t pres);

/* a message body's size: the same walk with no output */
static uint64_t pb_msg_size(const enc_t* E, const onode* x, uint64_t e, uint64_t pres) {
  enc_t S = *E;
  S.out = NULL;
  S.pos = 0;
  pb_enc_msg(&S, x, e, pres);
  return S.pos;
}

static void pb_enc_entry(enc_t* E, const onode* m, uint64_t j, uint64_t ep) {
  const onode* kv[2] = {m->key, m->val};
  for (int k = 0; k < 2; k++) {
    const onode* t = kv[k];
    const uint64_t tag = ((uint64_t)(k + 1) << 3) | (uint64_t)pb_wt_of(t);
    pb_put_uv(E, tag);
    if (t->kind == NK_SCALAR) {
      int fixed, zero;
      const uint64_t v = pb_wire(E, t, j, &fixed, &zero);
      pb_put_scalar(E, v, fixed);
    } else if (t->kind == NK_STRING || t->kind == NK_RAW) {
      const kx_column* c = &E->in->cols[t->col];
      const uint64_t a = arr_get(c, t->level, j), z = arr_get(c, t->level, j + 1);
      pb_put_uv(E, z - a);
      put_bytes(E, (const uint8_t*)c->data + a, z - a);
    } else {
      pb_put_uv(E, pb_msg_size(E, t, j, ep));
      pb_enc_msg(E, t, j, ep);
    }
  }
}

static void pb_enc_msg(enc_t* E, const onode* x, uint64_t e, uint64_t pres) {
  /* field-number order */
  int order[256];
  int nf = x->nfields < 256 ? x->nfields : 256;
  for (int i = 0; i < nf; i++) order[i] = i;
  for (int i = 1; i < nf; i++)
    for (int j = i; j > 0 && x->fields[order[j]].d->id < x->fields[order[j - 1]].d->id; j--) {
      int t = order[j]; order[j] = order[j - 1]; order[j - 1] = t;
    }
  for (int k = 0; k < nf; k++) {
    const ofield* G = &x->fields[order[k]];
    const onode* y = G->node;
    const int isset = G->pbit >= 0 && ((pres >> G->pbit) & 1);
    const int optional = G->d->req == KX_REQ_OPTIONAL;
    const uint64_t num = (uint64_t)(uint16_t)G->d->id;
    if (y->kind == NK_SCALAR) {
      int fixed, zero;
      const uint64_t v = pb_wire(E, y, e, &fixed, &zero);
      if (optional ? !isset : zero) continue;
      pb_put_uv(E, (num << 3) | (uint64_t)pb_wt_of(y));
      pb_put_scalar(E, v, fixed);
    } else if (y->kind == NK_STRING || y->kind == NK_RAW) {
      const kx_column* c = &E->in->cols[y->col];
      const uint64_t a = arr_get(c, y->level, e), z = arr_get(c, y->level, e + 1);
      if (y->kind == NK_RAW ? !isset : (optional ? !isset : z == a)) continue;
      pb_put_uv(E, (num << 3) | 2);
      pb_put_uv(E, z - a);
      put_bytes(E, (const uint8_t*)c->data + a, z - a);
    } else if (y->kind == NK_STRUCT) {
      if (!isset) continue;                                    /* nil message */
      pb_put_uv(E, (num << 3) | 2);
      pb_put_uv(E, pb_msg_size(E, y, e, pres));
      pb_enc_msg(E, y, e, pres);
    } else {
      const kx_column* rc = &E->in->cols[y->c_lo];
      const uint64_t a = arr_get(rc, y->level, e), z = arr_get(rc, y->level, e + 1);
      if (a == z) continue;
      if (y->kind == NK_LIST && y->elem->kind == NK_SCALAR) {  /* packed */
        uint64_t body = 0;
        uint8_t t[10];
        for (uint64_t j = a; j < z; j++) {
          int fixed, zero;
          const uint64_t v = pb_wire(E, y->elem, j, &fixed, &zero);
          body += fixed ? (uint64_t)fixed : kxo_put_uvarint(t, v);
        }
        pb_put_uv(E, (num << 3) | 2);
        pb_put_uv(E, body);
        for (uint64_t j = a; j < z; j++) {
          int fixed, zero;
          const uint64_t v = pb_wire(E, y->elem, j, &fixed, &zero);
          pb_put_scalar(E, v, fixed);
        }
        continue;
      }
      for (uint64_t j = a; j < z; j++) {
        const uint64_t ep = y->pres_col >= 0 ? val_get(E, y->pres_col, j) : 0;
        pb_put_uv(E, (num << 3) | 2);
        if (y->kind == NK_LIST) {
          const onode* el = y->elem;
          if (el->kind == NK_STRING || el->kind == NK_RAW) {
            const kx_column* c = &E->in->cols[el->col];
            const uint64_t sa = arr_get(c, el->level, j), sb = arr_get(c, el->level, j + 1);
            pb_put_uv(E, sb - sa);
            put_bytes(E, (const uint8_t*)c->data + sa, sb - sa);
          } else {
            pb_put_uv(E, pb_msg_size(E, el, j, ep));
            pb_enc_msg(E, el, j, ep);
          }
        } else {
          enc_t S = *E;
          S.out = NULL; S.pos = 0;
          pb_enc_entry(&S, y, j, ep);
          pb_put_uv(E, S.pos);
          pb_enc_entry(E, y, j, ep);
        }
      }
    }
  }
}

/* n records as the body of `message Batch { repeated Rec recs = 1; }`; offsets_out[r] = body start of
 * record r (as kxo_pb_encode), offsets_out[n] = total */
int kxo_npb_encode(const kx_struct_desc* structs, uint32_t nstructs, const kx_columns* in, uint64_t n,
                   uint8_t* out, uint64_t cap, uint64_t* offsets_out, uint64_t* total) {
  nplan* p = (nplan*)malloc(sizeof(nplan));
  int rc = nplan_build(p, structs, nstructs);
  if (!rc && !p->pb) rc = KX_ERR_INVALID_ARG;
  if (!rc) rc = ncheck_out(p, in);
  if (rc) { free(p); return rc; }
  enc_t E = {p, in, NULL, 0};
  uint64_t pos = 0;
  for (uint64_t r = 0; r < n; r++) {
    const uint64_t pres = in->presence ? in->presence[r] : 0;
    const uint64_t body = pb_msg_size(&E, p->rec, r, pres);
    uint8_t t[10];
    const size_t u = kxo_put_uvarint(t, body);
    if (out && pos + 1 + u + body <= cap) {
      out[pos] = 0x0A;
      memcpy(out + pos + 1, t, u);
      E.out = out;
      E.pos = pos + 1 + u;
      pb_enc_msg(&E, p->rec, r, pres);
      E.out = NULL;
    }
    if (offsets_out) offsets_out[r] = pos + 1 + u;
    pos += 1 + u + body;
  }
  if (offsets_out) offsets_out[n] = pos;
  *total = pos;
  free(p);
  return out && pos > cap ? KX_ERR_SIZE_LIMIT : KX_OK;
}
