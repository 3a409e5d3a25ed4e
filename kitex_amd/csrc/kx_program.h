// kx_program.h — the compiled schema ("program") the device kernels interpret.
//
// kx_schema_create flattens the IDL (include/kxcodec.h kx_struct_desc[]) into this fixed-size,
// position-independent table. It is copied to HBM once per (schema, device) and staged into LDS by
// every workgroup (≈2.5 KB), where the per-lane record parser reads it with ds_read.
//
// Flattening rules (identical to the CPU oracle's):
//  * depth-first over the IDL, struct fields inlined; every struct occurrence is an "instance" with a
//    unique set of leaf columns (non-recursive schemas only, depth < 8);
//  * every optional / struct / container field gets a presence bit (Go nil-ability);
//  * "flat field" index = position of a field in the instance-ordered field table (<= 64 in total),
//    so a single 64-bit mask holds the isset state of a whole record (required-field check,
//    struct_tpl.go:124-145).
#pragma once
#include <stdint.h>

#define KXP_MAX_FIELDS 64
#define KXP_MAX_INST 16
#define KXP_MAX_COLS 32
#define KXP_NV_MAX 16  // var slots (BYTES / LIST columns; a LIST_BYTES column takes 2) per flat schema

enum : uint8_t { KXP_K_FIXED = 1, KXP_K_BYTES = 2, KXP_K_LIST = 3, KXP_K_STRUCT = 4,
                 KXP_K_LISTB = 5,   // list/set<string>: column LIST_BYTES, slots vslot (elements) + vslot2 (bytes)
                 KXP_K_MAP = 6,     // map<K,V>: field kind only; columns col (keys), col + 1 (values)
                 KXP_K_LSTRUCT = 7 };  // list/set<S>, S of fixed scalars: field kind only; columns col ..
                                       // col + width - 1 (one per field of S, mside 3, sel_* below)

struct KxpField {      // 16 B
  int16_t id;
  uint8_t ttype;       // wire type (thrift TType)
  uint8_t elem;        // LIST/SET element type
  int8_t col;          // leaf column, -1 for STRUCT
  int8_t child;        // STRUCT: child instance
  int8_t pbit;         // presence bit or -1
  int8_t enc_next;     // next flat field in this instance's encoder order, -1 at the end
  uint8_t kind;        // KXP_K_*
  uint8_t width;       // FIXED: value width; LIST: element width
  uint8_t vslot;       // var slot (BYTES/LIST), 0xff otherwise
  uint8_t inst;        // owning instance
  uint8_t req;         // KX_REQ_*
  uint8_t flags;       // bit0: protobuf bytes (no UTF-8 check)
  uint8_t pb_wt;       // protobuf wire type for this field
  int8_t pb_next;      // next root field in field-number order (protobuf encode), -1 at the end
};

struct KxpInst {       // 32 B
  uint64_t req_mask;      // required flat fields of this instance
  uint64_t subtree_mask;  // flat fields of this instance and all descendants
  uint64_t pres_mask;     // presence bits of fields strictly inside this instance's subtree
  int8_t first;           // first flat field
  int8_t nfields;
  int8_t enc_first;       // first flat field in encoder order (-1 if no fields)
  int8_t parent;          // parent instance, -1 for the root
  int8_t ret_pred;        // predictor to resume with in the parent after this struct's STOP
  int8_t self_field;      // flat field (in the parent) holding this instance
  uint16_t vslot_mask;    // var slots inside this instance's subtree (KXP_NV_MAX = 16 bits)
};

struct KxpCol {        // 16 B
  uint8_t kind;        // KXP_K_FIXED / BYTES / LIST / LISTB (a map side: LIST or LISTB)
  uint8_t width;
  uint8_t elem;        // LIST element type (BOOL needs normalisation); map side: this side's type
  uint8_t vslot;       // 0xff for FIXED; LISTB: the elements slot
  int8_t field;        // flat field
  uint8_t ttype;
  uint8_t vslot2;      // LISTB: the bytes slot, else 0xff
  uint8_t mside;       // 1: map keys, 2: map values, 3: a field of a list<struct> element, 0: neither
  int64_t defv;        // FIXED default (bits)
};

// Canonical plan: the byte layout every record written by the encoder has (encoder order, all
// non-optional fields present, nil-free structs). Executed as a straight line of steps; a record
// that deviates at any step is re-parsed by the generic field loop.
enum : uint8_t { KXP_S_FIXED = 1, KXP_S_BYTES = 2, KXP_S_LIST = 3, KXP_S_STRUCT = 4, KXP_S_END = 5,
                 KXP_S_PB_VARINT = 6, KXP_S_PB_FIXED64 = 7, KXP_S_PB_LEN = 8 };
#define KXP_MAX_STEPS 96

struct KxpStep {       // 8 B
  uint32_t hdr;        // expected field header bytes: ttype | id_hi << 8 | id_lo << 16
  uint8_t kind;        // KXP_S_*
  uint8_t width;       // FIXED value width / LIST element width
  int8_t col;          // FIXED: column
  uint8_t vslot;       // BYTES / LIST: var slot
};

struct KxProgram {
  KxpField f[KXP_MAX_FIELDS];
  KxpInst inst[KXP_MAX_INST];
  KxpCol col[KXP_MAX_COLS];
  uint32_t nfields, ninst, ncols, nvar;
  uint32_t npres;
  uint32_t sig;          // first 3 wire bytes of a canonically encoded record (little-endian packed)
  uint32_t sig_len;      // 3, or 1 when the root encodes no fields before STOP
  uint32_t is_pb;
  uint8_t var_col[KXP_NV_MAX];  // var slot -> column
  uint64_t fixed_min;    // minimum encoded record size (optional unset, var empty)
  uint32_t nsteps;       // canonical plan length, 0 = no canonical fast path
  int32_t pb_first;      // first root field in field-number order (protobuf encode), -1 if none
  uint64_t canon_pres;   // presence word of a canonical record
  uint32_t sig_ambig;    // the signature is also the first header of a nested struct: validate candidates
  uint32_t sig2_off;     // canonical record: offset of the second field header (0: not fixed)
  uint32_t sig2;         // ... and its 3 bytes (a cheap pre-check before a full canonical parse)
  uint32_t npbsteps;     // protobuf canonical plan length (root fields in number order), 0 = none
  KxpStep steps[KXP_MAX_STEPS];
  // Protobuf canonical plan: one step per root field in field-number order (proto.Marshal's order);
  // hdr = tag bytes (bits 0-15) | tag length (16-17) | bool (bit 24) | bytes, no UTF-8 check (25)
  KxpStep pbsteps[KXP_MAX_FIELDS];
  // list<struct> element fields, per column (mside 3): the field id in S, required (1) or not, and the
  // column of S's first field (the element walker scans S's fields sel_first .. sel_first + n - 1)
  int16_t sel_id[KXP_MAX_COLS];
  uint8_t sel_req[KXP_MAX_COLS];
  uint8_t sel_first[KXP_MAX_COLS];
  uint8_t sel_n[KXP_MAX_COLS];
  // canonical plan: encoded bytes of a canonical record besides its var payloads (headers, fixed values,
  // string lengths, list headers, STOPs): BLength = canon_fixed + the var steps' payload bytes
  uint64_t canon_fixed;
};

// The canonical plan as the index pass walks it (a kernel parameter: uniform, loaded into SGPRs once per
// wave): the record is a chain of segments, each a fixed-size run (field headers with their values, struct
// headers, STOPs) whose header bytes are checked at known offsets, then at most one var field (string or
// numeric list) whose length moves the next segment. R2: [8 i64 fields] s9 | [] s10 | [STOP].
#define KXF_SEG 4
#define KXF_CHK 12
struct KxpFastSeg {
  uint16_t flen;              // bytes of the fixed run
  uint8_t nchk;               // header checks in it
  uint8_t vkind;              // 0: no var field (the record ends), 1: string / binary, 2: numeric list
  uint8_t vslot;              // var slot
  uint8_t vwidth;             // list element width
  uint16_t pad;
  uint32_t vhdr;              // the var field's header (3 bytes)
  uint16_t choff[KXF_CHK];    // check offsets in the run, in groups of 4 (ngrp groups; padding checks pass)
  uint32_t chval[KXF_CHK];    // expected bytes: a 3-byte header, (bit 31) a 1-byte STOP, (bit 30) padding
};
struct KxpFast {
  uint32_t nseg;
  uint32_t ok;                // 0: the plan does not fit (the step interpreter runs instead)
  KxpFastSeg seg[KXF_SEG];
};

// host: the segment form of a program's canonical plan
static inline void kxp_fast_plan(const KxProgram& P, KxpFast& F) {
  F = KxpFast{};
  if (!P.nsteps) return;
  uint32_t off = 0;
  bool ok = true;
  KxpFastSeg* G = &F.seg[0];
  F.nseg = 1;
  auto check = [&](uint32_t v) {
    if (G->nchk >= KXF_CHK || off > 0xffff) { ok = false; return; }
    G->choff[G->nchk] = (uint16_t)off;
    G->chval[G->nchk++] = v;
  };
  auto pad_groups = [&]() {   // checks come in groups of 4: fill the last group with passing checks
    while (G->nchk % 4) {
      if (G->nchk >= KXF_CHK) { ok = false; return; }
      G->choff[G->nchk] = 0;
      G->chval[G->nchk++] = 0x40000000u;
    }
  };
  for (uint32_t k = 0; k < P.nsteps && ok; k++) {
    const KxpStep& st = P.steps[k];
    switch (st.kind) {
      case KXP_S_FIXED: check(st.hdr & 0xffffffu); off += 3u + st.width; break;
      case KXP_S_STRUCT: check(st.hdr & 0xffffffu); off += 3u; break;
      case KXP_S_END: check(0x80000000u); off += 1u; break;
      case KXP_S_BYTES: case KXP_S_LIST:
        if (off > 0xffff || F.nseg >= KXF_SEG) { ok = false; break; }
        pad_groups();
        G->flen = (uint16_t)off;
        G->vkind = st.kind == KXP_S_BYTES ? 1 : 2;
        G->vslot = st.vslot;
        G->vwidth = st.width;
        G->vhdr = st.hdr & 0xffffffu;
        G = &F.seg[F.nseg++];
        off = 0;
        break;
      default: ok = false;
    }
  }
  if (off > 0xffff) ok = false;
  pad_groups();
  G->flen = (uint16_t)off;
  F.ok = ok ? 1u : 0u;
}

// The canonical plan as the fast emit pass executes it (emit_fast_kernel, T_CANON tiles): per segment the
// fixed fields of its run (value offset after the 3-byte header, wire type, column) and at most one string
// field after the run. Every offset inside a segment is a constant, so a record's fixed values are read
// with no dependence on each other; only the string lengths chain the segments. Schemas whose canonical
// plan holds a numeric list, more than KXE_SEG - 1 strings or more than KXE_FIX fixed fields in one run
// take the general emit pass (ok = 0).
#define KXE_SEG 4
#define KXE_FIX 16
struct KxpEmitFix {           // 4 B
  uint16_t off;               // value offset in the segment (past the field header)
  uint8_t ttype;              // wire type (BOOL: b == 1; BYTE / I16 / I32 / I64 / DOUBLE: big-endian)
  uint8_t col;                // FIXED column
};
struct KxpEmitSeg {           // 72 B
  uint16_t flen;              // bytes of the fixed run (headers, values, struct headers, STOPs)
  uint8_t nfix;
  uint8_t vkind;              // 0: the record ends with this run, 1: a string / binary field follows
  uint8_t vslot;              // its var slot
  uint8_t vcol;               // and column
  uint16_t pad;
  KxpEmitFix fix[KXE_FIX];
};
struct KxpEmit {
  uint32_t ok, nseg;
  KxpEmitSeg seg[KXE_SEG];
};

// host: the emit form of a program's canonical plan
static inline void kxp_emit_plan(const KxProgram& P, KxpEmit& E) {
  E = KxpEmit{};
  if (!P.nsteps || P.is_pb) return;
  uint32_t off = 0;
  bool ok = true;
  KxpEmitSeg* G = &E.seg[0];
  E.nseg = 1;
  for (uint32_t k = 0; k < P.nsteps && ok; k++) {
    const KxpStep& st = P.steps[k];
    switch (st.kind) {
      case KXP_S_FIXED:
        if (G->nfix >= KXE_FIX || st.col < 0 || off + 3 > 0xffff ||
            !(st.width == 1 || st.width == 2 || st.width == 4 || st.width == 8)) { ok = false; break; }
        G->fix[G->nfix++] = KxpEmitFix{(uint16_t)(off + 3), (uint8_t)(st.hdr & 0xff), (uint8_t)st.col};
        off += 3u + st.width;
        break;
      case KXP_S_STRUCT: off += 3u; break;
      case KXP_S_END: off += 1u; break;
      case KXP_S_BYTES: {
        const uint32_t c = st.vslot < KXP_NV_MAX ? P.var_col[st.vslot] : 0xffu;
        if (E.nseg >= KXE_SEG || off > 0xffff || c >= KXP_MAX_COLS || P.col[c].kind != KXP_K_BYTES) { ok = false; break; }
        G->flen = (uint16_t)off;
        G->vkind = 1;
        G->vslot = st.vslot;
        G->vcol = (uint8_t)c;
        G = &E.seg[E.nseg++];
        off = 0;
        break;
      }
      default: ok = false;   // numeric lists: the general emit pass (its wave-cooperative copy)
    }
  }
  if (off > 0xffff) ok = false;
  G->flen = (uint16_t)off;
  E.ok = ok ? 1u : 0u;
}

static_assert(sizeof(KxpEmitSeg) == 72, "KxpEmitSeg layout");
static_assert(sizeof(KxpField) == 16, "KxpField layout");
static_assert(sizeof(KxpInst) == 32, "KxpInst layout");
static_assert(sizeof(KxpCol) == 16, "KxpCol layout");
static_assert(sizeof(KxpStep) == 8, "KxpStep layout");
