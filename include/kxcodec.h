/*
 * kxcodec.h — C-ABI of the MI355X batch payload codec (libkxcodec.so).
 *
 * This is the drop-in boundary for Kitex's payload-codec hot path. Every entry point is plain C:
 * pointers + sizes, no exceptions, no torch/HIP C++ types (streams travel as `void*` = hipStream_t).
 * Device pointers are caller-owned hipMalloc'd memory unless a comment says "host".
 *
 * Reference interfaces each entry point replaces (paths relative to cloudwego/kitex):
 *   kx_schema_create ............ the generated per-type FastCodec trio is driven by the IDL; the schema
 *                                 is the flattened IDL (pkg/generic/descriptor/descriptor.go:64-80 model,
 *                                 tool/internal_pkg/pluginmode/thriftgo/struct_tpl.go:41-391 semantics)
 *   kx_thrift_decode_batch ...... thrift.FastCodec.FastRead (internal/mocks/thrift/k-mock.go:39-114,
 *                                 template struct_tpl.go:41-149) applied to N records, as called from
 *                                 fastUnmarshal (pkg/remote/codec/thrift/codec_fast.go:60-82) when the
 *                                 message lengths are known (offsets != NULL), or as the element loop of
 *                                 a list<Struct> (FieldFastReadList, struct_tpl.go:582-625) when the
 *                                 records are concatenated (offsets == NULL)
 *   kx_thrift_skip_batch ........ the skip decoder netpollSkipDecoder.SkipStruct/skipType
 *                                 (pkg/remote/codec/thrift/codec_apache.go:166-293) over N records
 *   kx_thrift_split_points ...... the same skip over one concatenated batch, keeping only the G + 1
 *                                 record boundaries that cut it into G shards of equal record counts
 *                                 (SURVEY.md §8e pass A; the reference's caller-side partition)
 *   kx_thrift_encoded_size_batch  thrift.FastCodec.BLength (k-mock.go:201-210; struct_tpl.go:266-391)
 *   kx_thrift_encode_batch ...... thrift.FastCodec.FastWriteNocopy (k-mock.go:190-199; struct_tpl.go:225-264,
 *                                 field reorder pkg tool/.../thriftgo/patcher.go:503-522)
 *   kx_pb_decode_batch .......... proto.Unmarshal of the Kitex-Protobuf body
 *                                 (pkg/remote/codec/protobuf/protobuf.go:209-216 -> service.go:358-365)
 *   kx_pb_encoded_size_batch .... proto.Size of each record + its Batch frame header
 *   kx_pb_encode_batch .......... proto.Marshal of the Kitex-Protobuf body (protobuf.go:64-134,
 *                                 deterministic field-number order) as a `repeated Rec recs = 1` stream
 *   kx_host_decode_batch ........ fastUnmarshal end to end from host (netpoll) memory: pinned H2D ->
 *                                 decode -> D2H (codec_fast.go:60-82 with the Next(dataLen) slice);
 *                                 kx_host_pb_decode_batch the same for protobufCodec.Unmarshal bodies
 *   kx_host_encode_batch ........ fastMarshal end to end to host memory: H2D of the columns -> encode ->
 *                                 D2H of the wire (codec_fast.go:40-58; thrift.go:106-160); kx_host_pb_
 *                                 encode_batch the same for protobufCodec.Marshal (protobuf.go:64-134)
 *   kx_shard_meta / kx_concat_plan / kx_concat_rebase: the concatenation of record-range shards decoded
 *                                 on several GPUs into one (the reference has no
 *                                 multi-device path, its caller partitions: pkg/remote/payload_codec.go:29-33)
 *   kx_thrift_encode_messages ... fastMarshal (codec_fast.go:40-58) over N messages: MessageBegin + Args wrapper
 *                                 + record + STOP on the device
 *   kx_thrift_decode_messages ... thriftCodec.Unmarshal over N framed messages (thrift.go:180-225):
 *                                 MessageBegin + Args{1: req} (k-mock.go:422-517) on the device
 *   kx_pb_decode_messages ....... protobufCodec.Unmarshal over N framed messages (protobuf.go:136-216)
 *   kx_crc32c_batch ............. crcPayloadValidator.Generate / getCRC32C (pkg/remote/codec/validate.go:
 *                                 183-217) over N payloads
 *   kx_frame_crc32c_validate .... payloadChecksumValidate + crcPayloadValidator.Validate (validate.go:91-127,
 *                                 190-201) of N TTHeader frames, as DecodeMeta runs it (default_codec.go:205-209)
 *   kx_thrift_raw_messages ...... binaryThriftCodec.Unmarshal (pkg/generic/binarythrift_codec.go:83-115,
 *                                 readBinaryMethod :185-199) over N raw messages; kx_thrift_set_seqids =
 *                                 SetSeqID (:117-175) in place
 *   kx_grpc_frame_scan .......... decodeGRPCFrame (pkg/remote/codec/grpc/grpc_compress.go:37-60) over N
 *                                 messages; kx_*_decode_grpc = grpcCodec.Decode bodies (grpc.go:202-270)
 *   kx_ctx_set_crc32c_check ..... CodecConfig{CRC32Check: true} (default_codec.go:70-92) for kx_*_decode_frames
 *   kx_strerror ................. error text; codes mirror pkg/remote/codec/perrors/protocol_error.go:28-36
 */
#ifndef KXCODEC_H_
#define KXCODEC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KX_ABI_VERSION 7  /* 7: the kx_host_* entries take every schema and report per-record codes
                             (record_status); 6: shard concatenation (kx_shard_meta, kx_concat_plan, kx_concat_rebase);
                             5: kx_status.var_total holds 16 var slots; kx_thrift_split_points */

/* ---- Thrift TType ids (gopkg protocol/thrift; pinned by pkg/protocol/bthrift/binary_test.go) ---- */
enum {
  KX_T_STOP = 0, KX_T_VOID = 1, KX_T_BOOL = 2, KX_T_BYTE = 3, KX_T_DOUBLE = 4,
  KX_T_I16 = 6, KX_T_I32 = 8, KX_T_I64 = 10, KX_T_STRING = 11, KX_T_STRUCT = 12,
  KX_T_MAP = 13, KX_T_SET = 14, KX_T_LIST = 15
};

/* ---- Thrift message types (WriteMessageBegin, binary_test.go:387-457) ---- */
enum { KX_MSG_CALL = 1, KX_MSG_REPLY = 2, KX_MSG_EXCEPTION = 3, KX_MSG_ONEWAY = 4 };

/* ---- return / status codes ----
 * 1..6 are the thrift TProtocolException type ids (perrors/protocol_error.go:28-36):
 * the Go shim maps any non-zero code to remote.NewTransError(remote.ProtocolError, ...)
 * exactly as fastUnmarshal does (codec_fast.go:65,69,79). */
enum {
  KX_OK = 0,
  KX_ERR_INVALID_DATA = 1,     /* unknown type id, required field missing, bad magic */
  KX_ERR_NEGATIVE_SIZE = 2,    /* negative string/list/map length */
  KX_ERR_SIZE_LIMIT = 3,       /* an output capacity (records / arena) is too small */
  KX_ERR_BAD_VERSION = 4,      /* MessageBegin / Kitex-PB magic mismatch */
  KX_ERR_NOT_IMPLEMENTED = 5,  /* schema shape not supported by this build */
  KX_ERR_DEPTH_LIMIT = 6,      /* skip recursion depth (64, codec_apache.go:167) exceeded */
  KX_ERR_EOF = 8,              /* record runs past the end of its buffer */
  KX_ERR_APPLICATION_EXCEPTION = 9, /* message of type EXCEPTION: a TApplicationException, not a
                                       record (thrift.go:192-195; decoded by the host shim) */
  KX_ERR_UNKNOWN_PROTOCOL = 10, /* framing sniff: no TTHeader / Mesh / Framed / PurePayload / Kitex-PB
                                  magic where one is required, or a malformed TTHeader / Mesh header
                                  (perrors UnknownProtocolError, type 0, default_codec.go:411-416) */
  KX_ERR_PAYLOAD_VALIDATION = 11, /* payload checksum mismatch (crcPayloadValidator.Validate, validate.go:190-201:
                                     kerrors.ErrPayloadValidation wrapping perrors.InvalidData) */
  KX_ERR_INVALID_ARG = 100,
  KX_ERR_HIP = 101,            /* a HIP runtime call failed */
  KX_ERR_NO_DEVICE = 102,
  KX_ERR_INTERNAL = 103        /* bounded spin expired / invariant broken */
};

/* ---- requiredness (thriftgo Requiredness; struct_tpl.go:55-58,313-340) ---- */
enum { KX_REQ_DEFAULT = 0, KX_REQ_REQUIRED = 1, KX_REQ_OPTIONAL = 2 };

/* ---- schema (flattened IDL) ---- */
typedef struct kx_field_desc {
  int16_t id;            /* thrift field id */
  uint8_t ttype;         /* KX_T_* of the field */
  uint8_t req;           /* KX_REQ_* */
  uint8_t elem_ttype;    /* LIST/SET: element KX_T_* (a scalar, STRING, or STRUCT: see below);
                            MAP: key KX_T_* | value KX_T_* << 4 (each a scalar or STRING) */
  uint8_t reserved0;     /* flags: KX_FIELD_BINARY (protobuf bytes), KX_FIELD_STRING_DEFAULT */
  int16_t child;         /* STRUCT (or LIST/SET of STRUCT): index of the (element) struct in the schema's
                            struct table; else -1 */
  int64_t default_bits;  /* scalar default value (two's complement / IEEE bits); a string field with
                            KX_FIELD_STRING_DEFAULT: pointer to its NUL-terminated default (nested schemas) */
} kx_field_desc;

typedef struct kx_struct_desc {
  const kx_field_desc* fields; /* host memory, IDL order */
  uint32_t nfields;
  uint32_t reserved0;          /* flags; of the root struct (index 0): KX_STRUCT_PROTOBUF */
} kx_struct_desc;

/* Kitex-Protobuf schemas (ABI v4). KX_STRUCT_PROTOBUF in the root struct's reserved0 marks every struct
 * of the table as a proto3 message: field ids are proto field numbers, and since proto3 fields have no
 * defaults, default_bits carries the proto scalar kind instead: bits 0..7 of the field itself (of its
 * elements for a repeated field, of its key for a map), bits 8..15 of a map's value.
 *   proto type                    ttype        kind
 *   int32, enum / int64           I32 / I64    KX_PB_NATURAL (varint; int32 sign-extends on the wire)
 *   uint32 / uint64               I32 / I64    KX_PB_UINT (uint32 zero-extends)
 *   sint32 / sint64               I32 / I64    KX_PB_SINT (zig-zag varint)
 *   fixed32, sfixed32, float      I32          KX_PB_FIXED (4 bytes LE; a float column holds its bits)
 *   fixed64, sfixed64             I64          KX_PB_FIXED (8 bytes LE)
 *   double / bool                 DOUBLE / BOOL KX_PB_NATURAL
 *   string / bytes                STRING       KX_PB_NATURAL (UTF-8 checked) / KX_PB_BYTES (or KX_FIELD_BINARY)
 *   message M                     STRUCT       child = M
 *   repeated T                    LIST         elem_ttype = T (child for messages), kind of T
 *   map<K, V>                     MAP          elem_ttype = K | V << 4, kinds K | V << 8
 * Columns follow the nested model below (flat proto3 schemas keep the flat layout). Decoding is
 * proto.Unmarshal (protobuf-go, google.golang.org/protobuf/encoding/protowire): a singular scalar or
 * string takes its last occurrence, a message field merges its occurrences, a repeated field appends
 * (packed and unpacked runs alike for scalars), a map appends its entries in wire order (building a Go
 * map by inserting them in order gives proto.Unmarshal's map: the last duplicate key wins; a missing key
 * or value is the zero value); unknown numbers and known numbers with another wire type are skipped;
 * `string` must be valid UTF-8 (KX_ERR_INVALID_DATA). Presence bits: message fields, proto3 `optional`
 * scalars (KX_REQ_OPTIONAL), repeated and map fields (the field occurred). Encoding is proto.Marshal:
 * field-number order, zero scalars and empty strings omitted (unless `optional` and present), a present
 * message written even when empty, repeated scalars packed, map entries with key and value always
 * written, in column order. */
#define KX_STRUCT_PROTOBUF 1u
enum { KX_PB_NATURAL = 0, KX_PB_SINT = 1, KX_PB_FIXED = 2, KX_PB_UINT = 3, KX_PB_BYTES = 4 };

typedef struct kx_schema kx_schema; /* opaque */

/* Column kinds produced by flattening (depth-first over the IDL, struct fields inlined). */
enum {
  KX_COL_FIXED = 1,      /* one value per record, width 1/2/4/8 bytes, host (little-endian) order */
  KX_COL_BYTES = 2,      /* string/binary: offsets[n+1] (bytes) + data arena */
  KX_COL_LIST = 3,       /* list/set of fixed scalars (or one side of a map of them):
                            offsets[n+1] (elements) + element arena */
  KX_COL_LIST_BYTES = 4, /* list/set of strings (or the string side of a map): offsets[n+1]
                            (elements), elem_offsets[elements+1] (bytes) + byte arena */
  KX_COL_LIST2 = 5,      /* scalars two container levels down (list<list<i64>>, map<K, list<i32>> values):
                            offsets[n+1] (outer elements), elem_offsets[outer+1] (inner elements), data */
  KX_COL_LIST2_BYTES = 6 /* strings two container levels down (map<string, list<string>> values):
                            offsets[n+1], elem_offsets[outer+1], sub_offsets[inner+1] (bytes), data */
};
/* A MAP field flattens to two consecutive columns, keys then values (each LIST or LIST_BYTES,
 * record offsets in entries); the value column's elem_ttype carries KX_ELEM_MAP_VALUE. Encoding
 * writes entries in column order (Go iterates a map in random order: its bytes are only
 * deterministic for maps of <= 1 entry, k-mock.go:225,259).
 * A LIST/SET of a struct S (field elem_ttype = KX_T_STRUCT, child = S) whose fields are all fixed-width
 * scalars (default or required) flattens to one LIST column per field of S, in S's IDL order, sharing
 * the record offsets (in elements); each column's elem_ttype is the field's type | KX_ELEM_STRUCT_FIELD,
 * its field_id / path end with S's field id. Decoding runs each element's FastRead (fields in any order,
 * unknown or mistyped fields skipped, the last duplicate wins, a missing field takes its default, a
 * missing required field is INVALID_DATA; FieldFastReadList + StructLikeFastRead, struct_tpl.go:583-625);
 * encoding writes every field of S in IDL order, then STOP (FieldFastWriteList, :1011-1036). Other
 * element structs (strings, nested structs or containers, optional fields) and containers of containers
 * compile to the nested model below (kx_schema_create falls back to it). */
#define KX_ELEM_MAP_VALUE 0x80
#define KX_ELEM_STRUCT_FIELD 0x40
/* Nested schemas (ABI v3; kx_schema_is_nested() == 1): any shape the generated FastRead handles whose
 * leaves are at most two container levels below the record. The column model generalises the one above:
 *  - every container field (list / set / map) opens a new element domain one level down; its elements'
 *    values live there: a scalar element or field is a LIST column (LIST2 two levels down), a string a
 *    LIST_BYTES (LIST2_BYTES) column; struct elements (list<S>, map<K, S>) are inlined field by field into
 *    the element domain (nested structs inside them too), a map is its key columns then its value columns;
 *  - columns are depth-first in IDL order; an element domain whose elements hold optional, struct or
 *    container fields gets one more column right after the domain's own columns: a LIST (LIST2) of u64
 *    presence words, one per element (elem_ttype = KX_ELEM_PRESENCE), with the bit layout of
 *    kx_columns.presence (column_info.presence_bit of a field inside an element is a bit of that word);
 *  - a container element (or map value) that is itself a container (list<list<i64>>, map<string,
 *    list<string>>) is described by field 0 of the struct `child` (a one-field "element type" struct;
 *    its id is ignored); a map value that is a struct: elem_ttype = key | KX_T_STRUCT << 4, child = S;
 *  - a recursive struct field (a struct that contains itself) keeps its encoded bytes: a BYTES
 *    (LIST_BYTES inside a container) column whose ttype (elem_ttype) is KX_T_STRUCT, delimited by the
 *    skip decoder on decode and written back verbatim on encode (an empty value encodes as STOP);
 *  - string fields may carry a default: kx_field_desc.default_bits = (int64_t)(intptr_t) of a
 *    NUL-terminated host string with KX_FIELD_STRING_DEFAULT set in reserved0 (copied at schema creation).
 * Semantics are those of the flat schemas (unknown / mistyped fields skipped, the last duplicate wins,
 * a repeated struct field is a fresh NewX(), missing required fields INVALID_DATA, absent fields take
 * their defaults) at every level. */
#define KX_ELEM_PRESENCE 0x20
#define KX_FIELD_BINARY 1
#define KX_FIELD_STRING_DEFAULT 2

typedef struct kx_column_info {
  uint32_t kind;        /* KX_COL_* */
  uint32_t width;       /* FIXED: value width; LIST: element width; BYTES / LIST_BYTES: 1 */
  uint8_t ttype;        /* wire type of the field (LIST/SET/MAP for containers) */
  uint8_t elem_ttype;   /* LIST / LIST_BYTES: element wire type */
  int16_t field_id;     /* id of the leaf field */
  int32_t presence_bit; /* bit in the presence word for this field, or -1 */
  uint32_t depth;       /* nesting depth (0 = root field) */
  int16_t path[8];      /* field ids from the root to this leaf */
  uint8_t level;        /* container levels above the leaf (0: one value per record) */
  uint8_t reserved1[3];
} kx_column_info;

/* A batch of decoded records in struct-of-arrays form. All pointers are DEVICE memory for the
 * *_batch calls and HOST memory for kx_host_* calls.
 * Offsets are unsigned, `offset_bytes` wide (4 = uint32_t, the default when 0; 8 = uint64_t). With
 * 4-byte offsets a column whose arena position would pass UINT32_MAX fails with KX_ERR_SIZE_LIMIT
 * (it never wraps); use 8-byte offsets for arenas of 4 GiB units and more. */
typedef struct kx_column {
  void* data;             /* FIXED: n*width bytes; BYTES/LIST/LIST_BYTES: arena */
  void* offsets;          /* BYTES/LIST/LIST_BYTES: n+1 entries (bytes / elements); FIXED: NULL */
  uint64_t capacity;      /* arena capacity in arena units (bytes; LIST: elements); FIXED: ignored */
  void* elem_offsets;     /* LIST_BYTES: byte offset of every element (elem_capacity+1 entries) */
  uint64_t elem_capacity; /* LIST_BYTES: element capacity */
  uint32_t offset_bytes;  /* 4 (or 0) / 8: width of offsets and elem_offsets entries */
  uint32_t flags;         /* KX_COLF_* */
  void* sub_offsets;      /* LIST2_BYTES: byte offset of every inner element (sub_capacity+1 entries) */
  uint64_t sub_capacity;  /* LIST2 / LIST2_BYTES: inner element capacity */
} kx_column;

/* KX_COLF_VIEW (decode, BYTES columns): zero-copy string views instead of copies. `offsets` receives
 * n (offset, length) pairs of offset_bytes each: record i's string is in[off .. off + len) of the
 * decode call's input (len 0 => off 0); `data` / `capacity` are ignored and no arena is written. The
 * input must outlive the columns (the no-copy reads of the generated code, e.g. unsafex string
 * views). With 4-byte pairs the input must be < 4 GiB (else KX_ERR_SIZE_LIMIT). Not accepted by the
 * encoders or the kx_host_* calls. */
#define KX_COLF_VIEW 1u

#define KX_MAX_COLUMNS 64
#define KX_MAX_STRUCTS 16

typedef struct kx_columns {
  kx_column cols[KX_MAX_COLUMNS];
  uint32_t ncols;       /* must equal kx_schema_num_columns() */
  uint32_t reserved0;
  uint64_t* presence;   /* n words (bit per presence-tracked field), required iff the schema has any */
} kx_columns;

/* Per-call status, written by the device (caller-owned DEVICE memory, 192 bytes, 8-aligned). */
typedef struct kx_status {
  int32_t code;         /* first error (lowest record index), 0 = OK */
  int32_t reserved0;
  uint64_t record;      /* index of the failing record */
  uint64_t offset;      /* byte offset of the failing record's start in the input */
  uint64_t n_records;   /* records decoded */
  uint64_t consumed;    /* input bytes consumed (concatenated mode) */
  uint64_t var_total[16]; /* required arena size (arena units) per var slot (ABI 5: 16 slots, was 8) */
  uint64_t diag[3];       /* decode diagnostics: [0] tiles re-walked from their true entry,
                             [1] groups of 64 tiles re-scanned by the chain pass, [2] concatenated:
                             tiles the fast index path left to the field loop; known offsets: 2 when
                             the length gather ran, 3 when its extents needed the repair pass */
} kx_status;

typedef struct kx_ctx kx_ctx; /* opaque; one per host thread / stream */

/* ---- lifecycle ---- */
int kx_abi_version(void);
const char* kx_strerror(int code);

int kx_schema_create(const kx_struct_desc* structs, uint32_t nstructs, kx_schema** out);
void kx_schema_destroy(kx_schema* s);
uint32_t kx_schema_num_columns(const kx_schema* s);
int kx_schema_column_info(const kx_schema* s, uint32_t col, kx_column_info* out);
uint32_t kx_schema_presence_bits(const kx_schema* s);
/* Minimum encoded size of a record (all var fields empty, optional fields unset). */
uint64_t kx_schema_min_record_size(const kx_schema* s);
/* 1 when the schema uses the nested model (see KX_ELEM_PRESENCE above): decode and encode run the nested
 * record walker (lane = record; boundaries of concatenated records from the skip pass), and the arena
 * sizes of a decode are obtained first with kx_thrift_decode_sizes. */
int kx_schema_is_nested(const kx_schema* s);

/* Device workspace (bytes) a kx_ctx holds for a decode of n records over in_len input bytes (known_offsets
 * != 0: offsets given), grow-only per ctx and stream. No reference counterpart (capacity planning): the
 * concatenated modes keep per-tile aggregates plus record-start slots sized from the mean record size
 * (DESIGN.md §2), e.g. 0.28 GB for 16 M R2 records (2.8 GB of input). */
uint64_t kx_decode_workspace_bytes(const kx_schema* s, uint64_t in_len, int known_offsets, uint64_t n);

int kx_ctx_create(int device, kx_ctx** out);
void kx_ctx_destroy(kx_ctx* c);
/* Decode pipelining of this ctx (a tuning knob; no reference counterpart). A batch of more than two
 * chunks of `chunk_bytes` input (rounded to whole 512 KiB groups of tiles; 0 = never chunk) is
 * decoded as a pipeline: the index pass of chunk k runs on a second stream of the ctx while chain +
 * emit of chunk k - 1 run on the caller's stream, `ahead` chunks apart at most, so the emit pass
 * re-reads input the index pass has just brought into the Infinity Cache. Results are identical
 * for every setting. Default: KX_CHUNK_MB environment variable, else 0 (off: on MI355X the
 * per-chunk chain step costs more than the cache re-read saves), ahead 1. */
int kx_ctx_set_pipeline(kx_ctx* c, uint64_t chunk_bytes, int ahead);

/* ---- Thrift binary: batched FastRead ----
 * offsets != NULL : record i is in[offsets[i] .. offsets[i+1]) (u64, n+1 entries, device). Each record
 *                   is decoded independently, trailing bytes inside the range are ignored and a read
 *                   past the range is KX_ERR_EOF (fastUnmarshal semantics, codec_fast.go:62-71).
 *                   record_status (optional, n bytes) receives each record's code.
 * offsets == NULL : exactly n records are concatenated from in[0]; the boundary of each is where its
 *                   FastRead stops (list<Struct> element loop). status->consumed = bytes used.
 * On return the work is enqueued on `stream`; status is final when the stream reaches this point. */
int kx_thrift_decode_batch(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                           const uint64_t* offsets, uint64_t n, const kx_columns* out,
                           uint8_t* record_status, kx_status* status, void* stream);

/* Nested schemas: the arena sizes a decode of this input needs, per column (host memory, 3 x ncols):
 * units[3c] = data units (bytes / elements), units[3c + 1] = elem_offsets entries - 1, units[3c + 2] =
 * sub_offsets entries - 1. Synchronous on `stream`. status (host) as the decode's (the first failing
 * record; its extents count as empty). Flat schemas: KX_ERR_NOT_IMPLEMENTED (status->var_total). */
int kx_thrift_decode_sizes(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                           const uint64_t* offsets, uint64_t n, uint64_t* units, kx_status* status, void* stream);
/* The same for bare bodies at explicit extents in[starts[i], ends[i]) (the sizing step of
 * kx_thrift_decode_extents; ttstream DecodePayload, pkg/remote/trans/ttstream/frame.go:223-233). */
int kx_thrift_decode_sizes_extents(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                                   const uint64_t* starts, const uint64_t* ends, uint64_t n, uint64_t* units,
                                   kx_status* status, void* stream);

/* Skip decoder over n concatenated records: writes record start offsets (n+1 entries, device u64). */
int kx_thrift_skip_batch(kx_ctx* c, const uint8_t* in, uint64_t in_len, uint64_t n,
                         uint64_t* offsets_out, kx_status* status, void* stream);

/* Split points of n concatenated records of schema s for `parts` shards (1 <= parts <= 65536):
 * points_out[k] (parts + 1 entries, device u64) = the start of record floor(k * n / parts), and
 * points_out[parts] = the end of record n - 1 (= status->consumed). Shard k is then the batch
 * in[points_out[k] .. points_out[k + 1]) of floor((k+1)n/parts) - floor(kn/parts) records. Runs the decode's
 * index pass (with the schema's fast path) and its chain, never the emit pass. A flat schema's
 * records are walked by its program (field types checked as in decode); a nested schema's by the skip
 * decoder (kx_thrift_skip_batch). On a decode error or EOF before n records the status is the
 * decode's and points_out is left unwritten. n == 0: every point is 0. */
int kx_thrift_split_points(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len, uint64_t n,
                           uint32_t parts, uint64_t* points_out, kx_status* status, void* stream);

/* ---- multi-GPU record-range shards: concatenation of decoded shards into one rank ----
 * The reference has no multi-device path (its caller partitions; pkg/remote/payload_codec.go:29-33 is the
 * per-message surface); this is the exchange a host runs after every rank decoded its record range:
 *   1. kx_shard_meta on every rank: its exchange header (device u64[kx_shard_meta_words(...)]);
 *   2. all-gather of the headers (ncclAllGather), copied to host on the root as metas[world][words];
 *   3. kx_concat_plan on the root: the pieces every rank sends (in piece order) and where they land,
 *      and the root's array sizes; the root allocates its output columns (8-byte offsets, 8-byte views);
 *   4. ncclGroupStart; per piece ncclSend on its rank / ncclRecv on the root; ncclGroupEnd. A piece of
 *      an offsets array (array < 3, or a view column's pairs) lands in the root's STAGING column
 *      (senders' offset width), every other piece in the output column;
 *   5. kx_concat_rebase on the root: staging offsets + the rank's rebase -> output, closing entries.
 * Header layout: [n, in_len, then per non-FIXED column in column order, per level j of its offsets chain
 * (depth 1 for BYTES / LIST, 2 for LIST_BYTES / LIST2, 3 for LIST2_BYTES) the first entry f_j and the units
 * u_j it spans: f_0 = offsets[0], u_0 = offsets[n] - f_0, f_{j+1} = next[f_j], u_{j+1} = next[f_j + u_j] -
 * f_{j+1}] (a view column's words are 0). Every rank must give its columns the same offset_bytes / flags. */
#define KX_PIECE_OFFSETS 0u       /* kx_column.offsets (a view column: its (offset, length) pairs) */
#define KX_PIECE_ELEM_OFFSETS 1u  /* kx_column.elem_offsets */
#define KX_PIECE_SUB_OFFSETS 2u   /* kx_column.sub_offsets */
#define KX_PIECE_DATA 3u          /* kx_column.data (FIXED values, arenas); presence words: column == KX_MAX_COLUMNS */
typedef struct kx_concat_piece {
  uint32_t rank;        /* sender */
  uint32_t column;      /* schema column, or KX_MAX_COLUMNS for the presence words */
  uint32_t array;       /* KX_PIECE_* */
  uint32_t elem_bytes;  /* bytes per element of the piece (the sender's width) */
  uint64_t src_first;   /* first element in the sender's array */
  uint64_t count;       /* elements */
  uint64_t dst_first;   /* first element in the root's array (staging for offsets / view pieces) */
  int64_t rebase;       /* offsets: added to every entry; views: input bytes before this rank (added to a
                           non-empty view's offset); 0 otherwise */
} kx_concat_piece;
typedef struct kx_concat_sizes {
  uint64_t n;                          /* records of the concatenation */
  uint64_t in_len;                     /* input bytes of all ranks (views point into their concatenation) */
  uint64_t units[KX_MAX_COLUMNS][4];   /* per column and KX_PIECE_* array: entries before the closing one
                                          (offsets arrays hold units + 1 entries; data: its elements) */
} kx_concat_sizes;
/* infos / ncols: kx_schema_column_info of every column of the schema (host memory), which is all the
 * concatenation needs to know of it. */
uint32_t kx_shard_meta_words(const kx_column_info* infos, uint32_t ncols);
/* cols: this rank's decoded columns (device); writes the header to meta (device u64[kx_shard_meta_words]). */
int kx_shard_meta(kx_ctx* c, const kx_column_info* infos, uint32_t ncols, const kx_columns* cols, uint64_t n,
                  uint64_t in_len, uint64_t* meta, void* stream);
/* Host only (no device access). layout: any rank's columns (offset_bytes and flags are read, pointers
 * are not; presence != NULL when the records carry presence words). metas: host u64[world][words].
 * pieces: capacity *npieces on entry, the count on return (KX_ERR_SIZE_LIMIT, with the needed count,
 * when too small). Pieces are ordered by rank, then column, then array; empty pieces are listed. */
int kx_concat_plan(const kx_column_info* infos, uint32_t ncols, const kx_columns* layout, const uint64_t* metas,
                   uint32_t world, kx_concat_piece* pieces, uint32_t* npieces, kx_concat_sizes* sizes);
/* staging: the root's received offset arrays (offset_bytes = the senders'); out: the concatenated columns
 * (8-byte offsets and view pairs). Adds each offsets / view piece's rebase on the device and writes the
 * closing entry of every offsets array. pieces: host memory, as kx_concat_plan returned them. */
int kx_concat_rebase(kx_ctx* c, const kx_column_info* infos, uint32_t ncols, const kx_concat_piece* pieces,
                     uint32_t npieces, const kx_columns* staging, const kx_columns* out, const kx_concat_sizes* sizes,
                     void* stream);

/* ---- Thrift binary: batched BLength / FastWriteNocopy ---- */
int kx_thrift_encoded_size_batch(kx_ctx* c, const kx_schema* s, const kx_columns* in, uint64_t n,
                                 uint64_t* sizes_out, void* stream);
/* Writes the n encoded records back to back into out[0..). offsets_out (n+1, device, optional)
 * receives each record's start; status->consumed receives the total size. */
int kx_thrift_encode_batch(kx_ctx* c, const kx_schema* s, const kx_columns* in, uint64_t n,
                           uint8_t* out, uint64_t out_cap, uint64_t* offsets_out,
                           kx_status* status, void* stream);

/* fastMarshal over n messages (codec_fast.go:40-58; thriftCodec.Marshal, thrift.go:106-160): message i =
 * WriteMessageBegin(name, msg_type, seqids[i]) (strict binary, binary_test.go:387-457) + the method's
 * Args / Result struct whose field `body_field` (1 = Args{1: req}, 0 = Result{0: success}) is record i
 * (its FastWriteNocopy bytes, kx_thrift_encode_batch) + STOP (MockTestArgs.FastWriteNocopy,
 * k-mock.go:422-517). The records are first written to body_scratch (device, >= their total size, e.g.
 * the sum of kx_thrift_encoded_size_batch); out receives the n messages back to back
 * (sum of record sizes + n * (16 + name_len) bytes), offsets_out (n + 1, optional) their starts.
 * name: host memory. seqids: device i32[n]. Status: SIZE_LIMIT when scratch or out is too small. */
int kx_thrift_encode_messages(kx_ctx* c, const kx_schema* s, const kx_columns* in, uint64_t n, const char* name,
                              uint32_t name_len, int32_t msg_type, const int32_t* seqids, int32_t body_field,
                              uint8_t* body_scratch, uint64_t scratch_cap, uint8_t* out, uint64_t out_cap,
                              uint64_t* offsets_out, kx_status* status, void* stream);

/* ---- Kitex-Protobuf (proto3 body) ----
 * The schema's field ids are proto field numbers; ttype (and, with KX_STRUCT_PROTOBUF, the kind in
 * default_bits) selects the proto type, see KX_STRUCT_PROTOBUF above: scalars of every proto3 type,
 * strings / bytes, nested messages, repeated fields (packed and unpacked), maps, proto3 `optional`.
 * Flat messages run on the tile pipeline; anything else on the nested record walker. offsets semantics
 * as kx_thrift_decode_batch; with offsets == NULL the input is the body of
 * `message Batch { repeated Rec recs = 1; }`. */
int kx_pb_decode_batch(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                       const uint64_t* offsets, uint64_t n, const kx_columns* out,
                       uint8_t* record_status, kx_status* status, void* stream);
/* Framed size of each record (0x0A + uvarint(body) + body), device sizes_out[n]. */
int kx_pb_encoded_size_batch(kx_ctx* c, const kx_schema* s, const kx_columns* in, uint64_t n,
                             uint64_t* sizes_out, void* stream);
/* Writes the n records as the body of `message Batch { repeated Rec recs = 1; }`; offsets_out
 * (n+1, device, optional) receives each record's frame start; status->consumed the total size. */
int kx_pb_encode_batch(kx_ctx* c, const kx_schema* s, const kx_columns* in, uint64_t n,
                       uint8_t* out, uint64_t out_cap, uint64_t* offsets_out,
                       kx_status* status, void* stream);

/* ---- host-memory entry points (the netpoll buffer side) ----
 * in / out columns / record_status / status are HOST memory (pinned for full PCIe rate, or pageable).
 * Synchronous: every copy has completed when the call returns, on success and on error.
 * Every schema the device entry points take: flat columns of every kind (FIXED, BYTES, LIST, LIST_BYTES:
 * MockReq's map<string,string> and list<string>, k-mock.go:39-114; base.Base's Extra map), nested Thrift
 * schemas and nested Kitex-Protobuf messages (the record walker; LIST2 / LIST2_BYTES columns). A column's
 * capacities (capacity, elem_capacity, sub_capacity) are the units its host arrays hold; the device decides
 * the arena positions and only the units the records fill are copied back (status->var_total, a nested
 * schema's cursor totals); an arena too small is KX_ERR_SIZE_LIMIT.
 * With offsets (each message's length known from its framing) and n >= 64 Ki the batch is a pipeline of
 * 16 record-range chunks over three streams of the ctx: the H2D, the decode and the D2H of different chunks
 * overlap, each chunk continuing the previous one's arenas on the device. Without offsets: H2D, decode, D2H.
 * record_status (optional, n bytes): each record's code. With offsets every record is decoded on its own
 * (fastUnmarshal, codec_fast.go:62-71: a failing message fails alone, the others decode), so a caller can
 * fall back per message; status is the first failing record's (record = its index). Without offsets the
 * records from the failing one on carry its code. */
int kx_host_decode_batch(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                         const uint64_t* offsets, uint64_t n, const kx_columns* out, uint8_t* record_status,
                         kx_status* status);
/* The same for Kitex-Protobuf bodies (offsets semantics as kx_pb_decode_batch). */
int kx_host_pb_decode_batch(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                            const uint64_t* offsets, uint64_t n, const kx_columns* out, uint8_t* record_status,
                            kx_status* status);
/* fastMarshal from host memory (codec_fast.go:40-58 / thrift.go:106-160, the reply path): n records'
 * columns (HOST memory, pinned for full PCIe rate; flat or nested schemas, no views; elem_capacity /
 * sub_capacity = the entries - 1 their arrays hold) -> out[0 ..) (host) the records back to back, as
 * kx_thrift_encode_batch writes them; offsets_out (host, n + 1, optional) each record's start; status (host):
 * consumed = total bytes. SIZE_LIMIT when out_cap is too small: consumed is then the size the whole batch
 * needs, and out holds the records of the chunks that fitted (record_status 0 for them, SIZE_LIMIT for the
 * rest; optional, n bytes). With n >= 64 Ki a pipeline of 16 record-range chunks: the H2D of the columns,
 * the encode and the D2H of the wire of different chunks overlap. kx_host_pb_encode_batch: the
 * Kitex-Protobuf Batch body (kx_pb_encode_batch). */
int kx_host_encode_batch(kx_ctx* c, const kx_schema* s, const kx_columns* in, uint64_t n, uint8_t* out,
                         uint64_t out_cap, uint64_t* offsets_out, uint8_t* record_status, kx_status* status);
int kx_host_pb_encode_batch(kx_ctx* c, const kx_schema* s, const kx_columns* in, uint64_t n, uint8_t* out,
                            uint64_t out_cap, uint64_t* offsets_out, uint8_t* record_status, kx_status* status);

/* ---- message level: N framed RPC messages (framing already removed by the transport) ----
 * message i = in[offsets[i] .. offsets[i+1]) (u64, n+1 entries, device).
 * Thrift: MessageBegin (strict binary: i32 0x8001_00TT, string name, i32 seqid) + the method's
 *   argument / result struct; its field `body_field` (1 = Args{1: req}, 0 = Result{0: success}) of
 *   type STRUCT is the record decoded into `out` (schema `s` = that struct); every other field is
 *   skipped (skip decoder, depth 64). An absent record field decodes as an empty struct.
 *   (thriftCodec.Unmarshal, thrift.go:180-225; Args.FastRead, k-mock.go:422-517)
 * Protobuf: Kitex-PB meta header (u32 0x9001_0000 + type, u32-length method name, u32 seqid), the
 *   rest of the message is the proto body (protobufCodec.Unmarshal, protobuf.go:136-165).
 * msg_cols (optional, 3 entries): [0] method name (KX_COL_BYTES: offsets + arena), [1] message type
 *   (int32), [2] seqid (int32). Per-message codes in record_status (header errors, an EXCEPTION
 *   message = KX_ERR_APPLICATION_EXCEPTION, else the record's decode code); status as offsets mode
 *   (the first failing message; offset = its start). */
int kx_thrift_decode_messages(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                              const uint64_t* offsets, uint64_t n, int32_t body_field,
                              const kx_column* msg_cols, const kx_columns* out, uint8_t* record_status,
                              kx_status* status, void* stream);
int kx_pb_decode_messages(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                          const uint64_t* offsets, uint64_t n, const kx_column* msg_cols,
                          const kx_columns* out, uint8_t* record_status, kx_status* status, void* stream);

/* ---- socket buffer level: framing sniff (defaultCodec.DecodeMeta + checkPayload,
 *      default_codec.go:189-221, 328-427; Mesh header header_codec.go:192-212; TTHeader meta and
 *      info blocks per gopkg protocol/ttheader) ----
 * in = n frames back to back (device). Per frame: frame_offsets[i] (n + 1 entries; frame i =
 * [frame_offsets[i], frame_offsets[i+1])), the payload the payload codec reads = [payload_start[i],
 * payload_end[i]) (MessageBegin / Kitex-PB meta first; the Framed length and all headers removed),
 * kinds[i] (optional) = transport.Protocol (KX_TRANS_*) | KX_FRAME_PB | KX_FRAME_MESH.
 * PurePayload frames (no length prefix) are delimited by their MessageBegin + struct.
 * max_payload > 0: a longer payload is INVALID_DATA (checkPayloadSize, :429-434).
 * Status as concatenated decode: the first frame that cannot be delimited (UNKNOWN_PROTOCOL, EOF,
 * ...), status->n_records = frames delimited; boundaries are found in parallel on the device. */
enum {
  KX_TRANS_PURE = 0, KX_TRANS_TTHEADER = 2, KX_TRANS_FRAMED = 4, KX_TRANS_TTHEADER_FRAMED = 6,
  KX_FRAME_PB = 0x10, KX_FRAME_MESH = 0x20
};
int kx_frame_scan(kx_ctx* c, const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t max_payload,
                  uint64_t* frame_offsets, uint64_t* payload_start, uint64_t* payload_end, uint8_t* kinds,
                  kx_status* status, void* stream);
/* A socket buffer of n frames straight to columns: kx_frame_scan, then kx_*_decode_messages on the
 * payloads. frame_offsets (n + 1) and kinds are optional outputs. A frame that cannot be delimited
 * ends the batch: it and every later message get its code in record_status, and the call's status
 * is the scan's (record = that frame, offset = its start). */
int kx_thrift_decode_frames(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len, uint64_t n,
                            int32_t body_field, uint64_t max_payload, uint64_t* frame_offsets, uint8_t* kinds,
                            const kx_column* msg_cols, const kx_columns* out, uint8_t* record_status,
                            kx_status* status, void* stream);
int kx_pb_decode_frames(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len, uint64_t n,
                        uint64_t max_payload, uint64_t* frame_offsets, uint8_t* kinds, const kx_column* msg_cols,
                        const kx_columns* out, uint8_t* record_status, kx_status* status, void* stream);

/* ---- binary generic (raw) ingress: binaryThriftCodec (pkg/generic/binarythrift_codec.go) ----
 * kx_thrift_raw_messages: Unmarshal (:83-115) over n messages in[offsets[i] .. offsets[i+1]) (u64, n + 1):
 *   the request stays the raw message bytes (zero copy, nothing is parsed past the method name);
 *   msg_cols (optional, as kx_thrift_decode_messages) receive the method name (readBinaryMethod :185-199:
 *   u32 length at [4, 8), 0 < length <= size - 8), the message type (first u32 & 0xffff) and the seqid
 *   (the u32 after the name, 0 if absent). record_status: INVALID_DATA for a bad method length;
 *   APPLICATION_EXCEPTION for an EXCEPTION message (it takes the regular thriftCodec path, :88-90).
 * kx_thrift_set_seqids: SetSeqID (:117-134, getSeqID4Bytes :147-175) in place over n raw messages:
 *   the seqid of message i becomes seqids[i] (device i32); a message without a strict version is
 *   BAD_VERSION (INVALID_DATA when the first word is positive), a negative name length or a message
 *   too short for the seqid INVALID_DATA (that message is left untouched). */
int kx_thrift_raw_messages(kx_ctx* c, const uint8_t* in, uint64_t in_len, const uint64_t* offsets, uint64_t n,
                           const kx_column* msg_cols, uint8_t* record_status, kx_status* status, void* stream);
int kx_thrift_set_seqids(kx_ctx* c, uint8_t* in, uint64_t in_len, const uint64_t* offsets, uint64_t n,
                         const int32_t* seqids, uint8_t* record_status, kx_status* status, void* stream);

/* ---- gRPC length-prefixed messages (decodeGRPCFrame, pkg/remote/codec/grpc/grpc_compress.go:37-60;
 *      grpcCodec.Decode, grpc.go:202-260) ----
 * in = n messages back to back, each [u8 compressed flag][u32 BE length][payload] (the DATA frames of one
 * stream, HTTP/2 framing already removed). kx_grpc_frame_scan: frame_offsets (n + 1), payload
 * [payload_start[i], payload_end[i]) (the 5-byte prefix removed), flags[i] (optional) = the compressed-flag
 * byte; boundaries found in parallel on the device; a message cut short is KX_ERR_EOF, a payload longer
 * than max_payload (> 0) KX_ERR_INVALID_DATA; status as kx_frame_scan.
 * kx_thrift_decode_grpc / kx_pb_decode_grpc: scan, then each payload decoded as one record
 * (thrift.UnmarshalThriftData -> fastUnmarshal with dataLen = the payload, grpc.go:241-249; proto.Unmarshal
 * of the payload, :251-270). A compressed message (flag 1) gets KX_ERR_NOT_IMPLEMENTED (no decompressor
 * on the device: the reference's "kitex compression algorithm not found" when none is registered);
 * record_status / status as kx_*_decode_frames. */
int kx_grpc_frame_scan(kx_ctx* c, const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t max_payload,
                       uint64_t* frame_offsets, uint64_t* payload_start, uint64_t* payload_end, uint8_t* flags,
                       kx_status* status, void* stream);
int kx_thrift_decode_grpc(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len, uint64_t n,
                          uint64_t max_payload, uint64_t* frame_offsets, const kx_columns* out,
                          uint8_t* record_status, kx_status* status, void* stream);
int kx_pb_decode_grpc(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len, uint64_t n,
                      uint64_t max_payload, uint64_t* frame_offsets, const kx_columns* out, uint8_t* record_status,
                      kx_status* status, void* stream);

/* ---- CRC32C payload checksums (crcPayloadValidator, pkg/remote/codec/validate.go:168-217) ----
 * CRC-32C = crc32.Update(0, crc32.MakeTable(crc32.Castagnoli), payload) (getCRC32C, :208-217); the
 * header value is its big-endian lowercase hex (8 characters).
 * kx_crc32c_batch: crc_out[i] (device u32) = CRC-32C of in[offsets[i] .. offsets[i+1]) (n + 1 device u64
 *   offsets, e.g. kx_thrift_encode_batch's offsets_out): the Generate side. A range outside the input
 *   gives KX_ERR_INVALID_ARG in status (that range's crc_out = 0).
 * kx_frame_crc32c_validate: n frames starting at frame_offsets[i] (n + 1 entries, as kx_frame_scan writes
 *   them). For each TTHeader frame whose string-KV info holds "crc32c" (transmeta.HeaderCRC32C) with a
 *   non-empty value, the CRC-32C of the TTHeader payload (all bytes after the TTHeader, the Framed length
 *   prefix included: PayloadLen) must hex-encode to exactly that value, else record_status[i] =
 *   KX_ERR_PAYLOAD_VALIDATION. Frames of other framings, without the key or with an empty value pass
 *   (:95-99, :191-195). crc_out (optional) = the payload's CRC-32C (0 for non-TTHeader frames). Status:
 *   the first failing frame. */
int kx_crc32c_batch(kx_ctx* c, const uint8_t* in, uint64_t in_len, const uint64_t* offsets, uint64_t n,
                    uint32_t* crc_out, kx_status* status, void* stream);
int kx_frame_crc32c_validate(kx_ctx* c, const uint8_t* in, uint64_t in_len, const uint64_t* frame_offsets,
                             uint64_t n, uint32_t* crc_out, uint8_t* record_status, kx_status* status,
                             void* stream);
/* enable != 0: kx_*_decode_frames validate every TTHeader frame's CRC32C after the framing scan, as
 * NewDefaultCodecWithConfig(CodecConfig{CRC32Check: true}) does (default_codec.go:70-92); a failing frame's
 * message gets KX_ERR_PAYLOAD_VALIDATION (its record is not decoded). Default off. */
int kx_ctx_set_crc32c_check(kx_ctx* c, int enable);

/* ---- TTHeader streaming frames (ttstream DecodeFrame, pkg/remote/trans/ttstream/frame.go:137-185) ----
 * in = n frames of one connection back to back, each a TTHeader (gopkg protocol/ttheader) whose payload is
 * a bare struct (ProtocolIDThriftStruct / ProtobufStruct: gopkgthrift.FastMarshal, no MessageBegin,
 * frame.go:92-130, 192-233). Per frame: frame_offsets[i] (n + 1), payload [payload_start[i], payload_end[i])
 * (PayloadLen bytes after the header), frame_types[i] = KX_TTS_* from IntInfo[frame_type_key] (an
 * unknown value is KX_ERR_INVALID_DATA: "unexpected frame type", :166-167), stream_ids[i] = the TTHeader
 * seqid (the stream id, :170), method_pos[i] / method_len[i] = IntInfo[to_method_key] inside `in` (0 / 0
 * when absent, :169). A frame without the streaming flag is KX_ERR_INVALID_DATA (:143-145); a frame whose
 * magic is not TTHeader's, or whose header blocks are malformed, KX_ERR_UNKNOWN_PROTOCOL; a frame cut short
 * KX_ERR_EOF. Outputs other than frame_offsets are optional. Status as kx_frame_scan.
 * The int-info key of the frame type, its five values and the streaming flag live in the un-vendored
 * gopkg (ttheader.FrameType, FrameType*, HeaderFlagsStreaming): kx_ttstream_default_keys fills the values
 * this library assumes (parity unpinned); a caller with other constants passes its own.
 * ToMethod is transmeta.ToMethod (pkg/remote/transmeta/metakey.go:33, key 9). */
typedef struct kx_ttstream_keys {
  uint16_t frame_type_key;    /* IntInfo key of the frame type (ttheader.FrameType) */
  uint16_t to_method_key;     /* IntInfo key of the method (ttheader.ToMethod) */
  uint16_t streaming_flag;    /* ttheader.HeaderFlagsStreaming */
  uint16_t reserved;
  char type_names[5][8];      /* values for META, HEADER, DATA, TRAILER, RST (NUL-padded, <= 8 bytes) */
} kx_ttstream_keys;
enum { KX_TTS_META = 1, KX_TTS_HEADER = 2, KX_TTS_DATA = 3, KX_TTS_TRAILER = 4, KX_TTS_RST = 5 };
void kx_ttstream_default_keys(kx_ttstream_keys* keys);
int kx_ttstream_frame_scan(kx_ctx* c, const uint8_t* in, uint64_t in_len, uint64_t n, const kx_ttstream_keys* keys,
                           uint64_t* frame_offsets, uint64_t* payload_start, uint64_t* payload_end,
                           uint8_t* frame_types, int32_t* stream_ids, uint64_t* method_pos, uint32_t* method_len,
                           kx_status* status, void* stream);

/* ---- records at explicit extents (gopkgthrift.FastUnmarshal of each payload, ttstream DecodePayload
 *      frame.go:223-233; proto.Unmarshal for ProtobufStruct) ----
 * Record i = in[starts[i] .. ends[i]) (device u64 arrays, n entries each; extents may leave gaps, e.g. the
 * DATA-frame payloads kx_ttstream_frame_scan located). Semantics, record_status and status as the
 * known-offsets decode (offset = the failing record's start). */
int kx_thrift_decode_extents(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                             const uint64_t* starts, const uint64_t* ends, uint64_t n, const kx_columns* out,
                             uint8_t* record_status, kx_status* status, void* stream);
int kx_pb_decode_extents(kx_ctx* c, const kx_schema* s, const uint8_t* in, uint64_t in_len,
                         const uint64_t* starts, const uint64_t* ends, uint64_t n, const kx_columns* out,
                         uint8_t* record_status, kx_status* status, void* stream);

/* Kitex-Protobuf meta header (host memory; protobuf.go:77-90 / 136-165). */
uint64_t kx_pb_meta_length(uint32_t name_len);
int kx_pb_write_meta(uint8_t* buf, uint64_t cap, const char* name, uint32_t name_len, int32_t msg_type,
                     int32_t seqid, uint64_t* written);
int kx_pb_read_meta(const uint8_t* buf, uint64_t len, const char** name, uint32_t* name_len,
                    int32_t* msg_type, int32_t* seqid, uint64_t* consumed);

/* ---- Thrift MessageBegin (WriteMessageBegin / ReadMessageBegin, binary_test.go:387-457) ---- */
uint64_t kx_thrift_message_begin_length(uint32_t name_len);
int kx_thrift_write_message_begin(uint8_t* buf, uint64_t cap, const char* name, uint32_t name_len,
                                  int32_t msg_type, int32_t seqid, uint64_t* written);
int kx_thrift_read_message_begin(const uint8_t* buf, uint64_t len, const char** name,
                                 uint32_t* name_len, int32_t* msg_type, int32_t* seqid,
                                 uint64_t* consumed);

#ifdef __cplusplus
}
#endif
#endif /* KXCODEC_H_ */
