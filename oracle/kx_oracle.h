/*
 * kx_oracle.h — TEST INFRASTRUCTURE ONLY. CPU restatement of the reference (cloudwego/kitex) payload
 * codec semantics, used as the parity checker for the MI355X codec and as the CPU baseline in bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library. The
 * product (kitex_amd / libkxcodec.so) never links or calls it.
 *
 * Parity pinning: every primitive is checked against the reference's own known-answer tests
 * (pkg/protocol/bthrift/binary_test.go, pkg/remote/codec/thrift/thrift_data_test.go,
 * codec_apache_test.go) in tests/test_oracle_kat.py. The reference itself (Go, plus the un-vendored
 * github.com/cloudwego/gopkg v0.2.0) cannot be built or run here: no Go toolchain.
 */
#ifndef KX_ORACLE_H_
#define KX_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#include "../include/kxcodec.h"

#ifdef __cplusplus
extern "C" {
#endif

/* -------- thrift.Binary primitives (gopkg; KATs in bthrift/binary_test.go) -------- */
size_t kxo_write_field_begin(uint8_t* b, uint8_t ttype, int16_t id);      /* binary_test.go:56-75 */
size_t kxo_write_field_stop(uint8_t* b);                                  /* :83-87 */
size_t kxo_write_map_begin(uint8_t* b, uint8_t kt, uint8_t vt, int32_t n); /* :90-109 */
size_t kxo_write_list_begin(uint8_t* b, uint8_t et, int32_t n);           /* :118-136 */
size_t kxo_write_set_begin(uint8_t* b, uint8_t et, int32_t n);            /* :145-163 */
size_t kxo_write_bool(uint8_t* b, int v);                                 /* :172-196 */
size_t kxo_write_byte(uint8_t* b, int8_t v);                              /* :199-212 */
size_t kxo_write_i16(uint8_t* b, int16_t v);                              /* :215-228 */
size_t kxo_write_i32(uint8_t* b, int32_t v);                              /* :231-244 */
size_t kxo_write_i64(uint8_t* b, int64_t v);                              /* :247-260 */
size_t kxo_write_double(uint8_t* b, double v);                            /* :263-276 */
size_t kxo_write_string(uint8_t* b, const uint8_t* s, uint32_t n);        /* :279-322 */
size_t kxo_write_message_begin(uint8_t* b, const char* name, uint32_t n, int32_t type,
                               int32_t seqid);                            /* :387-457 */
size_t kxo_message_begin_length(uint32_t name_len);                       /* :338 */
int kxo_read_message_begin(const uint8_t* b, size_t len, uint32_t* name_off, uint32_t* name_len,
                           int32_t* type, int32_t* seqid, size_t* used);

/* -------- skip decoder: netpollSkipDecoder.skipType (codec_apache.go:191-293) -------- */
int kxo_skip(const uint8_t* b, size_t len, uint8_t ttype, int maxdepth, size_t* used);
/* SkipStruct over n concatenated records (codec_apache.go:166-172): offsets_out[n+1]. */
int kxo_skip_batch(const uint8_t* b, size_t len, uint64_t n, uint64_t* offsets_out,
                   uint64_t* n_done);

/* -------- schema flattening (independent of the product's) -------- */
int kxo_flatten(const kx_struct_desc* structs, uint32_t nstructs, kx_column_info* cols,
                uint32_t* ncols, uint32_t* npresence);

/* -------- generated FastRead over a batch (struct_tpl.go:41-149, 405-625) --------
 * Columns are HOST memory laid out exactly like the device API (kxcodec.h). */
int kxo_thrift_decode(const kx_struct_desc* structs, uint32_t nstructs, const uint8_t* in,
                      uint64_t in_len, const uint64_t* offsets, uint64_t n,
                      const kx_columns* out, uint8_t* record_status, kx_status* st);
/* Same, partitioned over `threads` pthreads (offsets required): the CPU baseline. */
int kxo_thrift_decode_mt(const kx_struct_desc* structs, uint32_t nstructs, const uint8_t* in,
                         uint64_t in_len, const uint64_t* offsets, uint64_t n,
                         const kx_columns* out, kx_status* st, int threads);

/* -------- generated BLength / FastWriteNocopy (struct_tpl.go:225-391, patcher.go:503-522) -------- */
int kxo_thrift_sizes(const kx_struct_desc* structs, uint32_t nstructs, const kx_columns* in,
                     uint64_t n, uint64_t* sizes);
int kxo_thrift_encode(const kx_struct_desc* structs, uint32_t nstructs, const kx_columns* in,
                      uint64_t n, uint8_t* out, uint64_t cap, uint64_t* offsets_out,
                      uint64_t* total);
int kxo_thrift_encode_mt(const kx_struct_desc* structs, uint32_t nstructs, const kx_columns* in,
                         uint64_t n, uint8_t* out, uint64_t cap, uint64_t* offsets_out,
                         uint64_t* total, int threads);

/* -------- Kitex-Protobuf (protobuf.go:32-47,64-216) + proto3 body -------- */
size_t kxo_pb_write_meta(uint8_t* b, const char* method, uint32_t n, int32_t msg_type,
                         int32_t seqid);
int kxo_pb_read_meta(const uint8_t* b, size_t len, uint32_t* method_off, uint32_t* method_len,
                     int32_t* msg_type, int32_t* seqid, size_t* used);
size_t kxo_put_uvarint(uint8_t* b, uint64_t v);
int kxo_get_uvarint(const uint8_t* b, size_t len, uint64_t* v, size_t* used);
int kxo_pb_decode(const kx_struct_desc* structs, uint32_t nstructs, const uint8_t* in,
                  uint64_t in_len, const uint64_t* offsets, uint64_t n, const kx_columns* out,
                  uint8_t* record_status, kx_status* st);
int kxo_pb_decode_mt(const kx_struct_desc* structs, uint32_t nstructs, const uint8_t* in,
                     uint64_t in_len, const uint64_t* offsets, uint64_t n, const kx_columns* out,
                     kx_status* st, int threads);
/* Encode n records as `Batch { repeated Rec recs = 1; }` (offsets_out: start of each record's body). */
int kxo_pb_encode(const kx_struct_desc* structs, uint32_t nstructs, const kx_columns* in,
                  uint64_t n, uint8_t* out, uint64_t cap, uint64_t* offsets_out, uint64_t* total);

/* -------- framing sniff and CRC32C payload validation (default_codec.go, validate.go) -------- */
int kxo_frame_one(const uint8_t* b, uint64_t len, uint64_t max_payload, uint64_t* flen, uint64_t* ps,
                  uint64_t* pe, uint8_t* kind);
int kxo_frame_scan(const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t max_payload, uint64_t* frame_offsets,
                   uint64_t* pay_start, uint64_t* pay_end, uint8_t* kinds, uint64_t* n_done);
int kxo_ttstream_frame_one(const uint8_t* b, uint64_t len, const kx_ttstream_keys* keys, uint64_t* flen,
                           uint64_t* ps, uint64_t* pe, uint8_t* ftype, int32_t* sid, uint64_t* mpos, uint32_t* mlen);
int kxo_ttstream_frame_scan(const uint8_t* in, uint64_t in_len, uint64_t n, const kx_ttstream_keys* keys,
                            uint64_t* frame_offsets, uint64_t* pay_start, uint64_t* pay_end, uint8_t* ftypes,
                            int32_t* sids, uint64_t* mpos, uint32_t* mlen, uint64_t* n_done);
int kxo_raw_messages(const uint8_t* in, uint64_t in_len, const uint64_t* offsets, uint64_t n, uint64_t* name_pos,
                     uint64_t* name_len, int32_t* msg_type, int32_t* seqid, uint8_t* rs);
int kxo_set_seqids(uint8_t* in, uint64_t in_len, const uint64_t* offsets, uint64_t n, const int32_t* seqids,
                   uint8_t* rs);
int kxo_grpc_frame_scan(const uint8_t* in, uint64_t in_len, uint64_t n, uint64_t max_payload,
                        uint64_t* frame_offsets, uint64_t* pay_start, uint64_t* pay_end, uint8_t* flags,
                        uint64_t* n_done);
uint32_t kxo_crc32c(uint32_t crc, const uint8_t* p, uint64_t n);
int kxo_crc32c_batch(const uint8_t* in, uint64_t in_len, const uint64_t* offsets, uint64_t n, uint32_t* crc_out);
int kxo_frame_crc32c_validate(const uint8_t* in, uint64_t in_len, const uint64_t* frame_offsets, uint64_t n,
                              uint32_t* crc_out, uint8_t* record_status, uint64_t* first_bad);

/* -------- synthetic inputs: splitmix64 -------- */
uint64_t kxo_splitmix64(uint64_t x);

/* nested schemas (kx_oracle_nested.c; include/kxcodec.h "Nested schemas") */
int kxo_nflatten(const kx_struct_desc* structs, uint32_t nstructs, kx_column_info* cols, uint32_t* ncols,
                 uint32_t* npresence);
int kxo_nthrift_decode(const kx_struct_desc* structs, uint32_t nstructs, const uint8_t* in, uint64_t in_len,
                       const uint64_t* offsets, uint64_t n, const kx_columns* out, uint8_t* record_status,
                       kx_status* st);
int kxo_nthrift_encode(const kx_struct_desc* structs, uint32_t nstructs, const kx_columns* in, uint64_t n,
                       uint8_t* out, uint64_t cap, uint64_t* sizes, uint64_t* offsets_out, uint64_t* total);
int kxo_is_nested(const kx_struct_desc* structs, uint32_t nstructs);
/* Kitex-Protobuf nested messages (KX_STRUCT_PROTOBUF; kx_oracle_nested.c): proto.Unmarshal / proto.Marshal */
int kxo_npb_decode(const kx_struct_desc* structs, uint32_t nstructs, const uint8_t* in, uint64_t in_len,
                   const uint64_t* offsets, uint64_t n, const kx_columns* out, uint8_t* record_status,
                   kx_status* st);
int kxo_npb_encode(const kx_struct_desc* structs, uint32_t nstructs, const kx_columns* in, uint64_t n,
                   uint8_t* out, uint64_t cap, uint64_t* offsets_out, uint64_t* total);

#ifdef __cplusplus
}
#endif
#endif
