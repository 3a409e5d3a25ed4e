// kx_shard.hip — concatenation of record-range shards into one rank (include/kxcodec.h
// "multi-GPU record-range shards"). The exchange itself (all-gather of the headers, point-to-point pieces)
// belongs to the host's collective library (RCCL over xGMI); what lives here is everything around it that
// needs the column layout: the per-rank header (a one-wave kernel reading the first and last offsets of
// every level of every var column), the plan (host: which element range of which array each rank sends
// and where it lands), and the rebase of the received offsets (a kernel adding each piece's base).
#include <string.h>

#include "kx_internal.h"

namespace {

int set_device(kx_ctx* c) {
  KX_HIP_CHECK(hipSetDevice(c->device));
  return KX_OK;
}

// offsets levels above the data array, per column kind (0: FIXED)
__host__ __device__ inline uint32_t col_depth(uint32_t kind) {
  switch (kind) {
    case KX_COL_BYTES: case KX_COL_LIST: return 1;
    case KX_COL_LIST_BYTES: case KX_COL_LIST2: return 2;
    case KX_COL_LIST2_BYTES: return 3;
    default: return 0;
  }
}

inline uint32_t data_width(const kx_column_info& ci) {
  switch (ci.kind) {
    case KX_COL_FIXED: case KX_COL_LIST: case KX_COL_LIST2: return ci.width;
    default: return 1;   // string bytes
  }
}

struct MetaCol {
  const void* arr[3];    // offsets, elem_offsets, sub_offsets
  uint32_t depth, ob, word, view;
};
struct MetaParams {
  MetaCol col[KX_MAX_COLUMNS];
  uint32_t ncols;
  uint64_t n, in_len;
  uint64_t* meta;
};

__device__ __forceinline__ uint64_t rd_off(const void* a, uint32_t ob, uint64_t i) {
  return ob == 8 ? ((const uint64_t*)a)[i] : (uint64_t)((const uint32_t*)a)[i];
}

// one lane per column: its chain of offsets arrays, level by level
__global__ void __launch_bounds__(64) meta_kernel(MetaParams p) {
  const uint32_t c = threadIdx.x;
  if (c == 0) { p.meta[0] = p.n; p.meta[1] = p.in_len; }
  if (c >= p.ncols || !p.col[c].depth) return;
  const MetaCol& M = p.col[c];
  uint64_t* w = p.meta + M.word;
  if (M.view) {
    for (uint32_t j = 0; j < M.depth; j++) { w[2 * j] = 0; w[2 * j + 1] = 0; }
    return;
  }
  uint64_t f = rd_off(M.arr[0], M.ob, 0), l = rd_off(M.arr[0], M.ob, p.n);
  w[0] = f;
  w[1] = l - f;
  for (uint32_t j = 1; j < M.depth; j++) {
    const uint64_t f2 = rd_off(M.arr[j], M.ob, f), l2 = rd_off(M.arr[j], M.ob, l);
    w[2 * j] = f2;
    w[2 * j + 1] = l2 - f2;
    f = f2;
    l = l2;
  }
}

// rebase jobs: dst[i] = src[i] + delta (offsets, src 4 or 8 bytes); views (src pairs of 4 bytes packed in one
// word, or of 8 bytes): (off + delta, len) when len != 0, else (0, 0); const: dst[0] = delta
enum : uint32_t { J_OFFS = 0, J_VIEW4 = 1, J_VIEW8 = 2, J_CONST = 3 };
struct RebaseJob {
  const void* src;
  uint64_t* dst;
  uint64_t count;
  int64_t delta;
  uint32_t src_bytes, mode;
};
constexpr int JOBS = 24;
struct RebaseParams {
  RebaseJob job[JOBS];
  uint32_t njobs;
};

__global__ void __launch_bounds__(256) rebase_kernel(RebaseParams p) {
  const uint32_t jb = blockIdx.y;
  if (jb >= p.njobs) return;
  const RebaseJob& J = p.job[jb];
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < J.count; i += stride) {
    switch (J.mode) {
      case J_OFFS:
        J.dst[i] = (J.src_bytes == 8 ? ((const uint64_t*)J.src)[i] : (uint64_t)((const uint32_t*)J.src)[i]) +
                   (uint64_t)J.delta;
        break;
      case J_VIEW4: {
        const uint64_t x = ((const uint64_t*)J.src)[i];
        const uint64_t len = x >> 32;
        J.dst[2 * i] = len ? (x & 0xffffffffull) + (uint64_t)J.delta : 0;
        J.dst[2 * i + 1] = len;
        break;
      }
      case J_VIEW8: {
        const uint64_t o = ((const uint64_t*)J.src)[2 * i], len = ((const uint64_t*)J.src)[2 * i + 1];
        J.dst[2 * i] = len ? o + (uint64_t)J.delta : 0;
        J.dst[2 * i + 1] = len;
        break;
      }
      default:
        J.dst[i] = (uint64_t)J.delta;
    }
  }
}

inline void* arr_of(const kx_column& k, uint32_t a) {
  return a == 0 ? k.offsets : a == 1 ? k.elem_offsets : a == 2 ? k.sub_offsets : k.data;
}

inline uint32_t off_bytes(const kx_column& k) { return k.offset_bytes == 8 ? 8u : 4u; }

}  // namespace

extern "C" {

uint32_t kx_shard_meta_words(const kx_column_info* infos, uint32_t ncols) {
  if (!infos || ncols > KX_MAX_COLUMNS) return 0;
  uint32_t w = 2;
  for (uint32_t c = 0; c < ncols; c++) w += 2 * col_depth(infos[c].kind);
  return w;
}

int kx_shard_meta(kx_ctx* c, const kx_column_info* infos, uint32_t ncols, const kx_columns* cols, uint64_t n,
                  uint64_t in_len, uint64_t* meta, void* stream) {
  if (!c || !infos || !cols || !meta || cols->ncols != ncols || ncols > KX_MAX_COLUMNS) return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  MetaParams p{};
  p.ncols = ncols;
  p.n = n;
  p.in_len = in_len;
  p.meta = meta;
  uint32_t w = 2;
  for (uint32_t k = 0; k < ncols; k++) {
    const kx_column& col = cols->cols[k];
    MetaCol& M = p.col[k];
    M.depth = col_depth(infos[k].kind);
    M.ob = off_bytes(col);
    M.word = w;
    M.view = (col.flags & KX_COLF_VIEW) ? 1u : 0u;
    for (uint32_t a = 0; a < 3; a++) M.arr[a] = arr_of(col, a);
    for (uint32_t a = 0; a < M.depth && !M.view; a++)
      if (!M.arr[a]) return KX_ERR_INVALID_ARG;
    w += 2 * M.depth;
  }
  hipLaunchKernelGGL(meta_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, p);
  KX_HIP_CHECK(hipGetLastError());
  return KX_OK;
}

int kx_concat_plan(const kx_column_info* infos, uint32_t ncols, const kx_columns* layout, const uint64_t* metas,
                   uint32_t world, kx_concat_piece* pieces, uint32_t* npieces, kx_concat_sizes* sizes) {
  if (!infos || !layout || !metas || !npieces || !sizes || world == 0 || layout->ncols != ncols ||
      ncols > KX_MAX_COLUMNS)
    return KX_ERR_INVALID_ARG;
  const uint32_t words = kx_shard_meta_words(infos, ncols);
  std::vector<uint32_t> word(ncols);
  for (uint32_t c = 0, w = 2; c < ncols; c++) { word[c] = w; w += 2 * col_depth(infos[c].kind); }
  auto M = [&](uint32_t r, uint32_t i) { return metas[(uint64_t)r * words + i]; };
  // prefix sums over ranks: records, input bytes, units of every level of every column
  std::vector<uint64_t> rec0(world + 1, 0), in0(world + 1, 0);
  for (uint32_t r = 0; r < world; r++) { rec0[r + 1] = rec0[r] + M(r, 0); in0[r + 1] = in0[r] + M(r, 1); }
  // base[(c * 3 + j) * (world + 1) + r]: units of level j of column c held by ranks before r
  std::vector<uint64_t> base((size_t)ncols * 3 * (world + 1), 0);
  auto B = [&](uint32_t c, uint32_t j, uint32_t r) -> uint64_t& { return base[((size_t)c * 3 + j) * (world + 1) + r]; };
  for (uint32_t c = 0; c < ncols; c++)
    for (uint32_t j = 0; j < col_depth(infos[c].kind); j++)
      for (uint32_t r = 0; r < world; r++) B(c, j, r + 1) = B(c, j, r) + M(r, word[c] + 2 * j + 1);
  memset(sizes, 0, sizeof(*sizes));
  sizes->n = rec0[world];
  sizes->in_len = in0[world];
  uint32_t np = 0;
  const uint32_t cap = *npieces;
  auto add = [&](uint32_t r, uint32_t col, uint32_t a, uint32_t eb, uint64_t src, uint64_t cnt, uint64_t dst,
                 int64_t rb) {
    if (np < cap && pieces) pieces[np] = kx_concat_piece{r, col, a, eb, src, cnt, dst, rb};
    np++;
  };
  for (uint32_t c = 0; c < ncols; c++) {
    const kx_column_info& ci = infos[c];
    const uint32_t k = col_depth(ci.kind);
    const bool view = (layout->cols[c].flags & KX_COLF_VIEW) != 0;
    if (ci.kind == KX_COL_FIXED || view) sizes->units[c][view ? KX_PIECE_OFFSETS : KX_PIECE_DATA] = rec0[world];
    if (ci.kind == KX_COL_FIXED || view) continue;
    sizes->units[c][0] = rec0[world];
    for (uint32_t j = 1; j < k; j++) sizes->units[c][j] = B(c, j - 1, world);
    sizes->units[c][KX_PIECE_DATA] = B(c, k - 1, world);
  }
  for (uint32_t r = 0; r < world; r++) {
    const uint64_t n = M(r, 0);
    for (uint32_t c = 0; c < ncols; c++) {
      const kx_column_info& ci = infos[c];
      const kx_column& L = layout->cols[c];
      const uint32_t k = col_depth(ci.kind);
      if (ci.kind == KX_COL_FIXED) {
        add(r, c, KX_PIECE_DATA, ci.width, 0, n, rec0[r], 0);
        continue;
      }
      if (L.flags & KX_COLF_VIEW) {   // (offset, length) pairs: one u64 per record (4-byte pairs) or two
        add(r, c, KX_PIECE_OFFSETS, off_bytes(L) == 8 ? 16u : 8u, 0, n, rec0[r], (int64_t)in0[r]);
        continue;
      }
      const uint64_t w0 = word[c];
      add(r, c, KX_PIECE_OFFSETS, off_bytes(L), 0, n, rec0[r], (int64_t)(B(c, 0, r) - M(r, w0)));
      for (uint32_t j = 1; j < k; j++)
        add(r, c, j, off_bytes(L), M(r, w0 + 2 * (j - 1)), M(r, w0 + 2 * (j - 1) + 1), B(c, j - 1, r),
            (int64_t)(B(c, j, r) - M(r, w0 + 2 * j)));
      add(r, c, KX_PIECE_DATA, data_width(ci), M(r, w0 + 2 * (k - 1)), M(r, w0 + 2 * (k - 1) + 1), B(c, k - 1, r), 0);
    }
    if (layout->presence) add(r, KX_MAX_COLUMNS, KX_PIECE_DATA, 8, 0, n, rec0[r], 0);
  }
  const int rc = np > cap || (!pieces && np) ? KX_ERR_SIZE_LIMIT : KX_OK;
  *npieces = np;
  return rc;
}

int kx_concat_rebase(kx_ctx* c, const kx_column_info* infos, uint32_t ncols, const kx_concat_piece* pieces,
                     uint32_t npieces, const kx_columns* staging, const kx_columns* out, const kx_concat_sizes* sizes,
                     void* stream) {
  if (!c || !infos || (!pieces && npieces) || !staging || !out || !sizes || staging->ncols != ncols ||
      out->ncols != ncols || ncols > KX_MAX_COLUMNS)
    return KX_ERR_INVALID_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  RebaseParams p{};
  uint64_t maxc = 0;
  auto flush = [&]() -> int {
    if (!p.njobs) return KX_OK;
    const unsigned gx = (unsigned)kmax64(1, kmin64(256, (maxc + 255) / 256));
    hipLaunchKernelGGL(rebase_kernel, dim3(gx, p.njobs), dim3(256), 0, st, p);
    KX_HIP_CHECK(hipGetLastError());
    p.njobs = 0;
    maxc = 0;
    return KX_OK;
  };
  auto job = [&](const void* src, uint64_t* dst, uint64_t cnt, int64_t delta, uint32_t sb, uint32_t mode) -> int {
    if (!cnt) return KX_OK;
    if (!dst || (mode != J_CONST && !src)) return KX_ERR_INVALID_ARG;
    p.job[p.njobs++] = RebaseJob{src, dst, cnt, delta, sb, mode};
    maxc = kmax64(maxc, cnt);
    return p.njobs == JOBS ? flush() : KX_OK;
  };
  for (uint32_t i = 0; i < npieces; i++) {
    const kx_concat_piece& P = pieces[i];
    if (P.column >= ncols || P.array == KX_PIECE_DATA) continue;   // data pieces land in place
    const kx_column& S = staging->cols[P.column];
    const kx_column& O = out->cols[P.column];
    if (O.offset_bytes != 8) return KX_ERR_INVALID_ARG;   // the concatenation's offsets never wrap
    const char* src = (const char*)arr_of(S, P.array);
    uint64_t* dst = (uint64_t*)arr_of(O, P.array);
    if (S.flags & KX_COLF_VIEW) {
      if ((rc = job(src ? src + P.dst_first * P.elem_bytes : nullptr, dst ? dst + 2 * P.dst_first : nullptr, P.count,
                    P.rebase, P.elem_bytes, P.elem_bytes == 16 ? J_VIEW8 : J_VIEW4)))
        return rc;
    } else {
      if ((rc = job(src ? src + P.dst_first * P.elem_bytes : nullptr, dst ? dst + P.dst_first : nullptr, P.count,
                    P.rebase, P.elem_bytes, J_OFFS)))
        return rc;
    }
  }
  // closing entries: offsets array j ends at units[j] with the units of the next array
  for (uint32_t col = 0; col < ncols; col++) {
    const uint32_t k = col_depth(infos[col].kind);
    if (!k || (out->cols[col].flags & KX_COLF_VIEW)) continue;
    for (uint32_t j = 0; j < k; j++) {
      uint64_t* dst = (uint64_t*)arr_of(out->cols[col], j);
      const uint64_t next = sizes->units[col][j + 1 < k ? j + 1 : KX_PIECE_DATA];
      if ((rc = job(nullptr, dst ? dst + sizes->units[col][j] : nullptr, 1, (int64_t)next, 8, J_CONST))) return rc;
    }
  }
  return flush();
}

}  // extern "C"
