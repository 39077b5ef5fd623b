// SelectionExec (K3b): order-preserving compaction of the rows whose predicate is true.
// Build-defined operator (absent in the reference; interface PhysicalPlan K:442-446):
// a null predicate drops the row; the output keeps input row order (bit-exact parity).
//
// Algorithm (no atomics on the data path, deterministic):
//   1. k_tile_count : per 8192-row tile, popcount(mask & validity)      -> tile_counts
//   2. k_scan       : exclusive scan of tile counts (one block)          -> tile_offsets, total
//   3. k_compact    : per tile, 4 rows per lane; the lane's rank inside the wave comes from
//                     the 3 bit-planes of its per-lane count via ballot + mbcnt; wave totals are
//                     scanned through LDS; selected values are written at their final position.
// Traffic per input row: mask 1/8 B twice + every gathered column once + selected rows written.
#include "qe_internal.hpp"

namespace qe {

constexpr int FT_THREADS = 256;
constexpr int FT_ROWS_PER_LANE = 4;
constexpr int FT_ITERS = 8;
constexpr int64_t FT_TILE = (int64_t)FT_THREADS * FT_ROWS_PER_LANE * FT_ITERS;  // 8192 rows

__device__ __forceinline__ uint8_t sel_byte(const uint8_t* __restrict__ mv, const uint8_t* __restrict__ ml,
                                            int64_t byte, int64_t n) {
  uint8_t s = mv[byte];
  if (ml) s &= ml[byte];
  const int64_t r0 = byte << 3;
  if (r0 + 8 > n) s &= (uint8_t)((1u << (n - r0)) - 1);
  return s;
}

__global__ void __launch_bounds__(FT_THREADS) k_tile_count(const uint8_t* __restrict__ mv,
                                                           const uint8_t* __restrict__ ml, int64_t n,
                                                           int64_t* __restrict__ tile_counts) {
  __shared__ int64_t part[FT_THREADS / 64];
  const int64_t tile = blockIdx.x;
  const int64_t nbytes = (n + 7) >> 3;
  const int64_t b0 = tile * (FT_TILE / 8);  // 1024 bytes per tile, 4 per thread
  int c = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t b = b0 + k * FT_THREADS + threadIdx.x;
    if (b < nbytes) c += __popc(sel_byte(mv, ml, b, n));
  }
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int w = 0; w < FT_THREADS / 64; ++w) t += part[w];
    tile_counts[tile] = t;
  }
}

// Device-wide int64 exclusive scans. A 1024-thread block takes tiles of 8192 elements; wave w of
// the block holds elements 512 w + 64 k + lane (k < 8) of a tile, so every load and store
// instruction moves one contiguous 512-byte row (round 4 gave each thread 8 consecutive elements:
// 64-byte lane strides, and the one-block scan walked its chunks serially: 16.6 us per call for
// the CSV scan's 23.5K segment counts, 54 us for a 4M-row length column).
constexpr int GS_THREADS = 1024, GS_PER = 8;
constexpr int64_t GS_TILE = (int64_t)GS_THREADS * GS_PER;

__device__ __forceinline__ void tile_load(const int64_t* __restrict__ in, int64_t n, int64_t b0, int64_t (&v)[GS_PER]) {
  const int64_t e0 = b0 + (int64_t)(threadIdx.x >> 6) * 512 + (threadIdx.x & 63);
#pragma unroll
  for (int k = 0; k < GS_PER; ++k) v[k] = e0 + 64 * k < n ? in[e0 + 64 * k] : 0;
}

// Exclusive prefixes of a loaded tile (+ carry) stored to out; returns the tile's total.
__device__ __forceinline__ int64_t tile_scan_store(const int64_t (&v)[GS_PER], int64_t* __restrict__ out, int64_t n,
                                                   int64_t b0, int64_t carry, int64_t* wsum) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t run = 0, ex[GS_PER];
#pragma unroll
  for (int k = 0; k < GS_PER; ++k) {  // row k of the wave: inclusive lane scan, then the rows before
    int64_t x = v[k];
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int64_t y = __shfl_up(x, off);
      if (lane >= off) x += y;
    }
    ex[k] = run + x - v[k];
    run += __shfl(x, 63);
  }
  if (lane == 0) wsum[wid] = run;
  __syncthreads();
  int64_t wprefix = 0, all = 0;
#pragma unroll
  for (int w = 0; w < GS_THREADS / 64; ++w) {
    if (w < wid) wprefix += wsum[w];
    all += wsum[w];
  }
  __syncthreads();  // wsum is rewritten by the next tile
  const int64_t e0 = b0 + (int64_t)wid * 512 + lane;
#pragma unroll
  for (int k = 0; k < GS_PER; ++k)
    if (e0 + 64 * k < n) out[e0 + 64 * k] = carry + wprefix + ex[k];
  return all;
}

// One block, any n (writes the total to out[n], and to *total2 when given): KS_TILES tiles' loads
// are issued before the first of them is scanned, so up to KS_TILES tiles the block waits for
// memory once.
constexpr int KS_TILES = 1;
__global__ void __launch_bounds__(1024) k_scan(const int64_t* __restrict__ in, int64_t* __restrict__ out,
                                               int64_t n, int64_t* __restrict__ total2 = nullptr) {
  __shared__ int64_t wsum[16];
  int64_t carry = 0;
  for (int64_t g0 = 0; g0 < n; g0 += KS_TILES * GS_TILE) {
    int64_t v[KS_TILES][GS_PER];
#pragma unroll
    for (int t = 0; t < KS_TILES; ++t) tile_load(in, n, g0 + t * GS_TILE, v[t]);
#pragma unroll
    for (int t = 0; t < KS_TILES; ++t)
      if (g0 + t * GS_TILE < n) carry += tile_scan_store(v[t], out, n, g0 + t * GS_TILE, carry, wsum);
  }
  if (threadIdx.x == 0) {
    out[n] = carry;
    if (total2) *total2 = carry;
  }
}

__global__ void __launch_bounds__(GS_THREADS) k_scan_reduce(const int64_t* __restrict__ in, int64_t n,
                                                             int64_t* __restrict__ sums) {
  __shared__ int64_t wsum[GS_THREADS / 64];
  int64_t v[GS_PER];
  tile_load(in, n, blockIdx.x * GS_TILE, v);
  int64_t t = 0;
#pragma unroll
  for (int k = 0; k < GS_PER; ++k) t += v[k];
  for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t all = 0;
    for (int w = 0; w < GS_THREADS / 64; ++w) all += wsum[w];
    sums[blockIdx.x] = all;
  }
}

__global__ void __launch_bounds__(GS_THREADS) k_scan_apply(const int64_t* __restrict__ in, int64_t* __restrict__ out,
                                                            int64_t n, const int64_t* __restrict__ offs, int64_t nb) {
  __shared__ int64_t wsum[GS_THREADS / 64];
  int64_t v[GS_PER];
  tile_load(in, n, blockIdx.x * GS_TILE, v);
  (void)tile_scan_store(v, out, n, blockIdx.x * GS_TILE, offs[blockIdx.x], wsum);
  if (blockIdx.x == nb - 1 && threadIdx.x == 0) out[n] = offs[nb];
}

int exclusive_scan_i64(qe_ctx* ctx, const int64_t* in, int64_t* out, int64_t n) {
  if (n <= KS_TILES * GS_TILE) {
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, ctx->stream, in, out, n, (int64_t*)nullptr);
    return launch_check("k_scan");
  }
  const int64_t nb = (n + GS_TILE - 1) / GS_TILE;
  const size_t need = (size_t)(2 * nb + 2) * 8;
  if (need > ctx->scan_tmp_bytes) {
    if (ctx->scan_tmp) {
      QE_TRY(ctx_sync(ctx));
      QE_HIP(hipFree(ctx->scan_tmp));
    }
    ctx->scan_tmp = nullptr;
    ctx->scan_tmp_bytes = 0;
    QE_HIP(hipMalloc(&ctx->scan_tmp, need));
    ctx->scan_tmp_bytes = need;
  }
  int64_t* sums = (int64_t*)ctx->scan_tmp;
  int64_t* offs = sums + nb + 1;
  hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)nb), dim3(GS_THREADS), 0, ctx->stream, in, n, sums);
  QE_TRY(launch_check("k_scan_reduce"));
  hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, ctx->stream, sums, offs, nb, (int64_t*)nullptr);
  QE_TRY(launch_check("k_scan"));
  hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)nb), dim3(GS_THREADS), 0, ctx->stream, in, out, n, offs, nb);
  return launch_check("k_scan_apply");
}

struct GatherCol {
  const void* in;
  const uint8_t* in_valid;
  void* out;
  uint32_t* out_valid;  // zeroed by the host; whole words from the tile's LDS bitmap (atomicOr at its edges)
  int32_t width;        // 8, 4 or 1; 0 = UTF-8 (out = int64 {src offset, length} per selected row)
  int32_t pad;
  const int32_t* in_offs;  // UTF-8 input offsets
};

constexpr int FT_MAX_COLS = 8;
struct GatherArgs {
  GatherCol cols[FT_MAX_COLS];
  int32_t ncols;
};

__device__ __forceinline__ void gather_store(const GatherCol& c, int64_t row0, int nsel_mask, int64_t pos0,
                                             const int (&rank)[4], bool full, uint32_t* lbits, int64_t tb) {
  // Loads the lane's 4 rows (vectorised when the tile is full) and stores the selected ones.
  if (c.width == 0) {  // UTF-8: record (source byte offset, length); bytes are copied after the scan
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if ((nsel_mask >> j) & 1) {
        const int32_t s0 = c.in_offs[row0 + j], s1 = c.in_offs[row0 + j + 1];
        ((int2*)c.out)[pos0 + rank[j]] = make_int2(s0, s1 - s0);
      }
    }
  } else if (c.width == 8) {
    int64_t v[4];
    if (full) {
      typedef long long i64x2 __attribute__((ext_vector_type(2)));
      const i64x2* p = (const i64x2*)((const int64_t*)c.in + row0);
      const i64x2 a = p[0], b = p[1];
      v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (nsel_mask >> j) & 1 ? ((const int64_t*)c.in)[row0 + j] : 0;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if ((nsel_mask >> j) & 1) ((int64_t*)c.out)[pos0 + rank[j]] = v[j];
  } else if (c.width == 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if ((nsel_mask >> j) & 1) ((int32_t*)c.out)[pos0 + rank[j]] = ((const int32_t*)c.in)[row0 + j];
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if ((nsel_mask >> j) & 1) ((uint8_t*)c.out)[pos0 + rank[j]] = ((const uint8_t*)c.in)[row0 + j];
  }
  if (c.out_valid) {  // validity bits at tile-local output positions in LDS (written out per tile)
    const uint8_t vb = c.in_valid ? (uint8_t)(c.in_valid[row0 >> 3] >> (row0 & 7)) : (uint8_t)0xF;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (((nsel_mask >> j) & 1) && ((vb >> j) & 1)) {
        const int p = (int)(pos0 + rank[j] - tb);
        atomicOr(&lbits[p >> 5], 1u << (p & 31));
      }
    }
  }
}

// A tile's validity bits (LDS, tile-local compacted order) -> the output bitmap words of its range
// [tb, tb + total): words inside the range are this tile's alone (plain stores), the first and last
// may share bits with the neighbouring tiles (atomicOr into the zeroed bitmap).
__device__ __forceinline__ void flush_valid_bits(uint32_t* out_valid, const uint32_t* lbits, int64_t tb, int64_t total) {
  const int64_t w0 = tb >> 5;
  const int64_t nw = total ? ((tb + total - 1) >> 5) - w0 + 1 : 0;
  for (int64_t i = threadIdx.x; i < nw; i += blockDim.x) {
    const int64_t l0 = ((w0 + i) << 5) - tb;  // tile-local bit of the word's bit 0
    uint32_t v;
    if (l0 < 0) {
      v = lbits[0] << (uint32_t)(-l0);
    } else {
      const uint32_t q = (uint32_t)(l0 >> 5), sh = (uint32_t)(l0 & 31);
      v = sh ? (lbits[q] >> sh) | (lbits[q + 1] << (32u - sh)) : lbits[q];
    }
    uint32_t* dst = out_valid + (w0 + i);
    if (l0 >= 0 && l0 + 32 <= total) *dst = v;
    else if (v) atomicOr(dst, v);
  }
}

__global__ void __launch_bounds__(FT_THREADS) k_compact(const uint8_t* __restrict__ mv, const uint8_t* __restrict__ ml,
                                                        int64_t n, const int64_t* __restrict__ tile_offsets,
                                                        GatherArgs args) {
  __shared__ int wtot[FT_THREADS / 64];
  constexpr int VW = (int)(FT_TILE / 32) + 1;  // a tile's output validity words (+1: shifted reads)
  __shared__ uint32_t s_vb[FT_MAX_COLS][VW];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t tile = blockIdx.x;
  int64_t base = tile_offsets[tile];
  const int64_t tb = base;
  for (int k = 0; k < args.ncols; ++k)
    if (args.cols[k].out_valid)
      for (int i = threadIdx.x; i < VW; i += FT_THREADS) s_vb[k][i] = 0u;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int it = 0; it < FT_ITERS; ++it) {
    const int64_t row0 = tile * FT_TILE + (int64_t)it * (FT_THREADS * FT_ROWS_PER_LANE) +
                         (int64_t)threadIdx.x * FT_ROWS_PER_LANE;
    int sel = 0;
    if (row0 < n) sel = (sel_byte(mv, ml, row0 >> 3, n) >> (row0 & 7)) & 0xF;
    const int c = __popc(sel);
    // exclusive prefix of c over lanes, from its bit planes
    const uint64_t b0 = __ballot(c & 1), b1 = __ballot(c & 2), b2 = __ballot(c & 4);
    const int prefix = __popcll(b0 & lt) + 2 * __popcll(b1 & lt) + 4 * __popcll(b2 & lt);
    const int total = __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
    if (lane == 0) wtot[wid] = total;
    __syncthreads();
    int woff = 0, btot = 0;
#pragma unroll
    for (int w = 0; w < FT_THREADS / 64; ++w) {
      woff += w < wid ? wtot[w] : 0;
      btot += wtot[w];
    }
    if (sel) {
      int rank[4];
      int r = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        rank[j] = r;
        r += (sel >> j) & 1;
      }
      const int64_t pos0 = base + woff + prefix;
      const bool full = row0 + 4 <= n;
      for (int k = 0; k < args.ncols; ++k) gather_store(args.cols[k], row0, sel, pos0, rank, full, s_vb[k], tb);
    }
    base += btot;
    __syncthreads();
  }
  for (int k = 0; k < args.ncols; ++k)
    if (args.cols[k].out_valid) flush_valid_bits(args.cols[k].out_valid, s_vb[k], tb, base - tb);
}

// ---- UTF-8 gather: (src, len) pairs -> offsets (device-wide exclusive scan) -> bytes ------------
constexpr int SC_TILE = 2048;  // elements per tile, 8 per thread

__global__ void __launch_bounds__(256) k_len_tile_sum(const int2* __restrict__ sl, int64_t n, int64_t* __restrict__ sums) {
  __shared__ int64_t part[4];
  int64_t c = 0;
  const int64_t b0 = (int64_t)blockIdx.x * SC_TILE;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int64_t i = b0 + k * 256 + threadIdx.x;
    if (i < n) c += sl[i].y;
  }
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) sums[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// offsets[i] = tile_offset + exclusive prefix of lengths inside the tile; offsets[n] = total.
__global__ void __launch_bounds__(256) k_len_tile_scan(const int2* __restrict__ sl, int64_t n,
                                                       const int64_t* __restrict__ tile_off, int32_t* __restrict__ offs) {
  __shared__ int64_t wsum[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t base = (int64_t)blockIdx.x * SC_TILE + (int64_t)threadIdx.x * 8;  // 8 consecutive per thread
  int64_t v[8], t = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    v[k] = base + k < n ? sl[base + k].y : 0;
    t += v[k];
  }
  int64_t x = t;  // inclusive scan of thread totals within the wave
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  int64_t run = tile_off[blockIdx.x] + x - t;
  for (int w = 0; w < wid; ++w) run += wsum[w];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (base + k < n) offs[base + k] = (int32_t)run;
    run += v[k];
  }
}

__global__ void k_write_total(const int64_t* __restrict__ total, int32_t* __restrict__ offs, int64_t n) {
  offs[n] = (int32_t)*total;
}

__global__ void __launch_bounds__(256) k_copy_bytes(const int2* __restrict__ sl, const int32_t* __restrict__ offs,
                                                    const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int2 e = sl[i];
    const uint8_t* s = src + e.x;
    uint8_t* d = dst + offs[i];
    for (int k = 0; k < e.y; ++k) d[k] = s[k];
  }
}

struct FilterPlan {
  int64_t ntiles;
  int64_t* counts;   // ntiles
  int64_t* offsets;  // ntiles + 1
};

static int filter_prepare(qe_ctx* ctx, const qe_column* mask, FilterPlan* fp, int64_t* d_total = nullptr) {
  QE_CHECK(mask && mask->type == QE_TYPE_BOOL, QE_ERR_INVALID_ARG, "mask must be a BOOL column");
  QE_CHECK(mask->values || mask->length == 0, QE_ERR_INVALID_ARG, "null mask values");
  const int64_t n = mask->length;
  fp->ntiles = (int64_t)div_up((uint64_t)n, FT_TILE);
  void* s;
  QE_TRY(ctx_scratch(ctx, (size_t)(2 * fp->ntiles + 1) * 8, &s));
  fp->counts = (int64_t*)s;
  fp->offsets = fp->counts + fp->ntiles;
  if (n == 0) {
    QE_HIP(hipMemsetAsync(fp->offsets, 0, 8, ctx->stream));
    if (d_total) QE_HIP(hipMemsetAsync(d_total, 0, 8, ctx->stream));
    return QE_OK;
  }
  hipLaunchKernelGGL(k_tile_count, dim3((unsigned)fp->ntiles), dim3(FT_THREADS), 0, ctx->stream,
                     (const uint8_t*)mask->values, mask->validity, n, fp->counts);
  QE_TRY(launch_check("k_tile_count"));
  hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, ctx->stream, fp->counts, fp->offsets, fp->ntiles, d_total);
  return launch_check("k_scan");
}

static int read_total(qe_ctx* ctx, const FilterPlan& fp, int64_t* total) {
  void* h;
  QE_TRY(ctx_pinned(ctx, 8, &h));
  QE_HIP(hipMemcpyAsync(h, fp.offsets + fp.ntiles, 8, hipMemcpyDeviceToHost, ctx->stream));
  QE_TRY(ctx_sync(ctx));
  *total = *(int64_t*)h;
  return QE_OK;
}

}  // namespace qe

using namespace qe;

extern "C" {

int qe_filter_count(qe_ctx* ctx, const qe_column* mask, int64_t* out_count) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(out_count, QE_ERR_INVALID_ARG, "null out_count");
  FilterPlan fp;
  QE_TRY(filter_prepare(ctx, mask, &fp));
  return read_total(ctx, fp, out_count);
}

int qe_filter_apply(qe_ctx* ctx, const qe_column* mask, const qe_column* inputs, int32_t ncols, qe_column* outs,
                    int64_t* out_count) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(ncols >= 0 && ncols <= FT_MAX_COLS, QE_ERR_UNSUPPORTED, "at most %d columns per call", FT_MAX_COLS);
  QE_CHECK(ncols == 0 || (inputs && outs), QE_ERR_INVALID_ARG, "null column arrays");
  QE_CHECK(mask != nullptr, QE_ERR_INVALID_ARG, "null mask");
  const int64_t n = mask->length;
  GatherArgs args{};
  args.ncols = ncols;
  for (int i = 0; i < ncols; ++i) {
    const qe_column& in = inputs[i];
    qe_column& out = outs[i];
    QE_CHECK(in.length == n, QE_ERR_INVALID_ARG, "column %d has %lld rows, mask %lld", i, (long long)in.length,
             (long long)n);
    const bool utf8 = in.type == QE_TYPE_UTF8;
    QE_CHECK(is_fixed(in.type) || utf8, QE_ERR_UNSUPPORTED, "filter: column %d type %d not supported", i, in.type);
    QE_CHECK(out.type == in.type && (out.values || out.length == 0), QE_ERR_INVALID_ARG,
             "output %d must have the input's type", i);
    QE_CHECK(!in.validity || out.validity, QE_ERR_INVALID_ARG, "output %d needs a validity buffer", i);
    QE_CHECK(!utf8 || (in.offsets && out.offsets), QE_ERR_INVALID_ARG, "UTF8 column %d needs offsets", i);
    args.cols[i] = GatherCol{in.values, in.validity, out.values, in.validity ? (uint32_t*)out.validity : nullptr,
                             utf8 ? 0 : type_width(in.type), 0, utf8 ? in.offsets : nullptr};
  }
  FilterPlan fp;
  QE_TRY(filter_prepare(ctx, mask, &fp));
  int64_t total;
  QE_TRY(read_total(ctx, fp, &total));
  for (int i = 0; i < ncols; ++i) {
    QE_CHECK(outs[i].length >= total, QE_ERR_CAPACITY, "output %d holds %lld rows, need %lld", i,
             (long long)outs[i].length, (long long)total);
    if (args.cols[i].out_valid) {
      // atomicOr works on 32-bit words: the buffer must be 4-byte aligned and padded.
      QE_CHECK(((uintptr_t)outs[i].validity & 3) == 0, QE_ERR_INVALID_ARG, "validity buffer must be 4-byte aligned");
      QE_HIP(hipMemsetAsync(outs[i].validity, 0, (size_t)div_up((uint64_t)total, 32) * 4, ctx->stream));
    }
  }
  // UTF-8 columns: k_compact writes (src offset, length) pairs into scratch, then a scan + copy
  int nutf8 = 0;
  for (int i = 0; i < ncols; ++i) nutf8 += args.cols[i].width == 0;
  int2* pairs = nullptr;
  int64_t* tsum = nullptr;
  const int64_t stiles = (int64_t)div_up((uint64_t)(total > 0 ? total : 1), SC_TILE);
  if (nutf8 && total > 0) {
    // after the filter plan's tile arrays (2*ntiles+1 int64), keep them alive
    const size_t base = (size_t)(2 * fp.ntiles + 1) * 8;
    const size_t need = base + (size_t)nutf8 * total * sizeof(int2) + (size_t)(2 * stiles + 1) * 8 + 256;
    void* sb;
    QE_TRY(ctx_scratch(ctx, need, &sb));
    // the scratch may have moved: the tile offsets must be recomputed
    QE_TRY(filter_prepare(ctx, mask, &fp));
    pairs = (int2*)((char*)sb + ((base + 15) & ~size_t(15)));
    tsum = (int64_t*)(pairs + (size_t)nutf8 * total);
    int u = 0;
    for (int i = 0; i < ncols; ++i) {
      if (args.cols[i].width != 0) continue;
      args.cols[i].pad = u;
      args.cols[i].out = pairs + (size_t)u * total;
      ++u;
    }
  }
  if (total > 0 && ncols > 0) {
    hipLaunchKernelGGL(k_compact, dim3((unsigned)fp.ntiles), dim3(FT_THREADS), 0, ctx->stream,
                       (const uint8_t*)mask->values, mask->validity, n, fp.offsets, args);
    QE_TRY(launch_check("k_compact"));
  }
  for (int i = 0; i < ncols && total > 0; ++i) {
    if (args.cols[i].width != 0) continue;
    const int2* sl = (const int2*)args.cols[i].out;
    hipLaunchKernelGGL(k_len_tile_sum, dim3((unsigned)stiles), dim3(256), 0, ctx->stream, sl, total, tsum);
    QE_TRY(launch_check("k_len_tile_sum"));
    QE_TRY(exclusive_scan_i64(ctx, tsum, tsum + stiles, stiles));
    hipLaunchKernelGGL(k_len_tile_scan, dim3((unsigned)stiles), dim3(256), 0, ctx->stream, sl, total,
                       tsum + stiles, outs[i].offsets);
    QE_TRY(launch_check("k_len_tile_scan"));
    hipLaunchKernelGGL(k_write_total, dim3(1), dim3(1), 0, ctx->stream, tsum + 2 * stiles, outs[i].offsets, total);
    QE_TRY(launch_check("k_write_total"));
    const int64_t grid = std::min<int64_t>((int64_t)div_up((uint64_t)total, 256), (int64_t)ctx->num_cus * 8);
    hipLaunchKernelGGL(k_copy_bytes, dim3((unsigned)grid), dim3(256), 0, ctx->stream, sl, outs[i].offsets,
                       (const uint8_t*)inputs[i].values, (uint8_t*)outs[i].values, total);
    QE_TRY(launch_check("k_copy_bytes"));
  }
  for (int i = 0; i < ncols; ++i)
    if (args.cols[i].width == 0 && total == 0) QE_HIP(hipMemsetAsync(outs[i].offsets, 0, 4, ctx->stream));
  for (int i = 0; i < ncols; ++i) outs[i].length = total;
  if (out_count) *out_count = total;
  return QE_OK;
}

}  // extern "C"

extern "C" int qe_filter_apply_async(qe_ctx* ctx, const qe_column* mask, const qe_column* inputs, int32_t ncols,
                                     qe_column* outs, int64_t* d_count) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(ncols >= 0 && ncols <= FT_MAX_COLS, QE_ERR_UNSUPPORTED, "at most %d columns per call", FT_MAX_COLS);
  QE_CHECK(ncols == 0 || (inputs && outs), QE_ERR_INVALID_ARG, "null column arrays");
  QE_CHECK(mask != nullptr && d_count != nullptr, QE_ERR_INVALID_ARG, "null mask or count");
  const int64_t n = mask->length;
  GatherArgs args{};
  args.ncols = ncols;
  for (int i = 0; i < ncols; ++i) {
    const qe_column& in = inputs[i];
    const qe_column& out = outs[i];
    QE_CHECK(in.length == n, QE_ERR_INVALID_ARG, "column %d has %lld rows, mask %lld", i, (long long)in.length,
             (long long)n);
    QE_CHECK(is_fixed(in.type), QE_ERR_UNSUPPORTED,
             "stream-ordered filter: column %d type %d is not fixed-width (qe_filter_apply sizes UTF8 outputs)", i,
             in.type);
    QE_CHECK(out.type == in.type && (out.values || n == 0), QE_ERR_INVALID_ARG, "output %d must have the input's type", i);
    QE_CHECK(out.length >= n, QE_ERR_CAPACITY, "output %d holds %lld rows, need the mask's %lld (an upper bound)", i,
             (long long)out.length, (long long)n);
    QE_CHECK(!in.validity || (out.validity && ((uintptr_t)out.validity & 3) == 0), QE_ERR_INVALID_ARG,
             "output %d needs a 4-byte aligned validity buffer", i);
    args.cols[i] = GatherCol{in.values, in.validity, out.values, in.validity ? (uint32_t*)out.validity : nullptr,
                             type_width(in.type), 0, nullptr};
  }
  FilterPlan fp;
  QE_TRY(filter_prepare(ctx, mask, &fp, d_count));  // (the scan also leaves the count in *d_count)
  for (int i = 0; i < ncols; ++i)
    if (args.cols[i].out_valid && n > 0)
      QE_HIP(hipMemsetAsync(outs[i].validity, 0, (size_t)div_up((uint64_t)n, 32) * 4, ctx->stream));
  if (n > 0 && ncols > 0) {
    hipLaunchKernelGGL(k_compact, dim3((unsigned)fp.ntiles), dim3(FT_THREADS), 0, ctx->stream,
                       (const uint8_t*)mask->values, mask->validity, n, fp.offsets, args);
    QE_TRY(launch_check("k_compact"));
  }
  for (int i = 0; i < ncols; ++i) outs[i].length = n;
  return QE_OK;
}
