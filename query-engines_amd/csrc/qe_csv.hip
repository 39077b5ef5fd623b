// GPU CSV scan: CsvDataSource / ReaderIterator (Main.kt:204-357) turn a CSV file
// into Utf8 RecordBatches; this file does the tokenising on the device, from the file's bytes in
// HBM to device Utf8 columns.
//
// Grammar (restated identically in oracle/csv_ref.py; the reference delegates to univocity
// CsvParser with delimiter / line-separator detection and skipEmptyLines, K:290-297, whose version
// is unpinned):
//   * '"' toggles the quoted state wherever it occurs; outside quotes, '\n', "\r\n" and a lone '\r'
//     end a record and the delimiter byte ends a field;
//   * records whose bytes are all <= 0x20 (empty / blank lines) or whose first byte is '#'
//     (univocity's default comment character) are skipped; the first kept record is the header
//     when the file has one;
//   * a field value is its bytes with chars <= 0x20 trimmed from both ends; if that starts and ends
//     with '"' (length >= 2) the quotes are removed, "" becomes ", and the result is trimmed again
//     (K:263 calls String.trim() on every value); a missing trailing field reads as "" (K:263).
// Pipeline (all HBM-streaming, one wave per 16 KiB segment for the byte passes):
//   k_csv_count2   per segment: quotes, and terminators under both starting quote states
//   k_csv_seg_reduce / _apply: quote state at each segment start, terminator prefixes, line count
//   k_csv_terms<true> terminator positions (the line-end list)
//   k_csv_lines    per line (64 per wave, staged in LDS): projected field lengths, short values
//                  into a 16-byte stage (kept-line path k_csv_keep / k_csv_fields when a line is
//                  blank or a comment)
//   k_csv_len_*    reduce / scan / apply: every column's value byte starts and size in 3 launches
//   k_csv_copy_wave per projected column: Utf8 offsets + bytes
#include <vector>

#include "qe_internal.hpp"

struct qe_csv_table {
  qe_ctx* ctx = nullptr;
  const uint8_t* data = nullptr;  // the file bytes (the caller keeps them until the columns are built)
  int64_t rows = 0;
  int64_t consumed = 0;           // bytes up to and including the last record (all of them unless QE_CSV_PARTIAL_TAIL)
  int64_t stride = 0;             // entries per array of the block (>= rows + 1)
  int32_t nproj = 0;
  void* block = nullptr;          // per projected column: start i64, meta u32, byte start u32 [stride]
  uint8_t* stage_block = nullptr; // per projected column: 16 bytes per row (short unquoted values)
  std::vector<int64_t> total;     // per projected column: bytes
  std::vector<int64_t> maxlen;    // per projected column: longest value, bytes
  std::vector<qe_column> cols;    // materialised views (qe_csv_column), built on first request
  std::vector<void*> owned;
  // start: file position of the value, written only where the column build reads it (quoted, or
  // longer than its 16-byte stage); meta: output length | quoted << 31; bstart: the value's byte
  // start in the column (the Utf8 offsets, < 2^31), entry rows = the column's size
  int64_t* start(int c) { return (int64_t*)block + (size_t)c * stride; }
  uint32_t* meta(int c) { return (uint32_t*)((int64_t*)block + (size_t)nproj * stride) + (size_t)c * stride; }
  uint32_t* bstart(int c) { return meta(0) + (size_t)(nproj + c) * stride; }
  uint8_t* stage(int c) { return stage_block + (size_t)c * stride * 16; }
};

namespace qe {
namespace {

constexpr int SEG = 16 * 1024;  // bytes per wave-task: 16 steps x 64 lanes x 16 B
constexpr int CSV_MAX_FIELDS = 32;
constexpr int CSV_MAX_FIELD_INDEX = 1024;

struct Lane16 {
  uint32_t w[4];
  __device__ __forceinline__ uint32_t byte(int k) const { return (w[k >> 2] >> (8 * (k & 3))) & 0xFFu; }
};

__device__ __forceinline__ Lane16 load16(const uint8_t* data, int64_t nbytes, int64_t pos) {
  Lane16 v;
  if (pos + 16 <= nbytes) {
    const uint4 t = *(const uint4*)(data + pos);
    v.w[0] = t.x;
    v.w[1] = t.y;
    v.w[2] = t.z;
    v.w[3] = t.w;
  } else {
    v.w[0] = v.w[1] = v.w[2] = v.w[3] = 0;
    for (int k = 0; k < 16 && pos + k < nbytes; ++k) v.w[k >> 2] |= (uint32_t)data[pos + k] << (8 * (k & 3));
  }
  return v;
}

// Number of '"' bytes in the 16 bytes (bytes past the end read as 0).
__device__ __forceinline__ int quotes16(const Lane16& v) {
  int q = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t x = v.w[i] ^ 0x22222222u;  // zero byte where the byte is '"'
    // exact per-byte zero test (the (x - 0x01..) & ~x form has borrow false positives)
    q += __popc(~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu));
  }
  return q;
}

// Whether any of the 16 bytes may equal `b`: the classic has-zero-byte test (no false negatives;
// a false positive only sends the lane down the exact path). ~5 VALU ops per word.
__device__ __forceinline__ bool has_byte(const Lane16& v, uint32_t b) {
  const uint32_t rep = b * 0x01010101u;
  uint32_t any = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t x = v.w[i] ^ rep;
    any |= (x - 0x01010101u) & ~x & 0x80808080u;
  }
  return any != 0;
}

// Terminator mask (bit k = byte k ends a record) of a lane's 16 bytes, given the quote state at
// its first byte; returns the state after the 16 bytes.
// 16-bit mask of the bytes equal to `b` (exact SWAR byte compare, 4 bytes per word).
__device__ __forceinline__ uint32_t eq16(const Lane16& v, uint32_t b) {
  const uint32_t rep = b * 0x01010101u;
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t x = v.w[i] ^ rep;
    const uint32_t hb = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);  // bit 7 of each matching byte
    m |= (((hb >> 7) & 1u) | ((hb >> 14) & 2u) | ((hb >> 21) & 4u) | ((hb >> 28) & 8u)) << (4 * i);
  }
  return m;
}

// The '\n' bytes of 16 as bit 7 of each matching byte, per 32-bit word (no packing to a 16-bit mask:
// counts and positions come straight from these words, and the byte passes are VALU-bound).
__device__ __forceinline__ void nl_words(const Lane16& v, uint32_t (&h)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t x = v.w[i] ^ 0x0A0A0A0Au;
    h[i] = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
  }
}

// `next` = the byte after these 16 (the next lane's first byte, passed by shuffle; 0 past the end).
// `maybe_q` false: the caller knows the 16 bytes hold no '"'.
__device__ __forceinline__ uint32_t terms16(const Lane16& v, uint32_t next, int64_t nbytes, int64_t pos,
                                            uint32_t inq, uint32_t* inq_out, bool maybe_q = true) {
  if (!maybe_q || !has_byte(v, '"') || eq16(v, '"') == 0) {  // no quote: the state is constant (common case)
    *inq_out = inq;
    if (inq) return 0;
    // VALU-bound kernels (every wave instruction is 4 cycles on a SIMD): the '\n' mask directly, a
    // '\r' mask only where the cheap test sees one (a wave step nearly always holds a '\n' somewhere,
    // so testing for it first only added work)
    const uint32_t valid = pos + 16 <= nbytes ? 0xFFFFu : ((1u << (nbytes - pos)) - 1u);
    const uint32_t nl = eq16(v, '\n') & valid, cr = has_byte(v, '\r') ? (eq16(v, '\r') & valid) : 0u;
    const uint32_t next_nl = (nl >> 1) | ((pos + 16 < nbytes && next == '\n') ? 0x8000u : 0u);
    return nl | (cr & ~next_nl);
  }
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t c = v.byte(k);
    if (pos + k >= nbytes) break;
    if (c == '"') {
      inq ^= 1u;
    } else if (!inq) {
      if (c == '\n') {
        m |= 1u << k;
      } else if (c == '\r') {
        const uint32_t nx = k < 15 ? v.byte(k + 1) : (pos + 16 < nbytes ? next : 0u);
        const bool last = pos + k + 1 >= nbytes;
        if (last || nx != '\n') m |= 1u << k;
      }
    }
  }
  *inq_out = inq;
  return m;
}

// Terminator positions of every segment (the line-end list), given the quote state at each
// segment's start and its first line's index. HASQ / HASCR: the file holds a '"' / a '\r' at all
// (k_csv_count2 reports both); without them a step is only the '\n' compare (the byte passes are
// VALU-bound: tripdata, no quotes and no '\r', 160 -> ~110 VALU instructions per wave step).
template <bool HASQ, bool HASCR>
__global__ void __launch_bounds__(256) k_csv_terms(const uint8_t* __restrict__ data, int64_t nbytes, int64_t nseg,
                                                   const int64_t* __restrict__ seg_qstart,
                                                   const int64_t* __restrict__ seg_tstart, int64_t* __restrict__ ends) {
  const int lane = threadIdx.x & 63;
  const int64_t seg = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (seg >= nseg) return;
  const int64_t base = seg * SEG;
  const uint64_t below = (1ull << lane) - 1;
  uint32_t carry = HASQ ? (uint32_t)(seg_qstart[seg] & 1) : 0u;
  int64_t out = seg_tstart[seg];
  Lane16 vq[4];
  for (int step = 0; step < SEG / 1024; ++step) {
    const int64_t row0 = base + step * 1024;
    if (row0 >= nbytes) break;
    const int64_t pos = row0 + lane * 16;
    if ((step & 3) == 0) {  // 4 loads in flight per lane: this step and the next three
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t pu = pos + u * 1024;
        vq[u] = pu < nbytes ? load16(data, nbytes, pu) : Lane16{{0, 0, 0, 0}};
      }
    }
    Lane16 v;
    switch (step & 3) {  // constant indices keep vq in registers
      case 0: v = vq[0]; break;
      case 1: v = vq[1]; break;
      case 2: v = vq[2]; break;
      default: v = vq[3]; break;
    }
    bool mq = false;
    uint32_t inq0 = 0;
    uint64_t par = 0;
    if (HASQ) {
      mq = has_byte(v, '"');
      const uint32_t qodd = mq ? (uint32_t)(quotes16(v) & 1) : 0u;
      par = __ballot(qodd);
      inq0 = carry ^ ((uint32_t)__popcll(par & below) & 1u);
    }
    // byte after this lane's 16, for a '\r' there: the next lane's first byte (the shuffle runs on
    // the whole wave, before any lane branches off); lane 63 reads it (rare)
    uint32_t next = 0;
    if (HASCR) {
      next = (uint32_t)__shfl_down((int)(v.w[0] & 0xFFu), 1);
      if (lane == 63) next = (v.byte(15) == '\r' && pos + 16 < nbytes) ? data[pos + 16] : 0u;
    }
    // no quote, no '\r', a full chunk: the '\n' words directly (outside quotes) or nothing
    const bool plain = !mq && pos + 16 <= nbytes && (!HASCR || !has_byte(v, '\r'));
    uint32_t h[4] = {0, 0, 0, 0};
    uint32_t m = 0;
    if (plain) {
      if (!inq0) nl_words(v, h);
    } else {
      uint32_t inq1;  // (the state after the 16 bytes is unused here: the carry follows the ballot)
      m = terms16(v, next, nbytes, pos, inq0, &inq1, mq);
    }
    if (HASQ) carry ^= (uint32_t)__popcll(par) & 1u;
    const int c = plain ? __popc(h[0]) + __popc(h[1]) + __popc(h[2]) + __popc(h[3]) : __popc(m);  // 0..16
    // wave exclusive prefix and total of c from its 5 bit-planes (ballot + popcount, no LDS)
    int excl = 0, total = 0;
#pragma unroll
    for (int b = 0; b < 5; ++b) {
      const uint64_t plane = __ballot((c >> b) & 1);
      excl += __popcll(plane & below) << b;
      total += __popcll(plane) << b;
    }
    int64_t o = out + excl;
    if (plain) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {  // two 64-bit halves: fewer divergent loops than four words
        uint64_t hh = h[2 * i] | ((uint64_t)h[2 * i + 1] << 32);
        while (hh) {
          ends[o++] = pos + 8 * i + (__builtin_ctzll(hh) >> 3);
          hh &= hh - 1;
        }
      }
    } else {
      uint32_t mm = m;
      while (mm) {
        const int k = __builtin_ctz(mm);
        mm &= mm - 1;
        ends[o++] = pos + k;
      }
    }
    out += total;
  }
}

// One read of the file for the counting pass: per segment its quote count and its terminator
// count under both possible quote states at the segment's first byte (the state is the parity of
// all earlier quotes, known only after a scan of the quote counts). A lane without a quote gets
// both hypotheses from one mask: inside quotes nothing terminates. Replaces a quote pass plus a
// terminator pass that needed the scanned quote counts (two reads of the file).
__global__ void __launch_bounds__(256) k_csv_count2(const uint8_t* __restrict__ data, int64_t nbytes, int64_t nseg,
                                                    int64_t* __restrict__ seg_q, int64_t* __restrict__ seg_t0,
                                                    int64_t* __restrict__ seg_t1, uint8_t* __restrict__ seg_cr) {
  const int lane = threadIdx.x & 63;
  const int64_t seg = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (seg >= nseg) return;
  const int64_t base = seg * SEG;
  const uint64_t below = (1ull << lane) - 1;
  uint32_t rel = 0;  // parity of this segment's quotes before the current step
  int q = 0, c0 = 0, c1 = 0;
  bool anycr = false;  // a '\r' in the segment (the position pass then needs its '\r' handling)
  int64_t l0 = -1, l1 = -1;  // last terminator position under each hypothesis
  Lane16 vq[4];
  for (int step = 0; step < SEG / 1024; ++step) {
    const int64_t row0 = base + step * 1024;
    if (row0 >= nbytes) break;
    const int64_t pos = row0 + lane * 16;
    if ((step & 3) == 0) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t pu = pos + u * 1024;
        vq[u] = pu < nbytes ? load16(data, nbytes, pu) : Lane16{{0, 0, 0, 0}};
      }
    }
    Lane16 v;
    switch (step & 3) {
      case 0: v = vq[0]; break;
      case 1: v = vq[1]; break;
      case 2: v = vq[2]; break;
      default: v = vq[3]; break;
    }
    // (wave-uniform tests first: a step without any '"' or '\r' skips the parity ballot and the
    // next-byte shuffle — the pass is VALU-bound)
    const bool hasq = has_byte(v, '"');
    int nq = 0;
    uint32_t x = rel;  // state at this lane's first byte if the segment starts outside quotes
    uint64_t par = 0;
    if (__ballot(hasq)) {
      nq = hasq ? quotes16(v) : 0;
      q += nq;
      par = __ballot(nq & 1);
      x = rel ^ ((uint32_t)__popcll(par & below) & 1u);
    }
    const bool cr = has_byte(v, '\r');
    anycr |= cr;
    uint32_t next = 0;
    if (__ballot(cr)) {
      next = (uint32_t)__shfl_down((int)(v.w[0] & 0xFFu), 1);
      if (lane == 63) next = (v.byte(15) == '\r' && pos + 16 < nbytes) ? data[pos + 16] : 0u;
    }
    uint32_t dummy;
    if (nq == 0 && pos + 16 <= nbytes && !cr) {  // '\n' terminators only: straight from the words
      uint32_t h[4];
      nl_words(v, h);
      const int c = __popc(h[0]) + __popc(h[1]) + __popc(h[2]) + __popc(h[3]);
      if (c) {
        const int i = h[3] ? 3 : h[2] ? 2 : h[1] ? 1 : 0;
        const int64_t last = pos + 4 * i + ((31 - __builtin_clz(h[i])) >> 3);
        if (x) {
          c1 += c;
          l1 = last;
        } else {
          c0 += c;
          l0 = last;
        }
      }
    } else if (nq == 0) {
      const uint32_t mm = terms16(v, next, nbytes, pos, 0u, &dummy, false);
      if (mm) {
        const int64_t last = pos + 31 - __builtin_clz(mm);
        if (x) {
          c1 += __popc(mm);
          l1 = last;
        } else {
          c0 += __popc(mm);
          l0 = last;
        }
      }
    } else {
      const uint32_t m0 = terms16(v, next, nbytes, pos, x, &dummy);
      const uint32_t m1 = terms16(v, next, nbytes, pos, x ^ 1u, &dummy);
      c0 += __popc(m0);
      c1 += __popc(m1);
      if (m0) l0 = pos + 31 - __builtin_clz(m0);
      if (m1) l1 = pos + 31 - __builtin_clz(m1);
    }
    rel ^= (uint32_t)__popcll(par) & 1u;
  }
  for (int d = 32; d >= 1; d >>= 1) {
    q += __shfl_xor(q, d);
    c0 += __shfl_xor(c0, d);
    c1 += __shfl_xor(c1, d);
    l0 = max(l0, (int64_t)__shfl_xor(l0, d));
    l1 = max(l1, (int64_t)__shfl_xor(l1, d));
  }
  const bool segcr = __ballot(anycr) != 0;
  if (lane == 0) {
    seg_cr[seg] = segcr ? 1 : 0;
    seg_q[seg] = q;
    seg_t0[seg] = c0;
    seg_t1[seg] = c1;
    seg_t0[2 * nseg + seg] = l0;  // seg_l0 / seg_l1 follow the two count arrays
    seg_t1[2 * nseg + seg] = l1;
  }
}

// One read of the file that classifies its bytes four at a time (SWAR on 32-bit words) for the fast
// path of a file without '"' or '\r' (tripdata, K:1335): two bitmaps of one bit per byte, in byte
// order — '\n' and the delimiter — and per 16 KiB segment what k_csv_count2 reports for such a file
// (its '\n' count and last '\n'; no quote, so no quote state) plus one flag: the segment holds a '"'
// or a '\r'. The host then takes the general passes (k_csv_count2 ...) instead.
//   test of a word x against byte c < 0x80: s = ((x & 0x7F7F7F7F) ^ c) + 0x7F7F7F7F leaves bit 7 of
//   a byte clear iff its low seven bits equal c — for an ASCII byte, iff the byte is c (a byte
//   >= 0x80 is marked "no match" on a branch of its own);
//   16-bit mask in byte order: the bytes of (s & 0x80808080) dotted with weights 1, 2, 4, 8
//   (v_dot4_u32_u8) give 128 x the inverted nibble of each word.
// Requires delim < 0x80 (the host checks).
__device__ __forceinline__ uint32_t nib_mask16(const uint32_t (&s)[4]) {  // bit k: byte k matched
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) m += __builtin_amdgcn_udot4(s[i] & 0x80808080u, 0x08040201u, 0u, false) << (4 * i);
  return ~(m >> 7) & 0xFFFFu;
}

__global__ void __launch_bounds__(256) k_csv_classify(const uint8_t* __restrict__ data, int64_t nbytes, int64_t nseg,
                                                      uint32_t delim, uint16_t* __restrict__ nlbm,
                                                      uint16_t* __restrict__ dbm, int64_t* __restrict__ seg_q,
                                                      int64_t* __restrict__ seg_t0, int64_t* __restrict__ seg_t1,
                                                      uint8_t* __restrict__ seg_cr) {
  const int lane = threadIdx.x & 63;
  const int64_t seg = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (seg >= nseg) return;
  const int64_t base = seg * SEG;
  const uint32_t K7 = 0x7F7F7F7Fu, CN = 0x0A0A0A0Au, CQ = 0x22222222u, CR = 0x0D0D0D0Du, CD = delim * 0x01010101u;
  uint32_t qr = 0xFFFFFFFFu;  // AND of the '"' / '\r' tests: a clear bit 7 = one was seen
  int cnt = 0;
  int64_t last = -1;
  auto step_bytes = [&](const Lane16& v, int64_t pos) {
    uint32_t sn[4], sd[4], t[4], hi = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t a = v.w[i] & K7;
      sn[i] = (a ^ CN) + K7;
      sd[i] = (a ^ CD) + K7;
      t[i] = ((a ^ CQ) + K7) & ((a ^ CR) + K7);
      hi |= v.w[i];
    }
    if (hi & 0x80808080u) {  // bytes >= 0x80 (UTF-8) match no class
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t h = v.w[i] & 0x80808080u;
        sn[i] |= h;
        sd[i] |= h;
        t[i] |= h;
      }
    }
    qr &= t[0] & t[1] & t[2] & t[3];
    const uint32_t nl = nib_mask16(sn), dl = nib_mask16(sd);
    cnt += __popc(nl);
    if (nl) last = pos + 31 - __builtin_clz(nl);
    if (pos < nbytes) {
      nlbm[pos >> 4] = (uint16_t)nl;
      dbm[pos >> 4] = (uint16_t)dl;
    }
  };
  if (base + SEG <= nbytes) {
    // a whole segment inside the file: no bounds checks, eight 16-byte loads in flight per lane
    // (the checked form below issued four, each under a branch)
#pragma unroll
    for (int g = 0; g < SEG / 1024 / 8; ++g) {
      Lane16 v8[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 x = __builtin_nontemporal_load((const u32x4*)(data + base + (g * 8 + u) * 1024 + lane * 16));
        v8[u].w[0] = x.x;
        v8[u].w[1] = x.y;
        v8[u].w[2] = x.z;
        v8[u].w[3] = x.w;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) step_bytes(v8[u], base + (g * 8 + u) * 1024 + lane * 16);
    }
  } else {
    Lane16 vq[4];
    for (int step = 0; step < SEG / 1024; ++step) {
      const int64_t row0 = base + step * 1024;
      if (row0 >= nbytes) break;
      const int64_t pos = row0 + lane * 16;
      if ((step & 3) == 0) {  // 4 loads in flight per lane: this step and the next three
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t pu = pos + u * 1024;
          vq[u] = pu < nbytes ? load16(data, nbytes, pu) : Lane16{{0, 0, 0, 0}};
        }
      }
      Lane16 v;
      switch (step & 3) {  // constant indices keep vq in registers
        case 0: v = vq[0]; break;
        case 1: v = vq[1]; break;
        case 2: v = vq[2]; break;
        default: v = vq[3]; break;
      }
      step_bytes(v, pos);
    }
  }
  for (int d = 32; d >= 1; d >>= 1) {
    cnt += __shfl_xor(cnt, d);
    last = max(last, (int64_t)__shfl_xor(last, d));
  }
  const bool special = __ballot((qr & 0x80808080u) != 0x80808080u) != 0;
  if (lane == 0) {
    seg_cr[seg] = special ? 1 : 0;
    seg_q[seg] = special ? 1 : 0;
    seg_t0[seg] = cnt;
    seg_t1[seg] = 0;
    seg_t0[2 * nseg + seg] = last;  // seg_l0 / seg_l1 follow the two count arrays
    seg_t1[2 * nseg + seg] = -1;
  }
}

// The line-end list from the '\n' bitmap (fast path): one wave per 16 KiB segment, 256 bitmap bytes
// per lane read with two 16-byte loads, the wave prefix of the lanes' counts, then each lane's
// positions by count-trailing-zeros.
__global__ void __launch_bounds__(256) k_csv_ends_bm(const uint64_t* __restrict__ nlbm, int64_t nbytes, int64_t nseg,
                                                     const int64_t* __restrict__ seg_ts, int64_t* __restrict__ ends) {
  const int lane = threadIdx.x & 63;
  const int64_t seg = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (seg >= nseg) return;
  const uint64_t below = (1ull << lane) - 1;
  const int64_t b0 = seg * SEG + (int64_t)lane * 256;  // this lane's first byte
  uint64_t w[4] = {0, 0, 0, 0};
  if (b0 < nbytes) {
    const uint4* p = (const uint4*)(nlbm + (b0 >> 6));
    const uint4 x = p[0], y = p[1];
    w[0] = x.x | ((uint64_t)x.y << 32);
    w[1] = x.z | ((uint64_t)x.w << 32);
    w[2] = y.x | ((uint64_t)y.y << 32);
    w[3] = y.z | ((uint64_t)y.w << 32);
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // bits past the file's end (pieces the classify pass never wrote)
      const int64_t lo = b0 + 64 * k;
      if (lo >= nbytes) w[k] = 0;
      else if (nbytes - lo < 64) w[k] &= (1ull << (nbytes - lo)) - 1;
    }
  }
  const int c = __popcll(w[0]) + __popcll(w[1]) + __popcll(w[2]) + __popcll(w[3]);  // 0..256
  int excl = 0;
#pragma unroll
  for (int b = 0; b < 9; ++b) excl += __popcll(__ballot((c >> b) & 1) & below) << b;
  int64_t o = seg_ts[seg] + excl;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint64_t x = w[k];
    while (x) {
      ends[o++] = b0 + 64 * k + __builtin_ctzll(x);
      x &= x - 1;
    }
  }
}

// The segment plan: the quote state at each segment's start (parity of all earlier quotes), the
// terminator count under that state, its prefixes, and the last terminator's position — in two
// launches over blocks of 2048 segments. k_csv_seg_reduce: per block, its quote count and its
// terminator total and last terminator under both possible states at the block's start.
// k_csv_seg_apply: each block resolves its start state and prefixes from the blocks before it (a
// short serial pass over their totals), then writes its segments' quote and terminator prefixes;
// the last block also leaves the terminator count and the last terminator's position in host[0..1]
// (fine-grained pinned memory) for the one read-back that sizes the line list. (One 1024-thread
// block doing it all took 52 us on tripdata's 27K segments: a single CU's memory round trips.)
constexpr int SP_THREADS = 256, SP_TILE = SP_THREADS * 8;
struct SegAgg {
  int64_t q, t[2], last[2];  // [P]: the block starts inside quotes (P = 1) or not
  int64_t flags;             // bit 0: a '"' in the block; bit 1: a '\r'
};

__device__ __forceinline__ void seg_load(const int64_t* __restrict__ seg_q, const int64_t* __restrict__ t0,
                                         const int64_t* __restrict__ t1, int64_t nseg, int64_t g0, int64_t (&q)[8],
                                         int64_t (&a)[8], int64_t (&b)[8], int64_t (&la)[8], int64_t (&lb)[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int64_t e = tile_elem(g0, k);
    const bool in = e < nseg;
    q[k] = in ? seg_q[e] : 0;
    a[k] = in ? t0[e] : 0;
    b[k] = in ? t1[e] : 0;
    la[k] = in ? t0[2 * nseg + e] : -1;  // seg_l0 / seg_l1 follow the two count arrays
    lb[k] = in ? t1[2 * nseg + e] : -1;
  }
}

__global__ void __launch_bounds__(SP_THREADS) k_csv_seg_reduce(const int64_t* __restrict__ seg_q,
                                                               const int64_t* __restrict__ t0,
                                                               const int64_t* __restrict__ t1, int64_t nseg,
                                                               const uint8_t* __restrict__ seg_cr,
                                                               SegAgg* __restrict__ agg) {
  __shared__ int64_t ws[SP_THREADS / 64];
  __shared__ int64_t red[SP_THREADS / 64][5];
  int64_t q[8], a[8], b[8], la[8], lb[8], ex[8];
  const int64_t g0 = (int64_t)blockIdx.x * SP_TILE;
  seg_load(seg_q, t0, t1, nseg, g0, q, a, b, la, lb);
  int cr = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int64_t e = tile_elem(g0, k);
    if (e < nseg) cr |= seg_cr[e];
  }
  const bool anycr = __syncthreads_or(cr) != 0;
  const int64_t qt = tile_excl<int64_t, SP_THREADS / 64>(q, ex, ws);
  int64_t s0 = 0, s1 = 0, m0 = -1, m1 = -1;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const bool odd = ex[k] & 1;  // quotes before this segment within the block
    s0 += odd ? b[k] : a[k];
    s1 += odd ? a[k] : b[k];
    m0 = max(m0, odd ? lb[k] : la[k]);
    m1 = max(m1, odd ? la[k] : lb[k]);
  }
  for (int d = 32; d >= 1; d >>= 1) {
    s0 += __shfl_xor(s0, d);
    s1 += __shfl_xor(s1, d);
    m0 = max(m0, (int64_t)__shfl_xor(m0, d));
    m1 = max(m1, (int64_t)__shfl_xor(m1, d));
  }
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[wid][0] = s0;
    red[wid][1] = s1;
    red[wid][2] = m0;
    red[wid][3] = m1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    SegAgg g{qt, {0, 0}, {-1, -1}, (qt > 0 ? 1 : 0) | (anycr ? 2 : 0)};
    for (int w = 0; w < SP_THREADS / 64; ++w) {
      g.t[0] += red[w][0];
      g.t[1] += red[w][1];
      g.last[0] = max(g.last[0], red[w][2]);
      g.last[1] = max(g.last[1], red[w][3]);
    }
    agg[blockIdx.x] = g;
  }
}

__global__ void __launch_bounds__(SP_THREADS) k_csv_seg_apply(const int64_t* __restrict__ seg_q,
                                                              const int64_t* __restrict__ t0,
                                                              const int64_t* __restrict__ t1, int64_t nseg,
                                                              const SegAgg* __restrict__ agg, int64_t nb,
                                                              int64_t* __restrict__ seg_qs, int64_t* __restrict__ seg_ts,
                                                              int64_t* host) {
  __shared__ int64_t ws[SP_THREADS / 64];
  __shared__ int64_t base[2];
  const int64_t blk = blockIdx.x;
  if (threadIdx.x == 0) {  // this block's start state and prefixes from the blocks before it
    int64_t qp = 0, tp = 0, last = -1, fl = 0;
    for (int64_t j = 0; j < blk; ++j) {
      const SegAgg g = agg[j];
      const int P = (int)(qp & 1);
      tp += g.t[P];
      last = max(last, g.last[P]);
      qp += g.q;
      fl |= g.flags;
    }
    base[0] = qp;
    base[1] = tp;
    if (blk == nb - 1) {  // the file's totals
      const SegAgg g = agg[blk];
      const int P = (int)(qp & 1);
      const int64_t tall = tp + g.t[P];
      seg_qs[nseg] = qp + g.q;
      seg_ts[nseg] = tall;
      __hip_atomic_store(&host[0], tall, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&host[1], max(last, g.last[P]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&host[2], fl | g.flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  __syncthreads();
  const int64_t qp = base[0], tp = base[1];
  const int64_t g0 = blk * SP_TILE;
  int64_t q[8], a[8], b[8], la[8], lb[8], ex[8];
  seg_load(seg_q, t0, t1, nseg, g0, q, a, b, la, lb);
  (void)tile_excl<int64_t, SP_THREADS / 64>(q, ex, ws);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int64_t qs = qp + ex[k];
    const int64_t e = tile_elem(g0, k);
    if (e < nseg) seg_qs[e] = qs;
    q[k] = (qs & 1) ? b[k] : a[k];  // the terminator count under the segment's actual start state
  }
  (void)tile_excl<int64_t, SP_THREADS / 64>(q, ex, ws);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int64_t e = tile_elem(g0, k);
    if (e < nseg) seg_ts[e] = tp + ex[k];
  }
}

__global__ void k_csv_set_i64(int64_t* p, int64_t v) { *p = v; }

// Line i is [start(i), ends[i]) with start(0) = 0, start(i) = ends[i-1] + 1.
__device__ __forceinline__ int64_t line_start(const int64_t* ends, int64_t i) { return i == 0 ? 0 : ends[i - 1] + 1; }

__global__ void k_csv_keep(const uint8_t* __restrict__ data, const int64_t* __restrict__ ends, int64_t nlines,
                           int64_t* __restrict__ keep) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nlines; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = line_start(ends, i), e = ends[i];
    int64_t k = 0;
    if (s < e && data[s] != '#') {
      for (int64_t p = s; p < e; ++p)
        if (data[p] > 0x20) {
          k = 1;
          break;
        }
    }
    keep[i] = k;
  }
}

__global__ void k_csv_compact_lines(const int64_t* __restrict__ keep, const int64_t* __restrict__ kstart,
                                    int64_t nlines, int64_t* __restrict__ kept) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nlines; i += (int64_t)gridDim.x * blockDim.x)
    if (keep[i]) kept[kstart[i]] = i;
}

struct FieldArgs {
  int16_t slot[CSV_MAX_FIELD_INDEX];  // field index -> projected column slot, -1 = not projected
  int64_t* start[CSV_MAX_FIELDS];     // per column: byte position of the (trimmed, unquoted) value
  uint32_t* meta[CSV_MAX_FIELDS];     // per column: output length (after unescaping) | quoted << 31
  uint8_t* stage[CSV_MAX_FIELDS];     // per column: 16 bytes per row, the value when unquoted and <= 16 bytes
  int32_t max_field;                  // largest projected field index
  int32_t delim;
  uint64_t low_mask;                  // bit f: field f < 64 is projected (skips the table lookup)
  int16_t pf[CSV_MAX_FIELDS];         // the projected field indices, ascending
  int32_t npf;
  int32_t noq;                        // 1: the bytes hold no '"' at all (the line walk skips its quote test)
};

// Bytes of the file by global position: straight from HBM, or from a wave's LDS copy of a block.
struct GBytes {
  const uint8_t* d;
  int64_t nbytes;
  __device__ __forceinline__ uint32_t operator[](int64_t i) const { return d[i]; }
  __device__ __forceinline__ uint4 bytes16(int64_t s, int64_t n) const {  // bytes [s, s + n), n <= 16
    const int64_t a = s & ~(int64_t)15;
    if (a + 32 <= nbytes) {  // two aligned 16-byte loads and a funnel shift
      const int sh = (int)(s - a);
      const uint4 x = *(const uint4*)(d + a);
      unsigned __int128 v = ((unsigned __int128)(((uint64_t)x.w << 32) | x.z) << 64) | (((uint64_t)x.y << 32) | x.x);
      if (sh) {
        v >>= 8 * sh;
        if (sh + n > 16) {
          const uint4 y = *(const uint4*)(d + a + 16);
          const unsigned __int128 w = ((unsigned __int128)(((uint64_t)y.w << 32) | y.z) << 64) | (((uint64_t)y.y << 32) | y.x);
          v |= w << (128 - 8 * sh);
        }
      }
      if (n < 16) v &= (((unsigned __int128)1) << (8 * n)) - 1;
      return make_uint4((uint32_t)v, (uint32_t)(v >> 32), (uint32_t)(v >> 64), (uint32_t)(v >> 96));
    }
    uint64_t lo = 0, hi = 0;
    for (int64_t k = 0; k < n; ++k) {
      const uint64_t b = d[s + k];
      if (k < 8) lo |= b << (8 * k);
      else hi |= b << (8 * (k - 8));
    }
    return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
  }
  __device__ __forceinline__ Lane16 load16(int64_t a) const { return qe::load16(d, nbytes, a); }
};
struct LBytes {
  const uint8_t* L;  // LDS copy of [base, base + span), base 16-byte aligned
  int64_t base;
  __device__ __forceinline__ uint32_t operator[](int64_t i) const { return L[i - base]; }
  // bytes [s, s + n), n <= 16, zero-padded: two aligned 16-byte LDS reads and a funnel shift
  __device__ __forceinline__ uint4 bytes16(int64_t s, int64_t n) const {
    const int64_t o = s - base;
    const int sh = (int)(o & 15);
    const uint4 a = *(const uint4*)(L + (o - sh));
    unsigned __int128 v = ((unsigned __int128)(((uint64_t)a.w << 32) | a.z) << 64) | (((uint64_t)a.y << 32) | a.x);
    if (sh) {
      v >>= 8 * sh;
      if (sh + n > 16) {
        const uint4 b = *(const uint4*)(L + (o - sh) + 16);
        const unsigned __int128 w = ((unsigned __int128)(((uint64_t)b.w << 32) | b.z) << 64) | (((uint64_t)b.y << 32) | b.x);
        v |= w << (128 - 8 * sh);
      }
    }
    if (n < 16) v &= (((unsigned __int128)1) << (8 * n)) - 1;
    return make_uint4((uint32_t)v, (uint32_t)(v >> 32), (uint32_t)(v >> 64), (uint32_t)(v >> 96));
  }
  __device__ __forceinline__ Lane16 load16(int64_t a) const {  // a: 16-byte aligned, inside the copy
    const uint4 t = *(const uint4*)(L + (a - base));
    Lane16 v;
    v.w[0] = t.x;
    v.w[1] = t.y;
    v.w[2] = t.z;
    v.w[3] = t.w;
    return v;
  }
};

template <typename D>
__device__ __forceinline__ void trim(const D& d, int64_t& s, int64_t& e) {
  while (s < e && d[s] <= 0x20) ++s;
  while (e > s && d[e - 1] <= 0x20) --e;
}

template <typename D>
__device__ void record_field(const D& d, const FieldArgs& A, int f, int64_t s, int64_t e, int64_t row) {
  if (f > A.max_field) return;
  if (f < 64 && !((A.low_mask >> f) & 1)) return;
  const int sl = A.slot[f];
  if (sl < 0) return;
  trim(d, s, e);
  uint8_t q = 0;
  int64_t len = e - s;
  if (!A.noq && len >= 2 && d[s] == '"' && d[e - 1] == '"') {
    ++s;
    --e;
    // unescaped length: every "" pair counts once; then trim again (String.trim on the value)
    int64_t a = s, b = e;
    // trimming after unescaping: leading/trailing bytes <= 0x20 are never quotes, so trimming the
    // escaped span first gives the same bytes
    trim(d, a, b);
    int64_t n = 0;
    for (int64_t p = a; p < b; ++p) {
      if (d[p] == '"' && p + 1 < b && d[p + 1] == '"') ++p;
      ++n;
    }
    s = a;
    len = n;
    q = 1;
  }
  A.meta[sl][row] = (uint32_t)len | ((uint32_t)q << 31);
  // Short unquoted values are staged densely, 16 bytes per row, while the line sits in LDS; the
  // column build reads them there instead of gathering from every line of the file (and needs no
  // file position for them).
  if (!q && len <= 16) *(uint4*)(A.stage[sl] + row * 16) = d.bytes16(s, len);
  else A.start[sl][row] = s;
}

// One record [s, e): the projected fields' ranges into row `r` (missing fields read as "").
template <typename D>
__device__ void walk_record(const D& data, int64_t s, int64_t e, const FieldArgs& A, int32_t nproj, int64_t r) {
  for (int c = 0; c < nproj; ++c) A.meta[c][r] = 0;
  int f = 0;
  int64_t fs = s;
  uint32_t inq = 0;
  // 16-byte aligned loads; bytes outside [s, e) are skipped
  for (int64_t a = s & ~(int64_t)15; a < e && f <= A.max_field; a += 16) {
    const Lane16 v = data.load16(a);
    const uint32_t lo = (uint32_t)(s > a ? s - a : 0);
    const uint32_t hi = (uint32_t)(e - a < 16 ? e - a : 16);
    const uint32_t in = (hi >= 32 ? 0xFFFFu : ((1u << hi) - 1u)) & ~((1u << lo) - 1u);
    uint32_t q = (has_byte(v, '"') ? eq16(v, '"') : 0u) & in, d = eq16(v, (uint32_t)A.delim) & in;
    if (q == 0 && inq) continue;
    while (d && f <= A.max_field) {
      const int k = __builtin_ctz(d);
      // quote toggles before this delimiter
      const uint32_t before = q & ((1u << k) - 1u);
      inq ^= (uint32_t)__popc(before) & 1u;
      q &= ~((1u << k) - 1u);
      d &= d - 1;
      if (!inq) {
        record_field(data, A, f, fs, a + k, r);
        ++f;
        fs = a + k + 1;
      }
    }
    inq ^= (uint32_t)__popc(q) & 1u;
  }
  if (f <= A.max_field) record_field(data, A, f, fs, e, r);
}

// The delimiter bytes among a lane's 16 as bit 7 of each matching byte, in two 64-bit words (bytes
// 0-7 and 8-15), restricted to bytes [lo, hi): counts and positions come straight from these words
// (packing them to a 16-bit mask cost the line walk ~40 VALU instructions per 16 bytes).
__device__ __forceinline__ uint64_t byte_lowmask(int n) {  // bytes [0, n) of a 64-bit word, n in 0..8
  return n >= 8 ? ~0ull : ((1ull << (8 * n)) - 1ull);
}
__device__ __forceinline__ void delim_words(const Lane16& v, uint32_t delim, int lo, int hi, uint64_t& d0,
                                            uint64_t& d1) {
  const uint32_t rep = delim * 0x01010101u;
  uint32_t hb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t x = v.w[i] ^ rep;
    hb[i] = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
  }
  d0 = hb[0] | ((uint64_t)hb[1] << 32);
  d1 = hb[2] | ((uint64_t)hb[3] << 32);
  if (lo != 0 || hi != 16) {  // the line's first or last chunk
    d0 &= byte_lowmask(min(hi, 8)) & ~byte_lowmask(min(lo, 8));
    d1 &= byte_lowmask(max(hi - 8, 0)) & ~byte_lowmask(max(lo - 8, 0));
  }
}
// Byte index (0..15) of the k-th (0-based) delimiter of (d0, d1), which hold more than k.
__device__ __forceinline__ int nth_delim(uint64_t d0, uint64_t d1, int k) {
  const int c0 = __popcll(d0);
  uint64_t w = k < c0 ? d0 : d1;
  const int b = k < c0 ? 0 : 8;
  for (k = k < c0 ? k : k - c0; k > 0; --k) w &= w - 1;
  return b + (__builtin_ctzll(w) >> 3);
}

// walk_record for a line without a '"' byte (false: the line has one; nothing was written, the
// caller walks it with walk_record). No per-delimiter loop: a 16-byte chunk holding n delimiters
// ends fields f .. f + n - 1 at once, and only the projected fields among them (A.pf, ascending)
// locate their bounds by bit selection — the walk's work follows the projected fields, not the
// line's field count (the line pass is VALU-bound).
template <typename D>
__device__ bool walk_record_unquoted(const D& data, int64_t s, int64_t e, const FieldArgs& A, int32_t nproj, int64_t r) {
  int f = 0, t = 0;
  int64_t fs = s;
  for (int64_t a = s & ~(int64_t)15; a < e && t < A.npf; a += 16) {
    const Lane16 v = data.load16(a);
    const int lo = s > a ? (int)(s - a) : 0;
    const int hi = e - a < 16 ? (int)(e - a) : 16;
    if (!A.noq && has_byte(v, '"') &&
        (eq16(v, '"') & ((hi >= 16 ? 0xFFFFu : ((1u << hi) - 1u)) & ~((1u << lo) - 1u))))
      return false;
    uint64_t d0, d1;
    delim_words(v, (uint32_t)A.delim, lo, hi, d0, d1);
    const int n = __popcll(d0) + __popcll(d1);
    while (t < A.npf && A.pf[t] < f + n) {  // projected field A.pf[t] ends in this chunk
      const int ft = A.pf[t], k = ft - f;
      const int64_t st = k == 0 ? fs : a + nth_delim(d0, d1, k - 1) + 1;
      record_field(data, A, ft, st, a + nth_delim(d0, d1, k), r);
      ++t;
    }
    if (n) {
      fs = a + (d1 ? 8 + ((63 - __builtin_clzll(d1)) >> 3) : ((63 - __builtin_clzll(d0)) >> 3)) + 1;
      f += n;
    }
  }
  if (t < A.npf && A.pf[t] == f) {  // the line's last field
    record_field(data, A, f, fs, e, r);
    ++t;
  }
  for (; t < A.npf; ++t) A.meta[A.slot[A.pf[t]]][r] = 0;  // fields the line does not reach read as "" (K:263)
  return true;
}

// The field table in LDS: indexing kernel arguments by a per-lane field number would turn every
// field into a memory round trip.
__device__ __forceinline__ void stage_args(FieldArgs& S, const FieldArgs& A) {
  const int16_t* src = A.slot;
  for (int i = threadIdx.x; i <= A.max_field; i += blockDim.x) S.slot[i] = src[i];
  if (threadIdx.x < CSV_MAX_FIELDS) {
    S.start[threadIdx.x] = A.start[threadIdx.x];
    S.meta[threadIdx.x] = A.meta[threadIdx.x];
    S.stage[threadIdx.x] = A.stage[threadIdx.x];
  }
  if (threadIdx.x < CSV_MAX_FIELDS) S.pf[threadIdx.x] = A.pf[threadIdx.x];
  if (threadIdx.x == 0) {
    S.max_field = A.max_field;
    S.delim = A.delim;
    S.low_mask = A.low_mask;
    S.npf = A.npf;
    S.noq = A.noq;
  }
  __syncthreads();
}

__global__ void k_csv_fields(const uint8_t* __restrict__ data, int64_t nbytes, const int64_t* __restrict__ ends,
                             const int64_t* __restrict__ kept, int64_t first_row_line, int64_t nrows, FieldArgs Ag,
                             int32_t nproj) {
  __shared__ FieldArgs A;
  stage_args(A, Ag);
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t li = kept[first_row_line + r];
    walk_record(GBytes{data, nbytes}, line_start(ends, li), ends[li], A, nproj, r);
  }
}

// All lines at once, for files whose every line is a record (the common case; otherwise the
// host reruns the kept-line path above): one wave per 64 consecutive lines copies their bytes
// into LDS with coalesced 16-byte loads and each lane walks its line there (a lane per line
// reading HBM directly touches 64 different rows per load instruction). Lines whose block does
// not fit LB_BYTES walk HBM. Row r = line r + first (the header is line 0). `nskip` counts the
// lines that are not records (blank, or '#' first).
constexpr int LB_BYTES = 8192;
__global__ void __launch_bounds__(256) k_csv_lines(const uint8_t* __restrict__ data, int64_t nbytes,
                                                   const int64_t* __restrict__ ends, int64_t nlines, int64_t first,
                                                   FieldArgs Ag, int32_t nproj,
                                                   unsigned long long* __restrict__ nskip) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4][LB_BYTES];
  __shared__ FieldArgs A;
  stage_args(A, Ag);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint8_t* L = lds[wid];
  const int64_t wstride = (int64_t)gridDim.x * 4 * 64;
  for (int64_t l0 = ((int64_t)blockIdx.x * 4 + wid) * 64; l0 < nlines; l0 += wstride) {
    const int64_t li = l0 + lane;
    const bool live = li < nlines;
    const int64_t s = live ? line_start(ends, li) : 0, e = live ? ends[li] : 0;
    const int last = (int)(min(l0 + 63, nlines - 1) - l0);
    const int64_t base = __shfl(s, 0) & ~(int64_t)15;
    const int64_t span = __shfl(e, last) - base;
    const bool staged = span <= LB_BYTES;
    if (staged) {  // all of the block's loads in flight at once, then into LDS
      Lane16 v[LB_BYTES / 1024];
#pragma unroll
      for (int k = 0; k < LB_BYTES / 1024; ++k) {
        const int64_t off = (int64_t)k * 1024 + lane * 16;
        if (off < span) v[k] = load16(data, nbytes, base + off);
      }
#pragma unroll
      for (int k = 0; k < LB_BYTES / 1024; ++k) {
        const int64_t off = (int64_t)k * 1024 + lane * 16;
        if (off < span) *(uint4*)(L + off) = make_uint4(v[k].w[0], v[k].w[1], v[k].w[2], v[k].w[3]);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (live) {
      bool keep = false;
      if (staged) {
        const LBytes d{L, base};
        if (s < e && d[s] != '#')
          for (int64_t p = s; p < e && !keep; ++p) keep = d[p] > 0x20;
        if (keep && li >= first && !walk_record_unquoted(d, s, e, A, nproj, li - first))
          walk_record(d, s, e, A, nproj, li - first);
      } else {
        const GBytes d{data, nbytes};
        if (s < e && d[s] != '#')
          for (int64_t p = s; p < e && !keep; ++p) keep = d[p] > 0x20;
        if (keep && li >= first && !walk_record_unquoted(d, s, e, A, nproj, li - first))
          walk_record(d, s, e, A, nproj, li - first);
      }
      if (!keep) atomicAdd(nskip, 1ull);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the block's LDS is rewritten next
    __builtin_amdgcn_wave_barrier();
  }
}

// Bit index of the k-th (0-based) set bit of w, which has more than k.
__device__ __forceinline__ int select64(uint64_t w, int k) {
  int pos = 0;
  const int c = __popcll(w & 0xFFFFFFFFull);
  if (k >= c) {
    k -= c;
    w >>= 32;
    pos = 32;
  }
  uint32_t x = (uint32_t)w;
  int h = __popc(x & 0xFFFFu);
  if (k >= h) {
    k -= h;
    x >>= 16;
    pos += 16;
  }
  h = __popc(x & 0xFFu);
  if (k >= h) {
    k -= h;
    x >>= 8;
    pos += 8;
  }
  for (; k > 0; --k) x &= x - 1;
  return pos + __ffs(x) - 1;
}

// walk_record_unquoted on the delimiter bitmap (one bit per byte, k_csv_classify) instead of the
// line's bytes: a 64-byte stretch of the line is one 8-byte load (the wave's lines are consecutive,
// so its lanes share a few cached bitmap lines), a popcount and, for the projected fields ending
// there, a bit select. Bytes are touched only for the projected values (trim, 16-byte stage).
template <typename D>
__device__ __forceinline__ void walk_record_bm(const D& d, const uint64_t* __restrict__ dbm, int64_t s, int64_t e,
                                               const FieldArgs& A, int64_t r) {
  int f = 0, t = 0;
  int64_t fs = s;
  for (int64_t wb = s & ~(int64_t)63; wb < e && t < A.npf; wb += 64) {
    uint64_t w = dbm[wb >> 6];
    if (wb < s) w &= ~0ull << (s - wb);
    if (e - wb < 64) w &= (1ull << (e - wb)) - 1;
    const int n = __popcll(w);
    while (t < A.npf && A.pf[t] < f + n) {  // projected field A.pf[t] ends in this stretch
      const int ft = A.pf[t], k = ft - f;
      const int64_t st = k == 0 ? fs : wb + select64(w, k - 1) + 1;
      record_field(d, A, ft, st, wb + select64(w, k), r);
      ++t;
    }
    if (n) {
      fs = wb + (63 - __builtin_clzll(w)) + 1;
      f += n;
    }
  }
  if (t < A.npf && A.pf[t] == f) {  // the line's last field
    record_field(d, A, f, fs, e, r);
    ++t;
  }
  for (; t < A.npf; ++t) A.meta[A.slot[A.pf[t]]][r] = 0;  // fields the line does not reach read as "" (K:263)
}

// The fast path's line walk (a file without '"' or '\r'): k_csv_lines' shape — one wave per 64
// consecutive lines, their bytes staged in LDS with coalesced 16-byte loads — with the fields
// located on the delimiter bitmap (walk_record_bm) instead of classifying the bytes again. (A lane
// per line reading the bytes from HBM directly took 243 us on tripdata against 169 us staged.)
__global__ void __launch_bounds__(256) k_csv_lines_bm(const uint8_t* __restrict__ data, int64_t nbytes,
                                                      const uint64_t* __restrict__ dbm, const int64_t* __restrict__ ends,
                                                      int64_t nlines, int64_t first, FieldArgs Ag, int32_t nproj,
                                                      unsigned long long* __restrict__ nskip) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4][LB_BYTES];
  __shared__ FieldArgs A;
  stage_args(A, Ag);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint8_t* L = lds[wid];
  const int64_t wstride = (int64_t)gridDim.x * 4 * 64;
  for (int64_t l0 = ((int64_t)blockIdx.x * 4 + wid) * 64; l0 < nlines; l0 += wstride) {
    const int64_t li = l0 + lane;
    const bool live = li < nlines;
    const int64_t s = live ? line_start(ends, li) : 0, e = live ? ends[li] : 0;
    const int last = (int)(min(l0 + 63, nlines - 1) - l0);
    const int64_t base = __shfl(s, 0) & ~(int64_t)15;
    const int64_t span = __shfl(e, last) - base;
    const bool staged = span <= LB_BYTES;
    if (staged) {  // all of the block's loads in flight at once, then into LDS
      Lane16 v[LB_BYTES / 1024];
#pragma unroll
      for (int k = 0; k < LB_BYTES / 1024; ++k) {
        const int64_t off = (int64_t)k * 1024 + lane * 16;
        if (off < span) v[k] = load16(data, nbytes, base + off);
      }
#pragma unroll
      for (int k = 0; k < LB_BYTES / 1024; ++k) {
        const int64_t off = (int64_t)k * 1024 + lane * 16;
        if (off < span) *(uint4*)(L + off) = make_uint4(v[k].w[0], v[k].w[1], v[k].w[2], v[k].w[3]);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (live) {
      bool keep = false;
      if (staged) {
        const LBytes d{L, base};
        if (s < e && d[s] != '#')
          for (int64_t p = s; p < e && !keep; ++p) keep = d[p] > 0x20;
        if (keep && li >= first) walk_record_bm(d, dbm, s, e, A, li - first);
      } else {
        const GBytes d{data, nbytes};
        if (s < e && d[s] != '#')
          for (int64_t p = s; p < e && !keep; ++p) keep = d[p] > 0x20;
        if (keep && li >= first) walk_record_bm(d, dbm, s, e, A, li - first);
      }
      if (!keep) atomicAdd(nskip, 1ull);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the block's LDS is rewritten next
    __builtin_amdgcn_wave_barrier();
  }
}

// Byte starts of the projected columns' values (the Utf8 offsets): a scan of the lengths in meta,
// every column per launch (blockIdx.y = column). Per 8192-row tile its sum (int64), the tiles'
// prefixes, then each tile's rows in 32-bit arithmetic — exact whenever the column's size is below
// 2^31, which the host checks on the int64 total (round 5: int64 lengths, the generic int64 scan
// per column, then a kernel narrowing the starts to int32 offsets).
// (The longest value of each tile goes to maxs, same layout as sums.)
__global__ void __launch_bounds__(1024) k_csv_len_reduce(const uint32_t* __restrict__ meta0, int64_t stride, int64_t n,
                                                         int64_t nb, int64_t* __restrict__ sums,
                                                         int64_t* __restrict__ maxs) {
  __shared__ int64_t ws[16], wm[16];
  const uint32_t* __restrict__ m = meta0 + (size_t)blockIdx.y * stride;
  uint32_t v[8];
  tile_load_u32(m, (int64_t)blockIdx.x * 8192, n, v);
  int64_t t = 0, mx = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int64_t l = v[k] & 0x7FFFFFFFu;
    t += l;
    mx = max(mx, l);
  }
  for (int d = 32; d >= 1; d >>= 1) {
    t += __shfl_xor(t, d);
    mx = max(mx, (int64_t)__shfl_xor(mx, d));
  }
  if ((threadIdx.x & 63) == 0) {
    ws[threadIdx.x >> 6] = t;
    wm[threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t all = 0;
    for (int w = 0; w < 16; ++w) {
      all += ws[w];
      mx = max(mx, wm[w]);
    }
    sums[(size_t)blockIdx.y * (nb + 1) + blockIdx.x] = all;
    maxs[(size_t)blockIdx.y * (nb + 1) + blockIdx.x] = mx;
  }
}

// One block per column: the tile sums' exclusive prefixes in place, the column's size at entry n of
// its starts and in host[1 + c], its longest value in host[1 + nproj + c]; host[0] = *nskip
// (lines that are not records), so one sync returns everything the host needs.
__global__ void __launch_bounds__(1024) k_csv_len_scan(int64_t* __restrict__ sums, const int64_t* __restrict__ maxs,
                                                       int64_t nb, uint32_t* __restrict__ bstart0,
                                                       int64_t stride, int64_t n,
                                                       const unsigned long long* __restrict__ nskip, int64_t* host) {
  __shared__ int64_t ws[16];
  int64_t* __restrict__ sm = sums + (size_t)blockIdx.x * (nb + 1);
  const int64_t* __restrict__ mm = maxs + (size_t)blockIdx.x * (nb + 1);
  int64_t carry = 0, mx = 0;
  for (int64_t g0 = 0; g0 < nb; g0 += 8192) {
    int64_t v[8], ex[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t e = tile_elem(g0, k);
      v[k] = e < nb ? sm[e] : 0;
      if (e < nb) mx = max(mx, mm[e]);
    }
    const int64_t t = tile_excl(v, ex, ws);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t e = tile_elem(g0, k);
      if (e < nb) sm[e] = carry + ex[k];
    }
    carry += t;
  }
  for (int d = 32; d >= 1; d >>= 1) mx = max(mx, (int64_t)__shfl_xor(mx, d));
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = mx;  // (tile_excl's last barrier freed ws)
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 0; w < 16; ++w) mx = max(mx, ws[w]);
    __hip_atomic_store(&host[1 + gridDim.x + blockIdx.x], mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    sm[nb] = carry;
    bstart0[(size_t)blockIdx.x * stride + n] = (uint32_t)carry;
    __hip_atomic_store(&host[1 + blockIdx.x], carry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (blockIdx.x == 0)
      __hip_atomic_store(&host[0], nskip ? (int64_t)*nskip : (int64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void __launch_bounds__(1024) k_csv_len_apply(const uint32_t* __restrict__ meta0, int64_t stride, int64_t n,
                                                        int64_t nb, const int64_t* __restrict__ sums,
                                                        uint32_t* __restrict__ bstart0) {
  __shared__ uint32_t ws[16];
  const uint32_t* __restrict__ m = meta0 + (size_t)blockIdx.y * stride;
  uint32_t* __restrict__ b = bstart0 + (size_t)blockIdx.y * stride;
  const int64_t g0 = (int64_t)blockIdx.x * 8192;
  uint32_t v[8], ex[8];
  tile_load_u32(m, g0, n, v);
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] &= 0x7FFFFFFFu;
  (void)tile_excl(v, ex, ws);
  const uint32_t base = (uint32_t)sums[(size_t)blockIdx.y * (nb + 1) + blockIdx.x];
#pragma unroll
  for (int k = 0; k < 8; ++k) ex[k] += base;
  const int64_t e0 = tile_elem(g0, 0);
  if (e0 + 8 <= n) {
    *(uint4*)(b + e0) = make_uint4(ex[0], ex[1], ex[2], ex[3]);
    *(uint4*)(b + e0 + 4) = make_uint4(ex[4], ex[5], ex[6], ex[7]);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (e0 + k < n) b[e0 + k] = ex[k];
  }
}

// Offsets and bytes of one projected column into its Utf8 buffers. A wave takes 64 rows, puts their
// output offsets and byte sources in LDS, and its lanes then walk the wave's contiguous output range
// 4 bytes per lane — byte j's row found by binary search over the 64 offsets. Stores land
// contiguous across lanes, and the source loads are independent (not one dependent loop per row).
// A short unquoted value comes from its 16-byte stage, any other from the file. A wave holding a
// quoted field (escape-aware copy: `""` -> `"`) copies row by row. (One thread per row, byte by
// byte, took 132 / 95 us for tripdata's fare_amount / VendorID columns.)
__global__ void __launch_bounds__(256) k_csv_copy_wave(const uint8_t* __restrict__ data, const int64_t* __restrict__ start,
                                                       const uint32_t* __restrict__ meta, const uint8_t* __restrict__ stage,
                                                       const uint32_t* __restrict__ bstart, int64_t n,
                                                       int32_t* __restrict__ offs, uint8_t* __restrict__ out,
                                                       int lds_path) {
  __shared__ int32_t s_o[4][65];
  __shared__ int64_t s_s[4][64];  // source of the row's first byte: file position, or -1 - row (staged)
  __shared__ __attribute__((aligned(16))) uint8_t s_b[4][1056];  // a staged wave's output bytes
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const bool out16 = lds_path && ((uintptr_t)out & 15) == 0;
  for (int64_t r0 = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 64; r0 < n; r0 += nw * 64) {
    const int64_t r = r0 + lane;
    const bool in = r < n;
    const uint32_t mt = in ? meta[r] : 0u;
    const int64_t l = mt & 0x7FFFFFFFu;
    const bool q = mt >> 31;
    const bool staged = !q && l <= 16;
    const int32_t o = in ? (int32_t)bstart[r] : 0x7FFFFFFF;
    if (in) offs[r] = o;
    if (r == n - 1) offs[n] = (int32_t)bstart[n];
    if (__ballot(q)) {
      if (in) {
        uint8_t* dst = out + o;
        if (staged) {
          for (int64_t k = 0; k < l; ++k) dst[k] = stage[r * 16 + k];
        } else if (!q) {  // an unquoted field keeps any `""` verbatim
          const int64_t s = start[r];
          for (int64_t k = 0; k < l; ++k) dst[k] = data[s + k];
        } else {
          int64_t p = start[r];
          for (int64_t k = 0; k < l; ++k) {
            const uint8_t c = data[p];
            dst[k] = c;
            p += (c == '"' && data[p + 1] == '"') ? 2 : 1;
          }
        }
      }
      continue;
    }
    const int64_t rend = r0 + 64 < n ? r0 + 64 : n;
    if (out16 && !__ballot(in && !staged)) {
      // every value of the wave sits in its 16-byte stage (<= 1 KiB in all): one 16-byte load per
      // row, the bytes assembled in LDS at their output positions, then 16-byte stores of the
      // wave's output range (byte stores only at its two ends)
      const int32_t obeg = __shfl(o, 0), oend = (int32_t)bstart[rend];
      const int32_t a0 = obeg & ~15;
      uint8_t* B = s_b[w];
      if (in && l) {
        const uint4 st = *(const uint4*)(stage + r * 16);
        const uint64_t lo = ((uint64_t)st.y << 32) | st.x, hi = ((uint64_t)st.w << 32) | st.z;
        uint8_t* d = B + (o - a0);
        // 16 predicated byte stores with constant shifts (a loop over l was vectorised by the compiler
        // into dword / 16-byte LDS stores at unaligned addresses, and corrupted bytes)
#pragma unroll
        for (int k = 0; k < 16; ++k)
          if (k < (int)l) d[k] = (uint8_t)(k < 8 ? lo >> (8 * k) : hi >> (8 * (k - 8)));
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      for (int32_t c = a0 + lane * 16; c < oend; c += 1024) {
        if (c >= obeg && c + 16 <= oend) {
          *(uint4*)(out + c) = *(const uint4*)(B + (c - a0));
        } else {
          for (int k = 0; k < 16; ++k)
            if (c + k >= obeg && c + k < oend) out[c + k] = B[c + k - a0];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // s_b is rewritten next
      __builtin_amdgcn_wave_barrier();
      continue;
    }
    s_o[w][lane] = o;
    s_s[w][lane] = staged ? -1 - r : (in ? start[r] : 0);
    if (lane == 0) s_o[w][64] = (int32_t)bstart[rend];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int32_t obeg = s_o[w][0], oend = s_o[w][64];
    for (int32_t j = obeg + lane * 4; j < oend; j += 256) {
      int lo = 0, hi = 63;  // last row whose output starts at or before byte j
#pragma unroll
      for (int st = 0; st < 6; ++st) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_o[w][mid] <= j) lo = mid;
        else hi = mid - 1;
      }
      int row = lo;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int32_t b = j + k;
        if (b >= oend) break;
        while (s_o[w][row + 1] <= b) ++row;
        const int64_t src = s_s[w][row];
        out[b] = src < 0 ? stage[(-1 - src) * 16 + (b - s_o[w][row])] : data[src + (b - s_o[w][row])];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // s_o / s_s are rewritten next
    __builtin_amdgcn_wave_barrier();
  }
}

int dmalloc(qe_csv_table* t, size_t bytes, void** p) {
  if (dev_alloc(t->ctx, bytes ? bytes : 1, p) != QE_OK) return fail(QE_ERR_OOM, "device allocation of %zu bytes failed in CSV scan", bytes);
  t->owned.push_back(*p);
  return QE_OK;
}

int grid_for(qe_ctx* ctx, int64_t n, int threads = 256) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)div_up((uint64_t)(n > 0 ? n : 1), threads),
                                                      (int64_t)ctx->num_cus * 8));
}

int read_i64(qe_ctx* ctx, const int64_t* p, int64_t* out) {
  QE_HIP(hipMemcpyAsync(out, p, 8, hipMemcpyDeviceToHost, ctx->stream));
  QE_TRY(ctx_sync(ctx));
  return QE_OK;
}

// The value byte starts of every projected column for `rows` rows (their lengths in meta), the
// columns' sizes into t->total, and host[0] = *nskip (0 without one): one sync. Sets t->rows.
int column_sizes(qe_csv_table* t, int64_t rows, const unsigned long long* nskip, volatile int64_t* host) {
  qe_ctx* ctx = t->ctx;
  const int32_t nproj = t->nproj;
  t->rows = rows;
  t->total.assign((size_t)nproj, 0);
  t->maxlen.assign((size_t)nproj, 0);
  host[0] = 0;
  const int64_t nb = (int64_t)div_up((uint64_t)(rows > 0 ? rows : 1), 8192);
  void* p;
  QE_TRY(ctx_workspace(ctx, 3, (size_t)nproj * (size_t)(nb + 1) * 16, &p));
  int64_t* sums = (int64_t*)p;
  int64_t* maxs = sums + (size_t)nproj * (size_t)(nb + 1);
  if (rows > 0) {
    hipLaunchKernelGGL(k_csv_len_reduce, dim3((unsigned)nb, (unsigned)nproj), dim3(1024), 0, ctx->stream, t->meta(0),
                       t->stride, rows, nb, sums, maxs);
    QE_TRY(launch_check("k_csv_len_reduce"));
  } else {
    QE_HIP(hipMemsetAsync(sums, 0, (size_t)nproj * (size_t)(nb + 1) * 16, ctx->stream));
  }
  hipLaunchKernelGGL(k_csv_len_scan, dim3((unsigned)nproj), dim3(1024), 0, ctx->stream, sums, maxs, nb, t->bstart(0),
                     t->stride, rows, nskip, (int64_t*)host);
  QE_TRY(launch_check("k_csv_len_scan"));
  if (rows > 0) {
    hipLaunchKernelGGL(k_csv_len_apply, dim3((unsigned)nb, (unsigned)nproj), dim3(1024), 0, ctx->stream, t->meta(0),
                       t->stride, rows, nb, sums, t->bstart(0));
    QE_TRY(launch_check("k_csv_len_apply"));
  }
  QE_TRY(ctx_sync(ctx));
  // Lines that were not records left their rows' lengths unwritten: the sizes are meaningless and
  // the caller reruns the kept-line path (which rewrites every row) before it asks again.
  if (nskip && host[0] != 0) return QE_OK;
  for (int c = 0; c < nproj; ++c) {
    t->total[(size_t)c] = host[1 + c];
    t->maxlen[(size_t)c] = host[1 + nproj + c];
    QE_CHECK(t->total[(size_t)c] < (1ll << 31), QE_ERR_CAPACITY, "CSV column %d holds more than 2^31 bytes", c);
  }
  return QE_OK;
}

int csv_parse(qe_ctx* ctx, const uint8_t* data, int64_t nbytes, const qe_csv_options* opt, qe_csv_table* t) {
  const int32_t nproj = opt->nfields;
  QE_CHECK(nproj >= 1 && nproj <= CSV_MAX_FIELDS, QE_ERR_UNSUPPORTED, "CSV scan projects 1..%d fields (got %d)",
           CSV_MAX_FIELDS, nproj);
  QE_CHECK(opt->delimiter > 0 && opt->delimiter < 256 && opt->delimiter != '"' && opt->delimiter != '\n' &&
               opt->delimiter != '\r',
           QE_ERR_INVALID_ARG, "bad CSV delimiter %d", opt->delimiter);
  FieldArgs A;
  for (int i = 0; i < CSV_MAX_FIELD_INDEX; ++i) A.slot[i] = -1;
  A.max_field = -1;
  A.delim = opt->delimiter;
  A.low_mask = 0;
  for (int c = 0; c < nproj; ++c) {
    const int f = opt->field_index ? opt->field_index[c] : c;
    QE_CHECK(f >= 0 && f < CSV_MAX_FIELD_INDEX, QE_ERR_UNSUPPORTED, "CSV field index %d out of range", f);
    QE_CHECK(A.slot[f] < 0, QE_ERR_INVALID_ARG, "CSV field %d projected twice", f);
    A.slot[f] = (int16_t)c;
    A.max_field = std::max(A.max_field, f);
    if (f < 64) A.low_mask |= 1ull << f;
  }
  A.npf = 0;  // the projected field indices, ascending (walk_record_unquoted)
  for (int f = 0; f <= A.max_field; ++f)
    if (A.slot[f] >= 0) A.pf[A.npf++] = (int16_t)f;
  // ---- record terminators
  const int64_t nseg = (int64_t)div_up((uint64_t)(nbytes > 0 ? nbytes : 1), SEG);
  const int64_t spb = (int64_t)div_up((uint64_t)nseg, SP_TILE);
  const int wgrid = (int)div_up((uint64_t)nseg, 4);  // 4 waves per 256-thread block
  // the kernels below leave their few host-bound words in fine-grained pinned memory: one sync, no
  // read-back copies
  void* hp;
  QE_TRY(ctx_pinned_coherent(ctx, (size_t)(2 * nproj + 3) * 8, &hp));
  volatile int64_t* host = (volatile int64_t*)hp;
  void* p;
  int64_t* ends = nullptr;
  int64_t nterm = 0, last_end = -1;
  bool file_q = false, file_cr = false;
  int64_t* seg_qs = nullptr;
  int64_t* seg_ts = nullptr;
  QE_TRY(ctx_workspace(ctx, 0, (size_t)(8 * nseg + 6) * 8 + (size_t)div_up((uint64_t)nseg, SP_TILE) * sizeof(SegAgg) + (size_t)nseg,
                       &p));
  int64_t* seg_q = (int64_t*)p;
  seg_qs = seg_q + nseg;
  seg_ts = seg_qs + nseg + 1;
  int64_t* seg_t0 = seg_ts + nseg + 1;  // then seg_t1 [nseg], seg_l0 [nseg], seg_l1 [nseg]
  int64_t* seg_t1 = seg_t0 + nseg;
  SegAgg* agg = (SegAgg*)(seg_t1 + 3 * nseg);  // after seg_t1 / seg_l0 / seg_l1
  uint8_t* seg_cr = (uint8_t*)(agg + spb);
  // Fast path (a file without '"' or '\r', which only its bytes can tell): one classification pass
  // writes the '\n' and delimiter bitmaps and the segment counts; the line-end list and the line walk
  // then read bitmaps. A file with either byte reruns the general passes (k_csv_count2 ...).
  bool fast = nbytes > 0 && A.delim < 0x80;
  const size_t bmw = (size_t)div_up((uint64_t)(nbytes > 0 ? nbytes : 1), 64) + 4;  // 64-bit words per bitmap
  uint64_t* nlbm = nullptr;
  uint64_t* dbm = nullptr;
  auto plan = [&](bool classify) -> int {
    if (classify) {
      hipLaunchKernelGGL(k_csv_classify, dim3(wgrid), dim3(256), 0, ctx->stream, data, nbytes, nseg, (uint32_t)A.delim,
                         (uint16_t*)nlbm, (uint16_t*)dbm, seg_q, seg_t0, seg_t1, seg_cr);
      QE_TRY(launch_check("k_csv_classify"));
    } else if (nbytes > 0) {
      hipLaunchKernelGGL(k_csv_count2, dim3(wgrid), dim3(256), 0, ctx->stream, data, nbytes, nseg, seg_q, seg_t0, seg_t1,
                         seg_cr);
      QE_TRY(launch_check("k_csv_count2"));
    } else {
      QE_HIP(hipMemsetAsync(seg_q, 0, 8, ctx->stream));
      QE_HIP(hipMemsetAsync(seg_t0, 0, 16, ctx->stream));
      QE_HIP(hipMemsetAsync(seg_t0 + 2, 0xFF, 16, ctx->stream));  // no terminator (nseg == 1)
      QE_HIP(hipMemsetAsync(seg_cr, 0, 1, ctx->stream));
    }
    hipLaunchKernelGGL(k_csv_seg_reduce, dim3((unsigned)spb), dim3(SP_THREADS), 0, ctx->stream, seg_q, seg_t0, seg_t1, nseg,
                       seg_cr, agg);
    QE_TRY(launch_check("k_csv_seg_reduce"));
    hipLaunchKernelGGL(k_csv_seg_apply, dim3((unsigned)spb), dim3(SP_THREADS), 0, ctx->stream, seg_q, seg_t0, seg_t1, nseg,
                       agg, spb, seg_qs, seg_ts, (int64_t*)hp);
    QE_TRY(launch_check("k_csv_seg_apply"));
    return ctx_sync(ctx);
  };
  if (fast) {
    QE_TRY(ctx_workspace(ctx, 5, bmw * 16, &p));
    nlbm = (uint64_t*)p;
    dbm = nlbm + bmw;
    QE_TRY(plan(true));
    if (host[2] & 3) fast = false;  // a '"' or '\r': the general passes decide the records
  }
  if (!fast) QE_TRY(plan(false));
  nterm = host[0];
  last_end = host[1];
  file_q = (host[2] & 1) != 0;  // any '"' / '\r' in the bytes
  file_cr = (host[2] & 2) != 0;
  QE_TRY(ctx_workspace(ctx, 1, (size_t)(nterm + 2) * 8, &p));
  ends = (int64_t*)p;
  A.noq = file_q ? 0 : 1;
  QE_TRY(ctx_workspace(ctx, 4, (size_t)(2 * nterm + 5) * 8, &p));
  int64_t* keep = (int64_t*)p;
  int64_t* kstart = keep + nterm + 2;
  // bytes after the last terminator form a final record (also an unterminated quote at EOF), unless
  // the caller says more of the file follows (QE_CSV_PARTIAL_TAIL: they start its next chunk)
  const bool partial = (opt->flags & QE_CSV_PARTIAL_TAIL) != 0;
  const int64_t nlines = nterm + (!partial && last_end + 1 < nbytes ? 1 : 0);
  t->consumed = partial ? last_end + 1 : nbytes;
  const int64_t first = opt->has_header ? 1 : 0;
  t->nproj = nproj;
  t->data = data;
  t->stride = (nlines + 1 + 63) & ~(int64_t)63;  // every per-column array 256-byte aligned
  QE_TRY(dmalloc(t, (size_t)nproj * (size_t)t->stride * 16 + 64, &p));
  t->block = p;
  QE_TRY(dmalloc(t, (size_t)nproj * (size_t)t->stride * 16, &p));
  t->stage_block = (uint8_t*)p;
  for (int c = 0; c < nproj; ++c) {
    A.start[c] = t->start(c);
    A.meta[c] = t->meta(c);
    A.stage[c] = t->stage(c);
  }
  int64_t rows = 0;
  bool scanned = false;  // column sizes already known (the all-records fast path)
  const int64_t rows_all = std::max<int64_t>(0, nlines - first);
  if (nterm > 0 && fast) {
    hipLaunchKernelGGL(k_csv_ends_bm, dim3(wgrid), dim3(256), 0, ctx->stream, (const uint64_t*)nlbm, nbytes, nseg, seg_ts,
                       ends);
    QE_TRY(launch_check("k_csv_ends_bm"));
  } else if (nterm > 0) {
    auto kt = file_q ? (file_cr ? k_csv_terms<true, true> : k_csv_terms<true, false>)
                     : (file_cr ? k_csv_terms<false, true> : k_csv_terms<false, false>);
    hipLaunchKernelGGL(kt, dim3(wgrid), dim3(256), 0, ctx->stream, data, nbytes, nseg, seg_qs, seg_ts, ends);
    QE_TRY(launch_check("k_csv_terms<emit>"));
  }
  if (nlines > nterm) {
    hipLaunchKernelGGL(k_csv_set_i64, dim3(1), dim3(1), 0, ctx->stream, ends + nterm, nbytes);
    QE_TRY(launch_check("k_csv_set_i64"));
  }
  // ---- records and their projected fields
  if (nlines > 0) {
    // every line a record (the common case): one pass over the lines, no kept-line list
    unsigned long long* nskip = (unsigned long long*)keep;
    QE_HIP(hipMemsetAsync(nskip, 0, 8, ctx->stream));
    const int64_t blocks = std::min<int64_t>((int64_t)div_up(div_up((uint64_t)nlines, 64), 4), (int64_t)ctx->num_cus * 8);
    if (fast) {
      hipLaunchKernelGGL(k_csv_lines_bm, dim3((unsigned)blocks), dim3(256), 0, ctx->stream, data, nbytes,
                         (const uint64_t*)dbm, ends, nlines, first, A, nproj, nskip);
      QE_TRY(launch_check("k_csv_lines_bm"));
    } else {
      hipLaunchKernelGGL(k_csv_lines, dim3((unsigned)blocks), dim3(256), 0, ctx->stream, data, nbytes, ends, nlines, first,
                         A, nproj, nskip);
      QE_TRY(launch_check("k_csv_lines"));
    }
    // Speculatively every line a record (the common case): the columns' length scans run now, and
    // the skipped-line count and the column sizes come back with one sync.
    QE_TRY(column_sizes(t, rows_all, nskip, host));
    if (host[0] == 0) {
      rows = rows_all;
      scanned = true;
    } else {  // blank or comment lines: kept-line list, then the fields of the kept rows
      hipLaunchKernelGGL(k_csv_keep, dim3(grid_for(ctx, nlines)), dim3(256), 0, ctx->stream, data, ends, nlines, keep);
      QE_TRY(launch_check("k_csv_keep"));
      QE_TRY(exclusive_scan_i64(ctx, keep, kstart, nlines));
      int64_t nkept = 0;
      QE_TRY(read_i64(ctx, kstart + nlines, &nkept));
      QE_TRY(ctx_workspace(ctx, 2, (size_t)(nkept + 1) * 8, &p));
      int64_t* kept = (int64_t*)p;
      if (nkept > 0) {
        hipLaunchKernelGGL(k_csv_compact_lines, dim3(grid_for(ctx, nlines)), dim3(256), 0, ctx->stream, keep, kstart,
                           nlines, kept);
        QE_TRY(launch_check("k_csv_compact_lines"));
      }
      rows = std::max<int64_t>(0, nkept - first);
      if (rows > 0) {
        hipLaunchKernelGGL(k_csv_fields, dim3(grid_for(ctx, rows)), dim3(256), 0, ctx->stream, data, nbytes, ends, kept,
                           first, rows, A, nproj);
        QE_TRY(launch_check("k_csv_fields"));
      }
    }
  }
  if (scanned) return QE_OK;
  // ---- per column: byte positions of the values (scan of lengths) and the column's size
  return column_sizes(t, rows, nullptr, host);
}

bool copy_lds() {
  static const bool on = [] {
    const char* e = getenv("QE_CSV_COPY_LDS");
    return !(e && e[0] == '0');
  }();
  return on;
}

// Offsets + bytes of projected column c into dst (offsets for rows+1 entries, values >= total).
int build_column(qe_csv_table* t, int c, int32_t* offsets, uint8_t* values) {
  qe_ctx* ctx = t->ctx;
  const int64_t rows = t->rows;
  if (rows == 0) {
    QE_HIP(hipMemsetAsync(offsets, 0, 4, ctx->stream));
    return QE_OK;
  }
  hipLaunchKernelGGL(k_csv_copy_wave, dim3(grid_for(ctx, rows)), dim3(256), 0, ctx->stream, t->data, t->start(c),
                     t->meta(c), t->stage(c), t->bstart(c), rows, offsets, values, copy_lds() ? 1 : 0);
  return launch_check("k_csv_copy_wave");
}

}  // namespace
}  // namespace qe

using namespace qe;

extern "C" {

int qe_csv_parse(qe_ctx* ctx, const uint8_t* data, int64_t nbytes, const qe_csv_options* opt, qe_csv_table** out) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(opt && out && (data || nbytes == 0) && nbytes >= 0, QE_ERR_INVALID_ARG, "null argument");
  *out = nullptr;
  qe_csv_table* t = new qe_csv_table();
  t->ctx = ctx;
  const int rc = csv_parse(ctx, data, nbytes, opt, t);
  if (rc != QE_OK) {
    for (void* q : t->owned) dev_free(ctx, q);
    delete t;
    return rc;
  }
  *out = t;
  return QE_OK;
}

int qe_csv_rows(const qe_csv_table* t, int64_t* rows) {
  QE_CHECK(t && rows, QE_ERR_INVALID_ARG, "null argument");
  *rows = t->rows;
  return QE_OK;
}

int qe_csv_consumed(const qe_csv_table* t, int64_t* bytes) {
  QE_CHECK(t && bytes, QE_ERR_INVALID_ARG, "null argument");
  *bytes = t->consumed;
  return QE_OK;
}

int qe_csv_column(const qe_csv_table* tc, int32_t i, qe_column* out) {
  QE_CHECK(tc && out, QE_ERR_INVALID_ARG, "null argument");
  qe_csv_table* t = const_cast<qe_csv_table*>(tc);
  QE_CHECK(i >= 0 && i < t->nproj, QE_ERR_INVALID_ARG, "CSV column %d out of range", i);
  QE_TRY(ctx_enter(t->ctx));
  if (t->cols.empty()) t->cols.assign((size_t)t->nproj, qe_column{});
  qe_column& c = t->cols[(size_t)i];
  if (!c.offsets) {  // first request: build the column into table-owned buffers
    void* o;
    void* v;
    QE_TRY(dmalloc(t, (size_t)(t->rows + 1) * 4, &o));
    QE_TRY(dmalloc(t, (size_t)t->total[(size_t)i], &v));
    QE_TRY(build_column(t, i, (int32_t*)o, (uint8_t*)v));
    c.type = QE_TYPE_UTF8;
    c.length = t->rows;
    c.offsets = (int32_t*)o;
    c.values = v;
    // the parse's bound on the values' lengths travels with the column (a lone UTF8 GROUP BY key of
    // short values then needs no dictionary, qe_column.max_len)
    if (!t->maxlen.empty()) c.max_len = (int32_t)std::min<int64_t>(t->maxlen[(size_t)i], INT32_MAX);
  }
  *out = c;
  return QE_OK;
}

int qe_csv_column_bytes(const qe_csv_table* t, int32_t i, int64_t* nbytes) {
  QE_CHECK(t && nbytes, QE_ERR_INVALID_ARG, "null argument");
  QE_CHECK(i >= 0 && i < t->nproj, QE_ERR_INVALID_ARG, "CSV column %d out of range", i);
  *nbytes = t->total[(size_t)i];
  return QE_OK;
}

int qe_csv_column_max_len(const qe_csv_table* t, int32_t i, int64_t* nbytes) {
  QE_CHECK(t && nbytes, QE_ERR_INVALID_ARG, "null argument");
  QE_CHECK(i >= 0 && i < t->nproj, QE_ERR_INVALID_ARG, "CSV column %d out of range", i);
  *nbytes = t->maxlen.empty() ? 0 : t->maxlen[(size_t)i];
  return QE_OK;
}

int qe_csv_column_copy(const qe_csv_table* tc, int32_t i, qe_column* dst) {
  QE_CHECK(tc && dst, QE_ERR_INVALID_ARG, "null argument");
  qe_csv_table* t = const_cast<qe_csv_table*>(tc);
  QE_CHECK(i >= 0 && i < t->nproj, QE_ERR_INVALID_ARG, "CSV column %d out of range", i);
  QE_CHECK(dst->type == QE_TYPE_UTF8 && dst->offsets && dst->length >= t->rows, QE_ERR_INVALID_ARG,
           "destination must be UTF8 with room for %lld rows", (long long)t->rows);
  QE_CHECK(dst->values || t->total[(size_t)i] == 0, QE_ERR_CAPACITY, "destination values buffer required");
  QE_TRY(ctx_enter(t->ctx));
  QE_TRY(build_column(t, i, dst->offsets, (uint8_t*)dst->values));
  dst->length = t->rows;
  if (!t->maxlen.empty()) dst->max_len = (int32_t)std::min<int64_t>(t->maxlen[(size_t)i], INT32_MAX);
  return QE_OK;
}

int qe_csv_destroy(qe_csv_table* t) {
  if (!t) return QE_OK;
  (void)hipSetDevice(t->ctx->device);
  for (void* q : t->owned) dev_free(t->ctx, q);
  delete t;
  return QE_OK;
}

int qe_csv_record_end(const uint8_t* data, int64_t nbytes, int32_t eof, int64_t* cut) {
  QE_CHECK(cut && nbytes >= 0 && (data || nbytes == 0), QE_ERR_INVALID_ARG, "bad arguments");
  *cut = 0;
  if (eof) {
    *cut = nbytes;
    return QE_OK;
  }
  // quote parity of the whole buffer (it starts at a record boundary, outside quotes; '"' toggles
  // the quoted state anywhere, oracle/csv_ref.py split_records), then a walk back from the end to
  // the last terminator outside quotes: '\n', or a '\r' whose next byte is known not to be '\n'
  int64_t q = 0;
  for (int64_t i = 0; i < nbytes; ++i) q += data[i] == 0x22;
  for (int64_t i = nbytes - 1; i >= 0; --i) {
    const uint8_t c = data[i];
    if (c == 0x22) {
      --q;  // q = quotes in [0, i)
      continue;
    }
    if (q & 1) continue;  // inside a quoted field
    if (c == 0x0A || (c == 0x0D && i + 1 < nbytes && data[i + 1] != 0x0A)) {
      *cut = i + 1;
      return QE_OK;
    }
  }
  return QE_OK;
}

}  // extern "C"
