// Dictionary-keyed GROUP BY inside the C state, and partials merged or exchanged by key CONTENT.
//
// The reference groups by the `List` of key values, a Utf8 key being `String(bytes)` (K:620-627),
// and main() merges per-partition partials by those keys (K:1309-1325; its query, K:1336, groups by
// the Utf8 VendorID). The device table groups by one 64-bit word per row, so a UTF8 key — or a key
// list that does not pack into 63 bits — becomes dictionary codes (qe_strdict.hip). Codes are local
// to the dictionary that issued them: two partitions number the same string differently. So the
// dictionaries live inside the state (keys go in and come out as their declared columns), and
// partials move between states by content: the exporter decodes the keys of its records, routes each
// record by a content hash of its keys (qe_hash_partition: equal keys, same partition, on every
// rank), and ships the key values beside the records; the importer re-encodes them into its own
// dictionaries and rewrites the records' key words before merging them.
//
// Wire block (QE_KEYED_HEADER header, then 8-byte aligned sections):
//   records  nrec * rec_bytes   (key words 0 / 1 cleared: they are rebuilt by the importer)
//   per key  validity           nrec bytes (1 = non-null)
//            values             nrec * 8 (int64 / fp64 bits / sign-extended int32 / uint8 / bool)
//            or, UTF8:          nrec int32 lengths, then the bytes of the records in order
#include <vector>

#include "qe_internal.hpp"

namespace qe {

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int ensure(qe_ctx* ctx, size_t need) {
    need = std::max<size_t>(need, 64);
    if (need <= bytes) return QE_OK;
    dev_free(ctx, p);
    p = nullptr;
    bytes = 0;
    QE_TRY(dev_alloc(ctx, need, &p));
    bytes = need;
    return QE_OK;
  }
  void release(qe_ctx* ctx) {
    dev_free(ctx, p);
    p = nullptr;
    bytes = 0;
  }
};

constexpr uint64_t KEYED_MAGIC = 0x31444559454B4551ull;  // "QEKEYED1"
constexpr int SECT = 16;                                 // int64 words of section offsets per block

struct WireHeader {
  uint64_t magic;
  int64_t nrec;
  int64_t block_bytes;
  int32_t rec_bytes, nkeys;
  int32_t key_type[QE_MAX_KEYS];
  int64_t utf8_bytes[QE_MAX_KEYS];
  int64_t pad[6];
};
static_assert(sizeof(WireHeader) == QE_KEYED_HEADER, "keyed block header size");

inline int64_t pad8(int64_t x) { return (x + 7) & ~(int64_t)7; }
inline size_t bitmap_bytes(int64_t n) { return (size_t)div_up((uint64_t)std::max<int64_t>(n, 1), 32) * 4; }

// Section offsets of one block: [0] block start (set by the caller), [1] records, [2+k] validity of
// key k, [6+k] its values (or UTF8 lengths), [10+k] its UTF8 bytes; returns the block's size.
int64_t block_layout(int64_t nrec, int32_t rb, int nkeys, const int32_t* types, const int64_t* ub, int64_t* s) {
  for (int i = 0; i < SECT; ++i) s[i] = 0;
  int64_t o = QE_KEYED_HEADER;
  s[1] = o;
  o += nrec * rb;
  for (int k = 0; k < nkeys; ++k) {
    s[2 + k] = o;
    o += pad8(nrec);
    s[6 + k] = o;
    if (types[k] == QE_TYPE_UTF8) {
      o += pad8(4 * nrec);
      s[10 + k] = o;
      o += pad8(ub[k]);
    } else {
      o += 8 * nrec;
    }
  }
  return o;
}

// Columns as kernel arguments.
struct KCols {
  void* v[QE_MAX_KEYS];
  const uint8_t* valid[QE_MAX_KEYS];
  const int32_t* offs[QE_MAX_KEYS];
  int32_t type[QE_MAX_KEYS];
};

KCols kcols(const qe_column* c, int n) {
  KCols K{};
  for (int k = 0; k < n; ++k) {
    K.v[k] = c[k].values;
    K.valid[k] = c[k].validity;
    K.offs[k] = c[k].offsets;
    K.type[k] = c[k].type;
  }
  return K;
}

__device__ __forceinline__ bool bit_at(const uint8_t* b, int64_t i) { return !b || ((b[i >> 3] >> (i & 7)) & 1); }

__device__ __forceinline__ int64_t load_widened(const void* v, int32_t type, int64_t i) {
  switch (type) {
    case QE_TYPE_INT64:
    case QE_TYPE_FLOAT64: return ((const int64_t*)v)[i];
    case QE_TYPE_INT32:
    case QE_TYPE_DATE32: return ((const int32_t*)v)[i];
    case QE_TYPE_UINT8: return ((const uint8_t*)v)[i];
    default: return (((const uint8_t*)v)[i >> 3] >> (i & 7)) & 1;  // BOOL
  }
}

__device__ __forceinline__ void store_native(void* v, int32_t type, int64_t i, int64_t x) {
  switch (type) {
    case QE_TYPE_INT64:
    case QE_TYPE_FLOAT64: ((int64_t*)v)[i] = x; break;
    case QE_TYPE_INT32:
    case QE_TYPE_DATE32: ((int32_t*)v)[i] = (int32_t)x; break;
    default: ((uint8_t*)v)[i] = (uint8_t)x; break;
  }
}

// The wave's 64 bits of a bitmap, written as two whole 32-bit words by lane 0. Every lane calls it
// (i = the lane's row; the wave's rows start at a multiple of 64).
__device__ __forceinline__ void wave_bits(uint32_t* bm, int64_t i, int64_t n, bool bit) {
  const uint64_t b = __ballot(i < n && bit);
  if ((threadIdx.x & 63) == 0 && i < n) {
    bm[i >> 5] = (uint32_t)b;
    if (i + 32 < n) bm[(i >> 5) + 1] = (uint32_t)(b >> 32);
  }
}

// Exported records -> the device key columns the table grouped by (KeyMeta packing undone).
__global__ void k_rec_devkeys(const uint8_t* __restrict__ recs, int64_t n, int32_t rb, KeyMeta km, KCols o) {
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = base + threadIdx.x;
    int64_t key = 0;
    bool knull = false;
    if (i < n) {
      const int64_t* r = (const int64_t*)(recs + i * rb);
      key = r[0];
      knull = r[1] != 0;
    }
    for (int k = 0; k < km.nkeys; ++k) {
      bool ok;
      int64_t x;
      if (km.mode == 1) {
        ok = !knull;
        x = key;
      } else {
        ok = !((key >> km.nullbit[k]) & 1);
        x = (key >> km.shift[k]) & km.fmask[k];
        if (km.type[k] == QE_TYPE_INT32 || km.type[k] == QE_TYPE_DATE32) x = (int64_t)(int32_t)x;
      }
      if (i < n) store_native(o.v[k], km.type[k], i, ok ? x : 0);
      wave_bits((uint32_t*)o.valid[k], i, n, ok);
    }
  }
}

// Device key columns -> the records' key words (what the update kernels pack, qe_jit emit_keys).
__global__ void k_pack_devkeys(uint8_t* __restrict__ recs, int64_t n, int32_t rb, KeyMeta km, KCols in) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t key = 0, knull = 0;
    if (km.mode == 1) {
      const bool ok = bit_at(in.valid[0], i);
      int64_t x = ((const int64_t*)in.v[0])[i];
      if (km.type[0] == QE_TYPE_FLOAT64 && bits_f64(x) != bits_f64(x)) x = 0x7FF8000000000000ll;  // one NaN
      key = ok ? x : 0;
      knull = ok ? 0 : 1;
    } else if (km.mode == 2) {
      for (int k = 0; k < km.nkeys; ++k) {
        const bool ok = bit_at(in.valid[k], i);
        const int64_t x = load_widened(in.v[k], km.type[k], i);
        key |= ok ? (x & km.fmask[k]) << km.shift[k] : (int64_t)1 << km.nullbit[k];
      }
    }
    int64_t* r = (int64_t*)(recs + i * rb);
    r[0] = key;
    r[1] = knull;
  }
}

// Position of each row within its partition (order within a partition is free: records merge by
// key) and the partitions' counts: one cursor atomic per (wave, partition present).
__global__ void k_part_pos(const int32_t* __restrict__ part, int64_t n, unsigned long long* __restrict__ cursor,
                           int64_t* __restrict__ pos) {
  const int lane = threadIdx.x & 63;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = base + threadIdx.x;
    const bool has = i < n;
    const int32_t p = has ? part[i] : 0;
    uint64_t todo = __ballot(has);
    int64_t mine = 0;
    while (todo) {
      const int leader = __ffsll((long long)todo) - 1;
      const int32_t lp = __shfl(p, leader);
      const uint64_t same = __ballot(has && p == lp);
      unsigned long long b = 0;
      if (lane == leader) b = atomicAdd(&cursor[lp], (unsigned long long)__popcll(same));
      b = (unsigned long long)__shfl((long long)b, leader);
      if (has && p == lp) mine = (int64_t)b + __popcll(same & lt);
      todo &= ~same;
    }
    if (has) pos[i] = mine;
  }
}

// UTF8 key lengths in wire order (partition start + position), for the byte offsets' scan.
__global__ void k_wire_lens(const int32_t* __restrict__ offs, const uint8_t* __restrict__ valid,
                            const int32_t* __restrict__ part, const int64_t* __restrict__ pos,
                            const int64_t* __restrict__ start, int64_t n, int64_t* __restrict__ lw) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    lw[start[part[i]] + pos[i]] = bit_at(valid, i) ? (int64_t)(offs[i + 1] - offs[i]) : 0;
}

// ub[p * nk + k] = UTF8 bytes of key k in partition p.
__global__ void k_part_bytes(const int64_t* __restrict__ start, int32_t nparts, int32_t nk, const int64_t* b0,
                             const int64_t* b1, const int64_t* b2, const int64_t* b3, int64_t* __restrict__ ub) {
  const int64_t* bo[QE_MAX_KEYS] = {b0, b1, b2, b3};
  for (int p = threadIdx.x; p < nparts; p += blockDim.x)
    for (int k = 0; k < nk; ++k) ub[(int64_t)p * nk + k] = bo[k] ? bo[k][start[p + 1]] - bo[k][start[p]] : 0;
}

struct BOffs {
  const int64_t* b[QE_MAX_KEYS];  // wire-order exclusive byte offsets of each UTF8 key
};

__global__ void k_wire_gather(const uint8_t* __restrict__ recs, int64_t n, int32_t rb, int32_t nkeys,
                              const int32_t* __restrict__ part, const int64_t* __restrict__ pos,
                              const int64_t* __restrict__ start, const int64_t* __restrict__ sect, KCols keys,
                              BOffs bo, uint8_t* __restrict__ dst) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t p = part[i];
    const int64_t j = pos[i];
    const int64_t* S = sect + (int64_t)SECT * p;
    uint8_t* B = dst + S[0];
    const uint64_t* src = (const uint64_t*)(recs + i * rb);
    uint64_t* d = (uint64_t*)(B + S[1] + j * rb);
    d[0] = 0;
    d[1] = 0;
    for (int w = 2; w < rb / 8; ++w) d[w] = src[w];
    for (int k = 0; k < nkeys; ++k) {
      const bool ok = bit_at(keys.valid[k], i);
      B[S[2 + k] + j] = ok ? 1 : 0;
      if (keys.type[k] == QE_TYPE_UTF8) {
        const int32_t s0 = keys.offs[k][i];
        const int32_t len = ok ? keys.offs[k][i + 1] - s0 : 0;
        ((int32_t*)(B + S[6 + k]))[j] = len;
        const int64_t g = start[p] + j;
        uint8_t* bd = B + S[10 + k] + (bo.b[k][g] - bo.b[k][start[p]]);
        const uint8_t* bs = (const uint8_t*)keys.v[k] + s0;
        for (int32_t b = 0; b < len; ++b) bd[b] = bs[b];
      } else {
        ((int64_t*)(B + S[6 + k]))[j] = ok ? load_widened(keys.v[k], keys.type[k], i) : 0;
      }
    }
  }
}

// Received wire sections (validity bytes, 8-byte values) -> a column of the key's type.
__global__ void k_wire_to_col(const uint8_t* __restrict__ vb, const int64_t* __restrict__ v8, int64_t n, int32_t type,
                              void* __restrict__ out, uint32_t* __restrict__ bits) {
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = base + threadIdx.x;
    const bool ok = i < n && vb[i] != 0;
    const int64_t x = i < n && ok && v8 ? v8[i] : 0;
    wave_bits(bits, i, n, ok);
    if (type == QE_TYPE_BOOL) wave_bits((uint32_t*)out, i, n, x != 0);
    else if (v8 && i < n) store_native(out, type, i, x);
  }
}

__global__ void k_len_i64(const int32_t* __restrict__ l32, int64_t n, int64_t* __restrict__ l64) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    l64[i] = l32[i];
}

__global__ void k_off32(const int64_t* __restrict__ scan, int64_t n1, int32_t* __restrict__ offs) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n1; i += (int64_t)gridDim.x * blockDim.x)
    offs[i] = (int32_t)scan[i];
}

int grid_for(const qe_ctx* ctx, int64_t n) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)div_up((uint64_t)n, 256), (int64_t)ctx->num_cus * 8));
}

bool packs(int n, const int32_t* m) {
  if (n == 0) return true;
  if (n == 1 && (m[0] == QE_TYPE_INT64 || m[0] == QE_TYPE_FLOAT64)) return true;
  int bits = 0;
  for (int k = 0; k < n; ++k) {
    if (m[k] == QE_TYPE_INT32 || m[k] == QE_TYPE_DATE32) bits += 33;
    else if (m[k] == QE_TYPE_UINT8) bits += 9;
    else return false;
  }
  return bits <= 63;
}

}  // namespace

// Export preparation (qe_hashagg_export_keyed_sizes -> qe_hashagg_export_keyed).
struct KeyedPrep {
  bool valid = false;
  uint64_t version = 0;
  int32_t nparts = 0;
  int64_t n = 0;
  DevBuf recs, part, pos, cursor, start, sect, ub, lw[QE_MAX_KEYS], boff[QE_MAX_KEYS];
  DevBuf dk[QE_MAX_KEYS], dkv[QE_MAX_KEYS];                  // device keys of the records
  DevBuf mv[QE_MAX_KEYS], mvv[QE_MAX_KEYS];                  // tuple members
  DevBuf uo[QE_MAX_KEYS], ub8[QE_MAX_KEYS], uv[QE_MAX_KEYS];  // decoded UTF8 keys
  qe_column cols[QE_MAX_KEYS] = {};                            // the declared key columns of the records
  std::vector<int64_t> counts, block_off, block_bytes, ubh;
};

struct Keyed {
  int32_t norig = 0;
  int32_t orig[QE_MAX_KEYS] = {};    // declared key types
  int32_t member[QE_MAX_KEYS] = {};  // type after string coding (UTF8 -> INT32 / wide INT64 codes)
  qe_strdict* sdict[QE_MAX_KEYS] = {};
  bool sdict_owned[QE_MAX_KEYS] = {};
  qe_strdict* tdict = nullptr;  // key-tuple codes (members that do not pack)
  bool dict = false;            // the device keys are dictionary codes
  bool wide = false;            // a lone UTF8 key: wide INT64 codes
  int64_t expected = 1024;
  // encode outputs, two sets: a stream-ordered update's settle may re-read the previous set
  DevBuf code[2][QE_MAX_KEYS], cvalid[2][QE_MAX_KEYS], tcode[2];
  int cur = 0;
  // finalize intermediates
  DevBuf fkey[QE_MAX_KEYS], fkvalid[QE_MAX_KEYS], fmem[QE_MAX_KEYS], fmvalid[QE_MAX_KEYS];
  // import intermediates
  DevBuf irecs, ivb[QE_MAX_KEYS], iv8[QE_MAX_KEYS], il32[QE_MAX_KEYS], ibytes[QE_MAX_KEYS], ival[QE_MAX_KEYS],
      icol[QE_MAX_KEYS], il64[QE_MAX_KEYS], iscan[QE_MAX_KEYS], ioff[QE_MAX_KEYS];
  KeyedPrep prep;
  std::vector<DevBuf*> all() {
    std::vector<DevBuf*> v;
    for (int s = 0; s < 2; ++s) {
      for (int k = 0; k < QE_MAX_KEYS; ++k) v.insert(v.end(), {&code[s][k], &cvalid[s][k]});
      v.push_back(&tcode[s]);
    }
    for (int k = 0; k < QE_MAX_KEYS; ++k)
      v.insert(v.end(), {&fkey[k], &fkvalid[k], &fmem[k], &fmvalid[k], &ivb[k], &iv8[k], &il32[k], &ibytes[k],
                         &ival[k], &icol[k], &il64[k], &iscan[k], &ioff[k], &prep.lw[k], &prep.boff[k], &prep.dk[k],
                         &prep.dkv[k], &prep.mv[k], &prep.mvv[k], &prep.uo[k], &prep.ub8[k], &prep.uv[k]});
    v.insert(v.end(), {&irecs, &prep.recs, &prep.part, &prep.pos, &prep.cursor, &prep.start, &prep.sect, &prep.ub});
    return v;
  }
};

bool keyed_dict(const Keyed* K) { return K && K->dict; }
bool keyed_tuple(const Keyed* K) { return K && K->tdict; }

int keyed_create(qe_ctx* ctx, int32_t nkeys, const int32_t* types, int64_t expected, Keyed** out, int32_t* dev_nkeys,
                 int32_t* dev_types) {
  Keyed* K = new Keyed();
  K->norig = nkeys;
  K->expected = expected;
  int nutf8 = 0;
  for (int k = 0; k < nkeys; ++k) {
    const int32_t t = types[k];
    if (t != QE_TYPE_UTF8 && t != QE_TYPE_BOOL && !is_fixed(t)) {
      delete K;
      return fail(QE_ERR_UNSUPPORTED, "group key %d: type %d not supported", k, t);
    }
    K->orig[k] = t;
    nutf8 += t == QE_TYPE_UTF8;
  }
  K->wide = nkeys == 1 && nutf8 == 1;
  for (int k = 0; k < nkeys; ++k)
    K->member[k] = K->orig[k] == QE_TYPE_UTF8 ? (K->wide ? QE_TYPE_INT64 : QE_TYPE_INT32) : K->orig[k];
  int st = QE_OK;
  if (packs(nkeys, K->member)) {
    *dev_nkeys = nkeys;
    for (int k = 0; k < nkeys; ++k) dev_types[k] = K->member[k];
    K->dict = nutf8 > 0;
  } else {
    *dev_nkeys = 1;
    dev_types[0] = QE_TYPE_INT32;
    K->dict = true;
    st = qe_strdict_create(ctx, expected, &K->tdict);
  }
  // string dictionaries: a wide key's is created on its first long value (short values are their
  // own codes and never need one)
  for (int k = 0; k < nkeys && st == QE_OK; ++k)
    if (K->orig[k] == QE_TYPE_UTF8 && !K->wide) {
      st = qe_strdict_create(ctx, expected, &K->sdict[k]);
      K->sdict_owned[k] = st == QE_OK;
    }
  if (st != QE_OK) {
    keyed_destroy(ctx, K);
    return st;
  }
  *out = K;
  return QE_OK;
}

void keyed_destroy(qe_ctx* ctx, Keyed* K) {
  if (!K) return;
  for (DevBuf* b : K->all()) b->release(ctx);
  for (int k = 0; k < QE_MAX_KEYS; ++k)
    if (K->sdict_owned[k]) qe_strdict_destroy(K->sdict[k]);
  if (K->tdict) qe_strdict_destroy(K->tdict);
  delete K;
}

namespace {

int64_t dict_size(qe_strdict* d) {
  int64_t n = 0;
  if (d) (void)qe_strdict_size(d, &n);
  return n;
}

// Every value of lone-UTF8-key state so far is its own (packed) code: no dictionary holds a key.
bool all_packed(const Keyed* K, int k) { return K->wide && dict_size(K->sdict[k]) == 0; }

// The device key columns of rows given as the declared key columns (UTF8 encoded into this state's
// dictionaries, key tuples coded), written into buffer set `set`. mem[k]: the tuple members (or the
// device keys themselves when nothing is tuple-coded).
int encode_keys(qe_ctx* ctx, Keyed* K, uint64_t* ctl, const qe_column* keys, int set, qe_column* mem, qe_column* dev) {
  const int64_t n = K->norig ? keys[0].length : 0;
  for (int k = 0; k < K->norig; ++k) {
    const qe_column& c = keys[k];
    QE_CHECK(c.length == n, QE_ERR_INVALID_ARG, "group key %d has %lld rows, key 0 %lld", k, (long long)c.length,
             (long long)n);
    if (K->orig[k] != QE_TYPE_UTF8) {
      QE_CHECK(c.type == K->orig[k], QE_ERR_INVALID_ARG, "group key %d: type %d, declared %d", k, c.type, K->orig[k]);
      mem[k] = c;
      continue;
    }
    if (c.type == K->member[k] && K->sdict[k] && !K->sdict_owned[k]) {  // codes of a bound dictionary
      mem[k] = c;
      continue;
    }
    QE_CHECK(c.type == QE_TYPE_UTF8 && (c.offsets || n == 0), QE_ERR_INVALID_ARG, "group key %d must be UTF8", k);
    const bool w64 = K->member[k] == QE_TYPE_INT64;
    QE_TRY(K->code[set][k].ensure(ctx, (size_t)n * (w64 ? 8 : 4)));
    if (c.validity) QE_TRY(K->cvalid[set][k].ensure(ctx, bitmap_bytes(n)));
    qe_column cc{K->member[k], 0, n, c.validity ? (uint8_t*)K->cvalid[set][k].p : nullptr, K->code[set][k].p, nullptr};
    if (w64 && c.max_len >= 1 && c.max_len <= 7) {
      // every value is its own wide code: one stream-ordered kernel, no dictionary, checked against the
      // bound (a longer value fails the state's next read-back)
      QE_TRY(strdict_encode_packed_checked(ctx, &c, &cc, (unsigned long long*)(ctl + 3)));
    } else {
      if (!K->sdict[k]) {
        QE_TRY(qe_strdict_create(ctx, K->expected, &K->sdict[k]));
        K->sdict_owned[k] = true;
      }
      QE_TRY(qe_strdict_encode(K->sdict[k], &c, &cc));
    }
    mem[k] = cc;
  }
  if (K->tdict) {
    QE_TRY(K->tcode[set].ensure(ctx, (size_t)n * 4));
    qe_column tc{QE_TYPE_INT32, 0, n, nullptr, K->tcode[set].p, nullptr};
    QE_TRY(qe_strdict_encode_tuple(K->tdict, mem, K->norig, &tc));
    dev[0] = tc;
  } else {
    for (int k = 0; k < K->norig; ++k) dev[k] = mem[k];
  }
  return QE_OK;
}

// A decoded UTF8 column of `codes` (this state's key k) in the given buffers.
int decode_utf8(qe_ctx* ctx, Keyed* K, int k, const qe_column& codes, DevBuf& offs, DevBuf& bytes, DevBuf& valid,
                qe_column* out) {
  const int64_t n = codes.length;
  QE_TRY(offs.ensure(ctx, (size_t)(n + 1) * 4));
  if (codes.validity) QE_TRY(valid.ensure(ctx, bitmap_bytes(n)));
  const bool packed = all_packed(K, k);
  int64_t nb = 7 * n;
  if (!packed) QE_TRY(qe_strdict_decode_bytes(K->sdict[k], &codes, &nb));
  QE_TRY(bytes.ensure(ctx, (size_t)nb));
  *out = qe_column{QE_TYPE_UTF8, 0, n, codes.validity ? (uint8_t*)valid.p : nullptr, bytes.p, (int32_t*)offs.p};
  if (packed) return qe_strdict_decode_packed(ctx, &codes, out);
  return qe_strdict_decode(K->sdict[k], &codes, out);
}

// Buffers for a column of n rows of `type` (validity always) into `c`.
int column_in(qe_ctx* ctx, int32_t type, int64_t n, DevBuf& v, DevBuf& valid, qe_column* c) {
  const size_t vb = type == QE_TYPE_BOOL ? bitmap_bytes(n) : (size_t)n * type_width(type);
  QE_TRY(v.ensure(ctx, vb));
  QE_TRY(valid.ensure(ctx, bitmap_bytes(n)));
  *c = qe_column{type, 0, n, (uint8_t*)valid.p, v.p, nullptr};
  return QE_OK;
}

// Finalize's device key columns and tuple members: dev keys into K->fkey (or the caller's fixed key
// outputs), tuple members decoded into K->fmem (or, again, the caller's outputs). mem[k] = member k.
int finalize_members(qe_hashagg* h, Keyed* K, int64_t g, qe_column* out_keys, qe_column* out_aggs, bool keys_only,
                     qe_column* mem) {
  qe_ctx* ctx = hashagg_ctx(h);
  const HashaggInfo I = hashagg_info(h);
  qe_column dk[QE_MAX_KEYS];
  if (K->tdict) {
    QE_TRY(K->fkey[0].ensure(ctx, (size_t)g * 4));
    dk[0] = qe_column{QE_TYPE_INT32, 0, g, nullptr, K->fkey[0].p, nullptr};
  } else {
    for (int k = 0; k < K->norig; ++k) {
      if (K->orig[k] == QE_TYPE_UTF8 || !out_keys) QE_TRY(column_in(ctx, I.km.type[k], g, K->fkey[k], K->fkvalid[k], &dk[k]));
      else dk[k] = out_keys[k];
    }
  }
  int64_t g2 = 0;
  QE_TRY(hashagg_finalize_raw(h, dk, out_aggs, &g2, keys_only));
  QE_CHECK(g2 == g, QE_ERR_DEVICE, "group count changed during finalize");
  if (!K->tdict) {
    for (int k = 0; k < K->norig; ++k) mem[k] = dk[k];
    return QE_OK;
  }
  for (int k = 0; k < K->norig; ++k) {
    if (K->orig[k] == QE_TYPE_UTF8 || !out_keys) QE_TRY(column_in(ctx, K->member[k], g, K->fmem[k], K->fmvalid[k], &mem[k]));
    else mem[k] = out_keys[k];
  }
  if (g == 0) return QE_OK;
  return qe_strdict_decode_tuple(K->tdict, &dk[0], K->norig, mem);
}

}  // namespace

int keyed_update(qe_hashagg* h, const qe_column* keys, const qe_column* agg_inputs, const qe_column* mask) {
  const HashaggInfo I = hashagg_info(h);
  Keyed* K = I.keyed;
  K->cur ^= 1;
  qe_column mem[QE_MAX_KEYS], dev[QE_MAX_KEYS];
  QE_TRY(encode_keys(I.ctx, K, I.ctl, keys, K->cur, mem, dev));
  return hashagg_update_raw(h, dev, agg_inputs, mask);
}

int keyed_update_fused(qe_hashagg* h, const qe_column* cols, int32_t ncols, const qe_fused_spec* spec) {
  const HashaggInfo I = hashagg_info(h);
  Keyed* K = I.keyed;
  QE_CHECK(ncols >= 1 && ncols <= QE_MAX_COLS, QE_ERR_UNSUPPORTED, "fused plan takes 1..%d columns (got %d)",
           QE_MAX_COLS, ncols);
  qe_column kc[QE_MAX_KEYS];
  for (int k = 0; k < K->norig; ++k) {
    const int s = spec->key_cols[k];
    QE_CHECK(s >= 0 && s < ncols, QE_ERR_INVALID_ARG, "key %d: column slot %d out of range", k, s);
    kc[k] = cols[s];
  }
  K->cur ^= 1;
  qe_column mem[QE_MAX_KEYS], dev[QE_MAX_KEYS];
  QE_TRY(encode_keys(I.ctx, K, I.ctl, kc, K->cur, mem, dev));
  // the key slots now hold their codes (a UTF8 column can be nothing but a key in a plan); key-tuple
  // codes join as one more slot
  qe_column c2[QE_MAX_COLS];
  for (int c = 0; c < ncols; ++c) c2[c] = cols[c];
  qe_fused_spec s2 = *spec;
  for (int k = 0; k < K->norig; ++k)
    if (K->orig[k] == QE_TYPE_UTF8) c2[spec->key_cols[k]] = mem[k];
  int n2 = ncols;
  if (K->tdict) {
    QE_CHECK(ncols < QE_MAX_COLS, QE_ERR_UNSUPPORTED, "a fused plan over key-tuple codes takes at most %d columns",
             QE_MAX_COLS - 1);
    c2[n2] = dev[0];
    s2.key_cols[0] = n2++;
  }
  return hashagg_update_fused_raw(h, c2, n2, &s2);
}

int keyed_finalize(qe_hashagg* h, qe_column* out_keys, qe_column* out_aggs, int64_t* out_groups) {
  const HashaggInfo I = hashagg_info(h);
  Keyed* K = I.keyed;
  qe_ctx* ctx = I.ctx;
  int64_t g = 0;
  QE_TRY(qe_hashagg_num_groups(h, &g));
  if (out_groups) *out_groups = g;  // also on QE_ERR_CAPACITY: callers size the outputs from it
  QE_CHECK(out_keys, QE_ERR_INVALID_ARG, "null out_keys");
  for (int k = 0; k < K->norig; ++k) {
    const qe_column& c = out_keys[k];
    QE_CHECK(c.type == K->orig[k], QE_ERR_INVALID_ARG, "key output %d: type %d, expected %d", k, c.type, K->orig[k]);
    QE_CHECK(c.length >= g && (c.values || g == 0), QE_ERR_CAPACITY, "key output %d holds %lld rows, need %lld", k,
             (long long)c.length, (long long)g);
    QE_CHECK(!c.validity || ((uintptr_t)c.validity & 3) == 0, QE_ERR_INVALID_ARG, "validity must be 4-byte aligned");
    if (c.type == QE_TYPE_UTF8)
      QE_CHECK(c.offsets && c.validity, QE_ERR_INVALID_ARG, "UTF8 key output %d needs offsets and a validity buffer", k);
  }
  qe_column mem[QE_MAX_KEYS];
  QE_TRY(finalize_members(h, K, g, out_keys, out_aggs, false, mem));
  for (int k = 0; k < K->norig; ++k) {
    if (K->orig[k] != QE_TYPE_UTF8) {
      out_keys[k].length = g;
      continue;
    }
    qe_column o = out_keys[k];
    o.length = g;
    if (g == 0) {
      QE_HIP(hipMemsetAsync(o.offsets, 0, 4, ctx->stream));
    } else if (all_packed(K, k)) {
      QE_TRY(qe_strdict_decode_packed(ctx, &mem[k], &o));
    } else {
      QE_TRY(qe_strdict_decode_trusted(K->sdict[k], &mem[k], &o));
    }
    out_keys[k].length = g;
  }
  return QE_OK;
}

}  // namespace qe

using namespace qe;

namespace {

int check_same_layout(qe_hashagg* a, qe_hashagg* b) {
  const HashaggInfo A = hashagg_info(a), B = hashagg_info(b);
  bool same = A.keyed->norig == B.keyed->norig && A.naggs == B.naggs && A.rec_bytes == B.rec_bytes &&
              (A.flags & QE_HASHAGG_FAST_FP64) == (B.flags & QE_HASHAGG_FAST_FP64);
  for (int k = 0; same && k < A.keyed->norig; ++k) same = A.keyed->orig[k] == B.keyed->orig[k];
  for (int j = 0; same && j < A.naggs; ++j)
    same = A.aggs[j].fn == B.aggs[j].fn &&
           (A.aggs[j].fn == QE_AGG_COUNT_STAR || A.aggs[j].input_type == B.aggs[j].input_type);
  QE_CHECK(same, QE_ERR_INVALID_ARG, "the two states differ in key types, aggregates or options");
  return QE_OK;
}

// Block headers of `nblocks` received blocks (one read-back), validated against this state.
int read_headers(qe_ctx* ctx, const HashaggInfo& I, const uint8_t* blocks, int32_t nblocks, const int64_t* block_bytes,
                 std::vector<WireHeader>* hd, std::vector<int64_t>* off) {
  hd->assign((size_t)nblocks, WireHeader{});
  off->assign((size_t)nblocks, 0);
  int64_t o = 0;
  for (int b = 0; b < nblocks; ++b) {
    QE_CHECK(block_bytes[b] == 0 || block_bytes[b] >= QE_KEYED_HEADER, QE_ERR_INVALID_ARG,
             "block %d: %lld bytes is not a keyed block", b, (long long)block_bytes[b]);
    (*off)[(size_t)b] = o;
    if (block_bytes[b]) QE_HIP(hipMemcpyAsync(&(*hd)[(size_t)b], blocks + o, QE_KEYED_HEADER, hipMemcpyDeviceToHost, ctx->stream));
    o += block_bytes[b];
  }
  QE_TRY(ctx_sync(ctx));
  const Keyed* K = I.keyed;
  for (int b = 0; b < nblocks; ++b) {
    if (!block_bytes[b]) continue;
    const WireHeader& H = (*hd)[(size_t)b];
    QE_CHECK(H.magic == KEYED_MAGIC, QE_ERR_INVALID_ARG, "block %d is not a keyed partial block", b);
    bool same = H.rec_bytes == I.rec_bytes && H.nkeys == K->norig && H.nrec >= 0;
    for (int k = 0; same && k < K->norig; ++k) same = H.key_type[k] == K->orig[k];
    QE_CHECK(same, QE_ERR_INVALID_ARG, "block %d: key types or record layout differ from this state's", b);
    int64_t s[SECT];
    QE_CHECK(block_layout(H.nrec, H.rec_bytes, H.nkeys, H.key_type, H.utf8_bytes, s) == block_bytes[b] &&
                 H.block_bytes == block_bytes[b],
             QE_ERR_INVALID_ARG, "block %d: size %lld does not match its header", b, (long long)block_bytes[b]);
  }
  return QE_OK;
}

int import_keyed(qe_hashagg* h, const void* blocks_v, int32_t nblocks, const int64_t* block_bytes, int64_t* nrec_out) {
  const HashaggInfo I = hashagg_info(h);
  Keyed* K = I.keyed;
  qe_ctx* ctx = I.ctx;
  const uint8_t* blocks = (const uint8_t*)blocks_v;
  std::vector<WireHeader> hd;
  std::vector<int64_t> off;
  QE_TRY(read_headers(ctx, I, blocks, nblocks, block_bytes, &hd, &off));
  int64_t N = 0, ub[QE_MAX_KEYS] = {0, 0, 0, 0};
  for (int b = 0; b < nblocks; ++b)
    if (block_bytes[b]) {
      N += hd[(size_t)b].nrec;
      for (int k = 0; k < K->norig; ++k) ub[k] += hd[(size_t)b].utf8_bytes[k];
    }
  if (nrec_out) *nrec_out = N;
  if (N == 0) return QE_OK;
  const int32_t rb = I.rec_bytes;
  for (int k = 0; k < K->norig; ++k)
    QE_CHECK(ub[k] < (1ll << 31), QE_ERR_CAPACITY, "key %d: received strings exceed 2^31 bytes", k);
  // the blocks' sections, concatenated
  QE_TRY(K->irecs.ensure(ctx, (size_t)N * rb));
  for (int k = 0; k < K->norig; ++k) {
    QE_TRY(K->ivb[k].ensure(ctx, (size_t)N));
    if (K->orig[k] == QE_TYPE_UTF8) {
      QE_TRY(K->il32[k].ensure(ctx, (size_t)N * 4));
      QE_TRY(K->ibytes[k].ensure(ctx, (size_t)ub[k]));
    } else {
      QE_TRY(K->iv8[k].ensure(ctx, (size_t)N * 8));
    }
  }
  int64_t r = 0, ubo[QE_MAX_KEYS] = {0, 0, 0, 0};
  for (int b = 0; b < nblocks; ++b) {
    if (!block_bytes[b]) continue;
    const WireHeader& H = hd[(size_t)b];
    const int64_t m = H.nrec;
    if (m == 0) continue;
    int64_t s[SECT];
    (void)block_layout(m, rb, H.nkeys, H.key_type, H.utf8_bytes, s);
    const uint8_t* B = blocks + off[(size_t)b];
    QE_HIP(hipMemcpyAsync((uint8_t*)K->irecs.p + r * rb, B + s[1], (size_t)m * rb, hipMemcpyDeviceToDevice, ctx->stream));
    for (int k = 0; k < K->norig; ++k) {
      QE_HIP(hipMemcpyAsync((uint8_t*)K->ivb[k].p + r, B + s[2 + k], (size_t)m, hipMemcpyDeviceToDevice, ctx->stream));
      if (K->orig[k] == QE_TYPE_UTF8) {
        QE_HIP(hipMemcpyAsync((int32_t*)K->il32[k].p + r, B + s[6 + k], (size_t)m * 4, hipMemcpyDeviceToDevice,
                              ctx->stream));
        if (H.utf8_bytes[k])
          QE_HIP(hipMemcpyAsync((uint8_t*)K->ibytes[k].p + ubo[k], B + s[10 + k], (size_t)H.utf8_bytes[k],
                                hipMemcpyDeviceToDevice, ctx->stream));
        ubo[k] += H.utf8_bytes[k];
      } else {
        QE_HIP(hipMemcpyAsync((int64_t*)K->iv8[k].p + r, B + s[6 + k], (size_t)m * 8, hipMemcpyDeviceToDevice,
                              ctx->stream));
      }
    }
    r += m;
  }
  // the declared key columns of the N records
  qe_column cols[QE_MAX_KEYS];
  const int grid = grid_for(ctx, N);
  for (int k = 0; k < K->norig; ++k) {
    QE_TRY(K->ival[k].ensure(ctx, bitmap_bytes(N)));
    if (K->orig[k] == QE_TYPE_UTF8) {
      QE_TRY(K->il64[k].ensure(ctx, (size_t)N * 8));
      QE_TRY(K->iscan[k].ensure(ctx, (size_t)(N + 1) * 8));
      QE_TRY(K->ioff[k].ensure(ctx, (size_t)(N + 1) * 4));
      hipLaunchKernelGGL(k_wire_to_col, dim3(grid), dim3(256), 0, ctx->stream, (const uint8_t*)K->ivb[k].p,
                         (const int64_t*)nullptr, N, QE_TYPE_UTF8, (void*)nullptr, (uint32_t*)K->ival[k].p);
      QE_TRY(launch_check("k_wire_to_col"));
      hipLaunchKernelGGL(k_len_i64, dim3(grid), dim3(256), 0, ctx->stream, (const int32_t*)K->il32[k].p, N,
                         (int64_t*)K->il64[k].p);
      QE_TRY(launch_check("k_len_i64"));
      QE_TRY(exclusive_scan_i64(ctx, (const int64_t*)K->il64[k].p, (int64_t*)K->iscan[k].p, N));
      hipLaunchKernelGGL(k_off32, dim3(grid_for(ctx, N + 1)), dim3(256), 0, ctx->stream, (const int64_t*)K->iscan[k].p,
                         N + 1, (int32_t*)K->ioff[k].p);
      QE_TRY(launch_check("k_off32"));
      cols[k] = qe_column{QE_TYPE_UTF8, 0, N, (uint8_t*)K->ival[k].p, K->ibytes[k].p, (int32_t*)K->ioff[k].p};
    } else {
      const int32_t t = K->orig[k];
      QE_TRY(K->icol[k].ensure(ctx, t == QE_TYPE_BOOL ? bitmap_bytes(N) : (size_t)N * type_width(t)));
      hipLaunchKernelGGL(k_wire_to_col, dim3(grid), dim3(256), 0, ctx->stream, (const uint8_t*)K->ivb[k].p,
                         (const int64_t*)K->iv8[k].p, N, t, K->icol[k].p, (uint32_t*)K->ival[k].p);
      QE_TRY(launch_check("k_wire_to_col"));
      cols[k] = qe_column{t, 0, N, (uint8_t*)K->ival[k].p, K->icol[k].p, nullptr};
    }
  }
  // re-encode by content into this state's dictionaries, rebuild the records' key words, merge
  qe_column dev[QE_MAX_KEYS];
  if (K->dict) {
    qe_column mem[QE_MAX_KEYS];
    K->cur ^= 1;
    QE_TRY(encode_keys(ctx, K, I.ctl, cols, K->cur, mem, dev));
  } else {
    for (int k = 0; k < K->norig; ++k) dev[k] = cols[k];
  }
  const KCols dk = kcols(dev, I.km.nkeys);
  hipLaunchKernelGGL(k_pack_devkeys, dim3(grid), dim3(256), 0, ctx->stream, (uint8_t*)K->irecs.p, N, rb, I.km, dk);
  QE_TRY(launch_check("k_pack_devkeys"));
  return hashagg_import_raw(h, K->irecs.p, N);
}

}  // namespace

extern "C" {

int qe_hashagg_finalize_sizes(qe_hashagg* h, int64_t* groups, int64_t* key_bytes) {
  QE_CHECK(h && groups, QE_ERR_INVALID_ARG, "null argument");
  const HashaggInfo I = hashagg_info(h);
  QE_TRY(ctx_enter(I.ctx));
  Keyed* K = I.keyed;
  QE_TRY(qe_hashagg_num_groups(h, groups));
  if (!key_bytes) return QE_OK;
  const int64_t g = *groups;
  bool need = false;
  for (int k = 0; k < K->norig; ++k) {
    key_bytes[k] = 0;
    if (K->orig[k] != QE_TYPE_UTF8) continue;
    if (all_packed(K, k)) key_bytes[k] = 7 * g;
    else need = true;
  }
  if (!need || g == 0) return QE_OK;
  qe_column mem[QE_MAX_KEYS];
  QE_TRY(finalize_members(h, K, g, nullptr, nullptr, true, mem));
  for (int k = 0; k < K->norig; ++k)
    if (K->orig[k] == QE_TYPE_UTF8 && !all_packed(K, k)) QE_TRY(qe_strdict_decode_bytes(K->sdict[k], &mem[k], &key_bytes[k]));
  return QE_OK;
}

int qe_hashagg_key_bytes_bound(qe_hashagg* h, int32_t key, int64_t* per_group) {
  QE_CHECK(h && per_group, QE_ERR_INVALID_ARG, "null argument");
  const HashaggInfo I = hashagg_info(h);
  Keyed* K = I.keyed;
  QE_CHECK(K && key >= 0 && key < K->norig, QE_ERR_INVALID_ARG, "no key %d", key);
  *per_group = K->orig[key] == QE_TYPE_UTF8 && !K->tdict && all_packed(K, key) ? 7 : 0;
  return QE_OK;
}

int qe_hashagg_export_keyed_sizes(qe_hashagg* h, int32_t nparts, int64_t* block_bytes) {
  QE_CHECK(h && block_bytes && nparts >= 1, QE_ERR_INVALID_ARG, "bad arguments");
  const HashaggInfo I = hashagg_info(h);
  qe_ctx* ctx = I.ctx;
  QE_TRY(ctx_enter(ctx));
  Keyed* K = I.keyed;
  KeyedPrep& P = K->prep;
  P.valid = false;
  int64_t n = 0;  // records (a group with exact-SUM E words exports more than one)
  QE_TRY(hashagg_export_counts_raw(h, 1, &n));
  const int32_t rb = I.rec_bytes;
  const int nk = K->norig;
  // the records, then their declared key columns
  QE_TRY(P.recs.ensure(ctx, (size_t)n * rb));
  if (n) QE_TRY(hashagg_export_raw(h, 1, P.recs.p));
  qe_column dk[QE_MAX_KEYS];
  for (int k = 0; k < I.km.nkeys; ++k) QE_TRY(column_in(ctx, I.km.type[k], n, P.dk[k], P.dkv[k], &dk[k]));
  const int grid = grid_for(ctx, n);
  if (n && I.km.nkeys) {
    hipLaunchKernelGGL(k_rec_devkeys, dim3(grid), dim3(256), 0, ctx->stream, (const uint8_t*)P.recs.p, n, rb, I.km,
                       kcols(dk, I.km.nkeys));
    QE_TRY(launch_check("k_rec_devkeys"));
  }
  qe_column mem[QE_MAX_KEYS];
  if (K->tdict) {
    for (int k = 0; k < nk; ++k) QE_TRY(column_in(ctx, K->member[k], n, P.mv[k], P.mvv[k], &mem[k]));
    if (n) QE_TRY(qe_strdict_decode_tuple(K->tdict, &dk[0], nk, mem));
  } else {
    for (int k = 0; k < nk; ++k) mem[k] = dk[k];
  }
  for (int k = 0; k < nk; ++k) {
    if (K->orig[k] == QE_TYPE_UTF8) {
      QE_TRY(decode_utf8(ctx, K, k, mem[k], P.uo[k], P.ub8[k], P.uv[k], &P.cols[k]));
      if (n == 0) QE_HIP(hipMemsetAsync(P.cols[k].offsets, 0, 4, ctx->stream));
    } else {
      P.cols[k] = mem[k];
    }
  }
  // destination partition of every record by key content, its position there, the counts
  QE_TRY(P.part.ensure(ctx, (size_t)n * 4));
  QE_TRY(P.pos.ensure(ctx, (size_t)n * 8));
  QE_TRY(P.cursor.ensure(ctx, (size_t)nparts * 8));
  if (nparts == 1 || nk == 0) {
    QE_HIP(hipMemsetAsync(P.part.p, 0, (size_t)n * 4, ctx->stream));
  } else if (n) {
    QE_TRY(qe_hash_partition(ctx, P.cols, nk, nparts, (int32_t*)P.part.p));
  }
  QE_HIP(hipMemsetAsync(P.cursor.p, 0, (size_t)nparts * 8, ctx->stream));
  if (n) {
    hipLaunchKernelGGL(k_part_pos, dim3(grid), dim3(256), 0, ctx->stream, (const int32_t*)P.part.p, n,
                       (unsigned long long*)P.cursor.p, (int64_t*)P.pos.p);
    QE_TRY(launch_check("k_part_pos"));
  }
  P.counts.assign((size_t)nparts, 0);
  QE_HIP(hipMemcpyAsync(P.counts.data(), P.cursor.p, (size_t)nparts * 8, hipMemcpyDeviceToHost, ctx->stream));
  QE_TRY(ctx_sync(ctx));
  std::vector<int64_t> start((size_t)nparts + 1, 0);
  for (int p = 0; p < nparts; ++p) start[(size_t)p + 1] = start[(size_t)p] + P.counts[(size_t)p];
  QE_TRY(P.start.ensure(ctx, ((size_t)nparts + 1) * 8));
  QE_HIP(hipMemcpyAsync(P.start.p, start.data(), ((size_t)nparts + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  // UTF8 bytes per partition: lengths in wire order, their scan, the partitions' spans
  P.ubh.assign((size_t)nparts * std::max(nk, 1), 0);
  bool any_utf8 = false;
  const int64_t* bo[QE_MAX_KEYS] = {nullptr, nullptr, nullptr, nullptr};
  for (int k = 0; k < nk; ++k) {
    if (K->orig[k] != QE_TYPE_UTF8) continue;
    any_utf8 = true;
    QE_TRY(P.lw[k].ensure(ctx, (size_t)n * 8));
    QE_TRY(P.boff[k].ensure(ctx, (size_t)(n + 1) * 8));
    if (n) {
      hipLaunchKernelGGL(k_wire_lens, dim3(grid), dim3(256), 0, ctx->stream, P.cols[k].offsets, P.cols[k].validity,
                         (const int32_t*)P.part.p, (const int64_t*)P.pos.p, (const int64_t*)P.start.p, n,
                         (int64_t*)P.lw[k].p);
      QE_TRY(launch_check("k_wire_lens"));
      QE_TRY(exclusive_scan_i64(ctx, (const int64_t*)P.lw[k].p, (int64_t*)P.boff[k].p, n));
    } else {
      QE_HIP(hipMemsetAsync(P.boff[k].p, 0, 8, ctx->stream));
    }
    bo[k] = (const int64_t*)P.boff[k].p;
  }
  if (any_utf8) {
    QE_TRY(P.ub.ensure(ctx, (size_t)nparts * nk * 8));
    hipLaunchKernelGGL(k_part_bytes, dim3(1), dim3(256), 0, ctx->stream, (const int64_t*)P.start.p, nparts, nk, bo[0],
                       bo[1], bo[2], bo[3], (int64_t*)P.ub.p);
    QE_TRY(launch_check("k_part_bytes"));
    QE_HIP(hipMemcpyAsync(P.ubh.data(), P.ub.p, (size_t)nparts * nk * 8, hipMemcpyDeviceToHost, ctx->stream));
  }
  QE_TRY(ctx_sync(ctx));
  // block layouts
  std::vector<int64_t> sect((size_t)nparts * SECT);
  P.block_off.assign((size_t)nparts, 0);
  P.block_bytes.assign((size_t)nparts, 0);
  int64_t o = 0;
  for (int p = 0; p < nparts; ++p) {
    int64_t ub[QE_MAX_KEYS] = {0, 0, 0, 0};
    for (int k = 0; k < nk; ++k) ub[k] = P.ubh[(size_t)p * nk + k];
    int64_t* s = &sect[(size_t)p * SECT];
    const int64_t bytes = block_layout(P.counts[(size_t)p], rb, nk, K->orig, ub, s);
    s[0] = o;
    P.block_off[(size_t)p] = o;
    P.block_bytes[(size_t)p] = bytes;
    block_bytes[p] = bytes;
    o += bytes;
  }
  QE_TRY(P.sect.ensure(ctx, sect.size() * 8));
  QE_HIP(hipMemcpyAsync(P.sect.p, sect.data(), sect.size() * 8, hipMemcpyHostToDevice, ctx->stream));
  QE_TRY(ctx_sync(ctx));  // (the host vectors above go out of scope)
  P.valid = true;
  P.version = I.version;
  P.nparts = nparts;
  P.n = n;
  return QE_OK;
}

int qe_hashagg_export_keyed(qe_hashagg* h, int32_t nparts, void* dst) {
  QE_CHECK(h && nparts >= 1 && dst, QE_ERR_INVALID_ARG, "bad arguments");
  const HashaggInfo I = hashagg_info(h);
  qe_ctx* ctx = I.ctx;
  QE_TRY(ctx_enter(ctx));
  Keyed* K = I.keyed;
  KeyedPrep& P = K->prep;
  QE_CHECK(P.valid && P.version == I.version && P.nparts == nparts, QE_ERR_INVALID_ARG,
           "call qe_hashagg_export_keyed_sizes with these partitions first (the state changed since)");
  const int nk = K->norig;
  std::vector<WireHeader> hd((size_t)nparts);
  for (int p = 0; p < nparts; ++p) {
    WireHeader& H = hd[(size_t)p];
    memset(&H, 0, sizeof H);
    H.magic = KEYED_MAGIC;
    H.nrec = P.counts[(size_t)p];
    H.block_bytes = P.block_bytes[(size_t)p];
    H.rec_bytes = I.rec_bytes;
    H.nkeys = nk;
    for (int k = 0; k < nk; ++k) {
      H.key_type[k] = K->orig[k];
      H.utf8_bytes[k] = K->orig[k] == QE_TYPE_UTF8 ? P.ubh[(size_t)p * nk + k] : 0;
    }
    QE_HIP(hipMemcpyAsync((uint8_t*)dst + P.block_off[(size_t)p], &H, QE_KEYED_HEADER, hipMemcpyHostToDevice, ctx->stream));
  }
  if (P.n) {
    BOffs bo{};
    for (int k = 0; k < nk; ++k) bo.b[k] = K->orig[k] == QE_TYPE_UTF8 ? (const int64_t*)P.boff[k].p : nullptr;
    hipLaunchKernelGGL(k_wire_gather, dim3(grid_for(ctx, P.n)), dim3(256), 0, ctx->stream, (const uint8_t*)P.recs.p,
                       P.n, I.rec_bytes, nk, (const int32_t*)P.part.p, (const int64_t*)P.pos.p,
                       (const int64_t*)P.start.p, (const int64_t*)P.sect.p, kcols(P.cols, nk), bo, (uint8_t*)dst);
    QE_TRY(launch_check("k_wire_gather"));
  }
  return ctx_sync(ctx);  // the headers' host copies
}

int qe_hashagg_import_keyed(qe_hashagg* h, const void* blocks, int32_t nblocks, const int64_t* block_bytes) {
  QE_CHECK(h && nblocks >= 0 && (block_bytes || nblocks == 0), QE_ERR_INVALID_ARG, "bad arguments");
  QE_TRY(ctx_enter(hashagg_ctx(h)));
  for (int b = 0; b < nblocks; ++b) QE_CHECK(blocks || block_bytes[b] == 0, QE_ERR_INVALID_ARG, "null blocks");
  return import_keyed(h, blocks, nblocks, block_bytes, nullptr);
}

int qe_hashagg_merge(qe_hashagg* dst, qe_hashagg* src) {
  QE_CHECK(dst && src && dst != src, QE_ERR_INVALID_ARG, "bad arguments");
  qe_ctx* ctx = hashagg_ctx(dst);
  QE_CHECK(hashagg_ctx(src) == ctx, QE_ERR_INVALID_ARG, "the two states must share one qe_ctx (one stream)");
  QE_TRY(ctx_enter(ctx));
  QE_TRY(check_same_layout(dst, src));
  const HashaggInfo D = hashagg_info(dst), S = hashagg_info(src);
  void* buf = nullptr;
  int st;
  if (!keyed_dict(D.keyed) && !keyed_dict(S.keyed)) {  // raw key words mean the same in both
    int64_t cnt = 0;
    QE_TRY(qe_hashagg_export_counts(src, 1, &cnt));
    if (!cnt) return QE_OK;
    QE_TRY(dev_alloc(ctx, (size_t)cnt * S.rec_bytes, &buf));
    st = hashagg_export_raw(src, 1, buf);
    if (st == QE_OK) st = hashagg_import_raw(dst, buf, cnt);
  } else {
    int64_t bytes = 0;
    QE_TRY(qe_hashagg_export_keyed_sizes(src, 1, &bytes));
    QE_TRY(dev_alloc(ctx, (size_t)bytes, &buf));
    st = qe_hashagg_export_keyed(src, 1, buf);
    if (st == QE_OK) st = import_keyed(dst, buf, 1, &bytes, nullptr);
  }
  dev_free(ctx, buf);  // stream-ordered: reused only after the import's work
  return st;
}

int qe_hashagg_bind_key_dict(qe_hashagg* h, int32_t key, qe_strdict* dict) {
  QE_CHECK(h && dict, QE_ERR_INVALID_ARG, "null argument");
  const HashaggInfo I = hashagg_info(h);
  Keyed* K = I.keyed;
  QE_CHECK(I.version == 0, QE_ERR_INVALID_ARG, "bind the key dictionary before the first update");
  QE_CHECK(key >= 0 && key < K->norig && !K->tdict, QE_ERR_INVALID_ARG, "key %d is not a device key of this state", key);
  const int32_t t = K->orig[key];
  QE_CHECK(t == QE_TYPE_INT32 || (t == QE_TYPE_INT64 && K->norig == 1), QE_ERR_INVALID_ARG,
           "a dictionary binds to an INT32 key (or a lone INT64 key of wide codes), not type %d", t);
  QE_CHECK(!K->sdict[key], QE_ERR_INVALID_ARG, "key %d already has a dictionary", key);
  K->orig[key] = QE_TYPE_UTF8;
  K->member[key] = t;
  K->sdict[key] = dict;
  K->sdict_owned[key] = false;
  K->wide = t == QE_TYPE_INT64;
  K->dict = true;
  return QE_OK;
}

}  // extern "C"
