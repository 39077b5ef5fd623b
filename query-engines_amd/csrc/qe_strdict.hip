// UTF-8 group keys for HashAggregateExec (Main.kt:620-627: the row key is String(bytes), looked up
// in a HashMap<List<Any?>, ...> by content equality). The device replaces that HashMap's string
// hashing/equality with a string dictionary that gives every distinct byte string a dense, stable
// int32 code; the hash aggregate then groups by codes (bit-exact integer work) and finalize
// decodes the codes back to strings.
//
// Layout in HBM (all owned by the dictionary, sized for growth):
//   slots    s_hash[cap] (u64, 0 = empty; hashes are forced nonzero), s_code[cap] (i32, -1 = not
//            yet published, -2 = insertion failed for capacity) — open addressing, linear probing,
//            cap = 2 * ccap so the load factor stays <= 1/2;
//   codes    code_off[ccap] (i64 arena offset), code_len[ccap] (i32), code_hash[ccap] (u64);
//   arena    the distinct strings' bytes, bump-allocated.
// Equality is byte equality of the full string (the 64-bit hash only filters). Insertion: CAS the
// hash into an empty slot; the winner copies its bytes to the arena, takes the next code and
// publishes it. A row that meets a matching hash whose code is not yet published does not wait:
// it is marked in a retry bitmap and resolved by a second pass after the kernel boundary.
// Capacity overflow (codes, arena or probe limit) flags the batch; the host grows the arrays,
// rebuilds the slots from the code arrays (codes keep their numbers) and re-runs the batch.
#include "qe_internal.hpp"

struct qe_strdict;

namespace qe {

namespace {

struct DictDev {
  uint64_t* s_hash;
  int32_t* s_code;
  uint64_t mask;  // cap - 1
  int64_t* code_off;
  int32_t* code_len;
  uint64_t* code_hash;
  int64_t ccap;
  uint8_t* arena;
  int64_t acap;
  unsigned int* ncodes;
  unsigned long long* arena_used;
  unsigned int* flags;  // [0] overflow, [1] unresolved rows
};

constexpr int R_RETRY = -1, R_OVERFLOW = -2, R_CLAIMED = -3;

__device__ __forceinline__ uint64_t load_u64_unaligned(const uint8_t* p, int n) {
  uint64_t w = 0;
  if (n >= 8) {
    __builtin_memcpy(&w, p, 8);
  } else {
    for (int k = 0; k < n; ++k) w |= (uint64_t)p[k] << (8 * k);
  }
  return w;
}

__device__ __forceinline__ uint64_t str_hash(const uint8_t* p, int len) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ ((uint64_t)len * 0xC2B2AE3D27D4EB4Full);
  int i = 0;
  for (; i + 8 <= len; i += 8) h = fmix64(h ^ load_u64_unaligned(p + i, 8)) + 0x165667B19E3779F9ull;
  if (i < len) h = fmix64(h ^ load_u64_unaligned(p + i, len - i) ^ ((uint64_t)(len - i) << 59));
  h = fmix64(h);
  return h ? h : 1;
}

__device__ __forceinline__ bool bytes_equal(const uint8_t* a, const uint8_t* b, int len) {
  int i = 0;
  for (; i + 8 <= len; i += 8)
    if (load_u64_unaligned(a + i, 8) != load_u64_unaligned(b + i, 8)) return false;
  for (; i < len; ++i)
    if (a[i] != b[i]) return false;
  return true;
}

// Once the code arrays are full the batch will run again after growth: lookups stop early and
// no slot is claimed for a key that cannot get a code (a claimed-but-failed slot costs every
// later probe a step). Plain loads: a stale value only delays the exit.
__device__ __forceinline__ bool dict_full(const DictDev& D) {
  return *(volatile const uint32_t*)&D.flags[0] != 0 ||
         (int64_t)__hip_atomic_load(D.ncodes, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= D.ccap;
}

// probes before a lookup gives up (flags overflow: the slots grow and the batch runs again);
// the slot table stays at most half full, so only a table flooded by failed claims gets here
constexpr uint64_t MAX_PROBES = 1024;


// Probes for a key of hash h (`eq(code)` compares the key stored under a code with this row's).
// Returns its code, R_RETRY (a matching hash not yet published), R_OVERFLOW, or R_CLAIMED: this
// lane claimed an empty slot (*claimed) and must allocate and publish the code.
template <typename Eq>
__device__ int dict_probe(const DictDev& D, uint64_t h, Eq eq, uint64_t* claimed) {
  if (*(volatile const uint32_t*)&D.flags[0]) return R_OVERFLOW;
  uint64_t slot = h & D.mask;
  for (uint64_t probe = 0; probe <= D.mask && probe < MAX_PROBES; ++probe, slot = (slot + 1) & D.mask) {
    uint64_t sh = __hip_atomic_load(&D.s_hash[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (sh == 0) {
      if (dict_full(D)) {
        atomicOr(&D.flags[0], 1u);
        return R_OVERFLOW;
      }
      const uint64_t prev = atomicCAS((unsigned long long*)&D.s_hash[slot], 0ull, (unsigned long long)h);
      if (prev == 0) {
        *claimed = slot;
        return R_CLAIMED;
      }
      sh = prev;
    }
    if (sh == h) {
      const int c = __hip_atomic_load(&D.s_code[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      if (c == -1) return R_RETRY;  // claimed, not yet published: a retry pass takes the row
      if (c == R_OVERFLOW) return R_OVERFLOW;
      if (eq(c)) return c;
    }
  }
  atomicOr(&D.flags[0], 1u);
  return R_OVERFLOW;
}

// Code c (or R_OVERFLOW when c < 0) for a claimed slot: key bytes at arena offset a (`put`),
// code arrays, then the release store that publishes the slot.
template <typename Put>
__device__ __forceinline__ int dict_publish(const DictDev& D, uint64_t slot, uint64_t h, int len, int64_t a,
                                            int64_t cc, Put put) {
  int c = R_OVERFLOW;
  if (cc >= 0 && cc < D.ccap) {
    put(D.arena + a);
    D.code_off[cc] = a;
    D.code_len[cc] = len;
    D.code_hash[cc] = h;
    c = (int)cc;
  }
  __threadfence();
  __hip_atomic_store(&D.s_code[slot], c, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  if (c < 0) atomicOr(&D.flags[0], 1u);
  return c;
}

// One lane on its own (retry passes): arena bytes first, a code only if they fit, so every code
// below ccap is published.
template <typename Put>
__device__ int dict_insert_one(const DictDev& D, uint64_t slot, uint64_t h, int len, Put put) {
  const unsigned long long a = atomicAdd(D.arena_used, (unsigned long long)len);
  int64_t cc = -1;
  if ((int64_t)(a + len) <= D.acap) cc = (int64_t)atomicAdd(D.ncodes, 1u);
  return dict_publish(D, slot, h, len, (int64_t)a, cc, put);
}

// The whole (converged) wave: lanes with `claim` get arena bytes and codes with ONE atomic per
// wave on each counter — high-cardinality batches insert many keys per wave, and per-lane
// atomics on the two counters serialise the chip. Same allocation rule as dict_insert_one.
template <typename Put>
__device__ int dict_insert_wave(const DictDev& D, bool claim, uint64_t slot, uint64_t h, int len, Put put,
                                int lane) {
  const uint64_t cm = __ballot(claim);
  if (!cm) return R_OVERFLOW;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  const long long x = claim ? len : 0;
  long long inc = x;
  for (int off = 1; off < 64; off <<= 1) {
    const long long y = __shfl_up(inc, off);
    if (lane >= off) inc += y;
  }
  const long long total = __shfl(inc, 63);
  const int first = __ffsll((long long)cm) - 1;
  unsigned long long abase = 0;
  if (lane == first) abase = atomicAdd(D.arena_used, (unsigned long long)total);
  abase = __shfl(abase, first);
  const int64_t a = (int64_t)abase + (inc - x);
  const bool fits = claim && a + len <= D.acap;
  const uint64_t fm = __ballot(fits);
  unsigned int cbase = 0;
  if (fm) {
    const int f0 = __ffsll((long long)fm) - 1;
    if (lane == f0) cbase = atomicAdd(D.ncodes, (unsigned int)__popcll(fm));
    cbase = __shfl(cbase, f0);
  }
  if (!claim) return R_OVERFLOW;
  return dict_publish(D, slot, h, len, a, fits ? (int64_t)cbase + __popcll(fm & lt) : -1, put);
}

// code >= 0, R_RETRY or R_OVERFLOW for one string on its own.
__device__ int dict_find_or_insert(const DictDev& D, const uint8_t* p, int len, uint64_t h) {
  uint64_t slot = 0;
  const int r = dict_probe(
      D, h, [&](int c) { return D.code_len[c] == len && bytes_equal(D.arena + D.code_off[c], p, len); }, &slot);
  if (r != R_CLAIMED) return r;
  return dict_insert_one(D, slot, h, len, [&](uint8_t* dst) {
    for (int k = 0; k < len; ++k) dst[k] = p[k];
  });
}

constexpr int ENC_THREADS = 256;

// Wide (int64) key codes (qe_strdict_encode64): a key of at most 7 bytes IS its code — its bytes in
// bits 0..55 (little-endian) and its length in bits 56..58 — and never touches the dictionary; a
// longer key is WIDE_DICT | its dictionary code. Equal strings get equal codes either way, a short
// and a long string never collide, and bit 63 stays clear (the hash aggregate's empty key is
// INT64_MIN).
constexpr int WIDE_MAX = 7;
constexpr uint64_t WIDE_DICT = 1ull << 62;
__device__ __forceinline__ int64_t wide_pack(uint64_t w, int len) {
  return (int64_t)((w & ((1ull << 56) - 1)) | ((uint64_t)len << 56));
}
__device__ __forceinline__ void put_code(int32_t* codes, int64_t* codes64, int64_t i, int c) {
  if (codes64) codes64[i] = c >= 0 ? (int64_t)(WIDE_DICT | (uint64_t)c) : 0;
  else codes[i] = c >= 0 ? c : 0;
}

__device__ __forceinline__ void encode_row(const DictDev& D, const int32_t* offs, const uint8_t* bytes, int64_t i,
                                           int32_t* codes, int64_t* codes64, uint32_t* retry) {
  const int32_t s0 = offs[i], len = offs[i + 1] - s0;
  const uint8_t* p = bytes + s0;
  const int c = dict_find_or_insert(D, p, len, str_hash(p, len));
  put_code(codes, codes64, i, c);
  if (c == R_RETRY) {
    atomicOr(&retry[i >> 5], 1u << (i & 31));
    atomicAdd(&D.flags[1], 1u);
  }
}

// Per-workgroup LDS cache of resolved strings: low-cardinality keys (the reference's VendorID)
// resolve without touching the global table, whose slots all rows would otherwise hit. An entry
// is published with state 2 after its fields are written. Only keys of up to 40 bytes are cached
// (they compare entirely in LDS); longer keys always take the global path.
constexpr int LC_SLOTS = 512, LC_BYTES = 40;
struct LdsCache {
  uint32_t state[LC_SLOTS];  // 0 empty, 1 being written, 2 ready
  uint64_t hash[LC_SLOTS];
  int32_t len[LC_SLOTS];
  int32_t code[LC_SLOTS];
  uint64_t head[LC_SLOTS][LC_BYTES / 8];
};

// LDS cache lookup / insert: linear probing over LC_PROBES slots (entries are never removed, so
// an empty slot ends a lookup). A key whose home slots are all taken just stays uncached.
constexpr int LC_PROBES = 8;
__device__ __forceinline__ int lc_find(LdsCache& C, uint64_t h, int32_t len, const uint64_t (&hd)[LC_BYTES / 8]) {
  int slot = (int)(h & (LC_SLOTS - 1));
  for (int q = 0; q < LC_PROBES; ++q, slot = (slot + 1) & (LC_SLOTS - 1)) {
    const uint32_t st = __hip_atomic_load(&C.state[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (st == 0) return -1;
    if (st == 2 && C.hash[slot] == h && C.len[slot] == len) {
      bool eq = true;
#pragma unroll
      for (int k = 0; k < LC_BYTES / 8; ++k) eq &= C.head[slot][k] == hd[k];
      if (eq) return C.code[slot];
    }
  }
  return -1;
}

__device__ __forceinline__ void lc_insert(LdsCache& C, uint64_t h, int32_t len, const uint64_t (&hd)[LC_BYTES / 8],
                                          int code) {
  int slot = (int)(h & (LC_SLOTS - 1));
  for (int q = 0; q < LC_PROBES; ++q, slot = (slot + 1) & (LC_SLOTS - 1)) {
    if (atomicCAS(&C.state[slot], 0u, 1u) == 0u) {
      C.hash[slot] = h;
      C.len[slot] = len;
      C.code[slot] = code;
#pragma unroll
      for (int k = 0; k < LC_BYTES / 8; ++k) C.head[slot][k] = hd[k];
      __hip_atomic_store(&C.state[slot], 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      return;
    }
  }
}

// Leader election: the first missing lane holding the same key (hash, length and the five head
// words all equal); lanes with dedup false lead themselves. Costs shuffles per DISTINCT key of
// the wave, no memory traffic — the lookups that follow run in parallel.
__device__ __forceinline__ int wave_leader(bool miss, bool dedup, uint64_t h, int32_t len,
                                           const uint64_t (&hd)[LC_BYTES / 8], int lane) {
  int leader = lane;
  uint64_t rest = __ballot(miss && dedup);
  while (rest) {
    const int k = __ffsll((long long)rest) - 1;
    bool same = ((rest >> lane) & 1) && __shfl(h, k) == h && __shfl(len, k) == len;
#pragma unroll
    for (int w = 0; w < LC_BYTES / 8; ++w) same = same && __shfl(hd[w], k) == hd[w];
    if (same) leader = k;
    rest &= ~__ballot(same) & ~(1ull << k);
  }
  return leader;
}

__device__ __forceinline__ void head32(const uint8_t* p, int len, uint64_t (&h)[LC_BYTES / 8]) {
#pragma unroll
  for (int k = 0; k < LC_BYTES / 8; ++k) {
    const int o = 8 * k;
    h[k] = o < len ? load_u64_unaligned(p + o, len - o >= 8 ? 8 : len - o) : 0;
  }
}

// One row's full lookup (LDS cache, then the wave's leaders on the global table, inserting new keys),
// for every lane of the converged wave at once; a row another wave has claimed but not published is
// deferred (s_def) or marked for the retry pass. The slow path of k_dict_encode's steps.
struct EncShared {
  LdsCache C;
  int wg_full;  // a lane of this workgroup saw the dictionary full: the batch reruns
  int ndef;
  int64_t def[2048];
};
constexpr int DEF_CAP = 2048;

__device__ __forceinline__ void encode_lookup(const DictDev& D, EncShared& S, const int32_t* __restrict__ offs,
                                              const uint8_t* __restrict__ bytes, int64_t n, int64_t i, bool live,
                                              int32_t* __restrict__ codes, int64_t* __restrict__ codes64,
                                              uint32_t* __restrict__ retry, int lane) {
  int32_t len = 0;
  const uint8_t* p = bytes;
  uint64_t h = 0;
  uint64_t hd[LC_BYTES / 8] = {0, 0, 0, 0, 0};
  int c = -1;
  if (live) {
    const int32_t s0 = offs[i];
    len = offs[i + 1] - s0;
    p = bytes + s0;
    h = str_hash(p, len);
    head32(p, len, hd);
    if (len <= LC_BYTES) c = lc_find(S.C, h, len, hd);
  }
  // misses: the first lane of each distinct key in the wave looks it up, all leaders at once
  // (keys over 40 bytes: every lane for itself); the other lanes take their leader's code
  const bool miss = live && c < 0;
  if (__ballot(miss)) {
    const int leader = wave_leader(miss, len <= LC_BYTES, h, len, hd, lane);
    const bool lead = miss && leader == lane;
    int code = 0;
    uint64_t gslot = 0;
    if (lead)
      code = dict_probe(
          D, h, [&](int cc) { return D.code_len[cc] == len && bytes_equal(D.arena + D.code_off[cc], p, len); },
          &gslot);
    const bool claim = lead && code == R_CLAIMED;
    const int pc = dict_insert_wave(D, claim, gslot, h, len, [&](uint8_t* dst) {
      for (int k = 0; k < len; ++k) dst[k] = p[k];
    }, lane);
    if (claim) code = pc;
    // a key another wave has claimed but not yet published: its insert is a few stores away (every
    // workgroup is resident and the claimer waits for nobody), so wait a little for it rather than
    // defer the row (at a batch's start every wave of the grid meets the new keys at once). After
    // this wave's own inserts, so a claimer in this wave has published.
    if (lead && code == R_RETRY) {
      auto eq = [&](int cc) { return D.code_len[cc] == len && bytes_equal(D.arena + D.code_off[cc], p, len); };
      for (int t = 0; t < 64 && code == R_RETRY; ++t) {
        __builtin_amdgcn_s_sleep(2);
        code = dict_probe(D, h, eq, &gslot);
      }
      if (code == R_CLAIMED)  // (a hash collision past the claimed slot) this lane inserts alone
        code = dict_insert_one(D, gslot, h, len, [&](uint8_t* dst) {
          for (int k = 0; k < len; ++k) dst[k] = p[k];
        });
    }
    if (lead && code >= 0 && len <= LC_BYTES) lc_insert(S.C, h, len, hd, code);
    code = __shfl(code, leader);
    if (miss) c = code;
  }
  if (live && i < n) {  // (the other lanes' rows are not this call's: the caller wrote them)
    put_code(codes, codes64, i, c);
    if (c == R_OVERFLOW) S.wg_full = 1;
    if (c == R_RETRY) {
      const int d = atomicAdd(&S.ndef, 1);
      if (d < DEF_CAP) {
        S.def[d] = i;
      } else {
        atomicOr(&retry[i >> 5], 1u << (i & 31));
        atomicAdd(&D.flags[1], 1u);
      }
    }
  }
}

// str_hash of a key of at most 8 bytes held in one word (what str_hash computes for it).
__device__ __forceinline__ uint64_t str_hash_short(uint64_t w, int len) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ ((uint64_t)len * 0xC2B2AE3D27D4EB4Full);
  if (len == 8) h = fmix64(h ^ w) + 0x165667B19E3779F9ull;
  else if (len > 0) h = fmix64(h ^ w ^ ((uint64_t)len << 59));
  h = fmix64(h);
  return h ? h : 1;
}

// 1024-thread workgroups, one per CU (one LDS cache per CU, warmed once; 16 waves to hide the
// offset -> byte -> cache latency chain). A wave step takes 256 rows, 4 per lane (rows
// base + 64 r + lane): their offsets and key words load together, then each key of at most 8 bytes
// is looked up in the LDS cache by its one word; every other row (longer keys, cache misses while
// the cache warms) takes encode_lookup. Round 4 ran one row per lane per step, 8 waves per CU:
// 112 us for tripdata's 4M VendorIDs.
// WIDE (int64 codes): keys of at most 7 bytes are packed in place, only longer keys look up.
constexpr int ENC_BLOCK = 1024;
template <bool WIDE>
__global__ void __launch_bounds__(ENC_BLOCK) k_dict_encode(DictDev D, const int32_t* __restrict__ offs,
                                                           const uint8_t* __restrict__ bytes,
                                                           const uint8_t* __restrict__ valid, int64_t n,
                                                           int32_t* __restrict__ codes, int64_t* __restrict__ codes64,
                                                           uint32_t* __restrict__ retry) {
  __shared__ EncShared S;
  for (int k = threadIdx.x; k < LC_SLOTS; k += blockDim.x) S.C.state[k] = 0;
  if (threadIdx.x == 0) {
    S.wg_full = 0;
    S.ndef = 0;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t wstride = ((int64_t)gridDim.x * blockDim.x >> 6) * 256;
  for (int64_t base = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x - lane) * 4; base < n; base += wstride) {
    if (*(volatile int*)&S.wg_full) break;  // uniform per wave (LDS)
    int64_t row[4];
    bool live[4];
    int32_t s0[4], len[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      row[r] = base + 64 * r + lane;
      live[r] = row[r] < n && (!valid || ((valid[row[r] >> 3] >> (row[r] & 7)) & 1));
      s0[r] = live[r] ? offs[row[r]] : 0;
      len[r] = live[r] ? offs[row[r] + 1] : 0;
    }
    uint64_t w[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      len[r] -= s0[r];
      w[r] = (live[r] && len[r] <= 8) ? load_u64_unaligned(bytes + s0[r], len[r]) : 0ull;
    }
    qu32 slow = 0;
    if (WIDE) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (live[r] && len[r] > WIDE_MAX) slow |= 1u << r;
        else if (row[r] < n) codes64[row[r]] = live[r] ? wide_pack(w[r], len[r]) : 0;
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int c = -1;
        if (live[r] && len[r] <= 8) {
          const uint64_t h = str_hash_short(w[r], len[r]);
          const uint64_t hd[LC_BYTES / 8] = {w[r], 0, 0, 0, 0};
          c = lc_find(S.C, h, len[r], hd);
        }
        if (live[r] && c < 0) slow |= 1u << r;
        else if (row[r] < n) codes[row[r]] = live[r] ? c : 0;
      }
    }
    // rows the cache did not answer: the full lookup, one row position at a time (rolled: its
    // code is large and runs only while the cache warms or for long keys)
#pragma unroll 1
    for (int r = 0; r < 4; ++r) {
      const bool sl = (slow >> r) & 1;
      if (!__ballot(sl)) continue;
      const int64_t i = base + 64 * r + lane;
      encode_lookup(D, S, offs, bytes, n, i, sl, codes, WIDE ? codes64 : nullptr, retry, lane);
    }
  }
  __syncthreads();
  const int nd = S.ndef < DEF_CAP ? S.ndef : DEF_CAP;
  for (int d = threadIdx.x; d < nd; d += blockDim.x) {
    const int64_t i = S.def[d];
    const int32_t s0 = offs[i], len = offs[i + 1] - s0;
    const uint8_t* p = bytes + s0;
    const uint64_t h = str_hash(p, len);
    int c = -1;
    if (len <= LC_BYTES) {
      uint64_t hd[LC_BYTES / 8];
      head32(p, len, hd);
      c = lc_find(S.C, h, len, hd);
    }
    if (c < 0) c = dict_find_or_insert(D, p, len, h);
    put_code(codes, WIDE ? codes64 : nullptr, i, c);
    if (c == R_OVERFLOW) S.wg_full = 1;
    if (c == R_RETRY) {
      atomicOr(&retry[i >> 5], 1u << (i & 31));
      atomicAdd(&D.flags[1], 1u);
    }
  }
}

// Second pass over the rows of `retry_in` (all codes seen by pass 1 are published by now).
__global__ void __launch_bounds__(ENC_THREADS) k_dict_encode_retry(DictDev D, const int32_t* __restrict__ offs,
                                                                   const uint8_t* __restrict__ bytes, int64_t n,
                                                                   int32_t* __restrict__ codes,
                                                                   int64_t* __restrict__ codes64,
                                                                   const uint32_t* __restrict__ retry_in,
                                                                   uint32_t* __restrict__ retry_out) {
  const int64_t words = (n + 31) >> 5;
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < words; w += (int64_t)gridDim.x * blockDim.x) {
    uint32_t bits = retry_in[w];
    while (bits) {
      const int j = __builtin_ctz(bits);
      bits &= bits - 1;
      encode_row(D, offs, bytes, (w << 5) + j, codes, codes64, retry_out);
    }
  }
}

// ---- composite keys: a row's key tuple as 5 words (up to 4 keys + a null-flag word) -------------
// Key k occupies word k (fp64 NaN canonicalised: Double.equals puts every NaN in one group, and
// +0.0 / -0.0 stay apart); word 4 holds the null flags. Every tuple is 40 bytes, so tuple arenas
// stay 8-byte aligned and compare word by word.
constexpr int TW = 5;
enum : int32_t { TK_I64 = 0, TK_F64 = 1, TK_I32 = 2, TK_U8 = 3, TK_BOOL = 4 };
struct TupleCols {
  const void* v[QE_MAX_KEYS];
  const uint8_t* valid[QE_MAX_KEYS];
  int32_t kind[QE_MAX_KEYS];
  int32_t nkeys;
};

__device__ __forceinline__ void tuple_words(const TupleCols& T, int64_t i, uint64_t (&w)[TW]) {
  uint64_t flags = 0;
#pragma unroll
  for (int k = 0; k < QE_MAX_KEYS; ++k) {
    uint64_t x = 0;
    if (k < T.nkeys) {
      const bool ok = !T.valid[k] || ((T.valid[k][i >> 3] >> (i & 7)) & 1);
      if (ok) {
        switch (T.kind[k]) {
          case TK_I64: x = ((const uint64_t*)T.v[k])[i]; break;
          case TK_F64: {
            x = ((const uint64_t*)T.v[k])[i];
            const double d = bits_f64((int64_t)x);
            if (d != d) x = 0x7FF8000000000000ull;
            break;
          }
          case TK_I32: x = (uint32_t)((const int32_t*)T.v[k])[i]; break;
          case TK_U8: x = ((const uint8_t*)T.v[k])[i]; break;
          default: x = (((const uint8_t*)T.v[k])[i >> 3] >> (i & 7)) & 1u; break;
        }
      } else {
        flags |= 1ull << k;
      }
    }
    w[k] = x;
  }
  w[TW - 1] = flags;
}

__device__ __forceinline__ uint64_t tuple_hash(const uint64_t (&w)[TW]) {
  uint64_t h = 0x9E3779B97F4A7C15ull;
#pragma unroll
  for (int k = 0; k < TW; ++k) h = fmix64(h ^ w[k]) + 0x165667B19E3779F9ull;
  h = fmix64(h);
  return h ? h : 1;
}

__device__ __forceinline__ bool tuple_eq(const DictDev& D, int c, const uint64_t (&w)[TW]) {
  const uint64_t* t = (const uint64_t*)(D.arena + D.code_off[c]);
  bool eq = true;
#pragma unroll
  for (int k = 0; k < TW; ++k) eq &= t[k] == w[k];
  return eq;
}

__device__ __forceinline__ void tuple_put(uint8_t* dst, const uint64_t (&w)[TW]) {
#pragma unroll
  for (int k = 0; k < TW; ++k) ((uint64_t*)dst)[k] = w[k];
}

__device__ int tuple_find_or_insert(const DictDev& D, const uint64_t (&w)[TW], uint64_t h) {
  uint64_t slot = 0;
  const int r = dict_probe(D, h, [&](int c) { return tuple_eq(D, c, w); }, &slot);
  if (r != R_CLAIMED) return r;
  return dict_insert_one(D, slot, h, 8 * TW, [&](uint8_t* dst) { tuple_put(dst, w); });
}

__global__ void __launch_bounds__(ENC_THREADS) k_tuple_encode(DictDev D, TupleCols T, int64_t n,
                                                              int32_t* __restrict__ codes,
                                                              uint32_t* __restrict__ retry) {
  __shared__ LdsCache C;
  __shared__ int wg_full;  // a lane of this workgroup saw the dictionary full: the batch reruns
  for (int k = threadIdx.x; k < LC_SLOTS; k += blockDim.x) C.state[k] = 0;
  if (threadIdx.x == 0) wg_full = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t start = blockIdx.x * (int64_t)blockDim.x + threadIdx.x - lane;
  for (int64_t i0 = start; i0 < n; i0 += stride) {
    if (*(volatile int*)&wg_full) break;  // uniform per wave (LDS)
    const int64_t i = i0 + lane;
    const bool live = i < n;
    uint64_t w[TW] = {0, 0, 0, 0, 0};
    uint64_t h = 0;
    int c = -1;
    if (live) {
      tuple_words(T, i, w);
      h = tuple_hash(w);
      c = lc_find(C, h, 8 * TW, w);
    }
    const bool miss = live && c < 0;
    if (__ballot(miss)) {
      const int leader = wave_leader(miss, true, h, 8 * TW, w, lane);
      const bool lead = miss && leader == lane;
      int code = 0;
      uint64_t gslot = 0;
      if (lead) code = dict_probe(D, h, [&](int cc) { return tuple_eq(D, cc, w); }, &gslot);
      const bool claim = lead && code == R_CLAIMED;
      const int pc = dict_insert_wave(D, claim, gslot, h, 8 * TW, [&](uint8_t* dst) { tuple_put(dst, w); }, lane);
      if (claim) code = pc;
      if (lead && code >= 0) lc_insert(C, h, 8 * TW, w, code);
      code = __shfl(code, leader);
      if (miss) c = code;
    }
    if (live) {
      codes[i] = c >= 0 ? c : 0;
      if (c == R_OVERFLOW) wg_full = 1;
      if (c == R_RETRY) {
        atomicOr(&retry[i >> 5], 1u << (i & 31));
        atomicAdd(&D.flags[1], 1u);
      }
    }
  }
}

__global__ void __launch_bounds__(ENC_THREADS) k_tuple_encode_retry(DictDev D, TupleCols T, int64_t n,
                                                                    int32_t* __restrict__ codes,
                                                                    const uint32_t* __restrict__ retry_in,
                                                                    uint32_t* __restrict__ retry_out) {
  const int64_t words = (n + 31) >> 5;
  for (int64_t wd = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; wd < words; wd += (int64_t)gridDim.x * blockDim.x) {
    uint32_t bits = retry_in[wd];
    while (bits) {
      const int j = __builtin_ctz(bits);
      bits &= bits - 1;
      const int64_t i = (wd << 5) + j;
      uint64_t w[TW];
      tuple_words(T, i, w);
      const int c = tuple_find_or_insert(D, w, tuple_hash(w));
      codes[i] = c >= 0 ? c : 0;
      if (c == R_RETRY) {
        atomicOr(&retry_out[i >> 5], 1u << (i & 31));
        atomicAdd(&D.flags[1], 1u);
      }
    }
  }
}

struct TupleOut {
  void* v[QE_MAX_KEYS];
  uint8_t* valid[QE_MAX_KEYS];  // byte-addressed; 8 rows per thread own one byte each
  int32_t kind[QE_MAX_KEYS];
  int32_t nkeys;
};

__global__ void k_tuple_decode(const int32_t* __restrict__ codes, int64_t n, int64_t ncodes,
                               const int64_t* __restrict__ code_off, const uint8_t* __restrict__ arena, TupleOut O,
                               unsigned int* __restrict__ bad) {
  const int64_t groups = (n + 7) >> 3;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < groups; g += (int64_t)gridDim.x * blockDim.x) {
    uint8_t vb[QE_MAX_KEYS] = {0, 0, 0, 0};
    uint8_t bb[QE_MAX_KEYS] = {0, 0, 0, 0};
    for (int j = 0; j < 8; ++j) {
      const int64_t i = (g << 3) + j;
      if (i >= n) break;
      const int32_t c = codes[i];
      if (c < 0 || c >= ncodes) {
        atomicOr(bad, 1u);
        continue;
      }
      const uint64_t* t = (const uint64_t*)(arena + code_off[c]);
      const uint64_t flags = t[TW - 1];
#pragma unroll
      for (int k = 0; k < QE_MAX_KEYS; ++k) {
        if (k >= O.nkeys) break;
        const uint64_t x = t[k];
        if (!((flags >> k) & 1)) vb[k] |= (uint8_t)(1u << j);
        switch (O.kind[k]) {
          case TK_I64:
          case TK_F64: ((uint64_t*)O.v[k])[i] = x; break;
          case TK_I32: ((uint32_t*)O.v[k])[i] = (uint32_t)x; break;
          case TK_U8: ((uint8_t*)O.v[k])[i] = (uint8_t)x; break;
          default: bb[k] |= (uint8_t)((x & 1u) << j); break;
        }
      }
    }
    for (int k = 0; k < O.nkeys; ++k) {
      if (O.valid[k]) O.valid[k][g] = vb[k];
      if (O.kind[k] == TK_BOOL) ((uint8_t*)O.v[k])[g] = bb[k];
    }
  }
}

// ---- content-hash partitioning of rows (exchange of dictionary-keyed partials) -------------------
struct HashCols {
  const void* v[QE_MAX_KEYS];
  const uint8_t* valid[QE_MAX_KEYS];
  const int32_t* offs[QE_MAX_KEYS];  // UTF8
  int32_t kind[QE_MAX_KEYS];         // TK_* or 5 = UTF8
  int32_t ncols;
};
constexpr int32_t TK_UTF8 = 5;

__global__ void k_hash_partition(HashCols H, int64_t n, int32_t nparts, int32_t* __restrict__ part) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t h = 0x2545F4914F6CDD1Dull;
    for (int k = 0; k < H.ncols; ++k) {
      uint64_t x;
      const bool ok = !H.valid[k] || ((H.valid[k][i >> 3] >> (i & 7)) & 1);
      if (!ok) {
        x = 0x6A09E667F3BCC909ull;  // null member
      } else {
        switch (H.kind[k]) {
          case TK_UTF8: {
            const int32_t s0 = H.offs[k][i];
            x = str_hash((const uint8_t*)H.v[k] + s0, H.offs[k][i + 1] - s0);
            break;
          }
          case TK_F64: {
            x = ((const uint64_t*)H.v[k])[i];
            const double d = bits_f64((int64_t)x);
            if (d != d) x = 0x7FF8000000000000ull;  // Double.equals: every NaN is one key
            break;
          }
          case TK_I64: x = ((const uint64_t*)H.v[k])[i]; break;
          case TK_I32: x = (uint32_t)((const int32_t*)H.v[k])[i]; break;
          case TK_U8: x = ((const uint8_t*)H.v[k])[i]; break;
          default: x = (((const uint8_t*)H.v[k])[i >> 3] >> (i & 7)) & 1u; break;
        }
      }
      h = fmix64(h ^ x) + 0x165667B19E3779F9ull * (uint64_t)(k + 1);
    }
    h = fmix64(h);
    part[i] = (int32_t)(((h >> 32) * (uint64_t)nparts) >> 32);
  }
}

__global__ void k_dict_rebuild(DictDev D, int64_t ncodes) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < ncodes; c += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t h = D.code_hash[c];
    uint64_t slot = h & D.mask;
    for (;;) {
      if (atomicCAS((unsigned long long*)&D.s_hash[slot], 0ull, (unsigned long long)h) == 0) {
        D.s_code[slot] = (int32_t)c;
        break;
      }
      slot = (slot + 1) & D.mask;
    }
  }
}

// Code i of a codes column: int32 (WIDE false) or a wide int64 code; *len its key's length, *c its
// dictionary code (-1: packed in the wide code itself), false if out of range.
template <bool WIDE>
__device__ __forceinline__ bool code_at(const void* codes, int64_t i, const int32_t* code_len, int64_t ncodes,
                                        int64_t* len, int64_t* c, uint64_t* packed) {
  if (WIDE) {
    const uint64_t x = (uint64_t)((const int64_t*)codes)[i];
    if (!(x & WIDE_DICT)) {
      *len = (int64_t)((x >> 56) & 0xFF);
      *c = -1;
      *packed = x;
      return (x >> 59) == 0 && *len <= WIDE_MAX;
    }
    const uint64_t d = x & ~WIDE_DICT;
    if (d >= (uint64_t)ncodes) return false;
    *c = (int64_t)d;
  } else {
    const int32_t d = ((const int32_t*)codes)[i];
    if (d < 0 || d >= ncodes) return false;
    *c = d;
  }
  *len = code_len[*c];
  return true;
}

template <bool WIDE>
__global__ void k_dict_decode_len(const void* __restrict__ codes, const uint8_t* __restrict__ valid, int64_t n,
                                  const int32_t* __restrict__ code_len, int64_t ncodes, int64_t* __restrict__ lens,
                                  unsigned int* __restrict__ bad) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t l = 0;
    if (!valid || ((valid[i >> 3] >> (i & 7)) & 1)) {
      int64_t c;
      uint64_t packed;
      if (!code_at<WIDE>(codes, i, code_len, ncodes, &l, &c, &packed)) {
        atomicOr(bad, 1u);
        l = 0;
      }
    }
    lens[i] = l;
  }
}

template <bool WIDE>
__global__ void k_dict_decode_copy(const void* __restrict__ codes, const uint8_t* __restrict__ valid, int64_t n,
                                   const int64_t* __restrict__ code_off, const int32_t* __restrict__ code_len,
                                   int64_t ncodes, const uint8_t* __restrict__ arena, const int64_t* __restrict__ starts,
                                   int32_t* __restrict__ out_offs, uint8_t* __restrict__ out_bytes) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= n; i += (int64_t)gridDim.x * blockDim.x) {
    out_offs[i] = (int32_t)starts[i];
    if (i == n) continue;
    if (valid && !((valid[i >> 3] >> (i & 7)) & 1)) continue;
    int64_t l, c;
    uint64_t packed = 0;
    if (!code_at<WIDE>(codes, i, code_len, ncodes, &l, &c, &packed)) continue;  // (reported by decode_len)
    uint8_t* dst = out_bytes + starts[i];
    if (c < 0) {
      for (int k = 0; k < l; ++k) dst[k] = (uint8_t)(packed >> (8 * k));
    } else {
      const uint8_t* src = arena + code_off[c];
      for (int64_t k = 0; k < l; ++k) dst[k] = src[k];
    }
  }
}

// Wide codes of UTF8 values all known to be at most WIDE_MAX bytes (qe_strdict_encode_packed): the
// code is the value itself, no dictionary — a streaming pass (offsets, up to 8 key bytes, one code
// per row), and no control-block read-back: the caller's next kernel can follow on the stream.
__global__ void __launch_bounds__(256) k_pack_codes(const int32_t* __restrict__ offs, const uint8_t* __restrict__ bytes,
                                                    const uint8_t* __restrict__ valid, int64_t n,
                                                    int64_t* __restrict__ codes64,
                                                    unsigned long long* __restrict__ err) {
  bool too_long = false;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const bool live = !valid || ((valid[i >> 3] >> (i & 7)) & 1);
    int64_t c = 0;
    if (live) {
      const int32_t s0 = offs[i];
      const int32_t full = offs[i + 1] - s0;
      const int len = min(full, WIDE_MAX);
      too_long |= full > WIDE_MAX;
      c = wide_pack(load_u64_unaligned(bytes + s0, len), len);
    }
    codes64[i] = c;
  }
  // the caller's length bound was wrong: flag it (one atomic per wave that saw such a value)
  const unsigned long long b = __ballot(too_long);
  if (err && b && (int)(threadIdx.x & 63) == __ffsll((long long)b) - 1) atomicOr(err, (unsigned long long)CTL_KEY_TOO_LONG);
}

// Decode of packed wide codes in one 1024-thread block (small results: a finalize's groups): the
// lengths, their prefixes (tile by tile) and the bytes, where the general decode runs a length
// pass, a device scan and a copy pass.
__global__ void __launch_bounds__(1024) k_unpack_codes_small(const int64_t* __restrict__ codes,
                                                             const uint8_t* __restrict__ valid, int64_t n,
                                                             int32_t* __restrict__ out_offs, uint8_t* __restrict__ out) {
  __shared__ int32_t ws[16];
  int32_t carry = 0;
  for (int64_t g0 = 0; g0 < n; g0 += 8192) {
    int32_t v[8], ex[8];
    uint64_t x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t e = tile_elem(g0, k);
      const bool live = e < n && (!valid || ((valid[e >> 3] >> (e & 7)) & 1));
      x[k] = live ? (uint64_t)codes[e] : 0ull;
      v[k] = (int32_t)((x[k] >> 56) & 7);
    }
    const int32_t t = tile_excl(v, ex, ws);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t e = tile_elem(g0, k);
      if (e >= n) continue;
      const int32_t o = carry + ex[k];
      out_offs[e] = o;
      for (int b = 0; b < v[k]; ++b) out[o + b] = (uint8_t)(x[k] >> (8 * b));
    }
    carry += t;
  }
  if (threadIdx.x == 0) out_offs[n] = carry;
}

}  // namespace

}  // namespace qe

using namespace qe;

struct qe_strdict {
  qe_ctx* ctx = nullptr;
  uint64_t cap = 0;  // slots (power of two)
  int64_t ccap = 0, acap = 0;
  uint64_t* s_hash = nullptr;
  int32_t* s_code = nullptr;
  int64_t* code_off = nullptr;
  int32_t* code_len = nullptr;
  uint64_t* code_hash = nullptr;
  uint8_t* arena = nullptr;
  // ctl: ncodes (u32) | pad | arena_used (u64) | flags[2] (u32)
  uint8_t* ctl = nullptr;
  int64_t ncodes = 0;
  int64_t arena_used = 0;
  int32_t mode = 0;  // 0 unused, 1 strings, 2 key tuples (kinds below)
  // the last qe_strdict_decode_bytes: its string starts stay in ctx scratch until the next
  // ctx_scratch call, so a qe_strdict_decode of the same codes right after reuses them
  const void* dec_codes = nullptr;
  const uint8_t* dec_valid = nullptr;
  int64_t dec_n = -1, dec_total = 0;
  uint64_t dec_epoch = 0;
  int32_t tuple_nkeys = 0;
  int32_t tuple_type[QE_MAX_KEYS] = {0, 0, 0, 0};

  unsigned int* d_ncodes() { return (unsigned int*)ctl; }
  unsigned long long* d_arena_used() { return (unsigned long long*)(ctl + 8); }
  unsigned int* d_flags() { return (unsigned int*)(ctl + 16); }
  DictDev dev() {
    return DictDev{s_hash, s_code, cap - 1, code_off, code_len, code_hash, ccap, arena, acap,
                   d_ncodes(), d_arena_used(), d_flags()};
  }
};

namespace {

int dict_free(qe_strdict* d) {
  void* ptrs[] = {d->s_hash, d->s_code, d->code_off, d->code_len, d->code_hash, d->arena, d->ctl};
  for (void* p : ptrs) dev_free(d->ctx, p);
  return QE_OK;
}

int grow_slots(qe_strdict* d, uint64_t cap) {
  qe_ctx* ctx = d->ctx;
  dev_free(ctx, d->s_hash);
  dev_free(ctx, d->s_code);
  d->s_hash = nullptr;
  d->s_code = nullptr;
  QE_TRY(dev_alloc(ctx, cap * 8, (void**)&d->s_hash));
  QE_TRY(dev_alloc(ctx, cap * 4, (void**)&d->s_code));
  d->cap = cap;
  QE_HIP(hipMemsetAsync(d->s_hash, 0, cap * 8, ctx->stream));
  QE_HIP(hipMemsetAsync(d->s_code, 0xFF, cap * 4, ctx->stream));
  if (d->ncodes > 0) {
    const int grid = (int)std::min<int64_t>((int64_t)div_up((uint64_t)d->ncodes, 256), (int64_t)ctx->num_cus * 8);
    hipLaunchKernelGGL(k_dict_rebuild, dim3(grid), dim3(256), 0, ctx->stream, d->dev(), d->ncodes);
    QE_TRY(launch_check("k_dict_rebuild"));
  }
  return QE_OK;
}

template <typename T>
int grow_array(qe_ctx* ctx, T** p, int64_t old_n, int64_t new_n) {
  T* q = nullptr;
  QE_TRY(dev_alloc(ctx, (size_t)new_n * sizeof(T), (void**)&q));
  if (*p) {
    if (old_n > 0) QE_HIP(hipMemcpyAsync(q, *p, (size_t)old_n * sizeof(T), hipMemcpyDeviceToDevice, ctx->stream));
    dev_free(ctx, *p);
  }
  *p = q;
  return QE_OK;
}

// Reads the control block back; returns the flags.
int read_ctl(qe_strdict* d, uint32_t* overflow, uint32_t* unresolved) {
  uint8_t h[24];
  QE_HIP(hipMemcpyAsync(h, d->ctl, 24, hipMemcpyDeviceToHost, d->ctx->stream));
  QE_TRY(ctx_sync(d->ctx));
  uint32_t nc;
  uint64_t au;
  memcpy(&nc, h, 4);
  memcpy(&au, h + 8, 8);
  memcpy(overflow, h + 16, 4);
  memcpy(unresolved, h + 20, 4);
  d->ncodes = std::min<int64_t>((int64_t)nc, d->ccap);  // codes >= ccap were never published
  d->arena_used = (int64_t)au;
  return QE_OK;
}

int write_ctl(qe_strdict* d) {
  uint8_t h[24] = {0};
  const uint32_t nc = (uint32_t)d->ncodes;
  const uint64_t au = (uint64_t)d->arena_used;
  memcpy(h, &nc, 4);
  memcpy(h + 8, &au, 8);
  QE_HIP(hipMemcpyAsync(d->ctl, h, 24, hipMemcpyHostToDevice, d->ctx->stream));
  QE_TRY(ctx_sync(d->ctx));
  return QE_OK;
}

}  // namespace

extern "C" {

int qe_strdict_create(qe_ctx* ctx, int64_t expected_distinct, qe_strdict** out) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(out, QE_ERR_INVALID_ARG, "null argument");
  *out = nullptr;
  qe_strdict* d = new qe_strdict();
  d->ctx = ctx;
  int64_t cc = 1024;
  while (cc < expected_distinct && cc < (1ll << 30)) cc <<= 1;
  d->ccap = cc;
  d->acap = std::max<int64_t>(1 << 16, cc * 16);
  int st = QE_OK;
  if ((st = grow_array(ctx, &d->code_off, 0, d->ccap)) != QE_OK || (st = grow_array(ctx, &d->code_len, 0, d->ccap)) ||
      (st = grow_array(ctx, &d->code_hash, 0, d->ccap)) || (st = grow_array(ctx, &d->arena, 0, d->acap)) ||
      (st = grow_array(ctx, &d->ctl, 0, 24)) || (st = grow_slots(d, (uint64_t)d->ccap * 2))) {
    dict_free(d);
    delete d;
    return st;
  }
  if (hipMemsetAsync(d->ctl, 0, 24, ctx->stream) != hipSuccess) {  // ncodes, arena_used, flags = 0: no host copy
    dict_free(d);
    delete d;
    return fail(QE_ERR_DEVICE, "strdict control block init failed");
  }
  *out = d;
  return QE_OK;
}

int qe_strdict_destroy(qe_strdict* d) {
  if (!d) return QE_OK;
  (void)hipSetDevice(d->ctx->device);
  dict_free(d);
  delete d;
  return QE_OK;
}

int qe_strdict_size(qe_strdict* d, int64_t* n) {
  QE_CHECK(d && n, QE_ERR_INVALID_ARG, "null argument");
  *n = d->ncodes;
  return QE_OK;
}

}  // extern "C"

namespace {

// Bytes spanned by a UTF8 column's values (offsets[n] - offsets[0]; one read-back on the ctx stream).
int column_span(qe_ctx* ctx, const qe_column* in, int64_t* out) {
  void* pin;
  QE_TRY(ctx_pinned(ctx, 8, &pin));
  QE_HIP(hipMemcpyAsync(pin, in->offsets + in->length, 4, hipMemcpyDeviceToHost, ctx->stream));
  QE_HIP(hipMemcpyAsync((int32_t*)pin + 1, in->offsets, 4, hipMemcpyDeviceToHost, ctx->stream));
  QE_TRY(ctx_sync(ctx));
  int32_t o[2];
  memcpy(o, pin, 8);
  *out = (int64_t)o[0] - o[1];
  return QE_OK;
}

// Pass 1 over all rows, retry passes until every row resolved; on overflow grow the code arrays /
// arena, rebuild the slots and run the batch again (re-encoding is idempotent).
template <typename Pass1, typename Retry>
int encode_loop(qe_strdict* d, int64_t n, int64_t batch_bytes, Pass1 pass1, Retry retry_pass,
                const qe_column* span_col = nullptr) {
  // batch_bytes < 0: the bytes of UTF8 column `span_col`, read back only if the arena has to grow
  // (the common batch skips that host round trip)
  qe_ctx* ctx = d->ctx;
  const int64_t words = (int64_t)div_up((uint64_t)n, 32);
  void* s;
  QE_TRY(ctx_scratch(ctx, (size_t)words * 8, &s));
  uint32_t* retry[2] = {(uint32_t*)s, (uint32_t*)s + words};
  for (int attempt = 0; attempt < 64; ++attempt) {
    QE_HIP(hipMemsetAsync(retry[0], 0, (size_t)words * 4, ctx->stream));
    QE_HIP(hipMemsetAsync(d->d_flags(), 0, 8, ctx->stream));
    QE_TRY(pass1(retry[0]));
    uint32_t ovf = 0, unres = 0;
    QE_TRY(read_ctl(d, &ovf, &unres));
    int cur = 0;
    for (int pass = 0; pass < 64 && unres && !ovf; ++pass) {
      QE_HIP(hipMemsetAsync(retry[1 - cur], 0, (size_t)words * 4, ctx->stream));
      QE_HIP(hipMemsetAsync(d->d_flags() + 1, 0, 4, ctx->stream));
      QE_TRY(retry_pass(retry[cur], retry[1 - cur], words));
      QE_TRY(read_ctl(d, &ovf, &unres));
      cur = 1 - cur;
    }
    if (!ovf && !unres) return QE_OK;
    // grow: codes x4 (slots follow), arena to twice what is in use plus this batch's bytes
    // distinct keys <= codes so far + this batch's rows: grow 16x, never past that bound
    int64_t bound = 1024;
    while (bound < d->ncodes + n && bound < (1ll << 31)) bound <<= 1;
    const int64_t new_ccap = d->ncodes * 2 >= d->ccap ? std::max(d->ccap, std::min(d->ccap * 16, bound)) : d->ccap;
    const int64_t used = std::min<int64_t>(d->arena_used, d->acap);
    if (batch_bytes < 0 && d->arena_used + 64 > d->acap) QE_TRY(column_span(ctx, span_col, &batch_bytes));
    const int64_t new_acap = d->arena_used + 64 > d->acap ? std::max<int64_t>(d->acap * 2, used * 2 + batch_bytes)
                                                           : d->acap;
    QE_CHECK(new_ccap <= (1ll << 31), QE_ERR_CAPACITY, "more than 2^31 distinct keys");
    if (new_ccap != d->ccap) {
      QE_TRY(grow_array(ctx, &d->code_off, d->ncodes, new_ccap));
      QE_TRY(grow_array(ctx, &d->code_len, d->ncodes, new_ccap));
      QE_TRY(grow_array(ctx, &d->code_hash, d->ncodes, new_ccap));
      d->ccap = new_ccap;
    }
    if (new_acap != d->acap) {
      QE_TRY(grow_array(ctx, &d->arena, used, new_acap));
      d->acap = new_acap;
    }
    if (d->arena_used > d->acap) d->arena_used = used;  // drop reservations past the old end
    if (d->mode == 2) d->arena_used = (d->arena_used + 7) & ~7ll;  // tuples stay 8-byte aligned
    QE_TRY(write_ctl(d));
    QE_TRY(grow_slots(d, (uint64_t)d->ccap * 2));  // also clears failed (-2) slots
  }
  return fail(QE_ERR_DEVICE, "key dictionary did not converge");
}

int32_t tuple_kind(int32_t type) {
  switch (type) {
    case QE_TYPE_INT64: return TK_I64;
    case QE_TYPE_FLOAT64: return TK_F64;
    case QE_TYPE_INT32:
    case QE_TYPE_DATE32: return TK_I32;
    case QE_TYPE_UINT8: return TK_U8;
    case QE_TYPE_BOOL: return TK_BOOL;
    default: return -1;
  }
}

}  // namespace

extern "C" {

int qe_strdict_encode(qe_strdict* d, const qe_column* in, qe_column* codes) {
  QE_CHECK(d && in && codes, QE_ERR_INVALID_ARG, "null argument");
  qe_ctx* ctx = d->ctx;
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(in->type == QE_TYPE_UTF8 && in->offsets, QE_ERR_UNSUPPORTED, "string dictionary input must be UTF8");
  QE_CHECK(d->mode != 2, QE_ERR_INVALID_ARG, "dictionary holds key tuples, not strings");
  QE_CHECK(codes->type == QE_TYPE_INT32 || codes->type == QE_TYPE_INT64, QE_ERR_INVALID_ARG,
           "codes column must be INT32 (dictionary codes) or INT64 (wide codes)");
  const bool wide = codes->type == QE_TYPE_INT64;
  int32_t* c32 = wide ? nullptr : (int32_t*)codes->values;
  int64_t* c64 = wide ? (int64_t*)codes->values : nullptr;
  const int64_t n = in->length;
  QE_CHECK(codes->length >= n && (codes->values || n == 0), QE_ERR_CAPACITY, "codes column too small");
  QE_CHECK(!in->validity || codes->validity, QE_ERR_INVALID_ARG, "codes validity buffer required");
  d->mode = 1;
  codes->length = n;
  if (n == 0) return QE_OK;
  if (in->validity)
    QE_HIP(hipMemcpyAsync(codes->validity, in->validity, (size_t)div_up((uint64_t)n, 8), hipMemcpyDeviceToDevice,
                          ctx->stream));  // an input bitmap may be Arrow-minimal: ceil(n/8) bytes
  // one 1024-thread workgroup per CU: every workgroup warms its LDS cache once, so few, long-lived
  // workgroups send few lookups of the hot keys to the global table
  const int grid = (int)std::min<int64_t>((int64_t)div_up((uint64_t)n, 4 * ENC_BLOCK), (int64_t)ctx->num_cus);
  return encode_loop(
      d, n, -1,
      [&](uint32_t* retry) {
        if (wide)
          hipLaunchKernelGGL(k_dict_encode<true>, dim3(grid), dim3(ENC_BLOCK), 0, ctx->stream, d->dev(), in->offsets,
                             (const uint8_t*)in->values, in->validity, n, c32, c64, retry);
        else
          hipLaunchKernelGGL(k_dict_encode<false>, dim3(grid), dim3(ENC_BLOCK), 0, ctx->stream, d->dev(), in->offsets,
                             (const uint8_t*)in->values, in->validity, n, c32, c64, retry);
        return launch_check("k_dict_encode");
      },
      [&](const uint32_t* rin, uint32_t* rout, int64_t words) {
        const int g2 = (int)std::min<int64_t>((int64_t)div_up((uint64_t)words, 256), (int64_t)ctx->num_cus * 4);
        hipLaunchKernelGGL(k_dict_encode_retry, dim3(g2), dim3(256), 0, ctx->stream, d->dev(), in->offsets,
                           (const uint8_t*)in->values, n, c32, c64, rin, rout);
        return launch_check("k_dict_encode_retry");
      },
      in);
}

int qe_strdict_encode_tuple(qe_strdict* d, const qe_column* keys, int32_t nkeys, qe_column* codes) {
  QE_CHECK(d && keys && codes, QE_ERR_INVALID_ARG, "null argument");
  qe_ctx* ctx = d->ctx;
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(nkeys >= 1 && nkeys <= QE_MAX_KEYS, QE_ERR_UNSUPPORTED, "key tuples take 1..%d columns", QE_MAX_KEYS);
  QE_CHECK(d->mode != 1, QE_ERR_INVALID_ARG, "dictionary holds strings, not key tuples");
  QE_CHECK(codes->type == QE_TYPE_INT32, QE_ERR_INVALID_ARG, "codes column must be INT32");
  const int64_t n = keys[0].length;
  TupleCols T{};
  T.nkeys = nkeys;
  for (int k = 0; k < nkeys; ++k) {
    QE_CHECK(keys[k].length == n, QE_ERR_INVALID_ARG, "key %d has %lld rows, key 0 %lld", k,
             (long long)keys[k].length, (long long)n);
    const int32_t kind = tuple_kind(keys[k].type);
    QE_CHECK(kind >= 0, QE_ERR_UNSUPPORTED, "key %d: type %d cannot be part of a key tuple (encode UTF8 first)", k,
             keys[k].type);
    QE_CHECK(keys[k].values || n == 0, QE_ERR_INVALID_ARG, "key %d: null values", k);
    if (d->mode == 2)
      QE_CHECK(d->tuple_nkeys == nkeys && d->tuple_type[k] == keys[k].type, QE_ERR_INVALID_ARG,
               "key %d: type %d differs from the dictionary's tuple layout", k, keys[k].type);
    T.v[k] = keys[k].values;
    T.valid[k] = keys[k].validity;
    T.kind[k] = kind;
  }
  QE_CHECK(codes->length >= n && (codes->values || n == 0), QE_ERR_CAPACITY, "codes column too small");
  if (d->mode == 0) {
    d->mode = 2;
    d->tuple_nkeys = nkeys;
    for (int k = 0; k < nkeys; ++k) d->tuple_type[k] = keys[k].type;
  }
  codes->length = n;
  if (n == 0) return QE_OK;
  if (codes->validity)  // a tuple with null members is still a (non-null) group key
    QE_HIP(hipMemsetAsync(codes->validity, 0xFF, (size_t)div_up((uint64_t)n, 32) * 4, ctx->stream));
  const int grid = (int)std::min<int64_t>((int64_t)div_up((uint64_t)n, 4 * ENC_BLOCK), (int64_t)ctx->num_cus);
  return encode_loop(
      d, n, 8 * TW * std::min<int64_t>(n, 1 << 20),
      [&](uint32_t* retry) {
        hipLaunchKernelGGL(k_tuple_encode, dim3(grid), dim3(ENC_THREADS), 0, ctx->stream, d->dev(), T, n,
                           (int32_t*)codes->values, retry);
        return launch_check("k_tuple_encode");
      },
      [&](const uint32_t* rin, uint32_t* rout, int64_t words) {
        const int g2 = (int)std::min<int64_t>((int64_t)div_up((uint64_t)words, 256), (int64_t)ctx->num_cus * 4);
        hipLaunchKernelGGL(k_tuple_encode_retry, dim3(g2), dim3(256), 0, ctx->stream, d->dev(), T, n,
                           (int32_t*)codes->values, rin, rout);
        return launch_check("k_tuple_encode_retry");
      });
}

int qe_hash_partition(qe_ctx* ctx, const qe_column* cols, int32_t ncols, int32_t nparts, int32_t* part) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(cols && part && ncols >= 1 && ncols <= QE_MAX_KEYS, QE_ERR_INVALID_ARG, "1..%d key columns", QE_MAX_KEYS);
  QE_CHECK(nparts >= 1, QE_ERR_INVALID_ARG, "nparts must be >= 1");
  const int64_t n = cols[0].length;
  HashCols H{};
  H.ncols = ncols;
  for (int k = 0; k < ncols; ++k) {
    QE_CHECK(cols[k].length == n, QE_ERR_INVALID_ARG, "column %d length differs", k);
    const int32_t kind = cols[k].type == QE_TYPE_UTF8 ? TK_UTF8 : tuple_kind(cols[k].type);
    QE_CHECK(kind >= 0, QE_ERR_UNSUPPORTED, "column %d: type %d cannot be hashed", k, cols[k].type);
    QE_CHECK(kind != TK_UTF8 || cols[k].offsets, QE_ERR_INVALID_ARG, "UTF8 column %d without offsets", k);
    H.v[k] = cols[k].values;
    H.valid[k] = cols[k].validity;
    H.offs[k] = cols[k].offsets;
    H.kind[k] = kind;
  }
  if (n == 0) return QE_OK;
  const int grid = (int)std::min<int64_t>((int64_t)div_up((uint64_t)n, 256), (int64_t)ctx->num_cus * 8);
  hipLaunchKernelGGL(k_hash_partition, dim3(grid), dim3(256), 0, ctx->stream, H, n, nparts, part);
  return launch_check("k_hash_partition");
}

int qe_strdict_decode_tuple(qe_strdict* d, const qe_column* codes, int32_t nkeys, qe_column* outs) {
  QE_CHECK(d && codes && outs, QE_ERR_INVALID_ARG, "null argument");
  qe_ctx* ctx = d->ctx;
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(d->mode == 2 && d->tuple_nkeys == nkeys, QE_ERR_INVALID_ARG, "dictionary does not hold %d-key tuples",
           nkeys);
  QE_CHECK(codes->type == QE_TYPE_INT32, QE_ERR_INVALID_ARG, "codes column must be INT32");
  const int64_t n = codes->length;
  TupleOut O{};
  O.nkeys = nkeys;
  for (int k = 0; k < nkeys; ++k) {
    QE_CHECK(outs[k].type == d->tuple_type[k], QE_ERR_INVALID_ARG, "output %d: type %d, tuple holds %d", k,
             outs[k].type, d->tuple_type[k]);
    QE_CHECK(outs[k].length >= n && (outs[k].values || n == 0), QE_ERR_CAPACITY, "output %d too small", k);
    O.v[k] = outs[k].values;
    O.valid[k] = outs[k].validity;
    O.kind[k] = tuple_kind(outs[k].type);
    outs[k].length = n;
  }
  if (n == 0) return QE_OK;
  void* s;
  QE_TRY(ctx_scratch(ctx, 8, &s));
  QE_HIP(hipMemsetAsync(s, 0, 4, ctx->stream));
  const int grid = (int)std::min<int64_t>((int64_t)div_up(div_up((uint64_t)n, 8), 256), (int64_t)ctx->num_cus * 8);
  hipLaunchKernelGGL(k_tuple_decode, dim3(grid), dim3(256), 0, ctx->stream, (const int32_t*)codes->values, n,
                     d->ncodes, d->code_off, d->arena, O, (unsigned int*)s);
  QE_TRY(launch_check("k_tuple_decode"));
  uint32_t bad = 0;
  QE_HIP(hipMemcpyAsync(&bad, s, 4, hipMemcpyDeviceToHost, ctx->stream));
  QE_TRY(ctx_sync(ctx));
  QE_CHECK(bad == 0, QE_ERR_INVALID_ARG, "code out of range for this dictionary");
  return QE_OK;
}

int qe_strdict_decode_bytes(qe_strdict* d, const qe_column* codes, int64_t* out_bytes) {
  QE_CHECK(d && codes && out_bytes, QE_ERR_INVALID_ARG, "null argument");
  qe_ctx* ctx = d->ctx;
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(codes->type == QE_TYPE_INT32 || codes->type == QE_TYPE_INT64, QE_ERR_INVALID_ARG,
           "codes column must be INT32 or INT64 (wide codes)");
  const int64_t n = codes->length;
  *out_bytes = 0;
  if (n == 0) return QE_OK;
  void* s;
  QE_TRY(ctx_scratch(ctx, (size_t)(2 * n + 2) * 8, &s));
  int64_t* lens = (int64_t*)s;
  int64_t* starts = lens + n;
  unsigned int* bad = (unsigned int*)(starts + n + 1);
  QE_HIP(hipMemsetAsync(bad, 0, 4, ctx->stream));
  const int grid = (int)std::min<int64_t>((int64_t)div_up((uint64_t)n, 256), (int64_t)ctx->num_cus * 8);
  if (codes->type == QE_TYPE_INT64)
    hipLaunchKernelGGL(k_dict_decode_len<true>, dim3(grid), dim3(256), 0, ctx->stream, codes->values, codes->validity,
                       n, d->code_len, d->ncodes, lens, bad);
  else
    hipLaunchKernelGGL(k_dict_decode_len<false>, dim3(grid), dim3(256), 0, ctx->stream, codes->values,
                       codes->validity, n, d->code_len, d->ncodes, lens, bad);
  QE_TRY(launch_check("k_dict_decode_len"));
  QE_TRY(exclusive_scan_i64(ctx, lens, starts, n));
  int64_t h[2] = {0, 0};
  QE_HIP(hipMemcpyAsync(h, starts + n, 8, hipMemcpyDeviceToHost, ctx->stream));
  QE_HIP(hipMemcpyAsync(h + 1, bad, 4, hipMemcpyDeviceToHost, ctx->stream));
  QE_TRY(ctx_sync(ctx));
  QE_CHECK((uint32_t)h[1] == 0, QE_ERR_INVALID_ARG, "code out of range for this dictionary");
  *out_bytes = h[0];
  d->dec_codes = codes->values;
  d->dec_valid = codes->validity;
  d->dec_n = n;
  d->dec_total = h[0];
  d->dec_epoch = ctx->scratch_epoch;
  return QE_OK;
}

static int strdict_decode(qe_strdict* d, const qe_column* codes, qe_column* out, bool trusted) {
  QE_CHECK(d && codes && out, QE_ERR_INVALID_ARG, "null argument");
  qe_ctx* ctx = d->ctx;
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(out->type == QE_TYPE_UTF8 && out->offsets, QE_ERR_INVALID_ARG, "output must be UTF8 with offsets");
  const int64_t n = codes->length;
  QE_CHECK(!codes->validity || out->validity, QE_ERR_INVALID_ARG, "output validity buffer required");
  int64_t total = 0;
  if (trusted && codes->type == QE_TYPE_INT64 && d->ncodes == 0 && n > 0 && n < (1ll << 28)) {
    // every code is packed (no long key was ever inserted): lengths and starts on the device, no
    // host round trip; the caller's values buffer holds WIDE_MAX bytes per row
    void* sp;
    QE_TRY(ctx_scratch(ctx, (size_t)(2 * n + 2) * 8, &sp));
    int64_t* lens = (int64_t*)sp;
    int64_t* starts = lens + n;
    unsigned int* bad = (unsigned int*)(starts + n + 1);
    const int g = (int)std::min<int64_t>((int64_t)div_up((uint64_t)n, 256), (int64_t)ctx->num_cus * 8);
    hipLaunchKernelGGL(k_dict_decode_len<true>, dim3(g), dim3(256), 0, ctx->stream, codes->values, codes->validity, n,
                       d->code_len, d->ncodes, lens, bad);
    QE_TRY(launch_check("k_dict_decode_len"));
    QE_TRY(exclusive_scan_i64(ctx, lens, starts, n));
    total = 0;
  } else if (d->dec_codes == codes->values && d->dec_valid == codes->validity && d->dec_n == n && n > 0 &&
      d->dec_epoch == ctx->scratch_epoch) {
    total = d->dec_total;  // qe_strdict_decode_bytes of these codes just ran: its starts are in scratch
  } else {
    QE_TRY(qe_strdict_decode_bytes(d, codes, &total));  // leaves starts in scratch
  }
  d->dec_codes = nullptr;
  QE_CHECK(total < (1ll << 31), QE_ERR_CAPACITY, "decoded strings exceed 2^31 bytes");
  out->length = n;
  if (n == 0) {
    QE_HIP(hipMemsetAsync(out->offsets, 0, 4, ctx->stream));
    return QE_OK;
  }
  QE_CHECK(out->values || (total == 0 && !trusted), QE_ERR_CAPACITY, "output values buffer required");
  const int64_t* starts = (const int64_t*)ctx->scratch + n;
  const int grid = (int)std::min<int64_t>((int64_t)div_up((uint64_t)n + 1, 256), (int64_t)ctx->num_cus * 8);
  if (codes->type == QE_TYPE_INT64)
    hipLaunchKernelGGL(k_dict_decode_copy<true>, dim3(grid), dim3(256), 0, ctx->stream, codes->values, codes->validity,
                       n, d->code_off, d->code_len, d->ncodes, d->arena, starts, out->offsets, (uint8_t*)out->values);
  else
    hipLaunchKernelGGL(k_dict_decode_copy<false>, dim3(grid), dim3(256), 0, ctx->stream, codes->values,
                       codes->validity, n, d->code_off, d->code_len, d->ncodes, d->arena, starts, out->offsets,
                       (uint8_t*)out->values);
  QE_TRY(launch_check("k_dict_decode_copy"));
  if (codes->validity)
    QE_HIP(hipMemcpyAsync(out->validity, codes->validity, (size_t)div_up((uint64_t)n, 8),
                          hipMemcpyDeviceToDevice, ctx->stream));
  return QE_OK;
}

int qe_strdict_decode(qe_strdict* d, const qe_column* codes, qe_column* out) {
  return strdict_decode(d, codes, out, false);
}

int qe_strdict_decode_trusted(qe_strdict* d, const qe_column* codes, qe_column* out) {
  return strdict_decode(d, codes, out, true);
}

int qe_strdict_encode_packed(qe_ctx* ctx, const qe_column* in, qe_column* codes) {
  QE_CHECK(ctx && in && codes, QE_ERR_INVALID_ARG, "null argument");
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(in->type == QE_TYPE_UTF8 && in->offsets, QE_ERR_UNSUPPORTED, "packed codes take a UTF8 column");
  QE_CHECK(codes->type == QE_TYPE_INT64, QE_ERR_INVALID_ARG, "packed codes are INT64 (wide codes)");
  const int64_t n = in->length;
  QE_CHECK(codes->length >= n && (codes->values || n == 0), QE_ERR_CAPACITY, "codes column too small");
  QE_CHECK(!in->validity || codes->validity, QE_ERR_INVALID_ARG, "codes validity buffer required");
  codes->length = n;
  if (n == 0) return QE_OK;
  if (in->validity)
    QE_HIP(hipMemcpyAsync(codes->validity, in->validity, (size_t)div_up((uint64_t)n, 8), hipMemcpyDeviceToDevice,
                          ctx->stream));
  const int grid = (int)std::min<int64_t>((int64_t)div_up((uint64_t)n, 256), (int64_t)ctx->num_cus * 8);
  hipLaunchKernelGGL(k_pack_codes, dim3(grid), dim3(256), 0, ctx->stream, in->offsets, (const uint8_t*)in->values,
                     in->validity, n, (int64_t*)codes->values, (unsigned long long*)nullptr);
  return launch_check("k_pack_codes");
}

int qe_strdict_decode_packed(qe_ctx* ctx, const qe_column* codes, qe_column* out) {
  QE_CHECK(ctx && codes && out, QE_ERR_INVALID_ARG, "null argument");
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(codes->type == QE_TYPE_INT64, QE_ERR_INVALID_ARG, "packed codes are INT64 (wide codes)");
  QE_CHECK(out->type == QE_TYPE_UTF8 && out->offsets, QE_ERR_INVALID_ARG, "output must be UTF8 with offsets");
  const int64_t n = codes->length;
  QE_CHECK(n < (1ll << 28), QE_ERR_CAPACITY, "packed decode takes fewer than 2^28 rows");
  QE_CHECK(!codes->validity || out->validity, QE_ERR_INVALID_ARG, "output validity buffer required");
  QE_CHECK(out->values || n == 0, QE_ERR_CAPACITY, "output values buffer required (7 bytes per row)");
  out->length = n;
  if (n == 0) {
    QE_HIP(hipMemsetAsync(out->offsets, 0, 4, ctx->stream));
    return QE_OK;
  }
  if (n <= 65536) {
    hipLaunchKernelGGL(k_unpack_codes_small, dim3(1), dim3(1024), 0, ctx->stream, (const int64_t*)codes->values,
                       codes->validity, n, out->offsets, (uint8_t*)out->values);
    QE_TRY(launch_check("k_unpack_codes_small"));
  } else {
    void* sp;
    QE_TRY(ctx_scratch(ctx, (size_t)(2 * n + 2) * 8, &sp));
    int64_t* lens = (int64_t*)sp;
    int64_t* starts = lens + n;
    unsigned int* bad = (unsigned int*)(starts + n + 1);
    const int g = (int)std::min<int64_t>((int64_t)div_up((uint64_t)n + 1, 256), (int64_t)ctx->num_cus * 8);
    hipLaunchKernelGGL(k_dict_decode_len<true>, dim3(g), dim3(256), 0, ctx->stream, codes->values, codes->validity, n,
                       nullptr, (int64_t)0, lens, bad);
    QE_TRY(launch_check("k_dict_decode_len"));
    QE_TRY(exclusive_scan_i64(ctx, lens, starts, n));
    hipLaunchKernelGGL(k_dict_decode_copy<true>, dim3(g), dim3(256), 0, ctx->stream, codes->values, codes->validity, n,
                       nullptr, nullptr, (int64_t)0, nullptr, starts, out->offsets, (uint8_t*)out->values);
    QE_TRY(launch_check("k_dict_decode_copy"));
  }
  if (codes->validity)
    QE_HIP(hipMemcpyAsync(out->validity, codes->validity, (size_t)div_up((uint64_t)n, 8), hipMemcpyDeviceToDevice,
                          ctx->stream));
  return QE_OK;
}

}  // extern "C"

int qe::strdict_encode_packed_checked(qe_ctx* ctx, const qe_column* in, qe_column* codes, unsigned long long* err) {
  const int64_t n = in->length;
  codes->length = n;
  if (n == 0) return QE_OK;
  if (in->validity)
    QE_HIP(hipMemcpyAsync(codes->validity, in->validity, (size_t)div_up((uint64_t)n, 8), hipMemcpyDeviceToDevice,
                          ctx->stream));
  const int grid = (int)std::min<int64_t>((int64_t)div_up((uint64_t)n, 256), (int64_t)ctx->num_cus * 8);
  hipLaunchKernelGGL(k_pack_codes, dim3(grid), dim3(256), 0, ctx->stream, in->offsets, (const uint8_t*)in->values,
                     in->validity, n, (int64_t*)codes->values, err);
  return launch_check("k_pack_codes");
}
