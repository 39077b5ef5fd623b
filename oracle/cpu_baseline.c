/*
 * ORACLE (test infrastructure + timed CPU baseline only — never linked into the product).
 *
 * Reference-faithful C restatement of the kquerydiy CPU path for the headline query
 *   SELECT k, SUM(a+b), COUNT(*), MIN(a), MAX(b) FROM t WHERE a > K GROUP BY k
 * as the reference's operator chain would execute it (folkol/query-engines kquerydiy/src/Main.kt):
 *   - per input batch, SelectionExec materialises the selected rows (build-defined operator),
 *   - ProjectionExec evaluates a+b into a new column (K:589-594),
 *   - HashAggregateExec.execute loops row at a time (K:620): it builds the row's key as a List of
 *     boxed values (K:621-626; ArrayList + Object[] + java.lang.Long from a per-thread bump
 *     allocator that is collected after each batch), looks it up in a chained hash map
 *     (java.util.HashMap, K:616/K:627: List.hashCode / List.equals, node per group) and calls each
 *     Accumulator through a virtual interface (K:519-522, K:628-631) with a boxed Long per input.
 *   - partition parallelism mirrors main() (K:1309-1325): T partitions aggregated concurrently,
 *     then a final merge of the partial maps.
 * The synthetic columns are regenerated here bit-for-bit (splitmix64, oracle/gen.py) before the
 * timed region starts.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static uint64_t gen_u64(uint64_t seed, uint64_t col, uint64_t row) {
  return splitmix64(seed ^ (col * 0x9E3779B97F4A7C15ull) ^ row);
}

/* ---- JVM object model the reference's row loop allocates (K:620-631) ----------------------------
 * Per selected row the reference builds the group key as a Kotlin List of boxed values
 * (`groupKeys.map { it.getValue(rowIndex) }`, K:621-626: an ArrayList plus its Object[] plus a
 * java.lang.Long per key value), and passes every aggregate input to its Accumulator boxed
 * (`aggrInputValues[i].getValue(rowIndex)`, K:628-631). Those objects come from the thread's
 * allocation buffer (bump pointer) and die young: here a per-thread arena that is reset after
 * every input batch (a minor collection whose survivors are only the map's keys, copied out on
 * insert). Long.valueOf's cache of -128..127 is modelled (no allocation for those values). */
typedef struct {
  uint64_t hdr; /* mark + class words of a JVM object header, compressed */
  int64_t v;
} jlong_box; /* java.lang.Long */

typedef struct {
  uint64_t hdr;
  int32_t len, pad;
  jlong_box* e[1];
} jarray1; /* Object[1] */

typedef struct {
  uint64_t hdr;
  int32_t size, modcount;
  jarray1* data;
} jlist; /* java.util.ArrayList of one key */

typedef struct {
  char* base;
  size_t off, cap;
} arena;

static jlong_box g_long_cache[256]; /* Long.valueOf cache, -128..127 */
static pthread_once_t g_cache_once = PTHREAD_ONCE_INIT;
static void init_long_cache(void) {
  for (int i = 0; i < 256; ++i) g_long_cache[i] = (jlong_box){0x1ull, (int64_t)i - 128};
}

static void* arena_alloc(arena* a, size_t n) {
  n = (n + 7) & ~(size_t)7;
  if (a->off + n > a->cap) { /* eden full mid-batch: a collection (nothing of earlier rows is live) */
    a->off = 0;
  }
  void* p = a->base + a->off;
  a->off += n;
  return p;
}

static jlong_box* box_long(arena* a, int64_t v) { /* Long.valueOf */
  if (v >= -128 && v <= 127) return &g_long_cache[v + 128];
  jlong_box* b = (jlong_box*)arena_alloc(a, sizeof(jlong_box));
  b->hdr = 0x1ull;
  b->v = v;
  return b;
}

static jlist* key_list(arena* a, jlong_box* k) { /* listOf(boxed key) built by map { } */
  jarray1* arr = (jarray1*)arena_alloc(a, sizeof(jarray1));
  arr->hdr = 0x1ull;
  arr->len = 1;
  arr->e[0] = k;
  jlist* l = (jlist*)arena_alloc(a, sizeof(jlist));
  l->hdr = 0x1ull;
  l->size = 1;
  l->modcount = 0;
  l->data = arr;
  return l;
}

/* ---- the Accumulator interface (K:519-522), inputs boxed (null = NULL pointer) --------------- */
typedef struct accumulator accumulator;
struct accumulator {
  void (*accumulate)(accumulator*, const jlong_box*);
  int has;
  int64_t value;
};

static void sum_acc(accumulator* a, const jlong_box* x) {
  if (!x) return;
  a->value = (int64_t)((uint64_t)a->value + (uint64_t)x->v);
  a->has = 1;
}
static void count_acc(accumulator* a, const jlong_box* x) {
  (void)x;
  a->value += 1;
  a->has = 1;
}
static void min_acc(accumulator* a, const jlong_box* x) {
  if (!x) return;
  if (!a->has || x->v < a->value) a->value = x->v;
  a->has = 1;
}
static void max_acc(accumulator* a, const jlong_box* x) { /* MaxAccumulator K:540-557 */
  if (!x) return;
  if (!a->has) {
    a->value = x->v;
    a->has = 1;
  } else if (x->v > a->value) {
    a->value = x->v;
  }
}

/* ---- java.util.HashMap<List<Any?>, List<Accumulator>> (K:616, K:627) --------------------------- */
typedef struct node {
  jlist* key; /* survivor copy of the row's key list */
  uint32_t hash;
  struct node* next;
  accumulator acc[4];
} node;

typedef struct {
  node** buckets;
  size_t nbuckets;
  size_t size;
} hashmap;

static uint32_t list_hash(const jlist* k) { /* List.hashCode (31 * 1 + Long.hashCode) + HashMap.hash */
  uint32_t h = 1;
  for (int32_t i = 0; i < k->size; ++i) {
    const jlong_box* e = k->data->e[i];
    h = 31u * h + (e ? (uint32_t)(e->v ^ ((uint64_t)e->v >> 32)) : 0u);
  }
  return h ^ (h >> 16);
}

static int list_equals(const jlist* x, const jlist* y) { /* List.equals -> Long.equals per element */
  if (x->size != y->size) return 0;
  for (int32_t i = 0; i < x->size; ++i) {
    const jlong_box *a = x->data->e[i], *b = y->data->e[i];
    if ((a == NULL) != (b == NULL)) return 0;
    if (a && a->v != b->v) return 0;
  }
  return 1;
}

static jlist* list_survivor(const jlist* k) { /* the key object outlives the batch: copy it out */
  jlist* l = (jlist*)malloc(sizeof(jlist) + sizeof(jarray1) + sizeof(jlong_box));
  jarray1* arr = (jarray1*)(l + 1);
  jlong_box* b = (jlong_box*)(arr + 1);
  *l = *k;
  l->data = arr;
  *arr = *k->data;
  if (k->data->e[0]) {
    *b = *k->data->e[0];
    arr->e[0] = b;
  }
  return l;
}

static void map_init(hashmap* m) {
  m->nbuckets = 16;
  m->buckets = (node**)calloc(m->nbuckets, sizeof(node*));
  m->size = 0;
}

static void map_grow(hashmap* m) {
  size_t nb = m->nbuckets * 2;
  node** b = (node**)calloc(nb, sizeof(node*));
  for (size_t i = 0; i < m->nbuckets; ++i) {
    node* n = m->buckets[i];
    while (n) {
      node* nx = n->next;
      size_t j = n->hash & (nb - 1);
      n->next = b[j];
      b[j] = n;
      n = nx;
    }
  }
  free(m->buckets);
  m->buckets = b;
  m->nbuckets = nb;
}

static node* map_get_or_put(hashmap* m, const jlist* key) {
  uint32_t h = list_hash(key);
  node* n = m->buckets[h & (m->nbuckets - 1)];
  for (; n; n = n->next)
    if (n->hash == h && list_equals(n->key, key)) return n;
  n = (node*)calloc(1, sizeof(node));
  n->key = list_survivor(key);
  n->hash = h;
  n->acc[0].accumulate = sum_acc;
  n->acc[1].accumulate = count_acc;
  n->acc[2].accumulate = min_acc;
  n->acc[3].accumulate = max_acc;
  size_t b = h & (m->nbuckets - 1);
  n->next = m->buckets[b];
  m->buckets[b] = n;
  if (++m->size > m->nbuckets * 3 / 4) map_grow(m);
  return n;
}

static void map_free(hashmap* m) {
  for (size_t i = 0; i < m->nbuckets; ++i) {
    node* n = m->buckets[i];
    while (n) {
      node* nx = n->next;
      free(n->key);
      free(n);
      n = nx;
    }
  }
  free(m->buckets);
}

static int64_t key_of(const node* n) { return n->key->data->e[0]->v; }

/* ---- one partition: batches of BATCH rows through Selection -> Projection -> HashAggregate ---- */
#define BATCH 65536
#define EDEN_BYTES ((size_t)16 << 20)

typedef struct {
  const int64_t *k, *a, *b;
  int64_t n, threshold;
  hashmap map;
} part;

static void run_partition(part* p) {
  pthread_once(&g_cache_once, init_long_cache);
  int64_t* sk = (int64_t*)malloc(BATCH * sizeof(int64_t));
  int64_t* sa = (int64_t*)malloc(BATCH * sizeof(int64_t));
  int64_t* sb = (int64_t*)malloc(BATCH * sizeof(int64_t));
  int64_t* proj = (int64_t*)malloc(BATCH * sizeof(int64_t));
  arena eden = {(char*)malloc(EDEN_BYTES), 0, EDEN_BYTES};
  map_init(&p->map);
  for (int64_t s = 0; s < p->n; s += BATCH) {
    const int64_t m = p->n - s < BATCH ? p->n - s : BATCH;
    /* SelectionExec: evaluate predicate, materialise selected rows */
    int64_t c = 0;
    for (int64_t i = 0; i < m; ++i) {
      if (p->a[s + i] > p->threshold) {
        sk[c] = p->k[s + i];
        sa[c] = p->a[s + i];
        sb[c] = p->b[s + i];
        ++c;
      }
    }
    /* ProjectionExec: a + b (JVM Long wrap) */
    for (int64_t i = 0; i < c; ++i) proj[i] = (int64_t)((uint64_t)sa[i] + (uint64_t)sb[i]);
    /* HashAggregateExec row loop (K:620-631): boxed key list, getOrPut, boxed accumulator inputs */
    for (int64_t i = 0; i < c; ++i) {
      jlist* key = key_list(&eden, box_long(&eden, sk[i]));
      node* n = map_get_or_put(&p->map, key);
      n->acc[0].accumulate(&n->acc[0], box_long(&eden, proj[i]));
      n->acc[1].accumulate(&n->acc[1], box_long(&eden, 1));
      n->acc[2].accumulate(&n->acc[2], box_long(&eden, sa[i]));
      n->acc[3].accumulate(&n->acc[3], box_long(&eden, sb[i]));
    }
    eden.off = 0; /* minor collection: this batch's row objects are dead */
  }
  free(eden.base);
  free(sk);
  free(sa);
  free(sb);
  free(proj);
}

static void* part_main(void* arg) {
  run_partition((part*)arg);
  return NULL;
}

typedef struct {
  int64_t *k, *a, *b;
  int64_t row0, n, nkeys;
  uint64_t seed;
} gen_job;

static void* gen_main(void* arg) { /* untimed: regenerate the synthetic rows (oracle/gen.py) */
  gen_job* g = (gen_job*)arg;
  for (int64_t i = 0; i < g->n; ++i) {
    const uint64_t r = (uint64_t)(g->row0 + i);
    g->k[i] = (int64_t)(gen_u64(g->seed, 0, r) % (uint64_t)g->nkeys);
    g->a[i] = (int64_t)(gen_u64(g->seed, 1, r) % (1ull << 20));
    g->b[i] = (int64_t)(gen_u64(g->seed, 2, r) % (1ull << 20));
  }
  return NULL;
}

typedef struct {
  int64_t key;
  int64_t sum, count, min, max;
} qe_group_out;

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* Returns seconds spent in the (timed) query; fills out[] (cap entries) and *ngroups.
 * Data: k = u0 % 1024, a = u1 % 2^20, b = u2 % 2^20 for rows row0..row0+rows-1. */
double qe_cpu_c4(int64_t row0, int64_t rows, uint64_t seed, int threads, int64_t threshold, int64_t nkeys,
                 qe_group_out* out, int64_t cap, int64_t* ngroups) {
  if (threads < 1) threads = 1;
  int64_t* k = (int64_t*)malloc(rows * sizeof(int64_t));
  int64_t* a = (int64_t*)malloc(rows * sizeof(int64_t));
  int64_t* b = (int64_t*)malloc(rows * sizeof(int64_t));
  part* parts = (part*)calloc(threads, sizeof(part));
  pthread_t* tid = (pthread_t*)calloc(threads, sizeof(pthread_t));
  const int64_t per = (rows + threads - 1) / threads;
  gen_job* jobs = (gen_job*)calloc(threads, sizeof(gen_job));
  for (int t = 0; t < threads; ++t) {
    const int64_t s = t * per, e = (s + per < rows) ? s + per : rows;
    jobs[t] = (gen_job){k + s, a + s, b + s, row0 + s, e > s ? e - s : 0, nkeys, seed};
    pthread_create(&tid[t], NULL, gen_main, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  free(jobs);
  const double t0 = now_s();
  for (int t = 0; t < threads; ++t) {
    const int64_t s = t * per, e = (s + per < rows) ? s + per : rows;
    parts[t].k = k + s;
    parts[t].a = a + s;
    parts[t].b = b + s;
    parts[t].n = e > s ? e - s : 0;
    parts[t].threshold = threshold;
    pthread_create(&tid[t], NULL, part_main, &parts[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  /* final merge of the partial maps, in partition order (K:1314-1325) */
  hashmap fin;
  map_init(&fin);
  for (int t = 0; t < threads; ++t) {
    for (size_t i = 0; i < parts[t].map.nbuckets; ++i) {
      for (node* n = parts[t].map.buckets[i]; n; n = n->next) {
        node* f = map_get_or_put(&fin, n->key);
        jlong_box s0 = {1, n->acc[0].value}, s2 = {1, n->acc[2].value}, s3 = {1, n->acc[3].value};
        f->acc[0].accumulate(&f->acc[0], &s0);
        f->acc[1].value += n->acc[1].value;
        f->acc[1].has = 1;
        f->acc[2].accumulate(&f->acc[2], n->acc[2].has ? &s2 : NULL);
        f->acc[3].accumulate(&f->acc[3], n->acc[3].has ? &s3 : NULL);
      }
    }
  }
  const double t1 = now_s();
  int64_t g = 0;
  for (size_t i = 0; i < fin.nbuckets; ++i) {
    for (node* n = fin.buckets[i]; n; n = n->next) {
      if (g < cap && out) {
        out[g].key = key_of(n);
        out[g].sum = n->acc[0].value;
        out[g].count = n->acc[1].value;
        out[g].min = n->acc[2].value;
        out[g].max = n->acc[3].value;
      }
      ++g;
    }
  }
  *ngroups = g;
  map_free(&fin);
  for (int t = 0; t < threads; ++t) map_free(&parts[t].map);
  free(parts);
  free(tid);
  free(k);
  free(a);
  free(b);
  return t1 - t0;
}

/* ---- a tuned CPU implementation of the same query, reported beside the port ("plus
 * a vectorised CPU path for honesty"): no boxing, no per-batch materialisation; each thread
 * filters, projects and aggregates into its own open-addressing table (linear probing, keys not
 * assumed dense), then the tables merge in thread order. Same results as qe_cpu_c4. */
#define FAST_SLOTS 4096
#define FAST_EMPTY INT64_MIN

typedef struct {
  const int64_t *k, *a, *b;
  int64_t n, threshold;
  int64_t key[FAST_SLOTS], sum[FAST_SLOTS], cnt[FAST_SLOTS], mn[FAST_SLOTS], mx[FAST_SLOTS];
  int overflow;
} fast_part;

static inline uint32_t fast_slot(int64_t k) {
  uint64_t h = (uint64_t)k * 0x9E3779B97F4A7C15ull;
  return (uint32_t)(h >> 52); /* 12 bits */
}

static void* fast_main(void* arg) {
  fast_part* p = (fast_part*)arg;
  for (int s = 0; s < FAST_SLOTS; ++s) p->key[s] = FAST_EMPTY;
  const int64_t thr = p->threshold;
  for (int64_t i = 0; i < p->n; ++i) {
    const int64_t a = p->a[i];
    if (a <= thr) continue;
    const int64_t k = p->k[i], b = p->b[i];
    uint32_t s = fast_slot(k);
    int probes = 0;
    while (p->key[s] != k && p->key[s] != FAST_EMPTY) {
      s = (s + 1) & (FAST_SLOTS - 1);
      if (++probes == FAST_SLOTS) {
        p->overflow = 1;
        return NULL;
      }
    }
    if (p->key[s] == FAST_EMPTY) {
      p->key[s] = k;
      p->sum[s] = 0;
      p->cnt[s] = 0;
      p->mn[s] = INT64_MAX;
      p->mx[s] = INT64_MIN;
    }
    p->sum[s] = (int64_t)((uint64_t)p->sum[s] + (uint64_t)a + (uint64_t)b);
    p->cnt[s] += 1;
    if (a < p->mn[s]) p->mn[s] = a;
    if (b > p->mx[s]) p->mx[s] = b;
  }
  return NULL;
}

/* Returns seconds of the timed query (generation untimed), or -1 if a thread's table overflowed
 * (more than FAST_SLOTS groups). */
double qe_cpu_c4_fast(int64_t row0, int64_t rows, uint64_t seed, int threads, int64_t threshold, int64_t nkeys,
                      qe_group_out* out, int64_t cap, int64_t* ngroups) {
  if (threads < 1) threads = 1;
  int64_t* k = (int64_t*)malloc(rows * sizeof(int64_t));
  int64_t* a = (int64_t*)malloc(rows * sizeof(int64_t));
  int64_t* b = (int64_t*)malloc(rows * sizeof(int64_t));
  fast_part* parts = (fast_part*)calloc(threads, sizeof(fast_part));
  pthread_t* tid = (pthread_t*)calloc(threads, sizeof(pthread_t));
  const int64_t per = (rows + threads - 1) / threads;
  gen_job* jobs = (gen_job*)calloc(threads, sizeof(gen_job));
  for (int t = 0; t < threads; ++t) {
    const int64_t s = t * per, e = (s + per < rows) ? s + per : rows;
    jobs[t] = (gen_job){k + s, a + s, b + s, row0 + s, e > s ? e - s : 0, nkeys, seed};
    pthread_create(&tid[t], NULL, gen_main, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  free(jobs);
  const double t0 = now_s();
  for (int t = 0; t < threads; ++t) {
    const int64_t s = t * per, e = (s + per < rows) ? s + per : rows;
    parts[t].k = k + s;
    parts[t].a = a + s;
    parts[t].b = b + s;
    parts[t].n = e > s ? e - s : 0;
    parts[t].threshold = threshold;
    pthread_create(&tid[t], NULL, fast_main, &parts[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  /* merge the thread tables in thread order into the first */
  fast_part* f = &parts[0];
  int bad = f->overflow;
  for (int t = 1; t < threads && !bad; ++t) {
    fast_part* p = &parts[t];
    bad |= p->overflow;
    for (int s = 0; s < FAST_SLOTS && !bad; ++s) {
      if (p->key[s] == FAST_EMPTY) continue;
      const int64_t key = p->key[s];
      uint32_t d = fast_slot(key);
      int probes = 0;
      while (f->key[d] != key && f->key[d] != FAST_EMPTY) {
        d = (d + 1) & (FAST_SLOTS - 1);
        if (++probes == FAST_SLOTS) {
          bad = 1;
          break;
        }
      }
      if (bad) break;
      if (f->key[d] == FAST_EMPTY) {
        f->key[d] = key;
        f->sum[d] = 0;
        f->cnt[d] = 0;
        f->mn[d] = INT64_MAX;
        f->mx[d] = INT64_MIN;
      }
      f->sum[d] = (int64_t)((uint64_t)f->sum[d] + (uint64_t)p->sum[s]);
      f->cnt[d] += p->cnt[s];
      if (p->mn[s] < f->mn[d]) f->mn[d] = p->mn[s];
      if (p->mx[s] > f->mx[d]) f->mx[d] = p->mx[s];
    }
  }
  const double t1 = now_s();
  int64_t g = 0;
  for (int s = 0; s < FAST_SLOTS && !bad; ++s) {
    if (f->key[s] == FAST_EMPTY) continue;
    if (g < cap && out) out[g] = (qe_group_out){f->key[s], f->sum[s], f->cnt[s], f->mn[s], f->mx[s]};
    ++g;
  }
  *ngroups = g;
  free(parts);
  free(tid);
  free(k);
  free(a);
  free(b);
  return bad ? -1.0 : t1 - t0;
}

/* ---- C5 (BASELINE configs[4]) with exact fp64 sums: the full-size per-group check's oracle ----------
 * SELECT l_returnflag, l_linestatus, SUM(l_quantity), SUM(l_extendedprice),
 *        SUM(l_extendedprice * (1 - l_discount)), SUM(l_extendedprice * (1 - l_discount) * (1 + l_tax)),
 *        AVG(l_extendedprice), COUNT(*)
 * WHERE l_shipdate <= 2400 AND l_discount >= 0.05 AND l_discount <= 0.07 AND l_quantity < 24
 * GROUP BY l_returnflag, l_linestatus          (kquery/workloads.py c5_spec; columns datasource.py)
 * Rows are regenerated bit for bit (generator column ids 10..16). Each fp64 value is added EXACTLY:
 * as an integer in units of 2^-80 (every value of this data is a multiple of that, checked; the
 * per-group totals stay below 2^125), so the sums are the exact sums of the rows' fp64 values —
 * the reference's sequential loop with exact arithmetic. The caller rounds them once (Python
 * Fraction -> float). out[g * 8 + ...], g = returnflag * 2 + linestatus:
 *   [0] COUNT(*)  [1] SUM(quantity) (int64, wraps)  [2..3] SUM(price)  [4..5] SUM(price*(1-d))
 *   [6..7] SUM(price*(1-d)*(1+t)); each exact sum as (signed high 64 bits, low 64 bits).
 * Returns seconds, or -1 if a value was not a multiple of 2^-80. */
typedef struct {
  int64_t row0, n;
  uint64_t seed;
  int64_t cnt[6], sq[6];
  __int128 s[3][6];
  int bad;
} c5_job;

static int c5_fixed(double v, __int128* out) { /* v * 2^80 as an exact integer */
  if (v == 0.0) {
    *out = 0;
    return 1;
  }
  int e;
  const double m = frexp(v, &e);              /* v = m * 2^e, 0.5 <= |m| < 1 */
  const int64_t M = (int64_t)ldexp(m, 53);    /* exact: 53-bit mantissa */
  const int sh = e - 53 + 80;
  if (sh >= 0) {
    if (sh > 70) return 0;
    *out = (__int128)M << sh;
    return 1;
  }
  if (-sh >= 63 || (M & ((1ll << -sh) - 1)) != 0) return 0;
  *out = (__int128)(M >> -sh);
  return 1;
}

static void* c5_main(void* arg) {
  c5_job* j = (c5_job*)arg;
  for (int64_t i = 0; i < j->n; ++i) {
    const uint64_t r = (uint64_t)(j->row0 + i);
    const int64_t qty = (int64_t)(gen_u64(j->seed, 10, r) % 50ull);
    const double price = (double)(gen_u64(j->seed, 11, r) % 10000000ull) * 0.01;
    const double disc = (double)(gen_u64(j->seed, 12, r) % 11ull) * 0.01;
    const double tax = (double)(gen_u64(j->seed, 13, r) % 9ull) * 0.01;
    const int flag = (int)(gen_u64(j->seed, 14, r) % 3ull);
    const int status = (int)(gen_u64(j->seed, 15, r) % 2ull);
    const int32_t ship = (int32_t)(gen_u64(j->seed, 16, r) % 2557ull);
    if (!(ship <= 2400 && disc >= 0.05 && disc <= 0.07 && qty < 24)) continue;
    const double dp = price * (1.0 - disc);
    const double dpt = dp * (1.0 + tax);
    const int g = flag * 2 + status;
    __int128 a, b, c;
    if (!c5_fixed(price, &a) || !c5_fixed(dp, &b) || !c5_fixed(dpt, &c)) {
      j->bad = 1;
      continue;
    }
    j->cnt[g] += 1;
    j->sq[g] = (int64_t)((uint64_t)j->sq[g] + (uint64_t)qty);
    j->s[0][g] += a;
    j->s[1][g] += b;
    j->s[2][g] += c;
  }
  return NULL;
}

double qe_cpu_c5_exact(int64_t row0, int64_t rows, uint64_t seed, int threads, int64_t* out) {
  if (threads < 1) threads = 1;
  c5_job* jobs = (c5_job*)calloc(threads, sizeof(c5_job));
  pthread_t* tid = (pthread_t*)calloc(threads, sizeof(pthread_t));
  const int64_t per = (rows + threads - 1) / threads;
  const double t0 = now_s();
  for (int t = 0; t < threads; ++t) {
    const int64_t s = t * per, e = (s + per < rows) ? s + per : rows;
    jobs[t].row0 = row0 + s;
    jobs[t].n = e > s ? e - s : 0;
    jobs[t].seed = seed;
    pthread_create(&tid[t], NULL, c5_main, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
  int bad = 0;
  for (int g = 0; g < 6; ++g) {
    int64_t cnt = 0;
    uint64_t sq = 0;
    __int128 s[3] = {0, 0, 0};
    for (int t = 0; t < threads; ++t) {
      bad |= jobs[t].bad;
      cnt += jobs[t].cnt[g];
      sq += (uint64_t)jobs[t].sq[g];
      for (int k = 0; k < 3; ++k) s[k] += jobs[t].s[k][g];
    }
    out[g * 8 + 0] = cnt;
    out[g * 8 + 1] = (int64_t)sq;
    for (int k = 0; k < 3; ++k) {
      out[g * 8 + 2 + 2 * k] = (int64_t)(s[k] >> 64);
      out[g * 8 + 3 + 2 * k] = (int64_t)(uint64_t)s[k];
    }
  }
  const double t1 = now_s();
  free(jobs);
  free(tid);
  return bad ? -1.0 : t1 - t0;
}
