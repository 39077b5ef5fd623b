/* TEST INFRASTRUCTURE (SURVEY §5 sanitizers): the oracle's C restatement (oracle/cpu_baseline.c)
 * under AddressSanitizer + UBSan, multi-threaded. Prints "key sum count min max" per group in key
 * order; tests/test_sanitizers.py compares with the Python oracle. */
#include <stdio.h>
#include <stdlib.h>

#include "../../oracle/cpu_baseline.c"

static int by_key(const void* x, const void* y) {
  const qe_group_out *a = (const qe_group_out*)x, *b = (const qe_group_out*)y;
  return (a->key > b->key) - (a->key < b->key);
}

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  const int64_t row0 = atoll(argv[1]), rows = atoll(argv[2]);
  const int threads = atoi(argv[3]);
  qe_group_out* out = (qe_group_out*)calloc(2048, sizeof(qe_group_out));
  int64_t ng = 0;
  qe_cpu_c4(row0, rows, 42, threads, 1 << 19, 1024, out, 2048, &ng);
  qsort(out, (size_t)ng, sizeof(qe_group_out), by_key);
  for (int64_t i = 0; i < ng; ++i)
    printf("%lld %lld %lld %lld %lld\n", (long long)out[i].key, (long long)out[i].sum, (long long)out[i].count,
           (long long)out[i].min, (long long)out[i].max);
  free(out);
  return 0;
}
