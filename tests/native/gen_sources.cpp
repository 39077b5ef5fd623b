// Host program (no GPU): emits the select-project kernel sources that qe_select_project would
// compile with hipRTC, for a few plan shapes and every tile-order mode, into argv[1]/. The CPU
// suite then compiles each for gfx950 with hipcc (tests/test_jit_sources.py), so a generator
// change that emits invalid HIP fails here rather than on the GPU box.
#include <stdio.h>
#include <string.h>

#include <string>

#include "qe_internal.hpp"

using namespace qe;

static qe_pred_term term(int col, int op, int64_t lit) {
  qe_pred_term t;
  memset(&t, 0, sizeof t);
  t.col = col;
  t.op = op;
  t.rhs_col = -1;
  t.lit.type = QE_TYPE_INT64;
  t.lit.bits = lit;
  return t;
}

static int emit(const char* dir, const char* name, const qe_column* cols, int ncols, const qe_pred_term* terms,
                int nterms, const qe_agg_program* outs, int nout) {
  Plan P;
  bool col_f64[QE_MAX_COLS];
  if (compile_inputs(cols, ncols, -1, nterms, terms, &P, col_f64) != QE_OK) {
    fprintf(stderr, "%s: compile_inputs: %s\n", name, qe_last_error());
    return 1;
  }
  int32_t out_kind[QE_MAX_AGGS];
  P.naggs = nout;
  for (int k = 0; k < nout; ++k) {
    bool is_f = false, nullable = false;
    if (compile_program(cols, ncols, col_f64, outs[k], k, &P.aggs[k], &is_f, &nullable) != QE_OK) {
      fprintf(stderr, "%s: compile_program: %s\n", name, qe_last_error());
      return 1;
    }
    out_kind[k] = (is_f ? 8 : 8) | (nullable ? 0x100 : 0);
  }
  const int modes[] = {SP_COUNTER, SP_PERSIST, SP_COUNT, SP_WRITE, SP_WRITE_SCAN};
  for (int m : modes) {
    std::string src;
    if (!gen_selproj_source(P, out_kind, nout, &src, m)) {
      fprintf(stderr, "%s: mode %d not generated\n", name, m);
      return 1;
    }
    const std::string path = std::string(dir) + "/" + name + "_m" + std::to_string(m) + ".hip";
    FILE* f = fopen(path.c_str(), "w");
    if (!f) return 1;
    fwrite(src.data(), 1, src.size(), f);
    fclose(f);
    printf("%s\n", path.c_str());
  }
  // register-resident one-pass kernel (SP_RESIDENT) at 40 rows per thread, where the plan takes it
  // (and its several-rounds form, file suffix _m6)
  const int R = selproj_resident_rows(P, out_kind, nout, 10000000, 256);
  for (int multi = 0; R > 0 && multi < 2; ++multi) {
    std::string src;
    if (!gen_selproj_resident_source(P, out_kind, nout, R | (multi ? 0x100 : 0), &src)) {
      fprintf(stderr, "%s: resident mode not generated\n", name);
      return 1;
    }
    const std::string path = std::string(dir) + "/" + name + "_m" + std::to_string(SP_RESIDENT + multi) + ".hip";
    FILE* f = fopen(path.c_str(), "w");
    if (!f) return 1;
    fwrite(src.data(), 1, src.size(), f);
    fclose(f);
    printf("%s\n", path.c_str());
  }
  return 0;
}

static int write_src(const char* dir, const std::string& name, const std::string& src) {
  const std::string path = std::string(dir) + "/" + name + ".hip";
  FILE* f = fopen(path.c_str(), "w");
  if (!f) return 1;
  fwrite(src.data(), 1, src.size(), f);
  fclose(f);
  printf("%s\n", path.c_str());
  return 0;
}

// Fused GROUP BY plan (key in slot 0; aggregates given as (fn, acc, program)) with two key-hash
// buckets: the two-pass fused kernel, the spilling first pass (spill_update) and the qe_pagg pass
// over its records.
struct AggIn {
  int fn, acc;
  const qe_agg_program* prog;  // null: COUNT(*)
};
static int emit_agg(const char* dir, const char* name, const qe_column* cols, int ncols, const qe_pred_term* terms,
                    int nterms, const AggIn* aggs, int naggs, int log2) {
  Plan P;
  bool col_f64[QE_MAX_COLS];
  if (compile_inputs(cols, ncols, -1, nterms, terms, &P, col_f64) != QE_OK) {
    fprintf(stderr, "%s: compile_inputs: %s\n", name, qe_last_error());
    return 1;
  }
  P.key_mode = 1;
  P.nkeys = 1;
  P.key_col[0] = 0;
  P.key_f64 = 0;
  P.naggs = naggs;
  for (int j = 0; j < naggs; ++j) {
    memset(&P.aggs[j], 0, sizeof P.aggs[j]);
    bool is_f = false, nullable = false;
    if (aggs[j].prog && compile_program(cols, ncols, col_f64, *aggs[j].prog, j, &P.aggs[j], &is_f, &nullable) != QE_OK) {
      fprintf(stderr, "%s: compile_program: %s\n", name, qe_last_error());
      return 1;
    }
    P.aggs[j].fn = aggs[j].fn;
    P.aggs[j].acc = aggs[j].acc;
    P.aggs[j].track_nn = nullable ? 1 : 0;
    P.aggs[j].pkind = aggs[j].prog ? 2 : 0;  // token program (compile_plan's general form)
  }
  // the same input summed twice (SUM and AVG of one column): one shared LDS accumulator, as
  // compile_plan marks it
  for (int j = 1; j < naggs; ++j)
    if (aggs[j].prog && aggs[j].prog == aggs[0].prog && aggs[j].acc == aggs[0].acc) P.aggs[j].share = 1;
  P.mp_n = 2;
  P.mp_pass = 0;
  std::string a, b, c;
  size_t lds = 0;
  if (!gen_fused_source(P, log2, &a, &lds, false) || !gen_fused_source(P, log2, &b, &lds, true) ||
      !gen_pagg_source(P, log2, &c, &lds, true, true)) {
    fprintf(stderr, "%s: fused / spill / pagg source not generated\n", name);
    return 1;
  }
  // radix-partitioned path: staged chunked scatter over 64 buckets, records row-major and
  // chunk-columnar (QE_PART_SOA), and the chunk-columnar aggregation pass
  std::string d, e, f;
  P.mp_n = 0;
  if (!gen_pscatter_staged_source(P, 6, &d, true, false) || !gen_pscatter_staged_source(P, 6, &e, true, true) ||
      !gen_pagg_source(P, log2, &f, &lds, true, false)) {
    fprintf(stderr, "%s: partition sources not generated\n", name);
    return 1;
  }
  // 32-bit records (Plan.part_narrow; wide again where a word is fp64 or a row index): staged
  // chunked and direct scatters, chunked and unchunked aggregation passes
  std::string g, h, i, j, i2;
  P.part_narrow = 1;
  // (i2: the fast aggregation pass with 2048 groups per bucket: its largest table, no regrouping)
  if (!gen_pscatter_staged_source(P, 6, &g, true, false) || !gen_part_source(P, 10, true, &h) ||
      !gen_pagg_source(P, log2, &i, &lds, true, false) || !gen_pagg_source(P, log2, &j, &lds, false, false) ||
      !gen_pagg_source(P, log2, &i2, &lds, true, false, 2048)) {
    fprintf(stderr, "%s: narrow partition sources not generated\n", name);
    return 1;
  }
  // 32-bit records of the spilling pass and their (record-major) aggregation pass
  std::string k, l;
  P.mp_n = 2;
  if (!gen_fused_source(P, log2, &k, &lds, true) || !gen_pagg_source(P, log2, &l, &lds, true, false)) {
    fprintf(stderr, "%s: narrow spill sources not generated\n", name);
    return 1;
  }
  // compact LDS table (Plan.lds_compact) where the plan shape allows it
  P.mp_n = 0;
  P.part_narrow = 0;
  P.lds_compact = 6080;
  std::string m, m2;
  if (compact_ok(P)) {
    if (!gen_fused_source(P, log2, &m, &lds, false) || write_src(dir, std::string(name) + "_fused_compact", m)) {
      fprintf(stderr, "%s: compact fused source not generated\n", name);
      return 1;
    }
    // the spilling pass over a compact kept table (32-bit spill records)
    P.mp_n = 2;
    P.part_narrow = 1;
    if (!gen_fused_source(P, log2, &m2, &lds, true) || write_src(dir, std::string(name) + "_spill_compact", m2)) {
      fprintf(stderr, "%s: compact spill source not generated\n", name);
      return 1;
    }
    // ... with the spilled share in 4 sub-buckets
    std::string m4;
    P.mp_n = 5;
    if (!gen_fused_source(P, log2, &m4, &lds, true) || write_src(dir, std::string(name) + "_spill_compact_sb4", m4)) {
      fprintf(stderr, "%s: compact spill source (4 sub-buckets) not generated\n", name);
      return 1;
    }
    P.mp_n = 0;
  }
  P.lds_compact = 0;
  // single-pass fused kernel (mp_n = 0): exact fp64 SUM plans add through the per-wave fx queue
  std::string q1;
  if (!gen_fused_source(P, log2, &q1, &lds, false) || write_src(dir, std::string(name) + "_fused1", q1)) {
    fprintf(stderr, "%s: single-pass fused source not generated\n", name);
    return 1;
  }
  return write_src(dir, std::string(name) + "_fused", a) | write_src(dir, std::string(name) + "_spill", b) |
         write_src(dir, std::string(name) + "_pagg", c) | write_src(dir, std::string(name) + "_pscatter", d) |
         write_src(dir, std::string(name) + "_pscatter_soa", e) | write_src(dir, std::string(name) + "_pagg_rows", f) |
         write_src(dir, std::string(name) + "_pscatter_n32", g) |
         write_src(dir, std::string(name) + "_pdirect_n32", h) | write_src(dir, std::string(name) + "_pagg_n32", i) |
         write_src(dir, std::string(name) + "_pagg_unchunked_n32", j) |
         write_src(dir, std::string(name) + "_pagg_big_n32", i2) |
         write_src(dir, std::string(name) + "_spill_n32", k) | write_src(dir, std::string(name) + "_pagg_soa_n32", l);
}

// The C5 plan (BASELINE configs[4], kquery/workloads.py c5_spec): 7 columns, 4 predicate terms, two
// packed uint8 keys, SUM(qty) int64, 3 exact fp64 SUMs and an AVG sharing the first one's
// accumulator, COUNT(*); single pass over a 256-slot table (the fx queue path).
static int emit_c5(const char* dir) {
  static int64_t i64d[64];
  static double f64d[64];
  static uint8_t u8d[64];
  static int32_t i32d[64];
  qe_column cols[7];
  memset(cols, 0, sizeof cols);
  const int32_t types[7] = {QE_TYPE_INT64, QE_TYPE_FLOAT64, QE_TYPE_FLOAT64, QE_TYPE_FLOAT64, QE_TYPE_UINT8,
                            QE_TYPE_UINT8, QE_TYPE_DATE32};
  void* vals[7] = {i64d, f64d, f64d, f64d, u8d, u8d, i32d};
  for (int c = 0; c < 7; ++c) {
    cols[c].type = types[c];
    cols[c].length = 1000;
    cols[c].values = vals[c];
  }
  qe_pred_term t[4] = {term(6, QE_OP_LE, 2400), term(2, QE_OP_GE, 0), term(2, QE_OP_LE, 0), term(0, QE_OP_LT, 24)};
  for (int i = 1; i <= 2; ++i) {
    t[i].lit.type = QE_TYPE_FLOAT64;
    const double d = i == 1 ? 0.05 : 0.07;
    memcpy(&t[i].lit.bits, &d, 8);
  }
  Plan P;
  bool col_f64[QE_MAX_COLS];
  if (compile_inputs(cols, 7, -1, 4, t, &P, col_f64) != QE_OK) return 1;
  P.key_mode = 2;
  P.nkeys = 2;
  P.key_col[0] = 4;
  P.key_col[1] = 5;
  P.key_shift[0] = 0;
  P.key_fmask[0] = 0xFF;
  P.key_nullbit[0] = 8;
  P.key_shift[1] = 9;
  P.key_fmask[1] = 0xFF;
  P.key_nullbit[1] = 17;
  auto tok = [](int op, int arg, double lit) {
    qe_token k;
    memset(&k, 0, sizeof k);
    k.op = op;
    k.arg = arg;
    if (op == QE_TOK_LIT) {
      k.lit.type = QE_TYPE_FLOAT64;
      memcpy(&k.lit.bits, &lit, 8);
    }
    return k;
  };
  qe_agg_program pr[5];
  memset(pr, 0, sizeof pr);
  pr[0].ntokens = 1;
  pr[0].tokens[0] = tok(QE_TOK_COL, 0, 0);
  pr[1].ntokens = 1;
  pr[1].tokens[0] = tok(QE_TOK_COL, 1, 0);
  const qe_token dp[5] = {tok(QE_TOK_COL, 1, 0), tok(QE_TOK_LIT, 0, 1.0), tok(QE_TOK_COL, 2, 0), tok(QE_TOK_SUB, 0, 0),
                          tok(QE_TOK_MUL, 0, 0)};
  pr[2].ntokens = 5;
  for (int i = 0; i < 5; ++i) pr[2].tokens[i] = dp[i];
  pr[3] = pr[2];
  pr[3].ntokens = 9;
  pr[3].tokens[5] = tok(QE_TOK_LIT, 0, 1.0);
  pr[3].tokens[6] = tok(QE_TOK_COL, 3, 0);
  pr[3].tokens[7] = tok(QE_TOK_ADD, 0, 0);
  pr[3].tokens[8] = tok(QE_TOK_MUL, 0, 0);
  pr[4] = pr[1];
  const int fns[6] = {QE_AGG_SUM, QE_AGG_SUM, QE_AGG_SUM, QE_AGG_SUM, QE_AGG_AVG, QE_AGG_COUNT_STAR};
  const int accs[6] = {ACC_SUM_I, ACC_SUM_X, ACC_SUM_X, ACC_SUM_X, ACC_SUM_X, ACC_NONE};
  P.naggs = 6;
  for (int j = 0; j < 6; ++j) {
    memset(&P.aggs[j], 0, sizeof P.aggs[j]);
    if (j < 5) {
      bool is_f = false, nullable = false;
      if (compile_program(cols, 7, col_f64, pr[j], j, &P.aggs[j], &is_f, &nullable) != QE_OK) return 1;
      P.aggs[j].pkind = P.aggs[j].ntok == 1 ? 1 : 2;
      P.aggs[j].col = P.aggs[j].tok[0].arg;
    }
    P.aggs[j].fn = fns[j];
    P.aggs[j].acc = accs[j];
  }
  P.aggs[4].share = 2;  // AVG(l_extendedprice) reads SUM(l_extendedprice)'s accumulator
  std::string src;
  size_t lds = 0;
  if (!gen_fused_source(P, 8, &src, &lds, false)) return 1;
  return write_src(dir, "c5_fused1", src);
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  static int64_t dummy[64];
  qe_column cols[3];
  memset(cols, 0, sizeof cols);
  for (int c = 0; c < 3; ++c) {
    cols[c].type = QE_TYPE_INT64;
    cols[c].length = 1000;
    cols[c].values = dummy;
  }
  // C2: a > 2^19, project a + b
  qe_pred_term t0 = term(0, QE_OP_GT, 1 << 19);
  qe_agg_program add;
  memset(&add, 0, sizeof add);
  add.ntokens = 3;
  add.tokens[0].op = QE_TOK_COL;
  add.tokens[0].arg = 0;
  add.tokens[1].op = QE_TOK_COL;
  add.tokens[1].arg = 1;
  add.tokens[2].op = QE_TOK_ADD;
  int rc = emit(argv[1], "c2", cols, 2, &t0, 1, &add, 1);
  // nullable inputs, two outputs (a + b, c), two predicate terms
  static uint8_t vdummy[64];
  cols[1].validity = vdummy;
  qe_pred_term t2[2] = {term(0, QE_OP_GT, 5), term(2, QE_OP_LE, 100)};
  qe_agg_program outs[2];
  outs[0] = add;
  memset(&outs[1], 0, sizeof outs[1]);
  outs[1].ntokens = 1;
  outs[1].tokens[0].op = QE_TOK_COL;
  outs[1].tokens[0].arg = 2;
  rc |= emit(argv[1], "nullable", cols, 3, t2, 2, outs, 2);
  // C4: SELECT k, SUM(a+b), COUNT(*), MIN(a), MAX(b) WHERE a > 2^19 GROUP BY k (slots k, a, b)
  cols[1].validity = nullptr;
  qe_pred_term t4 = term(1, QE_OP_GT, 1 << 19);
  qe_agg_program ab = add, pa, pb;
  ab.tokens[0].arg = 1;
  ab.tokens[1].arg = 2;
  memset(&pa, 0, sizeof pa);
  pa.ntokens = 1;
  pa.tokens[0].op = QE_TOK_COL;
  pa.tokens[0].arg = 1;
  pb = pa;
  pb.tokens[0].arg = 2;
  const AggIn c4[4] = {{QE_AGG_SUM, ACC_SUM_I, &ab}, {QE_AGG_COUNT_STAR, ACC_NONE, nullptr},
                       {QE_AGG_MIN, ACC_MIN_I, &pa}, {QE_AGG_MAX, ACC_MAX_I, &pb}};
  rc |= emit_agg(argv[1], "c4", cols, 3, &t4, 1, c4, 4, 12);
  // nullable key and an fp64 MAX (records carry flags and the global row index)
  static double fdummy[64];
  cols[0].validity = vdummy;
  cols[2].type = QE_TYPE_FLOAT64;
  cols[2].values = fdummy;
  cols[2].validity = vdummy;
  const AggIn fx[2] = {{QE_AGG_MAX, ACC_MAX_F, &pb}, {QE_AGG_COUNT_STAR, ACC_NONE, nullptr}};
  rc |= emit_agg(argv[1], "f64max", cols, 3, &t4, 1, fx, 2, 11);
  // deterministic state: fp64 SUM and AVG in exact fixed point (ACC_SUM_X)
  const AggIn dx[3] = {{QE_AGG_SUM, ACC_SUM_X, &pb}, {QE_AGG_AVG, ACC_SUM_X, &pb}, {QE_AGG_COUNT_STAR, ACC_NONE, nullptr}};
  rc |= emit_agg(argv[1], "det", cols, 3, &t4, 1, dx, 3, 10);
  rc |= emit_c5(argv[1]);
  return rc;
}
