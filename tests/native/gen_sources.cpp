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
  return 0;
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
  return rc;
}
