/*
 * oracle/cosine_topk.c — TEST INFRASTRUCTURE ONLY (the parity checker).
 *
 * CPU restatement of the reference ranker, iris_evaluate.py:383-386
 * (src/benchmark/):
 *     similarity = torch.mm(query_features, gallery_features.t())   # :383
 *     ranks = np.argsort(-similarity, axis=1)                        # :386
 * with two deliberate, documented refinements:
 *   - the ranking order is STABLE: score descending, then gallery index
 *     ascending (np.argsort's default kind is not stable on AVX-512 hosts);
 *   - each score is the fp32 dot product evaluated as the fixed fmaf chain
 *     librr's MFMA kernel performs (v_mfma_f32_32x32x2_f32 accumulates
 *     k-ordered, one rounding per product): within every 16-deep chunk c of
 *     the descriptor, k = 16c+0, 16c+8, 16c+1, 16c+9, ..., 16c+7, 16c+15.
 *     `order` = 1 selects the alternative lane-half order (16c+8 first) and
 *     `order` = 2 a plain sequential chain k = 0..d-1, for diagnosis.
 * Torch's own sgemm order is unspecified; the golden fixtures (tests/golden/,
 * produced by the reference's op sequence) pin these scores within 1e-5 and
 * the ranks up to near-ties.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library; the product path never does.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static float dot_mfma_order(const float* a, const float* b, int d, int order) {
  float acc = 0.0f;
  if (order == 2) {
    for (int k = 0; k < d; ++k) acc = fmaf(a[k], b[k], acc);
    return acc;
  }
  const int nchunk = (d + 15) / 16;
  for (int c = 0; c < nchunk; ++c) {
    for (int e = 0; e < 8; ++e) {
      const int k0 = 16 * c + e, k1 = 16 * c + 8 + e;
      const float a0 = k0 < d ? a[k0] : 0.0f, b0 = k0 < d ? b[k0] : 0.0f;
      const float a1 = k1 < d ? a[k1] : 0.0f, b1 = k1 < d ? b[k1] : 0.0f;
      if (order == 0) {
        acc = fmaf(a0, b0, acc);
        acc = fmaf(a1, b1, acc);
      } else {
        acc = fmaf(a1, b1, acc);
        acc = fmaf(a0, b0, acc);
      }
    }
  }
  return acc;
}

/* scores[i][j] = <q_i, g_j>, [nq][n] */
void rr_oracle_scores(const float* q, int nq, const float* g, long long n, int d, int order, float* scores) {
  for (int i = 0; i < nq; ++i)
    for (long long j = 0; j < n; ++j) scores[(long long)i * n + j] = dot_mfma_order(q + (long long)i * d, g + j * d, d, order);
}

typedef struct {
  float s;
  long long i;
} item_t;

/* score desc, index asc; -0.0 == +0.0; NaN after every number (including
 * -inf), NaNs by index: np.argsort(-similarity, kind="stable") order
 * (iris_evaluate.py:386; numpy sorts NaN last) */
static int cmp_item(const void* pa, const void* pb) {
  const item_t* a = (const item_t*)pa;
  const item_t* b = (const item_t*)pb;
  const int na = isnan(a->s), nb = isnan(b->s);
  if (na != nb) return na ? 1 : -1;
  if (a->s > b->s) return -1;
  if (a->s < b->s) return 1;
  return (a->i < b->i) ? -1 : (a->i > b->i);
}

/* Stable top-k of each row of scores [nq][n]; rows shorter than k are padded
 * with (-inf, -1).  out_idx = column + idx_offset. */
void rr_oracle_topk_rows(const float* scores, int nq, long long n, int k, long long idx_offset, float* out_s,
                         long long* out_i) {
  item_t* buf = (item_t*)malloc(sizeof(item_t) * (size_t)(n > 0 ? n : 1));
  for (int q = 0; q < nq; ++q) {
    for (long long j = 0; j < n; ++j) {
      buf[j].s = scores[(long long)q * n + j];
      buf[j].i = j;
    }
    qsort(buf, (size_t)n, sizeof(item_t), cmp_item);
    for (int r = 0; r < k; ++r) {
      if (r < n) {
        out_s[(long long)q * k + r] = buf[r].s;
        out_i[(long long)q * k + r] = buf[r].i + idx_offset;
      } else {
        out_s[(long long)q * k + r] = -INFINITY;
        out_i[(long long)q * k + r] = -1;
      }
    }
  }
  free(buf);
}

/* Fused restatement: scores in MFMA order + stable top-k, without holding the
 * whole [nq][n] matrix (one query row at a time). */
void rr_oracle_cosine_topk(const float* q, int nq, const float* g, long long n, int d, int k, long long idx_offset,
                           int order, float* out_s, long long* out_i) {
  float* row = (float*)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
  for (int i = 0; i < nq; ++i) {
    for (long long j = 0; j < n; ++j) row[j] = dot_mfma_order(q + (long long)i * d, g + j * d, d, order);
    rr_oracle_topk_rows(row, 1, n, k, idx_offset, out_s + (long long)i * k, out_i + (long long)i * k);
  }
  free(row);
}

/* k-way merge of partial top-k lists [nparts][nq][kin] (idx < 0 = padding)
 * into the stable top-kout per query. */
void rr_oracle_topk_merge(const float* ps, const long long* pi, int nparts, int nq, int kin, int kout, float* os,
                          long long* oi) {
  item_t* buf = (item_t*)malloc(sizeof(item_t) * (size_t)nparts * kin + 1);
  for (int q = 0; q < nq; ++q) {
    long long c = 0;
    for (int p = 0; p < nparts; ++p)
      for (int r = 0; r < kin; ++r) {
        const long long o = ((long long)p * nq + q) * kin + r;
        if (pi[o] < 0) continue;
        buf[c].s = ps[o];
        buf[c].i = pi[o];
        ++c;
      }
    qsort(buf, (size_t)c, sizeof(item_t), cmp_item);
    for (int r = 0; r < kout; ++r) {
      if (r < c) {
        os[(long long)q * kout + r] = buf[r].s;
        oi[(long long)q * kout + r] = buf[r].i;
      } else {
        os[(long long)q * kout + r] = -INFINITY;
        oi[(long long)q * kout + r] = -1;
      }
    }
  }
  free(buf);
}
