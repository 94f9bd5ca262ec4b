/* oracle_check.c — the oracle's C restatement (oracle/cosine_topk.c) under
 * AddressSanitizer + UBSan: scores, stable top-k with n < k padding, NaN rows,
 * exact ties, and the k-way merge with padding entries.  Exit 0 = clean. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

void rr_oracle_scores(const float* q, int nq, const float* g, long long n, int d, int order, float* scores);
void rr_oracle_topk_rows(const float* scores, int nq, long long n, int k, long long idx_offset, float* out_s,
                         long long* out_i);
void rr_oracle_cosine_topk(const float* q, int nq, const float* g, long long n, int d, int k, long long idx_offset,
                           int order, float* out_s, long long* out_i);
void rr_oracle_topk_merge(const float* ps, const long long* pi, int nparts, int nq, int kin, int kout, float* os,
                          long long* oi);

int main(void) {
  int fail = 0;
  const int nq = 3, n = 37, d = 20, k = 50;
  float* q = malloc(sizeof(float) * nq * d);
  float* g = malloc(sizeof(float) * n * d);
  srand(3);
  for (int i = 0; i < nq * d; ++i) q[i] = (float)rand() / RAND_MAX - 0.5f;
  for (int i = 0; i < n * d; ++i) g[i] = (float)rand() / RAND_MAX - 0.5f;
  for (int j = 0; j < d; ++j) g[10 * d + j] = g[3 * d + j];  /* exact tie */
  g[5 * d + 2] = NAN;                                         /* a NaN row */
  float* sc = malloc(sizeof(float) * nq * n);
  for (int order = 0; order < 3; ++order) rr_oracle_scores(q, nq, g, n, d, order, sc);
  float* os = malloc(sizeof(float) * nq * k);
  long long* oi = malloc(sizeof(long long) * nq * k);
  rr_oracle_cosine_topk(q, nq, g, n, d, k, 7, 0, os, oi);
  for (int i = 0; i < nq; ++i) {
    if (oi[i * k + n - 1] != 5 + 7 || !isnan(os[i * k + n - 1])) fail = 1;  /* NaN row last */
    for (int r = n; r < k; ++r)
      if (oi[i * k + r] != -1 || !isinf(os[i * k + r])) fail = 1;            /* padding */
  }
  /* merge two partial lists, the second half padding */
  float* ps = malloc(sizeof(float) * 2 * nq * k);
  long long* pi = malloc(sizeof(long long) * 2 * nq * k);
  for (int p = 0; p < 2; ++p)
    for (int i = 0; i < nq * k; ++i) {
      ps[p * nq * k + i] = os[i];
      pi[p * nq * k + i] = oi[i] < 0 ? -1 : oi[i] + p * 1000;
    }
  float* ms = malloc(sizeof(float) * nq * 10);
  long long* mi = malloc(sizeof(long long) * nq * 10);
  rr_oracle_topk_merge(ps, pi, 2, nq, k, 10, ms, mi);
  for (int i = 0; i < nq; ++i)
    if (mi[i * 10] != oi[i * k] || mi[i * 10 + 1] != oi[i * k] + 1000) fail = 1;  /* equal scores: index asc */
  rr_oracle_topk_rows(sc, nq, n, 4, 0, os, oi);
  free(q); free(g); free(sc); free(os); free(oi); free(ps); free(pi); free(ms); free(mi);
  printf("oracle_check: %s\n", fail ? "FAILED" : "ok");
  return fail;
}
