// abi_check.cpp — drives librr's C-ABI host logic under AddressSanitizer
// (sanitizers on the host side; the GPU pool runs no GPU ASan).
// Built by tests/asan/build.sh against a librr whose HOST code carries
// -fsanitize=address (hipcc -Xarch_host -fsanitize=address); device code is
// unchanged.
//   abi_check cpu : null-handle / bad-device rejection on every entry point,
//                   workspace-size arithmetic at extreme shapes (no GPU needed)
//   abi_check gpu : a real handle: argument validation of every entry point
//                   (bad shapes, null and misaligned pointers, short
//                   workspaces), tuning keys, then small end-to-end calls
//                   (cosine top-k, prefilter, merge, conv, GeM, L2) on the device
// Exit 0 = every expectation held and ASan reported nothing.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/rr.h"

static int g_fail = 0;
#define EXPECT(cond)                                                        \
  do {                                                                      \
    if (!(cond)) {                                                          \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_fail;                                                             \
    }                                                                       \
  } while (0)

static void cpu_checks() {
  EXPECT(std::strstr(rr_version(), "gfx950") != nullptr);
  rr_handle_t h = nullptr;
  EXPECT(rr_create(-1, &h) != RR_OK && h == nullptr);
  EXPECT(rr_create(1 << 20, &h) != RR_OK && h == nullptr);
  EXPECT(rr_create(0, nullptr) == RR_EINVAL);
  EXPECT(rr_destroy(nullptr) == RR_EINVAL);
  EXPECT(std::strlen(rr_last_error(nullptr)) > 0);
  int dev = -5;
  EXPECT(rr_get_device(nullptr, &dev) == RR_EINVAL && dev == -5);
  EXPECT(rr_set_tuning(nullptr, RR_TUNE_S3_CFG, 1) == RR_EINVAL);
  EXPECT(rr_timing_enable(nullptr, 1) == RR_EINVAL);
  EXPECT(rr_timing_collect(nullptr, 0, nullptr, nullptr) == RR_EINVAL);
  // every compute entry rejects a null handle before touching anything
  EXPECT(rr_cosine_topk(nullptr, nullptr, 1, nullptr, 1, 4, 1, 0, nullptr, nullptr, nullptr, 0, nullptr) == RR_EINVAL);
  EXPECT(rr_cosine_scores(nullptr, nullptr, 1, nullptr, 1, 4, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_topk_merge(nullptr, nullptr, nullptr, 1, 1, 1, 1, nullptr, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_quantize_rows(nullptr, nullptr, 1, 8, 1, nullptr, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_cosine_topk_lp(nullptr, nullptr, nullptr, 1, nullptr, nullptr, 1, 8, 1, 1, 0, nullptr, nullptr, nullptr, 0,
                           nullptr) == RR_EINVAL);
  EXPECT(rr_alpha_qe(nullptr, nullptr, 1, nullptr, 1, 4, nullptr, nullptr, 1, 1, 3.f, 0, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_prefilter_gallery_bound(nullptr, nullptr, nullptr, 1, 8, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_cosine_topk_prefilter(nullptr, nullptr, 1, nullptr, nullptr, nullptr, 1, 8, 1, 0, nullptr, nullptr, nullptr,
                                  0, nullptr) == RR_EINVAL);
  EXPECT(rr_pcaw_gram(nullptr, nullptr, 1, 4, nullptr, 0, nullptr, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_preprocess_u8(nullptr, nullptr, 1, 1, 1, nullptr, nullptr, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_preprocess_u8_ex(nullptr, nullptr, 1, 1, 1, nullptr, nullptr, 4, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_nchw_to_nhwc(nullptr, nullptr, 1, 1, 1, 1, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_nchw_to_nhwc_ex(nullptr, nullptr, 1, 1, 1, 1, 1, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_conv2d(nullptr, nullptr, 1, 1, 1, 1, nullptr, nullptr, 1, 1, 1, 1, 0, nullptr, 0, nullptr, nullptr) ==
         RR_EINVAL);
  EXPECT(rr_resize_bilinear(nullptr, nullptr, 1, 1, 1, 1, 1, 1, 0.f, 0.f, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_maxpool2d(nullptr, nullptr, 1, 1, 1, 1, 3, 2, 1, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_gem_pool(nullptr, nullptr, 1, 1, 1, 3.f, 1e-6f, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_l2_normalize(nullptr, nullptr, 1, 4, 1e-12f, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_linear(nullptr, nullptr, 1, 4, nullptr, nullptr, 1, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_linear_ex(nullptr, nullptr, 1, 4, nullptr, nullptr, 1, nullptr, 0, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_linear_bf16(nullptr, nullptr, 1, 8, nullptr, nullptr, 1, nullptr, 0, 0, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_layernorm(nullptr, nullptr, 4, 1, 4, nullptr, nullptr, 1e-5f, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_layernorm_ex(nullptr, nullptr, 4, 1, 4, nullptr, nullptr, 1e-5f, 0, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_patchify(nullptr, nullptr, 1, 16, 16, 3, 16, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_vit_tokens(nullptr, nullptr, 1, 1, 4, nullptr, nullptr, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_attention(nullptr, nullptr, 1, 1, 1, 64, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_attention_ex(nullptr, nullptr, 1, 1, 1, 64, 0, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_attention_bf16(nullptr, nullptr, 1, 1, 1, 64, 0, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_attention_bf16_qkv16(nullptr, nullptr, 1, 1, 1, 64, 0, nullptr, nullptr) == RR_EINVAL);
  // workspace arithmetic: worst-case candidate buffers at extreme shapes, no overflow
  const size_t w1 = rr_cosine_topk_workspace_size(4096, 200000000LL, 2048, 16384);
  EXPECT(w1 >= (size_t)4096 * (200000000ULL - 32768 + 16384) * 8);
  EXPECT(rr_cosine_topk_workspace_size(0, 10, 4, 1) >= 256);
  EXPECT(rr_cosine_topk_workspace_size(1, 0, 4, 1) > 0);
  const size_t w2 = rr_cosine_topk_prefilter_workspace_size(1280, 1600000, 2048, 100);
  EXPECT(w2 >= (size_t)1280 * 1600000 * 8);
  EXPECT(rr_cosine_topk_prefilter_workspace_size(-1, 10, 8, 1) == 0);
  EXPECT(rr_pcaw_gram_workspace_size(1600000, 2048) > (size_t)2048 * 2048 * 8);
  EXPECT(rr_pcaw_gram_workspace_size(-1, 8) == 0);
}

#define HIPCHK(x)                                                               \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(3);                                                             \
    }                                                                           \
  } while (0)

template <class T>
static T* dmalloc(size_t n) {
  void* p = nullptr;
  HIPCHK(hipMalloc(&p, n * sizeof(T) + 64));
  return (T*)p;
}

static void gpu_checks() {
  rr_handle_t h = nullptr;
  EXPECT(rr_create(0, &h) == RR_OK && h != nullptr);
  if (!h) return;
  int dev = -1;
  EXPECT(rr_get_device(h, &dev) == RR_OK && dev == 0);
  EXPECT(rr_set_tuning(h, 42, 1) == RR_EINVAL && std::strstr(rr_last_error(h), "unknown key"));
  EXPECT(rr_set_tuning(h, RR_TUNE_GEMM_CFG, 23) == RR_EINVAL);
  EXPECT(rr_set_tuning(h, RR_TUNE_S3_CFG, 6) == RR_OK && rr_set_tuning(h, RR_TUNE_S3_CFG, 0) == RR_OK);
  EXPECT(rr_timing_collect(h, 99, nullptr, nullptr) == RR_EINVAL);

  const int nq = 5, n = 9000, d = 64, k = 20;
  std::vector<float> hq(nq * d), hg((size_t)n * d);
  srand(7);
  for (auto& v : hq) v = (float)rand() / RAND_MAX - 0.5f;
  for (auto& v : hg) v = (float)rand() / RAND_MAX - 0.5f;
  float* q = dmalloc<float>(hq.size());
  float* g = dmalloc<float>(hg.size());
  HIPCHK(hipMemcpy(q, hq.data(), hq.size() * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(g, hg.data(), hg.size() * 4, hipMemcpyHostToDevice));
  float* os = dmalloc<float>(nq * k);
  long long* oi = dmalloc<long long>(nq * k);
  const size_t ws_n = rr_cosine_topk_workspace_size(nq, n, d, k);
  char* ws = dmalloc<char>(ws_n);
  // argument validation (never launches)
  EXPECT(rr_cosine_topk(h, q, nq, g, n, 6, k, 0, os, oi, ws, ws_n, nullptr) == RR_EINVAL);      // d % 4
  EXPECT(rr_cosine_topk(h, q, nq, g, n, d, 0, 0, os, oi, ws, ws_n, nullptr) == RR_EINVAL);      // k
  EXPECT(rr_cosine_topk(h, q, nq, g, n, d, 20000, 0, os, oi, ws, ws_n, nullptr) == RR_EINVAL);  // k > 16384
  const size_t ws_min = rr_cosine_topk_workspace_size_cap(nq, n, d, k, k);  // bounded: k candidates per query
  EXPECT(ws_min > 0 && ws_min < ws_n && rr_cosine_topk_cap_for(nq, n, d, k, ws_n) > k);
  EXPECT(rr_cosine_topk(h, q, nq, g, n, d, k, 0, os, oi, ws, ws_min - 1, nullptr) == RR_EWORKSPACE);
  EXPECT(rr_cosine_topk(h, q, nq, nullptr, n, d, k, 0, os, oi, ws, ws_n, nullptr) == RR_EINVAL);
  EXPECT(rr_cosine_topk(h, q + 1, nq, g, n, d, k, 0, os, oi, ws, ws_n, nullptr) == RR_EINVAL);  // misaligned
  EXPECT(rr_cosine_topk(h, q, nq, g, 0x100000000LL, d, k, 0, os, oi, ws, ws_n, nullptr) == RR_EINVAL);
  EXPECT(rr_conv2d(h, q, 1, 4, 4, 4, g, nullptr, 8, 9, 9, 1, 0, nullptr, 0, os, nullptr) == RR_EINVAL);  // empty out
  EXPECT(rr_alpha_qe(h, q, nq, g, n, d, oi, os, k, k + 1, 3.f, 0, q, nullptr) == RR_EINVAL);  // n > k
  EXPECT(rr_topk_merge(h, os, oi, 0, nq, k, k, os, oi, nullptr) == RR_EINVAL);
  EXPECT(rr_quantize_rows(h, q, nq, d, 3, g, nullptr, nullptr) == RR_EINVAL);
  EXPECT(rr_layernorm_ex(h, q, d, nq, d, nullptr, nullptr, 1e-5f, 7, g, nullptr) == RR_EINVAL);
  // small real calls
  EXPECT(rr_l2_normalize(h, q, nq, d, 1e-12f, q, nullptr) == RR_OK);
  EXPECT(rr_l2_normalize(h, g, n, d, 1e-12f, g, nullptr) == RR_OK);
  EXPECT(rr_cosine_topk(h, q, nq, g, n, d, k, 100, os, oi, ws, ws_n, nullptr) == RR_OK);
  std::vector<long long> hi(nq * k);
  std::vector<float> hs(nq * k);
  HIPCHK(hipMemcpy(hi.data(), oi, hi.size() * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(hs.data(), os, hs.size() * 4, hipMemcpyDeviceToHost));
  for (int i = 0; i < nq; ++i)
    for (int r = 0; r + 1 < k; ++r) EXPECT(hs[i * k + r] >= hs[i * k + r + 1] && hi[i * k + r] >= 100);
  // bounded workspaces: room for 400 candidates per query is plenty here (no
  // overflow, same result); room for k is not (the overflow int counts it)
  {
    int ovf = -1;
    const size_t b400 = rr_cosine_topk_workspace_size_cap(nq, n, d, k, 400);
    // (the 256-B rounding of the workspace may leave room for a few more)
    const long long c400 = rr_cosine_topk_cap_for(nq, n, d, k, b400);
    EXPECT(c400 >= 400 && rr_cosine_topk_workspace_size_cap(nq, n, d, k, c400) == b400);
    EXPECT(rr_cosine_topk(h, q, nq, g, n, d, k, 100, os, oi, ws, b400, nullptr) == RR_OK);
    HIPCHK(hipMemcpy(&ovf, ws + rr_cosine_topk_overflow_offset(nq, n, d, k), 4, hipMemcpyDeviceToHost));
    std::vector<long long> hb(nq * k);
    HIPCHK(hipMemcpy(hb.data(), oi, hb.size() * 8, hipMemcpyDeviceToHost));
    EXPECT(ovf == 0 && hb == hi);
    EXPECT(rr_cosine_topk(h, q, nq, g, n, d, k, 100, os, oi, ws, ws_min, nullptr) == RR_OK);
    HIPCHK(hipMemcpy(&ovf, ws + rr_cosine_topk_overflow_offset(nq, n, d, k), 4, hipMemcpyDeviceToHost));
    EXPECT(ovf > 0 && ovf <= nq);
    EXPECT(rr_cosine_topk(h, q, nq, g, n, d, k, 100, os, oi, ws, ws_n, nullptr) == RR_OK);  // restore os / oi
  }
  uint16_t* gb = dmalloc<uint16_t>((size_t)n * d);
  double* b3 = dmalloc<double>(3);
  EXPECT(rr_quantize_rows(h, g, n, d, 1, gb, nullptr, nullptr) == RR_OK);
  EXPECT(rr_prefilter_gallery_bound(h, g, gb, n, d, b3, nullptr) == RR_OK);
  const size_t pw_n = rr_cosine_topk_prefilter_workspace_size(nq, n, d, k);
  char* pws = dmalloc<char>(pw_n);
  float* os2 = dmalloc<float>(nq * k);
  long long* oi2 = dmalloc<long long>(nq * k);
  const size_t pw_min = rr_cosine_topk_prefilter_workspace_size_cap(nq, n, d, k, k);
  EXPECT(rr_cosine_topk_prefilter(h, q, nq, g, gb, b3, n, d, k, 100, os2, oi2, pws, pw_min - 8, nullptr) ==
         RR_EWORKSPACE);
  EXPECT(rr_cosine_topk_prefilter(h, q, nq, g, gb, b3, n, d, k, 100, os2, oi2, pws, pw_n, nullptr) == RR_OK);
  std::vector<long long> hi2(nq * k);
  HIPCHK(hipMemcpy(hi2.data(), oi2, hi2.size() * 8, hipMemcpyDeviceToHost));
  EXPECT(hi2 == hi);
  EXPECT(rr_topk_merge(h, os, oi, 1, nq, k, k / 2, os2, oi2, nullptr) == RR_OK);
  // a small conv + GeM
  float* x = dmalloc<float>(2 * 8 * 8 * 32);
  float* w = dmalloc<float>(64 * 9 * 32);
  float* y = dmalloc<float>(2 * 8 * 8 * 64);
  float* gp = dmalloc<float>(2 * 64);
  HIPCHK(hipMemset(x, 0, 2 * 8 * 8 * 32 * 4));
  HIPCHK(hipMemset(w, 0, 64 * 9 * 32 * 4));
  EXPECT(rr_conv2d(h, x, 2, 8, 8, 32, w, nullptr, 64, 3, 3, 1, 1, nullptr, 1, y, nullptr) == RR_OK);
  EXPECT(rr_gem_pool(h, y, 2, 64, 64, 3.f, 1e-6f, gp, nullptr) == RR_OK);
  EXPECT(rr_timing_enable(h, 1) == RR_OK);
  EXPECT(rr_l2_normalize(h, g, n, d, 1e-12f, g, nullptr) == RR_OK);
  double ms = -1;
  long long nl = -1;
  EXPECT(rr_timing_collect(h, 3, &ms, &nl) == RR_OK && nl == 1 && ms >= 0);
  HIPCHK(hipDeviceSynchronize());
  for (void* p : {(void*)q, (void*)g, (void*)os, (void*)oi, (void*)ws, (void*)gb, (void*)b3, (void*)pws, (void*)os2,
                  (void*)oi2, (void*)x, (void*)w, (void*)y, (void*)gp})
    HIPCHK(hipFree(p));
  EXPECT(rr_destroy(h) == RR_OK);
}

int main(int argc, char** argv) {
  const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
  cpu_checks();
  if (gpu) gpu_checks();
  std::printf("abi_check %s: %s (%d failures)\n", gpu ? "gpu" : "cpu", g_fail ? "FAILED" : "ok", g_fail);
  return g_fail ? 1 : 0;
}
