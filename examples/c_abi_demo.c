/*
 * c_abi_demo.c -- drive libfedavg_amd.so from plain C (no Python, no torch),
 * the way a non-Python host would bind the drop-in boundary.
 *
 *   gcc -O2 -ffp-contract=off -I include -I /opt/rocm/include -D__HIP_PLATFORM_AMD__ \
 *       examples/c_abi_demo.c -o examples/c_abi_demo \
 *       -L mobile-federated-learning_amd/lib -lfedavg_amd -L /opt/rocm/lib -lamdhip64 \
 *       -Wl,-rpath,$PWD/mobile-federated-learning_amd/lib -Wl,-rpath,/opt/rocm/lib
 *   ./examples/c_abi_demo [K] [P]
 *
 * Builds K synthetic clients, forms the weights with fedavg_weights_f32
 * (fedavg_trainer.py:444-447,453), reduces with fedavg_reduce_f32
 * (:450-457) and checks every element bit for bit against a scalar C loop in
 * the reference's order (no FMA: compile with -ffp-contract=off); then runs
 * the :291 distance pass and checks it against an fp64 C loop.
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fedavg_amd.h"

#define HIP_OK(x)                                                                \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 2;                                                                  \
    }                                                                            \
  } while (0)

static uint64_t rng = 88172645463325252ull;
static float urand(void) {  /* xorshift64 -> [-0.05, 0.05) */
  rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
  return (float)((double)(rng >> 11) / 9007199254740992.0 - 0.5) * 0.1f;
}

int main(int argc, char** argv) {
  const int64_t K = argc > 1 ? atoll(argv[1]) : 37;
  const int64_t P = argc > 2 ? atoll(argv[2]) : 1000003;
  const int64_t ld = (P + 63) / 64 * 64;
  printf("fedavg_abi_version=%d K=%lld P=%lld\n", fedavg_abi_version(), (long long)K, (long long)P);

  float* x = (float*)malloc(sizeof(float) * K * ld);
  int64_t* n = (int64_t*)malloc(sizeof(int64_t) * K);
  float* w = (float*)malloc(sizeof(float) * K);
  float* out = (float*)malloc(sizeof(float) * P);
  float* ref = (float*)malloc(sizeof(float) * P);
  double* sumsq = (double*)malloc(sizeof(double) * K);
  for (int64_t i = 0; i < K * ld; ++i) x[i] = urand();
  for (int64_t i = 0; i < K; ++i) n[i] = 1 + (int64_t)(rng % 1000);

  if (fedavg_weights_f32(n, K, w) != 0) { fprintf(stderr, "weights: %s\n", fedavg_last_error()); return 1; }

  float *dx, *dw, *dout;
  double *dws, *dsq;
  hipStream_t s;
  const int64_t nws = fedavg_client_sqdist_workspace(K, P);
  HIP_OK(hipStreamCreate(&s));
  HIP_OK(hipMalloc((void**)&dx, sizeof(float) * K * ld));
  HIP_OK(hipMalloc((void**)&dw, sizeof(float) * K));
  HIP_OK(hipMalloc((void**)&dout, sizeof(float) * P));
  HIP_OK(hipMalloc((void**)&dws, sizeof(double) * nws));
  HIP_OK(hipMalloc((void**)&dsq, sizeof(double) * K));
  HIP_OK(hipMemcpyAsync(dx, x, sizeof(float) * K * ld, hipMemcpyHostToDevice, s));
  HIP_OK(hipMemcpyAsync(dw, w, sizeof(float) * K, hipMemcpyHostToDevice, s));

  int rc = fedavg_reduce_f32(dx, K, P, ld, dw, dout, (void*)s);
  if (rc) { fprintf(stderr, "reduce rc=%d: %s\n", rc, fedavg_last_error()); return 1; }
  rc = fedavg_client_sqdist_f32(dx, K, P, ld, dout, dws, nws, dsq, (void*)s);
  if (rc) { fprintf(stderr, "sqdist rc=%d: %s\n", rc, fedavg_last_error()); return 1; }
  HIP_OK(hipMemcpyAsync(out, dout, sizeof(float) * P, hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(sumsq, dsq, sizeof(double) * K, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));

  /* reference order: acc = x0*w0; acc = acc + xi*wi (fedavg_trainer.py:455-457) */
  int64_t bad = 0;
  for (int64_t p = 0; p < P; ++p) {
    float acc = x[p] * w[0];
    for (int64_t i = 1; i < K; ++i) {
      const float t = x[i * ld + p] * w[i];
      acc = acc + t;
    }
    ref[p] = acc;
    if (memcmp(&acc, &out[p], sizeof(float)) != 0) ++bad;
  }
  double worst = 0.0;
  for (int64_t i = 0; i < K; ++i) {
    double e = 0.0;
    for (int64_t p = 0; p < P; ++p) {
      const float d = x[i * ld + p] - ref[p];
      e += (double)d * d;
    }
    const double rel = fabs(sumsq[i] - e) / (e > 0 ? e : 1.0);
    if (rel > worst) worst = rel;
  }
  printf("reduce: %lld / %lld elements differ (bit-exact check)\n", (long long)bad, (long long)P);
  printf("sqdist: max relative error vs fp64 C loop %.3e\n", worst);
  hipFree(dx); hipFree(dw); hipFree(dout); hipFree(dws); hipFree(dsq);
  hipStreamDestroy(s);
  const int ok = bad == 0 && worst < 1e-12;
  printf("%s\n", ok ? "C ABI demo OK" : "C ABI demo FAILED");
  return ok ? 0 : 1;
}
