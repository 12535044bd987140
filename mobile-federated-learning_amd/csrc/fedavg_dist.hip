// fedavg_dist.hip -- the post-aggregate client distance pass
// (fedavg_trainer.py:291) of libfedavg_amd.so.
#include "common.hpp"

namespace {
using namespace fedavg_impl;

// ---------------------------------------------------------------------------
// Post-aggregate client distances (fedavg_trainer.py:291): for every client i
//   sumsq[i] = sum_p fl32(x_i[p] - g[p])^2
// with the difference formed in fp32 exactly as the reference's
// `w[para] - w_glob[para]` forms it, each square exact in fp64 and the sum in
// fp64 (deterministic order: per-wave partials, then a fixed-order finalize).
// The reference's ATen fp32 norm accumulates in fp32 SIMD lanes; this is the
// accurate value it approximates.  HBM-read bound like the reduce: 4K+4 B per
// element.  Thread = C 16-B column slices (slice j at base + tid + 256j).
// ---------------------------------------------------------------------------
constexpr int kDistCols = 4;
constexpr int kDistRows = 4;

__device__ __forceinline__ double sq4(f32x4 d) {
  return static_cast<double>(d.x) * d.x + static_cast<double>(d.y) * d.y + static_cast<double>(d.z) * d.z +
         static_cast<double>(d.w) * d.w;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(kBlock) void client_sqdist_f32x4_kernel(
    const f32x4* __restrict__ X, int K, int64_t ld4, int64_t nvec, int tail, const f32x4* __restrict__ G,
    double* __restrict__ partials, int64_t nwaves) {
  constexpr int C = kDistCols;
  const int lane = threadIdx.x & 63;
  const int64_t wave_id = static_cast<int64_t>(blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6);
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kBlock * C + threadIdx.x;
  f32x4 g[C];
  int nv[C];  // valid elements of slice j (0..4): padding lanes never contribute
  bool valid[C];
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const int64_t v = base + static_cast<int64_t>(j) * kBlock;
    valid[j] = v < nvec;
    g[j] = valid[j] ? G[v] : f32x4{0.f, 0.f, 0.f, 0.f};
    nv[j] = !valid[j] ? 0 : (tail != 0 && v == nvec - 1 ? tail : 4);
  }
  const f32x4* col = X + base;
  int k = 0;
  for (; k < K; k += kDistRows) {
    const int rows = (K - k) < kDistRows ? (K - k) : kDistRows;
    f32x4 xs[kDistRows][C];
#pragma unroll
    for (int u = 0; u < kDistRows; ++u)
#pragma unroll
      for (int j = 0; j < C; ++j)
        xs[u][j] = (u < rows && valid[j]) ? ld<true>(col + static_cast<int64_t>(k + u) * ld4 + j * kBlock) : g[j];
#pragma unroll
    for (int u = 0; u < kDistRows; ++u) {
      if (u >= rows) break;
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < C; ++j) {
        f32x4 d = xs[u][j] - g[j];  // fp32 difference, as the reference forms it
        if (nv[j] < 4) {            // select (not multiply): padding may hold NaN/inf
          d.x = nv[j] > 0 ? d.x : 0.f;
          d.y = nv[j] > 1 ? d.y : 0.f;
          d.z = nv[j] > 2 ? d.z : 0.f;
          d.w = 0.f;
        }
        acc += sq4(d);
      }
      acc = wave_sum(acc);
      if (lane == 0) partials[static_cast<int64_t>(k + u) * nwaves + wave_id] = acc;
    }
  }
}

// sumsq[k] = sum over waves of partials[k][*], fixed order (block per client).
__global__ __launch_bounds__(kBlock) void client_sqdist_finalize_kernel(const double* __restrict__ partials,
                                                                        int64_t nwaves, double* __restrict__ out) {
  __shared__ double red[kBlock];
  const int64_t k = blockIdx.x;
  double s = 0.0;
  for (int64_t w = threadIdx.x; w < nwaves; w += kBlock) s += partials[k * nwaves + w];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = kBlock / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[k] = red[0];
}

int64_t sqdist_waves(int64_t P) {
  const int64_t nvec = (P + 3) / 4;
  const int64_t blocks = (nvec + kBlock * kDistCols - 1) / (kBlock * kDistCols);
  return blocks * (kBlock / 64);
}

}  // namespace

extern "C" {

int64_t fedavg_client_sqdist_workspace(int64_t K, int64_t P) {
  if (K <= 0 || P <= 0) return 0;
  return K * sqdist_waves(P);
}

int fedavg_client_sqdist_f32(const float* clients, int64_t K, int64_t P, int64_t ld, const float* glob,
                             double* workspace, int64_t workspace_elems, double* sumsq, void* stream) {
  const char* what = "fedavg_client_sqdist_f32";
  int rc = check_common(clients, K, P, ld, glob, sumsq, what);
  if (rc) return rc;
  if (P == 0) return set_error(FEDAVG_EINVAL, "%s: P must be >= 1", what);
  if (!aligned16(clients) || !aligned16(glob) || (ld % 4) != 0)
    return set_error(FEDAVG_EALIGN, "%s: needs 16-B aligned clients/glob and ld %% 4 == 0", what);
  const int64_t nwaves = sqdist_waves(P);
  if (!workspace || workspace_elems < K * nwaves)
    return set_error(FEDAVG_EINVAL, "%s: workspace needs %lld doubles", what, (long long)(K * nwaves));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t nvec = (P + 3) / 4;
  hipLaunchKernelGGL(client_sqdist_f32x4_kernel, dim3(static_cast<unsigned>(nwaves / (kBlock / 64))), dim3(kBlock),
                     0, s, reinterpret_cast<const f32x4*>(clients), static_cast<int>(K), ld / 4, nvec,
                     static_cast<int>(P & 3), reinterpret_cast<const f32x4*>(glob), workspace, nwaves);
  rc = launch_status(what);
  if (rc) return rc;
  hipLaunchKernelGGL(client_sqdist_finalize_kernel, dim3(static_cast<unsigned>(K)), dim3(kBlock), 0, s, workspace,
                     nwaves, sumsq);
  return launch_status(what);
}

}  // extern "C"
