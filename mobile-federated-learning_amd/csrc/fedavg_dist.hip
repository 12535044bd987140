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
// acc + the exact squares of d's four lanes, in fp64 with fused multiply-adds
// (this pass is tolerance-pinned, not bit-pinned: a fused square-add rounds
// once, so it is closer to the exact sum, and it halves the fp64 work)
__device__ __forceinline__ double sq4_add(double acc, f32x4 d) {
  const double x = d.x, y = d.y, z = d.z, w = d.w;
  acc = __builtin_fma(x, x, acc);
  acc = __builtin_fma(y, y, acc);
  acc = __builtin_fma(z, z, acc);
  return __builtin_fma(w, w, acc);
}

__device__ __forceinline__ double wave_sum(double v) { return wave_sum_dpp(v); }

// Block b of a launch covers C*256 column slices starting at slice
// b*C*256 of that launch's window; its waves write partials at global wave
// index wave_base + b*4 + wave.  U client rows are loaded per batch.
template <int U, int C>
__global__ __launch_bounds__(kBlock) void client_sqdist_f32x4_kernel(
    const f32x4* __restrict__ X, int K, int64_t ld4, int64_t nvec, int tail, const f32x4* __restrict__ G,
    double* __restrict__ partials, int64_t nwaves, int64_t wave_base) {
  const int lane = threadIdx.x & 63;
  const int64_t wave_id = wave_base + static_cast<int64_t>(blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6);
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
  for (int k = 0; k < K; k += U) {
    const int rows = (K - k) < U ? (K - k) : U;
    f32x4 xs[U][C];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < C; ++j)
        xs[u][j] = (u < rows && valid[j]) ? ld<true>(col + static_cast<int64_t>(k + u) * ld4 + j * kBlock) : g[j];
#pragma unroll
    for (int u = 0; u < U; ++u) {
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
        acc = sq4_add(acc, d);
      }
      acc = wave_sum(acc);
      if (lane == 0) partials[static_cast<int64_t>(k + u) * nwaves + wave_id] = acc;
    }
  }
}

// The same pass through buffer descriptors, split by column group.  A FULL
// group (every slice valid, no P % 4 tail) reads client row k through one
// descriptor whose base sits in SGPRs, with each lane's slice as a 32-bit
// offset shared by every row, and forms d = x - g with no masking at all --
// the reduce's register budget (reduce_f32x4_buf_kernel) plus the group's
// model slice g.  The ragged last group keeps per-slice masks and a record
// count that ends at the window's last float4 (lanes past it read 0).  Same
// per-wave partial layout as client_sqdist_f32x4_kernel<U, C>.
template <int U, int C>
__device__ __forceinline__ void sqdist_rows_store(double acc, double* partials, int64_t row, int64_t nwaves,
                                                  int64_t wave_id) {
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) partials[row * nwaves + wave_id] = acc;
}

// sum over a row's C slices of fl32(x - g)^2 in fp64, in ACC interleaved
// chains (slice j feeds chain j % ACC, the chains add pairwise at the end):
// ACC = 1 is one dependent chain of 4C fused square-adds per row
template <int C, int ACC>
__device__ __forceinline__ double sq_row(const f32x4 (&x)[C], const f32x4 (&g)[C]) {
  double a[ACC];
#pragma unroll
  for (int i = 0; i < ACC; ++i) a[i] = 0.0;
#pragma unroll
  for (int j = 0; j < C; ++j) a[j % ACC] = sq4_add(a[j % ACC], x[j] - g[j]);  // fp32 difference, as the reference
#pragma unroll
  for (int w = 1; w < ACC; w *= 2) {
#pragma unroll
    for (int i = 0; i + w < ACC; i += 2 * w) a[i] += a[i + w];
  }
  return a[0];
}

template <int U, int C, int MINW = 1, int ACC = 1>
__global__ __launch_bounds__(kBlock, MINW) void client_sqdist_buf_kernel(
    const f32x4* __restrict__ X, int K, int64_t ld4, int64_t nvec, int tail, const f32x4* __restrict__ G,
    double* __restrict__ partials, int64_t nwaves, int64_t wave_base) {
  const int64_t wave_id = wave_base + static_cast<int64_t>(blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6);
  constexpr int64_t span = static_cast<int64_t>(kBlock) * C;
  const int64_t blk0 = static_cast<int64_t>(blockIdx.x) * span;
  uint32_t off[C];
#pragma unroll
  for (int j = 0; j < C; ++j) off[j] = 16u * (threadIdx.x + j * kBlock);
  if (blk0 + span < nvec || (blk0 + span == nvec && tail == 0)) {
    constexpr int bytes = static_cast<int>(span * 16);
    f32x4 g[C];
    {
      const __amdgpu_buffer_rsrc_t rg = uniform_rsrc(G + blk0, bytes);
#pragma unroll
      for (int j = 0; j < C; ++j) g[j] = ld_rsrc_nt(rg, off[j]);
    }
    if constexpr (U == 0) {  // one row in flight while the previous one is summed
      const auto load_row = [&](f32x4 (&x)[C], int row) {
        const __amdgpu_buffer_rsrc_t r = uniform_rsrc(X + static_cast<int64_t>(row) * ld4 + blk0, bytes);
#pragma unroll
        for (int j = 0; j < C; ++j) x[j] = ld_rsrc_nt(r, off[j]);
      };
      f32x4 a[C], b[C];
      load_row(a, 0);
      int k = 0;
      for (; k + 2 <= K; k += 2) {
        load_row(b, k + 1);
        sqdist_rows_store<1, C>(sq_row<C, ACC>(a, g), partials, k, nwaves, wave_id);
        if (k + 2 < K) load_row(a, k + 2);
        sqdist_rows_store<1, C>(sq_row<C, ACC>(b, g), partials, k + 1, nwaves, wave_id);
      }
      if (k < K) sqdist_rows_store<1, C>(sq_row<C, ACC>(a, g), partials, k, nwaves, wave_id);
      return;
    }
    constexpr int UU = U > 0 ? U : 1;
    int k = 0;
    for (; k + UU <= K; k += UU) {
      f32x4 xs[UU][C];
#pragma unroll
      for (int u = 0; u < UU; ++u) {
        const __amdgpu_buffer_rsrc_t r = uniform_rsrc(X + static_cast<int64_t>(k + u) * ld4 + blk0, bytes);
#pragma unroll
        for (int j = 0; j < C; ++j) xs[u][j] = ld_rsrc_nt(r, off[j]);
      }
#pragma unroll
      for (int u = 0; u < UU; ++u) sqdist_rows_store<U, C>(sq_row<C, ACC>(xs[u], g), partials, k + u, nwaves, wave_id);
    }
    for (; k < K; ++k) {
      const __amdgpu_buffer_rsrc_t r = uniform_rsrc(X + static_cast<int64_t>(k) * ld4 + blk0, bytes);
      f32x4 x[C];
#pragma unroll
      for (int j = 0; j < C; ++j) x[j] = ld_rsrc_nt(r, off[j]);
      sqdist_rows_store<U, C>(sq_row<C, ACC>(x, g), partials, k, nwaves, wave_id);
    }
    return;
  }
  // ragged last group: masked slices, record count ends at the last float4
  const int64_t left = nvec - blk0;
  const int bytes = static_cast<int>((left < span ? left : span) * 16);
  int nv[C];  // valid elements of slice j (0..4): padding lanes never contribute
  f32x4 g[C];
  {
    const __amdgpu_buffer_rsrc_t rg = uniform_rsrc(G + blk0, bytes);
#pragma unroll
    for (int j = 0; j < C; ++j) {
      const int64_t v = blk0 + threadIdx.x + static_cast<int64_t>(j) * kBlock;
      nv[j] = v >= nvec ? 0 : (tail != 0 && v == nvec - 1 ? tail : 4);
      g[j] = ld_rsrc_nt(rg, off[j]);
    }
  }
  for (int k = 0; k < K; ++k) {
    const __amdgpu_buffer_rsrc_t r = uniform_rsrc(X + static_cast<int64_t>(k) * ld4 + blk0, bytes);
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < C; ++j) {
      f32x4 d = ld_rsrc_nt(r, off[j]) - g[j];
      if (nv[j] < 4) {  // select (not multiply): padding may hold NaN/inf
        d.x = nv[j] > 0 ? d.x : 0.f;
        d.y = nv[j] > 1 ? d.y : 0.f;
        d.z = nv[j] > 2 ? d.z : 0.f;
        d.w = 0.f;
      }
      acc = sq4_add(acc, d);
    }
    sqdist_rows_store<U, C>(acc, partials, k, nwaves, wave_id);
  }
}

// ---------------------------------------------------------------------------
// :291 for fp64 / fp16 / bf16 keys.  `w[para] - w_glob[para]` forms the
// difference in the key's own dtype (ATen: fp64 math for fp64; fp32 opmath
// rounded to fp16/bf16 for the 16-bit types), torch.cat then widens it
// exactly to the promoted dtype, and the norm squares and sums.  Here: the
// difference with the reference's rounding, then exact-ish fp64 squares and
// sum (fused square-adds), same per-wave partial layout and fixed-order
// finalize as the fp32 pass.  16-B slices: 2 fp64 or 8 fp16/bf16 elements.
// ---------------------------------------------------------------------------
struct DistF64 {
  using vec = f64x2;
  static constexpr int kLanes = 2;
  __device__ static double sq_add(double acc, vec x, vec g, int nv) {
    const vec d = x - g;  // fp64 difference, as the reference forms it
    if (nv > 0) acc = __builtin_fma(d.x, d.x, acc);
    if (nv > 1) acc = __builtin_fma(d.y, d.y, acc);
    return acc;
  }
};

template <typename R>
struct DistHalf {
  using vec = u16x8;
  static constexpr int kLanes = 8;
  __device__ static double sq_add(double acc, vec x, vec g, int nv) {
    u32x4 xu, gu;
    __builtin_memcpy(&xu, &x, 16);
    __builtin_memcpy(&gu, &g, 16);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // fl16(fl32(x) - fl32(g)): ATen's opmath subtraction rounded to the
      // key's 16-bit type, then widened exactly
      const f32x2 d = R::unpack(R::pack(opaque2(R::unpack(xu[j]) - R::unpack(gu[j]))));
      const double a = d.x, b = d.y;
      if (2 * j < nv) acc = __builtin_fma(a, a, acc);
      if (2 * j + 1 < nv) acc = __builtin_fma(b, b, acc);
    }
    return acc;
  }
};

template <class D, int U, int C>
__global__ __launch_bounds__(kBlock) void client_sqdist_vec_kernel(
    const typename D::vec* __restrict__ X, int K, int64_t ldv, int64_t nvec, int tail,
    const typename D::vec* __restrict__ G, double* __restrict__ partials, int64_t nwaves) {
  using vec = typename D::vec;
  const int lane = threadIdx.x & 63;
  const int64_t wave_id = static_cast<int64_t>(blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6);
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kBlock * C + threadIdx.x;
  vec g[C];
  int nv[C];  // valid elements of slice j: padding lanes never contribute
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const int64_t v = base + static_cast<int64_t>(j) * kBlock;
    nv[j] = v >= nvec ? 0 : (tail != 0 && v == nvec - 1 ? tail : D::kLanes);
    g[j] = nv[j] > 0 ? G[v] : vec{};
  }
  const vec* col = X + base;
  for (int k = 0; k < K; k += U) {
    const int rows = (K - k) < U ? (K - k) : U;
    vec xs[U][C];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < C; ++j)
        xs[u][j] = (u < rows && nv[j] > 0) ? ld<true>(col + static_cast<int64_t>(k + u) * ldv + j * kBlock) : g[j];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u >= rows) break;
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < C; ++j) acc = D::sq_add(acc, xs[u][j], g[j], nv[j]);
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

// Global-pointer schedule (the fp64/fp16/bf16 passes and the probe
// variants): 32 x 16-B loads in flight per thread (U4 x C8) in one launch;
// scripts/dist_variants.py (profiles/sweeps/r01_dist_*.jsonl) measured
// round-split launches within 1 % of it and U4 x C4 6 % behind.
constexpr int kDistCols = 8;
constexpr int kDistRows = 4;
// fp32 production (fedavg_client_sqdist_f32): the buffer-descriptor kernel at
// U2 x C16 in one launch -- full column groups read each row through one
// SGPR descriptor with no masking, 64 KiB contiguous per row per block, the
// reduce's winning shape: 6,818-6,840 GB/s vs 6,520-6,531 for the
// global-pointer U4 x C8 (scripts/dist_variants.py, profiles/r02/dist_variants.jsonl).
// U4 x C8 remains the fp64/fp16/bf16 passes' schedule.  Each row's fp64 sum
// runs as 4 interleaved chains (slice j into chain j % 4, added pairwise):
// 0.9-1.5 % faster than one chain of 64 dependent square-adds in three
// interleaved runs, 8 chains no better, 16 slower; a one-row-ahead pipeline
// (U = 0) loses 5 % -- two rows in flight per wave beat compute overlap
// (profiles/r02/sweeps/dist_chains.jsonl).
constexpr int kDistBufRows = 2;
constexpr int kDistBufCols = 16;
constexpr int kDistBufChains = 4;

// fp32 production column groups per thread: 16 while that still gives two
// workgroups per CU (the 25M-column target: 1,526), else 4 while it gives
// ~one per CU, else 2.  A small model's rows are short, and at 16 slices the
// launch had 37 workgroups for resnet56 (100 x 600K) and 74 for FEMNIST
// (10 x 1.2M).  rocprofv3 kernel time (profiles/r02/sweeps/dist_small_models.json):
// resnet56 275 -> 72 us (U8 x C2), FEMNIST 30.8 -> 12.7 us (U4 x C4),
// cfg4 500 x 1M 1,383 -> 391 us (U4 x C4), 100 x 3.125M 309 -> 197 us (U4 x C4).
int dist_cols(int64_t P) {
  const int64_t nvec = (P + 3) / 4;
  const int64_t cus = cu_count();
  if ((nvec + kBlock * 16 - 1) / (kBlock * 16) >= 2 * cus) return 16;
  if ((nvec + kBlock * 4 - 1) / (kBlock * 4) >= cus * 9 / 10) return 4;
  return 2;
}

int64_t sqdist_waves_for(int64_t P, int cols) {
  const int64_t nvec = (P + 3) / 4;
  const int64_t blocks = (nvec + kBlock * cols - 1) / (kBlock * cols);
  return blocks * (kBlock / 64);
}

template <int U, int C, bool BUF = false, int MINW = 1, int ACC = 1>
void launch_sqdist(const float* clients, int K, int64_t ld, int64_t P, const float* glob, double* partials,
                   int64_t nwaves, int max_blocks, hipStream_t s) {
  const int64_t nvec = (P + 3) / 4;
  const int64_t span = static_cast<int64_t>(kBlock) * C;
  const int64_t blocks = (nvec + span - 1) / span;
  const int64_t bpl = max_blocks > 0 ? max_blocks : blocks;
  const int64_t nl = (blocks + bpl - 1) / bpl;
  const int64_t per_blocks = (blocks + nl - 1) / nl;  // equal launches, whole blocks each
  const f32x4* X = reinterpret_cast<const f32x4*>(clients);
  const f32x4* Gv = reinterpret_cast<const f32x4*>(glob);
  for (int64_t b0 = 0; b0 < blocks; b0 += per_blocks) {
    const int64_t nb = (blocks - b0) < per_blocks ? (blocks - b0) : per_blocks;
    const int64_t v0 = b0 * span;
    const int64_t n = (nvec - v0) < nb * span ? (nvec - v0) : nb * span;
    const int tail = (v0 + n == nvec) ? static_cast<int>(P & 3) : 0;
    if constexpr (BUF)
      hipLaunchKernelGGL((client_sqdist_buf_kernel<U, C, MINW, ACC>), dim3(static_cast<unsigned>(nb)), dim3(kBlock), 0, s,
                         X + v0, K, ld / 4, n, tail, Gv + v0, partials, nwaves, b0 * (kBlock / 64));
    else
      hipLaunchKernelGGL((client_sqdist_f32x4_kernel<U, C>), dim3(static_cast<unsigned>(nb)), dim3(kBlock), 0, s,
                         X + v0, K, ld / 4, n, tail, Gv + v0, partials, nwaves, b0 * (kBlock / 64));
  }
}

#ifdef FEDAVG_TUNING  // the global-pointer variants (probe library)
int sqdist_impl(const float* clients, int64_t K, int64_t P, int64_t ld, const float* glob, double* workspace,
                int64_t workspace_elems, double* sumsq, int unroll, int cols, int max_blocks, void* stream) {
  const char* what = "fedavg_client_sqdist_f32";
  int rc = check_common(clients, K, P, ld, glob, sumsq, what);
  if (rc) return rc;
  if (P == 0) return set_error(FEDAVG_EINVAL, "%s: P must be >= 1", what);
  if (!aligned16(clients) || !aligned16(glob) || (ld % 4) != 0)
    return set_error(FEDAVG_EALIGN, "%s: needs 16-B aligned clients/glob and ld %% 4 == 0", what);
  if (cols != 4 && cols != 8) return set_error(FEDAVG_EMODE, "%s: cols must be 4 or 8", what);
  const int64_t nwaves = sqdist_waves_for(P, cols);
  if (!workspace || workspace_elems < K * nwaves)
    return set_error(FEDAVG_EINVAL, "%s: workspace needs %lld doubles", what, (long long)(K * nwaves));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int k = static_cast<int>(K);
  switch (unroll * 100 + cols) {
    case 404: launch_sqdist<4, 4>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 804: launch_sqdist<8, 4>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 408: launch_sqdist<4, 8>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 208: launch_sqdist<2, 8>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    default: return set_error(FEDAVG_EMODE, "%s: unsupported unroll=%d cols=%d", what, unroll, cols);
  }
  rc = launch_status(what);
  if (rc) return rc;
  hipLaunchKernelGGL(client_sqdist_finalize_kernel, dim3(static_cast<unsigned>(K)), dim3(kBlock), 0, s, workspace,
                     nwaves, sumsq);
  return launch_status(what);
}
#endif  // FEDAVG_TUNING

// fp64/fp16/bf16 passes: U4 x C8 while that gives ~one workgroup per CU,
// else U8 x C2 (the fp32 pass's short-row measurements, dist_cols)
constexpr int kDistSmallRows = 8;
constexpr int kDistSmallCols = 2;
int dist_vec_cols(int64_t nvec) {
  return (nvec + kBlock * kDistCols - 1) / (kBlock * kDistCols) >= cu_count() * 9 / 10 ? kDistCols : kDistSmallCols;
}

int64_t sqdist_vec_waves(int64_t nvec, int cols) {
  const int64_t blocks = (nvec + kBlock * cols - 1) / (kBlock * cols);
  return blocks * (kBlock / 64);
}

// One launch of client_sqdist_vec_kernel<D, 4, kDistCols> + the finalize.
// Rows: [K, ld] with 16-B aligned rows (ld a multiple of the 16-B lane count).
template <class D>
int sqdist_vec_impl(const void* clients, int64_t K, int64_t P, int64_t ld, const void* glob, double* workspace,
                    int64_t workspace_elems, double* sumsq, void* stream, const char* what) {
  int rc = check_common(clients, K, P, ld, glob, sumsq, what);
  if (rc) return rc;
  if (P == 0) return set_error(FEDAVG_EINVAL, "%s: P must be >= 1", what);
  constexpr int64_t lanes = D::kLanes;
  if (!aligned16(clients) || !aligned16(glob) || (ld % lanes) != 0)
    return set_error(FEDAVG_EALIGN, "%s: needs 16-B aligned clients/glob and ld %% %d == 0", what, (int)lanes);
  const int64_t nvec = (P + lanes - 1) / lanes;
  const int cols = dist_vec_cols(nvec);
  const int64_t nwaves = sqdist_vec_waves(nvec, cols);
  if (!workspace || workspace_elems < K * nwaves)
    return set_error(FEDAVG_EINVAL, "%s: workspace needs %lld doubles", what, (long long)(K * nwaves));
  hipStream_t s = static_cast<hipStream_t>(stream);
  using vec = typename D::vec;
  const int64_t blocks = (nvec + kBlock * cols - 1) / (kBlock * cols);
  if (cols == kDistCols)
    hipLaunchKernelGGL((client_sqdist_vec_kernel<D, kDistRows, kDistCols>), dim3(static_cast<unsigned>(blocks)),
                       dim3(kBlock), 0, s, reinterpret_cast<const vec*>(clients), static_cast<int>(K), ld / lanes, nvec,
                       static_cast<int>(P % lanes), reinterpret_cast<const vec*>(glob), workspace, nwaves);
  else
    hipLaunchKernelGGL((client_sqdist_vec_kernel<D, kDistSmallRows, kDistSmallCols>),
                       dim3(static_cast<unsigned>(blocks)), dim3(kBlock), 0, s, reinterpret_cast<const vec*>(clients),
                       static_cast<int>(K), ld / lanes, nvec, static_cast<int>(P % lanes),
                       reinterpret_cast<const vec*>(glob), workspace, nwaves);
  rc = launch_status(what);
  if (rc) return rc;
  hipLaunchKernelGGL(client_sqdist_finalize_kernel, dim3(static_cast<unsigned>(K)), dim3(kBlock), 0, s, workspace,
                     nwaves, sumsq);
  return launch_status(what);
}

int sqdist_buf_impl(const float* clients, int64_t K, int64_t P, int64_t ld, const float* glob, double* workspace,
                    int64_t workspace_elems, double* sumsq, int unroll, int cols, int max_blocks, void* stream,
                    const char* what) {
  int rc = check_common(clients, K, P, ld, glob, sumsq, what);
  if (rc) return rc;
  if (P == 0) return set_error(FEDAVG_EINVAL, "%s: P must be >= 1", what);
  if (!aligned16(clients) || !aligned16(glob) || (ld % 4) != 0)
    return set_error(FEDAVG_EALIGN, "%s: needs 16-B aligned clients/glob and ld %% 4 == 0", what);
  if (cols != 1 && cols != 2 && cols != 4 && cols != 8 && cols != 12 && cols != 16)
    return set_error(FEDAVG_EMODE, "%s: cols must be 1, 2, 4, 8, 12 or 16", what);
  const int64_t nwaves = sqdist_waves_for(P, cols);
  if (!workspace || workspace_elems < K * nwaves)
    return set_error(FEDAVG_EINVAL, "%s: workspace needs %lld doubles", what, (long long)(K * nwaves));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int k = static_cast<int>(K);
  switch (unroll * 100 + cols) {
    case 408: launch_sqdist<4, 8, true>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 804: launch_sqdist<8, 4, true>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 216: launch_sqdist<2, 16, true>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    // register-capped forms (launch_bounds min waves per SIMD 3 / 4): more
    // waves resident, fewer loads in flight per wave
    case 30216: launch_sqdist<2, 16, true, 3>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 40216: launch_sqdist<2, 16, true, 4>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 30408: launch_sqdist<4, 8, true, 3>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 116: launch_sqdist<1, 16, true>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 112: launch_sqdist<1, 12, true>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 212: launch_sqdist<2, 12, true>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 208: launch_sqdist<2, 8, true>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 808: launch_sqdist<8, 8, true>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    // 2 / 4 interleaved fp64 chains per row (codes + 1,000,000 x ACC)
    case 2000216: launch_sqdist<2, 16, true, 1, 2>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 4000216: launch_sqdist<2, 16, true, 1, 4>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 2000408: launch_sqdist<4, 8, true, 1, 2>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 4000408: launch_sqdist<4, 8, true, 1, 4>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 8000216: launch_sqdist<2, 16, true, 1, 8>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 16000216: launch_sqdist<2, 16, true, 1, 16>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    // U = 0: row k + 1 loads while row k is summed (one row of registers each)
    case 16: launch_sqdist<0, 16, true>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 4000016: launch_sqdist<0, 16, true, 1, 4>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 4000012: launch_sqdist<0, 12, true, 1, 4>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 4000008: launch_sqdist<0, 8, true, 1, 4>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    // 4 chains under a register cap (min waves per SIMD 3 / 4)
    case 4030212: launch_sqdist<2, 12, true, 3, 4>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 4030216: launch_sqdist<2, 16, true, 3, 4>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 4040208: launch_sqdist<2, 8, true, 4, 4>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 4030308: launch_sqdist<3, 8, true, 3, 4>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    // narrow column groups for small models (more workgroups per launch)
    case 4000404: launch_sqdist<4, 4, true, 1, 4>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 4000804: launch_sqdist<8, 4, true, 1, 4>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 4000402: launch_sqdist<4, 2, true, 1, 2>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 4000802: launch_sqdist<8, 2, true, 1, 2>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 4000801: launch_sqdist<8, 1, true, 1, 1>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 4001601: launch_sqdist<16, 1, true, 1, 1>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 4000116: launch_sqdist<1, 16, true, 1, 4>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    default: return set_error(FEDAVG_EMODE, "%s: unsupported unroll=%d cols=%d", what, unroll, cols);
  }
  rc = launch_status(what);
  if (rc) return rc;
  hipLaunchKernelGGL(client_sqdist_finalize_kernel, dim3(static_cast<unsigned>(K)), dim3(kBlock), 0, s, workspace,
                     nwaves, sumsq);
  return launch_status(what);
}

}  // namespace

extern "C" {

int64_t fedavg_client_sqdist_workspace(int64_t K, int64_t P) {
  if (K <= 0 || P <= 0) return 0;
  return K * sqdist_waves_for(P, dist_cols(P) < 4 ? dist_cols(P) : 4);  // production; any variant of >= 4 slices
}

int fedavg_client_sqdist_f32(const float* clients, int64_t K, int64_t P, int64_t ld, const float* glob,
                             double* workspace, int64_t workspace_elems, double* sumsq, void* stream) {
  // unroll codes: chains x 10000 + rows per batch (4 chains, at most one per slice)
  const int cols = P > 0 ? dist_cols(P) : kDistBufCols;
  const int rows = cols == 16 ? kDistBufRows : (cols == 4 ? 4 : 8);
  return sqdist_buf_impl(clients, K, P, ld, glob, workspace, workspace_elems, sumsq, kDistBufChains * 10000 + rows,
                         cols, 0, stream, "fedavg_client_sqdist_f32");
}

int64_t fedavg_client_sqdist_workspace_elems(int64_t K, int64_t P, int64_t elem_size) {
  if (K <= 0 || P <= 0 || (elem_size != 2 && elem_size != 4 && elem_size != 8)) return 0;
  const int64_t lanes = 16 / elem_size;
  const int64_t nvec = (P + lanes - 1) / lanes;
  return K * sqdist_vec_waves(nvec, dist_vec_cols(nvec));
}

int fedavg_client_sqdist_f64(const double* clients, int64_t K, int64_t P, int64_t ld, const double* glob,
                             double* workspace, int64_t workspace_elems, double* sumsq, void* stream) {
  return sqdist_vec_impl<DistF64>(clients, K, P, ld, glob, workspace, workspace_elems, sumsq, stream,
                                  "fedavg_client_sqdist_f64");
}

int fedavg_client_sqdist_f16(const uint16_t* clients, int64_t K, int64_t P, int64_t ld, const uint16_t* glob,
                             double* workspace, int64_t workspace_elems, double* sumsq, void* stream) {
  return sqdist_vec_impl<DistHalf<F16Pk>>(clients, K, P, ld, glob, workspace, workspace_elems, sumsq, stream,
                                          "fedavg_client_sqdist_f16");
}

int fedavg_client_sqdist_bf16(const uint16_t* clients, int64_t K, int64_t P, int64_t ld, const uint16_t* glob,
                              double* workspace, int64_t workspace_elems, double* sumsq, void* stream) {
  return sqdist_vec_impl<DistHalf<BF16Pk>>(clients, K, P, ld, glob, workspace, workspace_elems, sumsq, stream,
                                           "fedavg_client_sqdist_bf16");
}

#ifdef FEDAVG_TUNING  // probe library only (libfedavg_amd_probe.so)
int fedavg_client_sqdist_variant(const float* clients, int64_t K, int64_t P, int64_t ld, const float* glob,
                                 double* workspace, int64_t workspace_elems, double* sumsq, int unroll, int cols,
                                 int max_blocks, void* stream) {
  return sqdist_impl(clients, K, P, ld, glob, workspace, workspace_elems, sumsq, unroll, cols, max_blocks, stream);
}
#endif  // FEDAVG_TUNING

#ifdef FEDAVG_TUNING  // probe library only (libfedavg_amd_probe.so)
int fedavg_client_sqdist_buf(const float* clients, int64_t K, int64_t P, int64_t ld, const float* glob,
                             double* workspace, int64_t workspace_elems, double* sumsq, int unroll, int cols,
                             int max_blocks, void* stream) {
  return sqdist_buf_impl(clients, K, P, ld, glob, workspace, workspace_elems, sumsq, unroll, cols, max_blocks, stream,
                         "fedavg_client_sqdist_buf");
}
#endif  // FEDAVG_TUNING

}  // extern "C"
