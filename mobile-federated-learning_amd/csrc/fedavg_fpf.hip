// fedavg_fpf.hip -- the FPF2 bookkeeping of the round loop
// (fedavg_trainer.py:108-119, :209-210, :271-278, :314-327) on device-resident
// state: local_w_diffs [n_rows, ld], A_mat [ld], G_mat / local_itr_lst row /
// LRU_itr_lst [n_rows], all fp32 like the reference's tensors.
//
// Elementwise updates reproduce the reference's fp32 expressions operation by
// operation (no FMA: the library is built with -ffp-contract=off), so
// local_w_diffs, G_mat, local_itr_lst and LRU_itr_lst are bit-identical.  The
// two reductions -- global_w_diff.mean() (:319) and the row norms (:272) --
// accumulate in fp64 in a fixed order and round once (the norm's squares with
// explicit fp64 fused multiply-adds); the reference's fp32 reductions are
// within their own rounding error of that value.
//
// Padding lanes (columns P..ld) never contribute: every load past P is
// replaced by a select, so whatever the padding holds cannot leak in.
#include "common.hpp"

#include <math.h>

namespace {
using namespace fedavg_impl;

constexpr int kFpfRowsPerBlock = 4;
constexpr int kFpfMaxPartials = 1024;

__device__ __forceinline__ f32x4 masked(f32x4 v, int nv) {
  if (nv < 4) {
    v.x = nv > 0 ? v.x : 0.f;
    v.y = nv > 1 ? v.y : 0.f;
    v.z = nv > 2 ? v.z : 0.f;
    v.w = 0.f;
  }
  return v;
}

__device__ __forceinline__ int lanes_valid(int64_t v, int64_t P) {
  const int64_t rem = P - v * 4;
  return rem >= 4 ? 4 : (rem > 0 ? static_cast<int>(rem) : 0);
}

__device__ __forceinline__ double block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < kBlock / 64; ++w) s += red[w];
  return s;  // valid in thread 0
}

// :210  local_w_diffs[row_idx[k], :] = rows[k, :] - last_w   (fp32 difference)
__global__ __launch_bounds__(kBlock) void fpf_set_rows_kernel(f32x4* __restrict__ D, int64_t ld4, int64_t n_rows,
                                                              const int64_t* __restrict__ row_idx,
                                                              const f32x4* __restrict__ rows, int64_t ld_rows4,
                                                              const f32x4* __restrict__ last_w, int64_t P) {
  const int64_t r = row_idx[blockIdx.y];
  if (r < 0 || r >= n_rows) return;  // the host layer raises IndexError before launching
  const int64_t nvec = (P + 3) / 4;
  const f32x4* src = rows + static_cast<int64_t>(blockIdx.y) * ld_rows4;
  f32x4* dst = D + r * ld4;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; v < nvec;
       v += static_cast<int64_t>(gridDim.x) * kBlock)
    dst[v] = masked(src[v] - last_w[v], lanes_valid(v, P));
}

// :319 (first half): per-block fp64 partial sums of global_w_diff = w_glob - last_w.
__global__ __launch_bounds__(kBlock) void fpf_gdiff_partials_kernel(const f32x4* __restrict__ w_glob,
                                                                    const f32x4* __restrict__ last_w, int64_t P,
                                                                    double* __restrict__ partials) {
  __shared__ double red[kBlock / 64];
  const int64_t nvec = (P + 3) / 4;
  double s = 0.0;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; v < nvec;
       v += static_cast<int64_t>(gridDim.x) * kBlock) {
    const f32x4 g = masked(w_glob[v] - last_w[v], lanes_valid(v, P));
    s += static_cast<double>(g.x) + static_cast<double>(g.y) + static_cast<double>(g.z) + static_cast<double>(g.w);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

// :316-319  rows not in client_indexes: local_w_diffs -= global_w_diff;
//           A_mat = A_mat * (1 - 1/G2) + global_w_diff / G2 / global_w_diff.mean()
// Every block reduces the same partials in the same order, so all blocks see
// the same mean without another launch.
__global__ __launch_bounds__(kBlock) void fpf_end_round_kernel(f32x4* __restrict__ D, int64_t ld4, int64_t n_rows,
                                                               const uint8_t* __restrict__ keep_rows,
                                                               f32x4* __restrict__ A, const f32x4* __restrict__ w_glob,
                                                               const f32x4* __restrict__ last_w, int64_t P,
                                                               const double* __restrict__ partials, int nparts,
                                                               float g2, float c2) {
  __shared__ double red[kBlock / 64];
  __shared__ float mean_s;
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += kBlock) s += partials[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) mean_s = static_cast<float>(s / static_cast<double>(P));
  __syncthreads();
  const float mean = mean_s;
  const int64_t nvec = (P + 3) / 4;
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * kFpfRowsPerBlock;
  const int64_t r1 = r0 + kFpfRowsPerBlock < n_rows ? r0 + kFpfRowsPerBlock : n_rows;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; v < nvec;
       v += static_cast<int64_t>(gridDim.x) * kBlock) {
    const int nv = lanes_valid(v, P);
    const f32x4 g = masked(w_glob[v] - last_w[v], nv);
    if (blockIdx.y == 0) {
      const f32x4 a = A[v];
      f32x4 na;
      na.x = a.x * c2 + (g.x / g2) / mean;
      na.y = a.y * c2 + (g.y / g2) / mean;
      na.z = a.z * c2 + (g.z / g2) / mean;
      na.w = a.w * c2 + (g.w / g2) / mean;
      A[v] = nv == 4 ? na : f32x4{nv > 0 ? na.x : a.x, nv > 1 ? na.y : a.y, nv > 2 ? na.z : a.z, a.w};
    }
    for (int64_t r = r0; r < r1; ++r) {
      if (keep_rows[r]) continue;
      f32x4* p = D + r * ld4 + v;
      *p = *p - g;  // padding lanes: g == 0, D stays 0
    }
  }
}

// :321-327  local_itr_lst[round_idx, selected] = float(local_itr);
//           LRU_itr_lst += float(local_itr); LRU_itr_lst[selected] = 0   (LRU mode)
//           G_mat = G_mat * (1 - 1/G1) + local_itr_lst[round_idx, :] / G1
__global__ __launch_bounds__(kBlock) void fpf_update_g_kernel(float* __restrict__ G, float* __restrict__ itr_row,
                                                              float* __restrict__ lru,
                                                              const uint8_t* __restrict__ selected, int64_t n,
                                                              float local_itr, int record, float g1, float c1) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (r >= n) return;
  float it = itr_row[r];
  if (record) {
    if (selected[r]) it = local_itr;
    itr_row[r] = it;
    if (lru) lru[r] = selected[r] ? 0.f : lru[r] + local_itr;
  }
  G[r] = G[r] * c1 + it / g1;
}

// :272, :276-278  fpf[r] = norm(local_w_diffs[r] * A_mat) / G_mat[r], NaN/inf -> 0.
// One block per row; products rounded to fp32 like the reference's
// `local_w_diffs * A_mat`, squares and sum in fp64, one rounding at the end.
__device__ __forceinline__ double sq4_add(double acc, f32x4 q) {
  const double x = q.x, y = q.y, z = q.z, w = q.w;  // exact squares, one rounding per fused add
  acc = __builtin_fma(x, x, acc);
  acc = __builtin_fma(y, y, acc);
  acc = __builtin_fma(z, z, acc);
  return __builtin_fma(w, w, acc);
}

// The row is streamed with 8 x 16-B nontemporal loads in flight per thread
// (one block per row: 256 threads x 8 = 32 KiB per block-step); A_mat is
// re-read by every row, so its loads keep the default cache policy.
__global__ __launch_bounds__(kBlock) void fpf_index_kernel(const f32x4* __restrict__ D, int64_t ld4, int64_t P,
                                                           const f32x4* __restrict__ A, const float* __restrict__ G,
                                                           float* __restrict__ out) {
  constexpr int U = 8;
  __shared__ double red[kBlock / 64];
  const int64_t r = blockIdx.x;
  const int64_t nvec = (P + 3) / 4;
  const f32x4* row = D + r * ld4;
  double s = 0.0;
  for (int64_t v = threadIdx.x; v < nvec; v += U * kBlock) {
    // a full batch of U loads per thread, the last one predicated: every
    // thread keeps U loads in flight even when the row is short (P = 7,850)
    f32x4 d[U], a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool in = v + u * kBlock < nvec;
      d[u] = in ? ld<true>(row + v + u * kBlock) : f32x4{0.f, 0.f, 0.f, 0.f};
      a[u] = in ? A[v + u * kBlock] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) s = sq4_add(s, masked(d[u] * a[u], lanes_valid(v + u * kBlock, P)));
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    const float f = static_cast<float>(sqrt(s)) / G[r];
    out[r] = isfinite(f) ? f : 0.f;
  }
}

#ifdef FEDAVG_TUNING  // the column-window index variant (measurement only)
// :272 as a column-window pass (the reduce's access pattern).  Block
// (bx, by) covers C*256 column slices of rows [by*R, (by+1)*R) and walks
// those rows U at a time, so the blocks of a row group read one compact window
// of the same few rows together; each wave leaves one fp64 partial per row:
// partials[row][bx*4 + wave].  fpf_index_finalize_kernel then sums a row's
// partials in a fixed order (deterministic) and applies :272/:276-278.
template <int U, int C>
__global__ __launch_bounds__(kBlock) void fpf_index_partials_kernel(const f32x4* __restrict__ D, int64_t ld4,
                                                                    int64_t n_rows, int64_t P, int64_t rows_per_group,
                                                                    const f32x4* __restrict__ A,
                                                                    double* __restrict__ partials, int64_t nwc) {
  const int lane = threadIdx.x & 63;
  const int64_t nvec = (P + 3) / 4;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kBlock * C + threadIdx.x;
  const int64_t wave_col = static_cast<int64_t>(blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6);
  f32x4 a[C];
  int nv[C];
#pragma unroll
  for (int j = 0; j < C; ++j) {
    const int64_t v = base + static_cast<int64_t>(j) * kBlock;
    nv[j] = v < nvec ? lanes_valid(v, P) : 0;
    a[j] = nv[j] > 0 ? A[v] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * rows_per_group;
  const int64_t r1 = (r0 + rows_per_group) < n_rows ? (r0 + rows_per_group) : n_rows;
  for (int64_t r = r0; r < r1; r += U) {
    f32x4 d[U][C];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < C; ++j)
        d[u][j] = (r + u < r1 && nv[j] > 0) ? ld<true>(D + (r + u) * ld4 + base + j * kBlock)
                                            : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (r + u >= r1) break;
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < C; ++j) acc = sq4_add(acc, masked(d[u][j] * a[j], nv[j]));
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
      if (lane == 0) partials[(r + u) * nwc + wave_col] = acc;
    }
  }
}

__global__ __launch_bounds__(kBlock) void fpf_index_finalize_kernel(const double* __restrict__ partials, int64_t nwc,
                                                                    int64_t n_rows, const float* __restrict__ G,
                                                                    float* __restrict__ out) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (r >= n_rows) return;
  double s = 0.0;
  for (int64_t w = 0; w < nwc; ++w) s += partials[r * nwc + w];
  const float f = static_cast<float>(sqrt(s)) / G[r];
  out[r] = isfinite(f) ? f : 0.f;
}

int64_t index_col_blocks(int64_t P, int cols) {
  const int64_t nvec = (P + 3) / 4;
  return (nvec + static_cast<int64_t>(kBlock) * cols - 1) / (static_cast<int64_t>(kBlock) * cols);
}

// Row groups so that one launch holds about 3 blocks per CU.
int64_t index_row_groups(int64_t n_rows, int64_t col_blocks) {
  int64_t g = (3 * static_cast<int64_t>(cu_count()) + col_blocks - 1) / col_blocks;
  if (g < 1) g = 1;
  if (g > n_rows) g = n_rows;
  return g;
}

template <int U, int C>
void launch_index_windows(const float* diffs, int64_t n_rows, int64_t ld, int64_t P, const float* a_mat,
                          const float* g_mat, float* fpf, double* ws, int64_t groups, hipStream_t s) {
  const int64_t cb = index_col_blocks(P, C);
  const int64_t nwc = cb * (kBlock / 64);
  const int64_t rpg = (n_rows + groups - 1) / groups;
  const int64_t gy = (n_rows + rpg - 1) / rpg;
  hipLaunchKernelGGL((fpf_index_partials_kernel<U, C>), dim3(static_cast<unsigned>(cb), static_cast<unsigned>(gy)),
                     dim3(kBlock), 0, s, reinterpret_cast<const f32x4*>(diffs), ld / 4, n_rows, P, rpg,
                     reinterpret_cast<const f32x4*>(a_mat), ws, nwc);
  hipLaunchKernelGGL(fpf_index_finalize_kernel, dim3(static_cast<unsigned>((n_rows + kBlock - 1) / kBlock)),
                     dim3(kBlock), 0, s, ws, nwc, n_rows, g_mat, fpf);
}

#endif  // FEDAVG_TUNING

// :274, :276-278  fpf = LRU_itr_lst / G_mat, NaN/inf -> 0.
__global__ __launch_bounds__(kBlock) void fpf_index_lru_kernel(const float* __restrict__ lru,
                                                               const float* __restrict__ G, int64_t n,
                                                               float* __restrict__ out) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (r >= n) return;
  const float f = lru[r] / G[r];
  out[r] = isfinite(f) ? f : 0.f;
}

// ---------------------------------------------------------------------------
// Models with fp64 / fp16 / bf16 keys.  torch.cat at :210 and :316 promotes the
// per-key differences (each computed in its key's dtype) to T, the promoted
// dtype of all keys: local_w_diffs (fp32) receives fl32 of that, :317 runs in
// promote(fp32, T), and :319 runs in T -- so A_mat becomes fp64 after the first
// round of a model with an fp64 key, and a pure fp16/bf16 model forms the
// A_mat term in 16-bit arithmetic.  The model is described key by key in
// state_dict order (numel, cat offset, dtype group, offset in the group row,
// rounding of an fp32-stored integer key's difference to T); the clients'
// rows are the aggregate's per-dtype group rows.
// ---------------------------------------------------------------------------
struct FpfGroups {  // = fedavg_fpf_groups (include/fedavg_amd.h)
  const void* base[4];
  int64_t ld[4];
  int32_t kind[4];
};
enum : int { kF32 = 0, kF64 = 1, kF16 = 2, kBF16 = 3 };
// end_round_promoted only: the first fp64 round of a model whose A_mat is
// still the reference's fp32 tensor (a_mat holds its values widened exactly)
constexpr int kF64FromF32 = 4;
constexpr int kFpfKeyFields = 5;  // numel, cat_off, grp, grp_off, rnd

__device__ __forceinline__ float opaque1(float v) {
  asm volatile("" : "+v"(v));
  return v;
}

// fp32 -> fp16 / bf16 (RNE) -> fp32
__device__ __forceinline__ float rnd16(float x, int kind) {
  x = opaque1(x);
  return kind == kF16 ? static_cast<float>(static_cast<_Float16>(x)) : static_cast<float>(static_cast<__bf16>(x));
}

// element i of group grp: row `row` of cur minus row 0 of last, in the key's
// arithmetic (ATen computes a 16-bit difference in fp32 and rounds it)
__device__ __forceinline__ double cat_diff(const FpfGroups& cur, int64_t row, const FpfGroups& last, int grp,
                                           int64_t i, int rnd) {
  const int64_t o = row * cur.ld[grp] + i;
  switch (cur.kind[grp]) {
    case kF64:
      return static_cast<const double*>(cur.base[grp])[o] - static_cast<const double*>(last.base[grp])[i];
    case kF16:
      return rnd16(static_cast<float>(static_cast<const _Float16*>(cur.base[grp])[o]) -
                       static_cast<float>(static_cast<const _Float16*>(last.base[grp])[i]),
                   kF16);
    case kBF16:
      return rnd16(static_cast<float>(static_cast<const __bf16*>(cur.base[grp])[o]) -
                       static_cast<float>(static_cast<const __bf16*>(last.base[grp])[i]),
                   kBF16);
    default: {
      const float d = static_cast<const float*>(cur.base[grp])[o] - static_cast<const float*>(last.base[grp])[i];
      return rnd ? rnd16(d, rnd) : d;
    }
  }
}

// :210 / :316  out[row_idx[k]][c] = cat(w_k - last_w)[c] (fl32 of it into fp32
// rows, or the T value itself into an fp64 vector).  Column c belongs to the
// last key whose cat offset is <= c (empty keys lose the tie).
__global__ __launch_bounds__(kBlock) void fpf_cat_diff_kernel(const int64_t* __restrict__ keys, int64_t n_keys,
                                                              int64_t P, FpfGroups cur, FpfGroups last,
                                                              const int64_t* __restrict__ row_idx, int64_t n_rows,
                                                              void* __restrict__ out, int64_t ld_out, int out_f64) {
  const int64_t c = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (c >= P) return;
  const int64_t k = blockIdx.y;
  const int64_t r = row_idx ? row_idx[k] : k;
  if (r < 0 || r >= n_rows) return;  // the host layer raises IndexError before launching
  int64_t lo = 0, hi = n_keys - 1;
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (keys[mid * kFpfKeyFields + 1] <= c)
      lo = mid;
    else
      hi = mid - 1;
  }
  const int64_t* kj = keys + lo * kFpfKeyFields;
  const double v = cat_diff(cur, k, last, static_cast<int>(kj[2]), kj[3] + (c - kj[1]), static_cast<int>(kj[4]));
  if (out_f64)
    static_cast<double*>(out)[r * ld_out + c] = v;
  else
    static_cast<float*>(out)[r * ld_out + c] = static_cast<float>(v);
}

// :319 (first half) on the T-valued global_w_diff
__global__ __launch_bounds__(kBlock) void fpf_sum_f64_kernel(const double* __restrict__ x, int64_t P,
                                                             double* __restrict__ partials) {
  __shared__ double red[kBlock / 64];
  double s = 0.0;
  for (int64_t c = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; c < P;
       c += static_cast<int64_t>(gridDim.x) * kBlock)
    s += x[c];
  s = block_sum(s, red);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

// :316-319 with global_w_diff of dtype T (values in gd):
//   rows not in client_indexes: fl32(row - g) computed in promote(fp32, T);
//   A_mat = A_mat * (1 - 1/G2) + g / G2 / mean(g): fp64 for T = fp64 (A in
//   fp64), fp32 for T = fp32, and for T = fp16/bf16 the term g / G2 / mean is
//   16-bit (each op in fp32, rounded) and added to the fp32 A_mat.
template <int T>
__global__ __launch_bounds__(kBlock) void fpf_end_round_promoted_kernel(
    float* __restrict__ D, int64_t ld, int64_t n_rows, const uint8_t* __restrict__ keep_rows, void* __restrict__ A,
    const double* __restrict__ gd, int64_t P, const double* __restrict__ partials, int nparts, double g2, double c2) {
  __shared__ double red[kBlock / 64];
  __shared__ double mean_s;
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += kBlock) s += partials[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    const double m = s / static_cast<double>(P);
    mean_s = (T == kF64 || T == kF64FromF32) ? m
             : (T == kF32 ? static_cast<double>(static_cast<float>(m)) : rnd16(static_cast<float>(m), T));
  }
  __syncthreads();
  const double mean = mean_s;
  const float meanf = static_cast<float>(mean);
  const float g2f = static_cast<float>(g2), c2f = static_cast<float>(c2);
  constexpr bool F64 = T == kF64 || T == kF64FromF32;
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * kFpfRowsPerBlock;
  const int64_t r1 = r0 + kFpfRowsPerBlock < n_rows ? r0 + kFpfRowsPerBlock : n_rows;
  for (int64_t c = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; c < P;
       c += static_cast<int64_t>(gridDim.x) * kBlock) {
    const double g = gd[c];
    if (blockIdx.y == 0) {
      if constexpr (T == kF64) {
        double* a = static_cast<double*>(A);
        a[c] = a[c] * c2 + (g / g2) / mean;
      } else if constexpr (T == kF64FromF32) {
        // the reference's first promoted round: A_mat (fp32) * (1 - 1/G2) is an
        // fp32 product (the Python float cast to fp32), widened exactly when the
        // fp64 term is added -- fp64 A_mat from then on
        double* a = static_cast<double*>(A);
        a[c] = static_cast<double>(static_cast<float>(a[c]) * c2f) + (g / g2) / mean;
      } else if constexpr (T == kF32) {
        float* a = static_cast<float*>(A);
        a[c] = a[c] * c2f + (static_cast<float>(g) / g2f) / meanf;
      } else {
        float* a = static_cast<float*>(A);
        const float t = rnd16(rnd16(static_cast<float>(g) / g2f, T) / meanf, T);
        a[c] = a[c] * c2f + t;
      }
    }
    for (int64_t r = r0; r < r1; ++r) {
      if (keep_rows[r]) continue;
      float* p = D + r * ld + c;
      if constexpr (F64)
        *p = static_cast<float>(static_cast<double>(*p) - g);
      else
        *p = *p - static_cast<float>(g);
    }
  }
}

// :272, :276-278 once A_mat is fp64: norm(fl64(diff * A)) / G_mat in fp64
__global__ __launch_bounds__(kBlock) void fpf_index_f64a_kernel(const float* __restrict__ D, int64_t ld, int64_t P,
                                                                const double* __restrict__ A,
                                                                const float* __restrict__ G, double* __restrict__ out) {
  __shared__ double red[kBlock / 64];
  const int64_t r = blockIdx.x;
  const float* row = D + r * ld;
  double s = 0.0;
  for (int64_t c = threadIdx.x; c < P; c += kBlock) {
    const double q = static_cast<double>(row[c]) * A[c];
    s = __builtin_fma(q, q, s);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    const double f = sqrt(s) / static_cast<double>(G[r]);
    out[r] = isfinite(f) ? f : 0.0;
  }
}

unsigned col_blocks(int64_t P, int64_t cap) {
  const int64_t nvec = (P + 3) / 4;
  int64_t b = (nvec + kBlock - 1) / kBlock;
  if (b > cap) b = cap;
  return static_cast<unsigned>(b < 1 ? 1 : b);
}

int check_state(const void* diffs, int64_t n_rows, int64_t ld, int64_t P, const char* what) {
  if (n_rows <= 0 || n_rows > INT32_MAX) return set_error(FEDAVG_EINVAL, "%s: bad n_rows %lld", what, (long long)n_rows);
  if (P <= 0) return set_error(FEDAVG_EINVAL, "%s: P must be >= 1", what);
  if (ld < P || (ld % 4) != 0)
    return set_error(FEDAVG_EINVAL, "%s: need ld >= P and ld %% 4 == 0 (ld=%lld, P=%lld)", what, (long long)ld,
                     (long long)P);
  if (!diffs) return set_error(FEDAVG_EINVAL, "%s: null local_w_diffs", what);
  if (!aligned16(diffs)) return set_error(FEDAVG_EALIGN, "%s: local_w_diffs must be 16-B aligned", what);
  return FEDAVG_OK;
}

}  // namespace

extern "C" {

int fedavg_fpf_set_rows_f32(float* diffs, int64_t n_rows, int64_t ld, const int64_t* row_idx, int64_t K,
                            const float* rows, int64_t ld_rows, const float* last_w, int64_t P, void* stream) {
  const char* what = "fedavg_fpf_set_rows_f32";
  int rc = check_state(diffs, n_rows, ld, P, what);
  if (rc) return rc;
  if (K <= 0 || K > 65535) return set_error(FEDAVG_EINVAL, "%s: K must be in [1, 65535] (got %lld)", what, (long long)K);
  if (!row_idx || !rows || !last_w) return set_error(FEDAVG_EINVAL, "%s: null buffer", what);
  if (ld_rows < P || (ld_rows % 4) != 0) return set_error(FEDAVG_EINVAL, "%s: bad ld_rows", what);
  if (!aligned16(rows) || !aligned16(last_w))
    return set_error(FEDAVG_EALIGN, "%s: rows/last_w must be 16-B aligned", what);
  hipLaunchKernelGGL(fpf_set_rows_kernel, dim3(col_blocks(P, 256), static_cast<unsigned>(K)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), reinterpret_cast<f32x4*>(diffs), ld / 4, n_rows, row_idx,
                     reinterpret_cast<const f32x4*>(rows), ld_rows / 4, reinterpret_cast<const f32x4*>(last_w), P);
  return launch_status(what);
}

int64_t fedavg_fpf_workspace(int64_t P) {
  if (P <= 0) return 0;
  return col_blocks(P, kFpfMaxPartials);
}

int fedavg_fpf_end_round_f32(float* diffs, int64_t n_rows, int64_t ld, const uint8_t* keep_rows, float* a_mat,
                             const float* w_glob, const float* last_w, int64_t P, float g2, double* workspace,
                             int64_t workspace_elems, void* stream) {
  const char* what = "fedavg_fpf_end_round_f32";
  int rc = check_state(diffs, n_rows, ld, P, what);
  if (rc) return rc;
  if (!keep_rows || !a_mat || !w_glob || !last_w || !workspace) return set_error(FEDAVG_EINVAL, "%s: null buffer", what);
  if (!aligned16(a_mat) || !aligned16(w_glob) || !aligned16(last_w))
    return set_error(FEDAVG_EALIGN, "%s: A_mat/w_glob/last_w must be 16-B aligned", what);
  const unsigned nparts = col_blocks(P, kFpfMaxPartials);
  if (workspace_elems < nparts)
    return set_error(FEDAVG_EINVAL, "%s: workspace needs %u doubles", what, nparts);
  if (!(g2 != 0.f)) return set_error(FEDAVG_EINVAL, "%s: G2 must be nonzero", what);
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(fpf_gdiff_partials_kernel, dim3(nparts), dim3(kBlock), 0, s,
                     reinterpret_cast<const f32x4*>(w_glob), reinterpret_cast<const f32x4*>(last_w), P, workspace);
  rc = launch_status(what);
  if (rc) return rc;
  const float c2 = static_cast<float>(1.0 - 1.0 / static_cast<double>(g2));  // (1 - 1/G2) as a Python float
  const unsigned ry = static_cast<unsigned>((n_rows + kFpfRowsPerBlock - 1) / kFpfRowsPerBlock);
  hipLaunchKernelGGL(fpf_end_round_kernel, dim3(col_blocks(P, 512), ry), dim3(kBlock), 0, s,
                     reinterpret_cast<f32x4*>(diffs), ld / 4, n_rows, keep_rows, reinterpret_cast<f32x4*>(a_mat),
                     reinterpret_cast<const f32x4*>(w_glob), reinterpret_cast<const f32x4*>(last_w), P, workspace,
                     static_cast<int>(nparts), g2, c2);
  return launch_status(what);
}

int fedavg_fpf_update_g(float* g_mat, float* itr_row, float* lru_itr, const uint8_t* selected, int64_t n_rows,
                        float local_itr, int record, float g1, void* stream) {
  const char* what = "fedavg_fpf_update_g";
  if (n_rows <= 0) return set_error(FEDAVG_EINVAL, "%s: n_rows must be >= 1", what);
  if (!g_mat || !itr_row || !selected) return set_error(FEDAVG_EINVAL, "%s: null buffer", what);
  if (!(g1 != 0.f)) return set_error(FEDAVG_EINVAL, "%s: G1 must be nonzero", what);
  const float c1 = static_cast<float>(1.0 - 1.0 / static_cast<double>(g1));
  hipLaunchKernelGGL(fpf_update_g_kernel, dim3(static_cast<unsigned>((n_rows + kBlock - 1) / kBlock)), dim3(kBlock),
                     0, static_cast<hipStream_t>(stream), g_mat, itr_row, lru_itr, selected, n_rows, local_itr,
                     record ? 1 : 0, g1, c1);
  return launch_status(what);
}

int fedavg_fpf_index_f32(const float* diffs, int64_t n_rows, int64_t ld, int64_t P, const float* a_mat,
                         const float* g_mat, float* fpf, void* stream) {
  const char* what = "fedavg_fpf_index_f32";
  int rc = check_state(diffs, n_rows, ld, P, what);
  if (rc) return rc;
  if (!a_mat || !g_mat || !fpf) return set_error(FEDAVG_EINVAL, "%s: null buffer", what);
  if (!aligned16(a_mat)) return set_error(FEDAVG_EALIGN, "%s: A_mat must be 16-B aligned", what);
  hipLaunchKernelGGL(fpf_index_kernel, dim3(static_cast<unsigned>(n_rows)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), reinterpret_cast<const f32x4*>(diffs), ld / 4, P,
                     reinterpret_cast<const f32x4*>(a_mat), g_mat, fpf);
  return launch_status(what);
}

#ifdef FEDAVG_TUNING  // probe library only (libfedavg_amd_probe.so)
int64_t fedavg_fpf_index_workspace(int64_t n_rows, int64_t P) {
  if (n_rows <= 0 || P <= 0) return 0;
  return n_rows * index_col_blocks(P, 1) * (kBlock / 64);  // enough for every column width
}
#endif  // FEDAVG_TUNING

#ifdef FEDAVG_TUNING  // probe library only (libfedavg_amd_probe.so)
int fedavg_fpf_index_variant(const float* diffs, int64_t n_rows, int64_t ld, int64_t P, const float* a_mat,
                             const float* g_mat, float* fpf, double* workspace, int64_t workspace_elems, int unroll,
                             int cols, int row_groups, void* stream) {
  const char* what = "fedavg_fpf_index_variant";
  int rc = check_state(diffs, n_rows, ld, P, what);
  if (rc) return rc;
  if (!a_mat || !g_mat || !fpf || !workspace) return set_error(FEDAVG_EINVAL, "%s: null buffer", what);
  if (!aligned16(a_mat)) return set_error(FEDAVG_EALIGN, "%s: A_mat must be 16-B aligned", what);
  if (cols != 1 && cols != 2 && cols != 4 && cols != 8) return set_error(FEDAVG_EMODE, "%s: cols must be 1, 2, 4 or 8", what);
  const int64_t need = n_rows * index_col_blocks(P, cols) * (kBlock / 64);
  if (workspace_elems < need) return set_error(FEDAVG_EINVAL, "%s: workspace needs %lld doubles", what, (long long)need);
  const int64_t groups = row_groups > 0 ? (row_groups < n_rows ? row_groups : n_rows)
                                        : index_row_groups(n_rows, index_col_blocks(P, cols));
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (unroll * 100 + cols) {
    case 401: launch_index_windows<4, 1>(diffs, n_rows, ld, P, a_mat, g_mat, fpf, workspace, groups, s); break;
    case 801: launch_index_windows<8, 1>(diffs, n_rows, ld, P, a_mat, g_mat, fpf, workspace, groups, s); break;
    case 1601: launch_index_windows<16, 1>(diffs, n_rows, ld, P, a_mat, g_mat, fpf, workspace, groups, s); break;
    case 802: launch_index_windows<8, 2>(diffs, n_rows, ld, P, a_mat, g_mat, fpf, workspace, groups, s); break;
    case 404: launch_index_windows<4, 4>(diffs, n_rows, ld, P, a_mat, g_mat, fpf, workspace, groups, s); break;
    case 804: launch_index_windows<8, 4>(diffs, n_rows, ld, P, a_mat, g_mat, fpf, workspace, groups, s); break;
    case 408: launch_index_windows<4, 8>(diffs, n_rows, ld, P, a_mat, g_mat, fpf, workspace, groups, s); break;
    default: return set_error(FEDAVG_EMODE, "%s: unsupported unroll=%d cols=%d", what, unroll, cols);
  }
  return launch_status(what);
}
#endif  // FEDAVG_TUNING

int fedavg_fpf_cat_diff(const int64_t* keys, int64_t n_keys, int64_t P, const fedavg_fpf_groups* cur, int64_t K,
                        const fedavg_fpf_groups* last, const int64_t* row_idx, int64_t n_rows, void* out,
                        int64_t ld_out, int out_f64, void* stream) {
  const char* what = "fedavg_fpf_cat_diff";
  if (!keys || n_keys <= 0 || !cur || !last || !out) return set_error(FEDAVG_EINVAL, "%s: bad arguments", what);
  if (P <= 0 || ld_out < P) return set_error(FEDAVG_EINVAL, "%s: need 1 <= P <= ld_out", what);
  if (K <= 0 || K > 65535) return set_error(FEDAVG_EINVAL, "%s: K must be in [1, 65535] (got %lld)", what, (long long)K);
  if (n_rows <= 0 || (!row_idx && n_rows < K)) return set_error(FEDAVG_EINVAL, "%s: bad n_rows", what);
  FpfGroups c{}, l{};
  for (int g = 0; g < 4; ++g) {
    if (cur->kind[g] < kF32 || cur->kind[g] > kBF16 || cur->kind[g] != last->kind[g])
      return set_error(FEDAVG_EINVAL, "%s: group %d: bad or mismatched kind", what, g);
    c.base[g] = cur->base[g];
    c.ld[g] = cur->ld[g];
    c.kind[g] = cur->kind[g];
    l.base[g] = last->base[g];
    l.ld[g] = last->ld[g];
    l.kind[g] = last->kind[g];
  }
  hipLaunchKernelGGL(fpf_cat_diff_kernel, dim3(static_cast<unsigned>((P + kBlock - 1) / kBlock), static_cast<unsigned>(K)),
                     dim3(kBlock), 0, static_cast<hipStream_t>(stream), keys, n_keys, P, c, l, row_idx, n_rows, out,
                     ld_out, out_f64 ? 1 : 0);
  return launch_status(what);
}

int fedavg_fpf_end_round_promoted(float* diffs, int64_t n_rows, int64_t ld, const uint8_t* keep_rows, void* a_mat,
                                  const double* gdiff, int64_t P, int t_kind, float g2, double* workspace,
                                  int64_t workspace_elems, void* stream) {
  const char* what = "fedavg_fpf_end_round_promoted";
  int rc = check_state(diffs, n_rows, ld, P, what);
  if (rc) return rc;
  if (!keep_rows || !a_mat || !gdiff || !workspace) return set_error(FEDAVG_EINVAL, "%s: null buffer", what);
  const unsigned nparts = col_blocks(P, kFpfMaxPartials);
  if (workspace_elems < nparts) return set_error(FEDAVG_EINVAL, "%s: workspace needs %u doubles", what, nparts);
  if (!(g2 != 0.f)) return set_error(FEDAVG_EINVAL, "%s: G2 must be nonzero", what);
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(fpf_sum_f64_kernel, dim3(nparts), dim3(kBlock), 0, s, gdiff, P, workspace);
  rc = launch_status(what);
  if (rc) return rc;
  const double c2 = 1.0 - 1.0 / static_cast<double>(g2);  // (1 - 1/G2) as a Python float
  const dim3 grid(static_cast<unsigned>((P + kBlock - 1) / kBlock < 512 ? (P + kBlock - 1) / kBlock : 512),
                  static_cast<unsigned>((n_rows + kFpfRowsPerBlock - 1) / kFpfRowsPerBlock));
  const int np = static_cast<int>(nparts);
  switch (t_kind) {
    case kF32:
      hipLaunchKernelGGL(fpf_end_round_promoted_kernel<kF32>, grid, dim3(kBlock), 0, s, diffs, ld, n_rows, keep_rows,
                         a_mat, gdiff, P, workspace, np, static_cast<double>(g2), c2);
      break;
    case kF64:
      hipLaunchKernelGGL(fpf_end_round_promoted_kernel<kF64>, grid, dim3(kBlock), 0, s, diffs, ld, n_rows, keep_rows,
                         a_mat, gdiff, P, workspace, np, static_cast<double>(g2), c2);
      break;
    case kF64FromF32:
      hipLaunchKernelGGL(fpf_end_round_promoted_kernel<kF64FromF32>, grid, dim3(kBlock), 0, s, diffs, ld, n_rows,
                         keep_rows, a_mat, gdiff, P, workspace, np, static_cast<double>(g2), c2);
      break;
    case kF16:
      hipLaunchKernelGGL(fpf_end_round_promoted_kernel<kF16>, grid, dim3(kBlock), 0, s, diffs, ld, n_rows, keep_rows,
                         a_mat, gdiff, P, workspace, np, static_cast<double>(g2), c2);
      break;
    case kBF16:
      hipLaunchKernelGGL(fpf_end_round_promoted_kernel<kBF16>, grid, dim3(kBlock), 0, s, diffs, ld, n_rows, keep_rows,
                         a_mat, gdiff, P, workspace, np, static_cast<double>(g2), c2);
      break;
    default: return set_error(FEDAVG_EINVAL, "%s: t_kind must be 0..4 (got %d)", what, t_kind);
  }
  return launch_status(what);
}

int fedavg_fpf_index_f64(const float* diffs, int64_t n_rows, int64_t ld, int64_t P, const double* a_mat,
                         const float* g_mat, double* fpf, void* stream) {
  const char* what = "fedavg_fpf_index_f64";
  int rc = check_state(diffs, n_rows, ld, P, what);
  if (rc) return rc;
  if (!a_mat || !g_mat || !fpf) return set_error(FEDAVG_EINVAL, "%s: null buffer", what);
  hipLaunchKernelGGL(fpf_index_f64a_kernel, dim3(static_cast<unsigned>(n_rows)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), diffs, ld, P, a_mat, g_mat, fpf);
  return launch_status(what);
}

int fedavg_fpf_index_lru(const float* lru_itr, const float* g_mat, int64_t n_rows, float* fpf, void* stream) {
  const char* what = "fedavg_fpf_index_lru";
  if (n_rows <= 0) return set_error(FEDAVG_EINVAL, "%s: n_rows must be >= 1", what);
  if (!lru_itr || !g_mat || !fpf) return set_error(FEDAVG_EINVAL, "%s: null buffer", what);
  hipLaunchKernelGGL(fpf_index_lru_kernel, dim3(static_cast<unsigned>((n_rows + kBlock - 1) / kBlock)), dim3(kBlock),
                     0, static_cast<hipStream_t>(stream), lru_itr, g_mat, n_rows, fpf);
  return launch_status(what);
}

}  // extern "C"
