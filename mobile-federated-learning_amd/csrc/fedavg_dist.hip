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

// STYLE L > 0 (probe): each batch's U x C loads and squares interleaved in
// (row, slice) order with at most L loads of the wave in flight, as the
// zero-copy reduce's unit loop (fedavg_segments.hip, STYLE 2)
template <int U, int C, int MINW = 1, int ACC = 1, int STYLE = 0>
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
    if constexpr (STYLE > 0) {
      constexpr int L = STYLE, N = UU * C;
      for (; k + UU <= K; k += UU) {
        __amdgpu_buffer_rsrc_t rr[UU];
#pragma unroll
        for (int u = 0; u < UU; ++u) rr[u] = uniform_rsrc(X + static_cast<int64_t>(k + u) * ld4 + blk0, bytes);
        double a[UU][ACC];
#pragma unroll
        for (int u = 0; u < UU; ++u)
#pragma unroll
          for (int c = 0; c < ACC; ++c) a[u][c] = 0.0;
        f32x4 x[N];
#pragma unroll
        for (int i = 0; i < N + L; ++i) {
          if (i < N) x[i] = ld_rsrc_nt(rr[i / C], off[i % C]);
          if (i >= L) {
            const int j = i - L;
            a[j / C][(j % C) % ACC] = sq4_add(a[j / C][(j % C) % ACC], x[j] - g[j % C]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int u = 0; u < UU; ++u) {
#pragma unroll
          for (int w = 1; w < ACC; w *= 2) {
#pragma unroll
            for (int c = 0; c + w < ACC; c += 2 * w) a[u][c] += a[u][c + w];
          }
          sqdist_rows_store<U, C>(a[u][0], partials, k + u, nwaves, wave_id);
        }
      }
    }
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

// ---------------------------------------------------------------------------
// Aggregate (:450-457) and :291 in ONE pass over the client rows.  The
// reference reads every client's update twice per round: once to average it
// (:217) and once to measure ||w_i - w_glob|| (:291).  Both passes are
// HBM-read bound on the same K x P bytes, so fusing them halves the round's
// traffic -- if every column's K values are still on chip when that column's
// average is known.  A workgroup therefore owns tiles of S columns x all K
// rows staged in LDS (K x S x 4 bytes: 25.6 KB for K = 100, S = 64):
//   1. every row segment lands in LDS by LDS-DMA (global_load_lds_dwordx4,
//      1 KiB per wave instruction, no VGPR round trip).  The 16-B slots of
//      row r are XOR-swizzled by (r & 7): slot j holds the row's slice
//      j ^ (r & 7) (the swizzle is in the per-lane GLOBAL address; LDS stays
//      linear, as LDS-DMA requires), so threads reading one slice of 8
//      consecutive rows hit 8 different bank groups;
//   2. one thread per column runs the reference's sequential chain over the
//      K rows (fl32 products and sums in client order: the bits of
//      fedavg_reduce_f32) and stores the average to `out` and to LDS;
//   3. thread t owns row t % K and the slices t / K, t / K + q, ... (q =
//      256 / K threads per row), and adds fl32(x - g)^2 in fp64 to ONE
//      register accumulator that lives across all of the workgroup's tiles.
//      At the end the q accumulators of a row are added in a fixed order.
// A thread keeps one fp64 accumulator instead of one per row, so the kernel
// is LDS-bound, not register-bound: K = 100 x 64 columns runs 6 workgroups
// per CU.  Workgroups are persistent (grid = resident workgroups) and walk the
// tiles with a grid stride, so the running workgroups sweep one compact
// window of every row, as the round-split row reduce does.
// partials[k][workgroup], then the fixed-order finalize: deterministic.
// K <= 128 (q >= 2).
// ---------------------------------------------------------------------------

// rows -> LDS for the tile at column c0: slot i = row * V + j (LDS byte
// 16 i from `buf`) holds slice j ^ (row & 7) of the row segment
// Load slots per thread at the widest K each tile width serves (fused_cols):
// 300 x 32, 128 x 64, 64 x 128, 32 x 256 columns
template <int S>
constexpr int fused_slots() {
  return S == 32 ? 10 : 8;
}

// The byte offset (row * ld + slice) of each of this thread's load slots,
// the same for every tile: computed once per workgroup, so a tile's loads
// cost one 64-bit add each instead of the row / slice / swizzle arithmetic
template <int S>
struct FusedSlots {
  int64_t off[fused_slots<S>()];
};

template <int S>
__device__ __forceinline__ FusedSlots<S> fused_slots_of(int K, int64_t ld) {
  constexpr int V = S / 4;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  FusedSlots<S> sl;
#pragma unroll
  for (int m = 0; m < fused_slots<S>(); ++m) {
    const int i = wave * 64 + m * kBlock + lane;
    const int row = i / V;
    const int c = (i % V) ^ (row & 7);
    sl.off[m] = (static_cast<int64_t>(row) * ld + 4 * c) * 4;
  }
  return sl;
}

// a full tile's loads through the precomputed slots (the ragged last tile
// takes fused_load_tile, which masks slices past the model's end)
template <int S>
__device__ __forceinline__ void fused_load_full(const float* __restrict__ X, int K, int64_t c0,
                                                const FusedSlots<S>& sl, float* buf) {
  constexpr int V = S / 4;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nload = K * V;
  const char* base = reinterpret_cast<const char*>(X + c0);
#pragma unroll
  for (int m = 0; m < fused_slots<S>(); ++m) {
    const int i0 = wave * 64 + m * kBlock;
    if (i0 < nload && i0 + lane < nload)
      __builtin_amdgcn_global_load_lds((fused_gbl_t)(base + sl.off[m]), (fused_lds_t)(buf + 4 * i0), 16, 0, 2 /* nt */);
  }
}

template <int S>
__device__ __forceinline__ void fused_load_tile(const float* __restrict__ X, int K, int64_t ld, int64_t P, int64_t c0,
                                                float* buf) {
  constexpr int V = S / 4;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nload = K * V;
  const int ncols = P - c0 < S ? static_cast<int>(P - c0) : S;
  const int nv4 = (ncols + 3) >> 2;  // slices holding valid columns (the last may run into the row padding)
  for (int i0 = wave * 64; i0 < nload; i0 += kBlock) {
    const int i = i0 + lane;
    const int row = i / V;
    const int c = (i % V) ^ (row & 7);
    if (i < nload && c < nv4)
      __builtin_amdgcn_global_load_lds((fused_gbl_t)(X + static_cast<int64_t>(row) * ld + c0 + 4 * c),
                                       (fused_lds_t)(buf + 4 * i0), 16, 0, 2 /* nt */);
  }
}


template <int S, bool DB, int RW = 0, bool LOADS_ONLY = false, int RM = 1>
__global__ __launch_bounds__(kBlock) void reduce_sqdist_f32_kernel(const float* __restrict__ X, int K, int64_t ld,
                                                                   int64_t P, int64_t ntiles,
                                                                   const float* __restrict__ W,
                                                                   float* __restrict__ out,
                                                                   double* __restrict__ partials) {
  static_assert(S == 32 || S == 64 || S == 128 || S == 256, "tile widths: 32, 64, 128 or 256 columns");
  // one tile buffer [K][S] (swizzled slots) -- two when DB -- then the tile's average [S]
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tile_floats = K * S;
  float* gs = lds + (DB ? 2 : 1) * tile_floats;
  double acc[RM][4];  // four chains per row this thread owns (one per lane of a 16-B slice)
#pragma unroll
  for (int m = 0; m < RM; ++m) acc[m][0] = acc[m][1] = acc[m][2] = acc[m][3] = 0.0;
  double acc_rows[RW > 0 ? RW : 1];      // RW > 0: one accumulator per row of this wave
#pragma unroll
  for (int r = 0; r < (RW > 0 ? RW : 1); ++r) acc_rows[r] = 0.0;
  const FusedSlots<S> slots = fused_slots_of<S>(K, ld);
  int cur = 0;
  if (DB && static_cast<int64_t>(blockIdx.x) < ntiles)
    fused_load_tile<S>(X, K, ld, P, static_cast<int64_t>(blockIdx.x) * S, lds);
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    float* tile = lds + cur * tile_floats;
    const int64_t c0 = t * S;
    const int ncols = P - c0 < S ? static_cast<int>(P - c0) : S;
    if constexpr (DB) {
      barrier_loads();  // this tile has landed; every wave is done with the other buffer
      // 1. the next tile's rows stream into the other buffer while this one is used
      if (t + gridDim.x < ntiles) fused_load_tile<S>(X, K, ld, P, (t + gridDim.x) * S, lds + (cur ^ 1) * tile_floats);
    } else {
      if (ncols == S && !RW && K * (S / 4) <= fused_slots<S>() * kBlock)  // 1. rows -> LDS
        fused_load_full<S>(X, K, c0, slots, tile);
      else
        fused_load_tile<S>(X, K, ld, P, c0, tile);
      barrier_loads();
    }
    if constexpr (LOADS_ONLY) {  // probe: the tile traffic alone (one column of each tile stored)
      if (threadIdx.x == 0) out[c0] = tile[0];
      barrier_lds();
      continue;
    }
    fused_average<S>(tile, gs, K, W, ncols, out + c0);  // 2. the average of each column
    barrier_lds();
    if constexpr (RW > 0) {
      // 3'. rows wave + 4r (r < RW), S / 64 adjacent columns per lane, one
      //     register accumulator per row
      constexpr int PER = S / 64;
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        const int row = (threadIdx.x >> 6) + 4 * r;
        if (row < K) {
          const int c = (threadIdx.x & 63) * PER;
          const float* x = tile + row * S + ((((c >> 2) ^ (row & 7))) << 2) + (c & 3);
#pragma unroll
          for (int j = 0; j < PER; ++j) {
            const float d = x[j] - gs[c + j];  // fp32 difference, as the reference forms it
            const double dd = c + j < ncols ? static_cast<double>(d) : 0.0;  // select: padding may hold NaN/inf
            acc_rows[r] = __builtin_fma(dd, dd, acc_rows[r]);
          }
        }
      }
    } else {
      fused_squares<S, RM>(tile, gs, K, ncols, acc);  // 3. :291 squares of this thread's rows over its slices
    }
    if constexpr (DB)
      cur ^= 1;
    else
      barrier_lds();  // the tile is read out before the next one lands
  }
  if constexpr (RW > 0) {
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const int row = (threadIdx.x >> 6) + 4 * r;
      if (row < K) {
        const double sr = wave_sum_dpp(acc_rows[r]);
        if ((threadIdx.x & 63) == 0) partials[static_cast<int64_t>(row) * gridDim.x + blockIdx.x] = sr;
      }
    }
    return;
  }
  fused_finish<RM>(lds, acc, K, partials);
}

// (The LDS-DMA kernel serves 17-128 rows in production, fused_plan below.
// Round 2 ran it up to 300 clients with two rows per thread above 256:
// 200 x 10M 2.74 -> 1.84 ms, 300 x 5M 1.96 -> 1.58, but 500 x 11.2M 10.8 vs
// 7.26 ms for the two passes; profiles/r02/fused/fused_many_clients*_probe.jsonl.)

// the tile + its average, and at least the 256 doubles of the final per-row sums
inline int64_t fused_lds_bytes(int64_t K, int S, bool db = false) {
  const int64_t b = ((db ? 2 : 1) * K + 1) * S * 4;
  return b > kBlock * 8 ? b : kBlock * 8;
}

// Workgroups per CU the fused kernel keeps resident at this K (LDS-bound),
// after raising the kernel's dynamic LDS limit past 64 KiB where needed;
// cached per (device, S, K).  0 = the LDS request cannot be granted.
template <int S, bool DB = false, int RW = 0, bool LO = false, int RM = 1>
int fused_per_cu(int64_t K) {
  static std::mutex mu;
  static std::map<std::pair<int, int64_t>, int> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find({dev, K});
  if (it != cache.end()) return it->second;
  const auto kern = reduce_sqdist_f32_kernel<S, DB, RW, LO, RM>;
  const int64_t lds = fused_lds_bytes(K, S, DB);
  int per_cu = 0;
  if (lds > 65536 && hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                         hipFuncAttributeMaxDynamicSharedMemorySize,
                                         static_cast<int>(lds)) != hipSuccess) {
    (void)hipGetLastError();
  } else if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kBlock, static_cast<size_t>(lds)) !=
             hipSuccess) {
    (void)hipGetLastError();
    per_cu = 0;
  }
  cache[{dev, K}] = per_cu;
  return per_cu;
}

template <int S, bool DB = false, int RW = 0, bool LO = false, int RM = 1>
int64_t fused_grid(int64_t K, int64_t P, int blocks_per_cu) {
  const int per_cu = blocks_per_cu > 0 ? blocks_per_cu : fused_per_cu<S, DB, RW, LO, RM>(K);
  const int64_t ntiles = (P + S - 1) / S;
  const int64_t g = static_cast<int64_t>(per_cu) * cu_count();
  return ntiles < g ? ntiles : g;
}

template <int S, bool DB, int RW, bool LO, int RM>
int launch_fused_rm(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights, float* out,
                    double* partials, int64_t partial_elems, double* sumsq, int blocks_per_cu, hipStream_t s,
                    const char* what) {
  if (RW > 0 && K > 4 * RW) return set_error(FEDAVG_EMODE, "%s: %d rows per wave cover K <= %d", what, RW, 4 * RW);
  if (fused_per_cu<S, DB, RW, LO, RM>(K) <= 0)
    return set_error(FEDAVG_EMODE, "%s: the %d-column tile does not fit LDS at K = %lld", what, S, (long long)K);
  const int64_t ntiles = (P + S - 1) / S;
  const int64_t grid = fused_grid<S, DB, RW, LO, RM>(K, P, blocks_per_cu);
  if (partial_elems < K * grid)
    return set_error(FEDAVG_EINVAL, "%s: workspace needs %lld doubles", what, (long long)(K * grid));
  hipLaunchKernelGGL((reduce_sqdist_f32_kernel<S, DB, RW, LO, RM>), dim3(static_cast<unsigned>(grid)), dim3(kBlock),
                     static_cast<unsigned>(fused_lds_bytes(K, S, DB)), s, clients, static_cast<int>(K), ld, P, ntiles,
                     weights, out, partials);
  int rc = launch_status(what);
  if (rc) return rc;
  hipLaunchKernelGGL(client_sqdist_finalize_kernel, dim3(static_cast<unsigned>(K)), dim3(kBlock), 0, s, partials, grid,
                     sumsq);
  return launch_status(what);
}

// RM = rows per thread in the squares: 1 up to 256 rows, else 2
template <int S, bool DB = false, int RW = 0, bool LO = false>
int launch_fused(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights, float* out,
                 double* partials, int64_t partial_elems, double* sumsq, int blocks_per_cu, hipStream_t s,
                 const char* what) {
  if (K <= kBlock)
    return launch_fused_rm<S, DB, RW, LO, 1>(clients, K, P, ld, weights, out, partials, partial_elems, sumsq,
                                             blocks_per_cu, s, what);
  if constexpr (RW == 0 && !LO)
    return launch_fused_rm<S, DB, RW, LO, 2>(clients, K, P, ld, weights, out, partials, partial_elems, sumsq,
                                             blocks_per_cu, s, what);
  return set_error(FEDAVG_EMODE, "%s: this variant covers K <= %d", what, kBlock);
}

// ---------------------------------------------------------------------------
// Register-staged fused tiles (round 3).  The LDS-DMA form above fills a
// tile straight into LDS and has nothing in flight while a tile is averaged
// and squared; LDS-DMA also tops out near 6.5-6.8 TB/s chip-wide where
// register loads reach the row reduce's 7.1.  Here the tile goes through
// registers:
//   slot m of thread t holds row r0 + m R, 16-B slice sl of the tile
//   (V = S / 4 slices per row segment, R = 256 / V rows per slot round,
//   r0 = t / V, sl = t % V), so a wave instruction reads 64 / V row segments
//   of S x 4 bytes and the slot's LDS image is the linear 16 (t + 256 m);
// per tile:
//   1. the staged slots (loaded one tile earlier) are written to LDS,
//   2. the NEXT tile's loads are issued into the same registers -- they stay
//      in flight while this tile is averaged and squared,
//   3. the reference's sequential chain, one thread per column (S threads),
//   4. every thread squares its own slots against the tile's average; slot m
//      always belongs to the same row, so one fp64 accumulator per slot lives
//      across all tiles, and the V threads of a row (one per slice) are added
//      in a fixed order at the end: partials[row][workgroup].
// MODE 1 / 2 are traffic probes (1: loads only; 2: loads + LDS writes).
// ---------------------------------------------------------------------------
// FLAGS (probes): 1 = TILED buffer [ntiles][K][S] (each tile's rows contiguous);
// 2 = the workgroups of one XCD take contiguous tiles of a sweep (dispatch
// puts workgroup b on XCD b % 8); 4 = and the workgroups of one CU too
// (b, b + 256, ... share a CU).  Both remaps are bijections of the sweep: a
// different placement only changes the speed.
// DEPTH 2: two tiles' loads in flight per workgroup (two register stages,
// the tile in LDS a third).  MODE 3: loads only with no LDS at all (probe:
// the tile walk at the occupancy registers alone allow).
constexpr int rs_min_waves(int S, int DEPTH) {
  return DEPTH == 1 || S == 256 ? 1 : (S <= 64 ? 4 : (DEPTH == 2 ? 3 : 2));
}

template <int S, int SLOTS, int MODE = 0, int FLAGS = 0, int DEPTH = 1>
__global__ __launch_bounds__(kBlock, rs_min_waves(S, DEPTH)) void reduce_sqdist_rs_kernel(const float* __restrict__ X, int K, int64_t ld,
                                                                  int64_t P, int64_t ntiles,
                                                                  const float* __restrict__ W,
                                                                  float* __restrict__ out,
                                                                  double* __restrict__ partials) {
  static_assert(S == 32 || S == 64 || S == 128 || S == 256, "tile widths: 32, 64, 128 or 256 columns");
  static_assert(DEPTH >= 1 && DEPTH <= 3, "one to three tiles in flight");
  constexpr int V = S / 4;
  constexpr int R = kBlock / V;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* gs = lds + K * S;
  const int t = threadIdx.x;
  const int r0 = t / V, sl = t % V;
  const int nslot = r0 < K ? (K - r0 + R - 1) / R : 0;  // slots of this thread that hold a row
  constexpr bool TILED = (FLAGS & 1) != 0;
  const int64_t rstride = TILED ? S : ld;  // TILED: ld unused
  const char* p0 = reinterpret_cast<const char*>(X) + (static_cast<int64_t>(r0) * rstride + 4 * sl) * 4;
  const int64_t mstride = static_cast<int64_t>(R) * rstride * 4;
  f32x4* tile4 = reinterpret_cast<f32x4*>(lds);
  double acc[SLOTS];
#pragma unroll
  for (int m = 0; m < SLOTS; ++m) acc[m] = 0.0;

  // this thread's slots of tile `tt` into registers (slices past the model's
  // end are not loaded: the last row's would run off the allocation)
  const auto issue = [&](f32x4 (&xs)[SLOTS], int64_t tt) {
    const int64_t c0 = tt * S;
    const char* p = p0 + (TILED ? tt * K * S : c0) * 4;
    const bool slice_ok = c0 + 4 * sl < P;
#pragma unroll
    for (int m = 0; m < SLOTS; ++m)
      if (m < nslot && slice_ok) xs[m] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + m * mstride));
  };

  // one tile: staged slots -> LDS, refill the stage with tile `next`, average, squares
  const auto body = [&](f32x4 (&xs)[SLOTS], int64_t tt, int64_t next) {
    const int64_t c0 = tt * S;
    const int ncols = P - c0 < S ? static_cast<int>(P - c0) : S;
    if constexpr (MODE == 1 || MODE == 3) {
      float probe = 0.f;
#pragma unroll
      for (int m = 0; m < SLOTS; ++m)
        if (m < nslot) probe += xs[m].x;  // consume the loads
      if (next < ntiles) issue(xs, next);
      if (t == 0) out[c0] = probe;
      return;
    }
    barrier_lds();  // every wave is done with the previous tile
#pragma unroll
    for (int m = 0; m < SLOTS; ++m)
      if (m < nslot) tile4[t + kBlock * m] = xs[m];  // 1. (a ragged slice keeps stale data: never used)
    barrier_lds();
    if (next < ntiles) issue(xs, next);  // 2. that stage's next tile in flight
    if constexpr (MODE == 2) {
      if (t == 0) out[c0] = lds[0];
      return;
    }
    if (t < S) {  // 3. the average of column t, in the reference's order
      float a = lds[t] * W[0];
      constexpr int kUnroll = S == 64 ? 32 : 16;
#pragma unroll kUnroll
      for (int k = 1; k < K; ++k) {
        const float term = lds[k * S + t] * W[k];
        a = a + term;
      }
      gs[t] = a;
      if (t < ncols) out[c0 + t] = a;
    }
    barrier_lds();
    // 4. squares of this thread's slots: fl32(x - g) as the reference forms it, fp64 square-adds
    const f32x4 g = reinterpret_cast<const f32x4*>(gs)[sl];
    const int nv = ncols - 4 * sl;  // valid columns of this slice
    if (nv >= 4) {
#pragma unroll
      for (int m = 0; m < SLOTS; ++m)
        if (m < nslot) {
          const f32x4 d = tile4[t + kBlock * m] - g;
          const double dx = d.x, dy = d.y, dz = d.z, dw = d.w;
          acc[m] = __builtin_fma(dx, dx, acc[m]);
          acc[m] = __builtin_fma(dy, dy, acc[m]);
          acc[m] = __builtin_fma(dz, dz, acc[m]);
          acc[m] = __builtin_fma(dw, dw, acc[m]);
        }
    } else if (nv > 0) {  // ragged slice: select (not multiply) -- padding may hold NaN/inf
#pragma unroll
      for (int m = 0; m < SLOTS; ++m)
        if (m < nslot) {
          const f32x4 d = tile4[t + kBlock * m] - g;
          const double dx = d.x, dy = nv > 1 ? d.y : 0.f, dz = nv > 2 ? d.z : 0.f;
          acc[m] = __builtin_fma(dx, dx, acc[m]);
          acc[m] = __builtin_fma(dy, dy, acc[m]);
          acc[m] = __builtin_fma(dz, dz, acc[m]);
        }
    }
  };

  int64_t first = blockIdx.x;  // this workgroup's position in every sweep of gridDim.x tiles
  if constexpr ((FLAGS & 6) != 0) {
    const int64_t b = blockIdx.x, per_xcd = gridDim.x / 8;
    if constexpr ((FLAGS & 4) != 0) {
      const int64_t j = b / 8, per_cu = per_xcd / 32;
      first = (b % 8) * per_xcd + (j % 32) * per_cu + j / 32;
    } else {
      first = (b % 8) * per_xcd + b / 8;
    }
  }
  const int64_t G = gridDim.x;
  f32x4 xa[SLOTS];
  if (first < ntiles) issue(xa, first);
  if constexpr (DEPTH == 1) {
    for (int64_t tt = first; tt < ntiles; tt += G) body(xa, tt, tt + G);
  } else if constexpr (DEPTH == 2) {
    f32x4 xb[SLOTS];
    if (first + G < ntiles) issue(xb, first + G);
    for (int64_t tt = first; tt < ntiles; tt += 2 * G) {
      body(xa, tt, tt + 2 * G);
      if (tt + G >= ntiles) break;
      body(xb, tt + G, tt + 3 * G);
    }
  } else {
    f32x4 xb[SLOTS], xc[SLOTS];
    if (first + G < ntiles) issue(xb, first + G);
    if (first + 2 * G < ntiles) issue(xc, first + 2 * G);
    for (int64_t tt = first; tt < ntiles; tt += 3 * G) {
      body(xa, tt, tt + 3 * G);
      if (tt + G >= ntiles) break;
      body(xb, tt + G, tt + 4 * G);
      if (tt + 2 * G >= ntiles) break;
      body(xc, tt + 2 * G, tt + 5 * G);
    }
  }
  if constexpr (MODE != 0) return;
  // the V slot sums of a row are contiguous in red[]: row * V + slice = t + 256 m
  barrier_loads();
  double* red = reinterpret_cast<double*>(lds);
#pragma unroll
  for (int m = 0; m < SLOTS; ++m)
    if (m < nslot) red[t + kBlock * m] = acc[m];
  barrier_lds();
  for (int row = t; row < K; row += kBlock) {
    double s = red[row * V];
#pragma unroll
    for (int j = 1; j < V; ++j) s += red[row * V + j];
    partials[static_cast<int64_t>(row) * gridDim.x + blockIdx.x] = s;
  }
}

// LDS of a register-staged tile: [K][S] + the average [S]; the final per-row
// sums need K * V doubles (= K * S * 2 bytes, inside the tile)
inline int64_t fused_rs_lds_bytes(int64_t K, int S, int mode = 0) { return mode == 3 ? 0 : (K + 1) * S * 4; }

template <int S, int SLOTS, int MODE, int FLAGS = 0, int DEPTH = 1>
int fused_rs_per_cu(int64_t K) {
  static std::mutex mu;
  static std::map<std::pair<int, int64_t>, int> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find({dev, K});
  if (it != cache.end()) return it->second;
  const auto kern = reduce_sqdist_rs_kernel<S, SLOTS, MODE, FLAGS, DEPTH>;
  const int64_t lds = fused_rs_lds_bytes(K, S, MODE);
  int per_cu = 0;
  if (lds > 65536 && hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                         hipFuncAttributeMaxDynamicSharedMemorySize,
                                         static_cast<int>(lds)) != hipSuccess) {
    (void)hipGetLastError();
  } else if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kBlock, static_cast<size_t>(lds)) !=
             hipSuccess) {
    (void)hipGetLastError();
    per_cu = 0;
  }
  cache[{dev, K}] = per_cu;
  return per_cu;
}

template <int S, int SLOTS, int MODE, int FLAGS = 0, int DEPTH = 1>
int64_t fused_rs_grid(int64_t K, int64_t P, int blocks_per_cu) {
  const int per_cu = blocks_per_cu > 0 ? blocks_per_cu : fused_rs_per_cu<S, SLOTS, MODE, FLAGS, DEPTH>(K);
  const int64_t ntiles = (P + S - 1) / S;
  const int64_t g = static_cast<int64_t>(per_cu) * cu_count();
  return ntiles < g ? ntiles : g;
}

template <int S, int SLOTS, int MODE = 0, int FLAGS = 0, int DEPTH = 1>
int launch_fused_rs(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights, float* out,
                    double* partials, int64_t partial_elems, double* sumsq, int blocks_per_cu, hipStream_t s,
                    const char* what) {
  if ((K * S + 1023) / 1024 > SLOTS)
    return set_error(FEDAVG_EMODE, "%s: %d slots per thread cover K <= %d at %d columns", what, SLOTS,
                     SLOTS * 1024 / S, S);
  const int per_cu = fused_rs_per_cu<S, SLOTS, MODE, FLAGS, DEPTH>(K);
  if (per_cu <= 0)
    return set_error(FEDAVG_EMODE, "%s: the %d-column tile does not fit LDS at K = %lld", what, S, (long long)K);
  if (blocks_per_cu > per_cu)
    return set_error(FEDAVG_EMODE, "%s: %d workgroups per CU requested, %d resident", what, blocks_per_cu, per_cu);
  const int64_t ntiles = (P + S - 1) / S;
  const int64_t grid = fused_rs_grid<S, SLOTS, MODE, FLAGS, DEPTH>(K, P, blocks_per_cu);
  if ((FLAGS & 6) != 0 && (cu_count() != 256 || grid != (blocks_per_cu > 0 ? blocks_per_cu : per_cu) * 256LL))
    return set_error(FEDAVG_EMODE, "%s: the XCD / CU remaps need a full grid on 256 CUs", what);
  if (partial_elems < K * grid)
    return set_error(FEDAVG_EINVAL, "%s: workspace needs %lld doubles", what, (long long)(K * grid));
  hipLaunchKernelGGL((reduce_sqdist_rs_kernel<S, SLOTS, MODE, FLAGS, DEPTH>), dim3(static_cast<unsigned>(grid)),
                     dim3(kBlock), static_cast<unsigned>(fused_rs_lds_bytes(K, S, MODE)), s, clients, static_cast<int>(K), ld, P, ntiles,
                     weights, out, partials);
  int rc = launch_status(what);
  if (rc || MODE != 0) return rc;
  hipLaunchKernelGGL(client_sqdist_finalize_kernel, dim3(static_cast<unsigned>(K)), dim3(kBlock), 0, s, partials, grid,
                     sumsq);
  return launch_status(what);
}

// ---------------------------------------------------------------------------
// Wave-owned windows (round 3).  The tile kernels above share a tile between
// the 4 waves of a workgroup: one thread per COLUMN runs the chain from LDS,
// so every tile crosses LDS and a barrier, and each workgroup asks for K row
// segments of only S x 4 bytes at a time.  Here one WAVE owns a window of
// 64 x VEC columns and ALL K rows of it in registers (lane l: columns
// l*VEC .. l*VEC + VEC - 1 of every row; K x VEC VGPRs), so
//   - the chain is per lane, straight from registers (packed fp32 mul/add:
//     the bits of fedavg_reduce_f32), no LDS, no barrier;
//   - the squares are per lane as well, and row i's registers are reloaded
//     with the NEXT window's row i right after row i is squared: the next
//     window's K loads are issued during this window's squares (the
//     hardware's 63-load vmcnt cap throttles the issue, nothing else does),
//     so one register image serves both windows with no double buffer;
//   - a workgroup's NW waves take adjacent windows: NW x 64 x VEC x 4 bytes
//     of every row in flight together (2 KiB at VEC 2, NW 4).
// Row sums: a lane's fp64 partial of row i covers VEC columns; each batch of
// 8 rows is folded across the wave with v_permlane32_swap (8 rows -> 4
// registers, each row over 32 lanes), v_permlane16_swap (-> 2 registers, 16
// lanes per row) and one row_ror:8 exchange (-> 1 register: row 4h + [0, 2,
// 1, 3][l >> 4] in the 8 lanes l with (l >> 3) & 1 = h), added into one fp64
// accumulator per batch that lives across all windows; the 8-lane groups are
// summed once at the end (quad_perm / half-mirror DPP) -> partials[row][wave]
// -> the fixed-order finalize.  Deterministic; windows are read through one
// SGPR buffer descriptor per row whose range ends at the model's last 16-B
// slice (num_records 0 past the last window: the tail's reloads are dropped
// in the address unit, no traffic), columns past P inside the last slice are
// zeroed before the chain.
// MODE 256 (probe): the chain's weights by row broadcast (lane 16r + j of
// wvb[k] = row 16k + j's weight) in hand-pipelined 8-row blocks
// (chain8_row_bcast2): no v_readlane / LDS weight reads, four VALU a row.
// MODE 1: loads only (a traffic probe: wrong results).  MODE 4 (probe):
// squares in fp32 (the VEC columns' fl32(d*d) summed in fp32, widened once
// per row): the fp64 VALU stream's share of time and clock, measured.
// ---------------------------------------------------------------------------
// (window helpers: WinVec, fold32/16/8, win_batch_row, win_load, win_sq in common.hpp)

template <int KMAX, int VEC, int NW, int MODE = 0, int MINW = win_min_waves(KMAX, VEC)>
__global__ __launch_bounds__(64 * NW, MINW) void reduce_sqdist_win_kernel(
    const float* __restrict__ X, int K, int64_t ld, int64_t P, int64_t nwin, const float* __restrict__ W,
    float* __restrict__ out, double* __restrict__ partials) {
  typedef typename WinVec<VEC>::T V;
  constexpr int WC = 64 * VEC;
  constexpr int NB = (KMAX + 7) / 8;
  const int lane = threadIdx.x & 63;
  const int64_t GW = static_cast<int64_t>(gridDim.x) * NW;
  const int64_t gw = static_cast<int64_t>(blockIdx.x) * NW + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t voff = static_cast<uint32_t>(lane) * VEC * 4;
  const int64_t P4 = (P + 3) & ~static_cast<int64_t>(3);  // rows are read up to their last 16-B slice
  const int64_t row_bytes = ld * 4;
  const uint32_t rb32 = static_cast<uint32_t>(row_bytes);  // MODE 128: soffset steps
  const bool upper = (lane & 8) != 0;

  // window w's bytes per row (0: no such window -- its loads return 0 and move nothing)
  const auto win_bytes = [&](int64_t w) -> int {
    if (w >= nwin) return 0;
    const int64_t n = P4 - w * WC;
    return static_cast<int>((n < WC ? n : WC) * 4);
  };
  // Rows K..KMAX-1 are padding: loaded through an empty descriptor (0, no
  // traffic) and weighted -0.0 in the chain (x + (+0 * -0) == x for every x,
  // -0 and NaN included); their sums are never written.  Every row bound is
  // computed per window from an opaque copy of K: hoisted out of the window
  // loop the KMAX row masks would not fit the SGPRs.  Row i's descriptor base
  // advances one row per load through an opaque pointer for the same reason.
  // The LDS accumulators are per lane: no other lane touches them, no barrier.
  // LDS: the weights padded to KMAX with -0.0 (read as uniform 16-B
  // broadcasts in the chain), then each wave's per-batch row accumulators
  // [NB][64] (one fp64 per lane per batch: registers are the window's)
  __shared__ __attribute__((aligned(16))) float wl[(KMAX + 3) & ~3];
  __shared__ double accl[NW][NB][64];
  for (int i = threadIdx.x; i < ((KMAX + 3) & ~3); i += 64 * NW) wl[i] = i < K ? W[i] : -0.0f;
  float wv0 = lane < K ? W[lane] : -0.0f, wv1 = 64 + lane < K ? W[64 + lane] : -0.0f;  // LROWS: lane l = W[l], W[64 + l]
  constexpr bool BCW = (MODE & 256) != 0;
  static_assert(!BCW || (VEC == 2 && KMAX >= 16), "broadcast weights: VEC 2, 8-row blocks");
  float wvb[BCW ? (KMAX + 15) / 16 : 1];
  if constexpr (BCW) {
#pragma unroll
    for (int k = 0; k < (KMAX + 15) / 16; ++k) {
      const int row = 16 * k + (lane & 15);
      wvb[k] = row < K ? W[row] : -0.0f;
    }
  }
  double* acc = &accl[threadIdx.x >> 6][0][lane];
#pragma unroll
  for (int b = 0; b < NB; ++b) acc[64 * b] = 0.0;
  __syncthreads();
  // MODE 64 (probe): rows 0..E-1 of the next window are staged in LDS by
  // LDS-DMA before this window's chain (the VGPR rows free up only in the
  // squares), so E rows stay in flight through the chain; K > E
  constexpr bool LROWS = (MODE & 64) != 0;
  constexpr int E = LROWS ? 24 : 0;
  static_assert(!LROWS || VEC == 2, "LDS rows: 512-B row segments (2 x 64 lanes x 4 B)");
  __shared__ __attribute__((aligned(16))) float rowl[LROWS ? NW : 1][LROWS ? E : 1][LROWS ? WC : 1];
  float* myrows = &rowl[LROWS ? (threadIdx.x >> 6) : 0][0][0];
  // the wave's LDS slot base as a wave-uniform (SGPR) value: M0 for every DMA
  const uint32_t lds_base = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)myrows)));
  const auto dma_row = [&](int i, const char* rp, int bytes) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(rp), 0, bytes, 0x00020000);
    // two dword DMAs of 256 B (all 64 lanes: no exec branch around them)
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(uintptr_t)(lds_base + i * WC * 4), 4, lane * 4, 0, 0, 2);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(uintptr_t)(lds_base + i * WC * 4 + 256), 4, lane * 4 + 256,
                                             0, 0, 2);
  };
  V x[KMAX];
  {
    int Kw = K;
    asm volatile("" : "+s"(Kw));
    const int nb = win_bytes(gw);
    const char* rp = reinterpret_cast<const char*>(X + gw * WC);
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
      if (i < E) {
        asm volatile("" : "+s"(rp));
        dma_row(i, rp, nb);
        rp += row_bytes;
        continue;
      }
      asm volatile("" : "+s"(rp));
      x[i] = win_load<VEC>(__builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(rp), 0, i < Kw ? nb : 0, 0x00020000),
                           voff);
      rp += row_bytes;
    }
  }
  float probe = 0.f;
  for (int64_t w = gw; w < nwin; w += GW) {
    int Kw = K;
    asm volatile("" : "+s"(Kw));
    const int64_t c0 = w * WC;
    const int64_t cl = c0 + lane * VEC;  // this lane's first column
    const int nbn = win_bytes(w + GW);
    const char* rp = reinterpret_cast<const char*>(X + (w + GW) * WC);
    if constexpr (LROWS) {
      // this window's LDS rows have landed (the E oldest loads in flight:
      // at most the KMAX - E VGPR rows issued after them are outstanding)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(KMAX - E < 63 ? KMAX - E : 63) : "memory");  // (2 DMAs per LDS row)
#pragma unroll
      for (int i = 0; i < E; ++i) x[i] = *reinterpret_cast<const V*>(myrows + i * WC + lane * VEC);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read out before the next window's DMA lands
      const char* rq = reinterpret_cast<const char*>(X + (w + GW) * WC);
#pragma unroll
      for (int i = 0; i < E; ++i) {
        asm volatile("" : "+s"(rq));
        dma_row(i, rq, nbn);
        rq += row_bytes;
      }
      rp += E * row_bytes;  // the VGPR rows start at row E
    }
    // MODE 128 (probe): one descriptor per 8 rows with the row in soffset.
    // The range check covers soffset + voffset, so a group's record count
    // ends at its last existing row's window bytes (rows past K, and the
    // window past the model's last slice on that row, read 0); the other
    // rows of a ragged window read their padding (zeroed before the chain).
    // Needs 7 row pitches + a window < 4 GiB (the launcher checks).
    __amdgpu_buffer_rsrc_t grs;
    const char* gp = reinterpret_cast<const char*>(X + (w + GW) * WC) + E * row_bytes;
    const auto reload = [&](int i) {  // row i of the next window into x[i]
      if constexpr ((MODE & 128) != 0) {
        const int j = i & 7;
        if (j == 0) {
          asm volatile("" : "+s"(gp));
          const int rows = Kw - (i & ~7);  // rows of this group that exist
          const uint32_t nr = (nbn == 0 || rows <= 0)
                                  ? 0u
                                  : static_cast<uint32_t>((rows < 8 ? rows : 8) - 1) * rb32 + static_cast<uint32_t>(nbn);
          grs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(gp), 0, static_cast<int>(nr), 0x00020000);
          gp += 8 * row_bytes;
        }
        x[i] = win_load<VEC>(grs, voff, static_cast<uint32_t>(j) * rb32);
        return;
      }
      asm volatile("" : "+s"(rp));
      x[i] = win_load<VEC>(__builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(rp), 0, i < Kw ? nbn : 0, 0x00020000),
                           voff);
      rp += row_bytes;
    };
    if constexpr ((MODE & 1) != 0) {
#pragma unroll
      for (int i = 0; i < KMAX; ++i) {
#pragma unroll
        for (int v = 0; v < VEC; ++v) probe += x[i][v];
        if (i >= E) reload(i);
      }
      continue;
    }
    const bool ragged = c0 + WC > P;
    if (ragged) {  // columns past P (the last slice's padding) are zeroed: never NaN in the squares
#pragma unroll
      for (int i = 0; i < KMAX; ++i) {
#pragma unroll
        for (int v = 0; v < VEC; ++v)
          if (cl + v >= P) x[i][v] = 0.f;
      }
    }
    // the reference's chain, per lane: fl32(x_0 w_0), then + fl32(x_i w_i) in client order
    V a;
    if constexpr (BCW) {
      float a0 = -0.0f, a1 = -0.0f;  // fl32(-0.0 + p) is p, bit for bit
      float tc0 = mul_row_bcast<0>(wvb[0], x[0][0]), tc1 = mul_row_bcast<0>(wvb[0], x[0][1]);
      constexpr int NBLK = KMAX / 8, REM = KMAX % 8;
      static_for<NBLK>([&](auto bc) {
        constexpr int b = decltype(bc)::value;
        constexpr bool last = b == NBLK - 1 && REM == 0;
        chain8_row_bcast2<b % 2, last>(a0, a1, tc0, tc1, wvb[b / 2], wvb[last ? b / 2 : (b + 1) / 2], x + 8 * b);
      });
      static_for<REM>([&](auto rc) {  // the rows past the last 8-row block (tc: row 8 NBLK + r's product)
        constexpr int i = 8 * NBLK + decltype(rc)::value;
        float n0 = 0.f, n1 = 0.f;
        if constexpr (i + 1 < KMAX) {
          n0 = mul_row_bcast<i + 1>(wvb[(i + 1) / 16], x[i + 1][0]);
          n1 = mul_row_bcast<i + 1>(wvb[(i + 1) / 16], x[i + 1][1]);
        }
        a0 = a0 + tc0;
        a1 = a1 + tc1;
        tc0 = n0;
        tc1 = n1;
      });
      a[0] = a0;
      a[1] = a1;
    } else if constexpr (LROWS) {
      // weights from VGPR lanes (v_readlane): an LDS read here would wait for
      // the LDS-DMA just issued (the compiler cannot tell the arrays apart)
      asm volatile("" : "+v"(wv0), "+v"(wv1));  // re-read per window: not hoisted into SGPRs
#pragma unroll
      for (int i = 0; i < KMAX; ++i) {
        const float wi = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(i < 64 ? wv0 : wv1), i & 63));
        if (i == 0) {
          a = x[0] * wi;
        } else {
          const V t = x[i] * wi;
          a = a + t;
        }
      }
    } else {
    int wo = 0;  // re-read per window (an opaque LDS offset): not held in registers across windows
    asm volatile("" : "+v"(wo));
#pragma unroll
    for (int q = 0; q < (KMAX + 3) / 4; ++q) {
      const f32x4 w4 = *reinterpret_cast<const f32x4*>(&wl[wo + 4 * q]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = 4 * q + j;
        if (i == 0) {
          a = x[0] * w4[0];
        } else if (i < KMAX) {
          const V t = x[i] * w4[j];
          a = a + t;
        }
      }
    }
    }
    if (!ragged) {
      __builtin_nontemporal_store(static_cast<typename WinVec<VEC>::TA>(a), reinterpret_cast<typename WinVec<VEC>::TA*>(out + cl));
    } else {
#pragma unroll
      for (int v = 0; v < VEC; ++v)
        if (cl + v < P) out[cl + v] = a[v];
    }
    // squares of fl32(x - g), each row reloaded with the next window's row as soon as it is squared
    if constexpr ((MODE & 2) != 0) __builtin_amdgcn_s_setprio(2);  // probe: the reload issue first (no effect)
    if constexpr ((MODE & 16) != 0) __builtin_amdgcn_s_barrier();  // probe: the workgroup's waves reload in step
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      double p[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = 8 * b + j;
        p[j] = 0.0;
        if (i < KMAX) {
          if constexpr ((MODE & 4) != 0) {  // probe: fp32 squares
            const V d = x[i] - a;
            float sq = d[0] * d[0];
#pragma unroll
            for (int v = 1; v < VEC; ++v) sq = sq + d[v] * d[v];
            p[j] = static_cast<double>(sq);
          } else {
            p[j] = win_sq<VEC>(x[i] - a);
          }
          if (i >= E) reload(i);
        }
      }
      if constexpr ((MODE & 8) != 0) {  // probe: no folds (rows mixed: timing only)
        acc[64 * b] += ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
        continue;
      }
      const double q01 = fold32(p[0], p[1]), q23 = fold32(p[2], p[3]);
      const double q45 = fold32(p[4], p[5]), q67 = fold32(p[6], p[7]);
      acc[64 * b] += fold8(fold16(q01, q23), fold16(q45, q67), upper);
    }
    if constexpr ((MODE & 2) != 0) __builtin_amdgcn_s_setprio(0);
  }
  if constexpr ((MODE & 1) != 0) {
    if (probe == 12345.f) out[0] = probe;  // keep the loads
    return;
  }
  const int row_in = win_batch_row(lane);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    double s = acc[64 * b];
    s += dpp_move_f64<0xB1, 0xF>(s);   // quad_perm [1,0,3,2]
    s += dpp_move_f64<0x4E, 0xF>(s);   // quad_perm [2,3,0,1]
    s += dpp_move_f64<0x141, 0xF>(s);  // row_half_mirror: the other quad of the 8-lane group
    const int row = 8 * b + row_in;
    if ((lane & 7) == 0 && row < K) partials[static_cast<int64_t>(row) * GW + gw] = s;
  }
}

// waves of a window launch: every resident workgroup (persistent), or one
// per NW windows when the model has fewer
template <int KMAX, int VEC, int NW, int MODE = 0, int MINW = win_min_waves(KMAX, VEC)>
int64_t fused_win_waves(int64_t P, int blocks_per_cu) {
  const auto kern = reduce_sqdist_win_kernel<KMAX, VEC, NW, MODE, MINW>;
  const int64_t per_cu = blocks_per_cu > 0 ? blocks_per_cu : resident_blocks(kern, 64 * NW) / cu_count();
  const int64_t nwin = (P + 64 * VEC - 1) / (64 * VEC);
  const int64_t need = (nwin + NW - 1) / NW;
  const int64_t grid = per_cu * cu_count();
  return (grid < need ? grid : need) * NW;
}

template <int KMAX, int VEC, int NW, int MODE = 0, int MINW = win_min_waves(KMAX, VEC)>
int launch_fused_win(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights, float* out,
                     double* partials, int64_t partial_elems, double* sumsq, int blocks_per_cu, hipStream_t s,
                     const char* what) {
  if (K > KMAX) return set_error(FEDAVG_EMODE, "%s: this window kernel covers K <= %d", what, KMAX);
  if ((MODE & 64) != 0 && K <= 24) return set_error(FEDAVG_EMODE, "%s: LDS rows need K > 24", what);
  if ((MODE & 128) != 0 && ld * 4 * 7 + 64 * VEC * 4 >= (int64_t(1) << 32))
    return set_error(FEDAVG_EMODE, "%s: 8-row descriptors need 7 row pitches + a window < 4 GiB", what);
  const int64_t waves = fused_win_waves<KMAX, VEC, NW, MODE, MINW>(P, blocks_per_cu);
  if (waves <= 0) return set_error(FEDAVG_EMODE, "%s: the window kernel is not resident", what);
  if (partial_elems < K * waves)
    return set_error(FEDAVG_EINVAL, "%s: workspace needs %lld doubles", what, (long long)(K * waves));
  const int64_t nwin = (P + 64 * VEC - 1) / (64 * VEC);
  hipLaunchKernelGGL((reduce_sqdist_win_kernel<KMAX, VEC, NW, MODE, MINW>), dim3(static_cast<unsigned>(waves / NW)),
                     dim3(64 * NW), 0, s, clients, static_cast<int>(K), ld, P, nwin, weights, out, partials);
  int rc = launch_status(what);
  if (rc || (MODE & 1) != 0) return rc;
  hipLaunchKernelGGL(client_sqdist_finalize_kernel, dim3(static_cast<unsigned>(K)), dim3(kBlock), 0, s, partials,
                     waves, sumsq);
  return launch_status(what);
}

// ---------------------------------------------------------------------------
// Split-row windows (round 5) for 369-1024 rows.  The register-staged tiles
// ran 500 x 11.2M at 5.4 ms (52 % of HBM peak; a tile's K-step chain runs on
// 32 lanes only) and the two passes took over beyond 512 rows.  A workgroup of ns = ceil(K / KH) <=
// NSMAX waves owns a window of 64 x VEC columns; wave h holds rows h*KH ..
// h*KH + KH - 1 in registers.  The chain keeps the reference's order: wave 0
// runs its rows, hands its fp32 partial over LDS to wave 1, ... wave ns-1
// ends it and stores the average; then every wave squares its own rows
// against it and reloads them from the next window (as reduce_sqdist_win2).
// Rows past K load through an empty descriptor (+0) with weight -0.0, which
// leaves every chain value unchanged.
// PF > 0: the first PF rows of the next window are loaded into spare
// registers as the window starts, so HBM has work while the chain runs (at
// one workgroup per CU nothing else is in flight then: the reloads wait for
// the squares, the squares for the chain's last wave); after squaring row
// i < PF the wave takes the prefetched row instead of reloading it.
// LE > 0 (round 6 probe): rows PF .. PF+LE-1 of the next window go to LDS by
// LDS-DMA as the window starts (no registers: the row loads stream through
// the chain), and are read back in the squares in place of their reloads.
// MODE (probe, timing only): 1 = no chain (every wave takes x[0] as the
// average, no hand-offs), 2 = no squares (rows reloaded, nothing summed),
// 16 = the chain's weights by DPP broadcast: lane 16r + j of wv[k] holds row
// 16k + j's weight (every r), read once per launch, and row_newbcast:j hands
// it to the v_mul (no LDS reads and no lgkmcnt waits inside a turn),
// 8 = timeline: lane 0 of every wave of the first kStampBlocks workgroups
// stores s_memtime at five points of its first kStampWins windows, after the
// K x G partials (winn_stamp_elems; scripts/winn_timeline.py reads them).
// ---------------------------------------------------------------------------
// s_waitcnt vmcnt(0) expcnt(7) lgkmcnt(15) (gfx9 encoding: vmcnt in [3:0] and [15:14])
constexpr int kWaitVmcnt0 = 0x0F70;

template <int KH, int VEC, int NSMAX, int PF = 0, int LE = 0, int MODE = 0>
__global__ __launch_bounds__(64 * NSMAX, win_min_waves(KH, VEC)) void reduce_sqdist_winn_kernel(
    const float* __restrict__ X, int K, int64_t ld, int64_t P, int64_t nwin, const float* __restrict__ W,
    float* __restrict__ out, double* __restrict__ partials) {
  typedef typename WinVec<VEC>::T V;
  constexpr int WC = 64 * VEC;
  constexpr int NB = (KH + 7) / 8;
  constexpr int KP = (KH + 3) & ~3;
  const int lane = threadIdx.x & 63;
  const int h = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ns = __builtin_amdgcn_readfirstlane(static_cast<int>(blockDim.x >> 6));
  const int r0 = h * KH;
  const int64_t G = gridDim.x;
  const uint32_t voff = static_cast<uint32_t>(lane) * VEC * 4;
  const int64_t P4 = (P + 3) & ~static_cast<int64_t>(3);
  const int64_t row_bytes = ld * 4;
  const bool upper = (lane & 8) != 0;
  const auto win_bytes = [&](int64_t w) -> int {
    if (w >= nwin) return 0;
    const int64_t n = P4 - w * WC;
    return static_cast<int>((n < WC ? n : WC) * 4);
  };
  __shared__ __attribute__((aligned(16))) float wl[NSMAX][KP];
  __shared__ double accl[NSMAX][NB][64];
  __shared__ __attribute__((aligned(16))) V xa[64];
  static_assert(LE == 0 || VEC == 1, "LDS rows: 256-B row segments");
  static_assert(PF + LE <= KH, "prefetched rows");
  __shared__ __attribute__((aligned(16))) float rowl[LE > 0 ? NSMAX : 1][LE > 0 ? LE : 1][64];
  uint64_t* const stamps = reinterpret_cast<uint64_t*>(partials + static_cast<int64_t>(K) * G);
  int wi = 0;  // window count (timeline probe)
  const auto stamp = [&](int ph) __attribute__((always_inline)) {
    if constexpr ((MODE & 8) != 0) {
      if (blockIdx.x < kStampBlocks && wi < kStampWins) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        if (lane == 0) stamps[1 + ((int64_t(blockIdx.x) * NSMAX + h) * kStampWins + wi) * kStampSlots + ph] = t;
      }
    }
  };
  if constexpr ((MODE & 8) != 0) {
    if (blockIdx.x == 0 && threadIdx.x == 0) stamps[0] = kStampMagic;
  }
  for (int i = threadIdx.x; i < ns * KP; i += blockDim.x) {
    const int hh = i / KP, j = i % KP, row = hh * KH + j;
    wl[hh][j] = (j < KH && row < K) ? W[row] : -0.0f;
  }
  double* acc = &accl[h][0][lane];
#pragma unroll
  for (int b = 0; b < NB; ++b) acc[64 * b] = 0.0;
  __syncthreads();
  constexpr bool kBcastW = (MODE & 16) != 0;
  constexpr int NWV = kBcastW ? (KP + 15) / 16 : 1;
  float wv[NWV];
  if constexpr (kBcastW) {
#pragma unroll
    for (int k = 0; k < NWV; ++k) {
      const int j = 16 * k + (lane & 15);
      wv[k] = j < KP ? wl[h][j < KP ? j : 0] : 0.f;
    }
  }
  V x[KH];
  V xp[PF > 0 ? PF : 1];
  {
    int Kw = K;
    asm volatile("" : "+s"(Kw));
    const int nb = win_bytes(blockIdx.x);
    const char* rp = reinterpret_cast<const char*>(X + static_cast<int64_t>(blockIdx.x) * WC) + r0 * row_bytes;
#pragma unroll
    for (int i = 0; i < KH; ++i) {
      asm volatile("" : "+s"(rp));
      x[i] = win_load<VEC>(
          __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(rp), 0, r0 + i < Kw ? nb : 0, 0x00020000), voff);
      rp += row_bytes;
    }
  }
  const auto chain = [&](V& a, bool first) {
    if constexpr (kBcastW) {
      static_assert(VEC == 1 && KH % 16 == 0, "broadcast weights: one column per lane, 16-row groups");
      // the first turn starts from -0.0: fl32(-0.0 + p) is p, bit for bit
      float ac = first ? -0.0f : a[0];
      float tc = mul_row_bcast<0>(wv[0], x[0][0]);
      float xs[KH];
#pragma unroll
      for (int i = 0; i < KH; ++i) xs[i] = x[i][0];
      static_for<KH / 8>([&](auto bc) {
        constexpr int b = decltype(bc)::value;
        constexpr bool last = b == KH / 8 - 1;
        chain8_row_bcast<b % 2, last>(ac, tc, wv[b / 2], wv[last ? b / 2 : (b + 1) / 2], xs + 8 * b);
      });
      a[0] = ac;
      return;
    }
    int wo = h * KP;  // opaque: the weights are re-read per window, not held in registers
    asm volatile("" : "+v"(wo));
    const float* wp = &wl[0][0] + wo;
#pragma unroll
    for (int q = 0; q < KP / 4; ++q) {
      const f32x4 w4 = *reinterpret_cast<const f32x4*>(wp + 4 * q);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = 4 * q + j;
        if (i >= KH) continue;
        if (first && i == 0) {
          a = x[0] * w4[0];
        } else {
          const V t = x[i] * w4[j];
          a = a + t;
        }
      }
    }
  };
  for (int64_t w = blockIdx.x; w < nwin; w += G) {
    int Kw = K;
    asm volatile("" : "+s"(Kw));
    const int64_t c0 = w * WC;
    const int64_t cl = c0 + lane * VEC;
    const int nbn = win_bytes(w + G);
    const char* rp = reinterpret_cast<const char*>(X + (w + G) * WC) + r0 * row_bytes;
    stamp(0);
    if constexpr (PF > 0) {
      // this window's rows (reloaded in the last window's squares) first: a
      // pre-existing wait the compiler's waitcnt pass accounts for, so the
      // chain's uses of x[] need no wait on the prefetches issued below (it
      // otherwise entered the turn loop with vmcnt(0): every wave waited for
      // its prefetched rows of the NEXT window before its turn)
      __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
      stamp(1);
#pragma unroll
      for (int i = 0; i < PF; ++i) {
        asm volatile("" : "+s"(rp));
        xp[i] = win_load<VEC>(
            __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(rp), 0, r0 + i < Kw ? nbn : 0, 0x00020000), voff);
        rp += row_bytes;
      }
    }
    if constexpr (LE > 0) {
      // the last window's LDS rows have been read out (their ds_reads done)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      typedef __attribute__((address_space(3))) void* lds_ptr_t;
#pragma unroll
      for (int i = 0; i < LE; ++i) {
        asm volatile("" : "+s"(rp));
        const __amdgpu_buffer_rsrc_t r =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(rp), 0, r0 + PF + i < Kw ? nbn : 0, 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)&rowl[h][i][0], 4, lane * 4, 0, 0, 2);
        rp += row_bytes;
      }
    }
    const bool ragged = c0 + WC > P;
    if (ragged) {
#pragma unroll
      for (int i = 0; i < KH; ++i) {
#pragma unroll
        for (int v = 0; v < VEC; ++v)
          if (cl + v >= P) x[i][v] = 0.f;
      }
    }
    V a;
    if constexpr ((MODE & 1) != 0) {  // probe: no chain
      a = x[0];
    } else
    for (int st = 0; st < ns; ++st) {  // the chain, wave by wave in row order
      if (h == st) {
        stamp(2);
        if (st > 0) a = xa[lane];
        chain(a, st == 0);
        xa[lane] = a;
        stamp(3);
        if (st == ns - 1) {
          if (!ragged) {
            __builtin_nontemporal_store(static_cast<typename WinVec<VEC>::TA>(a),
                                        reinterpret_cast<typename WinVec<VEC>::TA*>(out + cl));
          } else {
#pragma unroll
            for (int v = 0; v < VEC; ++v)
              if (cl + v < P) out[cl + v] = a[v];
          }
        }
      }
      __syncthreads();
    }
    if constexpr ((MODE & 1) == 0) {
      if (h != ns - 1) a = xa[lane];
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      double p[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = 8 * b + j;
        p[j] = 0.0;
        if (i < KH) {
          if constexpr ((MODE & 2) == 0) p[j] = win_sq<VEC>(x[i] - a);
          if (i < PF) {
            x[i] = xp[i < PF ? i : 0];
          } else if (i < PF + LE) {
            x[i][0] = rowl[h][i - PF < LE ? i - PF : 0][lane];
          } else {
            asm volatile("" : "+s"(rp));
            x[i] = win_load<VEC>(
                __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(rp), 0, r0 + i < Kw ? nbn : 0, 0x00020000), voff);
            rp += row_bytes;
          }
        }
      }
      const double q01 = fold32(p[0], p[1]), q23 = fold32(p[2], p[3]);
      const double q45 = fold32(p[4], p[5]), q67 = fold32(p[6], p[7]);
      acc[64 * b] += fold8(fold16(q01, q23), fold16(q45, q67), upper);
    }
    stamp(4);
    __syncthreads();  // xa is read by every wave before the next window's chain rewrites it
    stamp(5);
    ++wi;
  }
  const int row_in = win_batch_row(lane);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    double s = acc[64 * b];
    s += dpp_move_f64<0xB1, 0xF>(s);
    s += dpp_move_f64<0x4E, 0xF>(s);
    s += dpp_move_f64<0x141, 0xF>(s);
    const int row = 8 * b + row_in;
    if ((lane & 7) == 0 && row < KH && r0 + row < K) partials[static_cast<int64_t>(r0 + row) * G + blockIdx.x] = s;
  }
}

// workgroups of the split window launch: the resident ones (ceil(K / KH)
// waves each) rounded down to a power of two per CU -- 3 workgroups of 5
// waves on a CU ran 12-15 % slower than 2 (profiles/r05/prefetch/) --, at
// most one per window
template <int KH, int VEC, int NSMAX, int PF = 0, int LE = 0, int MODE = 0>
int64_t fused_winn_grid(int64_t K, int64_t P, int blocks_per_cu) {
  const int ns = static_cast<int>((K + KH - 1) / KH);
  int64_t per_cu = blocks_per_cu;
  if (per_cu <= 0) {
    const int64_t r = resident_blocks(reduce_sqdist_winn_kernel<KH, VEC, NSMAX, PF, LE, MODE>, 64 * ns) / cu_count();
    per_cu = 0;  // none resident: the caller reports it (grid 0)
    if (r >= 1)
      for (per_cu = 1; per_cu * 2 <= r;) per_cu *= 2;
  }
  const int64_t nwin = (P + 64 * VEC - 1) / (64 * VEC);
  const int64_t grid = per_cu * cu_count();
  return grid < nwin ? grid : nwin;
}

template <int KH, int VEC, int NSMAX, int PF = 0, int LE = 0, int MODE = 0>
int launch_fused_winn(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights, float* out,
                      double* partials, int64_t partial_elems, double* sumsq, int blocks_per_cu, hipStream_t s,
                      const char* what) {
  if (K > NSMAX * KH) return set_error(FEDAVG_EMODE, "%s: this split window kernel covers K <= %d", what, NSMAX * KH);
  const int ns = static_cast<int>((K + KH - 1) / KH);
  const int64_t nwin = (P + 64 * VEC - 1) / (64 * VEC);
  const int64_t grid = fused_winn_grid<KH, VEC, NSMAX, PF, LE, MODE>(K, P, blocks_per_cu);
  if (grid <= 0) return set_error(FEDAVG_EMODE, "%s: the split window kernel is not resident", what);
  const int64_t need = K * grid + ((MODE & 8) != 0 ? winn_stamp_elems(NSMAX) : 0);
  if (partial_elems < need)
    return set_error(FEDAVG_EINVAL, "%s: workspace needs %lld doubles", what, (long long)need);
  hipLaunchKernelGGL((reduce_sqdist_winn_kernel<KH, VEC, NSMAX, PF, LE, MODE>), dim3(static_cast<unsigned>(grid)),
                     dim3(static_cast<unsigned>(64 * ns)), 0, s, clients, static_cast<int>(K), ld, P, nwin, weights,
                     out, partials);
  int rc = launch_status(what);
  if (rc) return rc;
  hipLaunchKernelGGL(client_sqdist_finalize_kernel, dim3(static_cast<unsigned>(K)), dim3(kBlock), 0, s, partials,
                     grid, sumsq);
  return launch_status(what);
}


// ---------------------------------------------------------------------------
// Split-row windows with point-to-point hand-offs (round 6).  The same work as
// reduce_sqdist_winn_kernel<64, 1, NSMAX, PF> -- wave h holds rows 64h ..
// 64h + 63 of a 64-column window, the chain runs wave by wave in row order,
// then every wave squares its rows against the average and reloads them from
// the next window -- without a workgroup barrier anywhere in the window loop:
//   * wave h > 0 starts its turn when wave h - 1's partial for this window is
//     in LDS (part[h - 1], flag[h - 1] = the window's sequence number), wave
//     ns - 1 publishes the average (avg, flag[NSMAX]); every other wave waits
//     for it before its squares;
//   * a wave's own rows are waited for at its turn (the compiler's vmcnt(PF):
//     the prefetched rows of the next window stay in flight), not at the
//     window's start;
//   * the squares and reloads run at a priority by wave (waves 0-3 first), so
//     the first waves' rows of the next window arrive first and their turns
//     start while the later waves' rows are still streaming.
// The timeline probe (winn, MODE 8) measured the barrier form's window as
// chain (14.4k cycles with the broadcast weights) + reload phase (9-12k)
// end to end: every turn waited at a barrier for the slowest wave's reloads.
// Hand-off safety: wave h writes part[h] for window s + 1 only after its
// squares of window s, i.e. after the average of s, i.e. after wave h + 1
// read part[h] for s; wave ns - 1 writes avg for s + 1 only after every other
// wave's turn of s + 1, each after its squares of s read avg.  Every wave runs
// the same windows, so every flag a wave waits for is set; the polls are
// bounded (kHandoffSpinMax) so a broken protocol ends in wrong sums (the parity
// tests), never in a hung grid.  Weights by row broadcast (chain8_row_bcast).
// MODE 8: the timeline stamps of the winn kernel.  Probes: MODE 1 polls
// with s_sleep 1 (the first form), 2 keeps every priority at 0, 4 keeps the
// turn at the squares' priority, 16 runs every wave's squares at priority 2, 32 by
// halves (waves 0-7 at 2, the rest at 1).
// ---------------------------------------------------------------------------
constexpr int kHandoffSpinMax = 1 << 16;  // x 16 polls of ~100 clocks (or x s_sleep 1): < 50 ms, a window is ~13 us

template <int NSMAX, int PF, int MODE = 0>
__global__ __launch_bounds__(64 * NSMAX, win_min_waves(64, 1)) void reduce_sqdist_winf_kernel(
    const float* __restrict__ X, int K, int64_t ld, int64_t P, int64_t nwin, const float* __restrict__ W,
    float* __restrict__ out, double* __restrict__ partials) {
  constexpr int KH = 64, WC = 64, NB = 8, NWV = 4;
  static_assert(PF >= 1 && PF <= KH, "prefetched rows");
  const int lane = threadIdx.x & 63;
  const int h = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ns = __builtin_amdgcn_readfirstlane(static_cast<int>(blockDim.x >> 6));
  const int r0 = h * KH;
  const int64_t G = gridDim.x;
  const uint32_t voff = static_cast<uint32_t>(lane) * 4;
  const int64_t P4 = (P + 3) & ~static_cast<int64_t>(3);
  const int64_t row_bytes = ld * 4;
  const bool upper = (lane & 8) != 0;
  const auto win_bytes = [&](int64_t w) -> int {
    if (w >= nwin) return 0;
    const int64_t n = P4 - w * WC;
    return static_cast<int>((n < WC ? n : WC) * 4);
  };
  __shared__ double accl[NSMAX][NB][64];
  __shared__ float part[NSMAX][64];
  __shared__ float avg[64];
  __shared__ int flag[NSMAX + 1];
  uint64_t* const stamps = reinterpret_cast<uint64_t*>(partials + static_cast<int64_t>(K) * G);
  int wi = 0;
  const auto stamp = [&](int ph) __attribute__((always_inline)) {
    if constexpr ((MODE & 8) != 0) {
      if (blockIdx.x < kStampBlocks && wi < kStampWins) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        if (lane == 0) stamps[1 + ((int64_t(blockIdx.x) * NSMAX + h) * kStampWins + wi) * kStampSlots + ph] = t;
      }
    }
  };
  if constexpr ((MODE & 8) != 0) {
    if (blockIdx.x == 0 && threadIdx.x == 0) stamps[0] = kStampMagic;
  }
  double* acc = &accl[h][0][lane];
#pragma unroll
  for (int b = 0; b < NB; ++b) acc[64 * b] = 0.0;
  if (threadIdx.x <= NSMAX) flag[threadIdx.x] = -1;
  float wv[NWV];  // lane 16r + j of wv[k]: row 16k + j's weight (-0.0 past K)
#pragma unroll
  for (int k = 0; k < NWV; ++k) {
    const int row = r0 + 16 * k + (lane & 15);
    wv[k] = row < K ? W[row] : -0.0f;
  }
  __syncthreads();
  // LDS pointers spelled out: a volatile access through a generic pointer is a
  // flat_load, whose wait is vmcnt(0) -- every row load of the wave
  typedef __attribute__((address_space(3))) volatile int lds_flag_t;
  const auto wait_flag = [&](int idx, int seq) __attribute__((always_inline)) {
    lds_flag_t* f = (lds_flag_t*)&flag[idx];
    // tight polls (no s_sleep): 600 x 10M 4.20 -> 4.09 ms, 1000 x 12.5M 7.97 -> 7.93
    // (profiles/r06/winf_modes/); MODE 1 is the s_sleep 1 form
    for (int it = 0; __builtin_amdgcn_readfirstlane(*f) != seq && it < kHandoffSpinMax * ((MODE & 1) ? 1 : 16); ++it)
      if constexpr ((MODE & 1) != 0) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
  };
  const auto publish = [&](int idx, int seq) __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the payload's ds_write is done
    *(lds_flag_t*)&flag[idx] = seq;
  };
  constexpr bool kPrio = (MODE & 2) == 0, kTurnPrio = kPrio && (MODE & 4) == 0;
  float x[KH];
  float xp[PF];
  {
    int Kw = K;
    asm volatile("" : "+s"(Kw));
    const int nb = win_bytes(blockIdx.x);
    const char* rp = reinterpret_cast<const char*>(X + static_cast<int64_t>(blockIdx.x) * WC) + r0 * row_bytes;
#pragma unroll
    for (int i = 0; i < KH; ++i) {
      asm volatile("" : "+s"(rp));
      x[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                           __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(rp), 0,
                                                                             r0 + i < Kw ? nb : 0, 0x00020000),
                                           static_cast<int>(voff), 0, 2));
      rp += row_bytes;
    }
  }
  int seq = 0;
  for (int64_t w = blockIdx.x; w < nwin; w += G, ++seq) {
    int Kw = K;
    asm volatile("" : "+s"(Kw));
    const int64_t c0 = w * WC;
    const int64_t cl = c0 + lane;
    const int nbn = win_bytes(w + G);
    const char* rp = reinterpret_cast<const char*>(X + (w + G) * WC) + r0 * row_bytes;
    stamp(0);
#pragma unroll
    for (int i = 0; i < PF; ++i) {  // the next window's first rows, in flight through the turn
      asm volatile("" : "+s"(rp));
      xp[i] = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(
                     __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(rp), 0, r0 + i < Kw ? nbn : 0, 0x00020000),
                     static_cast<int>(voff), 0, 2));
      rp += row_bytes;
    }
    const bool ragged = c0 + WC > P;
    if (ragged) {
#pragma unroll
      for (int i = 0; i < KH; ++i)
        if (cl >= P) x[i] = 0.f;
    }
    // the turn
    float a = -0.0f;  // fl32(-0.0 + p) is p, bit for bit: wave 0 starts the chain from it
    if (h > 0) {
      wait_flag(h - 1, seq);
      a = part[h - 1][lane];
    }
    stamp(2);
    if constexpr (kTurnPrio) __builtin_amdgcn_s_setprio(3);
    {
      float tc = mul_row_bcast<0>(wv[0], x[0]);
      static_for<KH / 8>([&](auto bc) {
        constexpr int b = decltype(bc)::value;
        constexpr bool last = b == KH / 8 - 1;
        chain8_row_bcast<b % 2, last>(a, tc, wv[b / 2], wv[last ? b / 2 : (b + 1) / 2], x + 8 * b);
      });
    }
    if (h < ns - 1) {
      part[h][lane] = a;
      publish(h, seq);
    } else {
      avg[lane] = a;
      publish(NSMAX, seq);
      if (!ragged) {
        __builtin_nontemporal_store(a, out + cl);
      } else if (cl < P) {
        out[cl] = a;
      }
    }
    stamp(3);
    if (h < ns - 1) {
      if constexpr (kTurnPrio) __builtin_amdgcn_s_setprio(0);
      wait_flag(NSMAX, seq);
      a = avg[lane];
    }
    // the squares, the next window's rows reloaded behind them: waves 0-3 first
    if constexpr ((MODE & 16) != 0) {  // probe: every wave's squares at priority 2
      __builtin_amdgcn_s_setprio(2);
    } else if constexpr ((MODE & 32) != 0) {  // probe: halves (waves 0-7 first)
      if (h < 8)
        __builtin_amdgcn_s_setprio(2);
      else
        __builtin_amdgcn_s_setprio(1);
    } else if constexpr (kPrio) {
      if (h < 4)
        __builtin_amdgcn_s_setprio(2);
      else if (h < 8)
        __builtin_amdgcn_s_setprio(1);
      else
        __builtin_amdgcn_s_setprio(0);
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      double p[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = 8 * b + j;
        const double d = static_cast<double>(x[i] - a);  // fp32 difference, as the reference forms it
        p[j] = d * d;
        if (i < PF) {
          x[i] = xp[i < PF ? i : 0];
        } else {
          asm volatile("" : "+s"(rp));
          x[i] = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(
                         __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(rp), 0, r0 + i < Kw ? nbn : 0, 0x00020000),
                         static_cast<int>(voff), 0, 2));
          rp += row_bytes;
        }
      }
      const double q01 = fold32(p[0], p[1]), q23 = fold32(p[2], p[3]);
      const double q45 = fold32(p[4], p[5]), q67 = fold32(p[6], p[7]);
      acc[64 * b] += fold8(fold16(q01, q23), fold16(q45, q67), upper);
    }
    __builtin_amdgcn_s_setprio(0);
    stamp(4);
    ++wi;
  }
  const int row_in = win_batch_row(lane);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    double sm = acc[64 * b];
    sm += dpp_move_f64<0xB1, 0xF>(sm);
    sm += dpp_move_f64<0x4E, 0xF>(sm);
    sm += dpp_move_f64<0x141, 0xF>(sm);
    const int row = 8 * b + row_in;
    if ((lane & 7) == 0 && r0 + row < K) partials[static_cast<int64_t>(r0 + row) * G + blockIdx.x] = sm;
  }
}

template <int NSMAX, int PF, int MODE = 0>
int64_t fused_winf_grid(int64_t K, int64_t P) {
  const int ns = static_cast<int>((K + 63) / 64);
  const int64_t r = resident_blocks(reduce_sqdist_winf_kernel<NSMAX, PF, MODE>, 64 * ns) / cu_count();
  int64_t per_cu = 0;
  if (r >= 1)
    for (per_cu = 1; per_cu * 2 <= r;) per_cu *= 2;
  const int64_t nwin = (P + 63) / 64;
  const int64_t grid = per_cu * cu_count();
  return grid < nwin ? grid : nwin;
}

template <int NSMAX, int PF, int MODE = 0>
int launch_fused_winf(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights, float* out,
                      double* partials, int64_t partial_elems, double* sumsq, hipStream_t s, const char* what) {
  if (K > NSMAX * 64 || K < 2)
    return set_error(FEDAVG_EMODE, "%s: these split windows cover 2 <= K <= %d", what, NSMAX * 64);
  const int ns = static_cast<int>((K + 63) / 64);
  const int64_t nwin = (P + 63) / 64;
  const int64_t grid = fused_winf_grid<NSMAX, PF, MODE>(K, P);
  if (grid <= 0) return set_error(FEDAVG_EMODE, "%s: the split window kernel is not resident", what);
  const int64_t need = K * grid + ((MODE & 8) != 0 ? winn_stamp_elems(NSMAX) : 0);
  if (partial_elems < need)
    return set_error(FEDAVG_EINVAL, "%s: workspace needs %lld doubles", what, (long long)need);
  hipLaunchKernelGGL((reduce_sqdist_winf_kernel<NSMAX, PF, MODE>), dim3(static_cast<unsigned>(grid)),
                     dim3(static_cast<unsigned>(64 * ns)), 0, s, clients, static_cast<int>(K), ld, P, nwin, weights,
                     out, partials);
  int rc = launch_status(what);
  if (rc) return rc;
  hipLaunchKernelGGL(client_sqdist_finalize_kernel, dim3(static_cast<unsigned>(K)), dim3(kBlock), 0, s, partials,
                     grid, sumsq);
  return launch_status(what);
}

#ifdef FEDAVG_TUNING
// ---------------------------------------------------------------------------
// Probe (round 3): split-row windows.  With K = 100 rows in one wave the
// window kernel above keeps more loads than the hardware's 63-load vmcnt cap
// can hold, so each window's reloads go out in two generations and the wave
// sits with nothing in flight between its last row's arrival and the first
// reload.  Here a workgroup of TWO waves owns a window: wave h holds rows
// h*KH .. h*KH + KH - 1 (KH <= 63: every reload of a window is in flight at
// once; KH x VEC registers, so three waves per SIMD at KH 50, VEC 2).  The
// chain stays the reference's sequential order: wave 0 runs rows 0..KH-1,
// hands its fp32 partial over LDS, wave 1 continues with rows KH..2KH-1 and
// returns the final average (two barriers per window).  Each wave squares and
// reloads its own rows; row sums as in reduce_sqdist_win_kernel, one partial
// per (row, workgroup).
// ---------------------------------------------------------------------------
template <int KH, int VEC>
__global__ __launch_bounds__(128, win_min_waves(KH, VEC)) void reduce_sqdist_win2_kernel(
    const float* __restrict__ X, int K, int64_t ld, int64_t P, int64_t nwin, const float* __restrict__ W,
    float* __restrict__ out, double* __restrict__ partials) {
  typedef typename WinVec<VEC>::T V;
  constexpr int WC = 64 * VEC;
  constexpr int NB = (KH + 7) / 8;
  constexpr int KP = (KH + 3) & ~3;
  const int lane = threadIdx.x & 63;
  const int h = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r0 = h * KH;
  const int64_t G = gridDim.x;
  const uint32_t voff = static_cast<uint32_t>(lane) * VEC * 4;
  const int64_t P4 = (P + 3) & ~static_cast<int64_t>(3);
  const int64_t row_bytes = ld * 4;
  const bool upper = (lane & 8) != 0;
  const auto win_bytes = [&](int64_t w) -> int {
    if (w >= nwin) return 0;
    const int64_t n = P4 - w * WC;
    return static_cast<int>((n < WC ? n : WC) * 4);
  };
  __shared__ __attribute__((aligned(16))) float wl[2][KP];
  __shared__ double accl[2][NB][64];
  __shared__ __attribute__((aligned(16))) V xa[64];
  for (int i = threadIdx.x; i < 2 * KP; i += 128) {
    const int hh = i / KP, j = i % KP, row = hh * KH + j;
    wl[hh][j] = (j < KH && row < K) ? W[row] : -0.0f;
  }
  double* acc = &accl[h][0][lane];
#pragma unroll
  for (int b = 0; b < NB; ++b) acc[64 * b] = 0.0;
  __syncthreads();
  V x[KH];
  {
    int Kw = K;
    asm volatile("" : "+s"(Kw));
    const int nb = win_bytes(blockIdx.x);
    const char* rp = reinterpret_cast<const char*>(X + static_cast<int64_t>(blockIdx.x) * WC) + r0 * row_bytes;
#pragma unroll
    for (int i = 0; i < KH; ++i) {
      asm volatile("" : "+s"(rp));
      x[i] = win_load<VEC>(
          __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(rp), 0, r0 + i < Kw ? nb : 0, 0x00020000), voff);
      rp += row_bytes;
    }
  }
  // a = a + fl32(x_i w_i) over this wave's rows (first: a = fl32(x_0 w_0) first)
  const auto chain = [&](V& a, bool first) {
    int wo = h * KP;  // opaque: the weights are re-read per window, not held in registers
    asm volatile("" : "+v"(wo));
    const float* wp = &wl[0][0] + wo;
#pragma unroll
    for (int q = 0; q < KP / 4; ++q) {
      const f32x4 w4 = *reinterpret_cast<const f32x4*>(wp + 4 * q);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = 4 * q + j;
        if (i >= KH) continue;
        if (first && i == 0) {
          a = x[0] * w4[0];
        } else {
          const V t = x[i] * w4[j];
          a = a + t;
        }
      }
    }
  };
  for (int64_t w = blockIdx.x; w < nwin; w += G) {
    int Kw = K;
    asm volatile("" : "+s"(Kw));
    const int64_t c0 = w * WC;
    const int64_t cl = c0 + lane * VEC;
    const int nbn = win_bytes(w + G);
    const char* rp = reinterpret_cast<const char*>(X + (w + G) * WC) + r0 * row_bytes;
    const bool ragged = c0 + WC > P;
    if (ragged) {
#pragma unroll
      for (int i = 0; i < KH; ++i) {
#pragma unroll
        for (int v = 0; v < VEC; ++v)
          if (cl + v >= P) x[i][v] = 0.f;
      }
    }
    V a;
    if (h == 0) {
      chain(a, true);
      xa[lane] = a;
    }
    __syncthreads();
    if (h == 1) {
      a = xa[lane];
      chain(a, false);
      xa[lane] = a;
      if (!ragged) {
        __builtin_nontemporal_store(static_cast<typename WinVec<VEC>::TA>(a), reinterpret_cast<typename WinVec<VEC>::TA*>(out + cl));
      } else {
#pragma unroll
        for (int v = 0; v < VEC; ++v)
          if (cl + v < P) out[cl + v] = a[v];
      }
    }
    __syncthreads();
    if (h == 0) a = xa[lane];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      double p[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = 8 * b + j;
        p[j] = 0.0;
        if (i < KH) {
          p[j] = win_sq<VEC>(x[i] - a);
          asm volatile("" : "+s"(rp));
          x[i] = win_load<VEC>(
              __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(rp), 0, r0 + i < Kw ? nbn : 0, 0x00020000), voff);
          rp += row_bytes;
        }
      }
      const double q01 = fold32(p[0], p[1]), q23 = fold32(p[2], p[3]);
      const double q45 = fold32(p[4], p[5]), q67 = fold32(p[6], p[7]);
      acc[64 * b] += fold8(fold16(q01, q23), fold16(q45, q67), upper);
    }
  }
  const int row_in = win_batch_row(lane);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    double s = acc[64 * b];
    s += dpp_move_f64<0xB1, 0xF>(s);
    s += dpp_move_f64<0x4E, 0xF>(s);
    s += dpp_move_f64<0x141, 0xF>(s);
    const int row = 8 * b + row_in;
    if ((lane & 7) == 0 && row < KH && r0 + row < K) partials[static_cast<int64_t>(r0 + row) * G + blockIdx.x] = s;
  }
}

template <int KH, int VEC>
int launch_fused_win2(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights, float* out,
                      double* partials, int64_t partial_elems, double* sumsq, int blocks_per_cu, hipStream_t s,
                      const char* what) {
  if (K > 2 * KH) return set_error(FEDAVG_EMODE, "%s: this split window kernel covers K <= %d", what, 2 * KH);
  const auto kern = reduce_sqdist_win2_kernel<KH, VEC>;
  const int64_t per_cu = blocks_per_cu > 0 ? blocks_per_cu : resident_blocks(kern, 128) / cu_count();
  const int64_t nwin = (P + 64 * VEC - 1) / (64 * VEC);
  int64_t grid = per_cu * cu_count();
  if (grid > nwin) grid = nwin;
  if (grid <= 0) return set_error(FEDAVG_EMODE, "%s: the split window kernel is not resident", what);
  if (partial_elems < K * grid)
    return set_error(FEDAVG_EINVAL, "%s: workspace needs %lld doubles", what, (long long)(K * grid));
  hipLaunchKernelGGL((reduce_sqdist_win2_kernel<KH, VEC>), dim3(static_cast<unsigned>(grid)), dim3(128), 0, s,
                     clients, static_cast<int>(K), ld, P, nwin, weights, out, partials);
  int rc = launch_status(what);
  if (rc) return rc;
  hipLaunchKernelGGL(client_sqdist_finalize_kernel, dim3(static_cast<unsigned>(K)), dim3(kBlock), 0, s, partials,
                     grid, sumsq);
  return launch_status(what);
}
#endif  // FEDAVG_TUNING

// Which one-read kernel serves K rows (production), from interleaved
// measurements of every candidate against the others and the two passes on
// ~4 GB of rows (scripts/fused_probe.py, profiles/r03/fused_rule/*.jsonl and
// profiles/r03/win/*.jsonl; ms):
//   long rows (>= 16 windows per wave), 17 <= K <= 128: the wave-owned
//   windows (reduce_sqdist_win_kernel), KMAX x VEC by K:
//     K <= 48   48 x 4 (1 KiB per wave per row; 24 x 41.7M 0.675 vs 0.697
//               LDS-DMA 128 and 0.687 at 32 x 4; 32 x 31.3M 0.715 vs 0.736;
//               48 x 20.8M 0.652 vs 0.687 LDS-DMA 256)
//     K <= 64   64 x 2 (64 x 10M 0.449 vs 0.464; 56 x 20M 0.841 vs 0.867)
//     K <= 80   80 x 2 (72 x 25M 1.311 vs 1.915 LDS-DMA 64; 80 x 25M 1.397
//               vs 2.124 -- the LDS-DMA tiles at 65-90 rows run far below
//               their K = 100 rate)
//     K <= 100  100 x 2 (100 x 25M 1.531-1.665 vs 1.601-1.797 by box; 90 x
//               25M 1.578 vs 2.440; 100 x 6.25M 0.431 vs 0.451)
//     K <= 128  128 x 1 (128 x 8M 0.693 vs 0.879; 112 x 8M 0.610 vs 0.640)
//   shorter rows (100 x 3.1M: window 0.230 vs 0.218; 65-96 rows from 400K
//   columns up stay on the windows, see kWinHoleMinP), other K:
//   K <= 16    register-staged, 256-column tiles (8 x 125M 0.896 vs 0.880
//              LDS-DMA; FEMNIST 10 x 1.2M 16.6 vs 22.2 us)
//   K <= 32    LDS-DMA, 128 columns (24 x 41.7M 0.733 vs 0.738 register-staged)
//   K <= 48    LDS-DMA, 256 columns (48 x 20.8M 0.737 vs 0.758 at 128)
//   K <= 64    LDS-DMA, 128 columns (64 x 10M 0.472 vs 0.486 register-staged)
//   K <= 128   LDS-DMA, 64 columns (100 x 25M 1.654 vs 1.753 register-staged)
//   K <= 192   register-staged, 64 columns, 16 slots (192 x 5.2M 0.778 vs
//              0.857 at 32 columns; the LDS-DMA kernel 0.829)
//   K <= 320   register-staged, 32 columns, 10 slots (224 x 4.5M 0.728 vs
//              1.03 at 64; 300 x 5M 1.08 vs 1.41 LDS-DMA vs 1.98 two passes)
//   K <= 368   register-staged, 32 columns, 16 slots (round 3: 500 x 11.2M
//              5.41 vs 6.88 ms for the two passes; 512 x 5M 2.58 vs 3.22)
//   K <= 1024  split-row windows (round 5, below: kFusedWinnMinK)
// Beyond 1024 rows the two passes (a workgroup holds at most 16 x 64 rows).
constexpr int kFusedNone = 0, kFusedLds = 1, kFusedRs = 2, kFusedWin = 3, kFusedWinn = 4;
constexpr int64_t kFusedRowsMaxK = 1024;
// split-row windows (reduce_sqdist_winn_kernel, 64 rows per wave, 64 columns)
// from 369 rows (round 5, scripts/fused_probe.py, profiles/r05/winn/, ms:
// 384 x 5M 1.455 vs 1.494 register-staged; 448 x 5M 1.60 vs 2.30; 500 x
// 11.2M 3.71 vs 5.37; 500 x 1.4M 0.54 vs 0.72; 512 x 5M 1.69 vs 2.59; but
// 352 x 5M 1.42 vs 1.36 and 300 x 5M 1.10 vs 1.05), up to 8 waves per
// workgroup to 512 rows, 16 beyond (640 x 3M 1.77 vs 2.46 for the two
// passes; 1000 x 12.5M 9.99 vs 15.05; 520 x 5M 2.71 vs 3.34)
constexpr int64_t kFusedWinnMinK = 369;
// (round 5: the barrier form with 8 prefetched rows, split_prefetch_rows)
// Round 6: the split windows run reduce_sqdist_winf_kernel (point-to-point
// hand-offs, broadcast weights) with 8 prefetched rows at <= 8 waves and 16
// beyond (profiles/r06/winf/, ms, barrier form vs winf: 1000 x 12.5M 9.06 vs
// 8.02; 999 x 10M+3 7.75 vs 6.44; 600 x 10M 5.13 vs 4.28; 513 x 3M 1.48 vs
// 1.26; 500 x 11.2M 3.66 vs 3.57; 400 x 10M 2.73 vs 2.60; 370 x 5M 1.25 vs
// 1.18; every output bit-identical).  FEDAVG_SPLIT_PREFETCH=0 keeps the
// barrier form without prefetch (A/B).
constexpr int kWinfPF8 = 8, kWinfPF16 = 16;
// With the prefetch the split windows also beat the register-staged tiles at
// 161-256 and 289-368 rows on long rows (profiles/r05/prefetch/, ms, tiles vs
// split: 170 x 5M 0.606 vs 0.593; 192 x 5M 0.725 vs 0.661; 240 x 5M 0.897 vs
// 0.822; 256 x 12M 2.53 vs 2.19; 290 x 5M 1.026 vs 0.998; 310 x 5M 1.092 vs
// 1.033; 352 x 5M 1.347 vs 1.178; 368 x 5M 1.427 vs 1.228), not at 140 x 5M
// (0.493 vs 0.529) or 270 x 5M (0.933 vs 0.981), and tie at 200 x 1.2M (18
// windows per workgroup): below 369 rows they take rounds of >= 24 windows
// per workgroup, and only with the prefetch on
// Round 6, the hand-off kernel (profiles/r06/winf_bands/, ms, plan then vs
// winf): 160 x 5M 0.615 vs 0.547; 260 x 5M 0.913 vs 0.851; 270 x 5M 0.939 vs
// 0.876; 288 x 5M 0.983 vs 0.923 (the old 257-288 gap); 200 x 1.2M (18
// windows per workgroup) 0.190 vs 0.182; 200 x 800K (12) 0.144 vs 0.126;
// 300-368 x 5M equal; below 160 the tiles keep it (150 x 5M 0.526 vs 0.536,
// 130 x 5M 0.459 vs 0.495)
constexpr int64_t kFusedWinnLowMinK = 160;
constexpr int64_t kFusedWinnLowMinPerBlock = 8;
constexpr int64_t kWinMinPerWave = 16;  // windows per wave below which the tile kernels keep the round
// ... except in the LDS-DMA tiles' weak band, 65-96 rows, where the windows
// win down to ~400K columns (profiles/r03/win/short_rows_*.jsonl, ms, tiles
// vs windows: 70 x 600K 0.052 vs 0.043; 70 x 3M 0.217 vs 0.143; 80 x 1.5M
// 0.129 vs 0.090; 90 x 600K 0.065 vs 0.051; 90 x 3M 0.285 vs 0.190; 92 x
// 1.5M 0.108 vs 0.102; 98 x 1.5M 0.109 vs 0.109; 100 x 600K 0.059 vs 0.059;
// 65 x 200K 0.022 vs 0.023)
constexpr int64_t kWinHoleMinK = 65, kWinHoleMaxK = 96, kWinHoleMinP = 400000;
struct FusedPlan {
  int kind, S, slots;  // kFusedWin: S = KMAX, slots = VEC
};

// The 81-100 band stages rows 0..23 of the next window in LDS (MODE 64):
// 100 x 25M 1.652 -> 1.646 ms, 100 x 25M+3 1.700 -> 1.690, 90 x 25M 1.607 ->
// 1.547 (profiles/r03/win/ldsrows.jsonl); every band has K > 24 rows
constexpr int kWin100Mode = 64;

// the window kernel instance for K rows ({kFusedNone} outside 17..128)
inline FusedPlan win_plan(int64_t K) {
  if (K <= 16 || K > 128) return {kFusedNone, 0, 0};
  if (K <= 48) return {kFusedWin, 48, 4};
  if (K <= 64) return {kFusedWin, 64, 2};
  if (K <= 80) return {kFusedWin, 80, 2};
  if (K <= 100) return {kFusedWin, 100, 2};
  return {kFusedWin, 128, 1};
}

// waves of the production window launch for plan `pl` (0: not a window plan)
inline int64_t win_waves(const FusedPlan& pl, int64_t P) {
  if (pl.kind != kFusedWin) return 0;
  switch (pl.S) {
    case 48: return fused_win_waves<48, 4, 4>(P, 0);
    case 64: return fused_win_waves<64, 2, 4>(P, 0);
    case 80: return fused_win_waves<80, 2, 4>(P, 0);
    case 100: return fused_win_waves<100, 2, 4, kWin100Mode>(P, 0);
    default: return fused_win_waves<128, 1, 4>(P, 0);
  }
}

inline FusedPlan fused_plan(int64_t K, int64_t P) {
  if (K < 1 || K > kFusedRowsMaxK) return {kFusedNone, 0, 0};
  const FusedPlan win = win_plan(K);
  if (win.kind == kFusedWin && ((P + 64 * win.slots - 1) / (64 * win.slots) >= kWinMinPerWave * win_waves(win, P) ||
                                 (K >= kWinHoleMinK && K <= kWinHoleMaxK && P >= kWinHoleMinP)))
    return win;
  if (K <= 16) return {kFusedRs, 256, 8};
  if (K <= 32) return {kFusedLds, 128, 0};
  if (K <= 48) return {kFusedLds, 256, 0};
  if (K <= 64) return {kFusedLds, 128, 0};
  if (K <= 128) return {kFusedLds, 64, 0};
  if (K >= kFusedWinnLowMinK && K < kFusedWinnMinK &&
      split_prefetch_rows() > 0) {
    const int64_t grid = fused_winf_grid<8, kWinfPF8>(K, P);
    if (grid > 0 && (P + 63) / 64 >= kFusedWinnLowMinPerBlock * grid) return {kFusedWinn, 64, 8};
  }
  if (K <= 192) return {kFusedRs, 64, 16};
  if (K <= 320) return {kFusedRs, 32, 10};
  if (K < kFusedWinnMinK) return {kFusedRs, 32, 16};
  return {kFusedWinn, 64, K <= 512 ? 8 : 16};  // S = rows per wave, slots = waves per workgroup (max)
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
//
// Between them, U4 x C8 when the 16-slice launch would end in a partly
// filled round of workgroups: a launch of g groups on r resident slots runs
// ceil(g / r) rounds, so 685 groups (cfg4, 500 x 11.2M) on 512 slots of the
// 16-slice kernel (2 per CU) fill 67 %, against 89 % for the 1,371 8-slice
// groups on its 768 slots (3 per CU).  scripts/dist_variants.py
// (profiles/r02/sweeps/dist_many_clients*.jsonl): 500 x 11.2M 4.10 -> 3.69 ms,
// 1000 x 12.5M 8.49 -> 8.03, 200 x 10M 1.52 -> 1.26; 100 x 25M keeps 16
// slices (1,526 groups, 99 %; 1.467 vs 1.600 ms at 8).
double round_fill(int64_t groups, int64_t slots) {
  if (slots <= 0) return 0.0;
  const int64_t rounds = (groups + slots - 1) / slots;
  return static_cast<double>(groups) / static_cast<double>(rounds * slots);
}

int dist_cols(int64_t P) {
  const int64_t nvec = (P + 3) / 4;
  const int64_t cus = cu_count();
  const int64_t g16 = (nvec + kBlock * 16 - 1) / (kBlock * 16);
  const int64_t g8 = (nvec + kBlock * 8 - 1) / (kBlock * 8);
  const int64_t slots16 = resident_blocks(client_sqdist_buf_kernel<2, 16, 1, 4>);
  const int64_t slots8 = resident_blocks(client_sqdist_buf_kernel<4, 8, 1, 4>);
  if (g16 >= 2 * cus) return round_fill(g8, slots8) > round_fill(g16, slots16) + 0.05 ? 8 : 16;
  if (g8 >= slots8) return 8;
  if ((nvec + kBlock * 4 - 1) / (kBlock * 4) >= cus * 9 / 10) return 4;
  return 2;
}

int64_t sqdist_waves_for(int64_t P, int cols) {
  const int64_t nvec = (P + 3) / 4;
  const int64_t blocks = (nvec + kBlock * cols - 1) / (kBlock * cols);
  return blocks * (kBlock / 64);
}

template <int U, int C, bool BUF = false, int MINW = 1, int ACC = 1, int STYLE = 0>
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
      hipLaunchKernelGGL((client_sqdist_buf_kernel<U, C, MINW, ACC, STYLE>), dim3(static_cast<unsigned>(nb)), dim3(kBlock), 0, s,
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
#ifdef FEDAVG_TUNING
    // interleaved loads and squares, L loads in flight: + 100000000 x L
    case 204000216: launch_sqdist<2, 16, true, 1, 4, 2>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 404000216: launch_sqdist<2, 16, true, 1, 4, 4>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 804000216: launch_sqdist<2, 16, true, 1, 4, 8>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 204000404: launch_sqdist<4, 4, true, 1, 4, 2>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 404000404: launch_sqdist<4, 4, true, 1, 4, 4>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 204000408: launch_sqdist<4, 8, true, 1, 4, 2>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
    case 404000408: launch_sqdist<4, 8, true, 1, 4, 4>(clients, k, ld, P, glob, workspace, nwaves, max_blocks, s); break;
#endif
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
  const int rows = cols == 16 ? kDistBufRows : (cols == 8 || cols == 4 ? 4 : 8);
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

// Aggregate + :291 sums in one pass for K <= kFusedRowsMaxK with 16-B
// aligned rows (fused_plan picks the kernel and tile); otherwise the two
// production passes back to back (fedavg_reduce_f32, then
// fedavg_client_sqdist_f32 on its output).  Either way `out` holds
// fedavg_reduce_f32's bits and sumsq the :291 sums.
int64_t fedavg_reduce_sqdist_workspace(int64_t K, int64_t P) {
  if (K <= 0 || P <= 0) return 0;
  const FusedPlan pl = fused_plan(K, P);
  const int64_t two_pass = fedavg_client_sqdist_workspace(K, P);
  int64_t fused = 0;
  if (pl.kind == kFusedWin) {
    fused = K * win_waves(pl, P);
  } else if (pl.kind == kFusedLds) {
    if (pl.S == 64) fused = K * fused_grid<64>(K, P, 0);
    if (pl.S == 128) fused = K * fused_grid<128>(K, P, 0);
    if (pl.S == 256) fused = K * fused_grid<256>(K, P, 0);
  } else if (pl.kind == kFusedWinn) {
    const bool pf = split_prefetch_rows() > 0;
    fused = K * (pl.slots == 8 ? (pf ? fused_winf_grid<8, kWinfPF8>(K, P) : fused_winn_grid<64, 1, 8>(K, P, 0))
                               : (pf ? fused_winf_grid<16, kWinfPF16>(K, P) : fused_winn_grid<64, 1, 16>(K, P, 0)));
  } else if (pl.kind == kFusedRs) {
    switch (pl.S * 100 + pl.slots) {
      case 25608: fused = K * fused_rs_grid<256, 8, 0>(K, P, 0); break;
      case 6416: fused = K * fused_rs_grid<64, 16, 0>(K, P, 0); break;
      case 3210: fused = K * fused_rs_grid<32, 10, 0>(K, P, 0); break;
      case 3216: fused = K * fused_rs_grid<32, 16, 0>(K, P, 0); break;
      default: break;
    }
  }
  return fused > two_pass ? fused : two_pass;
}

int fedavg_reduce_sqdist_f32(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights, float* out,
                             double* workspace, int64_t workspace_elems, double* sumsq, void* stream) {
  const char* what = "fedavg_reduce_sqdist_f32";
  int rc = check_common(clients, K, P, ld, weights, out, what);
  if (rc) return rc;
  if (!sumsq || !workspace) return set_error(FEDAVG_EINVAL, "%s: null workspace/sumsq", what);
  // both forms read the rows as 16-B slices (the two-pass fallback's distance
  // pass too): refuse unaligned rows up front rather than after the reduce
  if (!aligned16(clients) || (ld % 4) != 0)
    return set_error(FEDAVG_EALIGN, "%s: needs 16-B aligned rows and ld %% 4 == 0 (reduce alone: fedavg_reduce_f32)",
                     what);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (P == 0) {
    const hipError_t e = hipMemsetAsync(sumsq, 0, static_cast<size_t>(K) * sizeof(double), s);
    return e == hipSuccess ? FEDAVG_OK : set_error(-static_cast<int>(e), "%s: hipMemsetAsync failed", what);
  }
  const FusedPlan pl = fused_plan(K, P);
  if (pl.kind != kFusedNone && aligned4(out) && aligned4(weights)) {
    if (pl.kind == kFusedWin) {
      switch (pl.S) {
        case 48:
          return launch_fused_win<48, 4, 4>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq, 0, s,
                                            what);
        case 64:
          return launch_fused_win<64, 2, 4>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq, 0, s,
                                            what);
        case 80:
          return launch_fused_win<80, 2, 4>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq, 0, s,
                                            what);
        case 100:
          return launch_fused_win<100, 2, 4, kWin100Mode>(clients, K, P, ld, weights, out, workspace, workspace_elems,
                                                          sumsq, 0, s, what);
        default:
          return launch_fused_win<128, 1, 4>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq, 0, s,
                                             what);
      }
    }
    if (pl.kind == kFusedWinn) {
      const bool pf = split_prefetch_rows() > 0;
      if (pl.slots == 8 && pf)
        return launch_fused_winf<8, kWinfPF8>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq, s,
                                              what);
      if (pl.slots == 8)
        return launch_fused_winn<64, 1, 8>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq, 0, s,
                                           what);
      if (pf)
        return launch_fused_winf<16, kWinfPF16>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq, s,
                                                what);
      return launch_fused_winn<64, 1, 16>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq, 0, s,
                                          what);
    }
    if (pl.kind == kFusedLds) {
      if (pl.S == 64)
        return launch_fused<64>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq, 0, s, what);
      if (pl.S == 256)
        return launch_fused<256>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq, 0, s, what);
      return launch_fused<128>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq, 0, s, what);
    }
    switch (pl.S * 100 + pl.slots) {
      case 25608:
        return launch_fused_rs<256, 8>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq, 0, s, what);
      case 6416:
        return launch_fused_rs<64, 16>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq, 0, s, what);
      case 3210:
        return launch_fused_rs<32, 10>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq, 0, s, what);
      default:
        return launch_fused_rs<32, 16>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq, 0, s, what);
    }
  }
  rc = fedavg_reduce_f32(clients, K, P, ld, weights, out, stream);
  if (rc) return rc;
  return fedavg_client_sqdist_f32(clients, K, P, ld, out, workspace, workspace_elems, sumsq, stream);
}

// the production plan of fedavg_reduce_sqdist_f32 for K x P: kind x
// 1000000 + S x 100 + slots (kind 0 two passes, 1 LDS-DMA tiles, 2
// register-staged tiles, 3 wave-owned windows with S = KMAX, slots = VEC,
// 4 split-row windows with S = rows per wave, slots = most waves per group)
int64_t fedavg_fused_plan_of(int64_t K, int64_t P) {
  const FusedPlan pl = fused_plan(K, P);
  return static_cast<int64_t>(pl.kind) * 1000000 + pl.S * 100 + pl.slots;
}

#ifdef FEDAVG_TUNING  // probe library only (libfedavg_amd_probe.so)
// the fused pass with an explicit tile width (64 / 128 / 256 columns) and
// workgroups per CU (0 = as many as LDS allows); workspace >= K x grid
int fedavg_reduce_sqdist_f32_variant(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights,
                                     float* out, double* workspace, int64_t workspace_elems, double* sumsq, int cols,
                                     int blocks_per_cu, void* stream) {
  const char* what = "fedavg_reduce_sqdist_f32_variant";
  int rc = check_common(clients, K, P, ld, weights, out, what);
  if (rc) return rc;
  if (P == 0 || K > 1024 || !aligned16(clients) || (ld % 4) != 0 || !sumsq || !workspace)
    return set_error(FEDAVG_EINVAL, "%s: needs 1 <= K <= 1024, P >= 1, 16-B aligned rows", what);
  hipStream_t s = static_cast<hipStream_t>(stream);
  // cols + 1000: double-buffered tiles (the next tile's loads in flight while
  // one is used); + 10000: rows per wave with one register accumulator each
  switch (cols) {
#define FEDAVG_FUSED_CASE(C, DBUF, RWS)                                                                           \
  case C + (DBUF ? 1000 : 0) + (RWS ? 10000 : 0):                                                                \
    return launch_fused<C, DBUF, RWS>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq,         \
                                      blocks_per_cu, s, what);
    FEDAVG_FUSED_CASE(32, false, 0)
    FEDAVG_FUSED_CASE(64, false, 0)
    FEDAVG_FUSED_CASE(128, false, 0)
    FEDAVG_FUSED_CASE(256, false, 0)
    FEDAVG_FUSED_CASE(64, true, 0)
    FEDAVG_FUSED_CASE(128, true, 0)
    FEDAVG_FUSED_CASE(256, true, 0)
    FEDAVG_FUSED_CASE(64, false, 32)
    FEDAVG_FUSED_CASE(128, false, 32)
    FEDAVG_FUSED_CASE(256, false, 32)
    FEDAVG_FUSED_CASE(128, true, 32)
#undef FEDAVG_FUSED_CASE
    // + 100000: the tile loads alone (no average, no sums: a traffic probe, wrong results)
    case 100064: return launch_fused<64, false, 0, true>(clients, K, P, ld, weights, out, workspace, workspace_elems,
                                                         sumsq, blocks_per_cu, s, what);
    case 100128: return launch_fused<128, false, 0, true>(clients, K, P, ld, weights, out, workspace, workspace_elems,
                                                          sumsq, blocks_per_cu, s, what);
    case 101064: return launch_fused<64, true, 0, true>(clients, K, P, ld, weights, out, workspace, workspace_elems,
                                                        sumsq, blocks_per_cu, s, what);
    // register-staged tiles (reduce_sqdist_rs_kernel): 200000 + S; 210000 + S
    // with the slots of K = 100 at 128 / 256 columns; + 100000: loads only,
    // + 200000: loads + LDS writes (traffic probes, wrong results)
#define FEDAVG_RS_CASE(CODE, C, SL, MODE)                                                                         \
  case CODE:                                                                                                     \
    return launch_fused_rs<C, SL, MODE>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq,      \
                                        blocks_per_cu, s, what);
    FEDAVG_RS_CASE(200032, 32, 10, 0)
    FEDAVG_RS_CASE(200064, 64, 8, 0)
    FEDAVG_RS_CASE(200128, 128, 8, 0)
    FEDAVG_RS_CASE(200256, 256, 8, 0)
    FEDAVG_RS_CASE(210128, 128, 13, 0)
    FEDAVG_RS_CASE(210256, 256, 25, 0)
    FEDAVG_RS_CASE(300064, 64, 8, 1)
    FEDAVG_RS_CASE(310128, 128, 13, 1)
    FEDAVG_RS_CASE(310256, 256, 25, 1)
    FEDAVG_RS_CASE(400064, 64, 8, 2)
    FEDAVG_RS_CASE(410128, 128, 13, 2)
    FEDAVG_RS_CASE(410256, 256, 25, 2)
#undef FEDAVG_RS_CASE
    // + 1000000: the same over a TILED buffer [ceil(P / S)][K][S] (probe: is the
    // row-major tile walk limited by the spread of its K row segments?)
    case 1200064: return launch_fused_rs<64, 8, 0, 1>(clients, K, P, ld, weights, out, workspace, workspace_elems,
                                                         sumsq, blocks_per_cu, s, what);
    case 1300064: return launch_fused_rs<64, 8, 1, 1>(clients, K, P, ld, weights, out, workspace, workspace_elems,
                                                         sumsq, blocks_per_cu, s, what);
    case 1310128: return launch_fused_rs<128, 13, 1, 1>(clients, K, P, ld, weights, out, workspace,
                                                         workspace_elems, sumsq, blocks_per_cu, s, what);
    // + 2000000 / 4000000: XCD-contiguous / XCD- and CU-contiguous tile sweeps
    case 2200064: return launch_fused_rs<64, 8, 0, 2>(clients, K, P, ld, weights, out, workspace, workspace_elems,
                                                      sumsq, blocks_per_cu, s, what);
    case 2300064: return launch_fused_rs<64, 8, 1, 2>(clients, K, P, ld, weights, out, workspace, workspace_elems,
                                                      sumsq, blocks_per_cu, s, what);
    case 4200064: return launch_fused_rs<64, 8, 0, 4>(clients, K, P, ld, weights, out, workspace, workspace_elems,
                                                      sumsq, blocks_per_cu, s, what);
    case 4300064: return launch_fused_rs<64, 8, 1, 4>(clients, K, P, ld, weights, out, workspace, workspace_elems,
                                                      sumsq, blocks_per_cu, s, what);
    case 4200032: return launch_fused_rs<32, 10, 0, 4>(clients, K, P, ld, weights, out, workspace, workspace_elems,
                                                       sumsq, blocks_per_cu, s, what);
    // + 10000000: two tiles in flight per workgroup; 5300064 / 5310128: loads
    // only, no LDS (occupancy from registers alone)
    case 10200064: return launch_fused_rs<64, 8, 0, 0, 2>(clients, K, P, ld, weights, out, workspace,
                                                          workspace_elems, sumsq, blocks_per_cu, s, what);
    case 10200032: return launch_fused_rs<32, 10, 0, 0, 2>(clients, K, P, ld, weights, out, workspace,
                                                           workspace_elems, sumsq, blocks_per_cu, s, what);
    case 10200128: return launch_fused_rs<128, 8, 0, 0, 2>(clients, K, P, ld, weights, out, workspace,
                                                           workspace_elems, sumsq, blocks_per_cu, s, what);
    case 10300064: return launch_fused_rs<64, 8, 1, 0, 2>(clients, K, P, ld, weights, out, workspace,
                                                          workspace_elems, sumsq, blocks_per_cu, s, what);
    // many clients: S = 32 with 16 / 32 slots per thread (K <= 512 / 1024), S = 64 with 16 (K <= 256)
    case 200032 + 1600000: return launch_fused_rs<32, 16>(clients, K, P, ld, weights, out, workspace,
                                                         workspace_elems, sumsq, blocks_per_cu, s, what);
    case 200032 + 3200000: return launch_fused_rs<32, 32>(clients, K, P, ld, weights, out, workspace,
                                                         workspace_elems, sumsq, blocks_per_cu, s, what);
    case 200064 + 1600000: return launch_fused_rs<64, 16>(clients, K, P, ld, weights, out, workspace,
                                                         workspace_elems, sumsq, blocks_per_cu, s, what);
    case 5300064: return launch_fused_rs<64, 8, 3>(clients, K, P, ld, weights, out, workspace, workspace_elems,
                                                   sumsq, blocks_per_cu, s, what);
    // wide tiles with 2-3 tiles in flight (registers) beside the one in LDS:
    // 20000000 + DEPTH * 1000000 + S (K = 100: 13 slots at 128, 25 at 256)
    case 22000128: return launch_fused_rs<128, 13, 0, 0, 2>(clients, K, P, ld, weights, out, workspace,
                                                            workspace_elems, sumsq, blocks_per_cu, s, what);
    case 23000128: return launch_fused_rs<128, 13, 0, 0, 3>(clients, K, P, ld, weights, out, workspace,
                                                            workspace_elems, sumsq, blocks_per_cu, s, what);
    case 22000256: return launch_fused_rs<256, 25, 0, 0, 2>(clients, K, P, ld, weights, out, workspace,
                                                            workspace_elems, sumsq, blocks_per_cu, s, what);
    case 23000256: return launch_fused_rs<256, 25, 0, 0, 3>(clients, K, P, ld, weights, out, workspace,
                                                            workspace_elems, sumsq, blocks_per_cu, s, what);
    case 5310128: return launch_fused_rs<128, 13, 3>(clients, K, P, ld, weights, out, workspace, workspace_elems,
                                                     sumsq, blocks_per_cu, s, what);
    case 5310256: return launch_fused_rs<256, 25, 3>(clients, K, P, ld, weights, out, workspace, workspace_elems,
                                                     sumsq, blocks_per_cu, s, what);
    case 15300064: return launch_fused_rs<64, 8, 3, 0, 2>(clients, K, P, ld, weights, out, workspace,
                                                          workspace_elems, sumsq, blocks_per_cu, s, what);
    // wave-owned windows (reduce_sqdist_win_kernel): 60000000 + MODE *
    // 1000000 + NW * 10 + VEC at K <= 100; 70000000 + KMAX * 100 + NW * 10 + VEC
#define FEDAVG_WIN_CASE(VEC, NW, MODE)                                                                            \
  case 60000000 + MODE * 1000000 + NW * 10 + VEC:                                                                \
    return launch_fused_win<100, VEC, NW, MODE>(clients, K, P, ld, weights, out, workspace, workspace_elems,     \
                                                sumsq, blocks_per_cu, s, what);
    FEDAVG_WIN_CASE(2, 4, 1)
    FEDAVG_WIN_CASE(4, 4, 1)
    FEDAVG_WIN_CASE(2, 4, 2)
    FEDAVG_WIN_CASE(2, 4, 8)
    FEDAVG_WIN_CASE(2, 4, 16)
    FEDAVG_WIN_CASE(2, 8, 16)
    FEDAVG_WIN_CASE(2, 8, 0)
    FEDAVG_WIN_CASE(2, 4, 64)
    FEDAVG_WIN_CASE(2, 1, 64)
    FEDAVG_WIN_CASE(2, 2, 64)
    FEDAVG_WIN_CASE(2, 4, 128)
    FEDAVG_WIN_CASE(2, 4, 65)  // LDS rows, loads only (round 6 clock attribution)
    FEDAVG_WIN_CASE(2, 4, 68)  // LDS rows, fp32 squares
    FEDAVG_WIN_CASE(2, 4, 256)  // broadcast weights (round 6)
    FEDAVG_WIN_CASE(2, 4, 320)  // LDS rows + broadcast weights (round 6)
    case 60000000 + 192 * 1000000 + 42:  // LDS rows + 8-row descriptors
      return launch_fused_win<100, 2, 4, 192>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq,
                                              blocks_per_cu, s, what);
#define FEDAVG_WINK_CASE(KMAX, VEC, MINW)                                                                         \
  case 70000000 + KMAX * 100 + 40 + VEC:                                                                         \
    return launch_fused_win<KMAX, VEC, 4, 0, MINW>(clients, K, P, ld, weights, out, workspace, workspace_elems,  \
                                                   sumsq, blocks_per_cu, s, what);
    FEDAVG_WINK_CASE(100, 2, 2)
    FEDAVG_WINK_CASE(80, 2, 2)
    FEDAVG_WINK_CASE(64, 2, 3)
    FEDAVG_WINK_CASE(32, 4, 3)
    FEDAVG_WINK_CASE(48, 4, 2)
    FEDAVG_WINK_CASE(16, 4, 4)
    FEDAVG_WINK_CASE(128, 1, 2)
#undef FEDAVG_WINK_CASE
#undef FEDAVG_WIN_CASE
    // split-row windows (reduce_sqdist_win2_kernel): 80000000 + KH * 100 + VEC, K <= 2 KH
#define FEDAVG_WIN2_CASE(KH, VEC)                                                                                 \
  case 80000000 + KH * 100 + VEC:                                                                                \
    return launch_fused_win2<KH, VEC>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq,        \
                                      blocks_per_cu, s, what);
    FEDAVG_WIN2_CASE(50, 2)
    FEDAVG_WIN2_CASE(40, 2)
    FEDAVG_WIN2_CASE(32, 2)
    FEDAVG_WIN2_CASE(25, 4)
    FEDAVG_WIN2_CASE(60, 2)
    FEDAVG_WIN2_CASE(50, 4)
#undef FEDAVG_WIN2_CASE
    // split-row windows over ceil(K / KH) <= NSMAX waves (reduce_sqdist_winn_kernel):
    // 85000000 + NSMAX * 10000 + KH * 10 + VEC
#define FEDAVG_WINN_CASE(KH, VEC, NSMAX)                                                                          \
  case 85000000 + NSMAX * 10000 + KH * 10 + VEC:                                                                 \
    return launch_fused_winn<KH, VEC, NSMAX>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq,  \
                                             blocks_per_cu, s, what);
    FEDAVG_WINN_CASE(64, 1, 8)
    FEDAVG_WINN_CASE(64, 2, 8)
    FEDAVG_WINN_CASE(32, 2, 16)
    FEDAVG_WINN_CASE(128, 1, 4)
    FEDAVG_WINN_CASE(64, 1, 16)
#undef FEDAVG_WINN_CASE
    // the same (64 rows per wave, one column per lane) with PF rows of the next
    // window prefetched: 87000000 + PF * 100 + NSMAX
#define FEDAVG_WINNPF_CASE(NSMAX, PF)                                                                             \
  case 87000000 + PF * 100 + NSMAX:                                                                              \
    return launch_fused_winn<64, 1, NSMAX, PF>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq, \
                                               blocks_per_cu, s, what);
    FEDAVG_WINNPF_CASE(8, 4)
    FEDAVG_WINNPF_CASE(8, 8)
    FEDAVG_WINNPF_CASE(8, 12)
    FEDAVG_WINNPF_CASE(8, 16)
    FEDAVG_WINNPF_CASE(16, 2)
    FEDAVG_WINNPF_CASE(16, 4)
    FEDAVG_WINNPF_CASE(16, 6)
    FEDAVG_WINNPF_CASE(16, 8)
    FEDAVG_WINNPF_CASE(16, 10)
    FEDAVG_WINNPF_CASE(16, 12)
    FEDAVG_WINNPF_CASE(16, 16)
    FEDAVG_WINNPF_CASE(16, 24)
#undef FEDAVG_WINNPF_CASE
    // round 6: 128 rows per wave (2 waves per SIMD: 256 registers), half the
    // chain's hand-offs of the 64-row form and room for a deep prefetch:
    // 89000000 + PF * 100 + NSMAX
#define FEDAVG_WINN128_CASE(NSMAX, PF)                                                                            \
  case 89000000 + PF * 100 + NSMAX:                                                                              \
    return launch_fused_winn<128, 1, NSMAX, PF>(clients, K, P, ld, weights, out, workspace, workspace_elems,       \
                                                sumsq, blocks_per_cu, s, what);
    FEDAVG_WINN128_CASE(8, 0)
    FEDAVG_WINN128_CASE(8, 16)
    FEDAVG_WINN128_CASE(8, 32)
    FEDAVG_WINN128_CASE(8, 48)
    FEDAVG_WINN128_CASE(8, 64)
    FEDAVG_WINN128_CASE(8, 80)
#undef FEDAVG_WINN128_CASE
    // round 6: 64-row split windows with LE rows of the next window in LDS
    // (LDS-DMA through the chain) and timing modes: 88000000 + MODE * 100000
    // + LE * 100 + PF (NSMAX 16)
#define FEDAVG_WINNLE_CASE(PF, LE, MODE)                                                                         \
  case 88000000 + MODE * 100000 + LE * 100 + PF:                                                                 \
    return launch_fused_winn<64, 1, 16, PF, LE, MODE>(clients, K, P, ld, weights, out, workspace, workspace_elems, \
                                                      sumsq, blocks_per_cu, s, what);
    FEDAVG_WINNLE_CASE(8, 0, 1)
    FEDAVG_WINNLE_CASE(8, 0, 2)
    FEDAVG_WINNLE_CASE(8, 0, 3)
    FEDAVG_WINNLE_CASE(8, 8, 0)
    FEDAVG_WINNLE_CASE(8, 16, 0)
    FEDAVG_WINNLE_CASE(8, 22, 0)
    FEDAVG_WINNLE_CASE(0, 22, 0)
    FEDAVG_WINNLE_CASE(16, 22, 0)
    FEDAVG_WINNLE_CASE(8, 0, 8)
    FEDAVG_WINNLE_CASE(0, 0, 8)
    FEDAVG_WINNLE_CASE(16, 0, 8)
    FEDAVG_WINNLE_CASE(8, 0, 16)
    FEDAVG_WINNLE_CASE(8, 0, 24)
    FEDAVG_WINNLE_CASE(16, 0, 16)
#undef FEDAVG_WINNLE_CASE
    // round 6: split-row windows with point-to-point hand-offs
    // (reduce_sqdist_winf_kernel): 91000000 + MODE * 10000 + PF * 100 + NSMAX
#define FEDAVG_WINF_CASE(NSMAX, PF, MODE)                                                                        \
  case 91000000 + MODE * 10000 + PF * 100 + NSMAX:                                                              \
    return launch_fused_winf<NSMAX, PF, MODE>(clients, K, P, ld, weights, out, workspace, workspace_elems, sumsq, s, \
                                              what);
    FEDAVG_WINF_CASE(16, 8, 0)
    FEDAVG_WINF_CASE(16, 16, 0)
    FEDAVG_WINF_CASE(16, 8, 8)
    FEDAVG_WINF_CASE(8, 8, 0)
    FEDAVG_WINF_CASE(8, 16, 0)
    FEDAVG_WINF_CASE(16, 16, 1)
    FEDAVG_WINF_CASE(16, 16, 2)
    FEDAVG_WINF_CASE(16, 16, 4)
    FEDAVG_WINF_CASE(16, 24, 0)
    FEDAVG_WINF_CASE(16, 32, 0)
    FEDAVG_WINF_CASE(16, 16, 8)
    FEDAVG_WINF_CASE(16, 16, 9)
    FEDAVG_WINF_CASE(8, 8, 1)
    FEDAVG_WINF_CASE(8, 8, 2)
    FEDAVG_WINF_CASE(8, 16, 1)
    FEDAVG_WINF_CASE(8, 8, 8)
    FEDAVG_WINF_CASE(16, 16, 16)
    FEDAVG_WINF_CASE(16, 16, 32)
    FEDAVG_WINF_CASE(8, 8, 16)
    FEDAVG_WINF_CASE(8, 8, 32)
#undef FEDAVG_WINF_CASE
    default: return set_error(FEDAVG_EMODE, "%s: cols must be 32, 64, 128 or 256 (+1000: double-buffered)", what);
  }
}
#endif  // FEDAVG_TUNING

}  // extern "C"
