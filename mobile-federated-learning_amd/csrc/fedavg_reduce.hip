// fedavg_reduce.hip -- gfx950 (MI355X / CDNA4) kernels for the FedAvg
// server-side weighted reduction, plus the C ABI declared in
// include/fedavg_amd.h.
//
// Reference semantics (src/fedavg_trainer.py:441-458): for each element p,
//     acc = x[0][p] * w[0];  acc = acc + x[i][p] * w[i]  for i = 1..K-1
// evaluated left to right, one rounding per multiply and per add.  This file
// is compiled with -ffp-contract=off and also pins `fp contract(off)` below so
// the multiply+add pair is never fused into v_fma/v_fmac (a fused form rounds
// once and would not be bit-identical to the reference's ATen CPU ops).
//
// Roofline: 2 flops per 4-byte element read -> 0.5 flop/B; the kernels are
// HBM-read bound (4*K*P bytes in, 4*P out), never MFMA work.  Layout in HBM:
// one client-major [K, ld] buffer, each row one client's flattened
// state_dict; thread t owns the 16-byte column slice [4t, 4t+4) of every row
// and walks the client axis in order, so each wave-instruction reads 1 KiB of
// one row and a thread keeps UNROLL independent 16-B loads in flight.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <utility>

#include "fedavg_amd.h"
#include "fedavg_amd_tuning.h"

#pragma clang fp contract(off)

namespace {

constexpr int kBlock = 256;  // 4 waves of 64

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

thread_local char g_err[512] = "";

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    return set_error(-static_cast<int>(e), "%s: launch failed: %s", what, hipGetErrorString(e));
  }
  g_err[0] = '\0';
  return FEDAVG_OK;
}

__host__ __device__ inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
__host__ __device__ inline bool aligned4(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 3u) == 0; }

template <bool NT, typename T>
__device__ __forceinline__ T ld(const T* p) {
  if constexpr (NT) {
    return __builtin_nontemporal_load(p);
  } else {
    return *p;
  }
}

// ---------------------------------------------------------------------------
// fp32, bit-exact, float4 path.  One thread = one 16-B column slice.
//   X    : [K, ld] fp32 viewed as [K, ld4] float4 (16-B aligned, ld % 4 == 0)
//   nvec : ceil(P / 4) column slices; the last one stores only `tail` lanes
//          when P % 4 != 0 (its extra lanes read row padding, never stored).
// ---------------------------------------------------------------------------
template <int UNROLL, bool NT, bool OUT_VEC>
__global__ __launch_bounds__(kBlock) void reduce_f32x4_kernel(
    const f32x4* __restrict__ X, int K, int64_t ld4, int64_t nvec, int tail,
    const float* __restrict__ W, float* __restrict__ out) {
  const int64_t v = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (v >= nvec) return;
  const f32x4* col = X + v;

  f32x4 acc = ld<NT>(col) * W[0];  // fedavg_trainer.py:455  (i == 0)
  int k = 1;
  for (; k + UNROLL <= K; k += UNROLL) {
    f32x4 xs[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) xs[u] = ld<NT>(col + static_cast<int64_t>(k + u) * ld4);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const f32x4 term = xs[u] * W[k + u];  // fl32(p_i * w_i)
      acc = acc + term;                     // fedavg_trainer.py:457
    }
  }
  for (; k < K; ++k) {
    const f32x4 term = ld<NT>(col + static_cast<int64_t>(k) * ld4) * W[k];
    acc = acc + term;
  }

  float* o = out + v * 4;
  if (tail == 0 || v != nvec - 1) {
    if constexpr (OUT_VEC) {
      *reinterpret_cast<f32x4*>(o) = acc;
    } else {
      o[0] = acc.x; o[1] = acc.y; o[2] = acc.z; o[3] = acc.w;
    }
  } else {
    o[0] = acc.x;
    if (tail > 1) o[1] = acc.y;
    if (tail > 2) o[2] = acc.z;
  }
}

// ---------------------------------------------------------------------------
// fp32, bit-exact, variant family (benchmarking / tuning).  Same per-element
// order as reduce_f32x4_kernel; what changes is how much each thread keeps in
// flight and how the grid walks the columns:
//   U     client rows loaded per batch,
//   C     column slices per thread (slice j at base + tid + j*256, so a block
//         covers C*4 KiB contiguous bytes of every row),
//   PIPE  register double-buffering: batch b+1's loads are issued before
//         batch b is consumed, so 2*U*C loads can be in flight per thread,
//   grid  may be capped (grid-stride over column groups).
// ---------------------------------------------------------------------------
template <int U, int C, bool NT>
__device__ __forceinline__ void load_batch(f32x4 (&xs)[U][C], const f32x4* col, int k, int64_t ld4) {
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < C; ++j) xs[u][j] = ld<NT>(col + static_cast<int64_t>(k + u) * ld4 + j * kBlock);
}

template <int U, int C>
__device__ __forceinline__ void consume_batch(f32x4 (&acc)[C], const f32x4 (&xs)[U][C], const float* W, int k) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const float w = W[k + u];
#pragma unroll
    for (int j = 0; j < C; ++j) {
      const f32x4 term = xs[u][j] * w;
      acc[j] = acc[j] + term;
    }
  }
}

template <int U, int C, bool NT, bool PIPE>
__device__ __forceinline__ void reduce_full_group(f32x4 (&acc)[C], const f32x4* col, int K, int64_t ld4,
                                                  const float* __restrict__ W) {
  const float w0 = W[0];
#pragma unroll
  for (int j = 0; j < C; ++j) acc[j] = ld<NT>(col + j * kBlock) * w0;
  const int nb = (K - 1) / U;  // full batches after client 0
  int k = 1;
  if constexpr (PIPE) {
    f32x4 xa[U][C], xb[U][C];
    int b = 0;
    if (nb > 0) load_batch<U, C, NT>(xa, col, k, ld4);
    while (b < nb) {
      if (b + 1 < nb) load_batch<U, C, NT>(xb, col, k + U, ld4);
      consume_batch<U, C>(acc, xa, W, k);
      k += U;
      if (++b >= nb) break;
      if (b + 1 < nb) load_batch<U, C, NT>(xa, col, k + U, ld4);
      consume_batch<U, C>(acc, xb, W, k);
      k += U;
      ++b;
    }
  } else {
    for (int b = 0; b < nb; ++b, k += U) {
      f32x4 xs[U][C];
      load_batch<U, C, NT>(xs, col, k, ld4);
      consume_batch<U, C>(acc, xs, W, k);
    }
  }
  for (; k < K; ++k) {
    const float w = W[k];
#pragma unroll
    for (int j = 0; j < C; ++j) {
      const f32x4 term = ld<NT>(col + static_cast<int64_t>(k) * ld4 + j * kBlock) * w;
      acc[j] = acc[j] + term;
    }
  }
}

__device__ __forceinline__ void store_slice(float* out, int64_t v, int64_t nvec, int tail, f32x4 a) {
  float* o = out + v * 4;
  if (tail == 0 || v != nvec - 1) {
    *reinterpret_cast<f32x4*>(o) = a;
  } else {
    o[0] = a.x;
    if (tail > 1) o[1] = a.y;
    if (tail > 2) o[2] = a.z;
  }
}

template <int U, int C, bool NT, bool PIPE>
__global__ __launch_bounds__(kBlock) void reduce_f32x4_var_kernel(
    const f32x4* __restrict__ X, int K, int64_t ld4, int64_t nvec, int tail,
    const float* __restrict__ W, float* __restrict__ out) {
  const int64_t span = static_cast<int64_t>(kBlock) * C;
  for (int64_t base = static_cast<int64_t>(blockIdx.x) * span; base < nvec;
       base += static_cast<int64_t>(gridDim.x) * span) {
    if (base + span <= nvec) {
      f32x4 acc[C];
      reduce_full_group<U, C, NT, PIPE>(acc, X + base + threadIdx.x, K, ld4, W);
#pragma unroll
      for (int j = 0; j < C; ++j) store_slice(out, base + threadIdx.x + j * kBlock, nvec, tail, acc[j]);
    } else {
      for (int j = 0; j < C; ++j) {
        const int64_t v = base + threadIdx.x + j * kBlock;
        if (v >= nvec) break;
        f32x4 acc[1];
        reduce_full_group<U, 1, NT, false>(acc, X + v, K, ld4, W);
        store_slice(out, v, nvec, tail, acc[0]);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// fp32, bit-exact, BALANCED PERSISTENT schedule.  The column axis is cut into
// wave-slices (64 float4 = 1 KiB of one client row); the grid is the number
// of blocks the chip holds at once and block b owns the contiguous range
// [b*N/G, (b+1)*N/G) of the N full wave-slices.  It walks its range in steps
// of 4*C slices (wave w takes slices s+w, s+w+4, ..., so a step reads 4*C KiB
// contiguous bytes of each client row); in the last, partial step each wave
// takes the cw <= C slices still inside its range (cw is wave-uniform).  Every
// block therefore streams the same number of bytes (+-1 KiB x K) and the
// launch has no tail of half-empty block rounds, whatever K and P are.  The
// trailing partial wave-slice (nvec % 64 lanes) goes to the last block.
// ---------------------------------------------------------------------------
template <int U, int CW, bool NT>
__device__ __forceinline__ void balanced_body(const f32x4* col, int K, int64_t ld4, const float* W, float* out,
                                              int64_t v0, int64_t nvec, int tail) {
  f32x4 acc[CW];
  reduce_full_group<U, CW, NT, false>(acc, col, K, ld4, W);
#pragma unroll
  for (int j = 0; j < CW; ++j) store_slice(out, v0 + j * kBlock, nvec, tail, acc[j]);
}

template <int U, int C, bool NT, int CW>
__device__ __forceinline__ void balanced_dispatch(int cw, const f32x4* col, int K, int64_t ld4, const float* W,
                                                  float* out, int64_t v0, int64_t nvec, int tail) {
  if constexpr (CW >= 1) {
    if (cw == CW) {
      balanced_body<U, CW, NT>(col, K, ld4, W, out, v0, nvec, tail);
      return;
    }
    balanced_dispatch<U, C, NT, CW - 1>(cw, col, K, ld4, W, out, v0, nvec, tail);
  }
}

template <int U, int C, bool NT>
__global__ __launch_bounds__(kBlock) void reduce_balanced_f32x4_kernel(
    const f32x4* __restrict__ X, int K, int64_t ld4, int64_t nvec, int tail,
    const float* __restrict__ W, float* __restrict__ out) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t nws = nvec / 64;  // full wave-slices
  const int64_t G = gridDim.x, b = blockIdx.x;
  const int64_t ws0 = nws * b / G, ws1 = nws * (b + 1) / G;
  for (int64_t s = ws0; s < ws1; s += 4 * C) {
    const int64_t rem = ws1 - s;
    int cw = C;
    if (rem < 4 * C) cw = rem > wave ? static_cast<int>((rem - wave + 3) / 4) : 0;
    if (cw == 0) continue;
    const int64_t v0 = (s + wave) * 64 + lane;
    balanced_dispatch<U, C, NT, C>(cw, X + v0, K, ld4, W, out, v0, nvec, tail);
  }
  if (b == G - 1 && wave == 0 && nws * 64 < nvec) {
    const int64_t v = nws * 64 + lane;
    if (v < nvec) {
      f32x4 acc[1];
      reduce_full_group<U, 1, NT, false>(acc, X + v, K, ld4, W);
      store_slice(out, v, nvec, tail, acc[0]);
    }
  }
}

// ---------------------------------------------------------------------------
// fp32, bit-exact, LDS-DMA staging: every client-row load is a
// global_load_lds_dwordx4 (1 KiB per wave-instruction, `nt` when AUX == 2)
// into the wave's own LDS slots; after its own vmcnt(0) the wave reads the
// 16 B it loaded back with ds_read_b128 (lane l reads bytes [16l, 16l+16),
// conflict-free) and accumulates in the reference order.  No cross-wave LDS
// sharing, so no barrier: only the issuing wave's vmcnt orders its reads.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gbl_ptr_t;

template <int U, int C, int AUX>
__global__ __launch_bounds__(kBlock) void reduce_glds_f32x4_kernel(
    const f32x4* __restrict__ X, int K, int64_t ld4, int64_t nvec, int tail,
    const float* __restrict__ W, float* __restrict__ out) {
  constexpr int kSlot = 1024;  // bytes one wave-instruction lands
  __shared__ __attribute__((aligned(16))) char lds[(kBlock / 64) * U * C * kSlot];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  char* mine = lds + wave * (U * C * kSlot);
  const int64_t span = static_cast<int64_t>(kBlock) * C;
  for (int64_t base = static_cast<int64_t>(blockIdx.x) * span; base < nvec;
       base += static_cast<int64_t>(gridDim.x) * span) {
    if (base + span > nvec) {
      for (int j = 0; j < C; ++j) {
        const int64_t v = base + threadIdx.x + j * kBlock;
        if (v >= nvec) break;
        f32x4 acc1[1];
        reduce_full_group<8, 1, true, false>(acc1, X + v, K, ld4, W);
        store_slice(out, v, nvec, tail, acc1[0]);
      }
      continue;
    }
    const f32x4* col = X + base + threadIdx.x;
    f32x4 acc[C];
    const float w0 = W[0];
#pragma unroll
    for (int j = 0; j < C; ++j) acc[j] = ld<true>(col + j * kBlock) * w0;
    int k = 1;
    for (; k + U <= K; k += U) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < C; ++j)
          __builtin_amdgcn_global_load_lds(
              (gbl_ptr_t)(col + static_cast<int64_t>(k + u) * ld4 + j * kBlock),
              (lds_ptr_t)(mine + (u * C + j) * kSlot), 16, 0, AUX);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float w = W[k + u];
#pragma unroll
        for (int j = 0; j < C; ++j) {
          const f32x4 x = *reinterpret_cast<const f32x4*>(mine + (u * C + j) * kSlot + lane * 16);
          const f32x4 term = x * w;
          acc[j] = acc[j] + term;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slots free before the next batch lands
    }
    for (; k < K; ++k) {
      const float w = W[k];
#pragma unroll
      for (int j = 0; j < C; ++j) {
        const f32x4 term = ld<true>(col + static_cast<int64_t>(k) * ld4 + j * kBlock) * w;
        acc[j] = acc[j] + term;
      }
    }
#pragma unroll
    for (int j = 0; j < C; ++j) store_slice(out, base + threadIdx.x + j * kBlock, nvec, tail, acc[j]);
  }
}

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

// ---------------------------------------------------------------------------
// fp32, bit-exact, TILED layout: X is [ntiles][K][1024] (tile t holds columns
// [1024t, 1024t+1024) of every client, client-major inside the tile), so a
// block streams K * 4 KiB of contiguous memory instead of K rows 4*ld apart.
// ---------------------------------------------------------------------------
constexpr int kTile = kBlock * 4;  // floats per tile row (4 KiB)

template <int U, bool NT>
__global__ __launch_bounds__(kBlock) void reduce_tiled_f32x4_kernel(
    const f32x4* __restrict__ X, int K, int64_t P, const float* __restrict__ W, float* __restrict__ out) {
  const int64_t t = blockIdx.x;
  const f32x4* col = X + t * static_cast<int64_t>(K) * kBlock + threadIdx.x;
  f32x4 acc[1];
  reduce_full_group<U, 1, NT, true>(acc, col, K, kBlock, W);
  const int64_t p0 = t * kTile + static_cast<int64_t>(threadIdx.x) * 4;
  if (p0 + 4 <= P) {
    *reinterpret_cast<f32x4*>(out + p0) = acc[0];
  } else if (p0 < P) {
    out[p0] = acc[0].x;
    if (p0 + 1 < P) out[p0 + 1] = acc[0].y;
    if (p0 + 2 < P) out[p0 + 2] = acc[0].z;
  }
}

// fp32, bit-exact, scalar path for buffers that are not 16-B aligned.
__global__ __launch_bounds__(kBlock) void reduce_f32_scalar_kernel(
    const float* __restrict__ X, int K, int64_t ld, int64_t P,
    const float* __restrict__ W, float* __restrict__ out) {
  const int64_t p = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (p >= P) return;
  float acc = X[p] * W[0];
  for (int k = 1; k < K; ++k) {
    const float term = X[static_cast<int64_t>(k) * ld + p] * W[k];
    acc = acc + term;
  }
  out[p] = acc;
}

// fp32, bit-exact, pointer-array path: client k lives at ptrs[k] (device).
// Alignment is a per-client property, so the branch is wave-uniform.
template <bool OUT_VEC>
__global__ __launch_bounds__(kBlock) void reduce_ptrs_f32_kernel(
    const float* const* __restrict__ ptrs, int K, int64_t P,
    const float* __restrict__ W, float* __restrict__ out) {
  const int64_t v = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  const int64_t p0 = v * 4;
  if (p0 >= P) return;
  const int n = (P - p0) >= 4 ? 4 : static_cast<int>(P - p0);
  f32x4 acc;
  for (int k = 0; k < K; ++k) {
    const float* base = ptrs[k];
    f32x4 x;
    if (n == 4 && aligned16(base)) {
      x = *reinterpret_cast<const f32x4*>(base + p0);
    } else {
      x.x = base[p0];
      x.y = n > 1 ? base[p0 + 1] : 0.f;
      x.z = n > 2 ? base[p0 + 2] : 0.f;
      x.w = n > 3 ? base[p0 + 3] : 0.f;
    }
    const f32x4 term = x * W[k];
    acc = (k == 0) ? term : acc + term;
  }
  float* o = out + p0;
  if (n == 4) {
    if constexpr (OUT_VEC) {
      *reinterpret_cast<f32x4*>(o) = acc;
    } else {
      o[0] = acc.x; o[1] = acc.y; o[2] = acc.z; o[3] = acc.w;
    }
  } else {
    o[0] = acc.x;
    if (n > 1) o[1] = acc.y;
    if (n > 2) o[2] = acc.z;
  }
}

// ---------------------------------------------------------------------------
// fp64: the weight stays a double (ATen opmath for double).  16 B per thread.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void reduce_f64x2_kernel(
    const f64x2* __restrict__ X, int K, int64_t ld2, int64_t nvec, int tail,
    const double* __restrict__ W, double* __restrict__ out) {
  const int64_t v = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (v >= nvec) return;
  const f64x2* col = X + v;
  f64x2 acc = col[0] * W[0];
  int k = 1;
  for (; k + 4 <= K; k += 4) {
    f64x2 xs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) xs[u] = col[static_cast<int64_t>(k + u) * ld2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f64x2 term = xs[u] * W[k + u];
      acc = acc + term;
    }
  }
  for (; k < K; ++k) {
    const f64x2 term = col[static_cast<int64_t>(k) * ld2] * W[k];
    acc = acc + term;
  }
  double* o = out + v * 2;
  o[0] = acc.x;
  if (tail == 0 || v != nvec - 1) o[1] = acc.y;
}

__global__ __launch_bounds__(kBlock) void reduce_f64_scalar_kernel(
    const double* __restrict__ X, int K, int64_t ld, int64_t P,
    const double* __restrict__ W, double* __restrict__ out) {
  const int64_t p = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (p >= P) return;
  double acc = X[p] * W[0];
  for (int k = 1; k < K; ++k) {
    const double term = X[static_cast<int64_t>(k) * ld + p] * W[k];
    acc = acc + term;
  }
  out[p] = acc;
}

// ---------------------------------------------------------------------------
// fp16 / bf16: storage type kept, each op computed in fp32 and rounded back
// (ATen opmath float):  term = rh(f32(x) * w);  acc = rh(f32(acc) + f32(term)).
// ---------------------------------------------------------------------------
struct F16Rule {
  __device__ static float to_f32(unsigned short h) {
    _Float16 v;
    __builtin_memcpy(&v, &h, 2);
    return static_cast<float>(v);
  }
  __device__ static unsigned short from_f32(float f) {
    const _Float16 v = static_cast<_Float16>(f);  // v_cvt_f16_f32, round to nearest even
    unsigned short h;
    __builtin_memcpy(&h, &v, 2);
    return h;
  }
};

struct BF16Rule {
  __device__ static float to_f32(unsigned short h) {
    return __uint_as_float(static_cast<unsigned int>(h) << 16);
  }
  // c10::BFloat16 round_to_nearest_even: NaN -> 0x7FC0.
  __device__ static unsigned short from_f32(float f) {
    if (f != f) return 0x7FC0u;
    const unsigned int u = __float_as_uint(f);
    return static_cast<unsigned short>((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
  }
};

// The fp32 intermediate is made opaque to the instruction selector: without
// it gfx950 folds fpext -> fmul -> fptrunc into one v_fma_mixlo_f16, which
// rounds the exact product straight to f16 instead of f32-then-f16.
__device__ __forceinline__ float opaque(float v) {
  asm volatile("" : "+v"(v));
  return v;
}

template <typename R>
__device__ __forceinline__ unsigned short half_step(unsigned short acc, unsigned short x, float w, bool first) {
  const unsigned short term = R::from_f32(opaque(R::to_f32(x) * w));
  if (first) return term;
  return R::from_f32(opaque(R::to_f32(acc) + R::to_f32(term)));
}

// 8 halves (16 B) per thread when aligned; scalar elements otherwise.
template <typename R>
__global__ __launch_bounds__(kBlock) void reduce_half_kernel(
    const unsigned short* __restrict__ X, int K, int64_t ld, int64_t P, bool vec,
    const float* __restrict__ W, unsigned short* __restrict__ out) {
  const int64_t v = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (vec) {
    const int64_t p0 = v * 8;
    if (p0 >= P) return;
    const int n = (P - p0) >= 8 ? 8 : static_cast<int>(P - p0);
    u16x8 acc;
    for (int k = 0; k < K; ++k) {
      const u16x8 x = *reinterpret_cast<const u16x8*>(X + static_cast<int64_t>(k) * ld + p0);
      const float w = W[k];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = half_step<R>(acc[j], x[j], w, k == 0);
    }
    if (n == 8) {
      *reinterpret_cast<u16x8*>(out + p0) = acc;
    } else {
      for (int j = 0; j < n; ++j) out[p0 + j] = acc[j];
    }
  } else {
    const int64_t p = v;
    if (p >= P) return;
    unsigned short acc = 0;
    for (int k = 0; k < K; ++k) acc = half_step<R>(acc, X[static_cast<int64_t>(k) * ld + p], W[k], k == 0);
    out[p] = acc;
  }
}

// ---------------------------------------------------------------------------
// fp64 / fp16 / bf16 production kernels: the fp32 schedule (U-row batches,
// C 16-B slices per thread, nontemporal loads, round-split dispatch) over an
// element-op policy carrying each dtype's exact per-element rule.
// ---------------------------------------------------------------------------
struct OpF64 {
  using vec = f64x2;
  using wt = double;
  using elem = double;
  static constexpr int kLanes = 2;
  __device__ static vec first(vec x, wt w) { return x * w; }
  __device__ static vec step(vec acc, vec x, wt w) {
    const vec t = x * w;
    return acc + t;
  }
};

template <typename R>
struct OpHalf {
  using vec = u16x8;
  using wt = float;
  using elem = unsigned short;
  static constexpr int kLanes = 8;
  __device__ static vec first(vec x, wt w) {
    vec r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = half_step<R>(0, x[j], w, true);
    return r;
  }
  __device__ static vec step(vec acc, vec x, wt w) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = half_step<R>(acc[j], x[j], w, false);
    return acc;
  }
};

template <class Op, int U, int C, bool NT>
__device__ __forceinline__ void reduce_vec_group(typename Op::vec (&acc)[C], const typename Op::vec* col, int K,
                                                 int64_t ldv, const typename Op::wt* __restrict__ W) {
  using vec = typename Op::vec;
  const typename Op::wt w0 = W[0];
#pragma unroll
  for (int j = 0; j < C; ++j) acc[j] = Op::first(ld<NT>(col + j * kBlock), w0);
  int k = 1;
  for (; k + U <= K; k += U) {
    vec xs[U][C];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < C; ++j) xs[u][j] = ld<NT>(col + static_cast<int64_t>(k + u) * ldv + j * kBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const typename Op::wt w = W[k + u];
#pragma unroll
      for (int j = 0; j < C; ++j) acc[j] = Op::step(acc[j], xs[u][j], w);
    }
  }
  for (; k < K; ++k) {
    const typename Op::wt w = W[k];
#pragma unroll
    for (int j = 0; j < C; ++j) acc[j] = Op::step(acc[j], ld<NT>(col + static_cast<int64_t>(k) * ldv + j * kBlock), w);
  }
}

template <class Op>
__device__ __forceinline__ void store_vec(typename Op::elem* out, int64_t v, int64_t nvec, int tail,
                                          typename Op::vec a) {
  typename Op::elem* o = out + v * Op::kLanes;
  if (tail == 0 || v != nvec - 1) {
    *reinterpret_cast<typename Op::vec*>(o) = a;
  } else {
#pragma unroll
    for (int j = 0; j < Op::kLanes; ++j)
      if (j < tail) o[j] = a[j];
  }
}

template <class Op, int U, int C, bool NT>
__global__ __launch_bounds__(kBlock) void reduce_vec_kernel(
    const typename Op::vec* __restrict__ X, int K, int64_t ldv, int64_t nvec, int tail,
    const typename Op::wt* __restrict__ W, typename Op::elem* __restrict__ out) {
  const int64_t span = static_cast<int64_t>(kBlock) * C;
  for (int64_t base = static_cast<int64_t>(blockIdx.x) * span; base < nvec;
       base += static_cast<int64_t>(gridDim.x) * span) {
    if (base + span <= nvec) {
      typename Op::vec acc[C];
      reduce_vec_group<Op, U, C, NT>(acc, X + base + threadIdx.x, K, ldv, W);
#pragma unroll
      for (int j = 0; j < C; ++j) store_vec<Op>(out, base + threadIdx.x + j * kBlock, nvec, tail, acc[j]);
    } else {
      for (int j = 0; j < C; ++j) {
        const int64_t v = base + threadIdx.x + j * kBlock;
        if (v >= nvec) break;
        typename Op::vec acc1[1];
        reduce_vec_group<Op, U, 1, NT>(acc1, X + v, K, ldv, W);
        store_vec<Op>(out, v, nvec, tail, acc1[0]);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Split-client variant (tolerance-gated).  Block = SPLITS waves over the same
// 64 column slices; wave g owns the contiguous client range
// [g*K/SPLITS, (g+1)*K/SPLITS), keeps its partial sum in registers, stages
// it in LDS, and wave 0 combines the partials in group order.
// ---------------------------------------------------------------------------
template <int SPLITS>
__global__ __launch_bounds__(64 * SPLITS) void reduce_splitk_f32x4_kernel(
    const f32x4* __restrict__ X, int K, int64_t ld4, int64_t nvec, int tail,
    const float* __restrict__ W, float* __restrict__ out) {
  __shared__ f32x4 partial[SPLITS][64];
  const int lane = threadIdx.x & 63;
  const int g = threadIdx.x >> 6;
  const int64_t v = static_cast<int64_t>(blockIdx.x) * 64 + lane;
  const int k0 = static_cast<int>((static_cast<int64_t>(K) * g) / SPLITS);
  const int k1 = static_cast<int>((static_cast<int64_t>(K) * (g + 1)) / SPLITS);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (v < nvec && k1 > k0) {
    const f32x4* col = X + v;
    acc = col[static_cast<int64_t>(k0) * ld4] * W[k0];
    int k = k0 + 1;
    for (; k + 8 <= k1; k += 8) {
      f32x4 xs[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) xs[u] = col[static_cast<int64_t>(k + u) * ld4];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const f32x4 term = xs[u] * W[k + u];
        acc = acc + term;
      }
    }
    for (; k < k1; ++k) {
      const f32x4 term = col[static_cast<int64_t>(k) * ld4] * W[k];
      acc = acc + term;
    }
  }
  partial[g][lane] = acc;
  __syncthreads();
  if (g != 0 || v >= nvec) return;
  f32x4 s = partial[0][lane];
#pragma unroll
  for (int j = 1; j < SPLITS; ++j) {
    // groups with an empty client range (K < SPLITS) contribute nothing
    const int a = static_cast<int>((static_cast<int64_t>(K) * j) / SPLITS);
    const int b = static_cast<int>((static_cast<int64_t>(K) * (j + 1)) / SPLITS);
    if (b > a) s = s + partial[j][lane];
  }
  float* o = out + v * 4;
  if (tail == 0 || v != nvec - 1) {
    o[0] = s.x; o[1] = s.y; o[2] = s.z; o[3] = s.w;
  } else {
    o[0] = s.x;
    if (tail > 1) o[1] = s.y;
    if (tail > 2) o[2] = s.z;
  }
}

inline unsigned grid_for(int64_t items, int per_block) {
  return static_cast<unsigned>((items + per_block - 1) / per_block);
}

int check_common(const void* clients, int64_t K, int64_t P, int64_t ld, const void* weights,
                 const void* out, const char* what) {
  if (K <= 0) return set_error(FEDAVG_EINVAL, "%s: K must be >= 1 (got %lld)", what, (long long)K);
  if (K > INT32_MAX) return set_error(FEDAVG_EINVAL, "%s: K too large", what);
  if (P < 0) return set_error(FEDAVG_EINVAL, "%s: P must be >= 0", what);
  if (ld < P) return set_error(FEDAVG_EINVAL, "%s: ld (%lld) < P (%lld)", what, (long long)ld, (long long)P);
  if (P > 0 && (!clients || !weights || !out)) return set_error(FEDAVG_EINVAL, "%s: null buffer", what);
  return FEDAVG_OK;
}

template <int U, bool NT>
void launch_f32x4(const float* clients, int K, int64_t ld, int64_t P, const float* W, float* out,
                  hipStream_t s) {
  const int64_t nvec = (P + 3) / 4;
  const int tail = static_cast<int>(P & 3);
  const f32x4* X = reinterpret_cast<const f32x4*>(clients);
  if (aligned16(out)) {
    hipLaunchKernelGGL((reduce_f32x4_kernel<U, NT, true>), dim3(grid_for(nvec, kBlock)), dim3(kBlock), 0, s,
                       X, K, ld / 4, nvec, tail, W, out);
  } else {
    hipLaunchKernelGGL((reduce_f32x4_kernel<U, NT, false>), dim3(grid_for(nvec, kBlock)), dim3(kBlock), 0, s,
                       X, K, ld / 4, nvec, tail, W, out);
  }
}

int reduce_f32_impl(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights,
                    float* out, hipStream_t s, int unroll, int nontemporal, const char* what) {
  int rc = check_common(clients, K, P, ld, weights, out, what);
  if (rc) return rc;
  if (P == 0) return FEDAVG_OK;
  if (!aligned4(clients) || !aligned4(out) || !aligned4(weights))
    return set_error(FEDAVG_EALIGN, "%s: fp32 buffers must be 4-byte aligned", what);
  const int k = static_cast<int>(K);
  if (aligned16(clients) && (ld % 4) == 0) {
    switch (unroll * 2 + (nontemporal ? 1 : 0)) {
      case 4 * 2 + 0: launch_f32x4<4, false>(clients, k, ld, P, weights, out, s); break;
      case 4 * 2 + 1: launch_f32x4<4, true>(clients, k, ld, P, weights, out, s); break;
      case 8 * 2 + 0: launch_f32x4<8, false>(clients, k, ld, P, weights, out, s); break;
      case 8 * 2 + 1: launch_f32x4<8, true>(clients, k, ld, P, weights, out, s); break;
      case 16 * 2 + 0: launch_f32x4<16, false>(clients, k, ld, P, weights, out, s); break;
      case 16 * 2 + 1: launch_f32x4<16, true>(clients, k, ld, P, weights, out, s); break;
      default: return set_error(FEDAVG_EMODE, "%s: unsupported unroll %d", what, unroll);
    }
  } else {
    hipLaunchKernelGGL(reduce_f32_scalar_kernel, dim3(grid_for(P, kBlock)), dim3(kBlock), 0, s,
                       clients, k, ld, P, weights, out);
  }
  return launch_status(what);
}

template <int U, int C, bool NT, bool PIPE>
void launch_var(const float* clients, int K, int64_t ld, int64_t P, const float* W, float* out, int max_blocks,
                hipStream_t s) {
  const int64_t nvec = (P + 3) / 4;
  const int64_t span = static_cast<int64_t>(kBlock) * C;
  int64_t grid = (nvec + span - 1) / span;
  if (max_blocks > 0 && grid > max_blocks) grid = max_blocks;
  hipLaunchKernelGGL((reduce_f32x4_var_kernel<U, C, NT, PIPE>), dim3(static_cast<unsigned>(grid)), dim3(kBlock), 0,
                     s, reinterpret_cast<const f32x4*>(clients), K, ld / 4, nvec, static_cast<int>(P & 3), W, out);
}

template <int U, int C, int AUX>
void launch_glds(const float* clients, int K, int64_t ld, int64_t P, const float* W, float* out, int max_blocks,
                 hipStream_t s) {
  const int64_t nvec = (P + 3) / 4;
  const int64_t span = static_cast<int64_t>(kBlock) * C;
  int64_t grid = (nvec + span - 1) / span;
  if (max_blocks > 0 && grid > max_blocks) grid = max_blocks;
  hipLaunchKernelGGL((reduce_glds_f32x4_kernel<U, C, AUX>), dim3(static_cast<unsigned>(grid)), dim3(kBlock), 0, s,
                     reinterpret_cast<const f32x4*>(clients), K, ld / 4, nvec, static_cast<int>(P & 3), W, out);
}

// Blocks of a kernel the whole chip holds at once (occupancy x CUs), cached
// per (device, kernel) -- kernels of one signature share a template
// instantiation of this function, so the cache must be keyed by the kernel.
template <typename Kern>
int64_t resident_blocks(Kern kernel) {
  static std::mutex mu;
  static std::map<std::pair<int, const void*>, int64_t> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 1024;
  const auto key = std::make_pair(dev, reinterpret_cast<const void*>(kernel));
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, 0) != hipSuccess || per_cu <= 0) per_cu = 1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  const int64_t n = static_cast<int64_t>(per_cu) * cus;
  std::lock_guard<std::mutex> lk(mu);
  cache[key] = n;
  return n;
}

template <int U, int C, bool NT>
void launch_balanced(const float* clients, int K, int64_t ld, int64_t P, const float* W, float* out, int max_blocks,
                     hipStream_t s) {
  const int64_t nvec = (P + 3) / 4;
  const int64_t nws = nvec / 64;
  int64_t grid = max_blocks > 0 ? max_blocks : resident_blocks(reduce_balanced_f32x4_kernel<U, C, NT>);
  if (grid > nws) grid = nws > 0 ? nws : 1;
  hipLaunchKernelGGL((reduce_balanced_f32x4_kernel<U, C, NT>), dim3(static_cast<unsigned>(grid)), dim3(kBlock), 0, s,
                     reinterpret_cast<const f32x4*>(clients), K, ld / 4, nvec, static_cast<int>(P & 3), W, out);
}

// Round-split dispatch: the column range is cut into the fewest EQUAL
// launches whose blocks all fit on the chip at once (one resident round
// each).  Within a launch every block starts together and the running blocks
// sweep one compact window of every client row; the stream boundary between
// launches re-aligns them (a multi-round launch lets blocks drift apart and
// leaves a half-empty last round).
template <int U, int C, bool NT>
void launch_split(const float* clients, int K, int64_t ld, int64_t P, const float* W, float* out, int max_blocks,
                  hipStream_t s) {
  const int64_t nvec = (P + 3) / 4;
  const int64_t span = static_cast<int64_t>(kBlock) * C;
  const int64_t resident = max_blocks > 0 ? max_blocks : resident_blocks(reduce_f32x4_var_kernel<U, C, NT, false>);
  const int64_t blocks = (nvec + span - 1) / span;
  const int64_t nl = (blocks + resident - 1) / resident;
  const int64_t per = ((nvec + nl - 1) / nl + span - 1) / span * span;  // float4 columns per launch
  const f32x4* X = reinterpret_cast<const f32x4*>(clients);
  for (int64_t v0 = 0; v0 < nvec; v0 += per) {
    const int64_t n = (nvec - v0) < per ? (nvec - v0) : per;
    const int tail = (v0 + n == nvec) ? static_cast<int>(P & 3) : 0;
    hipLaunchKernelGGL((reduce_f32x4_var_kernel<U, C, NT, false>), dim3(static_cast<unsigned>((n + span - 1) / span)),
                       dim3(kBlock), 0, s, X + v0, K, ld / 4, n, tail, W, out + v0 * 4);
  }
}

int cu_count() {
  static std::mutex mu;
  static std::map<int, int> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  cache[dev] = cus;
  return cus;
}

// Windowed balanced dispatch: every launch has EXACTLY G blocks (a multiple
// of the CU count, so each CU gets the same number of equal-work blocks) and
// covers one window of ~G*4C wave-slices; inside the window the balanced
// kernel gives each block an equal contiguous share (+-1 KiB x K).  Windows
// are equal-sized and processed in order, so each launch sweeps one compact
// window of every client row.  max_blocks = G (0 = 3 x CUs).
template <int U, int C, bool NT>
void launch_window(const float* clients, int K, int64_t ld, int64_t P, const float* W, float* out, int max_blocks,
                   hipStream_t s) {
  const int64_t nvec = (P + 3) / 4;
  const int64_t G = max_blocks > 0 ? max_blocks : 3 * static_cast<int64_t>(cu_count());
  const int64_t win_ws = G * 4 * C;                   // wave-slices one window holds at full steps
  const int64_t nws = (nvec + 63) / 64;               // wave-slices incl. a partial last one
  const int64_t nl = (nws + win_ws - 1) / win_ws;
  const int64_t per_ws = (nws + nl - 1) / nl;         // equal windows, in wave-slices
  const f32x4* X = reinterpret_cast<const f32x4*>(clients);
  for (int64_t w0 = 0; w0 < nws; w0 += per_ws) {
    const int64_t v0 = w0 * 64;
    const int64_t n = std::min<int64_t>(per_ws * 64, nvec - v0);
    const int tail = (v0 + n == nvec) ? static_cast<int>(P & 3) : 0;
    int64_t grid = std::min<int64_t>(G, std::max<int64_t>(1, n / 64));
    hipLaunchKernelGGL((reduce_balanced_f32x4_kernel<U, C, NT>), dim3(static_cast<unsigned>(grid)), dim3(kBlock), 0,
                       s, X + v0, K, ld / 4, n, tail, W, out + v0 * 4);
  }
}

typedef void (*var_launcher)(const float*, int, int64_t, int64_t, const float*, float*, int, hipStream_t);

// pipe: 0 = plain register batches, 1 = register double-buffering, 2 = LDS-DMA staging,
//       3 = balanced persistent (grid = resident blocks unless max_blocks > 0),
//       4 = round-split launches of the plain kernel (max_blocks = blocks per round, 0 = resident),
//       5 = windowed balanced launches of exactly max_blocks blocks (0 = 3 x CUs)
template <int U, int C>
var_launcher pick_var2(int nt, int pipe) {
  if (pipe == 3) {
    if constexpr (U * C <= 32) return nt ? launch_balanced<U, C, true> : launch_balanced<U, C, false>;
    return nullptr;
  }
  if (pipe == 4) return nt ? launch_split<U, C, true> : launch_split<U, C, false>;
  if (pipe == 5) {
    if constexpr (U * C <= 64) return nt ? launch_window<U, C, true> : launch_window<U, C, false>;
    return nullptr;
  }
  if (pipe == 2) {
    if constexpr (U * C <= 16) return nt ? launch_glds<U, C, 2> : launch_glds<U, C, 0>;
    return nullptr;
  }
  if constexpr (U * C <= 32) {
    if (nt) return pipe ? launch_var<U, C, true, true> : launch_var<U, C, true, false>;
    return pipe ? launch_var<U, C, false, true> : launch_var<U, C, false, false>;
  } else {
    if (pipe) return nullptr;  // would spill
    return nt ? launch_var<U, C, true, false> : launch_var<U, C, false, false>;
  }
}

template <int U>
var_launcher pick_var1(int cols, int nt, int pipe) {
  switch (cols) {
    case 1: return pick_var2<U, 1>(nt, pipe);
    case 2: return pick_var2<U, 2>(nt, pipe);
    case 4: return pick_var2<U, 4>(nt, pipe);
    case 8:
      if constexpr (U <= 8) return pick_var2<U, 8>(nt, pipe);
      return nullptr;
    case 16:
      if constexpr (U <= 2) return pick_var2<U, 16>(nt, pipe);
      return nullptr;
    default: return nullptr;
  }
}

var_launcher pick_var(int unroll, int cols, int nt, int pipe) {
  switch (unroll) {
    case 32:  // deep batches for short rows / many clients (latency-bound shapes)
      if (cols == 1) return pick_var2<32, 1>(nt, pipe);
      if (cols == 2) return pick_var2<32, 2>(nt, pipe);
      return nullptr;
    case 1: return pick_var1<1>(cols, nt, pipe);
    case 2: return pick_var1<2>(cols, nt, pipe);
    case 4: return pick_var1<4>(cols, nt, pipe);
    case 8: return pick_var1<8>(cols, nt, pipe);
    case 16: return pick_var1<16>(cols, nt, pipe);
    default: return nullptr;
  }
}

// ---------------------------------------------------------------------------
// Production schedule for the exact fp32 reduce (fedavg_reduce_f32), chosen
// from the in-process A/B sweeps in profiles/ (scripts/kernel_variants.py):
//   * column slices per thread C: the widest of 8/4/2/1 that still gives a
//     launch >= 512 blocks (a block then reads C*4 KiB contiguous bytes of
//     each client row per step); U (rows per load batch) = 4 for C = 8, else 8
//     (32 and 32/16/8 16-B loads in flight per thread);
//   * round-split dispatch: the column range is cut into the fewest equal
//     launches of <= 768 blocks (2-3 blocks per CU) -- one resident round
//     each, so every launch's blocks start together and sweep one compact
//     window of every row (88% of HBM peak at K=100 x P=25M vs 76% for one
//     multi-round launch of the same kernel);
//   * nontemporal loads (the rows are read once), except for working sets of
//     64-240 MiB, which stay resident in the 256 MiB Infinity Cache across
//     back-to-back rounds when loaded with the default policy (there U = 16,
//     C = 4 was fastest: 89% vs 81% for C = 1).
// ---------------------------------------------------------------------------
struct Schedule {
  int unroll, cols, nt, blocks_per_launch;
};

constexpr int kBlocksPerLaunch = 768;

Schedule choose_schedule(int64_t K, int64_t P) {
  const int64_t nvec = (P + 3) / 4;
  Schedule sc{8, 1, 1, kBlocksPerLaunch};
  if (K <= 4) {
    // a block's work is tiny (K rows): one launch, many short blocks; round
    // splitting would only add launch boundaries (K=2..3 sweeps: +14-22 %)
    sc.cols = 1;
    sc.blocks_per_launch = 1 << 30;
  } else if (nvec >= int64_t(512) * kBlock * 8) {
    sc.unroll = 4, sc.cols = 8;
  } else if (nvec >= int64_t(512) * kBlock * 4) {
    sc.cols = 4;
  } else if (nvec >= int64_t(512) * kBlock * 2) {
    sc.cols = 2;
  } else {
    // short rows: few blocks, so each thread's client chain is the critical
    // path; deeper batches (16 rows) cut its round trips (+11-12 %), and with
    // many clients 4 slices per thread keep 64 loads in flight
    sc.unroll = 16;
    sc.cols = (K >= 500 && nvec >= int64_t(128) * kBlock * 4) ? 4 : 1;
  }
  const double bytes = 4.0 * static_cast<double>(K) * static_cast<double>(P);
  if (K > 4 && bytes > 64.0 * (1 << 20) && bytes <= 240.0 * (1 << 20)) {
    // Infinity-Cache-resident band: default-policy loads, and a deep, wide
    // per-thread batch (16 rows x 4 slices) measured fastest there
    sc.nt = 0;
    sc.unroll = 16;
    sc.cols = 4;
  }
  return sc;
}

void launch_production_f32(const float* clients, int K, int64_t ld, int64_t P, const float* W, float* out,
                           hipStream_t s) {
  const Schedule sc = choose_schedule(K, P);
  var_launcher fn = pick_var(sc.unroll, sc.cols, sc.nt, 4);
  fn(clients, K, ld, P, W, out, sc.blocks_per_launch, s);
}

// Round-split launches of reduce_vec_kernel (fp64 / fp16 / bf16).  The
// schedule is the fp32 one for the same number of 16-B column slices and the
// same byte footprint (choose_schedule takes fp32-equivalent element counts).
template <class Op, int U, int C, bool NT>
void launch_vec_split(const void* clients, int K, int64_t ld, int64_t P, const void* W, void* out, int bpl,
                      hipStream_t s) {
  using vec = typename Op::vec;
  const int64_t lanes = Op::kLanes;
  const int64_t nvec = (P + lanes - 1) / lanes;
  const int64_t span = static_cast<int64_t>(kBlock) * C;
  const int64_t blocks = (nvec + span - 1) / span;
  const int64_t nl = (blocks + bpl - 1) / bpl;
  const int64_t per = ((nvec + nl - 1) / nl + span - 1) / span * span;
  const vec* X = reinterpret_cast<const vec*>(clients);
  auto* O = reinterpret_cast<typename Op::elem*>(out);
  for (int64_t v0 = 0; v0 < nvec; v0 += per) {
    const int64_t n = (nvec - v0) < per ? (nvec - v0) : per;
    const int tail = (v0 + n == nvec) ? static_cast<int>(P % lanes) : 0;
    hipLaunchKernelGGL((reduce_vec_kernel<Op, U, C, NT>), dim3(static_cast<unsigned>((n + span - 1) / span)),
                       dim3(kBlock), 0, s, X + v0, K, ld / lanes, n, tail,
                       reinterpret_cast<const typename Op::wt*>(W), O + v0 * lanes);
  }
}

template <class Op, bool NT>
void launch_vec_nt(const Schedule& sc, const void* clients, int K, int64_t ld, int64_t P, const void* W, void* out,
                   hipStream_t s) {
  int key = sc.unroll * 100 + sc.cols;
  if constexpr (Op::kLanes == 8) {
    // fp16/bf16 unpack every 16-B vector into 8 fp32 lanes of work: halve the
    // rows per batch so the schedule stays spill-free (same bytes per block-step)
    switch (key) {
      case 408: key = 208; break;
      case 804: case 1604: key = 404; break;
      case 1601: key = 801; break;
      default: break;
    }
  }
  switch (key) {
    case 408: launch_vec_split<Op, 4, 8, NT>(clients, K, ld, P, W, out, sc.blocks_per_launch, s); break;
    case 208: launch_vec_split<Op, 2, 8, NT>(clients, K, ld, P, W, out, sc.blocks_per_launch, s); break;
    case 804: launch_vec_split<Op, 8, 4, NT>(clients, K, ld, P, W, out, sc.blocks_per_launch, s); break;
    case 404: launch_vec_split<Op, 4, 4, NT>(clients, K, ld, P, W, out, sc.blocks_per_launch, s); break;
    case 802: launch_vec_split<Op, 8, 2, NT>(clients, K, ld, P, W, out, sc.blocks_per_launch, s); break;
    case 801: launch_vec_split<Op, 8, 1, NT>(clients, K, ld, P, W, out, sc.blocks_per_launch, s); break;
    case 1604: launch_vec_split<Op, 16, 4, NT>(clients, K, ld, P, W, out, sc.blocks_per_launch, s); break;
    default: launch_vec_split<Op, 16, 1, NT>(clients, K, ld, P, W, out, sc.blocks_per_launch, s); break;
  }
}

// elem_bytes: 8 (fp64) or 2 (fp16/bf16).  The fp32 schedule is chosen for the
// problem with the same 16-B slice count and byte footprint.
template <class Op>
void launch_production_vec(const void* clients, int K, int64_t ld, int64_t P, const void* W, void* out,
                           hipStream_t s) {
  const int64_t f32_equiv = P * static_cast<int64_t>(16 / Op::kLanes) / 4;  // same bytes per row
  const Schedule sc = choose_schedule(K, f32_equiv);
  if (sc.nt)
    launch_vec_nt<Op, true>(sc, clients, K, ld, P, W, out, s);
  else
    launch_vec_nt<Op, false>(sc, clients, K, ld, P, W, out, s);
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int fedavg_abi_version(void) { return 1; }

const char* fedavg_last_error(void) { return g_err; }

int fedavg_reduce_f32(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights,
                      float* out, void* stream) {
  const char* what = "fedavg_reduce_f32";
  if (aligned16(clients) && aligned16(out) && (ld % 4) == 0 && P > 0 && K > 0) {
    int rc = check_common(clients, K, P, ld, weights, out, what);
    if (rc) return rc;
    if (!aligned4(weights)) return set_error(FEDAVG_EALIGN, "%s: weights must be 4-byte aligned", what);
    launch_production_f32(clients, static_cast<int>(K), ld, P, weights, out, static_cast<hipStream_t>(stream));
    return launch_status(what);
  }
  // unaligned buffers / odd row stride: the first-version kernels (same bits)
  return reduce_f32_impl(clients, K, P, ld, weights, out, static_cast<hipStream_t>(stream),
                         FEDAVG_DEFAULT_UNROLL, FEDAVG_DEFAULT_NONTEMPORAL, what);
}

int fedavg_f32_schedule(int64_t K, int64_t P, int* unroll, int* cols, int* nontemporal, int* launches) {
  if (K <= 0 || P < 0) return set_error(FEDAVG_EINVAL, "fedavg_f32_schedule: bad sizes");
  const Schedule sc = choose_schedule(K, P);
  const int64_t nvec = (P + 3) / 4;
  const int64_t span = static_cast<int64_t>(kBlock) * sc.cols;
  const int64_t blocks = (nvec + span - 1) / span;
  if (unroll) *unroll = sc.unroll;
  if (cols) *cols = sc.cols;
  if (nontemporal) *nontemporal = sc.nt;
  if (launches) *launches = static_cast<int>((blocks + sc.blocks_per_launch - 1) / sc.blocks_per_launch);
  return FEDAVG_OK;
}

int fedavg_reduce_f32_tuned(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights,
                            float* out, int unroll, int nontemporal, void* stream) {
  return reduce_f32_impl(clients, K, P, ld, weights, out, static_cast<hipStream_t>(stream), unroll,
                         nontemporal, "fedavg_reduce_f32_tuned");
}

int fedavg_reduce_f32_variant(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights,
                              float* out, int unroll, int nontemporal, int cols, int pipelined, int max_blocks,
                              void* stream) {
  const char* what = "fedavg_reduce_f32_variant";
  int rc = check_common(clients, K, P, ld, weights, out, what);
  if (rc) return rc;
  if (P == 0) return FEDAVG_OK;
  if (!aligned16(clients) || !aligned16(out) || (ld % 4) != 0)
    return set_error(FEDAVG_EALIGN, "%s: needs 16-B aligned clients/out and ld %% 4 == 0", what);
  var_launcher fn = pick_var(unroll, cols, nontemporal ? 1 : 0, pipelined);
  if (!fn) return set_error(FEDAVG_EMODE, "%s: unsupported unroll=%d cols=%d", what, unroll, cols);
  fn(clients, static_cast<int>(K), ld, P, weights, out, max_blocks, static_cast<hipStream_t>(stream));
  return launch_status(what);
}

int fedavg_reduce_tiled_f32(const float* tiles, int64_t K, int64_t P, const float* weights, float* out,
                            int unroll, void* stream) {
  const char* what = "fedavg_reduce_tiled_f32";
  int rc = check_common(tiles, K, P, P, weights, out, what);
  if (rc) return rc;
  if (P == 0) return FEDAVG_OK;
  if (!aligned16(tiles) || !aligned4(out)) return set_error(FEDAVG_EALIGN, "%s: tiles must be 16-B aligned", what);
  const int64_t ntiles = (P + kTile - 1) / kTile;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const f32x4* X = reinterpret_cast<const f32x4*>(tiles);
  const int k = static_cast<int>(K);
  switch (unroll) {
    case 4: hipLaunchKernelGGL((reduce_tiled_f32x4_kernel<4, false>), dim3(ntiles), dim3(kBlock), 0, s, X, k, P, weights, out); break;
    case 8: hipLaunchKernelGGL((reduce_tiled_f32x4_kernel<8, false>), dim3(ntiles), dim3(kBlock), 0, s, X, k, P, weights, out); break;
    case 16: hipLaunchKernelGGL((reduce_tiled_f32x4_kernel<16, false>), dim3(ntiles), dim3(kBlock), 0, s, X, k, P, weights, out); break;
    default: return set_error(FEDAVG_EMODE, "%s: unsupported unroll %d", what, unroll);
  }
  return launch_status(what);
}

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

int fedavg_reduce_ptrs_f32(const float* const* client_ptrs, int64_t K, int64_t P, const float* weights,
                           float* out, void* stream) {
  const char* what = "fedavg_reduce_ptrs_f32";
  int rc = check_common(client_ptrs, K, P, P, weights, out, what);
  if (rc) return rc;
  if (P == 0) return FEDAVG_OK;
  if (!aligned4(out) || !aligned4(weights)) return set_error(FEDAVG_EALIGN, "%s: out/weights misaligned", what);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t nvec = (P + 3) / 4;
  if (aligned16(out)) {
    hipLaunchKernelGGL(reduce_ptrs_f32_kernel<true>, dim3(grid_for(nvec, kBlock)), dim3(kBlock), 0, s,
                       client_ptrs, static_cast<int>(K), P, weights, out);
  } else {
    hipLaunchKernelGGL(reduce_ptrs_f32_kernel<false>, dim3(grid_for(nvec, kBlock)), dim3(kBlock), 0, s,
                       client_ptrs, static_cast<int>(K), P, weights, out);
  }
  return launch_status(what);
}

int fedavg_reduce_f64(const double* clients, int64_t K, int64_t P, int64_t ld, const double* weights,
                      double* out, void* stream) {
  const char* what = "fedavg_reduce_f64";
  int rc = check_common(clients, K, P, ld, weights, out, what);
  if (rc) return rc;
  if (P == 0) return FEDAVG_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uintptr_t m = 7u;
  if ((reinterpret_cast<uintptr_t>(clients) | reinterpret_cast<uintptr_t>(out) |
       reinterpret_cast<uintptr_t>(weights)) & m)
    return set_error(FEDAVG_EALIGN, "%s: fp64 buffers must be 8-byte aligned", what);
  if (aligned16(clients) && aligned16(out) && (ld % 2) == 0) {
    launch_production_vec<OpF64>(clients, static_cast<int>(K), ld, P, weights, out, s);
  } else {
    hipLaunchKernelGGL(reduce_f64_scalar_kernel, dim3(grid_for(P, kBlock)), dim3(kBlock), 0, s, clients,
                       static_cast<int>(K), ld, P, weights, out);
  }
  return launch_status(what);
}

static int reduce_half_entry(bool bf16, const uint16_t* clients, int64_t K, int64_t P, int64_t ld,
                             const float* weights, uint16_t* out, void* stream, const char* what) {
  int rc = check_common(clients, K, P, ld, weights, out, what);
  if (rc) return rc;
  if (P == 0) return FEDAVG_OK;
  if ((reinterpret_cast<uintptr_t>(clients) | reinterpret_cast<uintptr_t>(out)) & 1u)
    return set_error(FEDAVG_EALIGN, "%s: 16-bit buffers must be 2-byte aligned", what);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool vec = aligned16(clients) && aligned16(out) && (ld % 8) == 0;
  if (vec) {
    if (bf16)
      launch_production_vec<OpHalf<BF16Rule>>(clients, static_cast<int>(K), ld, P, weights, out, s);
    else
      launch_production_vec<OpHalf<F16Rule>>(clients, static_cast<int>(K), ld, P, weights, out, s);
    return launch_status(what);
  }
  const int64_t items = P;
  const auto* X = reinterpret_cast<const unsigned short*>(clients);
  auto* O = reinterpret_cast<unsigned short*>(out);
  if (bf16) {
    hipLaunchKernelGGL(reduce_half_kernel<BF16Rule>, dim3(grid_for(items, kBlock)), dim3(kBlock), 0, s, X,
                       static_cast<int>(K), ld, P, vec, weights, O);
  } else {
    hipLaunchKernelGGL(reduce_half_kernel<F16Rule>, dim3(grid_for(items, kBlock)), dim3(kBlock), 0, s, X,
                       static_cast<int>(K), ld, P, vec, weights, O);
  }
  return launch_status(what);
}

int fedavg_reduce_f16(const uint16_t* clients, int64_t K, int64_t P, int64_t ld, const float* weights,
                      uint16_t* out, void* stream) {
  return reduce_half_entry(false, clients, K, P, ld, weights, out, stream, "fedavg_reduce_f16");
}

int fedavg_reduce_bf16(const uint16_t* clients, int64_t K, int64_t P, int64_t ld, const float* weights,
                       uint16_t* out, void* stream) {
  return reduce_half_entry(true, clients, K, P, ld, weights, out, stream, "fedavg_reduce_bf16");
}

int fedavg_reduce_splitk_f32(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights,
                             float* out, int splits, void* stream) {
  const char* what = "fedavg_reduce_splitk_f32";
  if (splits == 1) return fedavg_reduce_f32(clients, K, P, ld, weights, out, stream);
  int rc = check_common(clients, K, P, ld, weights, out, what);
  if (rc) return rc;
  if (P == 0) return FEDAVG_OK;
  if (!aligned16(clients) || (ld % 4) != 0 || !aligned4(out))
    return set_error(FEDAVG_EALIGN, "%s: needs 16-B aligned clients and ld %% 4 == 0", what);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t nvec = (P + 3) / 4;
  const int tail = static_cast<int>(P & 3);
  const f32x4* X = reinterpret_cast<const f32x4*>(clients);
  const unsigned grid = grid_for(nvec, 64);
  const int k = static_cast<int>(K);
  switch (splits) {
    case 2: hipLaunchKernelGGL(reduce_splitk_f32x4_kernel<2>, dim3(grid), dim3(128), 0, s, X, k, ld / 4, nvec, tail, weights, out); break;
    case 4: hipLaunchKernelGGL(reduce_splitk_f32x4_kernel<4>, dim3(grid), dim3(256), 0, s, X, k, ld / 4, nvec, tail, weights, out); break;
    case 8: hipLaunchKernelGGL(reduce_splitk_f32x4_kernel<8>, dim3(grid), dim3(512), 0, s, X, k, ld / 4, nvec, tail, weights, out); break;
    default: return set_error(FEDAVG_EMODE, "%s: splits must be 1, 2, 4 or 8 (got %d)", what, splits);
  }
  return launch_status(what);
}

int fedavg_weights_f32(const int64_t* sample_nums, int64_t K, float* weights) {
  if (K <= 0 || !sample_nums || !weights) return set_error(FEDAVG_EINVAL, "fedavg_weights_f32: bad arguments");
  int64_t total = 0;
  for (int64_t i = 0; i < K; ++i) {
    if (sample_nums[i] < 0) return set_error(FEDAVG_EINVAL, "fedavg_weights_f32: negative sample count");
    total += sample_nums[i];
    if (total > (int64_t(1) << 53)) return set_error(FEDAVG_EINVAL, "fedavg_weights_f32: sum exceeds 2^53");
  }
  if (total == 0) return set_error(FEDAVG_EINVAL, "fedavg_weights_f32: sample counts sum to zero (ZeroDivisionError)");
  const double n = static_cast<double>(total);
  for (int64_t i = 0; i < K; ++i) {
    volatile double w = static_cast<double>(sample_nums[i]) / n;  // Python int / int (exact operands)
    weights[i] = static_cast<float>(w);                             // ATen double -> float scalar cast
  }
  g_err[0] = '\0';
  return FEDAVG_OK;
}

}  // extern "C"
