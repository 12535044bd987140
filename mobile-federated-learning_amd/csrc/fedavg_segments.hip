// fedavg_segments.hip -- zero-copy aggregation of DEVICE-resident clients.
//
// When the clients' state_dicts are already in HBM (client.py:96 without the
// .cpu()), the reduction (fedavg_trainer.py:450-457) and the :291 distance
// pass can read every client's tensors where they lie instead of packing them
// into [K, ld] rows first: packing moves 8 B per element (read + write) before
// the reduce reads 4 B again, so a round costs 12 B per element through rows
// and 4 B here.  The model's fp32 group is described by a key table
// (numel, output offset, source kind) and a pointer table [n_keys][K] (client
// k's address of key j).  Each key is cut into units of kSegSpan columns; a
// workgroup reduces one unit over all K clients with the production schedule
// (U4 client rows per batch, C4 16-B column slices per thread), reading each
// client through its pointer with dword-aligned 16-B loads (client tensors
// need only fp32 alignment; full units through a buffer descriptor per
// client, tails through global pointers), in the reference's client order with
// separately rounded products and sums -- the bits of fedavg_reduce_f32 on
// the packed rows.  Integer/bool keys (num_batches_tracked, ...) are converted
// to fp32 per element with static_cast, as the packers do.  Units are issued
// key-major in round-split launches of 3 x CUs workgroups, so a launch streams
// one compact window of every client's tensors, like the row-major reduce.
#include "common.hpp"
#include "staging.hpp"

#include <chrono>
#include <vector>

namespace {
using namespace fedavg_impl;
// the host-side staged layouts (key table, pointer table, descriptor table,
// workspace sizes): staging.hpp, which g++ also builds for the sanitizer fuzz
using fedavg_staging::kBool;
using fedavg_staging::kI16;
using fedavg_staging::kI32;
using fedavg_staging::kI64;
using fedavg_staging::kI8;
using fedavg_staging::kRaw;
using fedavg_staging::kSegDescMaxBytes;
using fedavg_staging::kSegUnitMapMax;
using fedavg_staging::kSegWinTablePad;
using fedavg_staging::kU8;
using fedavg_staging::kWinRsrcFlags;
using fedavg_staging::IntKey;
using fedavg_staging::round16;
using fedavg_staging::round_ws;
using fedavg_staging::RoundWs;
using fedavg_staging::seg_desc_bytes;
using fedavg_staging::SegKey;

typedef f32x4 f32x4_a4 __attribute__((aligned(4)));  // dword-aligned 16-B vector (client tensors, outputs)

// U4 x C4: units of 4,096 columns.  The multi-key sweep (scripts/
// segments_probe.py --model, profiles/r01_segments_models.jsonl) measured
// resnet56 x 100 at 113 us against 161 us for U4 x C8 (more units for the
// mid-size keys, cheaper masked tails), FEMNIST 19.1 vs 20.2 us, and the flat
// 25M-element key level (6,256 vs 6,226 GB/s); U2 x C16 loses 2.7x on resnet56.
constexpr int kSegU = 4;
constexpr int kSegC = 4;
constexpr int64_t kSegSpan = static_cast<int64_t>(kBlock) * kSegC * 4;  // columns per unit
// Round 3: full units run reduce_raw_unit's STYLE 2 -- loads and products
// interleaved in (row, slice) order with two loads of the wave in flight
// (a sched_barrier keeps the compiler from bunching a batch's loads) -- in
// launches of 2 workgroups per CU.  Interleaved against the round-2 schedule
// (U4 x C4, batch loads, 3 per CU) on separately allocated client tensors
// (scripts/segments_probe.py --model, profiles/r03/seg/models.jsonl): flat
// 100 x 25M 1.580 -> 1.444 ms (6,393 -> 6,996 GB/s), resnet18_gn x 500
// (62 keys) 3.683 -> 3.285 ms, resnet56 x 100 (small units, 8 per CU)
// 101.8 -> 94.6 us, FEMNIST x 10 17.4 -> 17.2 us; 3 per CU 1.479 ms, 4 loads
// in flight 1.498 ms, 64 KiB units (U2 x C16, 1 per CU) 1.473 ms.
constexpr int kSegStyle = 2;
constexpr int kSegBlocksPerCU = 2;
// Small models (fewer than 4 units of 4,096 columns per CU): units of 1,024
// columns (U4 x C1), up to 8 blocks per CU per launch -- 4x the workgroups.
// rocprofv3 kernel time per call (scripts/segments_probe.py --model,
// profiles/r02/sweeps/segments_small_models.json): resnet56 x 100 (350 keys)
// 90.0 -> 77.1 us, FEMNIST x 10 12.1 -> 10.9 us, MNIST-LR x 10 6.3 -> 4.3 us;
// the flat 25M key stays on C4 (1,577 vs 1,717 us at C1).
constexpr int kSegSmallC = 1;
constexpr int kSegSmallBlocksPerCU = 8;
constexpr int64_t kSegSmallUnitsPerCU = 4;
constexpr int64_t kSegSmallSpan = static_cast<int64_t>(kBlock) * kSegSmallC * 4;
// :291 on device-resident clients: U4 client rows per load batch; units of
// 8,192 columns (C8), or the small-model units of 1,024 (C1).  rocprofv3
// kernel time (scripts/segments_dist_probe.py, profiles/r02/sweeps/
// segments_dist.json): flat 100 x 25M 1,638 us at U4 x C8 vs 1,656 for the
// round-1 form (one client at a time, C4) and 1,681 at U4 x C4; resnet56 x 100
// 84.5 us at U4 x C1 vs 100.8 (one client at a time, C4); FEMNIST 13.8 vs 14.5.
constexpr int kSegDistU = 4;
constexpr int kSegDistC = 8;
constexpr int64_t kSegDistSpan = static_cast<int64_t>(kBlock) * kSegDistC * 4;
constexpr int64_t kSegSpanMaxBytes = static_cast<int64_t>(kBlock) * 16 * 16;  // widest unit (C = 16), bytes


// the key owning unit u (keys without units share their successor's start
// and lose the tie)
__device__ __forceinline__ int64_t find_key(const SegKey* __restrict__ keys, int64_t n_keys, int64_t u) {
  return wave_search_last_le([&](int64_t x) { return keys[x].unit_start; }, n_keys, u);
}

// Client addresses come from the pointer table as integers, so the compiler
// cannot infer their address space and would emit flat loads (which also
// count against lgkmcnt and stall the scalar pointer-table loads): every
// client access goes through an explicit global (address_space 1) pointer.
template <typename T>
using gptr = __attribute__((address_space(1))) const T*;

template <typename T>
__device__ __forceinline__ gptr<T> to_global(const void* p) {
  return (gptr<T>)(reinterpret_cast<uintptr_t>(p));
}

__device__ __forceinline__ f32x4 ldu(const float* p) { return __builtin_nontemporal_load(to_global<f32x4_a4>(p)); }

// Full units read through a buffer descriptor per client: the wave-uniform
// base (client pointer + unit start) goes to SGPRs via readfirstlane and each
// lane's slice is a 32-bit voffset shared by every client, so a load costs no
// 64-bit VGPR address (with plain global pointers the compiler hoists the
// loop-invariant part into one 64-bit VGPR pair per (client, slice) load,
// which caps the loads it keeps in flight).  aux 2 = nt, as ldu().
__device__ __forceinline__ __amdgpu_buffer_rsrc_t unit_rsrc(const float* unit_base) {
  return uniform_rsrc(unit_base, static_cast<int>(kSegSpanMaxBytes));
}

__device__ __forceinline__ f32x4 ldb(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) { return ld_rsrc_nt(r, byte_off); }

// elements [col, col + 4) of a unit with n columns: a full 16-B vector, or
// the valid head of one (the rest 0)
__device__ __forceinline__ f32x4 load_slice(const float* p, int64_t col, int64_t n) {
  if (col + 4 <= n) return ldu(p + col);
  const gptr<float> q = to_global<float>(p);
  f32x4 v{0.f, 0.f, 0.f, 0.f};
  if (col < n) v.x = q[col];
  if (col + 1 < n) v.y = q[col + 1];
  if (col + 2 < n) v.z = q[col + 2];
  return v;
}

__device__ __forceinline__ void store_slice_u(float* o, int64_t col, int64_t n, f32x4 a) {
  if (col + 4 <= n) {
    *reinterpret_cast<f32x4_a4*>(o + col) = a;
  } else if (col < n) {
    o[col] = a.x;
    if (col + 1 < n) o[col + 1] = a.y;
    if (col + 2 < n) o[col + 2] = a.z;
  }
}

__device__ __forceinline__ float load_cvt(const void* base, int64_t kind, int64_t e) {
  switch (kind) {
    case kI64: return static_cast<float>(to_global<int64_t>(base)[e]);
    case kI32: return static_cast<float>(to_global<int32_t>(base)[e]);
    case kI16: return static_cast<float>(to_global<int16_t>(base)[e]);
    case kI8: return static_cast<float>(to_global<int8_t>(base)[e]);
    case kU8: return static_cast<float>(to_global<uint8_t>(base)[e]);
    case kBool: return to_global<uint8_t>(base)[e] ? 1.0f : 0.0f;
    default: return to_global<float>(base)[e];
  }
}

// one unit of an fp32 key: FULL units (all kSegSpan columns) take the
// unconditional 16-B path with U rows per batch; the last unit of a key
// masks its tail slice element by element
// STYLE 1: the row reduce's loop shape (reduce_f32x4_buf_kernel): each
// batch's client addresses read from the table as the batch starts, the
// batch's loads then consume_batch -- the compiler interleaves loads and
// products as it does there (probe variants)
template <int U, int C, bool FULL, int STYLE = 0>
__device__ __forceinline__ void reduce_raw_unit(const int64_t* __restrict__ P, int K, int64_t c0, int64_t n,
                                                const float* __restrict__ W, float* __restrict__ o) {
  f32x4 acc[C];
  uint32_t off[C];  // byte offsets of this lane's slices inside the unit
#pragma unroll
  for (int s = 0; s < C; ++s) off[s] = 16u * (threadIdx.x + s * kBlock);
  const float w0 = W[0];
  const float* x0 = reinterpret_cast<const float*>(P[0]) + c0;
#pragma unroll
  for (int s = 0; s < C; ++s) {
    const int64_t col = 4 * (threadIdx.x + s * kBlock);
    acc[s] = (FULL ? ldb(unit_rsrc(x0), off[s]) : load_slice(x0, col, n)) * w0;  // :455, i == 0
  }
  const int nb = (K - 1) / U;
  int k = 1;
  if constexpr (FULL && STYLE >= 2) {
    // STYLE 2/3/4: loads and products interleaved in (row, slice) order with
    // at most L = 2/4/8 loads of this wave in flight (sched_barrier keeps the
    // compiler from hoisting the batch's loads into one burst)
    constexpr int L = STYLE == 2 ? 2 : (STYLE == 3 ? 4 : 8);
    constexpr int N = U * C;
    for (int b = 0; b < nb; ++b, k += U) {
      __amdgpu_buffer_rsrc_t rr[U];
      float w[U];
#pragma unroll
      for (int r = 0; r < U; ++r) {
        rr[r] = unit_rsrc(reinterpret_cast<const float*>(P[k + r]) + c0);
        w[r] = W[k + r];
      }
      f32x4 x[N];
#pragma unroll
      for (int i = 0; i < N + L; ++i) {
        if (i < N) x[i] = ldb(rr[i / C], off[i % C]);
        if (i >= L) {
          const int j = i - L;
          const f32x4 term = x[j] * w[j / C];
          acc[j % C] = acc[j % C] + term;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    for (; k < K; ++k) {
      const __amdgpu_buffer_rsrc_t rr = unit_rsrc(reinterpret_cast<const float*>(P[k]) + c0);
      const float w = W[k];
#pragma unroll
      for (int s = 0; s < C; ++s) {
        const f32x4 term = ldb(rr, off[s]) * w;
        acc[s] = acc[s] + term;
      }
    }
#pragma unroll
    for (int s = 0; s < C; ++s) *reinterpret_cast<f32x4_a4*>(o + 4 * (threadIdx.x + s * kBlock)) = acc[s];
    return;
  }
  if constexpr (FULL && STYLE == 1) {
    for (int b = 0; b < nb; ++b, k += U) {
      f32x4 xs[U][C];
#pragma unroll
      for (int r = 0; r < U; ++r) {
        const __amdgpu_buffer_rsrc_t rr = unit_rsrc(reinterpret_cast<const float*>(P[k + r]) + c0);
#pragma unroll
        for (int s = 0; s < C; ++s) xs[r][s] = ldb(rr, off[s]);
      }
      consume_batch<U, C>(acc, xs, W, k);
    }
    for (; k < K; ++k) {
      const __amdgpu_buffer_rsrc_t rr = unit_rsrc(reinterpret_cast<const float*>(P[k]) + c0);
      const float w = W[k];
#pragma unroll
      for (int s = 0; s < C; ++s) {
        const f32x4 term = ldb(rr, off[s]) * w;
        acc[s] = acc[s] + term;
      }
    }
#pragma unroll
    for (int s = 0; s < C; ++s) *reinterpret_cast<f32x4_a4*>(o + 4 * (threadIdx.x + s * kBlock)) = acc[s];
    return;
  }
  // the next batch's client addresses are loaded one batch ahead, so the
  // pointer-table latency overlaps the current batch's data loads
  int64_t nxt[U];
#pragma unroll
  for (int r = 0; r < U; ++r) nxt[r] = nb > 0 ? P[1 + r] : 0;
  for (int b = 0; b < nb; ++b, k += U) {
    int64_t cur[U];
#pragma unroll
    for (int r = 0; r < U; ++r) cur[r] = nxt[r];
    if (b + 1 < nb) {
#pragma unroll
      for (int r = 0; r < U; ++r) nxt[r] = P[k + U + r];
    }
    f32x4 xs[U][C];
#pragma unroll
    for (int r = 0; r < U; ++r) {
      const float* xr = reinterpret_cast<const float*>(cur[r]) + c0;
      if constexpr (FULL) {
        const __amdgpu_buffer_rsrc_t rr = unit_rsrc(xr);
#pragma unroll
        for (int s = 0; s < C; ++s) xs[r][s] = ldb(rr, off[s]);
      } else {
#pragma unroll
        for (int s = 0; s < C; ++s) xs[r][s] = load_slice(xr, 4 * (threadIdx.x + s * kBlock), n);
      }
    }
#pragma unroll
    for (int r = 0; r < U; ++r) {
      const float w = W[k + r];
#pragma unroll
      for (int s = 0; s < C; ++s) {
        const f32x4 term = xs[r][s] * w;  // :455 product, then the :457 sum, in client order
        acc[s] = acc[s] + term;
      }
    }
  }
  for (; k < K; ++k) {
    const float* xr = reinterpret_cast<const float*>(P[k]) + c0;
    const float w = W[k];
#pragma unroll
    for (int s = 0; s < C; ++s) {
      const int64_t col = 4 * (threadIdx.x + s * kBlock);
      const f32x4 term = (FULL ? ldb(unit_rsrc(xr), off[s]) : load_slice(xr, col, n)) * w;
      acc[s] = acc[s] + term;
    }
  }
#pragma unroll
  for (int s = 0; s < C; ++s) {
    const int64_t col = 4 * (threadIdx.x + s * kBlock);
    if (FULL)
      *reinterpret_cast<f32x4_a4*>(o + col) = acc[s];
    else
      store_slice_u(o, col, n, acc[s]);
  }
}

template <int U, int C, int STYLE = 0>
__global__ __launch_bounds__(kBlock) void reduce_segments_f32_kernel(const SegKey* __restrict__ keys,
                                                                     const int64_t* __restrict__ ptrs, int64_t n_keys,
                                                                     int64_t unit0, int K, const float* __restrict__ W,
                                                                     float* __restrict__ out) {
  constexpr int64_t span = static_cast<int64_t>(kBlock) * C * 4;  // columns per unit
  const int64_t u = unit0 + blockIdx.x;
  const int64_t j = find_key(keys, n_keys, u);
  const SegKey key = keys[j];
  const int64_t c0 = (u - key.unit_start) * span;
  const int64_t n = key.numel - c0 < span ? key.numel - c0 : span;
  const int64_t* P = ptrs + j * K;
  float* o = out + key.out_offset + c0;
  if (key.kind == kRaw) {
    if (n == span)
      reduce_raw_unit<U, C, true, STYLE>(P, K, c0, n, W, o);
    else
      reduce_raw_unit<1, C, false>(P, K, c0, n, W, o);
    return;
  }
  // integer / bool key: element by element, converted like the packers
  constexpr int kPer = 4 * C;
  float acc[kPer];
  const float w0 = W[0];
  const void* x0 = reinterpret_cast<const void*>(P[0]);
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int64_t e = threadIdx.x + static_cast<int64_t>(i) * kBlock;
    acc[i] = e < n ? load_cvt(x0, key.kind, c0 + e) * w0 : 0.f;
  }
  for (int k = 1; k < K; ++k) {
    const void* xk = reinterpret_cast<const void*>(P[k]);
    const float w = W[k];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int64_t e = threadIdx.x + static_cast<int64_t>(i) * kBlock;
      if (e < n) {
        const float term = load_cvt(xk, key.kind, c0 + e) * w;
        acc[i] = acc[i] + term;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int64_t e = threadIdx.x + static_cast<int64_t>(i) * kBlock;
    if (e < n) o[e] = acc[i];
  }
}

// fedavg_reduce_ptrs_f32: one key of P columns whose client addresses are
// already a device array [K] -- the same units, no table staging
template <int U, int C, int STYLE = kSegStyle>
__global__ __launch_bounds__(kBlock) void reduce_ptrs_f32_kernel(const int64_t* __restrict__ ptrs, int64_t P,
                                                                 int64_t unit0, int K, const float* __restrict__ W,
                                                                 float* __restrict__ out) {
  constexpr int64_t span = static_cast<int64_t>(kBlock) * C * 4;
  const int64_t c0 = (unit0 + blockIdx.x) * span;
  const int64_t n = P - c0 < span ? P - c0 : span;
  if (n == span)
    reduce_raw_unit<U, C, true, STYLE>(ptrs, K, c0, n, W, out + c0);
  else
    reduce_raw_unit<1, C, false>(ptrs, K, c0, n, W, out + c0);
}

__device__ __forceinline__ double sq4_add(double acc, f32x4 d) {
  const double x = d.x, y = d.y, z = d.z, w = d.w;
  acc = __builtin_fma(x, x, acc);
  acc = __builtin_fma(y, y, acc);
  acc = __builtin_fma(z, z, acc);
  return __builtin_fma(w, w, acc);
}

// one fp32 unit of :291 for U client rows per batch: the unit's model slice
// stays in registers, each batch loads U rows x C slices before any square is
// summed (full units through one buffer descriptor per client, the key's last
// unit masked), and every row's wave sum goes through DPP lane moves
template <int U, int C, bool FULL>
__device__ __forceinline__ void sqdist_raw_unit(const int64_t* __restrict__ P, int K, int64_t c0, int64_t n,
                                                const float* __restrict__ g, double* __restrict__ partials,
                                                int64_t nparts, int64_t part) {
  uint32_t off[C];
#pragma unroll
  for (int s = 0; s < C; ++s) off[s] = 16u * (threadIdx.x + s * kBlock);
  f32x4 gv[C];
#pragma unroll
  for (int s = 0; s < C; ++s) gv[s] = load_slice(g, 4 * (threadIdx.x + s * kBlock), n);
  const bool lane0 = (threadIdx.x & 63u) == 0;
  int k = 0;
  for (; k + U <= K; k += U) {
    f32x4 xs[U][C];
#pragma unroll
    for (int r = 0; r < U; ++r) {
      const float* xr = reinterpret_cast<const float*>(P[k + r]) + c0;
      if constexpr (FULL) {
        const __amdgpu_buffer_rsrc_t rr = unit_rsrc(xr);
#pragma unroll
        for (int s = 0; s < C; ++s) xs[r][s] = ldb(rr, off[s]);
      } else {
#pragma unroll
        for (int s = 0; s < C; ++s) xs[r][s] = load_slice(xr, 4 * (threadIdx.x + s * kBlock), n);
      }
    }
#pragma unroll
    for (int r = 0; r < U; ++r) {
      double acc = 0.0;
#pragma unroll
      for (int s = 0; s < C; ++s) acc = sq4_add(acc, xs[r][s] - gv[s]);  // fp32 difference, as the reference
      acc = wave_sum_dpp(acc);
      if (lane0) partials[static_cast<int64_t>(k + r) * nparts + part] = acc;
    }
  }
  for (; k < K; ++k) {
    const float* xk = reinterpret_cast<const float*>(P[k]) + c0;
    double acc = 0.0;
#pragma unroll
    for (int s = 0; s < C; ++s) acc = sq4_add(acc, load_slice(xk, 4 * (threadIdx.x + s * kBlock), n) - gv[s]);
    acc = wave_sum_dpp(acc);
    if (lane0) partials[static_cast<int64_t>(k) * nparts + part] = acc;
  }
}

// :291 on the same units: per client, sum over the unit's columns of
// fl32(x - g)^2 in fp64 (fused square-adds, as client_sqdist_f32x4_kernel),
// one partial per wave: partials[k][unit * 4 + wave].  Lanes past the unit's
// end contribute exactly 0 (x and g both read as 0 there).  Units are
// kBlock x C x 4 columns (the same table staging as the reduce with that span).
template <int U, int C>
__global__ __launch_bounds__(kBlock) void sqdist_segments_f32_kernel(const SegKey* __restrict__ keys,
                                                                     const int64_t* __restrict__ ptrs, int64_t n_keys,
                                                                     int64_t unit0, int K, const float* __restrict__ G,
                                                                     double* __restrict__ partials, int64_t nparts) {
  constexpr int64_t span = static_cast<int64_t>(kBlock) * C * 4;
  const int64_t u = unit0 + blockIdx.x;
  const int64_t j = find_key(keys, n_keys, u);
  const SegKey key = keys[j];
  const int64_t c0 = (u - key.unit_start) * span;
  const int64_t n = key.numel - c0 < span ? key.numel - c0 : span;
  const int64_t* P = ptrs + j * K;
  const float* g = G + key.out_offset + c0;
  const int64_t part = u * (kBlock / 64) + (threadIdx.x >> 6);
  if (key.kind == kRaw) {
    if (n == span)
      sqdist_raw_unit<U, C, true>(P, K, c0, n, g, partials, nparts, part);
    else
      sqdist_raw_unit<1, C, false>(P, K, c0, n, g, partials, nparts, part);
    return;
  }
  constexpr int kPer = 4 * C;
  const bool lane0 = (threadIdx.x & 63u) == 0;
  for (int k = 0; k < K; ++k) {
    const void* xk = reinterpret_cast<const void*>(P[k]);
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int64_t e = threadIdx.x + static_cast<int64_t>(i) * kBlock;
      if (e < n) {
        const double d = static_cast<double>(load_cvt(xk, key.kind, c0 + e) - g[e]);  // fp32 difference
        acc = __builtin_fma(d, d, acc);
      }
    }
    acc = wave_sum_dpp(acc);
    if (lane0) partials[static_cast<int64_t>(k) * nparts + part] = acc;
  }
}

// sumsq[k] = sum of partials[k][*] in a fixed order (one workgroup per client)
__global__ __launch_bounds__(kBlock) void segments_finalize_kernel(const double* __restrict__ partials, int64_t nparts,
                                                                   double* __restrict__ sumsq) {
  __shared__ double red[kBlock];
  const int64_t k = blockIdx.x;
  double s = 0.0;
  for (int64_t w = threadIdx.x; w < nparts; w += kBlock) s += partials[k * nparts + w];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = kBlock / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) sumsq[k] = red[0];
}

// Aggregate + :291 in ONE pass over device-resident clients' own tensors
// (fedavg_dist.hip's fused tiles on the key/pointer tables): a unit is S
// columns of one key x all K clients, staged in LDS -- full 16-B slices of
// fp32 keys by LDS-DMA straight from each client's tensor (16-B aligned
// sources: the host checks), the key's ragged last slice and integer/bool
// keys element by element (converted like the packers) -- then the
// reference's sequential average of each column and the per-row squares.
// The running workgroup keeps its rows' client addresses of the current key
// in registers (reloaded at a key change only).  K <= 256.
constexpr int kSegFusedRowsPerThread = 8;  // ceil(K * S / 4 / 256) slots per thread at K <= 128, S <= 64 ... 256

// MAP (round 4): `umap` maps every unit to its key (staged with the tables),
// and the NEXT unit's key and client addresses are fetched while this unit's
// loads are in flight -- the key by scalar loads, the addresses behind the
// tile's LDS-DMA, so both have arrived at the tile's barrier.  Without it a
// unit waits for a wave-wide search over the key table (two rounds of vector
// loads at 350 keys) and, at a key change, for its client addresses before
// its data loads can start: four dependent latencies per tile, and a small
// model's tiles change key almost every time.
// LADDR (round 5, with MAP): the current key's K client addresses live in
// LDS (after the tile and its average) instead of 8 + 8 int64 registers per
// thread (this slot's row address and the next key's): each slot reads its
// row's address with one ds_read_b64 when it issues the tile's loads, and at
// a key change threads 0..K-1 load the next key's addresses behind the tile's
// loads and write them to LDS after the tile's load barrier (every slot has
// read the old ones by then).  114 -> ~80 VGPRs: 6 workgroups per CU (the
// LDS bound, as the rows kernel's tiles) instead of 4.
template <int S, bool MAP = false, bool LADDR = false>
__global__ __launch_bounds__(kBlock, LADDR && S != 32 ? 6 : 1) void reduce_sqdist_segments_f32_kernel(const SegKey* __restrict__ keys,
                                                                            const int64_t* __restrict__ ptrs,
                                                                            int64_t n_keys, int64_t units, int K,
                                                                            const float* __restrict__ W,
                                                                            float* __restrict__ out,
                                                                            double* __restrict__ partials,
                                                                            const int* __restrict__ umap) {
  constexpr int V = S / 4;
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [K][S] swizzled tile, then the average [S]
  float* tile = lds;
  float* gs = lds + K * S;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nload = K * V;
  double acc[1][4] = {{0.0, 0.0, 0.0, 0.0}};
  int64_t cur_key = -1;
  int64_t src[kSegFusedRowsPerThread];  // client address of the row of this thread's m-th load slot
  const auto load_src = [&](const int64_t* P, int64_t (&d)[kSegFusedRowsPerThread]) __attribute__((always_inline)) {
#pragma unroll
    for (int m = 0; m < kSegFusedRowsPerThread; ++m) {
      const int i = wave * 64 + m * kBlock + lane;
      d[m] = i < nload ? P[i / V] : 0;
    }
  };
  int64_t u = blockIdx.x;
  int64_t j = 0;
  SegKey key{};
  static_assert(!LADDR || MAP, "LDS addresses come with the unit map");
  int64_t* addr = reinterpret_cast<int64_t*>(gs + S);  // LADDR: [K] client addresses of the current key
  if constexpr (MAP) {
    if (u < units) {
      j = umap[u];
      key = keys[j];
      if (key.kind == kRaw) {
        if constexpr (LADDR) {
          if (threadIdx.x < K) addr[threadIdx.x] = ptrs[j * K + threadIdx.x];
          __syncthreads();
        } else {
          load_src(ptrs + j * K, src);
        }
        cur_key = j;
      }
    }
  }
  for (; u < units; u += gridDim.x) {
    if constexpr (!MAP) {
      j = find_key(keys, n_keys, u);
      key = keys[j];
    }
    const int64_t c0 = (u - key.unit_start) * S;
    const int n = key.numel - c0 < S ? static_cast<int>(key.numel - c0) : S;
    const int64_t* P = ptrs + j * K;
    if (key.kind == kRaw) {
      if constexpr (!MAP) {
        if (j != cur_key) {
          cur_key = j;
          load_src(P, src);
        }
      }
      const int nfull = n >> 2;  // whole 16-B slices of this unit
      // LADDR: every slot's row address is read from LDS BEFORE the first
      // LDS-DMA is issued -- a ds_read after one would wait for it to land
      // (the compiler cannot tell the address block from the tile's bytes),
      // which serialised the slots (round 5: 71 us against the rows kernel's
      // 49 on the same bytes, SQ_WAIT_ANY 1.7x)
      int64_t base[kSegFusedRowsPerThread];
#pragma unroll
      for (int m = 0; m < kSegFusedRowsPerThread; ++m) {
        const int i = wave * 64 + m * kBlock + lane;
        base[m] = LADDR ? (i < nload ? addr[i / V] : 0) : src[m];
      }
#pragma unroll
      for (int m = 0; m < kSegFusedRowsPerThread; ++m) {
        const int i0 = wave * 64 + m * kBlock;
        const int i = i0 + lane;
        const int row = i / V;
        const int c = (i % V) ^ (row & 7);
        if (i0 < nload && i < nload && c < nfull)
          __builtin_amdgcn_global_load_lds((fused_gbl_t)(reinterpret_cast<const float*>(base[m]) + c0 + 4 * c),
                                           (fused_lds_t)(tile + 4 * i0), 16, 0, 2 /* nt */);
      }
      if (n & 3) {  // the key's ragged last slice, element by element (never past the tensor's end)
        for (int row = threadIdx.x; row < K; row += kBlock) {
          const gptr<float> x = to_global<float>(reinterpret_cast<const void*>(LADDR ? addr[row] : P[row]));
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int col = 4 * nfull + e;
            tile[fused_at<S>(row, col)] = col < n ? x[c0 + col] : 0.f;
          }
        }
      }
    } else {  // integer / bool key: converted element by element, as the packers do
      for (int idx = threadIdx.x; idx < K * S; idx += kBlock) {
        const int row = idx / S, col = idx % S;
        tile[fused_at<S>(row, col)] = col < n ? load_cvt(reinterpret_cast<const void*>(P[row]), key.kind, c0 + col) : 0.f;
      }
    }
    // MAP: the next unit's key (scalar loads) and, at a key change, its
    // client addresses (behind this tile's loads): in hand at the barrier
    int64_t jn = j;
    SegKey keyn = key;
    bool fresh = false;
    int64_t srcn[LADDR ? 1 : kSegFusedRowsPerThread];
    int64_t addr_next = 0;
    if constexpr (MAP) {
      const int64_t un = u + gridDim.x;
      if (un < units) {
        jn = umap[un];
        keyn = keys[jn];
        if (keyn.kind == kRaw && jn != cur_key) {
          if constexpr (LADDR) {
            if (threadIdx.x < K) addr_next = ptrs[jn * K + threadIdx.x];
          } else {
            load_src(ptrs + jn * K, srcn);
          }
          fresh = true;
        }
      }
    }
    barrier_loads();
    if constexpr (LADDR) {  // every slot has read this key's addresses: the next key's replace them
      if (fresh && threadIdx.x < K) addr[threadIdx.x] = addr_next;
    }
    fused_average<S>(tile, gs, K, W, n, out + key.out_offset + c0);
    barrier_lds();
    fused_squares<S, 1, true>(tile, gs, K, n, acc);  // full tiles unmasked (same VGPRs, round 4)
    barrier_lds();  // the tile is read out before the next one lands
    if constexpr (MAP) {
      j = jn;
      key = keyn;
      if (fresh) {
        if constexpr (!LADDR) {
#pragma unroll
          for (int m = 0; m < kSegFusedRowsPerThread; ++m) src[m] = srcn[m];
        }
        cur_key = jn;
      }
    }
  }
  fused_finish(lds, acc, K, partials);
}

// ---------------------------------------------------------------------------
// Zero-copy wave-owned windows (round 3): fedavg_dist.hip's
// reduce_sqdist_win_kernel on the key / pointer tables.  Each key is cut
// into windows of WC = 64 x VEC columns (stage_tables with that span); a
// wave holds one window of all K clients in registers, runs the reference's
// chain per lane, squares fl32(x - g) in fp64 and folds 8 rows at a time
// across the wave (common.hpp).
//   fast window (fp32 key, all WC columns): one SGPR buffer descriptor per
//     client; row i's registers are reloaded from the NEXT fast window's
//     client i right after row i is squared (its 8-row group's client
//     addresses come from the pointer table by scalar loads one group ahead);
//   slow window (a key's ragged last window): loaded after the squares by
//     one dword buffer load per element through a descriptor ranged to the
//     key, columns past it 0.
// fp32 keys only (the host checks): a model's integer / bool keys
// (BatchNorm's num_batches_tracked) are converted to fp32 columns on the
// device first and passed as fp32 keys (aggregate.py, round 4).
// The next window's key comes from a scalar scan forward from the current
// one (a wave's windows only move forward), so no vector load besides the
// rows is in flight in the loop.  Rows K..KMAX-1 are padding: empty
// descriptors (0, no traffic) or 0, weight -0.0, sums never written.  The
// pointer table is padded by kSegWinTablePad entries so every group's 8
// addresses load unconditionally (a padding row's is never dereferenced).
// ---------------------------------------------------------------------------
constexpr int64_t kSegWinMinPerWave = 16;  // windows per wave below which the LDS-DMA tiles keep the round

// DESC (round 5): every fast window's K client descriptors come from a
// descriptor table staged with the key table -- desc[j * KMAX + i] = {client
// i's address of key j (lo, hi), the key's byte length (0 for padding rows
// and empty keys), the buffer flags} -- by scalar loads from the constant
// address space (one s_load_dwordx16 per 4 rows), used in place as the row's
// buffer resource with the window's start in soffset.  The per-row
// v_readlane pair and the descriptor's SALU assembly (record count select,
// flags, mask) of the pointer form -- ~6 of a row's ~20 instructions per
// window -- are gone.  A window whose next one is ragged (or past the end)
// reloads from desc[n_keys * KMAX ..], KMAX null descriptors (record count
// 0: the loads return 0 and touch nothing), and the ragged window is loaded
// after the squares from the pointer table as before.
typedef __attribute__((address_space(4))) const u32x4* cdesc_t;

template <int KMAX, int VEC, int NW, bool DESC = false, int MINW = win_min_waves(KMAX, VEC)>
__global__ __launch_bounds__(64 * NW, MINW) void reduce_sqdist_segwin_kernel(
    const SegKey* __restrict__ keys, const int64_t* __restrict__ ptrs, int64_t n_keys, int64_t units, int K,
    const float* __restrict__ W, float* __restrict__ out, double* __restrict__ partials,
    const u32x4* __restrict__ desc) {
  typedef typename WinVec<VEC>::T V;
  constexpr int WC = 64 * VEC;
  constexpr int NB = (KMAX + 7) / 8;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t GW = static_cast<int64_t>(gridDim.x) * NW;
  const int64_t gw = static_cast<int64_t>(blockIdx.x) * NW + wv;
  const uint32_t voff = static_cast<uint32_t>(lane) * VEC * 4;
  const bool upper = (lane & 8) != 0;
  __shared__ __attribute__((aligned(16))) float wl[(KMAX + 3) & ~3];
  __shared__ double accl[NW][NB][64];
  for (int i = threadIdx.x; i < ((KMAX + 3) & ~3); i += 64 * NW) wl[i] = i < K ? W[i] : -0.0f;
  double* acc = &accl[wv][0][lane];
#pragma unroll
  for (int b = 0; b < NB; ++b) acc[64 * b] = 0.0;
  __syncthreads();

  V x[KMAX];
  // A window's K client addresses arrive as one vector load per 64 clients
  // (lane l: clients l and 64 + l), issued before the chain that precedes
  // their use -- the chain has waited for every older load by then -- and
  // row i reads its address with v_readlane (an SGPR pair: the descriptor
  // stays uniform).  Scalar loads would be hoisted for all KMAX rows at once.
  int64_t pv[2];
  const auto load_ptrs = [&](const int64_t* P) __attribute__((always_inline)) {
    const gptr<int64_t> q = to_global<int64_t>(P);
    pv[0] = q[lane];
    if constexpr (KMAX > 64) pv[1] = q[64 + lane];
  };
  const auto ptr_of = [&](int i) __attribute__((always_inline)) {
    const int64_t v = pv[i >> 6];
    int li = i & 63;
    asm volatile("" : "+s"(li));  // read where it is used: the KMAX addresses would not fit the SGPRs
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), li);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(static_cast<uint64_t>(v) >> 32), li);
    return reinterpret_cast<const float*>((static_cast<uint64_t>(hi) << 32) | lo);
  };
  // a slow window (a key's ragged last window) into x: one dword buffer load
  // per element through a descriptor whose range is that client's part of
  // the window (columns past the key read 0, nothing past it is touched).
  // No per-lane 64-bit address: the global-pointer form of this path held one
  // per row and made the 100-row instance spill.
  const auto load_slow = [&](int64_t c0, int n, int Kw) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
      const float* base = ptr_of(i) + c0;
      const __amdgpu_buffer_rsrc_t r =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, i < Kw ? n * 4 : 0, 0x00020000);
#pragma unroll
      for (int v = 0; v < VEC; ++v)
        x[i][v] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (lane * VEC + v) * 4, 0, 2));
    }
  };
  // client i of a fast window: the client's own address is the descriptor's
  // base and the window's start goes in soffset (one SGPR per window instead
  // of a 64-bit add per row); the range check covers soffset + voffset, so
  // the record count is the window's end byte -- 0 for padding rows (i >= Kw)
  // (the host keeps every key of a window plan under 2^30 elements)
  const auto load_fast = [&](int i, uint32_t soff, uint32_t nrec, int Kw) __attribute__((always_inline)) {
    x[i] = win_load<VEC>(
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ptr_of(i)), 0, i < Kw ? static_cast<int>(nrec) : 0,
                                          0x00020000),
        voff, soff);
  };
  // DESC: row i of the window whose descriptors start at `cd`
  const auto load_desc = [&](cdesc_t cd, int i, uint32_t soff) __attribute__((always_inline)) {
    const u32x4 d = cd[i];
    x[i] = win_load<VEC>(
        __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((static_cast<uint64_t>(d.y) << 32) | d.x), 0,
                                          static_cast<int>(d.z), static_cast<int>(d.w)),
        voff, soff);
  };

  // window / key indices in 32 bits (the host checks units < 2^31): 64-bit
  // compares run on the VALU, and a descriptor built from a VALU result
  // would cost a waterfall loop per load
  const int units32 = static_cast<int>(units), nkeys32 = static_cast<int>(n_keys);
  const int GW32 = static_cast<int>(GW);
  // valid columns of window `w` of a key with `numel` elements (uniform)
  const auto cols_of = [&](int64_t numel, int w) __attribute__((always_inline)) {
    const int64_t left = numel - static_cast<int64_t>(w) * WC;
    return (left >> 31) != 0 ? WC : (static_cast<int>(left) < WC ? static_cast<int>(left) : WC);
  };
  int u = static_cast<int>(gw), j = 0, n = 0;
  int64_t c0 = 0;
  if (u < units32) {
    j = __builtin_amdgcn_readfirstlane(static_cast<int>(find_key(keys, n_keys, u)));  // wave-wide search, then scans
    const SegKey key = keys[j];
    const int w = u - static_cast<int>(key.unit_start);
    c0 = static_cast<int64_t>(w) * WC;
    n = cols_of(key.numel, w);
    if (!DESC || n != WC) load_ptrs(ptrs + static_cast<int64_t>(j) * K);  // DESC: slow windows only
    if (n == WC) {
      if constexpr (DESC) {
        const cdesc_t cd = (cdesc_t)(desc + static_cast<int64_t>(j) * KMAX);
#pragma unroll
        for (int i = 0; i < KMAX; ++i) {
          load_desc(cd, i, static_cast<uint32_t>(c0 * 4));
          if ((i & 7) == 7) __builtin_amdgcn_sched_barrier(0);
        }
      } else {
#pragma unroll
        for (int i = 0; i < KMAX; ++i)
          load_fast(i, static_cast<uint32_t>(c0 * 4), static_cast<uint32_t>((c0 + WC) * 4), K);
      }
    } else {
      load_slow(c0, n, K);
    }
  }
  // DESC: the current key's output offset and the next-window key's fields
  // are kept in SGPRs and reloaded only when the scan moves to another key
  // (next_start: the first window of the key after it), so a window of a
  // long key issues no scalar load of the key table and waits on none
  int64_t cur_out = 0, kn_numel = 0;
  int kn_start = 0, next_start = 0x7fffffff;
  if (DESC && u < units32) {
    const SegKey k0 = keys[j];
    cur_out = k0.out_offset;
    kn_numel = k0.numel;
    kn_start = static_cast<int>(k0.unit_start);
    next_start = j + 1 < nkeys32 ? static_cast<int>(keys[j + 1].unit_start) : 0x7fffffff;
  }
  for (; u < units32; u += GW32) {
    int Kw = K;
    asm volatile("" : "+s"(Kw));
    const int64_t out_off = DESC ? cur_out : keys[j].out_offset;
    // the next window: its key by a forward scan
    const int un = u + GW32;
    int jn = j, nn = 0;
    int64_t c0n = 0;
    int64_t kn_out = cur_out;
    if (un < units32) {
      if constexpr (DESC) {
        while (un >= next_start) {  // keys without windows share their successor's start
          ++jn;
          const SegKey kk = keys[jn];
          kn_numel = kk.numel;
          kn_start = static_cast<int>(kk.unit_start);
          kn_out = kk.out_offset;
          next_start = jn + 1 < nkeys32 ? static_cast<int>(keys[jn + 1].unit_start) : 0x7fffffff;
        }
        const int w = un - kn_start;
        c0n = static_cast<int64_t>(w) * WC;
        nn = cols_of(kn_numel, w);
      } else {
        while (jn + 1 < nkeys32 && static_cast<int>(keys[jn + 1].unit_start) <= un) ++jn;
        const SegKey kn = keys[jn];
        const int w = un - static_cast<int>(kn.unit_start);
        c0n = static_cast<int64_t>(w) * WC;
        nn = cols_of(kn.numel, w);
      }
    }
    const bool fastn = un < units32 && nn == WC;
    // the next fast window's soffset and record count; no loads unless it is fast
    const uint32_t soffn = static_cast<uint32_t>(c0n * 4), nrecn = static_cast<uint32_t>((c0n + WC) * 4);
    int Kwn = fastn ? K : 0;
    asm volatile("" : "+s"(Kwn));
    // DESC: the next window's descriptors, or the null block when it is not fast
    const cdesc_t cdn = (cdesc_t)(desc + (fastn ? static_cast<int64_t>(jn) : n_keys) * KMAX);
    // the next window's addresses, before the chain (DESC: a slow next window only)
    if (!DESC || (un < units32 && !fastn)) load_ptrs(ptrs + static_cast<int64_t>(jn) * K);
    // the chain (a slow window's columns past its key are 0)
    int wo = 0;
    asm volatile("" : "+v"(wo));
    V a;
#pragma unroll
    for (int q = 0; q < (KMAX + 3) / 4; ++q) {
      const f32x4 w4 = *reinterpret_cast<const f32x4*>(&wl[wo + 4 * q]);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int i = 4 * q + jj;
        if (i == 0) {
          a = x[0] * w4[0];
        } else if (i < KMAX) {
          const V t = x[i] * w4[jj];
          a = a + t;
        }
      }
    }
    float* o = out + out_off + c0 + lane * VEC;
    if (n == WC) {
      if constexpr (DESC)  // streamed out, as the rows kernel's output
        __builtin_nontemporal_store(static_cast<typename WinVec<VEC>::TA>(a),
                                    reinterpret_cast<typename WinVec<VEC>::TA*>(o));
      else
        *reinterpret_cast<typename WinVec<VEC>::TA*>(o) = a;  // o: only dword-aligned (key offsets)
    } else {
#pragma unroll
      for (int v = 0; v < VEC; ++v)
        if (lane * VEC + v < n) o[v] = a[v];
    }
    // squares; row i reloaded from the next window right after (a slow next
    // window: empty descriptors here, its element loads after the squares)
    if constexpr (DESC) {
      // a batch's 8 descriptors were loaded during the previous batch: the
      // batch finalises them (their one wait on the scalar loads), issues the
      // NEXT batch's descriptor loads, then squares and reloads its rows
      u32x4 dc[8], dn[8];
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if (r < KMAX) dc[r] = cdn[r];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        uint32_t hi[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) hi[r] = dc[r].y & 0xffffu;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = 0; r < 8; ++r)
          if (b + 1 < NB && 8 * (b + 1) + r < KMAX) dn[r] = cdn[8 * (b + 1) + r];
        __builtin_amdgcn_sched_barrier(0);
        double p[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int i = 8 * b + r;
          p[r] = 0.0;
          if (i < KMAX) {
            p[r] = win_sq<VEC>(x[i] - a);
            x[i] = win_load<VEC>(__builtin_amdgcn_make_buffer_rsrc(
                                     reinterpret_cast<void*>((static_cast<uint64_t>(hi[r]) << 32) | dc[r].x), 0,
                                     static_cast<int>(dc[r].z), static_cast<int>(dc[r].w)),
                                 voff, soffn);
          }
        }
        const double q01 = fold32(p[0], p[1]), q23 = fold32(p[2], p[3]);
        const double q45 = fold32(p[4], p[5]), q67 = fold32(p[6], p[7]);
        acc[64 * b] += fold8(fold16(q01, q23), fold16(q45, q67), upper);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = 0; r < 8; ++r) dc[r] = dn[r];
      }
    } else {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        double p[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int i = 8 * b + r;
          p[r] = 0.0;
          if (i < KMAX) {
            p[r] = win_sq<VEC>(x[i] - a);
            load_fast(i, soffn, nrecn, Kwn);
          }
        }
        const double q01 = fold32(p[0], p[1]), q23 = fold32(p[2], p[3]);
        const double q45 = fold32(p[4], p[5]), q67 = fold32(p[6], p[7]);
        acc[64 * b] += fold8(fold16(q01, q23), fold16(q45, q67), upper);
      }
    }
    if (un < units32 && !fastn) {
      // a fresh opaque K: with the squares' Kw the compiler kept their KMAX
      // row masks (i < Kw) alive for these loads -- 139 SGPRs spilled to
      // VGPR lanes, two v_writelane per row in the squares loop
      int Ks = K;
      asm volatile("" : "+s"(Ks));
      load_slow(c0n, nn, Ks);
    }
    j = jn;
    c0 = c0n;
    n = nn;
    cur_out = kn_out;
  }
  const int row_in = win_batch_row(lane);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    double sm = acc[64 * b];
    sm += dpp_move_f64<0xB1, 0xF>(sm);
    sm += dpp_move_f64<0x4E, 0xF>(sm);
    sm += dpp_move_f64<0x141, 0xF>(sm);
    const int row = 8 * b + row_in;
    if ((lane & 7) == 0 && row < K) partials[static_cast<int64_t>(row) * GW + gw] = sm;
  }
}

// Zero-copy split-row windows (round 5): fedavg_dist.hip's
// reduce_sqdist_winn_kernel on the key / pointer tables, for 257-1024
// device-resident clients (the tiles stop at 256).  A workgroup of ns =
// ceil(K / 64) waves owns a window of 64 columns of one key; wave h holds
// clients 64h .. 64h + 63 in registers, one dword per lane.  The chain runs
// wave by wave in client order, handed over LDS; the last wave stores the
// average, then every wave squares its rows against it and reloads them from
// the next window (its 64 client addresses: one vector load per wave, read
// per row with v_readlane, as the pointer form of the one-wave windows).  A
// key's ragged last window loads element by element through descriptors
// ranged to the key.  fp32 keys only (integer keys arrive as fp32 scratch).
// ---------------------------------------------------------------------------
template <int NSMAX>
__global__ __launch_bounds__(64 * NSMAX, win_min_waves(64, 1)) void reduce_sqdist_segwinn_kernel(
    const SegKey* __restrict__ keys, const int64_t* __restrict__ ptrs, int64_t n_keys, int64_t units, int K,
    const float* __restrict__ W, float* __restrict__ out, double* __restrict__ partials) {
  constexpr int KH = 64, WC = 64, NB = 8;
  const int lane = threadIdx.x & 63;
  const int h = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ns = __builtin_amdgcn_readfirstlane(static_cast<int>(blockDim.x >> 6));
  const int r0 = h * KH;
  const int G = static_cast<int>(gridDim.x);
  const uint32_t voff = static_cast<uint32_t>(lane) * 4;
  const bool upper = (lane & 8) != 0;
  __shared__ __attribute__((aligned(16))) float wl[NSMAX][KH];
  __shared__ double accl[NSMAX][NB][64];
  __shared__ float xa[64];
  for (int i = threadIdx.x; i < ns * KH; i += blockDim.x) wl[i / KH][i % KH] = i < K ? W[i] : -0.0f;
  double* acc = &accl[h][0][lane];
#pragma unroll
  for (int b = 0; b < NB; ++b) acc[64 * b] = 0.0;
  __syncthreads();

  float x[KH];
  int64_t pv = 0;  // lane l: client r0 + l's address of the window's key
  const auto load_ptrs = [&](const int64_t* P) __attribute__((always_inline)) {
    const gptr<int64_t> q = to_global<int64_t>(P);
    pv = r0 + lane < K ? q[r0 + lane] : 0;
  };
  const auto ptr_of = [&](int i) __attribute__((always_inline)) {
    int li = i;
    asm volatile("" : "+s"(li));
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(pv), li);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(static_cast<uint64_t>(pv) >> 32), li);
    return reinterpret_cast<const float*>((static_cast<uint64_t>(hi) << 32) | lo);
  };
  // a full window: the client's address as the base, the window's start in
  // soffset, the window's end byte as the record count (0: client >= K)
  const auto load_fast = [&](int i, uint32_t soff, uint32_t nrec, int Kw) __attribute__((always_inline)) {
    x[i] = __builtin_bit_cast(
        float, __builtin_amdgcn_raw_buffer_load_b32(
                   __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ptr_of(i)), 0,
                                                     r0 + i < Kw ? static_cast<int>(nrec) : 0, 0x00020000),
                   static_cast<int>(voff), static_cast<int>(soff), 2));
  };
  // a key's ragged last window: the descriptor's range is the client's part of it
  const auto load_slow = [&](int64_t c0, int n, int Kw) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < KH; ++i) {
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ptr_of(i) + c0), 0,
                                                                         r0 + i < Kw ? n * 4 : 0, 0x00020000);
      x[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, static_cast<int>(voff), 0, 2));
    }
  };
  const int units32 = static_cast<int>(units), nkeys32 = static_cast<int>(n_keys);
  const auto cols_of = [&](int64_t numel, int w) __attribute__((always_inline)) {
    const int64_t left = numel - static_cast<int64_t>(w) * WC;
    return (left >> 31) != 0 ? WC : (static_cast<int>(left) < WC ? static_cast<int>(left) : WC);
  };
  int u = static_cast<int>(blockIdx.x), j = 0, n = 0;
  int64_t c0 = 0;
  if (u < units32) {
    j = __builtin_amdgcn_readfirstlane(static_cast<int>(find_key(keys, n_keys, u)));
    const SegKey key = keys[j];
    const int w = u - static_cast<int>(key.unit_start);
    c0 = static_cast<int64_t>(w) * WC;
    n = cols_of(key.numel, w);
    load_ptrs(ptrs + static_cast<int64_t>(j) * K);
    if (n == WC) {
#pragma unroll
      for (int i = 0; i < KH; ++i) load_fast(i, static_cast<uint32_t>(c0 * 4), static_cast<uint32_t>((c0 + WC) * 4), K);
    } else {
      load_slow(c0, n, K);
    }
  }
  for (; u < units32; u += G) {
    const int64_t out_off = keys[j].out_offset;
    const int un = u + G;
    int jn = j, nn = 0;
    int64_t c0n = 0;
    if (un < units32) {
      while (jn + 1 < nkeys32 && static_cast<int>(keys[jn + 1].unit_start) <= un) ++jn;
      const SegKey kn = keys[jn];
      const int w = un - static_cast<int>(kn.unit_start);
      c0n = static_cast<int64_t>(w) * WC;
      nn = cols_of(kn.numel, w);
    }
    const bool fastn = un < units32 && nn == WC;
    const uint32_t soffn = static_cast<uint32_t>(c0n * 4), nrecn = static_cast<uint32_t>((c0n + WC) * 4);
    int Kwn = fastn ? K : 0;
    asm volatile("" : "+s"(Kwn));
    if (un < units32) load_ptrs(ptrs + static_cast<int64_t>(jn) * K);  // this window's rows are loaded
    float a = 0.f;
    for (int st = 0; st < ns; ++st) {  // the chain, wave by wave in client order
      if (h == st) {
        int wo = h * KH;
        asm volatile("" : "+v"(wo));
        const float* wp = &wl[0][0] + wo;
        if (st > 0) a = xa[lane];
#pragma unroll
        for (int q = 0; q < KH / 4; ++q) {
          const f32x4 w4 = *reinterpret_cast<const f32x4*>(wp + 4 * q);
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int i = 4 * q + jj;
            if (st == 0 && i == 0) {
              a = x[0] * w4[0];
            } else {
              const float t = x[i] * w4[jj];
              a = a + t;
            }
          }
        }
        xa[lane] = a;
        if (st == ns - 1 && lane < n) out[out_off + c0 + lane] = a;
      }
      __syncthreads();
    }
    if (h != ns - 1) a = xa[lane];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      double p[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int i = 8 * b + r;
        const double d = static_cast<double>(x[i] - a);  // fp32 difference, as the reference forms it
        p[r] = d * d;
        load_fast(i, soffn, nrecn, Kwn);
      }
      const double q01 = fold32(p[0], p[1]), q23 = fold32(p[2], p[3]);
      const double q45 = fold32(p[4], p[5]), q67 = fold32(p[6], p[7]);
      acc[64 * b] += fold8(fold16(q01, q23), fold16(q45, q67), upper);
    }
    if (un < units32 && !fastn) {
      int Ks = K;
      asm volatile("" : "+s"(Ks));
      load_slow(c0n, nn, Ks);
    }
    __syncthreads();  // every wave has read xa before the next window's chain rewrites it
    j = jn;
    c0 = c0n;
    n = nn;
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

// Zero-copy split-row windows with point-to-point hand-offs (round 6): the
// segwinn work on fedavg_dist.hip's reduce_sqdist_winf_kernel protocol -- no
// workgroup barrier in the window loop (wave h > 0 takes wave h - 1's partial
// from LDS behind a flag, the last wave publishes the average behind another),
// a wave waits for its own rows at its turn, the weights come by row
// broadcast, the squares and reloads run at a priority by wave, and the first
// PF rows of the next window are in flight through the turn.  The client
// addresses of the window after next load at the start of the squares, ahead
// of the reloads, so the next prefetch waits on them with the reloads still in
// flight (vmcnt counts in issue order); the key table is read through the
// constant address space (scalar loads: the key walk never waits on vmcnt).
// Hand-off safety and the bounded polls: see the rows kernel.
// UNI: every row load takes the client's address + the window's first column
// as its base and the window's columns as its range, so a key's ragged last
// window loads through the same instructions as a full one (lanes past it
// read 0).  Without it a ragged window reloads every row again after the
// squares (round 5's form), and the compiler, merging the two load paths,
// waits for all of a wave's rows at the start of its turn.
template <int NSMAX, int PF, bool UNI = true, int MODE = 0>
__global__ __launch_bounds__(64 * NSMAX, win_min_waves(64, 1)) void reduce_sqdist_segwinf_kernel(
    const SegKey* __restrict__ keys, const int64_t* __restrict__ ptrs, int64_t n_keys, int64_t units, int K,
    const float* __restrict__ W, float* __restrict__ out, double* __restrict__ partials) {
  constexpr int KH = 64, WC = 64, NB = 8, NWV = 4;
  static_assert(PF >= 1 && PF <= KH, "prefetched rows");
  constexpr int kSpinMax = 1 << 20;  // tight polls, as the rows kernel's
  const int lane = threadIdx.x & 63;
  const int h = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ns = __builtin_amdgcn_readfirstlane(static_cast<int>(blockDim.x >> 6));
  const int r0 = h * KH;
  const int G = static_cast<int>(gridDim.x);
  const uint32_t voff = static_cast<uint32_t>(lane) * 4;
  const bool upper = (lane & 8) != 0;
  __shared__ double accl[NSMAX][NB][64];
  __shared__ float part[NSMAX][64];
  __shared__ float avg[64];
  __shared__ int flag[NSMAX + 1];
  uint64_t* const stamps = reinterpret_cast<uint64_t*>(partials + static_cast<int64_t>(K) * G);
  int wi = 0;
  const auto stamp = [&](int ph) __attribute__((always_inline)) {  // MODE 8: the rows kernel's timeline
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
  float wv[NWV];  // lane 16r + j of wv[k]: client 16k + j's weight (-0.0 past K)
#pragma unroll
  for (int k = 0; k < NWV; ++k) {
    const int row = r0 + 16 * k + (lane & 15);
    wv[k] = row < K ? W[row] : -0.0f;
  }
  __syncthreads();
  typedef __attribute__((address_space(3))) volatile int lds_flag_t;
  const auto wait_flag = [&](int idx, int seq) __attribute__((always_inline)) {
    lds_flag_t* f = (lds_flag_t*)&flag[idx];
    for (int it = 0; __builtin_amdgcn_readfirstlane(*f) != seq && it < kSpinMax; ++it) {
    }
    asm volatile("" ::: "memory");
  };
  const auto publish = [&](int idx, int seq) __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    *(lds_flag_t*)&flag[idx] = seq;
  };
  const auto load_ptrs = [&](const int64_t* P) __attribute__((always_inline)) -> int64_t {
    const gptr<int64_t> q = to_global<int64_t>(P);
    return r0 + lane < K ? q[r0 + lane] : 0;
  };
  const auto ptr_of = [&](int64_t pv, int i) __attribute__((always_inline)) {
    int li = i;
    asm volatile("" : "+s"(li));
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(pv), li);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(static_cast<uint64_t>(pv) >> 32), li);
    return reinterpret_cast<const float*>((static_cast<uint64_t>(hi) << 32) | lo);
  };
  const auto load_fast = [&](int64_t pv, int i, uint32_t soff, uint32_t nrec, int Kw) __attribute__((always_inline)) {
    return __builtin_bit_cast(
        float, __builtin_amdgcn_raw_buffer_load_b32(
                   __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ptr_of(pv, i)), 0,
                                                     r0 + i < Kw ? static_cast<int>(nrec) : 0, 0x00020000),
                   static_cast<int>(voff), static_cast<int>(soff), 2));
  };
  const auto load_row = [&](int64_t pv, int i, int64_t c0_, int n_, int Kw) __attribute__((always_inline)) {
    return __builtin_bit_cast(
        float, __builtin_amdgcn_raw_buffer_load_b32(
                   __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ptr_of(pv, i) + c0_), 0,
                                                     r0 + i < Kw ? n_ * 4 : 0, 0x00020000),
                   static_cast<int>(voff), 0, 2));
  };
  float x[KH];
  float xp[PF];
  const auto load_slow = [&](int64_t pv, int64_t c0, int n, int Kw) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < KH; ++i) {
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ptr_of(pv, i) + c0), 0,
                                                                         r0 + i < Kw ? n * 4 : 0, 0x00020000);
      x[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, static_cast<int>(voff), 0, 2));
    }
  };
  const int units32 = static_cast<int>(units), nkeys32 = static_cast<int>(n_keys);
  const auto cols_of = [&](int64_t numel, int w) __attribute__((always_inline)) {
    const int64_t left = numel - static_cast<int64_t>(w) * WC;
    return (left >> 31) != 0 ? WC : (static_cast<int>(left) < WC ? static_cast<int>(left) : WC);
  };
  typedef __attribute__((address_space(4))) const SegKey ckey_t;
  ckey_t* const kc = (ckey_t*)keys;
  // window u_ of key j_ (walked forward from j_): its first column and width
  const auto locate = [&](int u_, int& j_, int64_t& c0_, int& n_) __attribute__((always_inline)) {
    while (j_ + 1 < nkeys32 && static_cast<int>(kc[j_ + 1].unit_start) <= u_) ++j_;
    const int w = u_ - static_cast<int>(kc[j_].unit_start);
    c0_ = static_cast<int64_t>(w) * WC;
    n_ = cols_of(kc[j_].numel, w);
  };
  int u = static_cast<int>(blockIdx.x), j = 0, n = 0;
  int64_t c0 = 0;
  int jn = 0, nn = 0;
  int64_t c0n = 0, pvn = 0;
  if (u < units32) {
    j = __builtin_amdgcn_readfirstlane(static_cast<int>(find_key(keys, n_keys, u)));
    locate(u, j, c0, n);
    jn = j;
    const int64_t pv0 = load_ptrs(ptrs + static_cast<int64_t>(j) * K);
    // the next window's addresses before this window's rows: the loop's
    // first prefetch then waits for them with the rows still in flight
    if (u + G < units32) {
      locate(u + G, jn, c0n, nn);
      pvn = load_ptrs(ptrs + static_cast<int64_t>(jn) * K);
    }
    if constexpr (UNI) {
#pragma unroll
      for (int i = 0; i < KH; ++i) x[i] = load_row(pv0, i, c0, n, K);
    } else if (n == WC) {
#pragma unroll
      for (int i = 0; i < KH; ++i)
        x[i] = load_fast(pv0, i, static_cast<uint32_t>(c0 * 4), static_cast<uint32_t>((c0 + WC) * 4), K);
    } else {
      load_slow(pv0, c0, n, K);
    }
  }
  // the first window's rows in: without this wait the compiler merges the
  // prologue's pending row loads into the loop's state and waits for ALL of
  // a wave's rows at every turn (vmcnt(PF)) instead of row by row
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  int seq = 0;
  for (; u < units32; u += G, ++seq) {
    const int64_t out_off = kc[j].out_offset;
    const int un = u + G, unn = un + G;
    const bool fastn = un < units32 && nn == WC;
    const uint32_t soffn = static_cast<uint32_t>(c0n * 4), nrecn = static_cast<uint32_t>((c0n + WC) * 4);
    int Kwn = (UNI ? un < units32 : fastn) ? K : 0;
    asm volatile("" : "+s"(Kwn));
    stamp(0);
#pragma unroll
    for (int i = 0; i < PF; ++i) xp[i] = UNI ? load_row(pvn, i, c0n, nn, Kwn) : load_fast(pvn, i, soffn, nrecn, Kwn);
    // the turn
    float a = -0.0f;  // fl32(-0.0 + p) is p, bit for bit
    if (h > 0) {
      wait_flag(h - 1, seq);
      a = part[h - 1][lane];
    }
    stamp(2);
    __builtin_amdgcn_s_setprio(3);
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
      if (lane < n) out[out_off + c0 + lane] = a;
    }
    stamp(3);
    if (h < ns - 1) {
      __builtin_amdgcn_s_setprio(0);
      wait_flag(NSMAX, seq);
      a = avg[lane];
    }
    // the window after next: its key and client addresses, ahead of the reloads
    int jnn = jn, nnn = 0;
    int64_t c0nn = 0, pvnn = 0;
    if (unn < units32) {
      locate(unn, jnn, c0nn, nnn);
      pvnn = load_ptrs(ptrs + static_cast<int64_t>(jnn) * K);
    }
    if (h < 4)
      __builtin_amdgcn_s_setprio(2);
    else if (h < 8)
      __builtin_amdgcn_s_setprio(1);
    else
      __builtin_amdgcn_s_setprio(0);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      double p[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int i = 8 * b + r;
        const double d = static_cast<double>(x[i] - a);  // fp32 difference, as the reference forms it
        p[r] = d * d;
        if (i < PF)
          x[i] = xp[i < PF ? i : 0];
        else
          x[i] = UNI ? load_row(pvn, i, c0n, nn, Kwn) : load_fast(pvn, i, soffn, nrecn, Kwn);
      }
      const double q01 = fold32(p[0], p[1]), q23 = fold32(p[2], p[3]);
      const double q45 = fold32(p[4], p[5]), q67 = fold32(p[6], p[7]);
      acc[64 * b] += fold8(fold16(q01, q23), fold16(q45, q67), upper);
    }
    if (!UNI && un < units32 && !fastn) {
      int Ks = K;
      asm volatile("" : "+s"(Ks));
      load_slow(pvn, c0n, nn, Ks);
    }
    __builtin_amdgcn_s_setprio(0);
    stamp(4);
    ++wi;
    j = jn;
    c0 = c0n;
    n = nn;
    jn = jnn;
    c0n = c0nn;
    nn = nnn;
    pvn = pvnn;
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

constexpr int64_t kSegSplitMaxK = 1024;  // the split-row windows' reach (16 waves of 64 clients)

// workgroups of the split-row window launch over `units` windows (0: not resident)
constexpr int kSegWinfPF8 = 8, kSegWinfPF16 = 16;  // prefetched rows at <= 8 / 16 waves

// FEDAVG_SEGWINN_BARRIER=1 keeps round 5's barrier form of the zero-copy
// split windows (A/B); the hand-off form is the default
inline bool seg_barrier_windows() {
  static const bool on = [] {
    const char* e = std::getenv("FEDAVG_SEGWINN_BARRIER");
    return e && e[0] == '1';
  }();
  return on;
}

// FEDAVG_SEGWINF_TWO_PATHS=1: the hand-off kernel with round 5's separate
// ragged-window reload (A/B against the uniform row loads)
inline bool seg_split_two_paths() {
  static const bool on = [] {
    const char* e = std::getenv("FEDAVG_SEGWINF_TWO_PATHS");
    return e && e[0] == '1';
  }();
  return on;
}

// FEDAVG_SEGWINF_STAMPS=1: the hand-off kernel's timeline build (MODE 8;
// the partials grow by winn_stamp_elems)
inline bool seg_split_stamps() {
  static const bool on = [] {
    const char* e = std::getenv("FEDAVG_SEGWINF_STAMPS");
    return e && e[0] == '1';
  }();
  return on;
}

inline int64_t segwinn_blocks(int64_t K, int64_t units) {
  const int ns = static_cast<int>((K + 63) / 64);
  const bool bar = seg_barrier_windows();
  int64_t res = ns <= 8 ? (bar ? resident_blocks(reduce_sqdist_segwinn_kernel<8>, 64 * ns)
                               : resident_blocks(reduce_sqdist_segwinf_kernel<8, kSegWinfPF8>, 64 * ns))
                        : (bar ? resident_blocks(reduce_sqdist_segwinn_kernel<16>, 64 * ns)
                               : resident_blocks(reduce_sqdist_segwinf_kernel<16, kSegWinfPF16>, 64 * ns));
  // workgroups per CU: the resident ones rounded down to a power of two, as
  // the rows kernel's grid (round 6, the hand-off kernel, resnet18_gn-shaped
  // rounds, profiles/r06/zc_percu/, ms: 257 clients 3 per CU 2.70 vs 2 2.32;
  // 300 2.83 vs 2.47; 129 clients 5 per CU 1.53 vs 4 1.47; 500 equal; the
  // barrier form's rule was 3 at 5 waves); FEDAVG_SEGWINN_PER_CU caps it
  static const int64_t per_cu_env = [] {
    const char* e = std::getenv("FEDAVG_SEGWINN_PER_CU");
    return e && e[0] ? static_cast<int64_t>(std::atoll(e)) : int64_t(0);
  }();
  const int64_t cus = cu_count();
  int64_t per_cu = per_cu_env;
  if (per_cu <= 0 && !bar) {
    const int64_t r = res / cus;
    per_cu = 0;
    if (r >= 1)
      for (per_cu = 1; per_cu * 2 <= r;) per_cu *= 2;
  } else if (per_cu <= 0) {
    per_cu = ns == 5 ? 3 : 0;  // the barrier form's rule (round 5)
  }
  if (per_cu > 0 && per_cu * cus < res) res = per_cu * cus;
  return units < res ? units : res;
}

// windows per wave below which the LDS-DMA tiles keep the round
// (kSegWinMinPerWave; FEDAVG_SEGWIN_MIN_PER_WAVE overrides it for probes)
inline int64_t segwin_min_per_wave() {
  static const int64_t v = [] {
    const char* e = std::getenv("FEDAVG_SEGWIN_MIN_PER_WAVE");
    return e && e[0] ? static_cast<int64_t>(std::atoll(e)) : kSegWinMinPerWave;
  }();
  return v;
}

// FEDAVG_SEGWIN=0 keeps the LDS-DMA tiles for every device round (probes, A/B)
inline bool segwin_disabled() {
  static const bool off = [] {
    const char* e = std::getenv("FEDAVG_SEGWIN");
    return e && e[0] == '0';
  }();
  return off;
}

// waves of a zero-copy window launch over `units` windows
template <int KMAX, int VEC, int NW, bool DESC = true>
int64_t segwin_waves(int64_t units) {
  const int64_t per_cu = resident_blocks(reduce_sqdist_segwin_kernel<KMAX, VEC, NW, DESC>, 64 * NW) / cu_count();
  const int64_t grid = per_cu * cu_count();
  const int64_t need = (units + NW - 1) / NW;
  return (grid < need ? grid : need) * NW;
}

// the window instance for K clients (0 outside 17..128).  Round 3 ran 81-100
// clients on the 128 x 1 instance because its 100 x 2 form spilled (device
// round 100 x 25M 3.66 ms, profiles/r03/segwin/); the spill was the slow
// path's per-lane 64-bit element addresses, gone with the buffer-load form
// (232 VGPRs, no scratch), so 81-100 clients take 100 x 2 as on rows
inline int segwin_kmax(int64_t K) {
  return K <= 16 || K > 128 ? 0 : (K <= 48 ? 48 : (K <= 64 ? 64 : (K <= 80 ? 80 : (K <= 100 ? 100 : 128))));
}
inline int segwin_vec(int kmax) { return kmax == 48 ? 4 : (kmax == 128 ? 1 : 2); }

inline int64_t segwin_waves_for(int kmax, int64_t units) {
  switch (kmax) {
    case 48: return segwin_waves<48, 4, 4>(units);
    case 64: return segwin_waves<64, 2, 4>(units);
    case 80: return segwin_waves<80, 2, 4>(units);
    case 100: return segwin_waves<100, 2, 4>(units);
    case 128: return segwin_waves<128, 1, 4>(units);
    default: return 0;
  }
}

constexpr int kSegFusedMaxK = kBlock;

// tile width: as fedavg_dist.hip's fused_cols (32 above 128 clients, 64 above
// 64, 128 up to 64, 256 up to 16); every width keeps <= 8 load slots per thread
inline int seg_fused_cols(int64_t K) { return K > 128 ? 32 : (K > 64 ? 64 : (K > 16 ? 128 : 256)); }

inline int64_t seg_fused_lds_bytes(int64_t K, int S, bool laddr = false) {
  const int64_t b = (K + 1) * S * 4 + (laddr ? K * 8 : 0);  // LADDR: + the key's K client addresses
  return b > kBlock * 8 ? b : kBlock * 8;
}

// FEDAVG_SEG_LADDR=0 keeps the tiles' client addresses in registers (probes, A/B)
inline bool seg_laddr_disabled() {
  static const bool off = [] {
    const char* e = std::getenv("FEDAVG_SEG_LADDR");
    return e && e[0] == '0';
  }();
  return off;
}

template <int S, bool MAP = false, bool LADDR = false>
int seg_fused_per_cu(int64_t K) {
  static std::mutex mu;
  static std::map<std::pair<int, int64_t>, int> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find({dev, K});
  if (it != cache.end()) return it->second;
  const auto kern = reduce_sqdist_segments_f32_kernel<S, MAP, LADDR>;
  const int64_t lds = seg_fused_lds_bytes(K, S, LADDR);
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

template <int S, bool MAP = false, bool LADDR = false>
int64_t seg_fused_grid(int64_t K, int64_t units) {
  const int64_t g = static_cast<int64_t>(seg_fused_per_cu<S, MAP, LADDR>(K)) * cu_count();
  return units < g ? units : g;
}

// resident workgroups per CU of any tile kernel form (the partials' bound)
template <int S>
int seg_fused_per_cu_max(int64_t K) {
  const int a = seg_fused_per_cu<S, false>(K), b = seg_fused_per_cu<S, true>(K),
            c = seg_fused_per_cu<S, true, true>(K);
  const int ab = a > b ? a : b;
  return ab > c ? ab : c;
}

int64_t units_of(const int64_t* numel, int64_t n_keys, int64_t span = kSegSpan) {
  int64_t units = 0;
  for (int64_t j = 0; j < n_keys; ++j) units += (numel[j] + span - 1) / span;
  return units;
}

// a model with fewer than kSegSmallUnitsPerCU units of kSegSpan per CU takes
// the narrow units (reduce and :291 alike)
bool segments_small(const int64_t* numel, int64_t n_keys) {
  if (!numel || n_keys <= 0) return false;
  for (int64_t j = 0; j < n_keys; ++j)
    if (numel[j] < 0) return false;  // stage_tables reports it
  return units_of(numel, n_keys) < kSegSmallUnitsPerCU * static_cast<int64_t>(cu_count());
}

// Validate the tables, write the device tables into host_ws, copy them to
// dev_ws on `s`.  Returns the unit count (> 0), 0 for an empty model, or a
// negative error code.
int64_t stage_tables(const char* what, const int64_t* client_ptrs, const int64_t* numel, const int64_t* offset,
                     const int64_t* kind, int64_t n_keys, int64_t K, void* host_ws, void* dev_ws, int64_t ws_bytes,
                     hipStream_t s, int64_t span = kSegSpan) {
  if (n_keys <= 0 || K <= 0 || K > INT32_MAX || !client_ptrs || !numel || !offset || !kind || !host_ws || !dev_ws)
    return set_error(FEDAVG_EINVAL, "%s: bad arguments", what);
  if (ws_bytes < fedavg_segments_workspace(K, n_keys))
    return set_error(FEDAVG_EINVAL, "%s: workspace needs %lld bytes", what,
                     (long long)fedavg_segments_workspace(K, n_keys));
  if (!aligned16(host_ws) || !aligned16(dev_ws)) return set_error(FEDAVG_EALIGN, "%s: workspaces must be 16-B aligned", what);
  if (!is_pinned_host_memory(host_ws)) return set_error(FEDAVG_EINVAL, "%s: host_ws is not pinned host memory", what);
  if (!is_device_memory(dev_ws)) return set_error(FEDAVG_EINVAL, "%s: dev_ws must be device memory", what);
  fedavg_staging::TablesOut st;
  fedavg_staging::Msg msg;
  if (const int rc = fedavg_staging::stage_segment_tables(client_ptrs, numel, offset, kind, n_keys, K, host_ws, ws_bytes,
                                                          span, &st, &msg))
    return set_error(rc, "%s: %s", what, msg.text);
  const int64_t units = st.units;
  if (units == 0) return 0;
  // a host address would fault the kernels: spot check of the first and last
  // source (the Python layer checks every tensor's device)
  if (!is_device_memory(st.first_src) || !is_device_memory(st.last_src))
    return set_error(FEDAVG_EINVAL, "%s: client sources must be device memory", what);
  const hipError_t e = hipMemcpyAsync(dev_ws, host_ws, static_cast<size_t>(fedavg_segments_workspace(K, n_keys)),
                                      hipMemcpyHostToDevice, s);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return set_error(-static_cast<int>(e), "%s: hipMemcpyAsync failed: %s", what, hipGetErrorString(e));
  }
  return units;
}

// round-split: equal launches of at most `cap` workgroups (production: 3 x
// CUs, the reduce's schedule); cap <= 0 = one launch
template <int U, int C, int STYLE = 0>
void launch_reduce_segments(const SegKey* keys, const int64_t* ptrs, int64_t n_keys, int64_t units, int64_t K,
                            const float* weights, float* out, int64_t cap, hipStream_t s) {
  if (cap <= 0) cap = units;
  const int64_t nl = (units + cap - 1) / cap;
  const int64_t per = (units + nl - 1) / nl;
  for (int64_t u0 = 0; u0 < units; u0 += per) {
    const int64_t nb = units - u0 < per ? units - u0 : per;
    hipLaunchKernelGGL((reduce_segments_f32_kernel<U, C, STYLE>), dim3(static_cast<unsigned>(nb)), dim3(kBlock), 0, s, keys,
                       ptrs, n_keys, u0, static_cast<int>(K), weights, out);
  }
}

// The fused pass a round takes: the wave-owned windows for 17-128 clients
// when every key is fp32 and each wave gets at least segwin_min_per_wave()
// windows, else the LDS-DMA tiles.  `span` is the unit width the key table is
// staged with.
struct SegFusedPlan {
  bool win;
  int kmax;
  int64_t span, waves;
};

// 257-1024 clients fuse only on the split-row windows: 32-bit buffer offsets
// per key, window indices in 32 bits
inline bool seg_split_ok(const int64_t* numel, int64_t n_keys) {
  if (!numel || n_keys <= 0 || n_keys >= (int64_t(1) << 31)) return false;
  for (int64_t j = 0; j < n_keys; ++j)
    if (numel[j] < 0 || numel[j] >= (int64_t(1) << 30)) return false;
  return units_of(numel, n_keys, 64) < (int64_t(1) << 31);
}

// 129-256 clients take the zero-copy split windows too when every workgroup
// gets >= kSegSplitMinPerBlock windows (round 6; profiles/r06/seg160/, seg129/,
// resnet18_gn-shaped device rounds, ms, tiles vs split windows: 129 2.07 vs
// 1.46; 150 2.29 vs 1.49; 160 2.44 vs 1.43; 200 2.90 vs 1.71; 256 4.12 vs
// 2.10; the one-wave windows keep <= 128: 100 0.79 vs 1.06, 120 0.97 vs 1.11)
constexpr int64_t kSegSplitMinK = 129, kSegSplitMinPerBlock = 8;
// FEDAVG_SEG_SPLIT_MIN_K overrides kSegSplitMinK (probes)
inline int64_t seg_split_min_k() {
  static const int64_t v = [] {
    const char* e = std::getenv("FEDAVG_SEG_SPLIT_MIN_K");
    return e && e[0] ? static_cast<int64_t>(std::atoll(e)) : kSegSplitMinK;
  }();
  return v;
}

SegFusedPlan seg_fused_plan(const int64_t* numel, int64_t n_keys, int64_t K, bool all_raw) {
  SegFusedPlan p{false, segwin_kmax(K), seg_fused_cols(K), 0};
  if (K >= seg_split_min_k() && K >= 2 && K <= kSegFusedMaxK && all_raw && !seg_barrier_windows() &&
      seg_split_ok(numel, n_keys)) {
    const int64_t units = units_of(numel, n_keys, 64);
    const int64_t blocks = segwinn_blocks(K, units);
    if (blocks > 0 && units >= kSegSplitMinPerBlock * blocks) {
      p.win = true;
      p.kmax = -1;
      p.span = 64;
      p.waves = blocks;
      return p;
    }
  }
  if (K > kSegFusedMaxK) {  // kmax -1: the split-row windows (the caller checked seg_split_ok)
    if (K <= kSegSplitMaxK && all_raw && seg_split_ok(numel, n_keys)) {
      p.win = true;
      p.kmax = -1;
      p.span = 64;
      p.waves = segwinn_blocks(K, units_of(numel, n_keys, 64));
    }
    return p;
  }
  // the windows address a key's bytes with 32-bit buffer offsets
  bool small_keys = numel != nullptr;
  for (int64_t j = 0; small_keys && j < n_keys; ++j) small_keys = numel[j] < (int64_t(1) << 30);
  if (p.kmax > 0 && all_raw && small_keys && n_keys > 0 && n_keys < (int64_t(1) << 31) && !segwin_disabled()) {
    const int64_t wc = 64 * segwin_vec(p.kmax);
    const int64_t wunits = units_of(numel, n_keys, wc);
    const int64_t waves = segwin_waves_for(p.kmax, wunits);
    if (waves > 0 && wunits >= segwin_min_per_wave() * waves && wunits < (int64_t(1) << 31)) {
      p.win = true;
      p.span = wc;
      p.waves = waves;
    }
  }
  return p;
}

// The fused launch (+ the sums' finalize) on tables staged with plan.span
int launch_seg_fused(const SegFusedPlan& p, const SegKey* keys, const int64_t* tptrs, int64_t n_keys, int64_t units,
                     int64_t K, const float* weights, float* out, double* partials, int64_t partial_elems,
                     double* sumsq, hipStream_t s, const char* what, const int* umap = nullptr,
                     const u32x4* desc = nullptr) {
  if (units == 0) {
    const hipError_t e = hipMemsetAsync(sumsq, 0, static_cast<size_t>(K) * sizeof(double), s);
    return e == hipSuccess ? FEDAVG_OK : set_error(-static_cast<int>(e), "%s: hipMemsetAsync failed", what);
  }
  // beyond kSegFusedMaxK clients only the split-row windows fuse: the tile
  // kernel loads at most kBlock client addresses per workgroup
  if (K > kSegFusedMaxK && !(p.win && p.kmax < 0))
    return set_error(FEDAVG_EMODE, "%s: K = %lld fuses only on the split-row windows", what, (long long)K);
  const int k32 = static_cast<int>(K);
  int64_t nparts = 0;
  if (p.win && p.kmax < 0) {  // split-row windows: p.waves workgroups of ceil(K / 64) waves
    if (p.waves <= 0) return set_error(FEDAVG_EMODE, "%s: the split window kernel is not resident", what);
    if (partial_elems < K * p.waves)
      return set_error(FEDAVG_EINVAL, "%s: partials need %lld doubles", what, (long long)(K * p.waves));
    const int ns = static_cast<int>((K + 63) / 64);
    const dim3 grid(static_cast<unsigned>(p.waves)), block(static_cast<unsigned>(64 * ns));
    if (K < 2)
      return set_error(FEDAVG_EMODE, "%s: the split windows take K >= 2", what);
    if (seg_barrier_windows()) {
      if (ns <= 8)
        hipLaunchKernelGGL((reduce_sqdist_segwinn_kernel<8>), grid, block, 0, s, keys, tptrs, n_keys, units, k32,
                           weights, out, partials);
      else
        hipLaunchKernelGGL((reduce_sqdist_segwinn_kernel<16>), grid, block, 0, s, keys, tptrs, n_keys, units, k32,
                           weights, out, partials);
    } else if (seg_split_stamps()) {  // timeline probe
      if (partial_elems < K * p.waves + winn_stamp_elems(16))
        return set_error(FEDAVG_EINVAL, "%s: the timeline needs %lld more doubles", what, (long long)winn_stamp_elems(16));
      if (ns <= 8)
        hipLaunchKernelGGL((reduce_sqdist_segwinf_kernel<8, kSegWinfPF8, true, 8>), grid, block, 0, s, keys, tptrs,
                           n_keys, units, k32, weights, out, partials);
      else
        hipLaunchKernelGGL((reduce_sqdist_segwinf_kernel<16, kSegWinfPF16, true, 8>), grid, block, 0, s, keys, tptrs,
                           n_keys, units, k32, weights, out, partials);
    } else if (seg_split_two_paths()) {  // A/B: ragged windows reloaded after the squares
      if (ns <= 8)
        hipLaunchKernelGGL((reduce_sqdist_segwinf_kernel<8, kSegWinfPF8, false>), grid, block, 0, s, keys, tptrs,
                           n_keys, units, k32, weights, out, partials);
      else
        hipLaunchKernelGGL((reduce_sqdist_segwinf_kernel<16, kSegWinfPF16, false>), grid, block, 0, s, keys, tptrs,
                           n_keys, units, k32, weights, out, partials);
    } else if (ns <= 8) {
      hipLaunchKernelGGL((reduce_sqdist_segwinf_kernel<8, kSegWinfPF8>), grid, block, 0, s, keys, tptrs, n_keys, units,
                         k32, weights, out, partials);
    } else {
      hipLaunchKernelGGL((reduce_sqdist_segwinf_kernel<16, kSegWinfPF16>), grid, block, 0, s, keys, tptrs, n_keys,
                         units, k32, weights, out, partials);
    }
    nparts = p.waves;
  } else if (p.win) {
    if (partial_elems < K * p.waves)
      return set_error(FEDAVG_EINVAL, "%s: partials need %lld doubles", what, (long long)(K * p.waves));
    const dim3 grid(static_cast<unsigned>(p.waves / 4)), block(256);
#define FEDAVG_SEGWIN(KM, VC)                                                                                       \
  if (desc)                                                                                                        \
    hipLaunchKernelGGL((reduce_sqdist_segwin_kernel<KM, VC, 4, true>), grid, block, 0, s, keys, tptrs, n_keys,     \
                       units, k32, weights, out, partials, desc);                                                  \
  else                                                                                                             \
    hipLaunchKernelGGL((reduce_sqdist_segwin_kernel<KM, VC, 4, false>), grid, block, 0, s, keys, tptrs, n_keys,    \
                       units, k32, weights, out, partials, nullptr);
    switch (p.kmax) {
      case 48: FEDAVG_SEGWIN(48, 4) break;
      case 64: FEDAVG_SEGWIN(64, 2) break;
      case 80: FEDAVG_SEGWIN(80, 2) break;
      case 100: FEDAVG_SEGWIN(100, 2) break;
      default: FEDAVG_SEGWIN(128, 1) break;
    }
#undef FEDAVG_SEGWIN
    nparts = p.waves;
  } else {
    const int S = static_cast<int>(p.span);
#define FEDAVG_SEG_FUSED(C)                                                                                        \
  if (S == C) {                                                                                                    \
    const bool la = umap && !seg_laddr_disabled();                                                                 \
    if ((la ? seg_fused_per_cu<C, true, true>(K) : (umap ? seg_fused_per_cu<C, true>(K) : seg_fused_per_cu<C>(K))) \
        <= 0)                                                                                                      \
      return set_error(FEDAVG_EMODE, "%s: tile does not fit LDS", what);                                           \
    nparts = la ? seg_fused_grid<C, true, true>(K, units)                                                          \
                : (umap ? seg_fused_grid<C, true>(K, units) : seg_fused_grid<C>(K, units));                        \
    if (partial_elems < K * nparts)                                                                                \
      return set_error(FEDAVG_EINVAL, "%s: partials need %lld doubles", what, (long long)(K * nparts));             \
    if (la)                                                                                                        \
      hipLaunchKernelGGL((reduce_sqdist_segments_f32_kernel<C, true, true>), dim3(static_cast<unsigned>(nparts)),   \
                         dim3(kBlock), static_cast<unsigned>(seg_fused_lds_bytes(K, C, true)), s, keys, tptrs,      \
                         n_keys, units, k32, weights, out, partials, umap);                                         \
    else if (umap)                                                                                                 \
      hipLaunchKernelGGL((reduce_sqdist_segments_f32_kernel<C, true>), dim3(static_cast<unsigned>(nparts)),         \
                         dim3(kBlock), static_cast<unsigned>(seg_fused_lds_bytes(K, C)), s, keys, tptrs, n_keys,    \
                         units, k32, weights, out, partials, umap);                                                 \
    else                                                                                                           \
      hipLaunchKernelGGL((reduce_sqdist_segments_f32_kernel<C>), dim3(static_cast<unsigned>(nparts)), dim3(kBlock),  \
                         static_cast<unsigned>(seg_fused_lds_bytes(K, C)), s, keys, tptrs, n_keys, units, k32,      \
                         weights, out, partials, nullptr);                                                          \
  }
    FEDAVG_SEG_FUSED(32)
    FEDAVG_SEG_FUSED(64)
    FEDAVG_SEG_FUSED(128)
    FEDAVG_SEG_FUSED(256)
#undef FEDAVG_SEG_FUSED
  }
  int rc = launch_status(what);
  if (rc) return rc;
  hipLaunchKernelGGL(segments_finalize_kernel, dim3(static_cast<unsigned>(K)), dim3(kBlock), 0, s, partials, nparts,
                     sumsq);
  return launch_status(what);
}

// ---------------------------------------------------------------------------
// A device-resident round in one call (round 4: fedavg_device_round_f32).
// The Python layer used to gather the group's pointer columns, convert the
// integer keys through a pack launch of its own, upload the weights and stage
// the tables in four steps (0.3 ms of host time for resnet56 x 100's 35,000
// tensors against a 0.08 ms kernel); here one pass over the walk's address
// table writes the key table, the key-major pointer table, the fp32 weights
// and the integer keys' conversion table into the pinned workspace, one H2D
// ships them, and the launches follow.
// Workspace layout (host and device alike, 16-B aligned parts):
//   SegKey[n_keys] | int64 ptrs[n_keys * K + kSegWinTablePad] | float w[K] |
//   IntKey[n_keys] | int64 int_src[n_keys * K]
// ---------------------------------------------------------------------------
// (IntKey, RoundWs / round_ws, the unit map's and the descriptor table's
// limits: staging.hpp; a tile round of more than kSegUnitMapMax units at
// 17-128 clients takes the windows)

// FEDAVG_SEGWIN_DESC=0 keeps the windows' pointer form (probes, A/B)
inline bool segwin_desc_disabled() {
  static const bool off = [] {
    const char* e = std::getenv("FEDAVG_SEGWIN_DESC");
    return e && e[0] == '0';
  }();
  return off;
}


// a fused round's integer / bool keys as fp32 columns of the [K, S] scratch:
// one wave per (key, client) item, the packers' static_cast (fedavg_pack.hip)
__global__ __launch_bounds__(64) void int_keys_to_f32_kernel(const IntKey* __restrict__ ik,
                                                             const int64_t* __restrict__ src, int K, int64_t S,
                                                             float* __restrict__ scratch) {
  const int64_t item = blockIdx.x;  // key q, client k: item = q * K + k
  const int64_t q = item / K, k = item - q * K;
  const IntKey key = ik[q];
  const void* p = reinterpret_cast<const void*>(src[item]);
  float* d = scratch + k * S + key.col;
  for (int64_t e = threadIdx.x; e < key.numel; e += 64) d[e] = load_cvt(p, key.kind, e);
}

}  // namespace

extern "C" {

int64_t fedavg_segments_workspace(int64_t K, int64_t n_keys) {
  return fedavg_staging::segments_workspace_bytes(K, n_keys);
}

int64_t fedavg_segments_partials(const int64_t* key_numel, int64_t n_keys, int64_t K) {
  if (!key_numel || n_keys <= 0 || K <= 0) return 0;
  return K * units_of(key_numel, n_keys, segments_small(key_numel, n_keys) ? kSegSmallSpan : kSegDistSpan) *
         (kBlock / 64);
}

int fedavg_reduce_ptrs_f32(const float* const* client_ptrs, int64_t K, int64_t P, const float* weights,
                           float* out, void* stream) {
  const char* what = "fedavg_reduce_ptrs_f32";
  int rc = check_common(client_ptrs, K, P, P, weights, out, what);
  if (rc) return rc;
  if (P == 0) return FEDAVG_OK;
  if (!aligned4(out) || !aligned4(weights)) return set_error(FEDAVG_EALIGN, "%s: out/weights misaligned", what);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool small = (P + kSegSpan - 1) / kSegSpan < kSegSmallUnitsPerCU * static_cast<int64_t>(cu_count());
  const int64_t span = small ? static_cast<int64_t>(kBlock) * kSegSmallC * 4 : kSegSpan;
  const int64_t units = (P + span - 1) / span;
  const int64_t cap = static_cast<int64_t>(small ? kSegSmallBlocksPerCU : kSegBlocksPerCU) * cu_count();
  const int64_t nl = (units + cap - 1) / cap;
  const int64_t per = (units + nl - 1) / nl;
  const auto* ptrs = reinterpret_cast<const int64_t*>(client_ptrs);
  for (int64_t u0 = 0; u0 < units; u0 += per) {
    const int64_t nb = units - u0 < per ? units - u0 : per;
    if (small)
      hipLaunchKernelGGL((reduce_ptrs_f32_kernel<kSegU, kSegSmallC>), dim3(static_cast<unsigned>(nb)), dim3(kBlock), 0,
                         s, ptrs, P, u0, static_cast<int>(K), weights, out);
    else
      hipLaunchKernelGGL((reduce_ptrs_f32_kernel<kSegU, kSegC>), dim3(static_cast<unsigned>(nb)), dim3(kBlock), 0, s,
                         ptrs, P, u0, static_cast<int>(K), weights, out);
  }
  return launch_status(what);
}

int fedavg_reduce_segments_f32(const int64_t* client_ptrs, const int64_t* key_numel, const int64_t* key_offset,
                               const int64_t* key_kind, int64_t n_keys, int64_t K, const float* weights, float* out,
                               void* host_ws, void* dev_ws, int64_t ws_bytes, void* stream) {
  const char* what = "fedavg_reduce_segments_f32";
  if (!weights || !out) return set_error(FEDAVG_EINVAL, "%s: null weights/out", what);
  if (!is_device_memory(out)) return set_error(FEDAVG_EINVAL, "%s: out must be device memory", what);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool small = segments_small(key_numel, n_keys);
  const int64_t span = small ? kSegSmallSpan : kSegSpan;
  const int64_t units = stage_tables(what, client_ptrs, key_numel, key_offset, key_kind, n_keys, K, host_ws, dev_ws,
                                     ws_bytes, s, span);
  if (units <= 0) return static_cast<int>(units);
  const auto* keys = static_cast<const SegKey*>(dev_ws);
  const auto* ptrs = reinterpret_cast<const int64_t*>(static_cast<const char*>(dev_ws) +
                                                      n_keys * static_cast<int64_t>(sizeof(SegKey)));
  if (small)
    launch_reduce_segments<kSegU, kSegSmallC, kSegStyle>(keys, ptrs, n_keys, units, K, weights, out,
                                                         static_cast<int64_t>(kSegSmallBlocksPerCU) * cu_count(), s);
  else
    launch_reduce_segments<kSegU, kSegC, kSegStyle>(keys, ptrs, n_keys, units, K, weights, out,
                                                    static_cast<int64_t>(kSegBlocksPerCU) * cu_count(), s);
  return launch_status(what);
}

int fedavg_client_sqdist_segments_f32(const int64_t* client_ptrs, const int64_t* key_numel, const int64_t* key_offset,
                                      const int64_t* key_kind, int64_t n_keys, int64_t K, const float* glob,
                                      double* partials, int64_t partial_elems, double* sumsq, void* host_ws,
                                      void* dev_ws, int64_t ws_bytes, void* stream) {
  const char* what = "fedavg_client_sqdist_segments_f32";
  if (!glob || !partials || !sumsq) return set_error(FEDAVG_EINVAL, "%s: null glob/partials/sumsq", what);
  if (!is_device_memory(glob) || !is_device_memory(partials) || !is_device_memory(sumsq))
    return set_error(FEDAVG_EINVAL, "%s: glob, partials and sumsq must be device memory", what);
  const int64_t need = fedavg_segments_partials(key_numel, n_keys, K);
  if (partial_elems < need) return set_error(FEDAVG_EINVAL, "%s: partials need %lld doubles", what, (long long)need);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool small = segments_small(key_numel, n_keys);
  const int64_t units = stage_tables(what, client_ptrs, key_numel, key_offset, key_kind, n_keys, K, host_ws, dev_ws,
                                     ws_bytes, s, small ? kSegSmallSpan : kSegDistSpan);
  if (units < 0) return static_cast<int>(units);
  if (units == 0) {
    const hipError_t e = hipMemsetAsync(sumsq, 0, static_cast<size_t>(K) * sizeof(double), s);
    return e == hipSuccess ? FEDAVG_OK : set_error(-static_cast<int>(e), "%s: hipMemsetAsync failed", what);
  }
  const auto* keys = static_cast<const SegKey*>(dev_ws);
  const auto* ptrs = reinterpret_cast<const int64_t*>(static_cast<const char*>(dev_ws) +
                                                      n_keys * static_cast<int64_t>(sizeof(SegKey)));
  const int64_t nparts = units * (kBlock / 64);
  if (small)
    hipLaunchKernelGGL((sqdist_segments_f32_kernel<kSegDistU, kSegSmallC>), dim3(static_cast<unsigned>(units)),
                       dim3(kBlock), 0, s, keys, ptrs, n_keys, int64_t(0), static_cast<int>(K), glob, partials, nparts);
  else
    hipLaunchKernelGGL((sqdist_segments_f32_kernel<kSegDistU, kSegDistC>), dim3(static_cast<unsigned>(units)),
                       dim3(kBlock), 0, s, keys, ptrs, n_keys, int64_t(0), static_cast<int>(K), glob, partials, nparts);
  int rc = launch_status(what);
  if (rc) return rc;
  hipLaunchKernelGGL(segments_finalize_kernel, dim3(static_cast<unsigned>(K)), dim3(kBlock), 0, s, partials, nparts,
                     sumsq);
  return launch_status(what);
}

// Aggregate + :291 sums in one pass over device-resident clients (K <= 256,
// every fp32 key's client tensors 16-B aligned): out as
// fedavg_reduce_segments_f32, sumsq as fedavg_client_sqdist_segments_f32 on
// that out.  partials : fedavg_reduce_sqdist_segments_partials(K) doubles.
int64_t fedavg_reduce_sqdist_segments_partials(int64_t K) {
  if (K <= 0 || K > kSegSplitMaxK) return 0;
  if (K > kSegFusedMaxK)  // the split-row windows (device round)
    return K * segwinn_blocks(K, INT64_MAX / 2) + (seg_split_stamps() ? winn_stamp_elems(16) : 0);
  const int S = seg_fused_cols(K);
  const int per_cu = S == 32 ? seg_fused_per_cu_max<32>(K)
                     : (S == 64 ? seg_fused_per_cu_max<64>(K)
                                : (S == 128 ? seg_fused_per_cu_max<128>(K) : seg_fused_per_cu_max<256>(K)));
  const int64_t tiles = K * static_cast<int64_t>(per_cu > 0 ? per_cu : 1) * cu_count();
  const int64_t windows = K * segwin_waves_for(segwin_kmax(K), INT64_MAX / 2);  // a full window launch
  const int64_t split = K >= seg_split_min_k() ? K * segwinn_blocks(K, INT64_MAX / 2) : 0;  // 129-256: split windows
  const int64_t need = tiles > windows ? tiles : windows;
  return (need > split ? need : split) + (seg_split_stamps() ? winn_stamp_elems(16) : 0);
}

int fedavg_reduce_sqdist_segments_f32(const int64_t* client_ptrs, const int64_t* key_numel, const int64_t* key_offset,
                                      const int64_t* key_kind, int64_t n_keys, int64_t K, const float* weights,
                                      float* out, double* partials, int64_t partial_elems, double* sumsq,
                                      void* host_ws, void* dev_ws, int64_t ws_bytes, void* stream) {
  const char* what = "fedavg_reduce_sqdist_segments_f32";
  if (!weights || !out || !partials || !sumsq) return set_error(FEDAVG_EINVAL, "%s: null weights/out/partials/sumsq", what);
  if (K < 1 || K > kSegFusedMaxK)
    return set_error(FEDAVG_EINVAL, "%s: K = %lld outside 1..%d (use the two passes)", what, (long long)K, kSegFusedMaxK);
  if (!is_device_memory(out) || !is_device_memory(partials) || !is_device_memory(sumsq))
    return set_error(FEDAVG_EINVAL, "%s: out, partials and sumsq must be device memory", what);
  if (client_ptrs && key_kind && key_numel)
    for (int64_t j = 0; j < n_keys; ++j)
      for (int64_t k = 0; k < K && key_kind[j] == kRaw && key_numel[j] > 0; ++k)
        if ((client_ptrs[k * n_keys + j] & 15) != 0)
          return set_error(FEDAVG_EALIGN, "%s: client %lld key %lld is not 16-B aligned (use the two passes)", what,
                           (long long)k, (long long)j);
  hipStream_t s = static_cast<hipStream_t>(stream);
  // long models, 17-128 clients, fp32 keys only: the zero-copy wave-owned windows
  bool all_raw = key_kind != nullptr && key_numel != nullptr;
  for (int64_t jk = 0; all_raw && jk < n_keys; ++jk) all_raw = key_numel[jk] >= 0 && key_kind[jk] == kRaw;
  const SegFusedPlan plan = seg_fused_plan(key_numel, n_keys, K, all_raw);
  if (plan.win && partial_elems < K * plan.waves)
    return set_error(FEDAVG_EINVAL, "%s: partials need %lld doubles", what, (long long)(K * plan.waves));
  const int64_t units = stage_tables(what, client_ptrs, key_numel, key_offset, key_kind, n_keys, K, host_ws, dev_ws,
                                     ws_bytes, s, plan.span);
  if (units < 0) return static_cast<int>(units);
  const auto* keys = static_cast<const SegKey*>(dev_ws);
  const auto* tptrs = reinterpret_cast<const int64_t*>(static_cast<const char*>(dev_ws) +
                                                       n_keys * static_cast<int64_t>(sizeof(SegKey)));
  return launch_seg_fused(plan, keys, tptrs, n_keys, units, K, weights, out, partials, partial_elems, sumsq, s, what);
}

int64_t fedavg_device_round_workspace(int64_t K, int64_t n_keys) {
  if (K <= 0 || n_keys <= 0) return 0;
  return round_ws(K, n_keys).end;
}

int64_t fedavg_device_round_scratch(const int64_t* key_numel, const int64_t* key_kind, int64_t n_keys, int64_t K) {
  if (!key_numel || !key_kind || n_keys <= 0 || K <= 0) return 0;
  int64_t S = 0;
  for (int64_t j = 0; j < n_keys; ++j)
    if (key_kind[j] != kRaw && key_numel[j] > 0) S += (key_numel[j] + 3) & ~int64_t(3);
  return K * S;
}

#ifdef FEDAVG_TUNING  // probe library only: host-side phase times of the last device round call
}  // extern "C"
namespace {
thread_local double g_round_phase_us[10];
thread_local int g_round_nphase = 0;
thread_local std::chrono::steady_clock::time_point g_round_t0;
}  // namespace
#define FEDAVG_ROUND_MARK(i)                                                                              \
  do {                                                                                                    \
    const auto t_ = std::chrono::steady_clock::now();                                                     \
    if ((i) == 0) g_round_t0 = t_;                                                                        \
    g_round_phase_us[i] = std::chrono::duration<double, std::micro>(t_ - g_round_t0).count();             \
    g_round_nphase = (i) + 1;                                                                             \
  } while (0)
extern "C" {
int fedavg_device_round_phases(double* us, int cap) {
  const int n = g_round_nphase < cap ? g_round_nphase : cap;
  for (int i = 0; i < n; ++i) us[i] = g_round_phase_us[i];
  return n;
}
#else
#define FEDAVG_ROUND_MARK(i) \
  do {                       \
  } while (0)
#endif

int fedavg_device_round_f32(const int64_t* client_ptrs, int64_t ptr_ld, const int64_t* key_index,
                            const int64_t* key_numel, const int64_t* key_offset, const int64_t* key_kind,
                            int64_t n_keys, int64_t K, const double* weights, float* out, double* partials,
                            int64_t partial_elems, double* sumsq, float* int_scratch, int64_t scratch_elems,
                            void* host_ws, void* dev_ws, int64_t ws_bytes, void* stream) {
  const char* what = "fedavg_device_round_f32";
  FEDAVG_ROUND_MARK(0);
  if (!client_ptrs || !key_numel || !key_offset || !key_kind || !weights || !out || n_keys <= 0 || K <= 0 ||
      K > INT32_MAX || n_keys >= (int64_t(1) << 31) || (!key_index && ptr_ld < n_keys) || !host_ws || !dev_ws)
    return set_error(FEDAVG_EINVAL, "%s: bad arguments", what);
  if (sumsq && !partials) return set_error(FEDAVG_EINVAL, "%s: sums need partials", what);
  const RoundWs L = round_ws(K, n_keys);
  if (ws_bytes < L.end) return set_error(FEDAVG_EINVAL, "%s: workspace needs %lld bytes", what, (long long)L.end);
  if (!aligned16(host_ws) || !aligned16(dev_ws)) return set_error(FEDAVG_EALIGN, "%s: workspaces must be 16-B aligned", what);
  if (!is_pinned_host_memory(host_ws)) return set_error(FEDAVG_EINVAL, "%s: host_ws is not pinned host memory", what);
  if (!is_device_memory(dev_ws) || !is_device_memory(out))
    return set_error(FEDAVG_EINVAL, "%s: dev_ws and out must be device memory", what);
  if (sumsq && (!is_device_memory(sumsq) || !is_device_memory(partials)))
    return set_error(FEDAVG_EINVAL, "%s: partials and sumsq must be device memory", what);
  FEDAVG_ROUND_MARK(1);  // argument and pointer-attribute checks
  const bool fuse_req = sumsq != nullptr && (K <= kSegFusedMaxK || (K <= kSegSplitMaxK && seg_split_ok(key_numel, n_keys)));
  // a fused round takes its integer keys as fp32 scratch columns: the window
  // kernels read fp32 only, and the tiles' in-kernel conversion (element by
  // element, one tile per key and client block) made resnet56 x 100's fused
  // tile kernel 104 us against 77 + 4.7 us with the conversion launch
  // (profiles/r04/segwin_layout/); the two-pass reduce converts in-kernel
  if (fuse_req && int_scratch) {
    int64_t n_int = 0;
    fedavg_staging::int_scratch_cols(key_numel, key_kind, n_keys, &n_int);
    if (n_int > 0 && !is_device_memory(int_scratch))
      return set_error(FEDAVG_EINVAL, "%s: the integer keys' scratch must be device memory", what);
  }
  FEDAVG_ROUND_MARK(2);  // key validation
  // Everything the host writes before the tables' H2D (staging.hpp): the key
  // validation, the pointer table (client-major walk: the walk's table was
  // just written by other threads in fedavg_collect_ext and read row by row
  // -- the order the hardware prefetcher follows -- the call took 73-78 us
  // right after a resnet56 x 100 walk, against 182-200 us filling key-major;
  // branch-free checks per row: 63-65 us, scripts/device_round_call_probe.py,
  // profiles/r04/device_round/), the integer keys' scratch columns, the plan,
  // the key table, the tiles' unit map or the windows' descriptor table, the
  // weights.
  SegFusedPlan plan{false, 0, 0, 0};
  const auto plan_fn = [&](bool fuse, bool all_raw) -> fedavg_staging::RoundPlan {
    if (fuse) {
      plan = seg_fused_plan(key_numel, n_keys, K, all_raw);
      return fedavg_staging::RoundPlan{plan.win, plan.kmax, plan.span, false};
    }
    const bool small = segments_small(key_numel, n_keys);
    return fedavg_staging::RoundPlan{false, 0, small ? kSegSmallSpan : kSegSpan, small};
  };
  const fedavg_staging::RoundIn rin{client_ptrs, ptr_ld, key_index, key_numel, key_offset, key_kind, n_keys, K,
                                    weights, reinterpret_cast<int64_t>(int_scratch), int_scratch ? scratch_elems : 0,
                                    fuse_req, segwin_desc_disabled()};
  fedavg_staging::RoundOut st;
  fedavg_staging::Msg msg;
  int rc = fedavg_staging::stage_device_round(rin, host_ws, ws_bytes, plan_fn, &st, &msg);
  if (rc) return set_error(rc, "%s: %s", what, msg.text);
  FEDAVG_ROUND_MARK(3);  // the pointer-table fill
  const bool fuse = st.fuse, converted = st.converted, small = st.plan.small;
  const int64_t units = st.units, S = st.S, n_int = st.n_int, moff = st.moff;
  const bool with_map = st.with_map, with_desc = st.with_desc;
  if (!st.first_src) {  // every key empty
    if (sumsq) {
      const hipError_t e = hipMemsetAsync(sumsq, 0, static_cast<size_t>(K) * sizeof(double), static_cast<hipStream_t>(stream));
      if (e != hipSuccess) return set_error(-static_cast<int>(e), "%s: hipMemsetAsync failed", what);
    }
    return sumsq ? FEDAVG_OK : 1;
  }
  // a host address would fault the kernels: spot check of the first and last
  // source (the Python layer checks every tensor's device)
  if (!is_device_memory(st.first_src) || !is_device_memory(st.last_src))
    return set_error(FEDAVG_EINVAL, "%s: client sources must be device memory", what);
  FEDAVG_ROUND_MARK(4);  // the sources' spot check
  FEDAVG_ROUND_MARK(5);  // plan, key table, weights (staged above)
  hipStream_t s = static_cast<hipStream_t>(stream);
  const hipError_t e = hipMemcpyAsync(dev_ws, host_ws, static_cast<size_t>(st.bytes), hipMemcpyHostToDevice, s);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return set_error(-static_cast<int>(e), "%s: hipMemcpyAsync failed: %s", what, hipGetErrorString(e));
  }
  FEDAVG_ROUND_MARK(6);  // the tables' H2D issued
  const char* db = static_cast<const char*>(dev_ws);
  const auto* keys = reinterpret_cast<const SegKey*>(db);
  const auto* tptrs = reinterpret_cast<const int64_t*>(db + L.ptrs);
  const auto* dw = reinterpret_cast<const float*>(db + L.w);
  if (converted) {
    if (n_int * K > INT32_MAX) return set_error(FEDAVG_EINVAL, "%s: too many integer keys", what);
    hipLaunchKernelGGL(int_keys_to_f32_kernel, dim3(static_cast<unsigned>(n_int * K)), dim3(64), 0, s,
                       reinterpret_cast<const IntKey*>(db + L.ik), reinterpret_cast<const int64_t*>(db + L.isrc),
                       static_cast<int>(K), S, int_scratch);
    rc = launch_status(what);
    if (rc) return rc;
  }
  FEDAVG_ROUND_MARK(7);  // the integer keys' launch
  if (fuse) {
    rc = launch_seg_fused(plan, keys, tptrs, n_keys, units, K, dw, out, partials, partial_elems, sumsq, s, what,
                          with_map ? reinterpret_cast<const int*>(db + moff) : nullptr,
                          with_desc ? reinterpret_cast<const u32x4*>(db + moff) : nullptr);
    FEDAVG_ROUND_MARK(8);  // the fused launch and the sums' finalize
    return rc ? rc : FEDAVG_OK;
  }
  if (small)
    launch_reduce_segments<kSegU, kSegSmallC, kSegStyle>(keys, tptrs, n_keys, units, K, dw, out,
                                                         static_cast<int64_t>(kSegSmallBlocksPerCU) * cu_count(), s);
  else
    launch_reduce_segments<kSegU, kSegC, kSegStyle>(keys, tptrs, n_keys, units, K, dw, out,
                                                    static_cast<int64_t>(kSegBlocksPerCU) * cu_count(), s);
  rc = launch_status(what);
  FEDAVG_ROUND_MARK(8);  // the reduce's launches
  return rc ? rc : 1;
}

// tuning hook (fedavg_amd_tuning.h): the zero-copy reduce with an explicit
#ifdef FEDAVG_TUNING  // probe library only (libfedavg_amd_probe.so)
// fedavg_client_sqdist_segments_f32 with an explicit (U, C): units of
// 1,024 x C columns; partials need K x units x 4 doubles for that span
int fedavg_client_sqdist_segments_f32_variant(const int64_t* client_ptrs, const int64_t* key_numel,
                                              const int64_t* key_offset, const int64_t* key_kind, int64_t n_keys,
                                              int64_t K, const float* glob, double* partials, int64_t partial_elems,
                                              double* sumsq, void* host_ws, void* dev_ws, int64_t ws_bytes,
                                              int unroll, int cols, void* stream) {
  const char* what = "fedavg_client_sqdist_segments_f32_variant";
  if (!glob || !partials || !sumsq || !key_numel || n_keys <= 0 || K <= 0)
    return set_error(FEDAVG_EINVAL, "%s: bad arguments", what);
  const int uc = unroll * 100 + cols;
  if (uc != 104 && uc != 204 && uc != 404 && uc != 804 && uc != 401 && uc != 801 && uc != 402 && uc != 802 &&
      uc != 208 && uc != 408)
    return set_error(FEDAVG_EMODE, "%s: unsupported (unroll, cols) = (%d, %d)", what, unroll, cols);
  const int64_t span = static_cast<int64_t>(kBlock) * cols * 4;
  const int64_t need = K * units_of(key_numel, n_keys, span) * (kBlock / 64);
  if (partial_elems < need) return set_error(FEDAVG_EINVAL, "%s: partials need %lld doubles", what, (long long)need);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t units = stage_tables(what, client_ptrs, key_numel, key_offset, key_kind, n_keys, K, host_ws, dev_ws,
                                     ws_bytes, s, span);
  if (units <= 0) return static_cast<int>(units);
  const auto* keys = static_cast<const SegKey*>(dev_ws);
  const auto* ptrs = reinterpret_cast<const int64_t*>(static_cast<const char*>(dev_ws) +
                                                      n_keys * static_cast<int64_t>(sizeof(SegKey)));
  const int64_t nparts = units * (kBlock / 64);
  const dim3 grid(static_cast<unsigned>(units));
  const int k = static_cast<int>(K);
  switch (uc) {
#define FEDAVG_SQSEG_CASE(U, C)                                                                                      \
  case U * 100 + C:                                                                                                  \
    hipLaunchKernelGGL((sqdist_segments_f32_kernel<U, C>), grid, dim3(kBlock), 0, s, keys, ptrs, n_keys, int64_t(0), \
                       k, glob, partials, nparts);                                                                   \
    break;
    FEDAVG_SQSEG_CASE(1, 4)
    FEDAVG_SQSEG_CASE(2, 4)
    FEDAVG_SQSEG_CASE(4, 4)
    FEDAVG_SQSEG_CASE(8, 4)
    FEDAVG_SQSEG_CASE(4, 1)
    FEDAVG_SQSEG_CASE(8, 1)
    FEDAVG_SQSEG_CASE(4, 2)
    FEDAVG_SQSEG_CASE(8, 2)
    FEDAVG_SQSEG_CASE(2, 8)
    FEDAVG_SQSEG_CASE(4, 8)
#undef FEDAVG_SQSEG_CASE
  }
  int rc = launch_status(what);
  if (rc) return rc;
  hipLaunchKernelGGL(segments_finalize_kernel, dim3(static_cast<unsigned>(K)), dim3(kBlock), 0, s, partials, nparts,
                     sumsq);
  return launch_status(what);
}
#endif  // FEDAVG_TUNING

// (U, C) schedule -- units of 1,024 x C columns -- and launch size; same bits
#ifdef FEDAVG_TUNING  // probe library only (libfedavg_amd_probe.so)
int fedavg_reduce_segments_f32_variant(const int64_t* client_ptrs, const int64_t* key_numel, const int64_t* key_offset,
                                       const int64_t* key_kind, int64_t n_keys, int64_t K, const float* weights,
                                       float* out, void* host_ws, void* dev_ws, int64_t ws_bytes, int unroll, int cols,
                                       int blocks_per_cu, void* stream) {
  const char* what = "fedavg_reduce_segments_f32_variant";
  if (!weights || !out) return set_error(FEDAVG_EINVAL, "%s: null weights/out", what);
  if (!is_device_memory(out)) return set_error(FEDAVG_EINVAL, "%s: out must be device memory", what);
  // unroll >= 100: STYLE unroll / 100 (1: the row reduce's loop shape; 2-4:
  // interleaved with 2 / 4 / 8 loads in flight) at unroll % 100
  const int uc = unroll * 100 + cols;
  if (uc != 408 && uc != 804 && uc != 208 && uc != 404 && uc != 802 && uc != 1602 && uc != 216 && uc != 116 &&
      uc != 801 && uc != 401 && uc != 1601 && uc != 402 && uc != 10216 && uc != 10404 && uc != 10408 &&
      uc != 10208 && uc != 10804 && uc != 20216 && uc != 30216 && uc != 40216 && uc != 20404 && uc != 30404 &&
      uc != 30408 && uc != 40408 && uc != 20401 && uc != 30401 && uc != 20408)
    return set_error(FEDAVG_EMODE, "%s: unsupported (unroll, cols) = (%d, %d)", what, unroll, cols);
  if (blocks_per_cu < 0) return set_error(FEDAVG_EINVAL, "%s: blocks_per_cu < 0", what);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t span = static_cast<int64_t>(kBlock) * cols * 4;
  const int64_t units = stage_tables(what, client_ptrs, key_numel, key_offset, key_kind, n_keys, K, host_ws, dev_ws,
                                     ws_bytes, s, span);
  if (units <= 0) return static_cast<int>(units);
  const auto* keys = static_cast<const SegKey*>(dev_ws);
  const auto* ptrs = reinterpret_cast<const int64_t*>(static_cast<const char*>(dev_ws) +
                                                      n_keys * static_cast<int64_t>(sizeof(SegKey)));
  const int64_t cap = static_cast<int64_t>(blocks_per_cu) * cu_count();
  switch (uc) {
    case 408: launch_reduce_segments<4, 8>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 804: launch_reduce_segments<8, 4>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 208: launch_reduce_segments<2, 8>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 404: launch_reduce_segments<4, 4>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 802: launch_reduce_segments<8, 2>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 1602: launch_reduce_segments<16, 2>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 216: launch_reduce_segments<2, 16>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 10216: launch_reduce_segments<2, 16, 1>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 10404: launch_reduce_segments<4, 4, 1>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 10408: launch_reduce_segments<4, 8, 1>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 10208: launch_reduce_segments<2, 8, 1>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 10804: launch_reduce_segments<8, 4, 1>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 20216: launch_reduce_segments<2, 16, 2>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 30216: launch_reduce_segments<2, 16, 3>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 40216: launch_reduce_segments<2, 16, 4>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 20404: launch_reduce_segments<4, 4, 2>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 30404: launch_reduce_segments<4, 4, 3>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 30408: launch_reduce_segments<4, 8, 3>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 40408: launch_reduce_segments<4, 8, 4>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 20408: launch_reduce_segments<4, 8, 2>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 20401: launch_reduce_segments<4, 1, 2>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 30401: launch_reduce_segments<4, 1, 3>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 801: launch_reduce_segments<8, 1>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 401: launch_reduce_segments<4, 1>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 1601: launch_reduce_segments<16, 1>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    case 402: launch_reduce_segments<4, 2>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
    default: launch_reduce_segments<1, 16>(keys, ptrs, n_keys, units, K, weights, out, cap, s); break;
  }
  return launch_status(what);
}
#endif  // FEDAVG_TUNING

}  // extern "C"
