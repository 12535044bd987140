// fedavg_variants.hip -- benchmarking variants of the exact fp32 kernel
// (include/fedavg_amd_tuning.h): first-version kernel, multi-column /
// double-buffered / LDS-DMA / balanced / round-split / windowed schedules and
// the tiled layout.  All produce the same bits as fedavg_reduce_f32; the
// production schedule is chosen in fedavg_reduce.hip from their sweeps
// (profiles/sweeps/).
#include "common.hpp"

namespace {
using namespace fedavg_impl;

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

int reduce_f32_tuned_impl(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights,
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
    return set_error(FEDAVG_EALIGN, "%s: the tuning hook needs 16-B aligned clients and ld %% 4 == 0", what);
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
    case 3:  // 768-float4 groups: a 781K-column chunk (N = 8) fills 255 CUs instead of 191 at C4
      if constexpr (U == 8 || U == 16) return pick_var2<U, 3>(nt, pipe);
      return nullptr;
    case 6:
      if constexpr (U == 4 || U == 8) return pick_var2<U, 6>(nt, pipe);
      return nullptr;
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
// HBM read-ceiling probe (measurement only): how fast can this chip stream a
// buffer with NO reduction structure?  The reduce's rate is judged against
// this as well as against the 8 TB/s spec.  Each thread keeps 8 x 16-B loads
// in flight and folds them into a register; a value-dependent store keeps
// the loads alive without writing anything in practice.
//   mode 0: grid-stride (thread v reads v, v + G*256, ...), nontemporal;
//   mode 1: block-contiguous ranges (block b sweeps its own 1/G of the
//           buffer, 32 KiB per block-step), nontemporal;
//   mode 2: mode 1 with default-policy loads.
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(kBlock) void probe_read_kernel(const f32x4* __restrict__ X, int64_t nvec,
                                                            float* __restrict__ sink) {
  constexpr int U = 8;
  constexpr bool NT = MODE != 2;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if constexpr (MODE == 0) {
    const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
    int64_t v = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    for (; v + (U - 1) * stride < nvec; v += U * stride) {
      f32x4 xs[U];
#pragma unroll
      for (int u = 0; u < U; ++u) xs[u] = ld<NT>(X + v + u * stride);
#pragma unroll
      for (int u = 0; u < U; ++u) acc += xs[u];
    }
    for (; v < nvec; v += stride) acc += ld<NT>(X + v);
  } else {
    const int64_t per = (nvec + gridDim.x - 1) / gridDim.x;
    const int64_t b0 = static_cast<int64_t>(blockIdx.x) * per;
    const int64_t b1 = (b0 + per) < nvec ? (b0 + per) : nvec;
    int64_t v = b0 + threadIdx.x;
    for (; v + (U - 1) * kBlock < b1; v += U * kBlock) {
      f32x4 xs[U];
#pragma unroll
      for (int u = 0; u < U; ++u) xs[u] = ld<NT>(X + v + u * kBlock);
#pragma unroll
      for (int u = 0; u < U; ++u) acc += xs[u];
    }
    for (; v < b1; v += kBlock) acc += ld<NT>(X + v);
  }
  if (acc.x + acc.y + acc.z + acc.w == 1234.5678f) sink[blockIdx.x] = acc.x;
}

// ---------------------------------------------------------------------------
// Co-scheduling probe (measurement only): a stand-in for a collective's
// kernel -- few workgroups, each wave holding ~260 VGPRs like RCCL's generic
// kernel on gfx950 (261 VGPR + 17 AGPR per its code-object metadata) -- that
// copies a buffer and then, optionally, stays resident for hold_us
// microseconds (a collective bound by xGMI rather than HBM spends most of its
// time resident and waiting).  Run next to the reduce it shows whether such a
// kernel finds room on the CUs while a reduce launch holds them.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock, 1) void probe_busy_copy_kernel(const f32x4* __restrict__ src,
                                                                   f32x4* __restrict__ dst, int64_t nvec,
                                                                   uint64_t hold_ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz constant clock
  constexpr int R = 36;  // float4 registers per thread: ~294 VGPRs per wave, as RCCL's kernel
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t v0 = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; v0 < nvec; v0 += stride * R) {
    f32x4 r[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int64_t v = v0 + i * stride;
      r[i] = v < nvec ? ld<true>(src + v) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int64_t v = v0 + i * stride;
      if (v < nvec) dst[v] = r[i];
    }
  }
  while (__builtin_amdgcn_s_memrealtime() - t0 < hold_ticks) __builtin_amdgcn_s_sleep(32);
}

// XCD-aware block order (measurement only).  The dispatcher hands workgroup i
// of a launch to XCD i % 8, so in launch order neighbouring 32-KiB column
// slices of a row sit on different XCDs (and L2s).  This variant renumbers
// the workgroups so XCD x works on one contiguous run of slices: logical
// block = start(x) + i / 8, a bijection for any grid size.  The reduce has no
// reuse across blocks, so this tests whether HBM/Infinity-Fabric locality of
// each XCD's stream matters for a pure read stream.
template <int U, int C, bool NT>
__global__ __launch_bounds__(kBlock) void reduce_f32x4_xcd_kernel(const f32x4* __restrict__ X, int K, int64_t ld4,
                                                                  int64_t nvec, int tail, const float* __restrict__ W,
                                                                  float* __restrict__ out) {
  constexpr int kXcds = 8;
  const int64_t G = gridDim.x, i = blockIdx.x;
  const int64_t q = G / kXcds, r = G % kXcds, x = i % kXcds;
  const int64_t b = x * q + (x < r ? x : r) + i / kXcds;
  const int64_t span = static_cast<int64_t>(kBlock) * C;
  const int64_t base = b * span;
  if (base >= nvec) return;
  if (base + span <= nvec) {
    f32x4 acc[C];
    reduce_full_group<U, C, NT, false>(acc, X + base + threadIdx.x, K, ld4, W);
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

// Shader-clock probe (measurement only): one wave per workgroup stamps the
// shader cycle counter (s_memtime) and the 100 MHz constant clock
// (s_memrealtime) `samples + 1` times, `interval_ticks` of the constant clock
// apart, sleeping in between.  Run beside a kernel on another stream, the
// stamps give the clock the chip holds while that kernel runs:
// MHz = d(s_memtime) / d(s_memrealtime) * 100 (MI355X_MICROARCH.md 'DVFS
// give-back' item 6).  Lane 0 writes (memtime, realtime) pairs to
// out[block][sample] with ordinary vector stores.
__global__ __launch_bounds__(64) void probe_clock_kernel(unsigned long long* __restrict__ out, int samples,
                                                         uint64_t interval_ticks) {
  unsigned long long* o = out + static_cast<int64_t>(blockIdx.x) * 2 * (samples + 1);
  uint64_t t_next = __builtin_amdgcn_s_memrealtime();
  for (int k = 0; k <= samples; ++k) {
    while (__builtin_amdgcn_s_memrealtime() < t_next) __builtin_amdgcn_s_sleep(8);
    unsigned long long c, r;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c)::"memory");
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r)::"memory");
    if (threadIdx.x == 0) {
      o[2 * k] = c;
      o[2 * k + 1] = r;
    }
    t_next = r + interval_ticks;
  }
}

// launch_split's equal round-split launches, with the XCD-aware order
template <int U, int C, bool NT>
void launch_split_xcd(const float* clients, int K, int64_t ld, int64_t P, const float* W, float* out, int max_blocks,
                      hipStream_t s) {
  const int64_t nvec = (P + 3) / 4;
  const int64_t span = static_cast<int64_t>(kBlock) * C;
  const int64_t resident = max_blocks > 0 ? max_blocks : resident_blocks(reduce_f32x4_xcd_kernel<U, C, NT>);
  const int64_t blocks = (nvec + span - 1) / span;
  const int64_t nl = (blocks + resident - 1) / resident;
  const int64_t per = ((nvec + nl - 1) / nl + span - 1) / span * span;
  const f32x4* X = reinterpret_cast<const f32x4*>(clients);
  for (int64_t v0 = 0; v0 < nvec; v0 += per) {
    const int64_t n = (nvec - v0) < per ? (nvec - v0) : per;
    const int tail = (v0 + n == nvec) ? static_cast<int>(P & 3) : 0;
    hipLaunchKernelGGL((reduce_f32x4_xcd_kernel<U, C, NT>), dim3(static_cast<unsigned>((n + span - 1) / span)),
                       dim3(kBlock), 0, s, X + v0, K, ld / 4, n, tail, W, out + v0 * 4);
  }
}

}  // namespace

extern "C" {

int fedavg_reduce_f32_tuned(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights,
                            float* out, int unroll, int nontemporal, void* stream) {
  return reduce_f32_tuned_impl(clients, K, P, ld, weights, out, static_cast<hipStream_t>(stream), unroll,
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

int fedavg_probe_read_f32x4(const float* buf, int64_t nvec, int mode, int blocks, int launches, float* sink,
                            void* stream) {
  const char* what = "fedavg_probe_read_f32x4";
  if (nvec < 0 || blocks <= 0 || launches <= 0 || mode < 0 || mode > 2 || (nvec > 0 && (!buf || !sink)))
    return set_error(FEDAVG_EINVAL, "%s: bad arguments", what);
  if (nvec == 0) return FEDAVG_OK;
  if (!aligned16(buf)) return set_error(FEDAVG_EALIGN, "%s: buffer must be 16-B aligned", what);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const f32x4* X = reinterpret_cast<const f32x4*>(buf);
  const int64_t per = (nvec + launches - 1) / launches;
  for (int64_t v0 = 0; v0 < nvec; v0 += per) {
    const int64_t n = (nvec - v0) < per ? (nvec - v0) : per;
    switch (mode) {
      case 0: hipLaunchKernelGGL(probe_read_kernel<0>, dim3(blocks), dim3(kBlock), 0, s, X + v0, n, sink); break;
      case 1: hipLaunchKernelGGL(probe_read_kernel<1>, dim3(blocks), dim3(kBlock), 0, s, X + v0, n, sink); break;
      default: hipLaunchKernelGGL(probe_read_kernel<2>, dim3(blocks), dim3(kBlock), 0, s, X + v0, n, sink); break;
    }
  }
  return launch_status(what);
}

int fedavg_probe_busy_copy(const void* src, void* dst, int64_t bytes, int blocks, int hold_us, void* stream) {
  const char* what = "fedavg_probe_busy_copy";
  if (bytes < 0 || blocks <= 0 || hold_us < 0 || (bytes > 0 && (!src || !dst)))
    return set_error(FEDAVG_EINVAL, "%s: bad arguments", what);
  if (!aligned16(src) || !aligned16(dst) || (bytes % 16) != 0)
    return set_error(FEDAVG_EALIGN, "%s: 16-B aligned buffers and sizes only", what);
  hipLaunchKernelGGL(probe_busy_copy_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), static_cast<const f32x4*>(src), static_cast<f32x4*>(dst),
                     bytes / 16, static_cast<uint64_t>(hold_us) * 100u);
  return launch_status(what);
}

int fedavg_probe_clock(unsigned long long* out, int blocks, int samples, int interval_us, void* stream) {
  const char* what = "fedavg_probe_clock";
  if (!out || blocks <= 0 || blocks > 1024 || samples <= 0 || samples > 100000 || interval_us <= 0)
    return set_error(FEDAVG_EINVAL, "%s: bad arguments", what);
  hipLaunchKernelGGL(probe_clock_kernel, dim3(static_cast<unsigned>(blocks)), dim3(64), 0,
                     static_cast<hipStream_t>(stream), out, samples, static_cast<uint64_t>(interval_us) * 100u);
  return launch_status(what);
}

int fedavg_stream_create_masked(int reserve_cus, int priority, void** stream) {
  const char* what = "fedavg_stream_create_masked";
  if (!stream || reserve_cus < 0) return set_error(FEDAVG_EINVAL, "%s: bad arguments", what);
  hipStream_t s = nullptr;
  hipError_t e;
  if (reserve_cus == 0) {
    e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority);
  } else {
    const int cus = cu_count();
    if (reserve_cus >= cus) return set_error(FEDAVG_EINVAL, "%s: cannot reserve %d of %d CUs", what, reserve_cus, cus);
    uint32_t mask[16] = {0};
    const int nwords = (cus + 31) / 32 > 16 ? 16 : (cus + 31) / 32;
    for (int c = 0; c < cus - reserve_cus && c < 512; ++c) mask[c / 32] |= 1u << (c % 32);
    e = hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(nwords), mask);
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return set_error(-static_cast<int>(e), "%s: %s", what, hipGetErrorString(e));
  }
  *stream = s;
  return FEDAVG_OK;
}

int fedavg_stream_destroy(void* stream) {
  const hipError_t e = hipStreamDestroy(static_cast<hipStream_t>(stream));
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return set_error(-static_cast<int>(e), "fedavg_stream_destroy: %s", hipGetErrorString(e));
  }
  return FEDAVG_OK;
}

int fedavg_reduce_f32_xcd(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights, float* out,
                          int max_blocks, void* stream) {
  const char* what = "fedavg_reduce_f32_xcd";
  if (K <= 0 || P <= 0 || ld < P || !clients || !weights || !out || K > INT32_MAX)
    return set_error(FEDAVG_EINVAL, "%s: bad arguments", what);
  if (!aligned16(clients) || !aligned16(out) || (ld % 4) != 0)
    return set_error(FEDAVG_EALIGN, "%s: needs 16-B aligned clients/out and ld %% 4 == 0", what);
  launch_split_xcd<4, 8, true>(clients, static_cast<int>(K), ld, P, weights, out, max_blocks,
                               static_cast<hipStream_t>(stream));
  return launch_status(what);
}

int fedavg_reduce_f32_buf(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights, float* out,
                          int unroll, int cols, int block, int max_blocks, void* stream) {
  const char* what = "fedavg_reduce_f32_buf";
  if (K <= 0 || P <= 0 || ld < P || !clients || !weights || !out || K > INT32_MAX)
    return set_error(FEDAVG_EINVAL, "%s: bad arguments", what);
  if (!aligned16(clients) || !aligned16(out) || (ld % 4) != 0)
    return set_error(FEDAVG_EALIGN, "%s: needs 16-B aligned clients/out and ld %% 4 == 0", what);
  const int k = static_cast<int>(K);
  hipStream_t s = static_cast<hipStream_t>(stream);
#define FEDAVG_BUF_CASE(U, C, B) \
  case (B) * 10000 + (U) * 100 + (C): launch_split_buf<U, C, B>(clients, k, ld, P, weights, out, max_blocks, s); break;
  switch (block * 10000 + unroll * 100 + cols) {
    FEDAVG_BUF_CASE(4, 8, 256)
    FEDAVG_BUF_CASE(8, 4, 256)
    FEDAVG_BUF_CASE(4, 4, 256)
    FEDAVG_BUF_CASE(2, 8, 256)
    FEDAVG_BUF_CASE(2, 16, 256)
    FEDAVG_BUF_CASE(1, 16, 256)
    FEDAVG_BUF_CASE(8, 8, 256)
    FEDAVG_BUF_CASE(4, 16, 256)
    FEDAVG_BUF_CASE(16, 1, 256)
    FEDAVG_BUF_CASE(16, 2, 256)
    FEDAVG_BUF_CASE(16, 4, 256)
    FEDAVG_BUF_CASE(8, 2, 256)
    FEDAVG_BUF_CASE(8, 1, 256)
    // 6 / 3 / 12 slices: 1,536- / 768-float4 column groups, one per CU for the
    // 1.56M / 781K-column chunks of the N = 8 (and N = 4) all-gather pipeline
    FEDAVG_BUF_CASE(4, 6, 256)
    FEDAVG_BUF_CASE(2, 6, 256)
    FEDAVG_BUF_CASE(8, 6, 256)
    FEDAVG_BUF_CASE(8, 3, 256)
    FEDAVG_BUF_CASE(4, 3, 256)
    FEDAVG_BUF_CASE(16, 3, 256)
    FEDAVG_BUF_CASE(2, 12, 128)
    FEDAVG_BUF_CASE(4, 6, 128)
    FEDAVG_BUF_CASE(8, 1, 128)
    FEDAVG_BUF_CASE(8, 2, 128)
    FEDAVG_BUF_CASE(8, 4, 128)
    FEDAVG_BUF_CASE(16, 1, 128)
    FEDAVG_BUF_CASE(16, 2, 128)
    FEDAVG_BUF_CASE(16, 4, 128)
    FEDAVG_BUF_CASE(4, 4, 128)
    FEDAVG_BUF_CASE(4, 8, 128)
    FEDAVG_BUF_CASE(8, 1, 64)
    FEDAVG_BUF_CASE(8, 2, 64)
    FEDAVG_BUF_CASE(8, 4, 64)
    FEDAVG_BUF_CASE(16, 1, 64)
    FEDAVG_BUF_CASE(16, 2, 64)
    FEDAVG_BUF_CASE(16, 4, 64)
    FEDAVG_BUF_CASE(4, 4, 64)
    FEDAVG_BUF_CASE(4, 8, 64)
    FEDAVG_BUF_CASE(32, 1, 64)
    FEDAVG_BUF_CASE(32, 2, 64)
    // block 1256 / 1512: the 256-thread U2 x C16 kernel with co-resident
    // workgroups remapped to adjacent column groups (cu_contiguous_group,
    // 256 / 512 slots per round)
    case 1256 * 10000 + 216: launch_split_buf<2, 16, 256, 256>(clients, k, ld, P, weights, out, max_blocks, s); break;
    case 1512 * 10000 + 216: launch_split_buf<2, 16, 256, 512>(clients, k, ld, P, weights, out, max_blocks, s); break;
    default:
      return set_error(FEDAVG_EMODE, "%s: unsupported unroll=%d cols=%d block=%d", what, unroll, cols, block);
  }
#undef FEDAVG_BUF_CASE
  return launch_status(what);
}

}  // extern "C"
