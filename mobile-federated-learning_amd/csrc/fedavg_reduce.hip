// fedavg_reduce.hip -- production kernels, schedule and C ABI of
// libfedavg_amd.so (include/fedavg_amd.h).  Shared device code and the
// reference semantics: common.hpp.
#include "common.hpp"

namespace fedavg_impl {

namespace {
thread_local char g_err[512] = "";
}  // namespace

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

const char* last_error_message() { return g_err; }

int check_common(const void* clients, int64_t K, int64_t P, int64_t ld, const void* weights,
                 const void* out, const char* what) {
  if (K <= 0) return set_error(FEDAVG_EINVAL, "%s: K must be >= 1 (got %lld)", what, (long long)K);
  if (K > INT32_MAX) return set_error(FEDAVG_EINVAL, "%s: K too large", what);
  if (P < 0) return set_error(FEDAVG_EINVAL, "%s: P must be >= 0", what);
  if (ld < P) return set_error(FEDAVG_EINVAL, "%s: ld (%lld) < P (%lld)", what, (long long)ld, (long long)P);
  if (P > 0 && (!clients || !weights || !out)) return set_error(FEDAVG_EINVAL, "%s: null buffer", what);
  return FEDAVG_OK;
}

}  // namespace fedavg_impl

namespace {
using namespace fedavg_impl;

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

// ---------------------------------------------------------------------------
// fp64: the weight stays a double (ATen opmath for double).  Scalar path for
// unaligned buffers; the production path is reduce_vec_kernel<OpF64> below.
// ---------------------------------------------------------------------------
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
  __device__ static vec finish(vec a) { return a; }
};

// Packed 16-bit rules: two elements per 32-bit word, fp32 math on pairs
// (v_pk_mul_f32 / v_pk_add_f32) and gfx950's two-at-a-time round-to-nearest-
// even conversions (v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32) -- about 5 VALU ops
// per element and client instead of ~14 for the integer bf16 rounding, which
// made the kernel ALU-bound.  For every non-NaN input the hardware rounding
// equals c10's (checked over all 2^32 fp32 patterns, tests/test_gpu_parity.py
// via fedavg_probe_cvt16); NaN is absorbing through the remaining mul/add
// steps, so canonicalising NaN to c10's 0x7FC0 once at the store (bf16) gives
// c10's bits for the whole reduction.
template <typename R>
struct OpHalfPk {
  using vec = u16x8;
  using wt = float;
  using elem = unsigned short;
  static constexpr int kLanes = 8;
  __device__ static vec first(vec x, wt w) {
    u32x4 xu, r;
    __builtin_memcpy(&xu, &x, 16);
    const f32x2 w2{w, w};
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = R::pack(opaque2(R::unpack(xu[j]) * w2));
    vec o;
    __builtin_memcpy(&o, &r, 16);
    return o;
  }
  __device__ static vec step(vec acc, vec x, wt w) {
    u32x4 xu, au;
    __builtin_memcpy(&xu, &x, 16);
    __builtin_memcpy(&au, &acc, 16);
    const f32x2 w2{w, w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const unsigned int t = R::pack(opaque2(R::unpack(xu[j]) * w2));       // fl16(x*w)
      au[j] = R::pack(opaque2(R::unpack(au[j]) + R::unpack(t)));             // fl16(acc + t)
    }
    vec o;
    __builtin_memcpy(&o, &au, 16);
    return o;
  }
  __device__ static vec finish(vec a) {
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = R::canon(a[j]);
    return a;
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
  __device__ static vec finish(vec a) { return a; }
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
  a = Op::finish(a);
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

// ---------------------------------------------------------------------------
// Small-round kernel (fedavg_round_f32 for rounds of a few MB): ONE launch
// instead of H2D + reduce + D2H.  It reads the packed client rows straight
// from pinned host memory (zero-copy over PCIe), keeps a copy of them in HBM
// for the round's later passes (the :291 distances, FPF :210), reduces in the
// reference's order -- acc = x0*w0, acc = acc + xk*wk, one rounding each, the
// same bits as every other exact kernel -- and writes the averaged model to
// HBM and to pinned host memory.  A tiny round is latency-bound: three
// stream operations (two DMA engine hand-offs) cost more than the bytes.
// ---------------------------------------------------------------------------
template <int U>
__global__ __launch_bounds__(kBlock) void round_small_f32x4_kernel(
    const f32x4* __restrict__ Xh, f32x4* __restrict__ Xd, int K, int64_t ld4, int64_t nvec, int tail,
    const float* __restrict__ Wh, float* __restrict__ Wd, float* __restrict__ out_d, float* __restrict__ out_h) {
  if (blockIdx.x == 0)
    for (int k = threadIdx.x; k < K; k += kBlock) Wd[k] = Wh[k];
  const int64_t v = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (v >= nvec) return;
  const f32x4* col = Xh + v;
  f32x4* dcol = Xd + v;
  f32x4 x0 = col[0];
  dcol[0] = x0;
  f32x4 acc = x0 * Wh[0];  // fedavg_trainer.py:455 (i == 0)
  int k = 1;
  for (; k + U <= K; k += U) {
    f32x4 xs[U];
#pragma unroll
    for (int u = 0; u < U; ++u) xs[u] = col[static_cast<int64_t>(k + u) * ld4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      dcol[static_cast<int64_t>(k + u) * ld4] = xs[u];
      const f32x4 term = xs[u] * Wh[k + u];
      acc = acc + term;  // fedavg_trainer.py:457
    }
  }
  for (; k < K; ++k) {
    const f32x4 x = col[static_cast<int64_t>(k) * ld4];
    dcol[static_cast<int64_t>(k) * ld4] = x;
    const f32x4 term = x * Wh[k];
    acc = acc + term;
  }
  store_slice(out_d, v, nvec, tail, acc);
  store_slice(out_h, v, nvec, tail, acc);
}

struct Schedule {
  int unroll, cols, nt, blocks_per_launch;
  int buf = 0;  // 1: reduce_f32x4_buf_kernel (per-row buffer descriptors); blocks_per_launch 0 = resident blocks
};

// Round-split launches hold 3 blocks per CU (768 on the 256-CU MI355X); the
// CU count is read from the device, so a partitioned GPU (fewer CUs per
// device) keeps one resident round per launch.
constexpr int kBlocksPerCU = 3;
inline int blocks_per_launch() { return kBlocksPerCU * cu_count(); }

constexpr int64_t kManyClients = 64;  // K from which the wider short-row schedules apply

// `resident_rows`: bytes of the row buffer the caller streams (K x ld); the
// Infinity-Cache band applies only when that whole buffer fits the band, so a
// column chunk of a wider shard (N > 1 pipeline) streams from HBM instead.
Schedule choose_schedule(int64_t K, int64_t P, double resident_rows = -1.0) {
  const int64_t nvec = (P + 3) / 4;
  Schedule sc{8, 1, 1, blocks_per_launch()};
  const int64_t full = 2 * static_cast<int64_t>(cu_count());  // blocks for a full-chip launch (512 on MI355X)
  if (K <= 4) {
    // a block's work is tiny (K rows): one launch, many short blocks; round
    // splitting would only add launch boundaries (K=2..3 sweeps: +14-22 %)
    sc.cols = 1;
    sc.blocks_per_launch = 1 << 30;
  } else if (nvec >= full * kBlock * 8) {
    sc.unroll = 4, sc.cols = 8;
  } else if (nvec >= full * kBlock * 4) {
    sc.cols = 4;
  } else if (nvec >= full * kBlock * 2) {
    sc.cols = 2;
  } else {
    // short rows: few blocks, so each thread's client chain is the critical
    // path; deeper batches (16 rows) cut its round trips (+11-12 %), and with
    // many clients 4 slices per thread keep 64 loads in flight
    sc.unroll = 16;
    sc.cols = (K >= 500 && nvec >= full / 4 * kBlock * 4) ? 4 : 1;
  }
  const double bytes = 4.0 * static_cast<double>(K) * static_cast<double>(P);
  const double span_bytes = resident_rows > bytes ? resident_rows : bytes;
  if (K > 4 && bytes > 64.0 * (1 << 20) && span_bytes <= 240.0 * (1 << 20)) {
    // Infinity-Cache-resident band: default-policy loads, and a deep, wide
    // per-thread batch (16 rows x 4 slices) measured fastest there
    sc.nt = 0;
    sc.unroll = 16;
    sc.cols = 4;
  }
  return sc;
}

// The fp32 kernel's own refinement (the fp64/fp16/bf16 paths keep
// choose_schedule): rows long enough for a full-chip launch (2 blocks per
// CU) of 16-slice groups take U2 x C16 through per-row buffer descriptors
// (reduce_f32x4_buf_kernel, 32-bit lane offsets shared by every row):
// 7.09-7.15 vs 6.96-7.05 TB/s at K=100 x 25M and 6.89 vs 6.49 at K=100 x 10M,
// interleaved (scripts/buf_probe.py, profiles/r01_buf_probe*.jsonl); below
// that width the 16-slice groups leave the launch short of blocks (4.4 TB/s
// at K=100 x 5M).
Schedule choose_f32_schedule(int64_t K, int64_t P, int64_t ld) {
  // a chunk of a wider row buffer (ld > P) is not cache-resident between
  // calls: K=100 x 390K chunks of a 3.125M-column shard (the N=8 pipeline)
  // run 3,971 GB/s in the Infinity-Cache schedule and 5,065 streamed
  // (U16 x C1 nt; profiles/r01_chunk_rotating.jsonl)
  Schedule sc = choose_schedule(K, P, 4.0 * static_cast<double>(K) * static_cast<double>(ld > P ? ld : P));
  const int64_t nvec = (P + 3) / 4;
  const int64_t full = 2 * static_cast<int64_t>(cu_count());
  if (sc.nt && sc.unroll == 4 && sc.cols == 8 && nvec >= full * kBlock * 16) {
    sc.unroll = 2;
    sc.cols = 16;
    sc.buf = 1;
  }
  // Few clients (5 <= K < 64) on rows below the 8-slice band: per-row buffer
  // descriptors with 1-2 slices per thread and a launch of every resident
  // block.  rocprofv3 kernel time, variants interleaved in one process, two
  // sweeps (scripts/buf_probe.py; profiles/r02/sweeps/small_k_*.json):
  //   4-slice band (2.1M <= P < 4.2M): U8 x C2 -- K=5 x 2.4M 0.68-0.73 x the
  //     time of U8 x C4 (nt), K=10 x 2.4M 0.72-0.73 x U16 x C4 (Infinity-Cache
  //     band), K=32 / 50 x 2.4M 0.89 / 0.94 x;
  //   shorter rows, 8 <= K <= 32, P >= 262K: U8 x C1 -- K=10 x 1.2M (FEMNIST)
  //     0.88 x, K=10 x 300K 0.69-0.73 x, K=20 / 32 x 1.2M 0.81-0.85 / 0.73 x,
  //     K=32 x 300K 0.80 x; K=5 and K=50 gain nothing there.
  // (K >= 64 keeps the rules above, tuned on the all-gather chunk shapes.)
  if (K >= 5 && K < kManyClients && nvec < full * kBlock * 8) {
    if (nvec >= full * kBlock * 4) {
      sc = Schedule{8, 2, 1, 0, 1};
    } else if (K >= 8 && K <= 32 && nvec >= full * kBlock / 2) {
      sc = Schedule{8, 1, 1, 0, 1};
    }
  }
  // short rows with many clients (the N > 1 all-gather chunks): 4 slices per
  // thread -- K=100 x 1.56M (N=2 chunk) 6,695 vs 6,178 GB/s at U8 x C2, and
  // K=100 x 781K (N=4 chunk) 6,741 vs 5,668 at U16 x C1
  // (profiles/r01_chunk_shapes.jsonl, interleaved)
  if (sc.nt && K >= kManyClients) {
    if (sc.unroll == 8 && sc.cols == 2) sc.cols = 4;
    if (sc.unroll == 16 && sc.cols == 1 && nvec >= full / 4 * kBlock * 4) sc.cols = 4;
    // Rows that give 3/4 to 1 block per CU at 6 (K >= 64) or 3 (K >= 256)
    // slices per thread: one resident block on (nearly) every CU beats
    // 1.5 blocks per CU at 4 slices.  Rotating-chunk sweep, interleaved,
    // bit-identical (profiles/r02/sweeps/short_row_c3_c6.jsonl): K=100 x 1.56M
    // (the N=2 chunk) 6,822 vs 6,585 GB/s at U8 x C4; K=500 x 702K (cfg4's
    // N=8 chunk) 6,856 vs 6,627 at U16 x C4.  (K=100 x 781K keeps U16 x C4:
    // 6,527 vs 6,200 at C3.)
    const int64_t cus = cu_count();
    if (nvec >= cus * 3 / 4 * kBlock * 6 && nvec <= cus * kBlock * 6) {
      sc.unroll = 4;
      sc.cols = 6;
    } else if (K >= 256 && nvec >= cus * 3 / 4 * kBlock * 3 && nvec <= cus * kBlock * 3) {
      sc.unroll = 8;
      sc.cols = 3;
    }
  }
  return sc;
}

void launch_production_f32(const float* clients, int K, int64_t ld, int64_t P, const float* W, float* out,
                           hipStream_t s, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr) {
  const Schedule sc = choose_f32_schedule(K, P, ld);
  const int bpl = sc.blocks_per_launch;
  const int key = sc.unroll * 100 + sc.cols;
  if (sc.buf) {
    switch (key) {
      case 801: launch_split_buf<8, 1>(clients, K, ld, P, W, out, bpl, s, e0, e1); return;
      case 802: launch_split_buf<8, 2>(clients, K, ld, P, W, out, bpl, s, e0, e1); return;
      default: launch_split_buf<2, 16>(clients, K, ld, P, W, out, bpl, s, e0, e1); return;
    }
  }
  if (sc.nt) {
    switch (key) {
      case 408: launch_split_ev<4, 8, true>(clients, K, ld, P, W, out, bpl, s, e0, e1); return;
      case 804: launch_split_ev<8, 4, true>(clients, K, ld, P, W, out, bpl, s, e0, e1); return;
      case 802: launch_split_ev<8, 2, true>(clients, K, ld, P, W, out, bpl, s, e0, e1); return;
      case 1604: launch_split_ev<16, 4, true>(clients, K, ld, P, W, out, bpl, s, e0, e1); return;
      case 1601: launch_split_ev<16, 1, true>(clients, K, ld, P, W, out, bpl, s, e0, e1); return;
      case 406: launch_split_ev<4, 6, true>(clients, K, ld, P, W, out, bpl, s, e0, e1); return;
      case 803: launch_split_ev<8, 3, true>(clients, K, ld, P, W, out, bpl, s, e0, e1); return;
      default: launch_split_ev<8, 1, true>(clients, K, ld, P, W, out, bpl, s, e0, e1); return;
    }
  }
  switch (key) {
    case 408: launch_split_ev<4, 8, false>(clients, K, ld, P, W, out, bpl, s, e0, e1); return;
    case 804: launch_split_ev<8, 4, false>(clients, K, ld, P, W, out, bpl, s, e0, e1); return;
    case 802: launch_split_ev<8, 2, false>(clients, K, ld, P, W, out, bpl, s, e0, e1); return;
    case 1604: launch_split_ev<16, 4, false>(clients, K, ld, P, W, out, bpl, s, e0, e1); return;
    case 1601: launch_split_ev<16, 1, false>(clients, K, ld, P, W, out, bpl, s, e0, e1); return;
    default: launch_split_ev<8, 1, false>(clients, K, ld, P, W, out, bpl, s, e0, e1); return;
  }
}

// fp32 buffers that are not all 16-B aligned (or an odd row stride): the
// first-version kernels, same per-element order and bits.
int reduce_f32_unaligned(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights, float* out,
                         hipStream_t s, const char* what) {
  int rc = check_common(clients, K, P, ld, weights, out, what);
  if (rc) return rc;
  if (P == 0) return FEDAVG_OK;
  if (!aligned4(clients) || !aligned4(out) || !aligned4(weights))
    return set_error(FEDAVG_EALIGN, "%s: fp32 buffers must be 4-byte aligned", what);
  if (aligned16(clients) && (ld % 4) == 0) {
    launch_f32x4<8, true>(clients, static_cast<int>(K), ld, P, weights, out, s);  // handles an unaligned out
  } else {
    hipLaunchKernelGGL(reduce_f32_scalar_kernel, dim3(grid_for(P, kBlock)), dim3(kBlock), 0, s, clients,
                       static_cast<int>(K), ld, P, weights, out);
  }
  return launch_status(what);
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

// fp64 / fp16 / bf16 through per-row buffer descriptors (the fp32
// reduce_f32x4_buf_kernel's addressing: SGPR-held row bases, 32-bit lane
// offsets shared by every row) -- same per-element rules and order as
// reduce_vec_kernel, so the same bits; the ragged last group takes the
// global-pointer path.
template <class Op, int U, int C>
__global__ __launch_bounds__(kBlock) void reduce_vec_buf_kernel(
    const typename Op::vec* __restrict__ X, int K, int64_t ldv, int64_t nvec, int tail,
    const typename Op::wt* __restrict__ W, typename Op::elem* __restrict__ out) {
  using vec = typename Op::vec;
  static_assert(sizeof(vec) == 16, "16-B vectors");
  constexpr int64_t span = static_cast<int64_t>(kBlock) * C;
  constexpr int bytes = static_cast<int>(span * 16);
  uint32_t off[C];
#pragma unroll
  for (int j = 0; j < C; ++j) off[j] = 16u * (threadIdx.x + j * kBlock);
  for (int64_t base = static_cast<int64_t>(blockIdx.x) * span; base < nvec;
       base += static_cast<int64_t>(gridDim.x) * span) {
    if (base + span <= nvec) {
      vec acc[C];
      {
        const __amdgpu_buffer_rsrc_t r0 = uniform_rsrc(X + base, bytes);
        const typename Op::wt w0 = W[0];
#pragma unroll
        for (int j = 0; j < C; ++j) acc[j] = Op::first(__builtin_bit_cast(vec, ld_rsrc_nt(r0, off[j])), w0);
      }
      int k = 1;
      for (; k + U <= K; k += U) {
        vec xs[U][C];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const __amdgpu_buffer_rsrc_t r = uniform_rsrc(X + static_cast<int64_t>(k + u) * ldv + base, bytes);
#pragma unroll
          for (int j = 0; j < C; ++j) xs[u][j] = __builtin_bit_cast(vec, ld_rsrc_nt(r, off[j]));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const typename Op::wt w = W[k + u];
#pragma unroll
          for (int j = 0; j < C; ++j) acc[j] = Op::step(acc[j], xs[u][j], w);
        }
      }
      for (; k < K; ++k) {
        const __amdgpu_buffer_rsrc_t r = uniform_rsrc(X + static_cast<int64_t>(k) * ldv + base, bytes);
        const typename Op::wt w = W[k];
#pragma unroll
        for (int j = 0; j < C; ++j) acc[j] = Op::step(acc[j], __builtin_bit_cast(vec, ld_rsrc_nt(r, off[j])), w);
      }
#pragma unroll
      for (int j = 0; j < C; ++j) store_vec<Op>(out, base + threadIdx.x + j * kBlock, nvec, tail, acc[j]);
    } else {
      for (int j = 0; j < C; ++j) {
        const int64_t v = base + threadIdx.x + j * kBlock;
        if (v >= nvec) break;
        vec acc1[1];
        reduce_vec_group<Op, U, 1, true>(acc1, X + v, K, ldv, W);
        store_vec<Op>(out, v, nvec, tail, acc1[0]);
      }
    }
  }
}

template <class Op, int U, int C>
void launch_vec_split_buf(const void* clients, int K, int64_t ld, int64_t P, const void* W, void* out, int bpl,
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
    hipLaunchKernelGGL((reduce_vec_buf_kernel<Op, U, C>), dim3(static_cast<unsigned>((n + span - 1) / span)),
                       dim3(kBlock), 0, s, X + v0, K, ld / lanes, n, tail,
                       reinterpret_cast<const typename Op::wt*>(W), O + v0 * lanes);
  }
}

template <class Op>
bool launch_vec_buf(int U, int C, const void* clients, int K, int64_t ld, int64_t P, const void* W, void* out,
                    int bpl, hipStream_t s) {
  switch (U * 100 + C) {
    case 804: launch_vec_split_buf<Op, 8, 4>(clients, K, ld, P, W, out, bpl, s); return true;
    case 408: launch_vec_split_buf<Op, 4, 8>(clients, K, ld, P, W, out, bpl, s); return true;
    case 216: launch_vec_split_buf<Op, 2, 16>(clients, K, ld, P, W, out, bpl, s); return true;
    case 404: launch_vec_split_buf<Op, 4, 4>(clients, K, ld, P, W, out, bpl, s); return true;
    case 208: launch_vec_split_buf<Op, 2, 8>(clients, K, ld, P, W, out, bpl, s); return true;
    default: return false;
  }
}

// fp16/bf16 schedule from the fp32 one for the same bytes per row.  Each 16-B
// vector unpacks into 8 fp32 lanes of work, so the deep fp32 batches are cut
// to stay spill-free -- except the large-P key: there the packed kernel wants
// the fp32 kernel's 32 x 16-B loads in flight per thread as U8 x C4 (158
// VGPRs), not U2 x C8 (16 loads): 6,543 vs 5,896 GB/s at K=100 x P=25M bf16
// and 6,641 vs 6,595 at K=500 x P=11.2M (profiles/sweeps/r01_half_*.jsonl).
inline int half_key(int key) {
  switch (key) {
    case 408: return 804;
    case 804: case 1604: return 404;
    case 1601: return 801;
    default: return key;
  }
}

template <class Op, bool NT>
void launch_vec_nt(const Schedule& sc, const void* clients, int K, int64_t ld, int64_t P, const void* W, void* out,
                   hipStream_t s) {
  int key = sc.unroll * 100 + sc.cols;
  if constexpr (Op::kLanes == 8) key = half_key(key);
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

#ifdef FEDAVG_TUNING
// Conversion probe (tests only): out[i] = the 16-bit rounding of the fp32
// bit pattern in[i] by mode 0 = BF16Pk (hardware), 1 = c10 integer RNE,
// 2 = F16Pk (hardware, packed), 3 = F16Rule (scalar v_cvt_f16_f32).
__global__ __launch_bounds__(kBlock) void probe_cvt16_kernel(const unsigned int* __restrict__ in, int64_t n,
                                                            int mode, unsigned short* __restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  const float f = __uint_as_float(in[i]);
  const f32x2 f2{f, 0.f};
  unsigned short h;
  switch (mode) {
    case 0: h = static_cast<unsigned short>(BF16Pk::pack(opaque2(f2)) & 0xFFFFu); break;
    case 1: h = BF16Rule::from_f32(opaque(f)); break;
    case 2: h = static_cast<unsigned short>(F16Pk::pack(opaque2(f2)) & 0xFFFFu); break;
    default: h = F16Rule::from_f32(opaque(f)); break;
  }
  out[i] = h;
}

#endif  // FEDAVG_TUNING

// elem_bytes: 8 (fp64) or 2 (fp16/bf16).  The fp32 schedule is chosen for the
// problem with the same 16-B slice count and byte footprint.
template <class Op>
void launch_production_vec(const void* clients, int K, int64_t ld, int64_t P, const void* W, void* out,
                           hipStream_t s) {
  const int64_t f32_equiv = P * static_cast<int64_t>(16 / Op::kLanes) / 4;  // same bytes per row
  if constexpr (Op::kLanes == 2) {
    // fp64 follows the fp32 kernel onto per-row buffer descriptors for long
    // rows: 7,113 vs 6,992 GB/s at K=100 x 12.5M fp64 (scripts/vec_buf_probe.py,
    // profiles/r01_vec_buf_probe.jsonl).  fp16/bf16 measured no gain (+0-1 %).
    const Schedule f = choose_f32_schedule(K, f32_equiv, ld * static_cast<int64_t>(16 / Op::kLanes) / 4);
    if (f.cols == 16) {
      launch_vec_split_buf<Op, 2, 16>(clients, K, ld, P, W, out, f.blocks_per_launch, s);
      return;
    }
  }
  const int64_t ld_equiv = ld * static_cast<int64_t>(16 / Op::kLanes) / 4;
  const Schedule sc = choose_schedule(K, f32_equiv, 4.0 * static_cast<double>(K) * static_cast<double>(ld_equiv));
  if (sc.nt)
    launch_vec_nt<Op, true>(sc, clients, K, ld, P, W, out, s);
  else
    launch_vec_nt<Op, false>(sc, clients, K, ld, P, W, out, s);
}

// Benchmarking hook (fedavg_reduce_half_variant): the packed fp16/bf16 kernel
// with an explicit (rows per batch U, 16-B slices per thread C) schedule,
// nontemporal loads and round-split at max_blocks blocks per launch.
template <class Op>
bool launch_half_variant(int U, int C, const void* clients, int K, int64_t ld, int64_t P, const void* W, void* out,
                         int bpl, hipStream_t s) {
  switch (U * 100 + C) {
    case 208: launch_vec_split<Op, 2, 8, true>(clients, K, ld, P, W, out, bpl, s); return true;
    case 408: launch_vec_split<Op, 4, 8, true>(clients, K, ld, P, W, out, bpl, s); return true;
    case 108: launch_vec_split<Op, 1, 8, true>(clients, K, ld, P, W, out, bpl, s); return true;
    case 404: launch_vec_split<Op, 4, 4, true>(clients, K, ld, P, W, out, bpl, s); return true;
    case 204: launch_vec_split<Op, 2, 4, true>(clients, K, ld, P, W, out, bpl, s); return true;
    case 804: launch_vec_split<Op, 8, 4, true>(clients, K, ld, P, W, out, bpl, s); return true;
    case 802: launch_vec_split<Op, 8, 2, true>(clients, K, ld, P, W, out, bpl, s); return true;
    case 402: launch_vec_split<Op, 4, 2, true>(clients, K, ld, P, W, out, bpl, s); return true;
    case 116: launch_vec_split<Op, 1, 16, true>(clients, K, ld, P, W, out, bpl, s); return true;
    case 216: launch_vec_split<Op, 2, 16, true>(clients, K, ld, P, W, out, bpl, s); return true;
    case 1601: launch_vec_split<Op, 16, 1, true>(clients, K, ld, P, W, out, bpl, s); return true;
    default: return false;
  }
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int fedavg_abi_version(void) { return 1; }

#ifdef FEDAVG_TUNING  // probe library only (libfedavg_amd_probe.so)
int fedavg_probe_cvt16(const uint32_t* in, int64_t n, int mode, uint16_t* out, void* stream) {
  if (n < 0 || !in || !out || mode < 0 || mode > 3)
    return set_error(FEDAVG_EINVAL, "fedavg_probe_cvt16: bad arguments");
  if (n == 0) return FEDAVG_OK;
  hipLaunchKernelGGL(probe_cvt16_kernel, dim3(static_cast<unsigned>((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), in, n, mode, out);
  return launch_status("fedavg_probe_cvt16");
}
#endif  // FEDAVG_TUNING

const char* fedavg_last_error(void) { return last_error_message(); }

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
  return reduce_f32_unaligned(clients, K, P, ld, weights, out, static_cast<hipStream_t>(stream), what);
}

int fedavg_reduce_f32_timed(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights,
                            float* out, void* stream, void* start_event, void* stop_event) {
  const char* what = "fedavg_reduce_f32_timed";
  if (!start_event || !stop_event) return set_error(FEDAVG_EINVAL, "%s: both events are required", what);
  if (!(aligned16(clients) && aligned16(out) && (ld % 4) == 0 && P > 0 && K > 0))
    return set_error(FEDAVG_EALIGN, "%s: the production (16-B aligned, P > 0) path only", what);
  int rc = check_common(clients, K, P, ld, weights, out, what);
  if (rc) return rc;
  if (!aligned4(weights)) return set_error(FEDAVG_EALIGN, "%s: weights must be 4-byte aligned", what);
  launch_production_f32(clients, static_cast<int>(K), ld, P, weights, out, static_cast<hipStream_t>(stream),
                        static_cast<hipEvent_t>(start_event), static_cast<hipEvent_t>(stop_event));
  return launch_status(what);
}

namespace {
// launches of launch_production_f32 for this schedule (buffer-descriptor
// schedules without a cap launch every resident block at once)
int production_launches(const Schedule& sc, int64_t P) {
  const int64_t nvec = (P + 3) / 4;
  const int64_t span = static_cast<int64_t>(kBlock) * sc.cols;
  const int64_t blocks = (nvec + span - 1) / span;
  int64_t per = sc.blocks_per_launch;
  if (per <= 0) {
    switch (sc.unroll * 100 + sc.cols) {
      case 801: per = resident_blocks(reduce_f32x4_buf_kernel<8, 1, kBlock, 0>, kBlock); break;
      case 802: per = resident_blocks(reduce_f32x4_buf_kernel<8, 2, kBlock, 0>, kBlock); break;
      default: per = resident_blocks(reduce_f32x4_buf_kernel<2, 16, kBlock, 0>, kBlock); break;
    }
  }
  return static_cast<int>((blocks + per - 1) / per);
}

void report_schedule(const Schedule& sc, int64_t P, int* unroll, int* cols, int* nontemporal, int* launches) {
  if (unroll) *unroll = sc.unroll;
  if (cols) *cols = sc.cols;
  if (nontemporal) *nontemporal = sc.buf ? 2 : sc.nt;
  if (launches) *launches = production_launches(sc, P);
}
}  // namespace

int fedavg_f32_schedule_ld(int64_t K, int64_t P, int64_t ld, int* unroll, int* cols, int* nontemporal,
                           int* launches) {
  if (K <= 0 || P < 0 || ld < P) return set_error(FEDAVG_EINVAL, "fedavg_f32_schedule_ld: bad sizes");
  report_schedule(choose_f32_schedule(K, P, ld), P, unroll, cols, nontemporal, launches);
  return FEDAVG_OK;
}

int fedavg_f32_schedule(int64_t K, int64_t P, int* unroll, int* cols, int* nontemporal, int* launches) {
  if (K <= 0 || P < 0) return set_error(FEDAVG_EINVAL, "fedavg_f32_schedule: bad sizes");
  report_schedule(choose_f32_schedule(K, P, P), P, unroll, cols, nontemporal, launches);
  return FEDAVG_OK;
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
      launch_production_vec<OpHalfPk<BF16Pk>>(clients, static_cast<int>(K), ld, P, weights, out, s);
    else
      launch_production_vec<OpHalfPk<F16Pk>>(clients, static_cast<int>(K), ld, P, weights, out, s);
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

#ifdef FEDAVG_TUNING  // probe library only (libfedavg_amd_probe.so)
int fedavg_reduce_vec_buf(int dtype, const void* clients, int64_t K, int64_t P, int64_t ld, const void* weights,
                          void* out, int unroll, int cols, int max_blocks, void* stream) {
  const char* what = "fedavg_reduce_vec_buf";
  int rc = check_common(clients, K, P, ld, weights, out, what);
  if (rc) return rc;
  if (P == 0) return FEDAVG_OK;
  const int lanes = dtype == 2 ? 2 : 8;
  if (dtype < 0 || dtype > 2) return set_error(FEDAVG_EMODE, "%s: dtype must be 0 (f16), 1 (bf16) or 2 (f64)", what);
  if (!aligned16(clients) || !aligned16(out) || (ld % lanes) != 0)
    return set_error(FEDAVG_EALIGN, "%s: needs 16-B aligned clients/out and ld %% %d == 0", what, lanes);
  const int bpl = max_blocks > 0 ? max_blocks : (1 << 30);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int k = static_cast<int>(K);
  bool ok;
  if (dtype == 2)
    ok = launch_vec_buf<OpF64>(unroll, cols, clients, k, ld, P, weights, out, bpl, s);
  else if (dtype == 1)
    ok = launch_vec_buf<OpHalfPk<BF16Pk>>(unroll, cols, clients, k, ld, P, weights, out, bpl, s);
  else
    ok = launch_vec_buf<OpHalfPk<F16Pk>>(unroll, cols, clients, k, ld, P, weights, out, bpl, s);
  if (!ok) return set_error(FEDAVG_EMODE, "%s: unsupported unroll=%d cols=%d", what, unroll, cols);
  return launch_status(what);
}
#endif  // FEDAVG_TUNING

#ifdef FEDAVG_TUNING  // probe library only (libfedavg_amd_probe.so)
int fedavg_reduce_half_variant(int bf16, const uint16_t* clients, int64_t K, int64_t P, int64_t ld,
                               const float* weights, uint16_t* out, int unroll, int cols, int max_blocks,
                               void* stream) {
  const char* what = "fedavg_reduce_half_variant";
  int rc = check_common(clients, K, P, ld, weights, out, what);
  if (rc) return rc;
  if (P == 0) return FEDAVG_OK;
  if (!aligned16(clients) || !aligned16(out) || (ld % 8) != 0)
    return set_error(FEDAVG_EALIGN, "%s: needs 16-B aligned clients/out and ld %% 8 == 0", what);
  const int bpl = max_blocks > 0 ? max_blocks : (1 << 30);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool ok = bf16 ? launch_half_variant<OpHalfPk<BF16Pk>>(unroll, cols, clients, static_cast<int>(K), ld, P,
                                                               weights, out, bpl, s)
                       : launch_half_variant<OpHalfPk<F16Pk>>(unroll, cols, clients, static_cast<int>(K), ld, P,
                                                              weights, out, bpl, s);
  if (!ok) return set_error(FEDAVG_EMODE, "%s: unsupported unroll=%d cols=%d", what, unroll, cols);
  return launch_status(what);
}
#endif  // FEDAVG_TUNING

#ifdef FEDAVG_TUNING  // probe library only (libfedavg_amd_probe.so)
int fedavg_half_schedule(int64_t K, int64_t P, int* unroll, int* cols, int* nontemporal, int* launches) {
  if (K <= 0 || P < 0) return set_error(FEDAVG_EINVAL, "fedavg_half_schedule: bad sizes");
  const Schedule sc = choose_schedule(K, P * 2 / 4);  // the fp32 problem with the same bytes per row
  const int key = half_key(sc.unroll * 100 + sc.cols);
  const int64_t nvec = (P + 7) / 8;
  const int64_t span = static_cast<int64_t>(kBlock) * (key % 100);
  const int64_t blocks = (nvec + span - 1) / span;
  if (unroll) *unroll = key / 100;
  if (cols) *cols = key % 100;
  if (nontemporal) *nontemporal = sc.nt;
  if (launches) *launches = static_cast<int>((blocks + sc.blocks_per_launch - 1) / sc.blocks_per_launch);
  return FEDAVG_OK;
}
#endif  // FEDAVG_TUNING

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

// A whole small round in ONE host call (the drop-in's path for models whose
// K x ld rows fit in a few MB, e.g. the reference's own MNIST-LR config): pack
// the clients' keys into the pinned rows (fedavg_pack_rows), round the
// weights to fp32, then one launch of round_small_f32x4_kernel (rows read
// from pinned memory and kept in HBM, reduce, result to HBM and to pinned
// memory) and wait.  The same steps through Python/torch cost ~100 us of host
// overhead per call.  Buffers: host_rows/host_w/host_out pinned host memory;
// dev_rows [K, ld], dev_w [K], dev_out [P] device memory (ld % 4 == 0,
// 16-B aligned).
int fedavg_round_f32(const fedavg_pack_item* items, int64_t n_items, float* host_rows, float* dev_rows, int64_t K,
                     int64_t P, int64_t ld, const double* weights, float* host_w, float* dev_w, float* dev_out,
                     float* host_out, int n_threads, void* stream) {
  const char* what = "fedavg_round_f32";
  int rc = check_common(dev_rows, K, P, ld, dev_w, dev_out, what);
  if (rc) return rc;
  if (P == 0) return FEDAVG_OK;
  if (!host_rows || !weights || !host_w || !host_out || (n_items > 0 && !items))
    return set_error(FEDAVG_EINVAL, "%s: null buffer", what);
  if (!aligned16(dev_rows) || !aligned16(dev_out) || (ld % 4) != 0 || !aligned4(dev_w))
    return set_error(FEDAVG_EALIGN, "%s: needs 16-B aligned dev_rows/dev_out and ld %% 4 == 0", what);
  rc = fedavg_pack_rows(items, n_items, host_rows, 4, n_threads);
  if (rc) return set_error(rc, "%s: bad pack items", what);
  for (int64_t i = 0; i < K; ++i) host_w[i] = static_cast<float>(weights[i]);  // ATen's scalar cast (:455)
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (!aligned16(host_rows) || !aligned16(host_out) || !aligned4(host_w))
    return set_error(FEDAVG_EALIGN, "%s: host_rows/host_out must be 16-B aligned", what);
  const int64_t nvec = (P + 3) / 4;
  hipLaunchKernelGGL(round_small_f32x4_kernel<16>, dim3(grid_for(nvec, kBlock)), dim3(kBlock), 0, s,
                     reinterpret_cast<const f32x4*>(host_rows), reinterpret_cast<f32x4*>(dev_rows),
                     static_cast<int>(K), ld / 4, nvec, static_cast<int>(P & 3), host_w, dev_w, dev_out, host_out);
  rc = launch_status(what);
  if (rc) return rc;
  const hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return set_error(-static_cast<int>(e), "%s: %s", what, hipGetErrorString(e));
  }
  return FEDAVG_OK;
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
