// common.hpp -- shared device code of libfedavg_amd.so (gfx950 / MI355X).
//
// Reference semantics (src/fedavg_trainer.py:441-458): for each element p,
//     acc = x[0][p] * w[0];  acc = acc + x[i][p] * w[i]  for i = 1..K-1
// evaluated left to right, one rounding per multiply and per add.  Every
// translation unit is compiled with -ffp-contract=off and this header pins
// `fp contract(off)` as well, so the multiply+add pair is never fused into
// v_fma/v_fmac (a fused form rounds once and is not bit-identical to the
// reference's ATen CPU ops).
//
// Roofline: 2 flops per 4-byte element read -> 0.5 flop/B; the kernels are
// HBM-read bound (4*K*P bytes in, 4*P out), never MFMA work.  Layout in HBM:
// one client-major [K, ld] buffer, each row one client's flattened
// state_dict.  A thread owns C 16-byte column slices (slice j at
// base + tid + 256*j) and walks the client axis in order, U rows per batch.
//
// Translation units: fedavg_reduce.hip (production kernels, schedule, C ABI),
// fedavg_variants.hip (benchmarking variants), fedavg_dist.hip (the :291
// distance pass).  Templates and inline helpers live here.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <tuple>
#include <mutex>
#include <utility>

#include "fedavg_amd.h"
#include "fedavg_amd_tuning.h"

#pragma clang fp contract(off)

namespace fedavg_impl {

constexpr int kBlock = 256;  // 4 waves of 64

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

// Packed 16-bit element rules (fp16 / bf16), shared by the reduce
// (fedavg_reduce.hip) and the distance pass (fedavg_dist.hip): two elements
// per 32-bit word, fp32 math on the pair, gfx950's two-at-a-time RNE
// conversions (v_cvt_pk_f16_f32 / v_cvt_pk_bf16_f32).  opaque2 keeps the
// compiler from fusing fpext -> op -> fptrunc into one mixed-precision op
// (which would round once instead of fp32-then-16-bit, as ATen does).
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x2 opaque2(f32x2 v) {
  asm volatile("" : "+v"(v));
  return v;
}

struct BF16Pk {
  __device__ static f32x2 unpack(unsigned int u) {
    return f32x2{__uint_as_float(u << 16), __uint_as_float(u & 0xFFFF0000u)};
  }
  __device__ static unsigned int pack(f32x2 f) {
    const bf16x2 b = __builtin_convertvector(f, bf16x2);
    unsigned int u;
    __builtin_memcpy(&u, &b, 4);
    return u;
  }
  __device__ static unsigned short canon(unsigned short h) { return (h & 0x7FFFu) > 0x7F80u ? 0x7FC0u : h; }
};

struct F16Pk {
  __device__ static f32x2 unpack(unsigned int u) {
    f16x2 h;
    __builtin_memcpy(&h, &u, 4);
    return __builtin_convertvector(h, f32x2);
  }
  __device__ static unsigned int pack(f32x2 f) {
    const f16x2 h = __builtin_convertvector(f, f16x2);
    unsigned int u;
    __builtin_memcpy(&u, &h, 4);
    return u;
  }
  __device__ static unsigned short canon(unsigned short h) { return h; }  // NaN payloads are not specified
};

// Error state (thread-local message), defined in fedavg_reduce.hip.
int set_error(int code, const char* fmt, ...);
int launch_status(const char* what);
const char* last_error_message();
int check_common(const void* clients, int64_t K, int64_t P, int64_t ld, const void* weights, const void* out,
                 const char* what);

__host__ __device__ inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
__host__ __device__ inline bool aligned4(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 3u) == 0; }

// hipPointerGetAttributes: is p device memory / pinned host memory of the
// runtime (host-side checks before a kernel dereferences caller addresses)
inline bool is_device_memory(const void* p) {
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return attr.type == hipMemoryTypeDevice;
}

inline bool is_pinned_host_memory(const void* p) {
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return attr.type == hipMemoryTypeHost;
}

// The largest i in [0, n) with start(i) <= g, for a nondecreasing start()
// with start(0) <= g: 64 probes per round across the wave, ballot, keep the
// last hit (a few rounds instead of a binary search's ~15 dependent loads for
// tables of tens of thousands of entries).  Every lane returns the same i.
template <typename Start>
__device__ __forceinline__ int64_t wave_search_last_le(Start start, int64_t n, int64_t g) {
  const int lane = static_cast<int>(threadIdx.x & 63u);
  int64_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const int64_t step = (hi - lo + 63) / 64;
    const int64_t idx = lo + lane * step;
    const bool hit = idx < hi && start(idx) <= g;
    const unsigned long long m = __ballot(hit);
    lo += (63 - __clzll(m)) * step;
    hi = hi < lo + step ? hi : lo + step;
  }
  return lo;
}

// Wave-wide fp64 sum through DPP lane moves (VALU, no LDS round trips):
// quad_perm [1,0,3,2] and [2,3,0,1] make quad sums, row_half_mirror and
// row_mirror make 16-lane row sums, row_bcast:15 (rows 1, 3) and row_bcast:31
// (rows 2, 3) carry them up to row 3; lane 63 then holds the total, read
// back as a wave-uniform value.  A __shfl_xor tree (ds_bpermute, an LDS
// round trip per step, 12 per fp64 sum) serialises ~6 LDS latencies per sum;
// the per-client sums of the :291 pass do one per client row.  Same addends,
// fixed order: deterministic, but not the shfl tree's bits.
// Timeline probes of the split windows (MODE 8): lane 0 of every wave of the
// first kStampBlocks workgroups stores s_memtime at up to kStampSlots points
// of its first kStampWins windows, after the K x G partials, behind a magic
// word (scripts/winn_timeline.py reads them)
constexpr int kStampBlocks = 8, kStampWins = 48, kStampSlots = 8;
constexpr uint64_t kStampMagic = 0x504D415453ull;  // "STAMP"
inline int64_t winn_stamp_elems(int nsmax) { return 1 + int64_t(kStampBlocks) * nsmax * kStampWins * kStampSlots; }

// f(std::integral_constant<int, I>{}) for I = 0 .. N-1, unrolled at compile
// time (DPP controls must be constants)
template <class F, int... Is>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// The sequential fp32 chain a = fl32(a + fl32(w_i x_i)) over 8 rows whose
// weights are lanes of one register: row i's weight is lane 16r + i % 16 of w,
// broadcast over its 16-lane row r by the multiply's own DPP operand
// (row_newbcast).  Software-pipelined by hand: the product of the block's
// first row arrives in tc, each add reads a product issued two instructions
// earlier, and tc leaves with the product of the next block's first row
// (lane 0 or 8, of wn when the next row starts a new 16).  The compiler's DPP
// combiner keeps row_newbcast as a separate v_mov_b32_dpp (and an s_nop after
// every inline v_mul), so the block is written out.  H = 0: rows of lanes
// 0..7, H = 1: lanes 8..15; LAST: no next row.
template <int H, bool LAST>
__device__ __forceinline__ void chain8_row_bcast(float& a, float& tc, float w, float wn, const float* x) {
  float t1;
#define FEDAVG_C8_MUL(T, X, L) "v_mul_f32_dpp " T ", %[w], " X " row_newbcast:" #L " row_mask:0xf bank_mask:0xf\n\t"
#define FEDAVG_C8_ADD(T) "v_add_f32_e32 %[a], %[a], " T "\n\t"
  if constexpr (H == 0) {
    if constexpr (LAST) {
      asm(FEDAVG_C8_MUL("%[t1]", "%[x1]", 1) FEDAVG_C8_ADD("%[tc]") FEDAVG_C8_MUL("%[tc]", "%[x2]", 2)
              FEDAVG_C8_ADD("%[t1]") FEDAVG_C8_MUL("%[t1]", "%[x3]", 3) FEDAVG_C8_ADD("%[tc]")
                  FEDAVG_C8_MUL("%[tc]", "%[x4]", 4) FEDAVG_C8_ADD("%[t1]") FEDAVG_C8_MUL("%[t1]", "%[x5]", 5)
                      FEDAVG_C8_ADD("%[tc]") FEDAVG_C8_MUL("%[tc]", "%[x6]", 6) FEDAVG_C8_ADD("%[t1]")
                          FEDAVG_C8_MUL("%[t1]", "%[x7]", 7) FEDAVG_C8_ADD("%[tc]") FEDAVG_C8_ADD("%[t1]")
          : [a] "+v"(a), [tc] "+v"(tc), [t1] "=&v"(t1)
          : [w] "v"(w), [x1] "v"(x[1]), [x2] "v"(x[2]), [x3] "v"(x[3]), [x4] "v"(x[4]), [x5] "v"(x[5]),
            [x6] "v"(x[6]), [x7] "v"(x[7]));
    } else {
      asm(FEDAVG_C8_MUL("%[t1]", "%[x1]", 1) FEDAVG_C8_ADD("%[tc]") FEDAVG_C8_MUL("%[tc]", "%[x2]", 2)
              FEDAVG_C8_ADD("%[t1]") FEDAVG_C8_MUL("%[t1]", "%[x3]", 3) FEDAVG_C8_ADD("%[tc]")
                  FEDAVG_C8_MUL("%[tc]", "%[x4]", 4) FEDAVG_C8_ADD("%[t1]") FEDAVG_C8_MUL("%[t1]", "%[x5]", 5)
                      FEDAVG_C8_ADD("%[tc]") FEDAVG_C8_MUL("%[tc]", "%[x6]", 6) FEDAVG_C8_ADD("%[t1]")
                          FEDAVG_C8_MUL("%[t1]", "%[x7]", 7) FEDAVG_C8_ADD("%[tc]")
                              FEDAVG_C8_MUL("%[tc]", "%[x8]", 8) FEDAVG_C8_ADD("%[t1]")
          : [a] "+v"(a), [tc] "+v"(tc), [t1] "=&v"(t1)
          : [w] "v"(w), [x1] "v"(x[1]), [x2] "v"(x[2]), [x3] "v"(x[3]), [x4] "v"(x[4]), [x5] "v"(x[5]),
            [x6] "v"(x[6]), [x7] "v"(x[7]), [x8] "v"(x[8]));
    }
  } else {
    if constexpr (LAST) {
      asm(FEDAVG_C8_MUL("%[t1]", "%[x1]", 9) FEDAVG_C8_ADD("%[tc]") FEDAVG_C8_MUL("%[tc]", "%[x2]", 10)
              FEDAVG_C8_ADD("%[t1]") FEDAVG_C8_MUL("%[t1]", "%[x3]", 11) FEDAVG_C8_ADD("%[tc]")
                  FEDAVG_C8_MUL("%[tc]", "%[x4]", 12) FEDAVG_C8_ADD("%[t1]") FEDAVG_C8_MUL("%[t1]", "%[x5]", 13)
                      FEDAVG_C8_ADD("%[tc]") FEDAVG_C8_MUL("%[tc]", "%[x6]", 14) FEDAVG_C8_ADD("%[t1]")
                          FEDAVG_C8_MUL("%[t1]", "%[x7]", 15) FEDAVG_C8_ADD("%[tc]") FEDAVG_C8_ADD("%[t1]")
          : [a] "+v"(a), [tc] "+v"(tc), [t1] "=&v"(t1)
          : [w] "v"(w), [x1] "v"(x[1]), [x2] "v"(x[2]), [x3] "v"(x[3]), [x4] "v"(x[4]), [x5] "v"(x[5]),
            [x6] "v"(x[6]), [x7] "v"(x[7]));
    } else {
      asm(FEDAVG_C8_MUL("%[t1]", "%[x1]", 9) FEDAVG_C8_ADD("%[tc]") FEDAVG_C8_MUL("%[tc]", "%[x2]", 10)
              FEDAVG_C8_ADD("%[t1]") FEDAVG_C8_MUL("%[t1]", "%[x3]", 11) FEDAVG_C8_ADD("%[tc]")
                  FEDAVG_C8_MUL("%[tc]", "%[x4]", 12) FEDAVG_C8_ADD("%[t1]") FEDAVG_C8_MUL("%[t1]", "%[x5]", 13)
                      FEDAVG_C8_ADD("%[tc]") FEDAVG_C8_MUL("%[tc]", "%[x6]", 14) FEDAVG_C8_ADD("%[t1]")
                          FEDAVG_C8_MUL("%[t1]", "%[x7]", 15) FEDAVG_C8_ADD("%[tc]")
                              "v_mul_f32_dpp %[tc], %[wn], %[x8] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
                                  FEDAVG_C8_ADD("%[t1]")
          : [a] "+v"(a), [tc] "+v"(tc), [t1] "=&v"(t1)
          : [w] "v"(w), [wn] "v"(wn), [x1] "v"(x[1]), [x2] "v"(x[2]), [x3] "v"(x[3]), [x4] "v"(x[4]),
            [x5] "v"(x[5]), [x6] "v"(x[6]), [x7] "v"(x[7]), [x8] "v"(x[8]));
    }
  }
#undef FEDAVG_C8_MUL
#undef FEDAVG_C8_ADD
}

// chain8_row_bcast for two columns per lane (window VEC 2): the rows' two
// products by the broadcast weight, then the two columns' adds of the row
// before (four instructions a row, each add reading a product issued four
// instructions earlier).  The block text is generated (rows 1..7, + row 8's
// product unless LAST).
template <int H, bool LAST, class V2>
__device__ __forceinline__ void chain8_row_bcast2(float& a0, float& a1, float& tc0, float& tc1, float w, float wn,
                                                  const V2* x) {
  float t10, t11;
  if constexpr (H == 0 && LAST) {
    asm("v_mul_f32_dpp %[t10], %[w], %[x10] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[t11], %[w], %[x11] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[tc0]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[tc1]\n\t"
          "v_mul_f32_dpp %[tc0], %[w], %[x20] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[tc1], %[w], %[x21] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[t10]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[t11]\n\t"
          "v_mul_f32_dpp %[t10], %[w], %[x30] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[t11], %[w], %[x31] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[tc0]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[tc1]\n\t"
          "v_mul_f32_dpp %[tc0], %[w], %[x40] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[tc1], %[w], %[x41] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[t10]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[t11]\n\t"
          "v_mul_f32_dpp %[t10], %[w], %[x50] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[t11], %[w], %[x51] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[tc0]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[tc1]\n\t"
          "v_mul_f32_dpp %[tc0], %[w], %[x60] row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[tc1], %[w], %[x61] row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[t10]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[t11]\n\t"
          "v_mul_f32_dpp %[t10], %[w], %[x70] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[t11], %[w], %[x71] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[tc0]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[tc1]\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[t10]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[t11]\n\t"
        : [a0] "+v"(a0), [a1] "+v"(a1), [tc0] "+v"(tc0), [tc1] "+v"(tc1), [t10] "=&v"(t10), [t11] "=&v"(t11)
        : [w] "v"(w), [x10] "v"(x[1][0]), [x11] "v"(x[1][1]), [x20] "v"(x[2][0]), [x21] "v"(x[2][1]), [x30] "v"(x[3][0]), [x31] "v"(x[3][1]), [x40] "v"(x[4][0]), [x41] "v"(x[4][1]), [x50] "v"(x[5][0]), [x51] "v"(x[5][1]), [x60] "v"(x[6][0]), [x61] "v"(x[6][1]), [x70] "v"(x[7][0]), [x71] "v"(x[7][1]));
  } else if constexpr (H == 0) {
    asm("v_mul_f32_dpp %[t10], %[w], %[x10] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[t11], %[w], %[x11] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[tc0]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[tc1]\n\t"
          "v_mul_f32_dpp %[tc0], %[w], %[x20] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[tc1], %[w], %[x21] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[t10]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[t11]\n\t"
          "v_mul_f32_dpp %[t10], %[w], %[x30] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[t11], %[w], %[x31] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[tc0]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[tc1]\n\t"
          "v_mul_f32_dpp %[tc0], %[w], %[x40] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[tc1], %[w], %[x41] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[t10]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[t11]\n\t"
          "v_mul_f32_dpp %[t10], %[w], %[x50] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[t11], %[w], %[x51] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[tc0]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[tc1]\n\t"
          "v_mul_f32_dpp %[tc0], %[w], %[x60] row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[tc1], %[w], %[x61] row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[t10]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[t11]\n\t"
          "v_mul_f32_dpp %[t10], %[w], %[x70] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[t11], %[w], %[x71] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[tc0]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[tc1]\n\t"
          "v_mul_f32_dpp %[tc0], %[w], %[x80] row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[tc1], %[w], %[x81] row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[t10]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[t11]\n\t"
        : [a0] "+v"(a0), [a1] "+v"(a1), [tc0] "+v"(tc0), [tc1] "+v"(tc1), [t10] "=&v"(t10), [t11] "=&v"(t11)
        : [w] "v"(w), [x10] "v"(x[1][0]), [x11] "v"(x[1][1]), [x20] "v"(x[2][0]), [x21] "v"(x[2][1]), [x30] "v"(x[3][0]), [x31] "v"(x[3][1]), [x40] "v"(x[4][0]), [x41] "v"(x[4][1]), [x50] "v"(x[5][0]), [x51] "v"(x[5][1]), [x60] "v"(x[6][0]), [x61] "v"(x[6][1]), [x70] "v"(x[7][0]), [x71] "v"(x[7][1]), [x80] "v"(x[8][0]), [x81] "v"(x[8][1]));
  } else if constexpr (LAST) {
    asm("v_mul_f32_dpp %[t10], %[w], %[x10] row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[t11], %[w], %[x11] row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[tc0]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[tc1]\n\t"
          "v_mul_f32_dpp %[tc0], %[w], %[x20] row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[tc1], %[w], %[x21] row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[t10]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[t11]\n\t"
          "v_mul_f32_dpp %[t10], %[w], %[x30] row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[t11], %[w], %[x31] row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[tc0]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[tc1]\n\t"
          "v_mul_f32_dpp %[tc0], %[w], %[x40] row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[tc1], %[w], %[x41] row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[t10]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[t11]\n\t"
          "v_mul_f32_dpp %[t10], %[w], %[x50] row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[t11], %[w], %[x51] row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[tc0]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[tc1]\n\t"
          "v_mul_f32_dpp %[tc0], %[w], %[x60] row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[tc1], %[w], %[x61] row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[t10]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[t11]\n\t"
          "v_mul_f32_dpp %[t10], %[w], %[x70] row_newbcast:15 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[t11], %[w], %[x71] row_newbcast:15 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[tc0]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[tc1]\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[t10]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[t11]\n\t"
        : [a0] "+v"(a0), [a1] "+v"(a1), [tc0] "+v"(tc0), [tc1] "+v"(tc1), [t10] "=&v"(t10), [t11] "=&v"(t11)
        : [w] "v"(w), [x10] "v"(x[1][0]), [x11] "v"(x[1][1]), [x20] "v"(x[2][0]), [x21] "v"(x[2][1]), [x30] "v"(x[3][0]), [x31] "v"(x[3][1]), [x40] "v"(x[4][0]), [x41] "v"(x[4][1]), [x50] "v"(x[5][0]), [x51] "v"(x[5][1]), [x60] "v"(x[6][0]), [x61] "v"(x[6][1]), [x70] "v"(x[7][0]), [x71] "v"(x[7][1]));
  } else {
    asm("v_mul_f32_dpp %[t10], %[w], %[x10] row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[t11], %[w], %[x11] row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[tc0]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[tc1]\n\t"
          "v_mul_f32_dpp %[tc0], %[w], %[x20] row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[tc1], %[w], %[x21] row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[t10]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[t11]\n\t"
          "v_mul_f32_dpp %[t10], %[w], %[x30] row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[t11], %[w], %[x31] row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[tc0]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[tc1]\n\t"
          "v_mul_f32_dpp %[tc0], %[w], %[x40] row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[tc1], %[w], %[x41] row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[t10]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[t11]\n\t"
          "v_mul_f32_dpp %[t10], %[w], %[x50] row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[t11], %[w], %[x51] row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[tc0]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[tc1]\n\t"
          "v_mul_f32_dpp %[tc0], %[w], %[x60] row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[tc1], %[w], %[x61] row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[t10]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[t11]\n\t"
          "v_mul_f32_dpp %[t10], %[w], %[x70] row_newbcast:15 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[t11], %[w], %[x71] row_newbcast:15 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[tc0]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[tc1]\n\t"
          "v_mul_f32_dpp %[tc0], %[wn], %[x80] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
          "v_mul_f32_dpp %[tc1], %[wn], %[x81] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
          "v_add_f32_e32 %[a0], %[a0], %[t10]\n\t"
          "v_add_f32_e32 %[a1], %[a1], %[t11]\n\t"
        : [a0] "+v"(a0), [a1] "+v"(a1), [tc0] "+v"(tc0), [tc1] "+v"(tc1), [t10] "=&v"(t10), [t11] "=&v"(t11)
        : [w] "v"(w), [wn] "v"(wn), [x10] "v"(x[1][0]), [x11] "v"(x[1][1]), [x20] "v"(x[2][0]), [x21] "v"(x[2][1]), [x30] "v"(x[3][0]), [x31] "v"(x[3][1]), [x40] "v"(x[4][0]), [x41] "v"(x[4][1]), [x50] "v"(x[5][0]), [x51] "v"(x[5][1]), [x60] "v"(x[6][0]), [x61] "v"(x[6][1]), [x70] "v"(x[7][0]), [x71] "v"(x[7][1]), [x80] "v"(x[8][0]), [x81] "v"(x[8][1]));
  }
}

// fl32(w[16r + I % 16] * x) by the same broadcast (the chain's first product)
template <int I>
__device__ __forceinline__ float mul_row_bcast(float w, float x) {
  float r;
  asm("v_mul_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(w), "v"(x), "n"(I % 16));
  return r;
}

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_move_f64(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(static_cast<uint32_t>(u)), CTRL, ROW_MASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(static_cast<uint32_t>(u >> 32)), CTRL, ROW_MASK, 0xF,
                                             false);
  return __builtin_bit_cast(double, (static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32) | static_cast<uint32_t>(lo));
}

__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += dpp_move_f64<0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
  v += dpp_move_f64<0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
  v += dpp_move_f64<0x141, 0xF>(v);  // row_half_mirror
  v += dpp_move_f64<0x140, 0xF>(v);  // row_mirror
  v += dpp_move_f64<0x142, 0xA>(v);  // row_bcast:15 into rows 1 and 3
  v += dpp_move_f64<0x143, 0xC>(v);  // row_bcast:31 into rows 2 and 3
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(u), 63);
  const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(u >> 32), 63);
  return __builtin_bit_cast(double, (static_cast<uint64_t>(hi) << 32) | lo);
}

inline unsigned grid_for(int64_t items, int per_block) {
  return static_cast<unsigned>((items + per_block - 1) / per_block);
}

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

// Blocks of a kernel the whole chip holds at once (occupancy x CUs), cached
// per (device, kernel) -- kernels of one signature share a template
// instantiation of this function, so the cache must be keyed by the kernel.
template <typename Kern>
int64_t resident_blocks(Kern kernel, int block = kBlock) {
  static std::mutex mu;
  static std::map<std::tuple<int, const void*, int>, int64_t> cache;  // per device, kernel and block size
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 1024;
  const auto key = std::make_tuple(dev, reinterpret_cast<const void*>(kernel), block);
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, 0) != hipSuccess || per_cu <= 0) per_cu = 1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  const int64_t n = static_cast<int64_t>(per_cu) * cus;
  std::lock_guard<std::mutex> lk(mu);
  cache[key] = n;
  return n;
}

inline int cu_count() {
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

// Round-split dispatch: the column range is cut into the fewest EQUAL
// launches whose blocks all fit on the chip at once (one resident round
// each).  Within a launch every block starts together and the running blocks
// sweep one compact window of every client row; the stream boundary between
// launches re-aligns them (a multi-round launch lets blocks drift apart and
// leaves a half-empty last round).
template <int U, int C, bool NT>
void launch_split_ev(const float* clients, int K, int64_t ld, int64_t P, const float* W, float* out, int max_blocks,
                     hipStream_t s, hipEvent_t ev_start, hipEvent_t ev_stop) {
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
    // launch-attached timing events: the first launch's start, the last one's end
    hipExtLaunchKernelGGL((reduce_f32x4_var_kernel<U, C, NT, false>), dim3(static_cast<unsigned>((n + span - 1) / span)),
                          dim3(kBlock), 0, s, v0 == 0 ? ev_start : nullptr, v0 + n >= nvec ? ev_stop : nullptr, 0,
                          X + v0, K, ld / 4, n, tail, W, out + v0 * 4);
  }
}

template <int U, int C, bool NT>
void launch_split(const float* clients, int K, int64_t ld, int64_t P, const float* W, float* out, int max_blocks,
                  hipStream_t s) {
  launch_split_ev<U, C, NT>(clients, K, ld, P, W, out, max_blocks, s, nullptr, nullptr);
}

// Row reduce through buffer descriptors: a full column group reads client
// row k through one descriptor whose base (row k + the group's first column)
// is wave-uniform and sits in SGPRs (readfirstlane), with the lane's slice as
// a 32-bit voffset shared by every row -- no 64-bit VGPR address per (row,
// slice) load.  aux 2 = nt.  Same per-element order as reduce_full_group, so
// the same bits; the ragged last group takes reduce_full_group's global path.
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* base, int bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo), 0, bytes,
                                           0x00020000);
}

__device__ __forceinline__ f32x4 ld_rsrc_nt(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>(byte_off), 0, 2));
}

// Column group of workgroup `b` in a one-round launch of `g` workgroups when
// the co-resident groups of a CU should take ADJACENT column groups: the
// dispatcher hands workgroup w to XCD w % 8 and, within it, fills the CUs in
// order, so w, w + S, w + 2S (S = slots per round, the CU count) share a CU.
// Slot r = b % S gets columns start_r + b / S with start_r = r*m + min(r, e)
// (g = S*m + e): a bijection that gives each CU one contiguous run.
__device__ __forceinline__ int64_t cu_contiguous_group(int64_t b, int64_t g, int64_t slots) {
  const int64_t m = g / slots, e = g % slots, r = b % slots, q = b / slots;
  return r * m + (r < e ? r : e) + q;
}

template <int U, int C, int BS = kBlock, int REMAP = 0>
__global__ __launch_bounds__(BS) void reduce_f32x4_buf_kernel(const f32x4* __restrict__ X, int K, int64_t ld4,
                                                              int64_t nvec, int tail, const float* __restrict__ W,
                                                              float* __restrict__ out) {
  constexpr int64_t span = static_cast<int64_t>(BS) * C;  // float4 columns per group
  constexpr int bytes = static_cast<int>(span * 16);
  uint32_t off[C];
#pragma unroll
  for (int j = 0; j < C; ++j) off[j] = 16u * (threadIdx.x + j * BS);
  const int64_t b0 = REMAP > 0 ? cu_contiguous_group(blockIdx.x, gridDim.x, REMAP) : blockIdx.x;
  for (int64_t base = b0 * span; base < nvec;
       base += static_cast<int64_t>(gridDim.x) * span) {
    if (base + span <= nvec) {
      f32x4 acc[C];
      const float w0 = W[0];
      {
        const __amdgpu_buffer_rsrc_t r0 = uniform_rsrc(X + base, bytes);
#pragma unroll
        for (int j = 0; j < C; ++j) acc[j] = ld_rsrc_nt(r0, off[j]) * w0;
      }
      const int nb = (K - 1) / U;
      int k = 1;
      for (int b = 0; b < nb; ++b, k += U) {
        f32x4 xs[U][C];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const __amdgpu_buffer_rsrc_t r = uniform_rsrc(X + static_cast<int64_t>(k + u) * ld4 + base, bytes);
#pragma unroll
          for (int j = 0; j < C; ++j) xs[u][j] = ld_rsrc_nt(r, off[j]);
        }
        consume_batch<U, C>(acc, xs, W, k);
      }
      for (; k < K; ++k) {
        const __amdgpu_buffer_rsrc_t r = uniform_rsrc(X + static_cast<int64_t>(k) * ld4 + base, bytes);
        const float w = W[k];
#pragma unroll
        for (int j = 0; j < C; ++j) {
          const f32x4 term = ld_rsrc_nt(r, off[j]) * w;
          acc[j] = acc[j] + term;
        }
      }
#pragma unroll
      for (int j = 0; j < C; ++j) store_slice(out, base + threadIdx.x + j * BS, nvec, tail, acc[j]);
    } else {
      for (int j = 0; j < C; ++j) {
        const int64_t v = base + threadIdx.x + j * BS;
        if (v >= nvec) break;
        f32x4 acc[1];
        reduce_full_group<U, 1, true, false>(acc, X + v, K, ld4, W);
        store_slice(out, v, nvec, tail, acc[0]);
      }
    }
  }
}

// launch_split's round-split schedule with the buffer-descriptor kernel, in
// blocks of BS threads (BS = 64: one wave per workgroup, for short rows whose
// 256-thread groups would leave the CUs unevenly loaded)
template <int U, int C, int BS = kBlock, int REMAP = 0>
void launch_split_buf(const float* clients, int K, int64_t ld, int64_t P, const float* W, float* out, int max_blocks,
                      hipStream_t s, hipEvent_t ev_start = nullptr, hipEvent_t ev_stop = nullptr) {
  const int64_t nvec = (P + 3) / 4;
  const int64_t span = static_cast<int64_t>(BS) * C;
  const int64_t resident =
      max_blocks > 0 ? max_blocks : resident_blocks(reduce_f32x4_buf_kernel<U, C, BS, REMAP>, BS);
  const int64_t blocks = (nvec + span - 1) / span;
  const int64_t nl = (blocks + resident - 1) / resident;
  const int64_t per = ((nvec + nl - 1) / nl + span - 1) / span * span;
  const f32x4* X = reinterpret_cast<const f32x4*>(clients);
  for (int64_t v0 = 0; v0 < nvec; v0 += per) {
    const int64_t n = (nvec - v0) < per ? (nvec - v0) : per;
    const int tail = (v0 + n == nvec) ? static_cast<int>(P & 3) : 0;
    hipExtLaunchKernelGGL((reduce_f32x4_buf_kernel<U, C, BS, REMAP>), dim3(static_cast<unsigned>((n + span - 1) / span)),
                          dim3(BS), 0, s, v0 == 0 ? ev_start : nullptr, v0 + n >= nvec ? ev_stop : nullptr, 0,
                          X + v0, K, ld / 4, n, tail, W, out + v0 * 4);
  }
}

// ---------------------------------------------------------------------------
// Fused aggregate + :291 tiles (fedavg_dist.hip: [K, ld] rows;
// fedavg_segments.hip: device-resident clients).  A workgroup stages a tile of
// S columns x all K rows in LDS -- row r's 16-B slot j holds the row's slice
// j ^ (r & 7) (XOR swizzle applied to the per-lane GLOBAL address, LDS-DMA
// keeps LDS linear) -- then:
//   fused_average : one thread per column, the reference's sequential chain
//                   over the K rows (:455-457, the bits of fedavg_reduce_f32),
//                   stored to `out` and to LDS (`gs`);
//   fused_squares : thread t owns row t % K and slices t / K, t / K + q, ...
//                   (q = 256 / K threads per row; above 256 rows, rows t,
//                   t + 256, ... whole): fl32(x - g)^2 in fp64 into four
//                   register chains per row that live across all tiles;
//   fused_finish  : the q threads of a row added in a fixed order ->
//                   partials[row][workgroup].
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void* fused_lds_t;
typedef const __attribute__((address_space(1))) void* fused_gbl_t;

// Barriers without the compiler's vmcnt(0) drain (a plain __syncthreads()
// would also wait for LDS-DMA loads meant to stay in flight across it).
__device__ __forceinline__ void barrier_lds() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void barrier_loads() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// LDS float index of (row, column) in a swizzled tile of S columns
template <int S>
__device__ __forceinline__ int fused_at(int row, int col) {
  return row * S + ((((col >> 2) ^ (row & 7))) << 2) + (col & 3);
}

template <int S>
__device__ __forceinline__ void fused_average(const float* tile, float* gs, int K, const float* __restrict__ W,
                                              int ncols, float* __restrict__ out) {
  if (threadIdx.x < S) {
    const int c = threadIdx.x;
    float a = tile[fused_at<S>(0, c)] * W[0];
    // 16 rows per batch: one s_load_dwordx16 of weights and 16 LDS reads per
    // wait (interleaved A/B, profiles/r02/fused/ab_chain_unroll16.jsonl:
    // 200 x 10M 1.693 -> 1.624 ms, 20 x 25M 0.428 -> 0.406, K = 100 equal);
    // 32 for the 64-column tiles of 65-128 clients (ab_chain_unroll32*.jsonl:
    // 100 x 25M 1.760 -> 1.668 ms; slower for the other widths)
    constexpr int kChainUnroll = S == 64 ? 32 : 16;
#pragma unroll kChainUnroll
    for (int k = 1; k < K; ++k) {
      const float term = tile[fused_at<S>(k, c)] * W[k];
      a = a + term;
    }
    gs[c] = a;
    if (c < ncols) out[c] = a;
  }
}

// RM = 1: K <= 256, thread t owns row t % K and slices t / K, t / K + q, ...
// (q = 256 / K); RM > 1: 256 < K <= 256 RM, thread t owns rows t, t + 256, ...
// and every slice of them.  acc[m][0..3]: four fp64 chains per owned row.
// UNMASKED: full tiles skip the padding selects (the rows kernel; the
// segments kernel keeps one masked path, which holds it to 6 workgroups/CU)
template <int S, int RM = 1, bool UNMASKED = true>
__device__ __forceinline__ void fused_squares(const float* tile, const float* gs, int K, int ncols,
                                              double (&acc)[RM][4]) {
  constexpr int V = S / 4;
  // a full tile (every column valid: all but a key's / the model's last) takes
  // no masks at all; the ragged one selects the padding out
  const auto sq_full = [&](double (&a)[4], f32x4 x, int c) {
    const f32x4 d = x - reinterpret_cast<const f32x4*>(gs)[c];  // fp32 difference, as the reference forms it
    const double dx = d.x, dy = d.y, dz = d.z, dw = d.w;
    a[0] = __builtin_fma(dx, dx, a[0]);
    a[1] = __builtin_fma(dy, dy, a[1]);
    a[2] = __builtin_fma(dz, dz, a[2]);
    a[3] = __builtin_fma(dw, dw, a[3]);
  };
  const auto sq = [&](double (&a)[4], f32x4 x, int c) {
    const f32x4 g = reinterpret_cast<const f32x4*>(gs)[c];
    const f32x4 d = x - g;        // fp32 difference, as the reference forms it
    const int n = ncols - 4 * c;  // valid columns of this slice (select, not multiply: padding may hold NaN/inf)
    if (n > 0) {
      const double dx = d.x, dy = n > 1 ? d.y : 0.f, dz = n > 2 ? d.z : 0.f, dw = n > 3 ? d.w : 0.f;
      a[0] = __builtin_fma(dx, dx, a[0]);
      a[1] = __builtin_fma(dy, dy, a[1]);
      a[2] = __builtin_fma(dz, dz, a[2]);
      a[3] = __builtin_fma(dw, dw, a[3]);
    }
  };
  const bool full = UNMASKED && ncols == S;
  if constexpr (RM == 1) {
    const int q = kBlock / K;
    const int my_row = threadIdx.x % K;
    const int my_sub = threadIdx.x / K;
    if (my_sub >= q) return;
    const int swz = my_row & 7;
    const f32x4* x4 = reinterpret_cast<const f32x4*>(tile) + my_row * V;
    if (full) {
      for (int c = my_sub; c < V; c += q) sq_full(acc[0], x4[c ^ swz], c);
    } else {
      for (int c = my_sub; c < V; c += q) sq(acc[0], x4[c ^ swz], c);
    }
  } else {
#pragma unroll
    for (int m = 0; m < RM; ++m) {
      const int row = threadIdx.x + m * kBlock;
      if (row < K) {
        const int swz = row & 7;
        const f32x4* x4 = reinterpret_cast<const f32x4*>(tile) + row * V;
        if (full) {
          for (int c = 0; c < V; ++c) sq_full(acc[m], x4[c ^ swz], c);
        } else {
          for (int c = 0; c < V; ++c) sq(acc[m], x4[c ^ swz], c);
        }
      }
    }
  }
}

// `lds` holds >= 256 doubles and no tile is in use or in flight any more
template <int RM = 1>
__device__ __forceinline__ void fused_finish(float* lds, const double (&acc)[RM][4], int K,
                                             double* __restrict__ partials) {
  barrier_loads();
  if constexpr (RM == 1) {
    const int q = kBlock / K;
    double* red = reinterpret_cast<double*>(lds);
    red[threadIdx.x] = (acc[0][0] + acc[0][1]) + (acc[0][2] + acc[0][3]);
    barrier_lds();
    if (threadIdx.x < K) {
      double s = red[threadIdx.x];
      for (int u = 1; u < q; ++u) s += red[threadIdx.x + u * K];
      partials[static_cast<int64_t>(threadIdx.x) * gridDim.x + blockIdx.x] = s;
    }
  } else {
#pragma unroll
    for (int m = 0; m < RM; ++m) {
      const int row = threadIdx.x + m * kBlock;
      if (row < K)
        partials[static_cast<int64_t>(row) * gridDim.x + blockIdx.x] = (acc[m][0] + acc[m][1]) + (acc[m][2] + acc[m][3]);
    }
  }
}

// ---------------------------------------------------------------------------
// Wave-owned windows (fedavg_dist.hip's reduce_sqdist_win_kernel and
// fedavg_segments.hip's zero-copy form): a wave holds 64 x VEC columns of all
// K rows in registers; each batch of 8 rows' fp64 partials is folded across
// the wave by v_permlane32_swap / v_permlane16_swap / one row_ror:8 exchange
// into one register (8 lanes per row, win_batch_row).
// ---------------------------------------------------------------------------
template <int VEC>
struct WinVec {
  typedef float T __attribute__((ext_vector_type(VEC)));
  // the same vector at dword alignment: window stores into outputs that are
  // only 4-B aligned (a key's offset inside the packed model is any element)
  typedef float TA __attribute__((ext_vector_type(VEC), aligned(4)));
};

// lanes 0-31: a's two halves added (lane l: a[l] + a[l + 32]); lanes 32-63: b's
__device__ __forceinline__ double fold32(double a, double b) {
  const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
  const auto lo = __builtin_amdgcn_permlane32_swap(static_cast<uint32_t>(ua), static_cast<uint32_t>(ub), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(static_cast<uint32_t>(ua >> 32), static_cast<uint32_t>(ub >> 32),
                                                   false, false);
  const double na = __builtin_bit_cast(double, (static_cast<uint64_t>(hi[0]) << 32) | lo[0]);
  const double nb = __builtin_bit_cast(double, (static_cast<uint64_t>(hi[1]) << 32) | lo[1]);
  return na + nb;
}

// 16-lane rows [a.r0 + a.r1, b.r0 + b.r1, a.r2 + a.r3, b.r2 + b.r3]
__device__ __forceinline__ double fold16(double a, double b) {
  const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
  const auto lo = __builtin_amdgcn_permlane16_swap(static_cast<uint32_t>(ua), static_cast<uint32_t>(ub), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(static_cast<uint32_t>(ua >> 32), static_cast<uint32_t>(ub >> 32),
                                                   false, false);
  const double na = __builtin_bit_cast(double, (static_cast<uint64_t>(hi[0]) << 32) | lo[0]);
  const double nb = __builtin_bit_cast(double, (static_cast<uint64_t>(hi[1]) << 32) | lo[1]);
  return na + nb;
}

// lanes with bit 3 clear keep a's value + the lane 8 above; set: b's + the lane 8 below
__device__ __forceinline__ double fold8(double a, double b, bool upper) {
  const double send = upper ? a : b;
  const double keep = upper ? b : a;
  return keep + dpp_move_f64<0x128, 0xF>(send);  // row_ror:8 = lane xor 8 within a 16-lane row
}

// batch row held by lane l after fold32 / fold16 / fold8
__device__ __forceinline__ int win_batch_row(int lane) {
  const int r = lane >> 4;
  return 4 * ((lane >> 3) & 1) + (((r & 1) << 1) | (r >> 1));
}

template <int VEC>
__device__ __forceinline__ typename WinVec<VEC>::T win_load(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t soff = 0) {
  typedef typename WinVec<VEC>::T V;
  if constexpr (VEC == 1)
    return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b32(r, static_cast<int>(off), static_cast<int>(soff), 2));
  else if constexpr (VEC == 2)
    return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b64(r, static_cast<int>(off), static_cast<int>(soff), 2));
  else
    return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>(off), static_cast<int>(soff), 2));
}

template <int VEC>
__device__ __forceinline__ double win_sq(typename WinVec<VEC>::T d) {
  double s = static_cast<double>(d[0]) * static_cast<double>(d[0]);
#pragma unroll
  for (int v = 1; v < VEC; ++v) s = __builtin_fma(static_cast<double>(d[v]), static_cast<double>(d[v]), s);
  return s;
}

// __launch_bounds__'s second argument is waves per SIMD: the window's KMAX x
// VEC registers (+ a quarter more at VEC 1: one square per row per lane
// before the folds) and ~40 others within 512 / waves
// rows of the next window the split-row window kernel on packed rows
// prefetches while the chain runs (reduce_sqdist_winn_kernel; the zero-copy
// form gained nothing from it); FEDAVG_SPLIT_PREFETCH=0 turns it
// off and gives 161-368 rows back to the tiles (A/B)
inline int split_prefetch_rows() {
  static const int v = [] {
    const char* e = std::getenv("FEDAVG_SPLIT_PREFETCH");
    return e && e[0] == '0' ? 0 : 8;
  }();
  return v;
}

constexpr int win_min_waves(int kmax, int vec) {
  const int regs = kmax * vec + (vec == 1 ? kmax / 4 : 0);
  return regs <= 88 ? 4 : (regs <= 128 ? 3 : (regs <= 216 ? 2 : 1));
}

}  // namespace fedavg_impl
