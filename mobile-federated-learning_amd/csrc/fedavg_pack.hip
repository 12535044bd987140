// fedavg_pack.hip -- packing DEVICE-resident client state_dicts into the
// [K, ld] client-major rows the reduction streams.
//
// The reference's clients return host state_dicts (client.py:96,
// `net.cpu().state_dict()`), but its aggregate (fedavg_trainer.py:441-458) is
// device-agnostic: with the clients' tensors left in HBM (the client trained
// on this GPU and the caller skipped the .cpu()) it reduces them where they
// lie.  The host packer (fedavg_host.cpp) cannot read HBM, and one device copy
// per key costs a launch each (35,000 for resnet56 x 100 clients), so this is
// the same item list as fedavg_pack_rows executed by ONE kernel.  Like the
// host packer it balances ELEMENTS, not items: wave w takes elements
// [w*kPackChunk, (w+1)*kPackChunk) of the items laid end to end (a prefix sum
// of numel built on the host and shipped with the items), finds its first
// item with a 64-way search across its lanes (a few probe rounds instead of a
// 15-level binary search for 35,000 items) and walks the items it overlaps.
// Waves, not workgroups, are the walkers: a model of many small keys
// (resnet56: 350 keys, most under 1,000 elements) is bound by the latency of
// each item's metadata load and copy, so more independent walkers finish it
// sooner.
// Raw copies move 16-B vectors: the destination is aligned by a short byte
// head, the source is then read with dword-aligned global_load_dwordx4 (fp32
// and fp64 always; fp16/bf16 when source and destination agree mod 4 bytes,
// element by element otherwise).  Integer/bool sources are converted to fp32
// element by element with static_cast, as the host packer and ATen's
// promotion of `int_tensor * python_float` do (fedavg_trainer.py:455); raw
// items are copied as bit patterns (NaN payloads kept).  HBM-bound: per
// element, the source bytes read + elem_size bytes written.
#include "common.hpp"
#include "staging.hpp"

namespace {
using namespace fedavg_impl;

constexpr int kPackThreads = 256;                                    // 4 waves per workgroup
constexpr int kWave = 64;
constexpr int kPackPer = 16;                                         // scalar loads in flight per lane
constexpr int kPackVecPer = 8;                                       // 16-B loads in flight per lane
constexpr int64_t kPackStep = static_cast<int64_t>(kWave) * kPackPer;  // elements per scalar pass
constexpr int64_t kPackChunk = 4096;                                 // elements per wave
constexpr int64_t kPackBlockElems = kPackChunk * (kPackThreads / kWave);

enum : int64_t { kRaw = 0, kI64 = 1, kI32 = 2, kI16 = 3, kI8 = 4, kU8 = 5, kBool = 6 };

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_a4 __attribute__((aligned(4)));  // dword-aligned 16-B source vector

struct Bits {
  template <typename T>
  __device__ T operator()(T v) const { return v; }
};
struct ToF32 {
  template <typename T>
  __device__ float operator()(T v) const { return static_cast<float>(v); }
};
struct BoolToF32 {
  __device__ float operator()(uint8_t v) const { return v ? 1.0f : 0.0f; }
};

__device__ __forceinline__ int lane_id() { return static_cast<int>(threadIdx.x & (kWave - 1)); }

// n elements src -> dst, converted by op, by one wave
template <typename S, typename D, typename Op>
__device__ __forceinline__ void pack_span(const S* __restrict__ src, D* __restrict__ dst, int64_t n, Op op) {
  const int lane = lane_id();
  for (int64_t base = 0; base < n; base += kPackStep) {
    S v[kPackPer];
#pragma unroll
    for (int j = 0; j < kPackPer; ++j) {
      const int64_t e = base + lane + j * kWave;
      if (e < n) v[j] = __builtin_nontemporal_load(src + e);
    }
#pragma unroll
    for (int j = 0; j < kPackPer; ++j) {
      const int64_t e = base + lane + j * kWave;
      if (e < n) dst[e] = op(v[j]);
    }
  }
}

// nb raw bytes src -> dst (elements of es bytes), by one wave
__device__ __forceinline__ void copy_raw(const char* __restrict__ s, char* __restrict__ d, int64_t nb, int es) {
  const uintptr_t da = reinterpret_cast<uintptr_t>(d);
  if (((reinterpret_cast<uintptr_t>(s) - da) & 3u) != 0) {  // cannot be dword-aligned together
    if (es == 2)
      pack_span(reinterpret_cast<const uint16_t*>(s), reinterpret_cast<uint16_t*>(d), nb / 2, Bits{});
    else if (es == 4)
      pack_span(reinterpret_cast<const uint32_t*>(s), reinterpret_cast<uint32_t*>(d), nb / 4, Bits{});
    else
      pack_span(reinterpret_cast<const uint64_t*>(s), reinterpret_cast<uint64_t*>(d), nb / 8, Bits{});
    return;
  }
  int64_t head = static_cast<int64_t>((16u - (da & 15u)) & 15u);
  if (head > nb) head = nb;
  const int64_t n16 = (nb - head) >> 4;
  const int64_t tail0 = head + (n16 << 4);
  const int lane = lane_id();
  if (lane < head) d[lane] = s[lane];
  if (lane < nb - tail0) d[tail0 + lane] = s[tail0 + lane];
  const u32x4_a4* vs = reinterpret_cast<const u32x4_a4*>(s + head);
  u32x4* vd = reinterpret_cast<u32x4*>(d + head);
  for (int64_t base = 0; base < n16; base += static_cast<int64_t>(kWave) * kPackVecPer) {
    u32x4 v[kPackVecPer];
#pragma unroll
    for (int j = 0; j < kPackVecPer; ++j) {
      const int64_t e = base + lane + j * kWave;
      if (e < n16) v[j] = __builtin_nontemporal_load(vs + e);
    }
#pragma unroll
    for (int j = 0; j < kPackVecPer; ++j) {
      const int64_t e = base + lane + j * kWave;
      if (e < n16) __builtin_nontemporal_store(v[j], vd + e);
    }
  }
}

__global__ __launch_bounds__(kPackThreads) void pack_rows_device_kernel(const fedavg_pack_item* __restrict__ items,
                                                                        const int64_t* __restrict__ start,
                                                                        int64_t n_items, int64_t total,
                                                                        char* __restrict__ dst_base, int es) {
  const int64_t g0 = static_cast<int64_t>(blockIdx.x) * kPackBlockElems + (threadIdx.x / kWave) * kPackChunk;
  if (g0 >= total) return;  // a wave past the end of the last workgroup's range
  const int64_t g1 = total - g0 < kPackChunk ? total : g0 + kPackChunk;
  for (int64_t i = wave_search_last_le([&](int64_t x) { return start[x]; }, n_items, g0); i < n_items; ++i) {
    const int64_t s0 = start[i];
    if (s0 >= g1) break;
    const fedavg_pack_item it = items[i];
    const int64_t a = (g0 > s0 ? g0 : s0) - s0;
    const int64_t z = (g1 < s0 + it.numel ? g1 : s0 + it.numel) - s0;
    if (z <= a) continue;
    const char* src = reinterpret_cast<const char*>(it.src);
    float* dstf = reinterpret_cast<float*>(dst_base) + it.dst_offset + a;
    switch (it.kind) {
      case kRaw: copy_raw(src + a * es, dst_base + (it.dst_offset + a) * es, (z - a) * es, es); break;
      case kI64: pack_span(reinterpret_cast<const int64_t*>(src) + a, dstf, z - a, ToF32{}); break;
      case kI32: pack_span(reinterpret_cast<const int32_t*>(src) + a, dstf, z - a, ToF32{}); break;
      case kI16: pack_span(reinterpret_cast<const int16_t*>(src) + a, dstf, z - a, ToF32{}); break;
      case kI8: pack_span(reinterpret_cast<const int8_t*>(src) + a, dstf, z - a, ToF32{}); break;
      case kU8: pack_span(reinterpret_cast<const uint8_t*>(src) + a, dstf, z - a, ToF32{}); break;
      case kBool: pack_span(reinterpret_cast<const uint8_t*>(src) + a, dstf, z - a, BoolToF32{}); break;
      default: break;  // rejected on the host
    }
  }
}

// Many tiny items (BatchNorm's num_batches_tracked: 1 element x 58 keys x
// K clients): one THREAD per item.  The wave-per-4,096-elements kernel above
// walks such items one after another -- a dependent load per item, ~4 ms for
// resnet56 x 100's 5,800 scalar items -- where here they all load at once.
__global__ __launch_bounds__(kPackThreads) void pack_small_items_kernel(const fedavg_pack_item* __restrict__ items,
                                                                        int64_t n_items, char* __restrict__ dst_base,
                                                                        int es) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kPackThreads + threadIdx.x;
  if (i >= n_items) return;
  const fedavg_pack_item it = items[i];
  const char* src = reinterpret_cast<const char*>(it.src);
  float* dstf = reinterpret_cast<float*>(dst_base) + it.dst_offset;
  for (int64_t e = 0; e < it.numel; ++e) {
    switch (it.kind) {
      case kRaw:
        if (es == 4)
          reinterpret_cast<uint32_t*>(dst_base)[it.dst_offset + e] = reinterpret_cast<const uint32_t*>(src)[e];
        else if (es == 8)
          reinterpret_cast<uint64_t*>(dst_base)[it.dst_offset + e] = reinterpret_cast<const uint64_t*>(src)[e];
        else
          reinterpret_cast<uint16_t*>(dst_base)[it.dst_offset + e] = reinterpret_cast<const uint16_t*>(src)[e];
        break;
      case kI64: dstf[e] = static_cast<float>(reinterpret_cast<const int64_t*>(src)[e]); break;
      case kI32: dstf[e] = static_cast<float>(reinterpret_cast<const int32_t*>(src)[e]); break;
      case kI16: dstf[e] = static_cast<float>(reinterpret_cast<const int16_t*>(src)[e]); break;
      case kI8: dstf[e] = static_cast<float>(reinterpret_cast<const int8_t*>(src)[e]); break;
      case kU8: dstf[e] = static_cast<float>(reinterpret_cast<const uint8_t*>(src)[e]); break;
      case kBool: dstf[e] = reinterpret_cast<const uint8_t*>(src)[e] ? 1.0f : 0.0f; break;
      default: break;  // rejected on the host
    }
  }
}

// items of at most this many elements on average (and none above kSmallItemMax)
// take pack_small_items_kernel
constexpr int64_t kSmallItemAvg = 64;
constexpr int64_t kSmallItemMax = 4096;

// the staged items | starts layout: staging.hpp (g++-built for the sanitizer fuzz)
int64_t items_bytes(int64_t n_items) { return fedavg_staging::pack_items_bytes(n_items); }

}  // namespace

extern "C" {

int64_t fedavg_pack_rows_device_workspace(int64_t n_items) {
  return fedavg_staging::pack_rows_device_workspace_bytes(n_items);
}

int fedavg_pack_rows_device(const fedavg_pack_item* items, int64_t n_items, void* dst_base, int64_t elem_size,
                            void* host_ws, void* dev_ws, int64_t ws_bytes, void* stream) {
  const char* what = "fedavg_pack_rows_device";
  if (n_items < 0 || (n_items > 0 && (!items || !dst_base || !host_ws || !dev_ws)) ||
      (elem_size != 2 && elem_size != 4 && elem_size != 8))
    return set_error(FEDAVG_EINVAL, "%s: bad arguments", what);
  if (n_items == 0) return FEDAVG_OK;
  if (ws_bytes < fedavg_pack_rows_device_workspace(n_items))
    return set_error(FEDAVG_EINVAL, "%s: workspace needs %lld bytes", what,
                     (long long)fedavg_pack_rows_device_workspace(n_items));
  if (!aligned16(host_ws) || !aligned16(dev_ws) || !aligned16(dst_base))
    return set_error(FEDAVG_EALIGN, "%s: dst_base and the workspaces must be 16-B aligned", what);
  if (!is_device_memory(dst_base) || !is_device_memory(dev_ws))
    return set_error(FEDAVG_EINVAL, "%s: dst_base and dev_ws must be device memory", what);
  if (!is_pinned_host_memory(host_ws)) return set_error(FEDAVG_EINVAL, "%s: host_ws is not pinned host memory", what);
  fedavg_staging::PackOut st;
  fedavg_staging::Msg msg;
  if (const int rc = fedavg_staging::stage_pack_items(items, n_items, elem_size, host_ws, ws_bytes, &st, &msg))
    return set_error(rc, "%s: %s", what, msg.text);
  const int64_t total = st.total, max_numel = st.max_numel;
  const void* first_src = st.first_src;
  const void* last_src = st.last_src;
  if (total == 0) return FEDAVG_OK;
  const int64_t blocks = (total + kPackBlockElems - 1) / kPackBlockElems;
  if (blocks > INT32_MAX) return set_error(FEDAVG_EINVAL, "%s: %lld elements exceed one launch", what, (long long)total);
  // the sources must live in HBM: a host address would fault the kernel
  // (spot check of the first and last source; the Python layer checks every
  // tensor's device)
  if (!is_device_memory(first_src) || !is_device_memory(last_src))
    return set_error(FEDAVG_EINVAL, "%s: item sources must be device memory", what);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const hipError_t e = hipMemcpyAsync(dev_ws, host_ws, static_cast<size_t>(fedavg_pack_rows_device_workspace(n_items)),
                                      hipMemcpyHostToDevice, s);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return set_error(-static_cast<int>(e), "%s: hipMemcpyAsync failed: %s", what, hipGetErrorString(e));
  }
  const auto* d_items = static_cast<const fedavg_pack_item*>(dev_ws);
  const auto* d_start = reinterpret_cast<const int64_t*>(static_cast<const char*>(dev_ws) + items_bytes(n_items));
  if (total <= kSmallItemAvg * n_items && max_numel <= kSmallItemMax) {
    hipLaunchKernelGGL(pack_small_items_kernel, dim3(static_cast<unsigned>((n_items + kPackThreads - 1) / kPackThreads)),
                       dim3(kPackThreads), 0, s, d_items, n_items, static_cast<char*>(dst_base), static_cast<int>(elem_size));
    return launch_status(what);
  }
  hipLaunchKernelGGL(pack_rows_device_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kPackThreads), 0, s, d_items,
                     d_start, n_items, total, static_cast<char*>(dst_base), static_cast<int>(elem_size));
  return launch_status(what);
}

}  // extern "C"
