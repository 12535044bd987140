// fedavg_xfer.hip -- host<->device transfers of the hot path: the averaged
// model's D2H (feeding load_state_dict, fedavg_trainer.py:219) and one rank's
// strided shard upload.
//
// D2H: two engines behind one entry point.  blocks == 0 is the runtime's
// hipMemcpyAsync; blocks > 0 is a zero-copy kernel with that fixed grid that
// writes straight into the mapped pinned buffer (nontemporal 16-B loads and
// stores).  The runtime copy's blit spreads over the whole chip and slows a
// concurrent reduce (0.19 -> 0.33 ms per streaming chunk), but it moves the
// bytes faster: a streaming round's finish at K=100 x P=25M measured 2.67 ms
// with it vs 3.0-3.1 ms with the 64-block kernel (3.3 / 3.5 ms at 128 / 256
// blocks), so 0 is the production default (aggregate.D2H_BLOCKS).
#include "common.hpp"

namespace {
using namespace fedavg_impl;

__global__ __launch_bounds__(kBlock) void copy_to_host_kernel(const f32x4* __restrict__ src, f32x4* __restrict__ dst,
                                                              int64_t nvec, const unsigned char* __restrict__ src_tail,
                                                              unsigned char* __restrict__ dst_tail, int tail_bytes) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; v < nvec; v += stride)
    __builtin_nontemporal_store(ld<true>(src + v), dst + v);
  if (blockIdx.x == 0 && static_cast<int>(threadIdx.x) < tail_bytes) dst_tail[threadIdx.x] = src_tail[threadIdx.x];
}

}  // namespace

extern "C" {

int fedavg_copy_to_host(const void* src, void* host_dst, int64_t bytes, int blocks, void* stream) {
  const char* what = "fedavg_copy_to_host";
  if (bytes < 0 || (bytes > 0 && (!src || !host_dst)))
    return set_error(FEDAVG_EINVAL, "%s: bad arguments", what);
  if (bytes == 0) return FEDAVG_OK;
  if (!aligned16(src) || !aligned16(host_dst))
    return set_error(FEDAVG_EALIGN, "%s: src and host_dst must be 16-B aligned", what);
  // only pinned (registered) host memory is reachable from the device
  if (!is_pinned_host_memory(host_dst)) return set_error(FEDAVG_EINVAL, "%s: host_dst is not pinned host memory", what);
  if (blocks < 0) return set_error(FEDAVG_EINVAL, "%s: blocks must be >= 0", what);
  if (blocks == 0) {
    const hipError_t e = hipMemcpyAsync(host_dst, src, static_cast<size_t>(bytes), hipMemcpyDeviceToHost,
                                        static_cast<hipStream_t>(stream));
    if (e != hipSuccess) {
      (void)hipGetLastError();
      return set_error(-static_cast<int>(e), "%s: hipMemcpyAsync failed: %s", what, hipGetErrorString(e));
    }
    return FEDAVG_OK;
  }
  const int64_t nvec = bytes / 16;
  const int tail = static_cast<int>(bytes - nvec * 16);
  const int64_t need = (nvec + kBlock - 1) / kBlock;
  const unsigned grid = static_cast<unsigned>(need < blocks ? (need < 1 ? 1 : need) : blocks);
  const auto* s8 = static_cast<const unsigned char*>(src);
  auto* d8 = static_cast<unsigned char*>(host_dst);
  hipLaunchKernelGGL(copy_to_host_kernel, dim3(grid), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                     static_cast<const f32x4*>(src), static_cast<f32x4*>(host_dst), nvec, s8 + nvec * 16,
                     d8 + nvec * 16, tail);
  return launch_status(what);
}

// One rank's P-shard of the pinned host [K, P] client buffer -> its device
// [K, ld] rows in ONE strided DMA (src pitch = the host
// row, width = the shard, height = K), instead of K row copies or a host-side
// gather into a contiguous temporary.
int fedavg_upload_shard(void* dst, int64_t dst_pitch_bytes, const void* host_src, int64_t src_pitch_bytes,
                        int64_t width_bytes, int64_t rows, void* stream) {
  const char* what = "fedavg_upload_shard";
  if (rows < 0 || width_bytes < 0 || dst_pitch_bytes < width_bytes || src_pitch_bytes < width_bytes)
    return set_error(FEDAVG_EINVAL, "%s: bad sizes (rows=%lld width=%lld dpitch=%lld spitch=%lld)", what,
                     (long long)rows, (long long)width_bytes, (long long)dst_pitch_bytes, (long long)src_pitch_bytes);
  if (rows == 0 || width_bytes == 0) return FEDAVG_OK;
  if (!dst || !host_src) return set_error(FEDAVG_EINVAL, "%s: null buffer", what);
  // async only from pinned memory; a pageable source would silently serialise
  if (!is_pinned_host_memory(host_src)) return set_error(FEDAVG_EINVAL, "%s: host_src is not pinned host memory", what);
  const hipError_t e = hipMemcpy2DAsync(dst, static_cast<size_t>(dst_pitch_bytes), host_src,
                                        static_cast<size_t>(src_pitch_bytes), static_cast<size_t>(width_bytes),
                                        static_cast<size_t>(rows), hipMemcpyHostToDevice,
                                        static_cast<hipStream_t>(stream));
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return set_error(-static_cast<int>(e), "%s: hipMemcpy2DAsync failed: %s", what, hipGetErrorString(e));
  }
  return FEDAVG_OK;
}

}  // extern "C"
