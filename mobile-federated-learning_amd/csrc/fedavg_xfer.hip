// fedavg_xfer.hip -- zero-copy device->host transfer of the averaged model
// (the D2H that feeds load_state_dict, fedavg_trainer.py:219).
//
// The runtime performs a device->pinned-host hipMemcpyAsync with a blit
// kernel that spreads over the whole chip; next to a running reduce it takes
// CU slots for as long as PCIe needs, and the reduce of a streaming round's
// next column chunk slowed from 0.19 to 0.33 ms (rocprofv3 timeline in
// DESIGN.md).  This kernel writes the chunk straight into the mapped pinned
// buffer with a small, fixed grid (nontemporal 16-B loads and stores): PCIe
// is the limit either way, and the reduce keeps the rest of the CUs.
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
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, host_dst) != hipSuccess || attr.type != hipMemoryTypeHost) {
    (void)hipGetLastError();
    return set_error(FEDAVG_EINVAL, "%s: host_dst is not pinned host memory", what);
  }
  if (blocks <= 0) blocks = 64;
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

}  // extern "C"
