// fedavg_host.cpp -- native host runtime of libfedavg_amd.so: packing client
// state_dicts into the pinned client-major staging rows the kernel streams.
//
// The reference hands aggregate() K host state_dicts (fedavg_trainer.py:199,
// client.py:96) and reduces them key by key (fedavg_trainer.py:450-457).  The
// drop-in packs every client's keys, in client 0's key order, into row i of a
// [K, ld] buffer so one H2D and one kernel cover the whole model.  Doing that
// with one torch copy per key costs ~9 us per key in Python (300 ms for
// resnet56 x 100 clients, 35,000 keys); here it is one call per group of rows:
// a persistent worker pool splits the total BYTES evenly (a 25M-element key is
// cut into slices, 350 tiny keys are batched), so both shapes stream at memcpy
// speed.  Integer/bool sources are promoted to fp32 with static_cast -- the
// same conversion ATen's TensorIterator applies when it promotes
// `int_tensor * python_float` to the default dtype (fedavg_trainer.py:455).
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "fedavg_amd.h"

namespace {

enum : int64_t {
  kRaw = 0,     // same dtype: elem_size bytes per element
  kI64 = 1,     // int64  -> fp32
  kI32 = 2,     // int32  -> fp32
  kI16 = 3,     // int16  -> fp32
  kI8 = 4,      // int8   -> fp32
  kU8 = 5,      // uint8  -> fp32
  kBool = 6,    // bool   -> fp32 (0.0 / 1.0)
};

template <typename S>
void convert(const void* src, float* dst, int64_t n) {
  const S* s = static_cast<const S*>(src);
  for (int64_t i = 0; i < n; ++i) dst[i] = static_cast<float>(s[i]);
}

void copy_range(const fedavg_pack_item& it, char* dst_base, int64_t elem_size, int64_t e0, int64_t e1) {
  const int64_t n = e1 - e0;
  if (n <= 0) return;
  if (it.kind == kRaw) {
    std::memcpy(dst_base + (it.dst_offset + e0) * elem_size,
                static_cast<const char*>(reinterpret_cast<const void*>(it.src)) + e0 * elem_size,
                static_cast<size_t>(n * elem_size));
    return;
  }
  float* dst = reinterpret_cast<float*>(dst_base) + it.dst_offset + e0;
  const char* src = reinterpret_cast<const char*>(it.src);
  switch (it.kind) {
    case kI64: convert<int64_t>(src + e0 * 8, dst, n); break;
    case kI32: convert<int32_t>(src + e0 * 4, dst, n); break;
    case kI16: convert<int16_t>(src + e0 * 2, dst, n); break;
    case kI8: convert<int8_t>(src + e0, dst, n); break;
    case kU8: convert<uint8_t>(src + e0, dst, n); break;
    case kBool: {
      const uint8_t* b = reinterpret_cast<const uint8_t*>(src + e0);
      for (int64_t i = 0; i < n; ++i) dst[i] = b[i] ? 1.0f : 0.0f;
      break;
    }
    default: break;
  }
}

int64_t item_bytes(const fedavg_pack_item& it, int64_t elem_size) {
  switch (it.kind) {
    case kRaw: return it.numel * elem_size;
    case kI64: return it.numel * 8;
    case kI32: return it.numel * 4;
    case kI16: return it.numel * 2;
    default: return it.numel;
  }
}

// Minimal persistent pool: run(n, fn) calls fn(t) for t in [0, n) on up to
// n threads (the caller is worker 0) and returns when all are done.
class Pool {
 public:
  static Pool& get() {
    static Pool p;
    return p;
  }

  void run(int n, const std::function<void(int)>& fn) {
    if (n <= 1) {
      fn(0);
      return;
    }
    std::lock_guard<std::mutex> call_lock(call_mu_);  // one parallel region at a time
    ensure(n - 1);
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &fn;
      njobs_ = n;
      next_.store(1);
      pending_ = n - 1;
      ++gen_;
    }
    cv_.notify_all();
    fn(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return pending_ == 0; });
    job_ = nullptr;
  }

  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }

 private:
  void ensure(int workers) {
    while (static_cast<int>(threads_.size()) < workers) threads_.emplace_back([this] { loop(); });
  }

  void loop() {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        job = job_;
      }
      for (;;) {
        const int t = next_.fetch_add(1);
        if (t >= njobs_) break;
        (*job)(t);
        std::lock_guard<std::mutex> lk(mu_);
        if (--pending_ == 0) done_cv_.notify_one();
      }
    }
  }

  std::mutex call_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> threads_;
  const std::function<void(int)>* job_ = nullptr;
  std::atomic<int> next_{0};
  int njobs_ = 0;
  int pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace

extern "C" int fedavg_pack_rows(const fedavg_pack_item* items, int64_t n_items, void* dst_base, int64_t elem_size,
                                int n_threads) {
  if (n_items < 0 || (n_items > 0 && (!items || !dst_base)) || (elem_size != 2 && elem_size != 4 && elem_size != 8))
    return FEDAVG_EINVAL;
  for (int64_t i = 0; i < n_items; ++i) {
    const fedavg_pack_item& it = items[i];
    if (it.numel < 0 || it.dst_offset < 0 || it.kind < kRaw || it.kind > kBool || (it.numel > 0 && !it.src))
      return FEDAVG_EINVAL;
    if (it.kind != kRaw && elem_size != 4) return FEDAVG_EINVAL;  // promotion targets fp32 only
  }
  // prefix sums of source bytes; each worker takes an equal byte range
  std::vector<int64_t> start(static_cast<size_t>(n_items) + 1, 0);
  for (int64_t i = 0; i < n_items; ++i) start[i + 1] = start[i] + item_bytes(items[i], elem_size);
  const int64_t total = start[n_items];
  if (total == 0) return FEDAVG_OK;
  constexpr int64_t kMinBytesPerThread = 1 << 20;  // below ~1 MiB a thread costs more than it saves
  int nt = std::max(1, std::min<int>(n_threads > 0 ? n_threads : 1,
                                     static_cast<int>((total + kMinBytesPerThread - 1) / kMinBytesPerThread)));
  char* dst = static_cast<char*>(dst_base);
  Pool::get().run(nt, [&](int t) {
    const int64_t b0 = total * t / nt, b1 = total * (t + 1) / nt;
    int64_t i = std::upper_bound(start.begin(), start.end(), b0) - start.begin() - 1;
    for (; i < n_items && start[i] < b1; ++i) {
      const fedavg_pack_item& it = items[i];
      const int64_t ib = start[i + 1] - start[i];
      if (ib == 0) continue;
      const int64_t per = ib / it.numel;  // source bytes per element
      const int64_t lo = std::max(b0, start[i]) - start[i];
      const int64_t hi = std::min(b1, start[i + 1]) - start[i];
      // element range [ceil(lo/per), ceil(hi/per)): each element is owned by
      // the worker whose byte range holds its first byte
      copy_range(it, dst, elem_size, (lo + per - 1) / per, (hi + per - 1) / per);
    }
  });
  return FEDAVG_OK;
}
