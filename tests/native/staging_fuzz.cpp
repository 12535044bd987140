// Sanitizer fuzz of the native host code (test infrastructure; no GPU).
//
//   g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all \
//       -I include -I mobile-federated-learning_amd/csrc tests/native/staging_fuzz.cpp \
//       mobile-federated-learning_amd/csrc/fedavg_host.cpp -pthread -o /tmp/staging_fuzz
//   /tmp/staging_fuzz [iterations] [seed]        (tests/test_native_sanitized.py runs it)
//
// What it checks, over random key tables and client counts:
// * fedavg_device_round_f32's host staging (staging.hpp stage_device_round)
//   for every plan form the round can take -- the LDS-DMA tiles with and
//   without the unit map, every window instance (KMAX 16/32/48/64/80/100/128)
//   with its descriptor table, the split-row windows, the non-fused reduce's
//   wide and narrow units -- with n_keys 1..5,000 and K 1..1,024, integer keys
//   converted or not, misaligned sources clearing the fused pass: the host
//   buffer is exactly round_ws(K, n_keys).end bytes (ASan flags any write past
//   it), every written byte lies below the bytes the H2D ships, and the
//   descriptor table / unit map / converted pointers hold what the kernels
//   expect;
// * stage_segment_tables and stage_pack_items into buffers of exactly their
//   workspace sizes;
// * the host packer fedavg_pack_rows (fedavg_host.cpp, the threaded pool)
//   against a scalar restatement, into a destination of exactly the bytes
//   the items cover.
// Exit status 0 = clean; any finding aborts (ASan/UBSan) or returns 1.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "fedavg_amd.h"
#include "staging.hpp"

using namespace fedavg_staging;

namespace {

int failures = 0;
#define CHECK(cond, ...)                                   \
  do {                                                     \
    if (!(cond)) {                                         \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                   \
      std::fprintf(stderr, "\n");                          \
      if (++failures > 20) std::exit(1);                   \
    }                                                      \
  } while (0)

// last byte index that differs from `fill` (-1: none)
int64_t last_written(const unsigned char* b, int64_t n, unsigned char fill) {
  for (int64_t i = n - 1; i >= 0; --i)
    if (b[i] != fill) return i;
  return -1;
}

struct Table {
  int64_t n_keys, K, ld;
  std::vector<int64_t> numel, offset, kind, key_index, ptrs;
  std::vector<double> weights;
  bool use_index;
};

Table random_table(std::mt19937_64& rng, int64_t n_keys, int64_t K) {
  Table t;
  t.n_keys = n_keys;
  t.K = K;
  t.use_index = rng() % 3 == 0;
  t.ld = t.use_index ? n_keys + static_cast<int64_t>(rng() % 7) : n_keys;
  t.numel.resize(n_keys);
  t.offset.resize(n_keys);
  t.kind.resize(n_keys);
  int64_t off = 0;
  const int int_share = static_cast<int>(rng() % 4);  // 0: no integer keys
  for (int64_t j = 0; j < n_keys; ++j) {
    const uint64_t r = rng();
    int64_t n;
    switch (r % 8) {
      case 0: n = 0; break;                                    // an empty key
      case 1: n = 1; break;                                    // scalar buffers (num_batches_tracked)
      case 2: n = static_cast<int64_t>(rng() % 100000); break;  // a large key
      default: n = static_cast<int64_t>(rng() % 2000); break;
    }
    t.numel[j] = n;
    t.offset[j] = off;
    off += n;
    t.kind[j] = (int_share && rng() % (8 / int_share) == 0) ? 1 + static_cast<int64_t>(rng() % 6) : kRaw;
  }
  if (t.use_index) {
    t.key_index.resize(n_keys);
    std::vector<int64_t> cols(t.ld);
    for (int64_t c = 0; c < t.ld; ++c) cols[c] = c;
    std::shuffle(cols.begin(), cols.end(), rng);
    for (int64_t j = 0; j < n_keys; ++j) t.key_index[j] = cols[j];
  }
  t.ptrs.assign(static_cast<size_t>(K * t.ld), 0);
  const bool misalign = rng() % 5 == 0;  // one 4-B aligned fp32 source: no fused pass
  for (int64_t k = 0; k < K; ++k)
    for (int64_t j = 0; j < n_keys; ++j) {
      const int64_t col = t.use_index ? t.key_index[j] : j;
      // fake device addresses (never dereferenced): 256-B apart per key, 1 GiB per client
      int64_t p = (int64_t(1) << 40) + k * (int64_t(1) << 30) + col * 4096;
      if (t.kind[j] != kRaw) p += 1 + static_cast<int64_t>(rng() % 3);  // integer sources: any alignment
      t.ptrs[static_cast<size_t>(k * t.ld + col)] = t.numel[j] > 0 ? p : (rng() % 2 ? 0 : p);
    }
  if (misalign) {
    for (int64_t j = 0; j < n_keys; ++j)
      if (t.kind[j] == kRaw && t.numel[j] > 0) {
        const int64_t col = t.use_index ? t.key_index[j] : j;
        t.ptrs[static_cast<size_t>((K - 1) * t.ld + col)] += 4;
        break;
      }
  }
  t.weights.resize(K);
  for (int64_t k = 0; k < K; ++k) t.weights[k] = 1.0 / static_cast<double>(k + 1);
  return t;
}

// the forms fedavg_device_round_f32's plan can take (seg_fused_plan / segments_small)
std::vector<RoundPlan> plan_forms(int64_t K) {
  std::vector<RoundPlan> f;
  for (int64_t span : {64, 128, 256, 512, 1024}) f.push_back(RoundPlan{false, 0, span, false});  // tiles
  const int kmaxes[] = {16, 32, 48, 64, 80, 100, 128};
  const int vecs[] = {4, 4, 4, 2, 2, 2, 1};
  for (int i = 0; i < 7; ++i)
    if (K <= kmaxes[i]) f.push_back(RoundPlan{true, kmaxes[i], 64 * vecs[i], false});
  f.push_back(RoundPlan{true, -1, 64, false});  // split-row windows
  return f;
}

void fuzz_device_round(std::mt19937_64& rng, int64_t n_keys, int64_t K, bool every_form) {
  const Table t = random_table(rng, n_keys, K);
  int64_t n_int = 0;
  const int64_t S = int_scratch_cols(t.numel.data(), t.kind.data(), n_keys, &n_int);
  const RoundWs L = round_ws(K, n_keys);
  std::vector<RoundPlan> forms = plan_forms(K);
  forms.push_back(RoundPlan{false, 0, 8192, false});  // non-fused: wide units
  forms.push_back(RoundPlan{false, 0, 1024, true});   // non-fused: narrow units
  if (!every_form) {  // a random trial: three forms, one fill pattern (the edges take all, both)
    std::shuffle(forms.begin(), forms.end(), rng);
    forms.resize(forms.size() < 3 ? forms.size() : 3);
  }
  const std::vector<unsigned char> fills = every_form ? std::vector<unsigned char>{0x00, 0xFF}
                                                      : std::vector<unsigned char>{static_cast<unsigned char>(rng())};
  for (const RoundPlan& form : forms) {
    const bool want_fuse = form.win || form.span <= 1024;
    for (unsigned char fill : fills) {
      // exactly the reserved bytes: ASan reports any write past them
      auto* buf = static_cast<unsigned char*>(std::malloc(static_cast<size_t>(L.end)));
      std::memset(buf, fill, static_cast<size_t>(L.end));
      RoundIn in{t.ptrs.data(), t.ld, t.use_index ? t.key_index.data() : nullptr, t.numel.data(), t.offset.data(),
                 t.kind.data(), n_keys, K, t.weights.data(), int64_t(1) << 44, K * S, want_fuse,
                 rng() % 8 == 0};
      bool fused_seen = false;
      const auto plan_fn = [&](bool fuse, bool) -> RoundPlan {
        fused_seen = fuse;
        return fuse ? form : RoundPlan{false, 0, form.small ? 1024 : 8192, form.small};
      };
      RoundOut st;
      Msg msg;
      const int rc = stage_device_round(in, buf, L.end, plan_fn, &st, &msg);
      CHECK(rc == FEDAVG_OK, "stage_device_round K=%lld n=%lld: %s", (long long)K, (long long)n_keys, msg.text);
      if (rc == FEDAVG_OK && st.first_src) {
        CHECK(st.bytes <= L.end, "bytes %lld > end %lld", (long long)st.bytes, (long long)L.end);
        const int64_t lw = last_written(buf, L.end, fill);
        CHECK(lw < st.bytes, "a staged byte (%lld) lies past the shipped bytes (%lld); K=%lld n=%lld kmax=%d",
              (long long)lw, (long long)st.bytes, (long long)K, (long long)n_keys, st.plan.kmax);
        CHECK(fused_seen == st.fuse, "plan_fn saw fuse=%d, round fuse=%d", fused_seen, st.fuse);
        if (st.with_desc)
          CHECK(st.moff + seg_desc_bytes(n_keys, st.plan.kmax) <= L.end, "descriptor table past the room");
        if (st.with_map) CHECK(st.moff + st.units * 4 <= L.end, "unit map past the room");
        const auto* hp = reinterpret_cast<const int64_t*>(buf + L.ptrs);
        if (st.with_desc) {  // the descriptors the windows load: client i's address of key j, its bytes
          const auto* hd = reinterpret_cast<const Desc*>(buf + st.moff);
          const int64_t km = st.plan.kmax;
          for (int64_t j = 0; j <= n_keys; j += 1 + n_keys / 64)
            for (int64_t i = 0; i < km; i += 1 + km / 16) {
              const Desc d = hd[j * km + i];
              const bool live = j < n_keys && t.numel[j] > 0 && i < K;
              const uint64_t p = live ? static_cast<uint64_t>(hp[j * K + i]) : 0;
              CHECK(d.addr_lo == static_cast<uint32_t>(p) && d.addr_hi == static_cast<uint32_t>(p >> 32) &&
                        d.records == (p ? static_cast<uint32_t>(t.numel[j] * 4) : 0u) && d.flags == kWinRsrcFlags,
                    "descriptor (%lld, %lld)", (long long)j, (long long)i);
            }
        }
        if (st.with_map) {  // the unit -> key map covers every unit with its key
          const auto* hm = reinterpret_cast<const int*>(buf + st.moff);
          const auto* hk = reinterpret_cast<const SegKey*>(buf);
          for (int64_t u = 0; u < st.units; u += 1 + st.units / 257) {
            const int64_t j = hm[u];
            CHECK(j >= 0 && j < n_keys && hk[j].unit_start <= u, "unit map at %lld", (long long)u);
          }
        }
        if (st.converted) {  // converted integer keys read their fp32 scratch columns
          const auto* hk = reinterpret_cast<const SegKey*>(buf);
          for (int64_t j = 0; j < n_keys; ++j) CHECK(hk[j].kind == kRaw, "converted key %lld kind", (long long)j);
          const auto* hik = reinterpret_cast<const IntKey*>(buf + L.ik);
          int64_t q = 0;
          for (int64_t j = 0; j < n_keys; ++j)
            if (t.kind[j] != kRaw && t.numel[j] > 0) {
              CHECK(hik[q].numel == t.numel[j] && hik[q].col + t.numel[j] <= S, "int key %lld", (long long)j);
              const int64_t p = hp[j * K + (K - 1)];
              CHECK(p == (int64_t(1) << 44) + ((K - 1) * S + hik[q].col) * 4, "scratch pointer of key %lld",
                    (long long)j);
              ++q;
            }
          CHECK(q == n_int, "converted %lld of %lld integer keys", (long long)q, (long long)n_int);
        }
        const auto* hw = reinterpret_cast<const float*>(buf + L.w);
        CHECK(hw[K - 1] == static_cast<float>(t.weights[K - 1]), "weights");
      }
      std::free(buf);
    }
  }
}

void fuzz_segment_tables(std::mt19937_64& rng, int64_t n_keys, int64_t K) {
  Table t = random_table(rng, n_keys, K);
  // stage_tables takes the client-major [K, n_keys] table without an index,
  // every non-empty source 4-B aligned for raw keys
  std::vector<int64_t> ptrs(static_cast<size_t>(K * n_keys));
  for (int64_t k = 0; k < K; ++k)
    for (int64_t j = 0; j < n_keys; ++j)
      ptrs[static_cast<size_t>(k * n_keys + j)] =
          (int64_t(1) << 40) + k * (int64_t(1) << 30) + j * 4096 + (t.kind[j] == kRaw ? 0 : 1);
  const int64_t ws = segments_workspace_bytes(K, n_keys);
  auto* buf = static_cast<unsigned char*>(std::malloc(static_cast<size_t>(ws)));
  TablesOut st;
  Msg msg;
  const int rc = stage_segment_tables(ptrs.data(), t.numel.data(), t.offset.data(), t.kind.data(), n_keys, K, buf, ws,
                                      int64_t(1) << (6 + rng() % 8), &st, &msg);
  CHECK(rc == FEDAVG_OK, "stage_segment_tables: %s", msg.text);
  std::free(buf);
}

void fuzz_pack(std::mt19937_64& rng) {
  const int64_t n_items = 1 + static_cast<int64_t>(rng() % 1500);
  const int64_t elem_size = (rng() % 4 == 0) ? 8 : 4;
  std::vector<std::vector<unsigned char>> srcs(static_cast<size_t>(n_items));
  std::vector<fedavg_pack_item> items(static_cast<size_t>(n_items));
  int64_t off = 0;
  for (int64_t i = 0; i < n_items; ++i) {
    const int64_t n = rng() % 64 == 0 ? static_cast<int64_t>(rng() % 200000) : static_cast<int64_t>(rng() % 700);
    const int64_t kind = (elem_size == 4 && rng() % 5 == 0) ? 1 + static_cast<int64_t>(rng() % 6) : kRaw;
    const int64_t src_es = kind == kRaw ? elem_size : (kind == 1 ? 8 : kind == 2 ? 4 : kind == 3 ? 2 : 1);
    auto& v = srcs[static_cast<size_t>(i)];
    v.resize(static_cast<size_t>(n * src_es));  // exactly the item's bytes (ASan-bounded)
    for (auto& c : v) c = static_cast<unsigned char>(rng());
    if (kind == kBool)
      for (auto& c : v) c &= 1;
    items[static_cast<size_t>(i)] =
        fedavg_pack_item{n ? reinterpret_cast<int64_t>(v.data()) : 0, n, off, kind};
    off += n + static_cast<int64_t>(rng() % 5);  // gaps between keys (row padding)
  }
  // workspace staging of the same items
  const int64_t ws = pack_rows_device_workspace_bytes(n_items);
  auto* wbuf = static_cast<unsigned char*>(std::malloc(static_cast<size_t>(ws)));
  PackOut po;
  Msg msg;
  int rc = stage_pack_items(items.data(), n_items, elem_size, wbuf, ws, &po, &msg);
  CHECK(rc == FEDAVG_OK, "stage_pack_items: %s", msg.text);
  std::free(wbuf);
  // the threaded host packer into exactly the covered bytes, against a scalar restatement
  const int64_t dst_bytes = off * elem_size;
  std::vector<unsigned char> dst(static_cast<size_t>(dst_bytes), 0), want(static_cast<size_t>(dst_bytes), 0);
  rc = fedavg_pack_rows(items.data(), n_items, dst.data(), elem_size, 1 + static_cast<int>(rng() % 8));
  CHECK(rc == FEDAVG_OK, "fedavg_pack_rows rc=%d", rc);
  for (const fedavg_pack_item& it : items) {
    const auto* s = reinterpret_cast<const unsigned char*>(it.src);
    for (int64_t e = 0; e < it.numel; ++e) {
      unsigned char* d = want.data() + (it.dst_offset + e) * elem_size;
      if (it.kind == kRaw) {
        std::memcpy(d, s + e * elem_size, static_cast<size_t>(elem_size));
        continue;
      }
      float f = 0;
      switch (it.kind) {
        case 1: { int64_t x; std::memcpy(&x, s + e * 8, 8); f = static_cast<float>(x); break; }
        case 2: { int32_t x; std::memcpy(&x, s + e * 4, 4); f = static_cast<float>(x); break; }
        case 3: { int16_t x; std::memcpy(&x, s + e * 2, 2); f = static_cast<float>(x); break; }
        case 4: f = static_cast<float>(static_cast<int8_t>(s[e])); break;
        case 5: f = static_cast<float>(s[e]); break;
        case 6: f = s[e] ? 1.0f : 0.0f; break;
      }
      std::memcpy(d, &f, 4);
    }
  }
  CHECK(dst == want, "fedavg_pack_rows output differs from the restatement (%lld items)", (long long)n_items);
}

}  // namespace

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 200;
  const uint64_t seed = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 1234;
  std::mt19937_64 rng(seed);
  // the edges first: 1 key / 1 client, the descriptor table's room switch
  // (2,047 / 2,048 keys at KMAX 128), the unit map's limit, the largest sizes
  const int64_t edges[][2] = {{1, 1}, {1, 1024}, {2047, 128}, {2048, 128}, {2049, 17}, {5000, 1}, {5000, 100},
                              {3, 1024}, {350, 100}, {62, 500}, {4095, 64}, {4096, 100}};
  for (const auto& e : edges) {
    fuzz_device_round(rng, e[0], e[1], true);
    fuzz_segment_tables(rng, e[0], e[1]);
  }
  for (int it = 0; it < iters; ++it) {
    const int64_t n_keys = rng() % 4 == 0 ? 1 + static_cast<int64_t>(rng() % 5000) : 1 + static_cast<int64_t>(rng() % 400);
    const int64_t K = rng() % 4 == 0 ? 1 + static_cast<int64_t>(rng() % 1024) : 1 + static_cast<int64_t>(rng() % 130);
    if (n_keys * K > 1500000) continue;  // bound the run time (the edges above cover the corners)
    fuzz_device_round(rng, n_keys, K, false);
    fuzz_segment_tables(rng, n_keys, K);
    if (it % 4 == 0) fuzz_pack(rng);
  }
  std::printf("staging fuzz: %d iterations, seed %llu, %d failures\n", iters, (unsigned long long)seed, failures);
  return failures ? 1 : 0;
}
