// Host-side staging of the table-driven device calls: workspace sizes and the
// bytes the host writes into the pinned workspace before ONE H2D ships them.
//
// HIP-free on purpose: g++ compiles this header with -fsanitize=address,
// undefined in tests/native/staging_fuzz.cpp, which fuzzes key counts, client
// counts and every fused-plan form and checks that every staged byte lies
// inside the room the sizing functions reserve (round 5 shipped a descriptor
// table written past round_ws's room for > 2,047 keys on a smaller window
// instance, found by reading the code; this makes that class of bug a test).
//
// Callers: fedavg_segments.hip (stage_tables, fedavg_device_round_f32),
// fedavg_pack.hip (fedavg_pack_rows_device).  The walk they stage is over the
// reference's state_dicts (client.py:96, fedavg_trainer.py:199).
#pragma once

#include <cstdarg>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "fedavg_amd.h"

namespace fedavg_staging {

// fedavg_pack_item.kind / SegKey.kind codes (include/fedavg_amd.h)
enum : int64_t { kRaw = 0, kI64 = 1, kI32 = 2, kI16 = 3, kI8 = 4, kU8 = 5, kBool = 6 };

// the device key table entry (fedavg_segments.hip's kernels read it)
struct SegKey {
  int64_t numel, out_offset, kind, unit_start;
};
// a fused round's integer key, converted into fp32 scratch columns
struct IntKey {
  int64_t numel, kind, col;  // col: the key's first column in a client's scratch row
};
// one window descriptor: a buffer resource (address lo, hi, record count, flags)
struct Desc {
  uint32_t addr_lo, addr_hi, records, flags;
};
static_assert(sizeof(SegKey) == 32 && sizeof(IntKey) == 24 && sizeof(Desc) == 16, "staged layouts");

// the pointer table is padded so the windows' 8-address groups load unconditionally
constexpr int64_t kSegWinTablePad = 128;
// the tile kernel's unit -> key map is staged for rounds of at most this many units
constexpr int64_t kSegUnitMapMax = 65536;
// the windows' descriptor table is staged for tables of at most this size
constexpr int64_t kSegDescMaxBytes = int64_t(4) << 20;
constexpr uint32_t kWinRsrcFlags = 0x00020000;

inline int64_t round16(int64_t b) { return (b + 15) & ~int64_t(15); }

// --- fedavg_segments_workspace: SegKey[n_keys] | int64 ptrs[n_keys * K + pad]
inline int64_t segments_workspace_bytes(int64_t K, int64_t n_keys) {
  if (K <= 0 || n_keys <= 0) return 0;
  return n_keys * static_cast<int64_t>(sizeof(SegKey)) +
         (n_keys * K + kSegWinTablePad) * static_cast<int64_t>(sizeof(int64_t));
}

// --- fedavg_device_round_f32's workspace (host and device alike, 16-B aligned parts):
//   SegKey[n_keys] | int64 ptrs[n_keys * K + pad] | float w[K] | IntKey[n_keys] |
//   int64 int_src[n_keys * K] | room for the unit map OR the descriptor table
struct RoundWs {
  int64_t ptrs, w, ik, isrc, end, desc_room;
};

inline int64_t seg_desc_bytes(int64_t n_keys, int64_t kmax = 128) {
  return (n_keys + 1) * kmax * static_cast<int64_t>(sizeof(Desc));
}

inline RoundWs round_ws(int64_t K, int64_t n_keys) {
  RoundWs r;
  r.ptrs = n_keys * static_cast<int64_t>(sizeof(SegKey));
  r.w = round16(r.ptrs + (n_keys * K + kSegWinTablePad) * static_cast<int64_t>(sizeof(int64_t)));
  r.ik = r.w + round16(K * static_cast<int64_t>(sizeof(float)));
  r.isrc = r.ik + round16(n_keys * static_cast<int64_t>(sizeof(IntKey)));
  const int64_t map_bytes = kSegUnitMapMax * static_cast<int64_t>(sizeof(int));
  const int64_t desc = seg_desc_bytes(n_keys) <= kSegDescMaxBytes ? seg_desc_bytes(n_keys) : 0;
  r.desc_room = map_bytes > desc ? map_bytes : desc;
  r.end = round16(r.isrc + n_keys * K * static_cast<int64_t>(sizeof(int64_t))) + r.desc_room;
  return r;
}

// --- fedavg_pack_rows_device's workspace: fedavg_pack_item[n] | int64 start[n + 1]
inline int64_t pack_items_bytes(int64_t n_items) { return n_items * static_cast<int64_t>(sizeof(fedavg_pack_item)); }
inline int64_t pack_rows_device_workspace_bytes(int64_t n_items) {
  if (n_items < 0) return -1;
  return pack_items_bytes(n_items) + (n_items + 1) * static_cast<int64_t>(sizeof(int64_t));
}

// error text of a refused staging (the callers hand it to set_error)
struct Msg {
  char text[256];
  int fail(int rc, const char* fmt, ...) __attribute__((format(printf, 3, 4))) {
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(text, sizeof(text), fmt, ap);
    va_end(ap);
    return rc;
  }
};

// ---------------------------------------------------------------------------
// stage_tables (fedavg_segments.hip): the key table and the key-major pointer
// table into host_ws (>= segments_workspace_bytes).  `units` = the units of
// `span` columns; first/last non-empty sources for the caller's spot check.
// ---------------------------------------------------------------------------
struct TablesOut {
  int64_t units;
  const void* first_src;
  const void* last_src;
};

inline int stage_segment_tables(const int64_t* client_ptrs, const int64_t* numel, const int64_t* offset,
                                const int64_t* kind, int64_t n_keys, int64_t K, void* host_ws, int64_t ws_bytes,
                                int64_t span, TablesOut* out, Msg* msg) {
  if (ws_bytes < segments_workspace_bytes(K, n_keys))
    return msg->fail(FEDAVG_EINVAL, "workspace needs %lld bytes", (long long)segments_workspace_bytes(K, n_keys));
  auto* hk = static_cast<SegKey*>(host_ws);
  auto* hp = reinterpret_cast<int64_t*>(static_cast<char*>(host_ws) + n_keys * static_cast<int64_t>(sizeof(SegKey)));
  *out = TablesOut{0, nullptr, nullptr};
  int64_t units = 0;
  for (int64_t j = 0; j < n_keys; ++j) {
    if (numel[j] < 0 || offset[j] < 0 || kind[j] < kRaw || kind[j] > kBool)
      return msg->fail(FEDAVG_EINVAL, "bad key %lld", (long long)j);
    hk[j] = SegKey{numel[j], offset[j], kind[j], units};
    units += (numel[j] + span - 1) / span;
    for (int64_t k = 0; k < K; ++k) {
      const int64_t p = client_ptrs[k * n_keys + j];
      if (numel[j] > 0) {
        if (p == 0 || (kind[j] == kRaw && (p & 3) != 0))
          return msg->fail(FEDAVG_EINVAL, "client %lld key %lld: null or misaligned source", (long long)k,
                           (long long)j);
        if (!out->first_src) out->first_src = reinterpret_cast<const void*>(p);
        out->last_src = reinterpret_cast<const void*>(p);
      }
      hp[j * K + k] = p;
    }
  }
  out->units = units;
  return FEDAVG_OK;
}

// ---------------------------------------------------------------------------
// fedavg_pack_rows_device: the items and their element starts into host_ws
// (>= pack_rows_device_workspace_bytes).
// ---------------------------------------------------------------------------
struct PackOut {
  int64_t total, max_numel;
  const void* first_src;
  const void* last_src;
};

inline int stage_pack_items(const fedavg_pack_item* items, int64_t n_items, int64_t elem_size, void* host_ws,
                            int64_t ws_bytes, PackOut* out, Msg* msg) {
  if (ws_bytes < pack_rows_device_workspace_bytes(n_items))
    return msg->fail(FEDAVG_EINVAL, "workspace needs %lld bytes", (long long)pack_rows_device_workspace_bytes(n_items));
  auto* h_items = static_cast<fedavg_pack_item*>(host_ws);
  auto* h_start = reinterpret_cast<int64_t*>(static_cast<char*>(host_ws) + pack_items_bytes(n_items));
  *out = PackOut{0, 0, nullptr, nullptr};
  int64_t total = 0;
  for (int64_t i = 0; i < n_items; ++i) {
    const fedavg_pack_item& it = items[i];
    if (it.numel < 0 || it.dst_offset < 0 || it.kind < kRaw || it.kind > kBool || (it.numel > 0 && !it.src) ||
        (it.kind != kRaw && elem_size != 4))
      return msg->fail(FEDAVG_EINVAL, "bad item %lld", (long long)i);
    h_items[i] = it;
    h_start[i] = total;
    total += it.numel;
    if (it.numel > out->max_numel) out->max_numel = it.numel;
    if (it.numel > 0) {
      if (!out->first_src) out->first_src = reinterpret_cast<const void*>(it.src);
      out->last_src = reinterpret_cast<const void*>(it.src);
    }
  }
  h_start[n_items] = total;
  out->total = total;
  return FEDAVG_OK;
}

// ---------------------------------------------------------------------------
// fedavg_device_round_f32: everything the host writes before the tables' H2D.
//
// `plan_fn(fuse, all_raw)` decides the round's form once the sources are known
// (a misaligned fp32 source clears `fuse`): win / kmax (window instance, -1 =
// the split-row windows) / span (the unit width the key table is staged with)
// / small (the narrow units of a non-fused round).  The fuzz harness passes
// every form; production passes seg_fused_plan (fedavg_segments.hip).
// ---------------------------------------------------------------------------
struct RoundPlan {
  bool win;
  int kmax;
  int64_t span;
  bool small;
};

struct RoundIn {
  const int64_t* client_ptrs;
  int64_t ptr_ld;
  const int64_t* key_index;  // null: key j is column j
  const int64_t* key_numel;
  const int64_t* key_offset;
  const int64_t* key_kind;
  int64_t n_keys, K;
  const double* weights;
  int64_t int_scratch;    // device address of the [K, S] fp32 scratch (0: none)
  int64_t scratch_elems;  // its floats
  bool fuse;            // the caller asked for the fused :291 sums (and K allows them)
  bool desc_disabled;   // FEDAVG_SEGWIN_DESC=0
};

struct RoundOut {
  RoundPlan plan;
  bool fuse, converted, with_map, with_desc;
  int64_t S, n_int, units, used, moff, bytes;  // bytes: what the H2D ships (from host_ws[0])
  const void* first_src;                        // null: every key is empty (nothing staged after the pointers)
  const void* last_src;
};

// the integer keys' scratch row width (fp32 columns, each key 4-aligned) and count
inline int64_t int_scratch_cols(const int64_t* key_numel, const int64_t* key_kind, int64_t n_keys, int64_t* n_int) {
  int64_t S = 0, n = 0;
  for (int64_t j = 0; j < n_keys; ++j)
    if (key_kind[j] != kRaw && key_numel[j] > 0) {
      S += (key_numel[j] + 3) & ~int64_t(3);
      ++n;
    }
  if (n_int) *n_int = n;
  return S;
}

template <class PlanFn>
int stage_device_round(const RoundIn& in, void* host_ws, int64_t ws_bytes, PlanFn&& plan_fn, RoundOut* out,
                       Msg* msg) {
  const int64_t n_keys = in.n_keys, K = in.K, ld = in.ptr_ld;
  const RoundWs L = round_ws(K, n_keys);
  if (ws_bytes < L.end) return msg->fail(FEDAVG_EINVAL, "workspace needs %lld bytes", (long long)L.end);
  char* hb = static_cast<char*>(host_ws);
  auto* hk = reinterpret_cast<SegKey*>(hb);
  auto* hp = reinterpret_cast<int64_t*>(hb + L.ptrs);
  auto* hw = reinterpret_cast<float*>(hb + L.w);
  auto* hik = reinterpret_cast<IntKey*>(hb + L.ik);
  auto* hsrc = reinterpret_cast<int64_t*>(hb + L.isrc);
  *out = RoundOut{};
  bool fuse = in.fuse;
  // keys: validation, the integer keys' scratch columns
  int64_t S = 0, n_int = 0;
  for (int64_t j = 0; j < n_keys; ++j) {
    const int64_t col = in.key_index ? in.key_index[j] : j;
    if (in.key_numel[j] < 0 || in.key_offset[j] < 0 || in.key_kind[j] < kRaw || in.key_kind[j] > kBool || col < 0 ||
        (in.key_index && col >= ld))
      return msg->fail(FEDAVG_EINVAL, "bad key %lld", (long long)j);
    if (in.key_kind[j] != kRaw && in.key_numel[j] > 0) {
      S += (in.key_numel[j] + 3) & ~int64_t(3);
      ++n_int;
    }
  }
  if (S >= (int64_t(1) << 31)) return msg->fail(FEDAVG_EINVAL, "integer keys too large");
  if (fuse && n_int > 0 && (in.int_scratch == 0 || (in.int_scratch & 15) != 0 || in.scratch_elems < K * S))
    return msg->fail(FEDAVG_EINVAL, "integer keys need an aligned device scratch of %lld floats", (long long)(K * S));
  // the pointer table, key-major, filled client-major (the order the walk's
  // table was written in); per key the masks its sources are checked with (a
  // non-empty key needs a non-null source; fp32 sources 4-B aligned, 16-B for
  // the fused pass)
  struct KeyFill {
    int64_t col, need, align, fuse_mask;
  };
  thread_local std::vector<KeyFill> kf;
  thread_local std::vector<int64_t> conv_j, conv_col;
  kf.resize(static_cast<size_t>(n_keys));
  for (int64_t j = 0; j < n_keys; ++j) {
    const bool live = in.key_numel[j] > 0, raw = in.key_kind[j] == kRaw;
    kf[j] = KeyFill{in.key_index ? in.key_index[j] : j, live ? 1 : 0, live && raw ? 3 : 0, live && raw ? 15 : 0};
  }
  int64_t fuse_bits = 0;
  for (int64_t k = 0; k < K; ++k) {
    const int64_t* row = in.client_ptrs + k * ld;
    int64_t bad = 0;
    for (int64_t j = 0; j < n_keys; ++j) {
      const KeyFill f = kf[j];
      const int64_t p = row[f.col];
      hp[j * K + k] = p;
      bad |= (f.need & static_cast<int64_t>(p == 0)) | (p & f.align);
      fuse_bits |= p & f.fuse_mask;
    }
    if (bad) {
      for (int64_t j = 0; j < n_keys; ++j) {
        const int64_t p = row[kf[j].col];
        if ((kf[j].need && p == 0) || (p & kf[j].align))
          return msg->fail(FEDAVG_EINVAL, "client %lld key %lld: null or misaligned source", (long long)k,
                           (long long)j);
      }
    }
  }
  if (fuse_bits) fuse = false;  // a misaligned fp32 source: the reduce alone (integer keys stay as they are)
  const bool converted = fuse && n_int > 0;
  // the converted integer keys: their sources into int_src, their table
  // entries pointed at their scratch columns
  conv_j.clear();
  conv_col.clear();
  if (converted) {
    int64_t soff = 0;
    for (int64_t j = 0; j < n_keys; ++j)
      if (in.key_kind[j] != kRaw && in.key_numel[j] > 0) {
        hik[conv_j.size()] = IntKey{in.key_numel[j], in.key_kind[j], soff};
        conv_j.push_back(j);
        conv_col.push_back(soff);
        soff += (in.key_numel[j] + 3) & ~int64_t(3);
      }
    for (size_t q = 0; q < conv_j.size(); ++q) {
      const int64_t j = conv_j[q];
      for (int64_t k = 0; k < K; ++k) {
        hsrc[static_cast<int64_t>(q) * K + k] = hp[j * K + k];
        hp[j * K + k] = in.int_scratch + (k * S + conv_col[q]) * static_cast<int64_t>(sizeof(float));
      }
    }
  }
  // the spot-checked sources: client 0's first and client K-1's last non-empty key
  for (int64_t j = 0; j < n_keys && !out->first_src; ++j)
    if (kf[j].need) out->first_src = reinterpret_cast<const void*>(in.client_ptrs[kf[j].col]);
  for (int64_t j = n_keys - 1; j >= 0 && !out->last_src; --j)
    if (kf[j].need) out->last_src = reinterpret_cast<const void*>(in.client_ptrs[(K - 1) * ld + kf[j].col]);
  out->fuse = fuse;
  out->converted = converted;
  out->S = S;
  out->n_int = n_int;
  if (!out->first_src) return FEDAVG_OK;  // every key empty
  // the unit width, then the key table
  const bool all_raw = converted || n_int == 0;
  const RoundPlan plan = plan_fn(fuse, all_raw);
  int64_t units = 0;
  for (int64_t j = 0; j < n_keys; ++j) {
    hk[j] = SegKey{in.key_numel[j], in.key_offset[j], converted ? kRaw : in.key_kind[j], units};
    units += (in.key_numel[j] + plan.span - 1) / plan.span;
  }
  // the tiles' unit -> key map, or the windows' descriptor table, right after
  // the last part in use, within the room round_ws reserved
  const int64_t used = converted ? L.isrc + n_int * K * static_cast<int64_t>(sizeof(int64_t)) : L.ik;
  const int64_t moff = round16(used);
  const bool with_map = fuse && !plan.win && units > 0 && units <= kSegUnitMapMax;
  if (with_map) {
    int* hm = reinterpret_cast<int*>(hb + moff);
    for (int64_t j = 0; j < n_keys; ++j) {
      const int64_t u1 = j + 1 < n_keys ? hk[j + 1].unit_start : units;
      for (int64_t u = hk[j].unit_start; u < u1; ++u) hm[u] = static_cast<int>(j);
    }
  }
  // the windows' descriptor table: client i's address of key j, the key's
  // byte length (every load's range check), the flags; padding rows and
  // empty keys get a record count of 0, and KMAX null descriptors follow the
  // last key (the reload target when the next window is not a full one).  A
  // table of more than 2,047 keys at KMAX 128 has no room reserved, and a
  // smaller KMAX's table must not overrun it.
  const int64_t dbytes = fuse && plan.win && plan.kmax > 0 ? seg_desc_bytes(n_keys, plan.kmax) : 0;
  const bool with_desc = fuse && plan.win && plan.kmax > 0 && dbytes <= kSegDescMaxBytes && dbytes <= L.desc_room &&
                         !in.desc_disabled;
  if (with_desc) {
    auto* hd = reinterpret_cast<Desc*>(hb + moff);
    const int64_t km = plan.kmax;
    for (int64_t j = 0; j <= n_keys; ++j) {
      const bool live = j < n_keys && in.key_numel[j] > 0;
      const uint32_t nrec = live ? static_cast<uint32_t>(in.key_numel[j] * 4) : 0u;
      for (int64_t i = 0; i < km; ++i) {
        const uint64_t p = live && i < K ? static_cast<uint64_t>(hp[j * K + i]) : 0;
        hd[j * km + i] = Desc{static_cast<uint32_t>(p), static_cast<uint32_t>(p >> 32), p ? nrec : 0u, kWinRsrcFlags};
      }
    }
  }
  // the reference's weights n_i / N (fedavg_trainer.py:453) rounded once to
  // fp32 (nearest even, the cast ATen applies to the scalar at :455)
  for (int64_t k = 0; k < K; ++k) hw[k] = static_cast<float>(in.weights[k]);
  out->plan = plan;
  out->with_map = with_map;
  out->with_desc = with_desc;
  out->units = units;
  out->used = used;
  out->moff = moff;
  out->bytes = with_map ? moff + units * static_cast<int64_t>(sizeof(int)) : (with_desc ? moff + dbytes : used);
  return FEDAVG_OK;
}

}  // namespace fedavg_staging
