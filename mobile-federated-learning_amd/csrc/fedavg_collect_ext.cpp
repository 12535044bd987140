// fedavg_collect_ext.cpp -- native walk over the clients' state_dicts.
//
// aggregate() must check every client's tensor for every key of client 0
// (fedavg_trainer.py:450-457 reads p_i[k] for all i, k) and gather its host
// address for the packer (csrc/fedavg_host.cpp).  In Python that costs about
// 0.75 us per tensor (26 ms for resnet56 x 100 clients, 35,000 tensors); here
// the dict lookups and tensor metadata are read through the torch C++ API.
//
// collect(dicts, names, template, device_index=-1, strict0=False) -> (ptrs[K, N] int64, bad_client, bad_key)
//   template[j] is client 0's tensor for names[j].  A client tensor passes
//   when it has the template's sizes and dtype and is contiguous, on the host
//   (device_index -1) or on HIP device `device_index` (device-resident clients).
//   On the first one that does not (or a missing key), the scan stops and
//   returns its (client, key) index so the Python layer can raise the
//   reference's exception or take its general path; otherwise (-1, -1).
//   strict0: client 0 must be a dict whose entries are exactly `names` in
//   order (else (None, 0, -1) at once) -- KeyTable.try_collect's check that a
//   table from an earlier round still fits, without a Python pass over the
//   key strings.
#include <torch/csrc/autograd/python_variable.h>
#include <torch/extension.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstring>
#include <vector>

#include <pybind11/stl.h>

namespace py = pybind11;

// Key equality without the Python API, for the walker threads: the key
// objects of different clients' state_dicts are equal strings but rarely the
// same objects (each net.cpu().state_dict() call builds its own names,
// client.py:96), so an identity test alone sends every client to the slow
// path.  Exact str objects compare by length, kind and bytes (immutable once
// ready; the cached hashes when both exist); anything else reports "unknown"
// and the caller falls back to PyObject_RichCompareBool under the GIL.
enum class KeyEq { kSame, kDiffer, kUnknown };
static inline KeyEq key_eq(PyObject* a, PyObject* b) {
  if (a == b) return KeyEq::kSame;
  if (!PyUnicode_CheckExact(a) || !PyUnicode_CheckExact(b) || !PyUnicode_IS_READY(a) || !PyUnicode_IS_READY(b))
    return KeyEq::kUnknown;
  const Py_ssize_t n = PyUnicode_GET_LENGTH(a);
  if (n != PyUnicode_GET_LENGTH(b) || PyUnicode_KIND(a) != PyUnicode_KIND(b)) return KeyEq::kDiffer;
  const Py_hash_t ha = reinterpret_cast<PyASCIIObject*>(a)->hash, hb = reinterpret_cast<PyASCIIObject*>(b)->hash;
  if (ha != -1 && hb != -1 && ha != hb) return KeyEq::kDiffer;
  return std::memcmp(PyUnicode_DATA(a), PyUnicode_DATA(b), static_cast<size_t>(n) * PyUnicode_KIND(a)) == 0
             ? KeyEq::kSame
             : KeyEq::kDiffer;
}

static py::tuple collect(py::list dicts, py::list names, py::list templ, int64_t device_index, bool strict0) {
  const Py_ssize_t K = PyList_GET_SIZE(dicts.ptr());
  const Py_ssize_t N = PyList_GET_SIZE(names.ptr());
  if (PyList_GET_SIZE(templ.ptr()) != N) throw std::invalid_argument("template/names length mismatch");
  std::vector<std::vector<int64_t>> sizes(N);
  std::vector<at::ScalarType> dtypes(N);
  for (Py_ssize_t j = 0; j < N; ++j) {
    PyObject* t = PyList_GET_ITEM(templ.ptr(), j);
    if (!THPVariable_Check(t)) throw std::invalid_argument("template entries must be tensors");
    const at::Tensor& ten = THPVariable_Unpack(t);
    sizes[j] = ten.sizes().vec();
    dtypes[j] = ten.scalar_type();
  }
  // the value objects, [K][N]: a dict whose entries are the names in order
  // (exact strings, key_eq) is read by PyDict_Next on torch's intra-op threads together with the
  // metadata checks below; any other mapping afterwards on this thread by
  // lookups (their new references held until the end).  The calling thread
  // keeps the GIL: no Python code runs meanwhile, and the threads call no
  // Python API besides PyDict_Next (no reference counts touched)
  std::vector<PyObject*> vals(static_cast<size_t>(K) * N);
  std::vector<PyObject*> owned;
  auto release = [&owned] {
    for (PyObject* o : owned) Py_DECREF(o);
    owned.clear();
  };
  std::vector<PyObject*> name_ptr(N);
  std::vector<Py_hash_t> name_hash(N);
  for (Py_ssize_t j = 0; j < N; ++j) {
    name_ptr[j] = PyList_GET_ITEM(names.ptr(), j);
    name_hash[j] = PyObject_Hash(name_ptr[j]);
    if (name_hash[j] == -1) {
      PyErr_Clear();
      return py::make_tuple(py::none(), 0, j);
    }
  }
  std::vector<PyObject*> dobj(K);
  for (Py_ssize_t i = 0; i < K; ++i) dobj[i] = PyList_GET_ITEM(dicts.ptr(), i);
  auto ptrs = torch::empty({static_cast<int64_t>(K), static_cast<int64_t>(N)}, torch::kInt64);
  int64_t* out = ptrs.data_ptr<int64_t>();
  std::vector<int64_t> bad(static_cast<size_t>(K), -1);  // per client: first failing key; kRedo: lookups
  constexpr int64_t kRedo = -2;
  // metadata checks and data pointers of client i (its vals filled)
  const auto check_client = [&](int64_t i) {
    PyObject* const* row = &vals[static_cast<size_t>(i) * N];
    // two prefetch stages: the TensorImpl kImpl keys ahead, then -- once it
    // has arrived -- the StorageImpl behind data_ptr() kStore keys ahead (the
    // third dependent miss of every tensor; 35,000 of them in a resnet56 x 100
    // round)
    constexpr Py_ssize_t kImpl = 16, kStore = 8;
    const auto impl_of = [&](Py_ssize_t j) -> c10::TensorImpl* {
      return THPVariable_CheckExact(row[j]) ? THPVariable_Unpack(row[j]).unsafeGetTensorImpl() : nullptr;
    };
    const auto prefetch_storage = [&](Py_ssize_t j) {
      if (c10::TensorImpl* ti = impl_of(j))
        if (ti->has_storage()) __builtin_prefetch(ti->unsafe_storage().unsafeGetStorageImpl());
    };
    for (Py_ssize_t j = 0; j < N && j < kImpl; ++j)
      if (c10::TensorImpl* ti = impl_of(j)) __builtin_prefetch(ti);
    for (Py_ssize_t j = 0; j < N && j < kStore; ++j) prefetch_storage(j);
    for (Py_ssize_t j = 0; j < N; ++j) {
      if (j + kImpl < N)
        if (c10::TensorImpl* ti = impl_of(j + kImpl)) __builtin_prefetch(ti);
      if (j + kStore < N) prefetch_storage(j + kStore);
      PyObject* t = row[j];
      // exact Tensor / Parameter only (no isinstance walk off the GIL
      // thread): a Tensor subclass goes to the general Python path
      bool ok = THPVariable_CheckExact(t);
      if (ok) {
        const at::Tensor& ten = THPVariable_Unpack(t);
        const bool where = device_index < 0 ? ten.is_cpu() : (ten.is_cuda() && ten.get_device() == device_index);
        ok = ten.scalar_type() == dtypes[j] && ten.sizes() == c10::IntArrayRef(sizes[j]) && where &&
             ten.is_contiguous();
        if (ok) out[i * N + j] = reinterpret_cast<int64_t>(ten.data_ptr());
      }
      if (!ok) {
        bad[i] = j;
        return;
      }
    }
  };
  at::parallel_for(0, K, 1, [&](int64_t i0, int64_t i1) {
    for (int64_t i = i0; i < i1; ++i) {
      PyObject* d = dobj[i];
      bool fast = PyDict_Check(d) && PyDict_Size(d) == N;
      if (fast) {
        Py_ssize_t pos = 0, j = 0;
        PyObject *key, *val;
        Py_hash_t h;
        PyObject** row = &vals[static_cast<size_t>(i) * N];
        thread_local std::vector<PyObject*> keys;
        keys.resize(N);
        // the dict's entry table in order: hashes against the names' (a miss
        // ends the fast walk), key and value objects prefetched together ...
        while (_PyDict_Next(d, &pos, &key, &val, &h)) {
          if (j >= N || (key != name_ptr[j] && h != name_hash[j])) {
            fast = false;
            break;
          }
          keys[j] = key;
          row[j++] = val;
          __builtin_prefetch(key);
          __builtin_prefetch(val);
        }
        fast = fast && j == N;
        // ... then the exact compare of every key (client i's own strings,
        // already on their way into the cache)
        for (Py_ssize_t jj = 0; fast && jj < N; ++jj)
          fast = key_eq(keys[jj], name_ptr[jj]) == KeyEq::kSame;
      }
      if (!fast) {
        bad[i] = kRedo;
        continue;
      }
      check_client(i);
    }
  });
  // strict0: client 0 must be a dict holding exactly `names`, in order (a
  // table reused from an earlier round; anything else takes a fresh table)
  if (strict0 && K > 0 && bad[0] == kRedo) return py::make_tuple(py::none(), 0, -1);
  for (Py_ssize_t i = 0; i < K; ++i) {  // other mappings / key objects: lookups on this thread
    if (bad[i] != kRedo) continue;
    bad[i] = -1;
    PyObject** row = &vals[static_cast<size_t>(i) * N];
    for (Py_ssize_t j = 0; j < N; ++j) {
      PyObject* t = PyObject_GetItem(dobj[i], name_ptr[j]);  // new reference
      if (!t) {
        PyErr_Clear();
        release();
        return py::make_tuple(py::none(), i, j);
      }
      owned.push_back(t);
      row[j] = t;
    }
    check_client(i);
  }
  release();  // the dicts keep their tensors alive
  for (Py_ssize_t i = 0; i < K; ++i)
    if (bad[i] >= 0) return py::make_tuple(py::none(), i, bad[i]);
  return py::make_tuple(ptrs, -1, -1);
}

// unpack(flat, offsets, shapes) -> [views]: view j is flat[offsets[j] :
// offsets[j] + numel(shapes[j])] shaped shapes[j] -- the averaged model's keys
// as views of the one host buffer the reduction wrote (the Python loop costs
// ~3.6 us per key: 1.3 ms for resnet56's 350 keys every round).
// the key views of flat (unpack's) for every (offset, shape); view j is
// handed to put(j, object) -- a list slot or a dict item
template <typename Put>
static void make_views(const at::Tensor& flat, py::list offsets, py::list shapes, Put put) {
  const Py_ssize_t N = PyList_GET_SIZE(offsets.ptr());
  if (PyList_GET_SIZE(shapes.ptr()) != N) throw std::invalid_argument("offsets/shapes length mismatch");
  if (flat.dim() != 1 || !flat.is_contiguous()) throw std::invalid_argument("flat must be a contiguous 1-D tensor");
  if (flat.requires_grad()) throw std::invalid_argument("unpack: flat must not require grad");
  std::vector<int64_t> size, stride;
  for (Py_ssize_t j = 0; j < N; ++j) {
    const int64_t off = PyLong_AsLongLong(PyList_GET_ITEM(offsets.ptr(), j));
    PyObject* shp = PyList_GET_ITEM(shapes.ptr(), j);
    const Py_ssize_t nd = PyTuple_GET_SIZE(shp);
    size.resize(nd);
    stride.resize(nd);
    int64_t numel = 1;
    for (Py_ssize_t d = nd - 1; d >= 0; --d) {
      size[d] = PyLong_AsLongLong(PyTuple_GET_ITEM(shp, d));
      stride[d] = numel;
      numel *= size[d];
    }
    if (off < 0 || off + numel > flat.numel()) throw std::out_of_range("unpack: key range outside the buffer");
    // a tensor on flat's storage with this key's sizes and offset, made
    // directly (as_strided's dispatch costs ~1.4 us a key: 0.5 ms for
    // resnet56's 350 keys, every round)
    auto impl = c10::make_intrusive<c10::TensorImpl>(c10::TensorImpl::VIEW, c10::Storage(flat.storage()),
                                                     flat.key_set(), flat.dtype());
    impl->set_sizes_and_strides(size, stride, std::make_optional<int64_t>(flat.storage_offset() + off));
    put(j, py::reinterpret_steal<py::object>(THPVariable_Wrap(at::Tensor(std::move(impl)))));
  }
}

static py::list unpack(const at::Tensor& flat, py::list offsets, py::list shapes) {
  py::list out(PyList_GET_SIZE(offsets.ptr()));
  make_views(flat, offsets, shapes, [&](Py_ssize_t j, py::object v) { out[j] = std::move(v); });
  return out;
}

// unpack_into(target, flat, names, offsets, shapes): target[names[j]] = view j
// (fedavg_trainer.py:455 assigns the averages into client 0's dict; existing
// keys keep their place) without an intermediate dict
static void unpack_into(py::object target, const at::Tensor& flat, py::list names, py::list offsets, py::list shapes) {
  if (PyList_GET_SIZE(names.ptr()) != PyList_GET_SIZE(offsets.ptr()))
    throw std::invalid_argument("names/offsets length mismatch");
  make_views(flat, offsets, shapes, [&](Py_ssize_t j, py::object v) {
    if (PyObject_SetItem(target.ptr(), PyList_GET_ITEM(names.ptr(), j), v.ptr()) != 0) throw py::error_already_set();
  });
}

// small_round(w_locals, names, templ, numel, offset, kind, shapes, P, ld, rows_host, rows_dev, w_host, w_dev,
//             round_fn, n_threads, stream, out_device) -> (status, out_dev, out_host)
//
// The whole host side of a small fp32 round in one call -- what aggregate()
// does in Python for a round whose key table is already known: the
// reference's weights n_i / N (fedavg_trainer.py:444-447, :453) from Python
// ints, the walk over every client's tensors (checked against the table like
// collect()), the pack-item list, ONE call of fedavg_round_f32 (pack + one
// kernel + wait; its address comes from the loaded libfedavg_amd.so) with
// the GIL released, and the averaged model's views written into
// w_locals[0][1] in key order (fedavg_trainer.py:449-457: the result IS
// client 0's dict).  status 0: done.  status 1: something the general path
// must see (a non-int or negative count, a zero total, a missing key or
// another shape/dtype/device, client 0 without exactly the table's keys in
// order, a repeated dict) -- nothing was written and the caller runs the
// general path, which raises the reference's exception or handles the case.
// A failing native call returns its negative code as status.
using round_fn_t = int (*)(const int64_t*, int64_t, float*, float*, int64_t, int64_t, int64_t, const double*, float*,
                           float*, float*, float*, int, void*);

static py::tuple small_round(py::list w_locals, py::list names, py::list templ, const std::vector<int64_t>& numel,
                             const std::vector<int64_t>& offset, const std::vector<int64_t>& kind, py::list shapes,
                             int64_t P, int64_t ld, int64_t rows_host, int64_t rows_dev, int64_t w_host,
                             int64_t w_dev, int64_t round_fn, int n_threads, int64_t stream, int64_t out_device) {
  const Py_ssize_t K = PyList_GET_SIZE(w_locals.ptr());
  const Py_ssize_t N = PyList_GET_SIZE(names.ptr());
  auto fallback = [] { return py::make_tuple(1, py::none(), py::none()); };
  if (K <= 0 || N <= 0 || static_cast<Py_ssize_t>(numel.size()) != N) return fallback();
  thread_local std::vector<double> weights;
  thread_local std::vector<PyObject*> dicts;
  thread_local std::vector<int64_t> items;
  weights.resize(K);
  dicts.resize(K);
  // counts and dicts (:444-447): exact ints only, summed in order
  int64_t total = 0;
  for (Py_ssize_t i = 0; i < K; ++i) {
    PyObject* pair = PyList_GET_ITEM(w_locals.ptr(), i);
    if (!PyTuple_Check(pair) || PyTuple_GET_SIZE(pair) != 2) return fallback();
    PyObject* n = PyTuple_GET_ITEM(pair, 0);
    if (!PyLong_CheckExact(n)) return fallback();
    int overflow = 0;
    const long long v = PyLong_AsLongLongAndOverflow(n, &overflow);
    if (overflow || v < 0 || v > (1LL << 53)) return fallback();
    total += v;
    if (total > (1LL << 53)) return fallback();
    weights[i] = static_cast<double>(v);
    dicts[i] = PyTuple_GET_ITEM(pair, 1);
    for (Py_ssize_t j = 0; j < i; ++j)
      if (dicts[j] == dicts[i]) return fallback();  // the general path raises (aliased rows)
  }
  if (total == 0) return fallback();  // ZeroDivisionError, raised by the general path
  for (Py_ssize_t i = 0; i < K; ++i) weights[i] = weights[i] / static_cast<double>(total);  // == Python n / N
  // client 0 must hold exactly the table's keys in order (the result replaces them in place)
  PyObject* d0 = dicts[0];
  if (!PyDict_Check(d0) || PyDict_Size(d0) != N) return fallback();
  {
    Py_ssize_t pos = 0, j = 0;
    PyObject *key, *val;
    while (PyDict_Next(d0, &pos, &key, &val)) {
      if (j >= N) return fallback();
      const int eq = PyObject_RichCompareBool(key, PyList_GET_ITEM(names.ptr(), j), Py_EQ);
      if (eq != 1) {
        if (eq < 0) PyErr_Clear();
        return fallback();
      }
      ++j;
    }
  }
  // the walk: every client's tensor for every key, checked against the table
  items.resize(static_cast<size_t>(K) * N * 4);
  for (Py_ssize_t i = 0; i < K; ++i) {
    PyObject* d = dicts[i];
    for (Py_ssize_t j = 0; j < N; ++j) {
      PyObject* t = PyObject_GetItem(d, PyList_GET_ITEM(names.ptr(), j));
      if (!t) {
        PyErr_Clear();
        return fallback();
      }
      bool ok = THPVariable_Check(t);
      if (ok) {
        const at::Tensor& ten = THPVariable_Unpack(t);
        const at::Tensor& tp = THPVariable_Unpack(PyList_GET_ITEM(templ.ptr(), j));
        // host clients only (client.py:96 returns net.cpu().state_dict()): the
        // packer reads them with the CPU
        ok = ten.scalar_type() == tp.scalar_type() && ten.sizes() == tp.sizes() && ten.is_contiguous() &&
             ten.is_cpu();
        if (ok) {
          int64_t* it = &items[(static_cast<size_t>(i) * N + j) * 4];
          it[0] = reinterpret_cast<int64_t>(ten.data_ptr());
          it[1] = numel[j];
          it[2] = static_cast<int64_t>(i) * ld + offset[j];
          it[3] = kind[j];
        }
      }
      Py_DECREF(t);  // the dict keeps the tensor alive
      if (!ok) return fallback();
    }
  }
  auto opts = at::TensorOptions().dtype(at::kFloat);
  at::Tensor out_host = at::empty({P}, opts.pinned_memory(true));
  at::Tensor out_dev = at::empty({P}, opts.device(at::Device(at::kCUDA, static_cast<c10::DeviceIndex>(out_device))));
  int rc;
  {
    py::gil_scoped_release nogil;
    rc = reinterpret_cast<round_fn_t>(round_fn)(items.data(), static_cast<int64_t>(K) * N,
                                                reinterpret_cast<float*>(rows_host), reinterpret_cast<float*>(rows_dev),
                                                K, P, ld, weights.data(), reinterpret_cast<float*>(w_host),
                                                reinterpret_cast<float*>(w_dev), out_dev.data_ptr<float>(),
                                                out_host.data_ptr<float>(), n_threads, reinterpret_cast<void*>(stream));
  }
  if (rc != 0) return py::make_tuple(rc, py::none(), py::none());
  // the averaged model's keys as views of out_host, written into client 0's dict
  std::vector<int64_t> size, stride;
  for (Py_ssize_t j = 0; j < N; ++j) {
    PyObject* shp = PyList_GET_ITEM(shapes.ptr(), j);
    const Py_ssize_t nd = PyTuple_GET_SIZE(shp);
    size.resize(nd);
    stride.resize(nd);
    int64_t n = 1;
    for (Py_ssize_t dd = nd - 1; dd >= 0; --dd) {
      size[dd] = PyLong_AsLongLong(PyTuple_GET_ITEM(shp, dd));
      stride[dd] = n;
      n *= size[dd];
    }
    py::object view = py::reinterpret_steal<py::object>(THPVariable_Wrap(out_host.as_strided(size, stride, offset[j])));
    if (PyObject_SetItem(d0, PyList_GET_ITEM(names.ptr(), j), view.ptr()) != 0) throw py::error_already_set();
  }
  return py::make_tuple(0, out_dev, out_host);
}

// verify_rows(w_locals, counts, names, templ, group, offset, kind, stage_ptr, stage_ld, stage_esize,
//             probes, seed, full_elems) -> (status, client, key, elements_checked)
//
// Does w_locals (the reference's :199 deep copies) hold what a streamed
// round's staging rows were packed from?  autostream.py fed each client's
// Client.train result to the packer while the loop went on; at :217 this
// walk checks
//   * len(w_locals) == len(counts) and every w_locals[i] is a (n, dict) pair
//     whose n == counts[i] (Python ==) and whose dict is not another
//     client's dict object;
//   * every client's dict holds exactly the table's keys in order (exact
//     string compares, key_eq; == on this thread for other key objects);
//   * at EVERY (client, key) pair, the value is an exact Tensor, contiguous,
//     on the host, with the template's dtype and sizes, and -- with
//     expect_version >= 0 -- its version counter is expect_version: the value
//     a fresh copy.deepcopy(tensor) carries (autostream measures it on the
//     running torch).  The reference's :199 deep copies are made after the
//     client's train() returned, so any in-place op on a w_locals tensor
//     between :199 and :217 (add_, clamp_, mul_, copy_, an optimizer step,
//     a slice assignment) moves that counter: such edits are caught every
//     round, deterministically, whatever positions they touch;
//   * element values at `probes` (client, key, position) triples drawn
//     afresh from `seed` every round -- every key at least once (at a random
//     client), the rest spread uniformly over all (client, key) pairs,
//     positions uniform inside the key -- against the pinned staging rows
//     the H2D copies uploaded (every element when the round has at most
//     `full_elems` of them), converted as the packer converts
//     (fp32/fp64/fp16/bf16 keys raw, integer/bool keys static_cast to fp32:
//     fedavg_host.cpp).  Equal converted values reduce to the same bits, so
//     a match is exactly the reduction's criterion at that element.
// The per-client walks run on torch's intra-op threads (see below).
//   * with `copies` (optional, one entry per client): where copies[i] is a
//     tuple, every value of client i IS (object identity) the tensor at that
//     position of the dict the loop's :199 copy.deepcopy returned for fed
//     client i (autostream records it in a one-shot __deepcopy__ hook).  A
//     tensor replaced between :199 and :217 -- by a fresh tensor or by
//     another deep copy, whose version counter is a deep copy's too -- is
//     caught deterministically; None entries skip the check.
// status 0: all checks passed; 1 count; 2 sample number; 3 not a (n, dict)
// pair; 4 repeated dict; 5 keys; 6 tensor metadata; 7 value (client, key);
// 8 version counter (client, key); 10 not the :199 deep copy's tensor
// (client, key).
namespace {
inline uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

struct Probe {
  const char* src;
  const char* dst;
  int kind;
  int esize;
  int i, j;
};

bool probe_equal(const Probe& p) {
  if (p.kind == 0) return std::memcmp(p.src, p.dst, static_cast<size_t>(p.esize)) == 0;
  float v;
  switch (p.kind) {  // fedavg_pack_item kinds (include/fedavg_amd.h), as fedavg_host.cpp converts
    case 1: { int64_t s; std::memcpy(&s, p.src, 8); v = static_cast<float>(s); break; }
    case 2: { int32_t s; std::memcpy(&s, p.src, 4); v = static_cast<float>(s); break; }
    case 3: { int16_t s; std::memcpy(&s, p.src, 2); v = static_cast<float>(s); break; }
    case 4: v = static_cast<float>(*reinterpret_cast<const int8_t*>(p.src)); break;
    case 5: v = static_cast<float>(*reinterpret_cast<const uint8_t*>(p.src)); break;
    case 6: v = *reinterpret_cast<const uint8_t*>(p.src) ? 1.0f : 0.0f; break;
    default: return false;
  }
  return std::memcmp(&v, p.dst, 4) == 0;
}
}  // namespace

static py::tuple verify_rows(py::list w_locals, py::list counts, py::list names, py::list templ,
                             const std::vector<int64_t>& group, const std::vector<int64_t>& offset,
                             const std::vector<int64_t>& kind, const std::vector<int64_t>& stage_ptr,
                             const std::vector<int64_t>& stage_ld, const std::vector<int64_t>& stage_esize,
                             int64_t probes, uint64_t seed, int64_t full_elems, int64_t expect_version,
                             py::object fed_keys, py::object copies) {
  const Py_ssize_t K = PyList_GET_SIZE(w_locals.ptr());
  const Py_ssize_t N = PyList_GET_SIZE(names.ptr());
  // (status, client, key, elements compared, (us before the walk, us in the
  // threaded walk, us after it, intra-op threads)) -- the timings for probes
  using clk = std::chrono::steady_clock;
  const auto t_entry = clk::now();
  auto t_walk0 = t_entry, t_walk1 = t_entry;
  const auto us = [](clk::time_point a, clk::time_point b) {
    return std::chrono::duration<double, std::micro>(b - a).count();
  };
  // walk_detail: summed us in the dict walks and in the tensor checks, the
  // slowest thread's us, the parallel chunks
  std::array<double, 4> walk_detail{0, 0, 0, 0};
  auto res = [&](int status, Py_ssize_t i, Py_ssize_t j, int64_t n) {
    const auto t_end = clk::now();
    return py::make_tuple(status, i, j, n,
                          py::make_tuple(us(t_entry, t_walk0), us(t_walk0, t_walk1), us(t_walk1, t_end),
                                         at::get_num_threads(), walk_detail[0], walk_detail[1], walk_detail[2],
                                         walk_detail[3]));
  };
  if (K != PyList_GET_SIZE(counts.ptr()) || K == 0) return res(1, -1, -1, 0);
  if (PyList_GET_SIZE(templ.ptr()) != N || static_cast<Py_ssize_t>(group.size()) != N ||
      static_cast<Py_ssize_t>(offset.size()) != N || static_cast<Py_ssize_t>(kind.size()) != N)
    throw std::invalid_argument("verify_rows: table arrays differ in length");
  std::vector<const at::Tensor*> tp(N);
  std::vector<int64_t> numel(N);
  for (Py_ssize_t j = 0; j < N; ++j) {
    PyObject* t = PyList_GET_ITEM(templ.ptr(), j);
    if (!THPVariable_Check(t)) throw std::invalid_argument("template entries must be tensors");
    tp[j] = &THPVariable_Unpack(t);
    numel[j] = tp[j]->numel();
    const int64_t g = group[j];
    if (g < 0 || g >= static_cast<int64_t>(stage_ptr.size())) throw std::invalid_argument("verify_rows: bad group");
  }
  // a round of at most full_elems elements (K x the table's elements) is
  // compared in full, every element of every client; larger ones by probes
  int64_t row_elems = 0;
  for (Py_ssize_t j = 0; j < N; ++j) row_elems += numel[j];
  const bool full = static_cast<int64_t>(K) * row_elems <= full_elems;
  // probe density: ~`probes` pairs over K x N, plus one anchor client per key
  const double frac = static_cast<double>(probes) / (static_cast<double>(K) * static_cast<double>(N));
  const uint64_t thresh = frac >= 1.0 ? ~0ull : static_cast<uint64_t>(frac * 18446744073709551615.0);
  std::vector<PyObject*> dicts(K);
  for (Py_ssize_t i = 0; i < K; ++i) {
    PyObject* pair = PyList_GET_ITEM(w_locals.ptr(), i);
    if (!PyTuple_Check(pair) || PyTuple_GET_SIZE(pair) != 2) return res(3, i, -1, 0);
    const int eq = PyObject_RichCompareBool(PyTuple_GET_ITEM(pair, 0), PyList_GET_ITEM(counts.ptr(), i), Py_EQ);
    if (eq != 1) {
      if (eq < 0) PyErr_Clear();
      return res(2, i, -1, 0);
    }
    PyObject* d = PyTuple_GET_ITEM(pair, 1);
    if (!PyDict_Check(d) || PyDict_Size(d) != N) return res(PyDict_Check(d) ? 5 : 3, i, -1, 0);
    dicts[i] = d;
  }
  {
    std::vector<PyObject*> sorted(dicts);
    std::sort(sorted.begin(), sorted.end());
    for (size_t a = 1; a < sorted.size(); ++a)
      if (sorted[a] == sorted[a - 1]) return res(4, -1, -1, 0);  // the plain path handles aliased clients
  }
  // One walk per client, clients split over torch's intra-op threads.  The
  // calling thread keeps the GIL throughout, so no Python code runs and no
  // object changes meanwhile; the threads read dict entry tables
  // (PyDict_Next: no reference counts touched) and tensor metadata, and call
  // nothing else of the Python API.  The walk is bound by cache misses on
  // scattered objects (resnet56 x 100: 35,000 tensors, ~150 ns each on one
  // thread), hence the threads and the prefetches a few keys ahead.
  // A dict whose keys are not the table's names as exact strings (key_eq)
  // is redone afterwards on this thread with == compares.
  std::vector<PyObject*> name_ptr(N);
  std::vector<Py_hash_t> name_hash(N);
  for (Py_ssize_t j = 0; j < N; ++j) {
    name_ptr[j] = PyList_GET_ITEM(names.ptr(), j);
    name_hash[j] = PyObject_Hash(name_ptr[j]);
    if (name_hash[j] == -1) {
      PyErr_Clear();
      return res(5, -1, j, 0);
    }
  }
  std::vector<PyObject*> vals(static_cast<size_t>(K) * N);
  std::vector<int64_t> status(static_cast<size_t>(K), 0);  // per client: 0, or (code << 32 | key)
  std::vector<int64_t> nprobe(static_cast<size_t>(K), 0);
  constexpr int64_t kRedo = -1;  // keys not identical: == compares on the GIL thread
  // The dict's entry table in order (_PyDict_Next): hashes against the
  // names' (a miss ends the fast walk), then every key compared exactly
  // (key_eq: each net.cpu().state_dict() builds its own name strings, so
  // the key objects are read -- prefetched with the values).  A dict whose
  // keys are not exact str objects equal to the names in order is redone on
  // this thread with ==.
  // fed_keys[i] (optional): the key objects of the dict fed as client i,
  // already matched exactly to the names when it was packed (collect).  The
  // loop's :199 copy.deepcopy keeps str keys as the same objects, so a key
  // identical to the fed one is the name without reading the string.
  std::vector<PyObject* const*> fk(static_cast<size_t>(K), nullptr);
  if (!fed_keys.is_none()) {
    if (!PyList_Check(fed_keys.ptr()) || PyList_GET_SIZE(fed_keys.ptr()) != K)
      throw std::invalid_argument("verify_rows: fed_keys must be a list with one key sequence per client");
    for (Py_ssize_t i = 0; i < K; ++i) {
      PyObject* ks = PyList_GET_ITEM(fed_keys.ptr(), i);
      if (PyTuple_Check(ks) && PyTuple_GET_SIZE(ks) == N) fk[i] = &PyTuple_GET_ITEM(ks, 0);
    }
  }
  std::vector<PyObject* const*> ck(static_cast<size_t>(K), nullptr);
  if (!copies.is_none()) {
    if (!PyList_Check(copies.ptr()) || PyList_GET_SIZE(copies.ptr()) != K)
      throw std::invalid_argument("verify_rows: copies must be a list with one entry per client");
    for (Py_ssize_t i = 0; i < K; ++i) {
      PyObject* cs = PyList_GET_ITEM(copies.ptr(), i);
      if (cs == Py_None) continue;
      if (!PyTuple_Check(cs) || PyTuple_GET_SIZE(cs) != N) return res(10, i, -1, 0);  // the copy had other keys
      ck[i] = &PyTuple_GET_ITEM(cs, 0);
    }
  }
  const auto fill_fast = [&](int64_t i) -> bool {
    Py_ssize_t pos = 0, j = 0;
    PyObject *key, *val;
    Py_hash_t h;
    PyObject** row = &vals[static_cast<size_t>(i) * N];
    PyObject* const* fed = fk[i];
    thread_local std::vector<PyObject*> keys;
    keys.resize(N);
    while (_PyDict_Next(dicts[i], &pos, &key, &val, &h)) {
      if (j >= N || (key != name_ptr[j] && h != name_hash[j])) return false;
      const bool known = key == name_ptr[j] || (fed && key == fed[j]);
      keys[j] = known ? nullptr : key;
      row[j++] = val;
      if (!known) __builtin_prefetch(key);
      __builtin_prefetch(val);
    }
    if (j != N) return false;
    for (Py_ssize_t jj = 0; jj < N; ++jj)
      if (keys[jj] && key_eq(keys[jj], name_ptr[jj]) != KeyEq::kSame) return false;
    return true;
  };
  // the VersionCounter object behind a tensor's _version (one more dependent
  // miss per tensor): VariableVersion is exactly one intrusive_ptr
  static_assert(sizeof(c10::VariableVersion) == sizeof(void*), "VariableVersion layout");
  const auto version_obj = [](c10::TensorImpl* ti) -> const void* {
    return *reinterpret_cast<void* const*>(&ti->version_counter());
  };
  // metadata checks and value probes of client i (its vals filled)
  const auto check_client = [&](int64_t i, std::vector<Probe>& todo) {
    todo.clear();
    int64_t st = 0;
    PyObject* const* row_vals = &vals[static_cast<size_t>(i) * N];
    // every (client, key) pair: the value's tensor checked (exact Tensor,
    // dtype, sizes, host, contiguous, version counter); the pairs probed this
    // round also have elements compared -- every key is probed at one client
    // or more each round (its anchor), so an edit of a key across clients is
    // always seen by value too.  The objects are cold (made seconds ago, by
    // the loop's :199 deep copies), so the walk goes in passes, each one a
    // run of independent loads the core overlaps instead of a chain of
    // dependent misses per tensor: the TensorImpls (their PyObjects were
    // prefetched by the dict walk), then every tensor's metadata with its
    // VersionCounter (and a probed pair's StorageImpl) prefetched, then the
    // versions and the value probes.
    const auto probed = [&](Py_ssize_t j, uint64_t* hp) {
      const uint64_t h = mix64(seed ^ mix64(static_cast<uint64_t>(i) * 0x100000001B3ull + static_cast<uint64_t>(j)));
      *hp = h;
      return full || h <= thresh ||
             static_cast<int64_t>(mix64(seed + static_cast<uint64_t>(j)) % static_cast<uint64_t>(K)) == i;
    };
    if (PyObject* const* cp = ck[i]) {  // the values the loop's :199 deep copy made (pointer compares)
      for (Py_ssize_t j = 0; j < N; ++j)
        if (row_vals[j] != cp[j]) {
          status[i] = (int64_t(10) << 32) | j;
          return;
        }
    }
    thread_local std::vector<c10::TensorImpl*> impls;
    impls.resize(N);
    for (Py_ssize_t j = 0; j < N; ++j) {
      c10::TensorImpl* ti =
          THPVariable_CheckExact(row_vals[j]) ? THPVariable_Unpack(row_vals[j]).unsafeGetTensorImpl() : nullptr;
      impls[j] = ti;
      if (ti) {  // the fields read below span the TensorImpl's first lines
        __builtin_prefetch(ti);
        __builtin_prefetch(reinterpret_cast<const char*>(ti) + 64);
        __builtin_prefetch(reinterpret_cast<const char*>(ti) + 128);
      }
    }
    for (Py_ssize_t j = 0; j < N && !st; ++j) {
      c10::TensorImpl* ti = impls[j];
      if (!ti) {  // a Tensor subclass: the plain path decides
        st = (int64_t(6) << 32) | j;
        break;
      }
      if (ti->dtype() != tp[j]->dtype() || ti->sizes() != tp[j]->sizes() || !ti->is_cpu() || !ti->is_contiguous()) {
        st = (int64_t(6) << 32) | j;
        break;
      }
      if (expect_version >= 0)
        if (const void* v = version_obj(ti)) __builtin_prefetch(v);
      uint64_t h;
      if (probed(j, &h) && ti->has_storage()) __builtin_prefetch(ti->unsafe_storage().unsafeGetStorageImpl());
    }
    for (Py_ssize_t j = 0; j < N && !st; ++j) {
      if (expect_version >= 0) {
        const c10::VariableVersion& vc = impls[j]->version_counter();
        if (!vc.enabled() || static_cast<int64_t>(vc.current_version()) != expect_version) {
          st = (int64_t(8) << 32) | j;
          break;
        }
      }
      const at::Tensor& ten = THPVariable_Unpack(row_vals[j]);
      uint64_t h;
      if (!probed(j, &h)) continue;
      const int64_t n = numel[j];
      if (n <= 0) continue;
      const int64_t g = group[j];
      const int es = static_cast<int>(stage_esize[g]);
      const int src_es = static_cast<int>(ten.element_size());
      const char* src = static_cast<const char*>(ten.data_ptr());
      const char* srow = reinterpret_cast<const char*>(stage_ptr[g]) + (i * stage_ld[g] + offset[j]) * es;
      if (full) {
        bool same = true;
        if (kind[j] == 0) {
          same = std::memcmp(src, srow, static_cast<size_t>(n) * es) == 0;
        } else {
          for (int64_t p = 0; p < n && same; ++p)
            same = probe_equal(Probe{src + p * src_es, srow + p * es, static_cast<int>(kind[j]), es, 0, 0});
        }
        if (!same) st = (int64_t(7) << 32) | j;
        nprobe[i] += n;
        continue;
      }
      for (int q = 0; q < 2; ++q) {  // two positions per probed pair
        const int64_t p = static_cast<int64_t>(mix64(h + 1 + q) % static_cast<uint64_t>(n));
        todo.push_back(Probe{src + p * src_es, srow + p * es, static_cast<int>(kind[j]), es, static_cast<int>(i),
                             static_cast<int>(j)});
      }
    }
    if (!st)
      for (const Probe& p : todo)
        if (!probe_equal(p)) {
          st = (int64_t(7) << 32) | p.j;
          break;
        }
    status[i] = st;
    nprobe[i] += static_cast<int64_t>(todo.size());
  };
  t_walk0 = clk::now();
  std::atomic<int64_t> fill_ns{0}, check_ns{0}, max_ns{0}, nchunks{0};
  at::parallel_for(0, K, 1, [&](int64_t i0, int64_t i1) {
    std::vector<Probe> todo;
    const auto c0 = clk::now();
    int64_t f = 0, c = 0;
    for (int64_t i = i0; i < i1; ++i) {
      const auto a = clk::now();
      const bool ok = fill_fast(i);
      const auto b = clk::now();
      f += std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
      if (!ok) {
        status[i] = kRedo;
        continue;
      }
      check_client(i, todo);
      c += std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - b).count();
    }
    const int64_t span = std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - c0).count();
    fill_ns += f;
    check_ns += c;
    nchunks += 1;
    int64_t m = max_ns.load();
    while (span > m && !max_ns.compare_exchange_weak(m, span)) {
    }
  });
  t_walk1 = clk::now();
  walk_detail = {fill_ns.load() / 1e3, check_ns.load() / 1e3, max_ns.load() / 1e3, static_cast<double>(nchunks.load())};
  {  // dicts whose keys are equal but not identical to the names: == on this thread
    std::vector<Probe> todo;
    for (Py_ssize_t i = 0; i < K; ++i) {
      if (status[i] != kRedo) continue;
      Py_ssize_t pos = 0, j = 0;
      PyObject *key, *val;
      status[i] = 0;
      while (PyDict_Next(dicts[i], &pos, &key, &val)) {
        if (j >= N) break;
        const int eq = key == name_ptr[j] ? 1 : PyObject_RichCompareBool(key, name_ptr[j], Py_EQ);
        if (eq != 1) {
          if (eq < 0) PyErr_Clear();
          break;
        }
        vals[static_cast<size_t>(i) * N + j++] = val;
      }
      if (j != N) {
        status[i] = (int64_t(5) << 32) | j;
        continue;
      }
      check_client(i, todo);
    }
  }
  int64_t total = 0;
  for (Py_ssize_t i = 0; i < K; ++i) {
    total += nprobe[i];
    if (status[i]) return res(static_cast<int>(status[i] >> 32), i, static_cast<Py_ssize_t>(status[i] & 0xffffffff), total);
  }
  return res(0, -1, -1, total);
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "native state_dict walk for mfl_amd (host metadata only)";
  m.def("collect", &collect, "validate clients against client 0 and gather data pointers", py::arg("dicts"),
        py::arg("names"), py::arg("templ"), py::arg("device_index") = -1, py::arg("strict0") = false);
  m.def("unpack", &unpack, "views of a flat buffer shaped like the key table's keys");
  m.def("unpack_into", &unpack_into, "those views assigned into a dict by key name");
  m.def("small_round", &small_round, "the host side of a small fp32 round in one call");
  m.def("verify_rows", &verify_rows,
        "w_locals against a streamed round's staging rows (every tensor's metadata and version counter, "
        "randomly sampled values)",
        py::arg("w_locals"), py::arg("counts"), py::arg("names"), py::arg("templ"), py::arg("group"),
        py::arg("offset"), py::arg("kind"), py::arg("stage_ptr"), py::arg("stage_ld"), py::arg("stage_esize"),
        py::arg("probes"), py::arg("seed"), py::arg("full_elems"), py::arg("expect_version") = -1,
        py::arg("fed_keys") = py::none(), py::arg("copies") = py::none());
}
