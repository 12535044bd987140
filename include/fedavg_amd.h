/*
 * fedavg_amd.h -- C ABI of the MI355X (gfx950) FedAvg weighted reduction.
 *
 * Replaces the inner loop of the reference's
 *     FedAvgTrainer.aggregate(self, w_locals)        src/fedavg_trainer.py:441-458
 * i.e. for every parameter element p:
 *     out[p] = (((x[0][p]*w[0]) + x[1][p]*w[1]) + ...) + x[K-1][p]*w[K-1]
 * computed in the reference's order (client 0 first, a multiply then an add
 * per client, never fused), so fp32 results are bit-identical to the
 * reference's torch CPU loop (fedavg_trainer.py:451-457).
 *
 * The reference has no FFI: its boundary is the Python method above.  These
 * entry points are what the Python drop-in (mobile-federated-learning_amd/)
 * binds through ctypes; INTEGRATION.md shows the binding.  The weight vector
 * w[i] = float(n_i / sum(n)) is formed on the host exactly as
 * fedavg_trainer.py:444-447,453 forms it (Python double, rounded to fp32 by
 * ATen), see fedavg_weights_f32() below.
 *
 * Conventions (all functions):
 *   - every buffer argument is DEVICE memory owned by the caller; nothing is
 *     allocated inside; calls are asynchronous and ordered on `stream`
 *     (a hipStream_t; NULL = the default stream), reentrant across streams;
 *   - return 0 on success, a negative FEDAVG_E* code for a rejected argument,
 *     or -(hipError_t) for a launch failure; fedavg_last_error() gives a
 *     thread-local message for the last failing call on this thread;
 *   - K == 0 is rejected (the reference returns the global model then,
 *     fedavg_trainer.py:442-443 -- the host layer handles that case);
 *     P == 0 is a no-op.
 */
#ifndef FEDAVG_AMD_H
#define FEDAVG_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FEDAVG_OK 0
#define FEDAVG_EINVAL (-10001)   /* bad size / stride / null pointer     */
#define FEDAVG_EALIGN (-10002)   /* misaligned buffer for this entry     */
#define FEDAVG_EMODE (-10003)    /* unknown mode / variant               */

/* ABI version: bumped on any signature change. */
int fedavg_abi_version(void);

/* Thread-local message for the last failing call on this thread ("" if none). */
const char* fedavg_last_error(void);

/*
 * fp32 sequential (bit-exact) reduce over a client-major packed buffer.
 *   clients : [K, ld] row-major fp32, row i = client i's flattened state_dict
 *             (fedavg_trainer.py:199 w_locals[i][1], keys concatenated in the
 *             order of w_locals[0][1].keys(), :450)
 *   weights : [K] fp32, weights[i] = fp32(n_i / N)                (:453)
 *   out     : [P] fp32
 *   ld      : row stride in elements, ld >= P.
 * Fast path: clients 16-B aligned and ld % 4 == 0 (float4 streaming); any
 * other alignment takes a scalar path with identical results.
 */
int fedavg_reduce_f32(const float* clients, int64_t K, int64_t P, int64_t ld,
                      const float* weights, float* out, void* stream);

/*
 * Same reduction over K separate device buffers (no packing):
 *   client_ptrs : DEVICE array [K] of device pointers, each to >= P floats.
 * Each pointer needs only fp32 (4-byte) alignment.  Runs the zero-copy
 * segments kernel (fedavg_segments.hip) on one key of P columns: units of
 * 4,096 columns, U4 client rows per batch, dword-aligned 16-B loads.
 */
int fedavg_reduce_ptrs_f32(const float* const* client_ptrs, int64_t K, int64_t P,
                           const float* weights, float* out, void* stream);

/*
 * fp64 keys keep fp64 (reference: `tensor_f64 * python_float` stays double,
 * the weight is not rounded to fp32).  weights : [K] double.
 */
int fedavg_reduce_f64(const double* clients, int64_t K, int64_t P, int64_t ld,
                      const double* weights, double* out, void* stream);

/*
 * fp16 / bf16 keys keep their dtype; each multiply and each add is computed
 * in fp32 and rounded to the storage type (ATen opmath), as the reference's
 * `acc += p * w` does for a half tensor.  Values are passed as raw 16-bit
 * patterns.  weights : [K] fp32.
 */
int fedavg_reduce_f16(const uint16_t* clients, int64_t K, int64_t P, int64_t ld,
                      const float* weights, uint16_t* out, void* stream);
int fedavg_reduce_bf16(const uint16_t* clients, int64_t K, int64_t P, int64_t ld,
                       const float* weights, uint16_t* out, void* stream);

/*
 * Tolerance-gated split-client variant (NOT bit-exact with the reference):
 * the client axis is cut into `splits` contiguous groups (1, 2, 4 or 8),
 * each group's partial sum is kept in registers, staged through LDS and the
 * groups are combined in a fixed order.  Deterministic run to run; matches
 * the reference within norm-wise relative 1e-6 on model-like data.  Useful
 * where P is too small to fill the GPU.  splits == 1 is the exact kernel.
 */
int fedavg_reduce_splitk_f32(const float* clients, int64_t K, int64_t P, int64_t ld,
                             const float* weights, float* out, int splits, void* stream);

/*
 * Post-aggregate client distances (fedavg_trainer.py:291, feeding delta at
 * :293): sumsq[i] = sum_p fl32(clients[i][p] - glob[p])^2, the difference
 * rounded to fp32 as the reference's `w[para] - w_glob[para]` does, squares
 * exact in fp64 and summed in fp64 in a fixed order (deterministic).  The
 * norm is fl32(sqrt(sumsq[i])).  glob : [P] fp32 (the reduce's output);
 * sumsq : [K] double; workspace : fedavg_client_sqdist_workspace(K, P)
 * doubles of device scratch.  Needs 16-B aligned clients/glob, ld % 4 == 0.
 */
int64_t fedavg_client_sqdist_workspace(int64_t K, int64_t P);
int fedavg_client_sqdist_f32(const float* clients, int64_t K, int64_t P, int64_t ld,
                             const float* glob, double* workspace, int64_t workspace_elems,
                             double* sumsq, void* stream);

/*
 * Aggregate and :291 in ONE pass over the client rows (fedavg_trainer.py:217
 * then :291 of the same round read the same K x P bytes twice):
 *   out   : fedavg_reduce_f32's result, the same bits;
 *   sumsq : fedavg_client_sqdist_f32(clients, ..., out, ...)'s sums, the
 *           same rounding rules (fp32 difference, fp64 squares and sum,
 *           fixed order; not necessarily the same summation tree).
 * Needs 16-B aligned rows and ld % 4 == 0 (FEDAVG_EALIGN otherwise, before
 * any work: fedavg_reduce_f32 alone takes unaligned rows).  K <= 1024 runs
 * a fused kernel: for 17-128 clients on long rows one wave per window of
 * 64 x VEC columns x all K rows in registers; from 369 clients (and at
 * 161-256 and 289-368 clients on long rows) a workgroup of ceil(K / 64)
 * waves per 64-column window, 64 rows per wave, the chain handed from wave
 * to wave in row order; otherwise tiles of K rows x 32-256
 * columns staged in LDS per workgroup (by LDS-DMA or through registers);
 * K > 1024 runs the two passes back to back (fedavg_fused_plan_of says
 * which).  workspace : fedavg_reduce_sqdist_workspace(K, P) doubles of
 * device scratch.  P == 0 writes sumsq = 0.
 */
int64_t fedavg_reduce_sqdist_workspace(int64_t K, int64_t P);
/* Which kernel fedavg_reduce_sqdist_f32 runs for K x P rows on the current
 * device: kind x 1000000 + S x 100 + slots.  kind 0: the two passes; 1:
 * LDS-DMA tiles of S columns; 2: register-staged tiles of S columns and
 * `slots` 16-B slots per thread; 3: wave-owned windows of KMAX = S rows and
 * VEC = slots columns per lane (17-128 clients on rows of >= 16 windows per
 * wave); 4: split-row windows of S = 64 rows per wave, at most `slots` waves
 * per workgroup (369-1024 clients; 161-256 and 289-368 on rows of >= 24
 * windows per workgroup). */
int64_t fedavg_fused_plan_of(int64_t K, int64_t P);
int fedavg_reduce_sqdist_f32(const float* clients, int64_t K, int64_t P, int64_t ld,
                             const float* weights, float* out, double* workspace,
                             int64_t workspace_elems, double* sumsq, void* stream);

/*
 * The same pass for fp64 / fp16 / bf16 keys (a state_dict group of that
 * dtype).  `w[para] - w_glob[para]` at :291 forms the difference in the
 * key's dtype -- fp64, or fp32 math rounded to fp16/bf16 (ATen opmath) --
 * and torch.cat widens it exactly, so sumsq[i] = sum_p d_i[p]^2 with d the
 * reference's rounded difference, squares and sum in fp64.  The caller adds
 * the groups' sums and rounds sqrt() to torch.cat's promoted dtype.
 * workspace : fedavg_client_sqdist_workspace_elems(K, P, elem_size) doubles
 * (elem_size 2, 4 or 8); rows 16-B aligned with ld a multiple of 16 B.
 */
int64_t fedavg_client_sqdist_workspace_elems(int64_t K, int64_t P, int64_t elem_size);
int fedavg_client_sqdist_f64(const double* clients, int64_t K, int64_t P, int64_t ld,
                             const double* glob, double* workspace, int64_t workspace_elems,
                             double* sumsq, void* stream);
int fedavg_client_sqdist_f16(const uint16_t* clients, int64_t K, int64_t P, int64_t ld,
                             const uint16_t* glob, double* workspace, int64_t workspace_elems,
                             double* sumsq, void* stream);
int fedavg_client_sqdist_bf16(const uint16_t* clients, int64_t K, int64_t P, int64_t ld,
                              const uint16_t* glob, double* workspace, int64_t workspace_elems,
                              double* sumsq, void* stream);

/*
 * FPF2 bookkeeping (fedavg_trainer.py:108-119 state, :209-210, :271-278,
 * :314-327), on device-resident state owned by the caller:
 *   diffs   : local_w_diffs, [n_rows, ld] fp32 (n_rows = client_num_in_total),
 *             zero-initialised; columns P..ld stay 0
 *   a_mat   : A_mat, [ld] fp32, initialised to ones
 *   g_mat   : G_mat, [n_rows] fp32, zeros; itr_row : row round_idx of
 *             local_itr_lst [comm_round, n_rows]; lru_itr : LRU_itr_lst or NULL
 * All updates are the reference's fp32 expressions, bit-identical, except
 * global_w_diff.mean() (:319) and the row norms (:272), which are summed in
 * fp64 in a fixed order and rounded once (within the reference's own fp32
 * rounding error).  Needs 16-B aligned diffs/rows/last_w/w_glob/a_mat and
 * ld % 4 == 0.
 *
 * set_rows (:210): diffs[row_idx[k]] = rows[k] - last_w for k < K (row_idx
 *   is DEVICE int64; out-of-range entries are skipped -- validate on the host).
 * end_round (:316-319): rows with keep_rows[r] == 0 (device uint8; 1 = in
 *   client_indexes) get diffs[r] -= (w_glob - last_w); A_mat EMA with the
 *   mean of (w_glob - last_w).  workspace: fedavg_fpf_workspace(P) doubles.
 * update_g (:321-327): if `record`, itr_row[selected] = local_itr and (when
 *   lru_itr != NULL) lru_itr = selected ? 0 : lru_itr + local_itr; then
 *   G_mat = G_mat * (1 - 1/g1) + itr_row / g1.
 * index (:272/:274, :276-278): fpf[r] = norm(diffs[r] * a_mat) / g_mat[r]
 *   (or lru_itr[r] / g_mat[r]), NaN/inf replaced by 0.  fpf is DEVICE fp32.
 */
int fedavg_fpf_set_rows_f32(float* diffs, int64_t n_rows, int64_t ld, const int64_t* row_idx,
                            int64_t K, const float* rows, int64_t ld_rows, const float* last_w,
                            int64_t P, void* stream);
int64_t fedavg_fpf_workspace(int64_t P);
int fedavg_fpf_end_round_f32(float* diffs, int64_t n_rows, int64_t ld, const uint8_t* keep_rows,
                             float* a_mat, const float* w_glob, const float* last_w, int64_t P,
                             float g2, double* workspace, int64_t workspace_elems, void* stream);
int fedavg_fpf_update_g(float* g_mat, float* itr_row, float* lru_itr, const uint8_t* selected,
                        int64_t n_rows, float local_itr, int record, float g1, void* stream);
int fedavg_fpf_index_f32(const float* diffs, int64_t n_rows, int64_t ld, int64_t P,
                         const float* a_mat, const float* g_mat, float* fpf, void* stream);
int fedavg_fpf_index_lru(const float* lru_itr, const float* g_mat, int64_t n_rows, float* fpf,
                         void* stream);

/*
 * FPF2 for models with fp64 / fp16 / bf16 keys (fedavg_trainer.py:210, :316-319,
 * :272 under torch.cat's promotion).  T = the promoted dtype of all keys.
 * The model is a DEVICE key table keys[n_keys][5] in state_dict order:
 *   numel, cat offset, dtype group (0..3), element offset in the group row,
 *   rounding of an fp32-stored integer key's difference (0 none, 2 fp16, 3 bf16:
 *   the integer difference cast to a 16-bit T)
 * and per-group row bases (fedavg_fpf_groups: row 0 of each group, row stride
 * in elements, kind 0 fp32 / 1 fp64 / 2 fp16 / 3 bf16; unused groups any kind
 * equal in cur and last).
 *
 * cat_diff (:210 / :316): out[r][c] = cat(cur_k - last)[c] for k < K, with
 *   r = row_idx[k] (DEVICE int64, out-of-range skipped) or k when row_idx is
 *   NULL; each key's difference is formed in the key's dtype; out is fp32
 *   (out_f64 = 0: fl32 of it, local_w_diffs) or fp64 (the T value itself).
 * end_round_promoted (:316-319): rows with keep_rows[r] == 0 get
 *   fl32(row - gdiff) computed in promote(fp32, T); A_mat EMA in T's arithmetic
 *   (t_kind 0 fp32 / 1 fp64 / 2 fp16 / 3 bf16; a_mat is fp64 [P] when t_kind
 *   is 1 or 4, else fp32) with the mean of gdiff (fp64 [P], T values) rounded
 *   to T.  t_kind 4: the first fp64 round, whose A_mat is still the
 *   reference's fp32 tensor: a_mat holds its values widened, and the
 *   A_mat * (1 - 1/G2) product is formed in fp32 as ATen does.
 * index_f64 (:272 once A_mat is fp64): fpf[r] = norm(diffs[r] * a_mat) /
 *   g_mat[r] in fp64, NaN/inf replaced by 0.  fpf is DEVICE fp64.
 */
typedef struct fedavg_fpf_groups {
  const void* base[4];
  int64_t ld[4];
  int32_t kind[4];
} fedavg_fpf_groups;
int fedavg_fpf_cat_diff(const int64_t* keys, int64_t n_keys, int64_t P, const fedavg_fpf_groups* cur,
                        int64_t K, const fedavg_fpf_groups* last, const int64_t* row_idx,
                        int64_t n_rows, void* out, int64_t ld_out, int out_f64, void* stream);
int fedavg_fpf_end_round_promoted(float* diffs, int64_t n_rows, int64_t ld, const uint8_t* keep_rows,
                                  void* a_mat, const double* gdiff, int64_t P, int t_kind, float g2,
                                  double* workspace, int64_t workspace_elems, void* stream);
int fedavg_fpf_index_f64(const float* diffs, int64_t n_rows, int64_t ld, int64_t P,
                         const double* a_mat, const float* g_mat, double* fpf, void* stream);

/*
 * Device -> pinned-host transfer of `bytes` bytes (the averaged model's D2H
 * feeding fedavg_trainer.py:219).  blocks == 0: the runtime's DMA copy
 * (hipMemcpyAsync; the production choice, fastest end to end).  blocks > 0:
 * a zero-copy kernel with a fixed grid of `blocks` workgroups writing straight
 * into the mapped pinned buffer, leaving the other CUs to a concurrent
 * reduce.  host_dst must be pinned host memory (checked with
 * hipPointerGetAttributes); src and host_dst 16-B aligned.
 */
int fedavg_copy_to_host(const void* src, void* host_dst, int64_t bytes, int blocks, void* stream);

/*
 * Input distribution of the P-sharded reduce: one
 * strided host->device DMA of `rows` rows of `width_bytes` each, from pinned
 * host memory with row pitch `src_pitch_bytes` (the full [K, P] client
 * buffer; host_src points at this rank's first column) into device rows of
 * pitch `dst_pitch_bytes` (this rank's [K, ld] buffer).  Replaces, for one
 * rank's columns, the per-client host tensors reaching the reduction
 * (fedavg_trainer.py:199 -> :450-457).  host_src must be pinned (checked);
 * stream-ordered and asynchronous.
 */
int fedavg_upload_shard(void* dst, int64_t dst_pitch_bytes, const void* host_src, int64_t src_pitch_bytes,
                        int64_t width_bytes, int64_t rows, void* stream);

/*
 * Host helper: weights[i] = (float)((double)n_i / (double)sum(n)) for integer
 * sample counts, exactly as Python's int/int true division followed by ATen's
 * double->float cast (fedavg_trainer.py:444-447,453).  Counts must be >= 0
 * and sum to a value <= 2^53; returns FEDAVG_EINVAL on a zero sum (the
 * reference raises ZeroDivisionError).  `weights` is HOST memory.
 */
int fedavg_weights_f32(const int64_t* sample_nums, int64_t K, float* weights);

/*
 * fedavg_reduce_f32 (aligned production path) with its kernel launches
 * bracketed by two caller-created hipEvent_t's attached to the launches
 * themselves (hipExtLaunchKernel): start_event fires when the first launch
 * starts, stop_event when the last one ends.  hipEventElapsedTime of the pair
 * is the reduce's kernel time with no extra barrier packets in the stream
 * (a separate hipEventRecord pair serialises back-to-back launches and cost
 * ~8 us per call on MI355X).  Same bits as fedavg_reduce_f32; the
 * measurement hook bench.py uses.  FEDAVG_EALIGN for the unaligned paths.
 */
int fedavg_reduce_f32_timed(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights,
                            float* out, void* stream, void* start_event, void* stop_event);

/*
 * The schedule fedavg_reduce_f32() uses for an aligned [K, P] problem:
 * rows per load batch, 16-B column slices per thread, the kernel and load
 * policy (nontemporal: 0 default-policy loads, 1 nontemporal loads through
 * global pointers, 2 nontemporal loads through per-row buffer descriptors),
 * and the number of round-split launches.  Host-only query (bench.py names the kernel from it).
 */
int fedavg_f32_schedule(int64_t K, int64_t P, int* unroll, int* cols, int* nontemporal, int* launches);
/* The same for P columns of a row buffer with row stride ld (a column chunk
 * of a wider shard when ld > P: no Infinity-Cache-resident schedule). */
int fedavg_f32_schedule_ld(int64_t K, int64_t P, int64_t ld, int* unroll, int* cols, int* nontemporal,
                           int* launches);


/*
 * Host runtime: pack client state_dicts into pinned client-major rows.
 *
 * One item per (client, key): copy `numel` elements from `src` (host, dense)
 * to element offset `dst_offset` of `dst_base` (host; for the packed [K, ld]
 * layout dst_offset = row * ld + key offset).  `kind` selects the source
 * type: 0 = same dtype as the destination (elem_size bytes per element);
 * 1..6 = int64, int32, int16, int8, uint8, bool promoted to fp32 with the
 * static_cast ATen applies to `int_tensor * python_float`
 * (fedavg_trainer.py:455).  Work is split evenly by bytes over `n_threads`
 * host threads (a persistent pool inside the library).  Replaces the
 * reference's per-key host loop over w_locals (fedavg_trainer.py:450-452) as
 * the way parameters reach the reduction.  Returns 0 or FEDAVG_EINVAL.
 */
typedef struct fedavg_pack_item {
  int64_t src;        /* host address of the first source element */
  int64_t numel;      /* elements to copy                        */
  int64_t dst_offset; /* destination element offset              */
  int64_t kind;       /* 0 raw, 1 i64, 2 i32, 3 i16, 4 i8, 5 u8, 6 bool */
} fedavg_pack_item;

int fedavg_pack_rows(const fedavg_pack_item* items, int64_t n_items, void* dst_base,
                     int64_t elem_size, int n_threads);

/*
 * Host runtime: one small round in a single call (the drop-in's path when a
 * round's fp32 rows are a few MB, e.g. the reference's MNIST-LR config):
 * fedavg_pack_rows(items -> host_rows), host_w[i] = (float)weights[i] (the
 * reference's Python-double weights n_i / N, fedavg_trainer.py:453, rounded as
 * ATen rounds the scalar at :455), then ONE kernel that reads the rows and
 * weights from pinned memory, copies them to dev_rows / dev_w (kept for the
 * round's later passes), reduces in the reference's order (the bits of
 * fedavg_reduce_f32) and writes the averaged model to dev_out and host_out;
 * then waits for `stream`.  host_rows [K, ld], host_w
 * [K], host_out [P]: pinned host memory; dev_rows [K, ld], dev_w [K], dev_out
 * [P]: device memory; ld % 4 == 0, rows/out buffers 16-B aligned.
 * Synchronous: on return host_out holds the result.
 */
int fedavg_round_f32(const fedavg_pack_item* items, int64_t n_items, float* host_rows, float* dev_rows, int64_t K,
                     int64_t P, int64_t ld, const double* weights, float* host_w, float* dev_w, float* dev_out,
                     float* host_out, int n_threads, void* stream);

/*
 * Device-resident clients: the reference's aggregate (fedavg_trainer.py:441-458)
 * reduces whatever device its state_dicts live on; when the clients' tensors
 * are already in HBM (client.py:96 without the .cpu()), this packs them into
 * the [K, ld] rows with ONE kernel instead of a host walk.  Same item list and
 * conversions as fedavg_pack_rows, but every item's src must be device memory
 * of the current device and dst_base is the device staging buffer.  The item
 * table and a chunk prefix sum are written to host_ws (pinned) and copied to
 * dev_ws (device) on `stream`, both of fedavg_pack_rows_device_workspace(n_items)
 * bytes, 16-B aligned; host_ws must not be rewritten until `stream` has passed
 * this call.  Stream-ordered and asynchronous.  Returns 0 or a negative code.
 */
int64_t fedavg_pack_rows_device_workspace(int64_t n_items);
int fedavg_pack_rows_device(const fedavg_pack_item* items, int64_t n_items, void* dst_base, int64_t elem_size,
                            void* host_ws, void* dev_ws, int64_t ws_bytes, void* stream);

/*
 * Zero-copy aggregation of device-resident clients (no [K, ld] rows): the fp32
 * group of the model as a key table -- key_numel / key_offset (element offset
 * in `out` / `glob`) / key_kind (fedavg_pack_item kinds: 0 fp32, 1..6 integer
 * and bool sources promoted to fp32) -- and client_ptrs [K][n_keys], the
 * device address of client k's tensor for key j (fp32 sources 4-B aligned).
 * fedavg_reduce_segments_f32 writes the averaged fp32 group into `out` [P]
 * with the bits of fedavg_reduce_f32 on the packed rows (fedavg_trainer.py:
 * 450-457); fedavg_client_sqdist_segments_f32 is fedavg_client_sqdist_f32 on
 * the same tables (:291; partials: fedavg_segments_partials doubles).  The
 * tables are staged through host_ws (pinned) into dev_ws (device), both
 * fedavg_segments_workspace(K, n_keys) bytes; host_ws must not be rewritten
 * until `stream` has passed the call.  Stream-ordered, asynchronous.
 */
int64_t fedavg_segments_workspace(int64_t K, int64_t n_keys);
int64_t fedavg_segments_partials(const int64_t* key_numel, int64_t n_keys, int64_t K);
int fedavg_reduce_segments_f32(const int64_t* client_ptrs, const int64_t* key_numel, const int64_t* key_offset,
                               const int64_t* key_kind, int64_t n_keys, int64_t K, const float* weights, float* out,
                               void* host_ws, void* dev_ws, int64_t ws_bytes, void* stream);
int fedavg_client_sqdist_segments_f32(const int64_t* client_ptrs, const int64_t* key_numel, const int64_t* key_offset,
                                      const int64_t* key_kind, int64_t n_keys, int64_t K, const float* glob,
                                      double* partials, int64_t partial_elems, double* sumsq, void* host_ws,
                                      void* dev_ws, int64_t ws_bytes, void* stream);
/*
 * Both in ONE pass over the clients' tensors (the fused tiles of
 * fedavg_reduce_sqdist_f32 on the same key/pointer tables): `out` with the
 * bits of fedavg_reduce_segments_f32, sumsq the :291 sums against that out.
 * Needs 1 <= K <= 256 and every fp32 key's client tensors 16-B aligned
 * (FEDAVG_EALIGN / FEDAVG_EINVAL otherwise: run the two calls above).
 * partials : fedavg_reduce_sqdist_segments_partials(K) doubles.
 */
int64_t fedavg_reduce_sqdist_segments_partials(int64_t K);
int fedavg_reduce_sqdist_segments_f32(const int64_t* client_ptrs, const int64_t* key_numel,
                                      const int64_t* key_offset, const int64_t* key_kind, int64_t n_keys,
                                      int64_t K, const float* weights, float* out, double* partials,
                                      int64_t partial_elems, double* sumsq, void* host_ws, void* dev_ws,
                                      int64_t ws_bytes, void* stream);

/*
 * A device-resident round's fp32 group in ONE call (the host side of
 * fedavg_trainer.py:441-458 after the walk over the clients' state_dicts,
 * with :291's sums when asked): replaces the per-round sequence "gather the
 * group's pointer columns, convert the integer keys, upload the weights,
 * stage the tables" with one pass over the walk's address table and one H2D.
 *   client_ptrs [K][ptr_ld]: client k's device address of every key of the
 *     model (the walk's table); key_index [n_keys]: the group key j's column
 *     in it (NULL: column j); key_numel / key_offset / key_kind as
 *     fedavg_reduce_segments_f32;
 *   weights [K]: the reference's n_i / N as host doubles, rounded here to
 *     fp32 (nearest even, as ATen rounds the scalar at :455);
 *   sumsq (NULL: the reduce alone) with partials :
 *     fedavg_reduce_sqdist_segments_partials(K) doubles;
 *   int_scratch: device fp32, fedavg_device_round_scratch(...) floats, 16-B
 *     aligned (NULL when that is 0): a fused round's integer / bool keys
 *     (BatchNorm's num_batches_tracked) are converted into it first;
 *   host_ws (pinned) / dev_ws (device): fedavg_device_round_workspace(K,
 *     n_keys) bytes, 16-B aligned; host_ws must not be rewritten until
 *     `stream` has passed the call.
 * Returns 0 when `out` and the sums were written (the fused pass), 1 when
 * only `out` was (sumsq NULL, K > 256 or an fp32 source not 16-B aligned:
 * the caller forms :291 with fedavg_client_sqdist_segments_f32), or a
 * negative code.  `out` has the bits of fedavg_reduce_segments_f32 either
 * way.  Stream-ordered and asynchronous.
 */
int64_t fedavg_device_round_workspace(int64_t K, int64_t n_keys);
int64_t fedavg_device_round_scratch(const int64_t* key_numel, const int64_t* key_kind, int64_t n_keys, int64_t K);
int fedavg_device_round_f32(const int64_t* client_ptrs, int64_t ptr_ld, const int64_t* key_index,
                            const int64_t* key_numel, const int64_t* key_offset, const int64_t* key_kind,
                            int64_t n_keys, int64_t K, const double* weights, float* out, double* partials,
                            int64_t partial_elems, double* sumsq, float* int_scratch, int64_t scratch_elems,
                            void* host_ws, void* dev_ws, int64_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* FEDAVG_AMD_H */
