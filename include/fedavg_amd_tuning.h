/*
 * fedavg_amd_tuning.h -- benchmarking hooks, exported ONLY by the probe
 * library libfedavg_amd_probe.so (the product library libfedavg_amd.so is
 * built without them).  Not part of the drop-in contract: scripts/ and the
 * variant tests load the probe library to A/B kernel variants in one process,
 * as the CDNA guide's rule 24 asks.  The probe library also exports every
 * product entry point of fedavg_amd.h (same sources, built with
 * -DFEDAVG_TUNING), so one handle serves a whole A/B run.
 */
#ifndef FEDAVG_AMD_TUNING_H
#define FEDAVG_AMD_TUNING_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Defaults of the first-version kernel (fedavg_reduce_f32_tuned; also the
 * path fedavg_reduce_f32 takes for buffers that are not 16-B aligned). */
#define FEDAVG_DEFAULT_UNROLL 8
#define FEDAVG_DEFAULT_NONTEMPORAL 0

/*
 * fedavg_reduce_f32 with explicit variant knobs:
 *   unroll      : client-axis loads kept in flight per thread (4, 8 or 16)
 *   nontemporal : 1 = streaming (nt) loads for the once-read client rows
 * Results are bit-identical for every variant (same per-element order).
 */
int fedavg_reduce_f32_tuned(const float* clients, int64_t K, int64_t P, int64_t ld,
                            const float* weights, float* out, int unroll, int nontemporal,
                            void* stream);

/*
 * Variant family of the exact fp32 kernel (same bits, different schedule):
 *   unroll     : client rows per load batch (1, 2, 4, 8, 16; 32 with cols <= 2)
 *   cols       : 16-B column slices per thread (1, 2, 4; 8 with unroll <= 8; 16 with unroll <= 2)
 *   pipelined  : 0 = register batches; 1 = register double-buffered batches
 *                (2*unroll*cols loads in flight); 2 = LDS-DMA staging
 *                (global_load_lds_dwordx4 into per-wave LDS slots, unroll*cols <= 16);
 *                3 = balanced persistent: grid = blocks resident on the chip, each block
 *                owns an equal contiguous range of 1 KiB wave-slices (unroll*cols <= 32);
 *                4 = round-split: the plain kernel (mode 0) launched over the fewest
 *                equal column ranges that each fit in one resident round;
 *                5 = windowed balanced: equal windows, each launched with exactly
 *                max_blocks blocks (0 = 3 x CUs), split evenly at 1 KiB granularity
 *   max_blocks : 0 = default grid (one block per column group; for pipelined == 3
 *                the resident block count); > 0 caps / sets the grid
 * Needs 16-B aligned clients/out and ld % 4 == 0.
 */
int fedavg_reduce_f32_variant(const float* clients, int64_t K, int64_t P, int64_t ld,
                              const float* weights, float* out, int unroll, int nontemporal,
                              int cols, int pipelined, int max_blocks, void* stream);

/*
 * Exact fp32 reduce over the TILED layout [ceil(P/1024)][K][1024]: tile t
 * holds columns [1024t, 1024t+1024) of every client, client-major inside the
 * tile (a block then streams K*4 KiB contiguous bytes).  Padding columns of
 * the last tile are read but never stored.
 */
int fedavg_reduce_tiled_f32(const float* tiles, int64_t K, int64_t P, const float* weights,
                            float* out, int unroll, void* stream);

/*
 * Test hook: out[i] = in[i] (fp32 bit pattern) rounded to 16 bits by the
 * production kernels' element rule -- mode 0: bf16, packed hardware RNE
 * (v_cvt_pk_bf16_f32); 1: bf16, c10's integer round_to_nearest_even;
 * 2: fp16, packed hardware (v_cvt_pk_f16_f32); 3: fp16, scalar
 * v_cvt_f16_f32.  Lets the GPU tests compare the rules over all 2^32 inputs.
 */
int fedavg_probe_cvt16(const uint32_t* in, int64_t n, int mode, uint16_t* out, void* stream);

/*
 * Packed fp16 (bf16 = 0) / bf16 (bf16 = 1) exact kernel with an explicit
 * schedule: unroll rows per batch x cols 16-B slices (8 halves) per thread,
 * (U, C) in {(1,8), (2,8), (4,8), (2,4), (4,4), (8,4), (4,2), (8,2), (1,16),
 * (2,16), (16,1)}; nontemporal loads; round-split launches of <= max_blocks
 * blocks (0 = one launch).  Same bits as fedavg_reduce_f16 / _bf16.
 * fedavg_half_schedule reports the production choice for [K, P].
 */
int fedavg_reduce_half_variant(int bf16, const uint16_t* clients, int64_t K, int64_t P, int64_t ld,
                               const float* weights, uint16_t* out, int unroll, int cols, int max_blocks,
                               void* stream);
int fedavg_half_schedule(int64_t K, int64_t P, int* unroll, int* cols, int* nontemporal, int* launches);

/*
 * Distance pass (fedavg_client_sqdist_f32) with an explicit schedule: unroll
 * client rows per batch x cols 16-B slices per thread ((4,4), (8,4), (4,8),
 * (2,8)), round-split launches of <= max_blocks blocks (0 = one launch).
 * workspace: fedavg_client_sqdist_workspace(K, P) doubles covers every
 * variant.  Per-wave partials differ with the schedule, so the fp64 sums may
 * differ in their last bits between variants (each one is deterministic).
 */
int fedavg_client_sqdist_variant(const float* clients, int64_t K, int64_t P, int64_t ld, const float* glob,
                                 double* workspace, int64_t workspace_elems, double* sumsq, int unroll, int cols,
                                 int max_blocks, void* stream);

/*
 * The FPF2 index (:272) as a column-window pass (measurement only): blocks
 * cover (column window x row group) and leave one fp64 partial per (row,
 * wave) in `workspace` (fedavg_fpf_index_workspace(n_rows, P) doubles), summed
 * per row in a fixed order.  unroll rows per batch x cols 16-B slices per
 * thread ((4,1), (8,1), (16,1), (8,2), (4,4), (8,4), (4,8)); row_groups
 * blocks along the rows (0 = about 3 blocks per CU).  Measured slower than
 * the production one-block-per-row fedavg_fpf_index_f32.
 */
int64_t fedavg_fpf_index_workspace(int64_t n_rows, int64_t P);
int fedavg_fpf_index_variant(const float* diffs, int64_t n_rows, int64_t ld, int64_t P, const float* a_mat,
                             const float* g_mat, float* fpf, double* workspace, int64_t workspace_elems, int unroll,
                             int cols, int row_groups, void* stream);

/*
 * HBM read-ceiling probe (measurement only): stream `nvec` 16-B vectors of a
 * device buffer with no reduction structure, in `launches` equal launches of
 * `blocks` workgroups each.  mode 0: grid-stride, nontemporal; 1: one
 * contiguous range per block, nontemporal; 2: as 1 with default-policy loads.
 * `sink` needs `blocks` floats (written only on an impossible value match).
 */
/* The production U4 x C8 nt reduce with an XCD-aware workgroup order (XCD x
 * takes one contiguous run of column slices); same round-split launches, same
 * bits.  Measurement only. */
int fedavg_reduce_f32_xcd(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights, float* out,
                          int max_blocks, void* stream);

/*
 * Zero-copy device-client reduce (fedavg_reduce_segments_f32, same tables and
 * workspaces) with an explicit schedule: unroll client pointers per load
 * batch x cols 16-B slices per thread, (U, C) in {(4,8) production, (8,4),
 * (2,8), (4,4), (8,2), (16,2), (2,16), (1,16)}; units of 1,024 x cols
 * columns; round-split launches of <= blocks_per_cu x CUs workgroups
 * (0 = one launch).  Same bits as the production call.
 */
/*
 * Host-side phase times of this thread's last fedavg_device_round_f32 call
 * (probe library build only): cumulative microseconds at up to `cap` marks
 * -- 0 start, 1 argument / pointer-attribute checks, 2 key validation, 3 the
 * pointer-table fill, 4 the sources' spot check, 5 plan + key table +
 * weights, 6 the tables' H2D issued, 7 the integer keys' launch, 8 the
 * reduce launches.  Returns the number of marks written.
 */
int fedavg_device_round_phases(double* us, int cap);
int fedavg_reduce_segments_f32_variant(const int64_t* client_ptrs, const int64_t* key_numel, const int64_t* key_offset,
                                       const int64_t* key_kind, int64_t n_keys, int64_t K, const float* weights,
                                       float* out, void* host_ws, void* dev_ws, int64_t ws_bytes, int unroll, int cols,
                                       int blocks_per_cu, void* stream);

/*
 * :291 on device-resident clients (fedavg_client_sqdist_segments_f32, same
 * tables and workspaces) with an explicit schedule: unroll client rows per
 * load batch x cols 16-B slices per thread, (U, C) in {(1,4), (2,4), (4,4),
 * (8,4), (4,1), (8,1), (4,2), (8,2), (2,8), (4,8)}; units of 1,024 x cols
 * columns; partials: K x units x 4 doubles for that unit size.
 */
int fedavg_client_sqdist_segments_f32_variant(const int64_t* client_ptrs, const int64_t* key_numel,
                                              const int64_t* key_offset, const int64_t* key_kind, int64_t n_keys,
                                              int64_t K, const float* glob, double* partials, int64_t partial_elems,
                                              double* sumsq, void* host_ws, void* dev_ws, int64_t ws_bytes,
                                              int unroll, int cols, void* stream);

/* The exact fp32 row reduce through buffer descriptors (one per client row
 * and column group, base in SGPRs, 32-bit lane offsets) in launch_split's
 * round-split schedule, workgroups of `block` threads (64, 128 or 256).
 * (unroll, cols, block): 256-thread groups (4,8) (8,4) (4,4) (2,8) (2,16)
 * (1,16) (8,8) (4,16) (16,1) (16,2) (16,4) (8,2) (8,1); 128 and 64 threads
 * (8,1) (8,2) (8,4) (16,1) (16,2) (16,4) (4,4) (4,8), plus (32,1) (32,2) at
 * 64.  max_blocks 0 = resident blocks.  Same bits. */
int fedavg_reduce_f32_buf(const float* clients, int64_t K, int64_t P, int64_t ld, const float* weights, float* out,
                          int unroll, int cols, int block, int max_blocks, void* stream);

/* The distance pass (fedavg_client_sqdist_f32) through buffer descriptors:
 * per block, one descriptor per client row and one for glob whose record
 * count ends at the last float4 (lanes past it read 0); (unroll, cols) in
 * {(4,8), (8,4), (2,16), (2,8), (8,8)}; round-split launches of <= max_blocks
 * blocks (0 = one launch).  Same workspace as fedavg_client_sqdist_f32. */
/* fedavg_reduce_sqdist_f32 with an explicit tile width (cols = 64, 128 or
 * 256 columns) and workgroups per CU (0 = as many as LDS allows); K <= 128,
 * workspace >= K x (blocks per CU x CUs) doubles.  Other codes select the
 * probe kernels listed at the switch in fedavg_dist.hip, among them the
 * wave-owned windows: 70000000 + KMAX x 100 + 40 + VEC (K <= KMAX; KMAX x
 * VEC in 16 x 4, 32 x 4, 48 x 4, 64 x 2, 80 x 2, 100 x 2, 128 x 1; workspace
 * >= K x 4 x workgroups). */
int fedavg_reduce_sqdist_f32_variant(const float* clients, int64_t K, int64_t P, int64_t ld,
                                     const float* weights, float* out, double* workspace,
                                     int64_t workspace_elems, double* sumsq, int cols,
                                     int blocks_per_cu, void* stream);
int fedavg_client_sqdist_buf(const float* clients, int64_t K, int64_t P, int64_t ld, const float* glob,
                             double* workspace, int64_t workspace_elems, double* sumsq, int unroll, int cols,
                             int max_blocks, void* stream);

/* fp16 (dtype 0) / bf16 (1) / fp64 (2) exact reduce through per-row buffer
 * descriptors (reduce_vec_buf_kernel; weights fp32 for fp16/bf16, fp64 for
 * fp64), (unroll, cols) in {(8,4), (4,8), (2,16), (4,4), (2,8)}; round-split
 * launches of <= max_blocks blocks (0 = one launch).  Same bits as
 * fedavg_reduce_f16 / _bf16 / _f64. */
int fedavg_reduce_vec_buf(int dtype, const void* clients, int64_t K, int64_t P, int64_t ld, const void* weights,
                          void* out, int unroll, int cols, int max_blocks, void* stream);

int fedavg_probe_read_f32x4(const float* buf, int64_t nvec, int mode, int blocks, int launches, float* sink,
                            void* stream);

/*
 * Co-scheduling probes (measurement only).  fedavg_probe_busy_copy: copy
 * `bytes` with `blocks` workgroups of a kernel holding ~294 registers per
 * wave, then keep every wave resident until hold_us microseconds after it
 * started -- a stand-in for a collective's kernel (RCCL's generic kernel on
 * gfx950 holds 261 VGPR + 17 AGPR; bound by xGMI, it stays resident).  fedavg_stream_create_masked: a non-blocking stream
 * whose kernels may use all CUs but the last `reserve_cus` (hip CU mask), or,
 * with reserve_cus == 0, a stream of the given priority; destroy it with
 * fedavg_stream_destroy.
 */
int fedavg_probe_busy_copy(const void* src, void* dst, int64_t bytes, int blocks, int hold_us, void* stream);
int fedavg_stream_create_masked(int reserve_cus, int priority, void** stream);

/*
 * Shader-clock probe (measurement only): `blocks` one-wave workgroups each
 * stamp (s_memtime, s_memrealtime) `samples + 1` times, `interval_us` apart,
 * into out[blocks][samples + 1][2] (uint64).  Launched on a side stream
 * beside a kernel, d(memtime) / d(realtime) * 100 is the shader clock in MHz
 * the chip holds while that kernel runs.
 */
int fedavg_probe_clock(unsigned long long* out, int blocks, int samples, int interval_us, void* stream);
int fedavg_stream_destroy(void* stream);

#ifdef __cplusplus
}
#endif

#endif /* FEDAVG_AMD_TUNING_H */
