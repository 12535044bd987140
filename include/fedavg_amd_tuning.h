/*
 * fedavg_amd_tuning.h -- benchmarking hooks of libfedavg_amd.so (not part of
 * the drop-in contract; bench.py uses them to A/B kernel variants in one
 * process, as the CDNA guide's rule 24 asks).
 */
#ifndef FEDAVG_AMD_TUNING_H
#define FEDAVG_AMD_TUNING_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Defaults used by fedavg_reduce_f32(). */
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

#ifdef __cplusplus
}
#endif

#endif /* FEDAVG_AMD_TUNING_H */
