/*
 * Development probes of botorch_amd (NOT the product ABI): timing and trace
 * entry points the tools/ scripts use.  Built only into
 * tools/libbotorch_amd_tools.so (`make tools`: the product sources compiled
 * with -DBO_TOOLS), never into botorch_amd/libbotorch_amd.so.
 */
#ifndef BOTORCH_AMD_TOOLS_H
#define BOTORCH_AMD_TOOLS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* fp64 VALU / LDS latency probe (tools/probe_rate.py): out[0..3] = s_memtime
 * ticks of 256 dependent FMAs, 256 x 8 independent FMAs, 64 rsq+2NR chains,
 * 256 dependent LDS reads, with `waves` waves in the workgroup. */
int bo_probe_valu_f64(int waves, long long* out, void* stream);

/* Task trace of the persistent Cholesky DAG (chol_dag.hip) on A (np x np,
 * np % 64 == 0): trace (device, >= 4 x tasks + 8 x np/64 int64) gets per task
 * [start, end, packed block/type/k/j, spin-wait ticks] (100 MHz); *ntasks
 * (HOST int) the count. */
int bo_probe_chol_dag(double* A, double* Linv, int64_t np, int* info, void* work,
                      long long* trace, int* ntasks, void* stream);

/* s_memtime ticks per 16 x 16 diagonal factor + inverse on one wave
 * (tools/probe_diag16.py): out[0..2] = DPP / readlane broadcasts / DPP factor
 * only; sink: one double of scratch. */
int bo_probe_diag16(long long* out, double* sink, void* stream);

/* One workgroup factors + inverts a 64 x 64 SPD A (row-major) reps times with
 * the DAG's diagonal-tile routine (variant 1 column owners, 0 four panels):
 * out = [L | L^{-1}], ct[0..7] the last rep's phase stamps, ct[8] all reps'
 * wall-clock ticks (tools/probe_potrf64.py). */
int bo_probe_potrf64(const double* A, double* out, long long* ct, int* info, int variant, int reps,
                     void* stream);

#ifdef __cplusplus
}
#endif

#endif /* BOTORCH_AMD_TOOLS_H */
