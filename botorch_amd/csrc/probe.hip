// Hardware probe of the v_mfma_f64_16x16x4_f64 accumulator map.
// A[i][k] = i for k == 0, 1 for k == 1, else 0;  B[k][j] = 16 for k == 0,
// j for k == 1, else 0   =>   D[i][j] = 16 i + j.  Lane l, register r of the
// result therefore reports the (row, col) it holds; tests compare it with
// mfma_row()/mfma_col() in common.h.
#include "common.h"

namespace {
__global__ void probe_kernel(double* out) {
  const int lane = threadIdx.x;
  const int i = lane & 15, k = lane >> 4;
  const double a = (k == 0) ? (double)i : (k == 1 ? 1.0 : 0.0);
  const double b = (k == 0) ? 16.0 : (k == 1 ? (double)i : 0.0);
  v4d acc = mfma_f64(a, b, v4d_zero());
  for (int r = 0; r < 4; ++r) {
    out[lane * 8 + r] = acc[r];
    out[lane * 8 + 4 + r] = (double)(mfma_row(lane, r) * 16 + mfma_col(lane));
  }
}
// Peak-rate probe: every wave issues `iters` x 8 independent back-to-back
// v_mfma_f64_16x16x4_f64 (operands in registers), 4 waves per CU-slot.  The
// MFMAs are inline asm on VGPR accumulators: written as builtins, the compiler
// copied all 8 accumulators VGPR -> AGPR -> VGPR around every iteration (128
// moves per 8 MFMAs), which capped the round-1 probe at 47 TF/s.  Dependent
// MFMAs are 8 apart (8 x 16 passes), beyond any srcC hazard window.
__global__ __launch_bounds__(256) void rate_kernel(int iters, double* out) {
  const int lane = threadIdx.x & 63;
  double a = 1.0 + 1e-3 * lane, b = 1.0 - 1e-3 * lane;
  v4d acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = v4d_zero();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc[j]) : "v"(a), "v"(b));
  }
  asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");  // last MFMAs retire before the reads
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  if (s == 12345.678) out[0] = s;  // keep live
}
#ifdef BO_TOOLS
// fp64 VALU latency / issue probe (one workgroup of `waves` waves; wave 0
// lane 0 records s_memtime ticks): out[0] = ticks for 256 dependent v_fma_f64,
// out[1] = ticks for 256 x 8 independent v_fma_f64 (8 chains), out[2] =
// ticks for 64 v_rsq_f64 + 2 Newton steps chained, out[3] = ticks for 256
// dependent ds_read_b64 -> v_add round trips (LDS latency).
__global__ void valu_probe_kernel(double seed, long long* out) {
  __shared__ double buf[256];
  const int tid = threadIdx.x;
  buf[tid & 255] = seed + tid;
  __syncthreads();
  double a = seed + tid, b = 1.0 + 1e-9 * tid;
  long long t0 = clock64();
#pragma unroll 16
  for (int i = 0; i < 256; ++i) a = fma(a, b, 1e-7);
  long long t1 = clock64();
  double c[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) c[j] = a + j;
  long long t2 = clock64();
#pragma unroll 4
  for (int i = 0; i < 256; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = fma(c[j], b, 1e-7);
  long long t3 = clock64();
  double r = c[0] + c[7] + 2.0;
#pragma unroll 4
  for (int i = 0; i < 64; ++i) {
    double q = __builtin_amdgcn_rsq(r);
    const double h = -0.5 * r;
    q = q * fma(h * q, q, 1.5);
    q = q * fma(h * q, q, 1.5);
    r = 2.0 + q;
  }
  long long t4 = clock64();
  int idx = tid & 255;
  double acc = 0.0;
  for (int i = 0; i < 256; ++i) {
    const double v = buf[idx];
    acc += v;
    idx = ((int)v + i) & 255;
  }
  long long t5 = clock64();
  if (tid == 0) {
    out[0] = t1 - t0;
    out[1] = t3 - t2;
    out[2] = t4 - t3;
    out[3] = t5 - t4;
  }
  if (a + r + acc == 1234.5) out[4] = 1;
}
#endif  // BO_TOOLS
}  // namespace

#ifdef BO_TOOLS  // development probe (tools/bo_tools.h), not the product ABI
extern "C" int bo_probe_valu_f64(int waves, long long* out, void* stream) {
  valu_probe_kernel<<<1, 64 * waves, 0, as_stream(stream)>>>(1.5, out);
  BO_LAUNCH_CHECK();
  return BO_OK;
}
#endif  // BO_TOOLS

// flops = blocks * 4 waves * iters * 8 * 2048
extern "C" int bo_probe_mfma_f64_rate(int blocks, int iters, double* out, void* stream) {
  rate_kernel<<<blocks, 256, 0, as_stream(stream)>>>(iters, out);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

extern "C" int bo_probe_mfma_f64_layout(double* out, void* stream) {
  probe_kernel<<<1, 64, 0, as_stream(stream)>>>(out);
  BO_LAUNCH_CHECK();
  return BO_OK;
}
