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
// v_mfma_f64_16x16x4_f64 (operands in registers), 4 waves per CU-slot.
__global__ __launch_bounds__(256) void rate_kernel(int iters, double* out) {
  const int lane = threadIdx.x & 63;
  double a = 1.0 + 1e-3 * lane, b = 1.0 - 1e-3 * lane;
  v4d acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = v4d_zero();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = mfma_f64(a, b, acc[j]);
  }
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  if (s == 12345.678) out[0] = s;  // keep live
}
}  // namespace

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
