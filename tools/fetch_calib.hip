// FETCH_SIZE calibration for the posterior GEMM's two load shapes
// (MI355X_MICROARCH.md §HBM: "other access widths are uncalibrated").
// Each kernel reads a 1 GiB buffer (past the 256 MiB Infinity Cache) exactly
// once:
//   wide  -- 16 B per lane, a wave reads 1 KiB contiguous (U rows in
//            post_partials_kernel, BO_LOAD_U);
//   seg   -- 8 B per lane, 16 lanes per 128-B row segment, 4 rows of stride
//            ld per instruction (the K*x^T operand loads, BO_LOAD_B).
// Run under `rocprofv3 --pmc FETCH_SIZE` and compare with the printed bytes.
// Build: hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void wide(const double2* __restrict__ a, int64_t n2, double* out) {
  double s = 0.0;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256) {
    const double2 v = a[i];
    s += v.x + v.y;
  }
  if (s == 12345.0) out[0] = s;  // never true for the zero-filled input: keeps the loads
}

// rows x ld doubles; a workgroup's 4 waves each take 4 rows x 128 columns
// blocks: per instruction lane l reads row r0 + (l >> 4), columns c0 + (l & 15) + 16 j
__global__ __launch_bounds__(256) void seg(const double* __restrict__ a, int rows, int ld, double* out) {
  double s = 0.0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nblk_c = ld / 128;
  const int64_t nblk = (int64_t)(rows / 4) * nblk_c;
  for (int64_t b = (int64_t)blockIdx.x * 4 + wave; b < nblk; b += (int64_t)gridDim.x * 4) {
    const int r0 = (int)(b / nblk_c) * 4, c0 = (int)(b % nblk_c) * 128;
    const double* p = a + (int64_t)(r0 + (lane >> 4)) * ld + c0 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += p[16 * j];
  }
  if (s == 12345.0) out[0] = s;
}

int main() {
  const int64_t bytes = 1ll << 30;
  const int64_t n = bytes / 8;
  double *a = nullptr, *out = nullptr;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&out, 8));
  CK(hipMemset(a, 0, bytes));
  const int ld = 8192, rows = (int)(n / ld);
  for (int rep = 0; rep < 3; ++rep) {
    wide<<<4096, 256>>>(reinterpret_cast<const double2*>(a), n / 2, out);
    CK(hipGetLastError());
    seg<<<4096, 256>>>(a, rows, ld, out);
    CK(hipGetLastError());
  }
  CK(hipDeviceSynchronize());
  std::printf("bytes per launch %lld (FETCH_SIZE in KiB should be %lld if counted exactly)\n",
              (long long)bytes, (long long)(bytes / 1024));
  CK(hipFree(a));
  CK(hipFree(out));
  return 0;
}
