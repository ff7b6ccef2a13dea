// FETCH_SIZE / WRITE_SIZE calibration for the access widths and patterns of this library's kernels
// (MI355X_MICROARCH.md: the x2 correction is calibrated for 16-B-per-lane streaming reads only).
// Every kernel reads (or writes) a known number of bytes of a 1.5 GiB buffer (larger than the
// 256 MiB Infinity Cache, so nothing stays resident between launches):
//   k_rd8      8 B per lane, coalesced (consecutive lanes, consecutive doubles) — k_cand/k_emit SoA loads
//   k_rd16    16 B per lane, coalesced — the guide's calibrated case
//   k_gather  k_prep's pattern: rows [12][S] of doubles, lane s visits the 12 rows in its own order
//   k_wr8      8 B per lane stores, coalesced
//   k_wr16    16 B per lane stores, coalesced
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
// Run:   rocprofv3 --pmc FETCH_SIZE --kernel-trace -d <dir> -- tools/fetch_calib   (and WRITE_SIZE)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k_rd8(const double* __restrict__ a, int64_t n, double* out) {
    double s = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 12345.678) out[0] = s;   // never true: keeps the loads
}
__global__ void k_rd16(const double2* __restrict__ a, int64_t n2, double* out) {
    double s = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x) {
        const double2 v = a[i];
        s += v.x + v.y;
    }
    if (s == 12345.678) out[0] = s;
}
// rows [12][S]; lane s reads row (k * 5 + s * 7) % 12 at visit k (a per-lane permutation: 5 is a unit mod 12)
__global__ void k_gather(const double* __restrict__ a, int64_t S, double* out) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    double acc = 0;
    for (int k = 0; k < 12; k++) {
        const int row = (int)((k * 5 + s * 7) % 12);
        acc += a[(int64_t)row * S + s];
        // some dependent arithmetic between visits, as k_prep's lane matching
        for (int j = 0; j < 64; j++) acc = acc * 0.999999 + 1e-9;
    }
    if (acc == 12345.678) out[0] = acc;
}
__global__ void k_wr8(double* a, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) a[i] = (double)i;
}
__global__ void k_wr16(double2* a, int64_t n2) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x) a[i] = make_double2((double)i, 1.0);
}

int main() {
    const int64_t n = (int64_t)192 << 20;          // 192 Mi doubles = 1.5 GiB
    double *a, *out;
    if (hipMalloc(&a, n * sizeof(double)) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    const int grid = 256 * 8 * 4, blk = 256;
    hipLaunchKernelGGL(k_wr8, dim3(grid), dim3(blk), 0, 0, a, n);
    hipLaunchKernelGGL(k_wr16, dim3(grid), dim3(blk), 0, 0, (double2*)a, n / 2);
    hipLaunchKernelGGL(k_rd8, dim3(grid), dim3(blk), 0, 0, a, n, out);
    hipLaunchKernelGGL(k_rd16, dim3(grid), dim3(blk), 0, 0, (const double2*)a, n / 2, out);
    const int64_t S = n / 12;
    hipLaunchKernelGGL(k_gather, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, 0, a, S, out);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("bytes per kernel: rd8/rd16/wr8/wr16 %lld, gather %lld (KiB: %lld / %lld)\n",
           (long long)(n * 8), (long long)(S * 12 * 8), (long long)(n * 8 / 1024), (long long)(S * 12 * 8 / 1024));
    return 0;
}
