// tools/valu_peak.hip — measured FP64 VALU issue rate of the MI355X (wave-instructions per cycle
// per SIMD and FLOP/s) for the roofline of the FP64-VALU-bound planner kernels. Each lane runs 8
// independent dependency chains (so issue, not latency, bounds), grid = 8 waves per SIMD on every
// CU. Prints one JSON line. Build: hipcc --offload-arch=gfx950 -O3 -o valu_peak valu_peak.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int kOp>
__global__ __launch_bounds__(256) void k_chain(double* out, int iters, double s) {
    double a0 = threadIdx.x * 1e-3, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < iters; i++) {
#define STEP(x)                                                        \
        if (kOp == 0) x = __builtin_fma(x, s, 0.5);                    \
        else if (kOp == 1) x = x * s;                                  \
        else if (kOp == 2) x = x + s;                                  \
        else if (kOp == 3) x = __builtin_amdgcn_rcp(x + s);           \
        else if (kOp == 4) x = __builtin_sqrt(x + s);                  \
        else if (kOp == 5) x = s / (x + 0.5);                          \
        else x = __builtin_fma(__builtin_fma(-(x + 0.5), __builtin_amdgcn_rcp(x + 0.5), 1.0), s, x);
        STEP(a0) STEP(a1) STEP(a2) STEP(a3) STEP(a4) STEP(a5) STEP(a6) STEP(a7)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

template <int kOp>
double run(double* d, int blocks, int iters, double s) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k_chain<kOp>, dim3(blocks), dim3(256), 0, 0, d, iters, s);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_chain<kOp>, dim3(blocks), dim3(256), 0, 0, d, iters, s);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms * 1e-3;
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 8;                 // 8 blocks x 4 waves = 32 waves per CU
    const int iters = 20000;
    double* d;
    hipMalloc(&d, sizeof(double) * blocks * 256);
    const char* names[7] = {"v_fma_f64", "v_mul_f64", "v_add_f64", "v_rcp_f64(+add)", "sqrt_f64(+add)",
                            "ieee_div_f64(+add)", "rcp+2fma(+2add)"};
    double secs[7] = {run<0>(d, blocks, iters, 0.999999), run<1>(d, blocks, iters, 0.999999),
                      run<2>(d, blocks, iters, 1e-9), run<3>(d, blocks, iters, 0.5), run<4>(d, blocks, iters, 0.5),
                      run<5>(d, blocks, iters, 0.7), run<6>(d, blocks, iters, 0.7)};
    const double waves = blocks * 4.0;
    printf("{\"cus\": %d, \"clock_mhz\": %d", cus, p.clockRate / 1000);
    for (int k = 0; k < 7; k++) {
        const double winstr = waves * iters * 8.0;          // wave-instructions of the op (k >= 3: op + add)
        printf(", \"%s\": {\"wave_instr_per_s\": %.4e, \"lane_ops_per_s\": %.4e}", names[k], winstr / secs[k],
               winstr * 64 / secs[k]);
    }
    printf("}\n");
    return 0;
}
