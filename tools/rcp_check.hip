// Accuracy of the hardware FP64 reciprocal and reciprocal square root (v_rcp_f64, v_rsq_f64) on
// gfx950: max error in ulps against the correctly rounded 1/x and 1/sqrt(x) (computed on the host
// in long double), over a log-uniform sweep of x. Usage: tools/rcp_check [n]
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
__global__ void k(const double* x, double* r, double* q, long n) {
    long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (i < n) { r[i] = __builtin_amdgcn_rcp(x[i]); q[i] = __builtin_amdgcn_rsq(x[i]); }
}
static double ulps(double got, long double want) {
    double w = (double)want;
    double u = std::nextafter(std::fabs(w), INFINITY) - std::fabs(w);
    return (double)std::fabs(((long double)got - want) / u);
}
int main(int argc, char** argv) {
    long n = argc > 1 ? atol(argv[1]) : 1 << 22;
    std::vector<double> x(n), r(n), q(n);
    unsigned long long s = 0x9E3779B97F4A7C15ull;
    for (long i = 0; i < n; i++) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        x[i] = std::ldexp(1.0 + (double)(s >> 11) * 0x1p-53, (int)(s % 80) - 40);
    }
    double *dx, *dr, *dq;
    hipMalloc(&dx, n * 8); hipMalloc(&dr, n * 8); hipMalloc(&dq, n * 8);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    k<<<(n + 255) / 256, 256>>>(dx, dr, dq, n);
    hipMemcpy(r.data(), dr, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(q.data(), dq, n * 8, hipMemcpyDeviceToHost);
    double mr = 0, mq = 0; long er = 0, eq = 0;
    for (long i = 0; i < n; i++) {
        const long double lx = x[i];
        const double a = ulps(r[i], 1.0L / lx), b = ulps(q[i], 1.0L / sqrtl(lx));
        if (a > mr) mr = a;
        if (b > mq) mq = b;
        er += r[i] != (double)(1.0L / lx);
        eq += q[i] != (double)(1.0L / sqrtl(lx));
    }
    printf("{\"n\": %ld, \"rcp_max_ulp\": %.3f, \"rcp_not_rn_frac\": %.4g, \"rsq_max_ulp\": %.3f, \"rsq_not_rn_frac\": %.4g}\n",
           n, mr, (double)er / n, mq, (double)eq / n);
    return 0;
}
