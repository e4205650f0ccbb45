// Accuracy of v_rcp_f64 / v_rsq_f64 alone and after one Newton step, against IEEE 1/b and
// 1/sqrt(b) (the tolerance triangulation's reciprocals).  hipcc -O3 --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

__global__ void probe(const double* b, int n, double* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = b[i];
    const double r0 = __builtin_amdgcn_rcp(x);
    double e = __builtin_fma(-x, r0, 1.0);
    const double r1 = __builtin_fma(r0, e, r0);
    const double q0 = __builtin_amdgcn_rsq(x);
    double t = x * q0;
    double f = __builtin_fma(-t, q0, 1.0);
    const double q1 = __builtin_fma(0.5 * q0, f, q0);
    out[6 * i + 0] = 1.0 / x;
    out[6 * i + 1] = r0;
    out[6 * i + 2] = r1;
    out[6 * i + 3] = 1.0 / sqrt(x);
    out[6 * i + 4] = q0;
    out[6 * i + 5] = q1;
}

static int64_t ulps(double a, double b) {
    int64_t x, y;
    memcpy(&x, &a, 8);
    memcpy(&y, &b, 8);
    return x > y ? x - y : y - x;
}

int main() {
    const int n = 1 << 22;
    std::vector<double> h(n);
    uint64_t s = 12345;
    for (int i = 0; i < n; i++) {
        s = s * 6364136223846793005ULL + 1442695040888963407ULL;
        h[i] = std::pow(10.0, -8.0 + 16.0 * ((s >> 11) * (1.0 / 9007199254740992.0)));
    }
    double *db, *dout;
    hipMalloc(&db, n * 8);
    hipMalloc(&dout, n * 48);
    hipMemcpy(db, h.data(), n * 8, hipMemcpyHostToDevice);
    probe<<<n / 256, 256>>>(db, n, dout);
    std::vector<double> o(6 * (size_t)n);
    hipMemcpy(o.data(), dout, n * 48, hipMemcpyDeviceToHost);
    int64_t m[4] = {0, 0, 0, 0};
    for (int i = 0; i < n; i++) {
        m[0] = std::max(m[0], ulps(o[6 * i], o[6 * i + 1]));
        m[1] = std::max(m[1], ulps(o[6 * i], o[6 * i + 2]));
        m[2] = std::max(m[2], ulps(o[6 * i + 3], o[6 * i + 4]));
        m[3] = std::max(m[3], ulps(o[6 * i + 3], o[6 * i + 5]));
    }
    printf("max ulp vs IEEE: rcp %lld, rcp+1 Newton %lld, rsq %lld, rsq+1 Newton %lld\n", (long long)m[0],
           (long long)m[1], (long long)m[2], (long long)m[3]);
    return 0;
}
