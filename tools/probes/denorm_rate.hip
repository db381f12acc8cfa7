// Subnormal-operand probe (gfx950, IEEE f32 denormals kept, as the product
// build): the same packed / plain f32 mul+add chains as valu_rate.hip on
// normal values and on subnormal values (every operand and result below
// 2^-126).  The Jacobi march keeps subnormals for bit parity with the
// reference; this measures whether they cost VALU cycles.  Diagnostic only.
//   hipcc --offload-arch=gfx950 -O3 denorm_rate.hip -o denorm_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

template <int N>
__global__ __launch_bounds__(256) void k_pk(float *out, float x0, float a, float b, int iters) {
    f2 x[N];
    for (int i = 0; i < N; ++i) x[i] = (f2){x0, x0};
    const f2 m = {a, a}, c = {b, b};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < N; ++i) x[i] = x[i] * m;
#pragma unroll
        for (int i = 0; i < N; ++i) x[i] = x[i] + c;
    }
    f2 s = x[0];
    for (int i = 1; i < N; ++i) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
}

template <int N>
__global__ __launch_bounds__(256) void k_sc(float *out, float x0, float a, float b, int iters) {
    float x[N];
    for (int i = 0; i < N; ++i) x[i] = x0;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < N; ++i) x[i] = x[i] * a;
#pragma unroll
        for (int i = 0; i < N; ++i) x[i] = x[i] + b;
    }
    float s = x[0];
    for (int i = 1; i < N; ++i) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const int wps = 4;   // waves per SIMD
    dim3 grid(ncu * wps), block(256);
    float *out;
    hipMalloc(&out, (size_t)grid.x * 256 * 4);
    const int iters = 20000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct Case { const char *name; float x0, a, b; } cases[] = {
        {"normal", 1.0f, 0.99999994f, 1e-7f},
        {"subnormal", 1e-39f, 0.99999994f, 1.4e-45f},
    };
    float *host = new float[(size_t)grid.x * 256];
    for (int rep = 0; rep < 2; ++rep)
        for (const Case &c : cases) {
            float ms_pk = 0, ms_sc = 0;
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_pk<8>, grid, block, 0, 0, out, c.x0, c.a, c.b, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms_pk, e0, e1);
            hipMemcpy(host, out, 4, hipMemcpyDeviceToHost);
            const float r_pk = host[0];
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_sc<16>, grid, block, 0, 0, out, c.x0, c.a, c.b, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms_sc, e0, e1);
            hipMemcpy(host, out, 4, hipMemcpyDeviceToHost);
            const double elem = (double)grid.x * 256 * iters * 2 * 16;
            const double simd_s = (double)ncu * 4;
            if (rep)
                printf("%-9s packed %.3f ms (%.1f elem-op/ns/SIMD, result %g)  plain %.3f ms (%.1f, result %g)\n",
                       c.name, ms_pk, elem / (ms_pk * 1e6) / simd_s, r_pk, ms_sc,
                       elem / (ms_sc * 1e6) / simd_s, host[0]);
        }
    delete[] host;
    return 0;
}
