// VALU issue-rate probe (gfx950): packed f32 (v_pk_mul_f32 / v_pk_add_f32)
// against plain f32 (v_mul_f32) on independent chains, every SIMD busy.
// Prints element-ops per cycle per SIMD for each form.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

template <int N>
__global__ __launch_bounds__(256) void k_pk(float *out, float a, int iters) {
    f2 x[N];
    for (int i = 0; i < N; ++i) x[i] = (f2){(float)threadIdx.x + i, (float)i};
    const f2 m = {a, a};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < N; ++i) x[i] = x[i] * m;
#pragma unroll
        for (int i = 0; i < N; ++i) x[i] = x[i] + m;
    }
    f2 s = x[0];
    for (int i = 1; i < N; ++i) s += x[i];
    if (s.x == 123.0f) out[threadIdx.x] = s.y;
}

template <int N>
__global__ __launch_bounds__(256) void k_sc(float *out, float a, int iters) {
    float x[N];
    for (int i = 0; i < N; ++i) x[i] = (float)threadIdx.x + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < N; ++i) x[i] = x[i] * a;
#pragma unroll
        for (int i = 0; i < N; ++i) x[i] = x[i] + a;
    }
    float s = x[0];
    for (int i = 1; i < N; ++i) s += x[i];
    if (s == 123.0f) out[threadIdx.x] = s;
}

int main() {
    float *out;
    hipMalloc(&out, 4096);
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 20000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int waves_per_simd : {1, 2, 4, 8}) {
        dim3 grid(ncu * waves_per_simd), block(256);
        for (int rep = 0; rep < 2; ++rep) {
            float ms_pk = 0, ms_sc = 0;
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_pk<8>, grid, block, 0, 0, out, 1.0000001f, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms_pk, e0, e1);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_sc<16>, grid, block, 0, 0, out, 1.0000001f, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms_sc, e0, e1);
            // element-ops: per thread iters * 2 ops * 16 elements
            const double elem = (double)grid.x * 256 * iters * 2 * 16;
            const double simd_s = (double)ncu * 4;
            if (rep)
                printf("waves/SIMD %d: packed %.3f ms (%.1f elem-op/ns/SIMD), plain %.3f ms (%.1f)\n",
                       waves_per_simd, ms_pk, elem / (ms_pk * 1e6) / simd_s, ms_sc,
                       elem / (ms_sc * 1e6) / simd_s);
        }
    }
    return 0;
}
