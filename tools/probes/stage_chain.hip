// Stage-chain probe (gfx950): the Jacobi march's per-slot arithmetic (8
// dependent stages of 2 DPP adds + 9 packed f32 ops on a 3-row register
// window per stage), no memory traffic, at 1-8 waves per SIMD.  Reports the
// VALU instruction rate against the ~4 cycles per wave64 VALU instruction
// measured by valu_rate.hip.  With ILP=2 each wave runs two independent
// marches interleaved.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float from_left(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float from_right(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x130, 0xf, 0xf, true));
}
__device__ __forceinline__ f2 upd(const f2 &B, const f2 &C, const f2 &Tp, const f2 &Rh, float r1, float r2, float r3) {
    const f2 h = {C.y + from_left(C.y), C.x + from_right(C.x)};
    const f2 v = Tp + B;
    const f2 pu = (h * r1 + v * r2 - Rh) * r3;
    return 0.75f * pu + 0.25f * C;
}

template <int T, int ILP>
struct M {
    f2 W[ILP][T][3];
    template <int V>
    __device__ __forceinline__ void slot(const f2 &in, const f2 &rh, float r1, float r2, float r3) {
#pragma unroll
        for (int q = 0; q < ILP; ++q) W[q][0][V % 3] = in + (float)q;
#pragma unroll
        for (int s = 1; s <= T; ++s)
#pragma unroll
            for (int q = 0; q < ILP; ++q) {
                f2 n = upd(W[q][s - 1][(V + 1) % 3], W[q][s - 1][(V + 2) % 3], W[q][s - 1][V % 3], rh, r1, r2, r3);
                if (s < T) W[q][s][V % 3] = n;
                else W[q][0][(V + 1) % 3] += n * 1e-30f;   // keep the last stage live
            }
    }
};

template <int T, int ILP>
__global__ __launch_bounds__(256) void k_chain(float *out, int slots, float r1, float r2, float r3) {
    M<T, ILP> m;
    for (int q = 0; q < ILP; ++q)
        for (int s = 0; s < T; ++s) m.W[q][s][0] = m.W[q][s][1] = m.W[q][s][2] = (f2){(float)threadIdx.x, 1.0f};
    f2 in = {1.0f, 2.0f}, rh = {0.5f, 0.25f};
    for (int k = 0; k < slots; k += 3) {
        m.template slot<0>(in, rh, r1, r2, r3);
        m.template slot<1>(in, rh, r1, r2, r3);
        m.template slot<2>(in, rh, r1, r2, r3);
        in += 1e-7f;
    }
    float s = 0;
    for (int q = 0; q < ILP; ++q)
        for (int t = 0; t < T; ++t) s += m.W[q][t][0].x + m.W[q][t][1].y;
    if (s == 1234.5f) out[threadIdx.x] = s;
}

template <int ILP>
void run(float *out, int ncu) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int slots = 3000;
    for (int wps : {1, 2, 3, 4, 6, 8}) {
        dim3 grid(ncu * wps), block(256);
        float ms = 0;
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL((k_chain<8, ILP>), grid, block, 0, 0, out, slots, 16777216.f, 16777216.f, 1.49e-8f);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
        }
        // VALU instructions per wave: slots * 8 stages * ILP * 11
        const double instr = (double)slots * 8 * ILP * 11 * wps;   // per SIMD
        printf("ILP %d waves/SIMD %d: %.3f ms, %.2f VALU instr/ns/SIMD (4-cycle issue at 2.3 GHz = 0.575)\n",
               ILP, wps, ms, instr / (ms * 1e6));
    }
}

int main() {
    float *out;
    (void)hipMalloc(&out, 4096);
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    run<1>(out, ncu);
    run<2>(out, ncu);
    return 0;
}
