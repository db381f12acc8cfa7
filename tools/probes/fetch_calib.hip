// FETCH_SIZE / WRITE_SIZE calibration probe (gfx950), MI355X_MICROARCH.md
// §HBM: "other access widths are uncalibrated: calibrate on a known byte count
// in your own access pattern".  Each kernel streams a known number of bytes
// with one access form the product kernels use:
//   k_rd_buf32 / k_rd_buf64 / k_rd_buf128  raw_buffer_load_b32/b64/b128 (the
//        Jacobi marches: kind 5 reads p' and rhs with b64, k_jacobi with b128)
//   k_rd_flat64 / k_rd_flat128             global (flat) float2 / float4 loads
//        (the predictor march, the corrector finish)
//   k_wr_buf64 / k_wr_flat128              b64 buffer stores / float4 stores
// over a 1 GiB buffer (4x the Infinity Cache: the reads reach HBM), one
// dispatch each, row-major coalesced like the marches (a wave covers a
// contiguous 64-lane span).  Run under rocprofv3 --pmc FETCH_SIZE and, in a
// separate pass, --pmc WRITE_SIZE; tools/pmc_calib.py divides the known bytes
// by the counters.  Diagnostic only (not part of the product).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, bytes, 0x00020000);
}

// Every kernel: grid-stride over `n` elements of W bytes; the sum goes to
// out[] only if it equals a sentinel, so the loads are never dead.
__global__ __launch_bounds__(kBlock) void k_rd_buf32(const float *p, size_t n, unsigned *out) {
    const __amdgpu_buffer_rsrc_t rs = rsrc(p, 0xFFFFFFFFu);
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
        acc += __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(i * 4), 0, 0);
    if (acc == 0x9E3779B9u) out[threadIdx.x] = acc;
}
__global__ __launch_bounds__(kBlock) void k_rd_buf64(const float *p, size_t n, unsigned *out) {
    const __amdgpu_buffer_rsrc_t rs = rsrc(p, 0xFFFFFFFFu);
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
        const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(i * 8), 0, 0);
        acc += v.x ^ v.y;
    }
    if (acc == 0x9E3779B9u) out[threadIdx.x] = acc;
}
__global__ __launch_bounds__(kBlock) void k_rd_buf128(const float *p, size_t n, unsigned *out) {
    const __amdgpu_buffer_rsrc_t rs = rsrc(p, 0xFFFFFFFFu);
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(i * 16), 0, 0);
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) out[threadIdx.x] = acc;
}
__global__ __launch_bounds__(kBlock) void k_rd_flat64(const float2 *p, size_t n, unsigned *out) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
        const float2 v = p[i];
        acc += v.x + v.y;
    }
    if (acc == 123.25f) out[threadIdx.x] = 1u;
}
__global__ __launch_bounds__(kBlock) void k_rd_flat128(const float4 *p, size_t n, unsigned *out) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
        const float4 v = p[i];
        acc += (v.x + v.y) + (v.z + v.w);
    }
    if (acc == 123.25f) out[threadIdx.x] = 1u;
}
__global__ __launch_bounds__(kBlock) void k_wr_buf64(float *p, size_t n) {
    const __amdgpu_buffer_rsrc_t rs = rsrc(p, 0xFFFFFFFFu);
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
        const u32x2 v = {(unsigned)i, (unsigned)(i >> 1)};
        __builtin_amdgcn_raw_buffer_store_b64(v, rs, (int)(i * 8), 0, 0);
    }
}
__global__ __launch_bounds__(kBlock) void k_wr_flat128(float4 *p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
        p[i] = make_float4((float)i, 1.f, 2.f, 3.f);
}

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

int main() {
    // 1 GiB - 64 KiB: buffer offsets (int) stay below 2^31 for every width
    const size_t bytes = (1ull << 30) - (1ull << 16);
    float *buf = nullptr;
    unsigned *out = nullptr;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&out, kBlock * 4));
    CHECK(hipMemset(buf, 0, bytes));
    CHECK(hipDeviceSynchronize());
    const dim3 grid(256 * 16), block(kBlock);
    // one warm-up pass of every kernel (first-launch code loads), then the
    // measured dispatch; the PMC summary averages per kernel over both, so
    // the printed bytes are per dispatch
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_rd_buf32, grid, block, 0, 0, buf, bytes / 4, out);
        hipLaunchKernelGGL(k_rd_buf64, grid, block, 0, 0, buf, bytes / 8, out);
        hipLaunchKernelGGL(k_rd_buf128, grid, block, 0, 0, buf, bytes / 16, out);
        hipLaunchKernelGGL(k_rd_flat64, grid, block, 0, 0, (const float2 *)buf, bytes / 8, out);
        hipLaunchKernelGGL(k_rd_flat128, grid, block, 0, 0, (const float4 *)buf, bytes / 16, out);
        hipLaunchKernelGGL(k_wr_buf64, grid, block, 0, 0, buf, bytes / 8);
        hipLaunchKernelGGL(k_wr_flat128, grid, block, 0, 0, (float4 *)buf, bytes / 16);
        CHECK(hipDeviceSynchronize());
    }
    CHECK(hipGetLastError());
    printf("{\"bytes_per_dispatch\": %zu, \"kernels\": [\"k_rd_buf32\", \"k_rd_buf64\", "
           "\"k_rd_buf128\", \"k_rd_flat64\", \"k_rd_flat128\", \"k_wr_buf64\", \"k_wr_flat128\"]}\n",
           bytes);
    CHECK(hipFree(buf));
    CHECK(hipFree(out));
    return 0;
}
