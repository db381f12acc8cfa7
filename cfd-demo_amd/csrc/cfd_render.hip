// cfd_render.hip — device-side snapshot derivation:
// the reference's only consumer of the solver state is App::update_simulation_view
// (src/app.rs:235-403), which copies u, v, p to the host every frame and there
// derives a scalar field (pressure, cell-centred velocity magnitude or
// vorticity), its min/max and an RGB colour ramp with the obstacle overlaid.
// Here all of it runs on the device and only the nx*ny RGBA8 image (or the
// derived f32 field) crosses PCIe.
//
// Arithmetic follows app.rs operation for operation (f32, no contraction,
// correctly rounded sqrt and division); `as u8` is Rust's saturating cast
// (NaN -> 0).  Min/max ignore NaN like the reference's `<` / `>` scans; they
// are reduced as order-preserving u32 keys (exact, order-independent).
#include "cfd_device.h"

namespace cfd {
namespace {

__device__ __forceinline__ uint32_t ord_key(float x) {   // f32 order -> u32 order
    const uint32_t b = __float_as_uint(x);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
    return v;
}

// Rust `f as u8`: saturating, NaN -> 0, truncation toward zero.
__device__ __forceinline__ uint32_t sat_u8(float x) {
    if (!(x > 0.0f)) return 0u;          // NaN, -0, negatives
    if (x >= 255.0f) return 255u;
    return (uint32_t)(int)x;
}

// Derived field of local row lj, column i (app.rs:290-303 velocity, :330-349 vorticity).
template <int MODE>
__device__ __forceinline__ float derive(const Geom &g, const Fields &f, int i, int lj) {
    const int nx = g.nx;
    const long W = nx + 1;
    if (MODE == CFD_VIS_PRESSURE) return f.p[(long)lj * nx + i];
    if (MODE == CFD_VIS_VELOCITY) {
        const float u_left = f.u[i + lj * W];
        const float u_right = f.u[i + 1 + lj * W];
        const float u_cell = 0.5f * (u_left + u_right);
        const float v_bottom = f.v[i + (long)lj * nx];
        const float v_top = f.v[i + (long)(lj + 1) * nx];
        const float v_cell = 0.5f * (v_bottom + v_top);
        return __builtin_sqrtf(u_cell * u_cell + v_cell * v_cell);
    }
    // vorticity: interior cells j in 1..ny-1, i in 1..nx-1 (exclusive), else 0
    const int j = g.j0 + lj;
    if (j < 1 || j > g.ny - 2 || i < 1 || i > nx - 2) return 0.0f;
    const float u_bottom = 0.5f * (f.u[i + lj * W] + f.u[i + 1 + lj * W]);
    const float u_top = 0.5f * (f.u[i + (lj + 1) * W] + f.u[i + 1 + (lj + 1) * W]);
    const float du_dy = (u_top - u_bottom) / g.dy;
    const float v_left = 0.5f * (f.v[i + (long)lj * nx] + f.v[i + (long)(lj + 1) * nx]);
    const float v_right = 0.5f * (f.v[i + 1 + (long)lj * nx] + f.v[i + 1 + (long)(lj + 1) * nx]);
    const float dv_dx = (v_right - v_left) / g.dx;
    return dv_dx - du_dy;
}

// Field (optional output) + its min/max keys, block-reduced, into 2 spread sets.
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_vis_field(Geom g, Fields f, float *out,
                                                      uint32_t *slots) {
    const size_t n = (size_t)g.nx * g.nyl;
    const size_t tid = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    uint32_t kmax = 0u, kmin = 0u;   // max key, max ~key (0 = none seen)
    for (size_t k = tid; k < n; k += stride) {
        const int lj = (int)(k / (size_t)g.nx), i = (int)(k % (size_t)g.nx);
        const float x = derive<MODE>(g, f, i, lj);
        if (out) out[k] = x;
        if (x == x) {
            const uint32_t key = ord_key(x);
            kmax = max(kmax, key);
            kmin = max(kmin, ~key);
        }
    }
    kmax = wave_max_u32(kmax);
    kmin = wave_max_u32(kmin);
    __shared__ uint32_t red[kBlock / 64][2];
    const int wv = (int)threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[wv][0] = kmax;
        red[wv][1] = kmin;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        uint32_t r = 0u;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) r = max(r, red[w][threadIdx.x]);
        if (r) atomicMax(&slots[(size_t)threadIdx.x * kResSlots * kResStride +
                                (blockIdx.x & (kResSlots - 1)) * kResStride], r);
    }
}

__device__ __forceinline__ float key_max(uint32_t k) {   // -inf when nothing was seen
    if (!k) return -__builtin_inff();
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}
__device__ __forceinline__ float key_min(uint32_t nk) {  // +inf when nothing was seen
    if (!nk) return __builtin_inff();
    const uint32_t k = ~nk;
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// Colour ramp + obstacle overlay (app.rs:257-283 and the identical blocks of
// the other two modes).  RGBA8 in memory order r, g, b, a (egui Color32).
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_vis_color(Geom g, Fields f, const float *field,
                                                      uint32_t *px, const uint32_t *keys,
                                                      int has_cyl, float cx, float cy,
                                                      float radius) {
    const size_t n = (size_t)g.nx * g.nyl;
    const size_t tid = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const float min_val = key_min(keys[1]);
    float max_val = key_max(keys[0]);
    if (fabsf(max_val - min_val) < 1e-6f) max_val = min_val + 1.0f;
    const float range = max_val - min_val;
    for (size_t k = tid; k < n; k += stride) {
        const int lj = (int)(k / (size_t)g.nx), i = (int)(k % (size_t)g.nx);
        const float val = field ? field[k] : derive<MODE>(g, f, i, lj);
        const float norm = (val - min_val) / range;
        uint32_t p = sat_u8(norm * 255.0f) | (sat_u8((1.0f - norm) * 255.0f) << 16) | 0xFF000000u;
        if (has_cyl) {
            const float x = ((float)i + 0.5f) * g.dx;
            const float y = ((float)(g.j0 + lj) + 0.5f) * g.dy;
            const float ddx = x - cx, ddy = y - cy;
            if (__builtin_sqrtf(ddx * ddx + ddy * ddy) <= radius) p = 0xFF808080u;
        }
        px[k] = p;
    }
}

inline int vis_grid(size_t n) {
    size_t b = (n + kBlock - 1) / kBlock;
    return (int)(b < 4096 ? (b ? b : 1) : 4096);
}

}  // namespace

void launch_vis_field(const Geom &g, const Fields &f, int mode, float *out, uint32_t *slots,
                      hipStream_t s) {
    const int G = vis_grid((size_t)g.nx * g.nyl);
    if (mode == CFD_VIS_PRESSURE)
        hipLaunchKernelGGL(k_vis_field<CFD_VIS_PRESSURE>, dim3(G), dim3(kBlock), 0, s, g, f, out, slots);
    else if (mode == CFD_VIS_VELOCITY)
        hipLaunchKernelGGL(k_vis_field<CFD_VIS_VELOCITY>, dim3(G), dim3(kBlock), 0, s, g, f, out, slots);
    else
        hipLaunchKernelGGL(k_vis_field<CFD_VIS_VORTICITY>, dim3(G), dim3(kBlock), 0, s, g, f, out, slots);
}

void launch_vis_color(const Geom &g, const Fields &f, int mode, const float *field, uint32_t *px,
                      const uint32_t *keys, int has_cyl, float cx, float cy, float radius,
                      hipStream_t s) {
    const int G = vis_grid((size_t)g.nx * g.nyl);
    if (mode == CFD_VIS_PRESSURE)
        hipLaunchKernelGGL(k_vis_color<CFD_VIS_PRESSURE>, dim3(G), dim3(kBlock), 0, s, g, f, field,
                           px, keys, has_cyl, cx, cy, radius);
    else if (mode == CFD_VIS_VELOCITY)
        hipLaunchKernelGGL(k_vis_color<CFD_VIS_VELOCITY>, dim3(G), dim3(kBlock), 0, s, g, f, field,
                           px, keys, has_cyl, cx, cy, radius);
    else
        hipLaunchKernelGGL(k_vis_color<CFD_VIS_VORTICITY>, dim3(G), dim3(kBlock), 0, s, g, f, field,
                           px, keys, has_cyl, cx, cy, radius);
}

}  // namespace cfd
