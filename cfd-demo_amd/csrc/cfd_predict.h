// cfd_predict.h — the reference's u / v predictor face arithmetic, shared by
// the predictor kernels (cfd_kernels.hip) and the fused predictor/divergence
// march (cfd_predict_march.hip).  Each helper takes a stencil accessor A
// (A.U(di, dj), A.V(di, dj)): global memory (GAcc) or registers, so every
// kernel evaluates the same expressions in the same order, bit for bit.
#pragma once
#include "cfd_device.h"

namespace cfd {
namespace {

// Stencil access for the predictors: U(di, dj) / V(di, dj) are the u / v
// values at flat offset (di, dj) from the cell — flat row-major indexing, so
// the reference's wrap-around reads across row ends (U(nx+1, j) == U(0, j+1))
// come out as they do in model.rs.
struct GAcc {
    const float *u, *v;
    long c, cv;
    int W, nx;
    __device__ __forceinline__ float U(int di, int dj) const { return u[c + di + (long)dj * W]; }
    __device__ __forceinline__ float V(int di, int dj) const { return v[cv + di + (long)dj * nx]; }
};

// ---------------------------------------------------------- u predictor (K1)

// u* on global rows 1..=ny-2, faces 1..=nx (model.rs:538-580 + compute_ustar
// :382-436).  One thread per face; neighbour reuse comes from L1/L2.  Flux
// velocities are the raw v values (get_v_north/south :1056-1069).
// INT: the caller guarantees an interior face (3 <= i <= nx-2, 2 <= j <=
// ny-3), where every column / row test of the second-order faces holds.
template <int SCHEME, int SP, bool INT = false, class A>
__device__ __forceinline__ float u_pred_val(const Geom &g, const Fields &f, float dt,
                                            int i, int lj, const A &a) {
    const int nx = g.nx, ny = g.ny, W = nx + 1;
    const int j = g.j0 + lj;
    const float uc = a.U(0, 0), ue1 = a.U(1, 0), uw1 = a.U(-1, 0), un1 = a.U(0, 1), us1 = a.U(0, -1);
    const float vn = a.V(0, 1), vs = a.V(0, 0);
    float ue, uw, un, us;
    if (SCHEME == 0) {
        // u_face_{e,w,n,s}_first_order (:893-908, :929-941, :966-981, :1011-1026)
        ue = ((uc + ue1) * 0.5f >= 0.0f) ? uc : ue1;
        uw = ((uw1 + uc) * 0.5f >= 0.0f) ? uw1 : uc;
        un = (vn >= 0.0f) ? uc : un1;
        us = (vs >= 0.0f) ? us1 : uc;
    } else {
        // The reference's bounds checks on flat indices reduce, over the faces
        // it predicts (1 <= i <= nx, 1 <= j <= ny-2, pitch W = nx+1, length
        // W*ny), to plain row / column tests:
        //   (i+1) + j*W + 1 < W*ny  <=>  i+2 < W*(ny-j), true as ny-j >= 2;
        //   i + (j+2)*W < W*ny      <=>  i < W*(ny-j-2)  <=>  j < ny-2.
        // Every candidate is formed and the upwind decision selects one
        // (same values as the reference's if / else chains; selects instead
        // of divergent branches).
        // u_face_e_second_order (:911-926)
        const float ue_p = (INT || i > 1) ? 1.5f * uc - 0.5f * a.U(-1, 0) : uc;
        const float ue_m = (INT || i < nx - 1) ? 1.5f * ue1 - 0.5f * a.U(2, 0) : ue1;
        ue = (uc >= 0.0f) ? ue_p : ue_m;
        // u_face_w_second_order (:944-963)
        const float uw_p = (INT || i > 2) ? 1.5f * uw1 - 0.5f * a.U(-2, 0) : uw1;
        const float uw_m = (INT || i < nx) ? 1.5f * uc - 0.5f * ue1 : uc;
        uw = (uw1 >= 0.0f) ? uw_p : uw_m;
        // u_face_n_second_order (:992-1008), decision on averaged v (:983-989)
        const float vnb = 0.5f * (a.V(-1, 1) + a.V(0, 1));
        const float un_p = (INT || j > 1) ? 1.5f * uc - 0.5f * us1 : uc;
        const float un_m = (INT || j < ny - 2) ? 1.5f * un1 - 0.5f * a.U(0, 2) : un1;
        un = (vnb >= 0.0f) ? un_p : un_m;
        // u_face_s_second_order (:1037-1053), decision on averaged v (:1028-1034)
        const float vsb = 0.5f * (a.V(-1, 0) + a.V(0, 0));
        const float us_p = (INT || j > 1) ? 1.5f * us1 - 0.5f * a.U(0, -2) : us1;
        const float us_m = (INT || j < ny) ? 1.5f * uc - 0.5f * un1 : uc;
        us = (vsb >= 0.0f) ? us_p : us_m;
    }
    const float dx = g.dx, dy = g.dy, nu = g.nu;
    const float f_e = ue * ue;
    const float f_w = uw * uw;
    const float f_n = vn * un;
    const float f_s = vs * us;
    const float convective = sdiv<SP>(f_e - f_w, dx, g.r_dx) + sdiv<SP>(f_n - f_s, dy, g.r_dy);
    const float laplace = sdiv<SP>(ue1 - 2.0f * uc + uw1, dx * dx, g.r_dxx) +
                          sdiv<SP>(un1 - 2.0f * uc + us1, dy * dy, g.r_dyy);
    float r = uc + dt * (-convective + nu * laplace);
    if (f.any_pmask && (f.mask_u[(long)lj * W + i] & 1)) r = 0.0f;
    return r;
}

// ---------------------------------------------------------- v predictor (K2)

// v* on global rows 1..=ny-1, columns 1..=nx-1 (model.rs:586-670 +
// compute_vstar :439-521).  Advecting u is the raw face value U(i+1,j),
// U(i,j).  SecondOrder: the lane of column nx-1 is never filled (:647-650),
// so all six inputs are 0.0 there.
// INT: interior face (2 <= i <= nx-3, 2 <= j <= ny-2): every column / row test
// of the second-order faces holds.
template <int SCHEME, int SP, bool INT = false, class A>
__device__ __forceinline__ float v_pred_val(const Geom &g, const Fields &f, float dt,
                                            int i, int lj, const A &a) {
    const int nx = g.nx, ny = g.ny;
    const int j = g.j0 + lj;
    const long cv = (long)lj * nx + i;
    const float vc = a.V(0, 0), ve1 = a.V(1, 0), vw1 = a.V(-1, 0), vn1 = a.V(0, 1), vs1 = a.V(0, -1);
    float uE = a.U(1, 0), uW = a.U(0, 0);
    float ve, vw, vn, vs;
    if (SCHEME == 0) {
        // v_face_{e,w,n,s}_first_order(_scalar) (:1073-1095, :1116-1142, :1163-1185, :1207-1229)
        ve = (uE >= 0.0f) ? vc : ve1;
        vw = (uW >= 0.0f) ? vw1 : vc;
        vn = (0.5f * (vc + vn1) >= 0.0f) ? vc : vn1;
        vs = (0.5f * (vs1 + vc) >= 0.0f) ? vs1 : vc;
    } else if (!INT && i >= nx - 1) {
        uE = 0.0f;
        uW = 0.0f;
        ve = vw = vn = vs = 0.0f;
    } else {
        // Bounds checks on flat indices over the faces predicted here
        // (1 <= i <= nx-2, 1 <= j <= ny-1, length nx*(ny+1)):
        //   i + j*nx + 2 < nx*(ny+1)      <=>  i+2 < nx*(ny+1-j), true;
        //   i + (j+2)*nx < nx*(ny+1)      <=>  j <= ny-2.
        // v_face_e_second_order (:1098-1113)
        const float ve_p = (INT || i > 0) ? 1.5f * vc - 0.5f * vw1 : vc;
        const float ve_m = (INT || i < nx - 2) ? 1.5f * ve1 - 0.5f * a.V(2, 0) : ve1;
        ve = (uE >= 0.0f) ? ve_p : ve_m;
        // v_face_w_second_order (:1145-1160)
        const float vw_p = (INT || i > 1) ? 1.5f * vw1 - 0.5f * a.V(-2, 0) : vw1;
        const float vw_m = (INT || i < nx - 1) ? 1.5f * vc - 0.5f * ve1 : vc;
        vw = (uW >= 0.0f) ? vw_p : vw_m;
        // v_face_n_second_order (:1188-1204)
        const float vn_p = (INT || j > 1) ? 1.5f * vc - 0.5f * vs1 : vc;
        const float vn_m = (INT || j < ny - 1) ? 1.5f * vn1 - 0.5f * a.V(0, 2) : vn1;
        vn = (0.5f * (vc + vn1) >= 0.0f) ? vn_p : vn_m;
        // v_face_s_second_order (:1232-1248)
        const float vs_p = (INT || j > 1) ? 1.5f * vs1 - 0.5f * a.V(0, -2) : vs1;
        const float vs_m = (INT || j < ny) ? 1.5f * vc - 0.5f * vn1 : vc;
        vs = (0.5f * (vs1 + vc) >= 0.0f) ? vs_p : vs_m;
    }
    float r;
    if (f.any_pmask && (f.mask_v[cv] & 1)) {
        r = 0.0f;
    } else {
        const float dx = g.dx, dy = g.dy, nu = g.nu;
        const float f_e = uE * ve;
        const float f_w = uW * vw;
        const float f_n = vn * vn;
        const float f_s = vs * vs;
        const float convective = sdiv<SP>(f_e - f_w, dx, g.r_dx) + sdiv<SP>(f_n - f_s, dy, g.r_dy);
        const float laplace = sdiv<SP>(ve1 - 2.0f * vc + vw1, dx * dx, g.r_dxx) +
                              sdiv<SP>(vn1 - 2.0f * vc + vs1, dy * dy, g.r_dyy);
        r = vc + dt * (-convective + nu * laplace);
    }
    return r;
}

}  // namespace
}  // namespace cfd
