// Where does the dispatcher put the waves of a workgroup?  (r6 store-wave
// study.)  Each workgroup of NW waves holds the LDS of the Jacobi march
// (18 KiB static + the 24 KiB pad) and each wave VGPRS registers (forced by a
// clobber), spins ~SPIN_US and records its HW_ID / XCC_ID and start / end
// (s_memrealtime, 100 MHz).  The host reports per configuration: workgroups
// resident per CU at once, waves per SIMD at once, and the SIMD of wave k
// relative to wave 0.
//   hipcc --offload-arch=gfx950 -O2 wave_place.hip -o wave_place && ./wave_place
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            return 1;                                                             \
        }                                                                         \
    } while (0)

struct Rec {
    unsigned hw, xcc;
    unsigned long long t0, t1;
};

template <int NW, int VG>
__global__ __launch_bounds__(NW * 64) void k_place(Rec *out, int spin_ticks) {
    __shared__ float lds[18432 / 4];
    extern __shared__ float pad[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    lds[threadIdx.x] = (float)t0;
    if (VG == 104) asm volatile("" ::: "v103");
    if (VG == 96) asm volatile("" ::: "v95");
    unsigned long long t = t0;
    while (t - t0 < (unsigned long long)spin_ticks) {
        __builtin_amdgcn_s_sleep(2);
        t = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    if (lane == 0) {
        Rec r;
        r.hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
        r.xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));
        r.t0 = t0;
        r.t1 = t;
        out[blockIdx.x * NW + wave] = r;   // vector store
        pad[0] = lds[(threadIdx.x + 64) % (NW * 64)];
    }
}

template <int NW, int VG>
int run(const char *name, int nwg, int spin_us, int pad_bytes = 24576) {
    Rec *d;
    CHECK(hipMalloc(&d, sizeof(Rec) * nwg * NW));
    CHECK(hipMemset(d, 0, sizeof(Rec) * nwg * NW));
    hipLaunchKernelGGL((k_place<NW, VG>), dim3(nwg), dim3(NW * 64), pad_bytes, 0, d, spin_us * 100);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    std::vector<Rec> h(nwg * NW);
    CHECK(hipMemcpy(h.data(), d, sizeof(Rec) * h.size(), hipMemcpyDeviceToHost));
    CHECK(hipFree(d));
    // CU key: xcc, se, sh, cu
    auto cu_of = [](const Rec &r) {
        return (int)((r.xcc & 15) << 8 | ((r.hw >> 13) & 7) << 5 | ((r.hw >> 12) & 1) << 4 | ((r.hw >> 8) & 15));
    };
    auto simd_of = [](const Rec &r) { return (int)((r.hw >> 4) & 3); };
    // concurrency: at the midpoint of each wave's life, count the waves of its
    // CU / SIMD alive at that time
    std::map<int, std::vector<int>> by_cu;   // CU -> wave indices
    for (int i = 0; i < (int)h.size(); ++i) by_cu[cu_of(h[i])].push_back(i);
    std::map<int, int> wg_hist, simd_hist, rel[NW];
    std::map<int, int> prod_simd_hist;   // NW=5: waves 0..3 per SIMD at once
    for (auto &kv : by_cu) {
        const auto &v = kv.second;
        for (int i : v) {
            if (i % NW) continue;   // one sample per workgroup (its wave 0)
            const unsigned long long tm = (h[i].t0 + h[i].t1) / 2;
            std::map<int, int> wgs;
            int sw[4] = {0, 0, 0, 0}, sp[4] = {0, 0, 0, 0};
            for (int j : v)
                if (h[j].t0 <= tm && h[j].t1 >= tm) {
                    wgs[j / NW] = 1;
                    ++sw[simd_of(h[j])];
                    if (j % NW < NW - 1 || NW == 4) ++sp[simd_of(h[j])];
                }
            ++wg_hist[(int)wgs.size()];
            for (int s = 0; s < 4; ++s) {
                ++simd_hist[sw[s]];
                ++prod_simd_hist[sp[s]];
            }
        }
    }
    for (int i = 0; i < (int)h.size(); ++i) {
        const int w0 = i - i % NW;
        ++rel[i % NW][(simd_of(h[i]) - simd_of(h[w0]) + 4) % 4];
    }
    int cus = (int)by_cu.size();
    printf("{\"config\": \"%s\", \"workgroups\": %d, \"waves_per_wg\": %d, \"cus_seen\": %d, ", name, nwg, NW, cus);
    printf("\"wgs_per_cu_at_once\": {");
    bool first = true;
    for (auto &kv : wg_hist) printf("%s\"%d\": %d", first ? "" : ", ", kv.first, kv.second), first = false;
    printf("}, \"waves_per_simd_at_once\": {");
    first = true;
    for (auto &kv : simd_hist) printf("%s\"%d\": %d", first ? "" : ", ", kv.first, kv.second), first = false;
    printf("}, \"all_but_last_wave_per_simd\": {");
    first = true;
    for (auto &kv : prod_simd_hist) printf("%s\"%d\": %d", first ? "" : ", ", kv.first, kv.second), first = false;
    printf("}, \"simd_of_wave_k_minus_wave0\": [");
    for (int k = 0; k < NW; ++k) {
        printf("%s[", k ? ", " : "");
        for (int s = 0; s < 4; ++s) printf("%s%d", s ? ", " : "", rel[k].count(s) ? rel[k][s] : 0);
        printf("]");
    }
    unsigned long long lo = ~0ull, hi = 0;
    for (auto &r : h) lo = std::min(lo, r.t0), hi = std::max(hi, r.t1);
    printf("], \"span_us\": %.1f}\n", (hi - lo) / 100.0);
    return 0;
}

int main() {
    // 768 = 3 workgroups on each of 256 CUs, 1024 = 4
    if (run<4, 104>("4 waves, 104 VGPRs (the march today)", 768, 40)) return 1;
    if (run<5, 104>("5 waves, 104 VGPRs (march + store wave)", 768, 40)) return 1;
    if (run<5, 96>("5 waves, 96 VGPRs", 768, 40)) return 1;
    if (run<4, 104>("4 waves, 104 VGPRs, 1024 workgroups, 8 KiB pad (3 march + store wave)", 1024, 40, 8192)) return 1;
    return 0;
}
