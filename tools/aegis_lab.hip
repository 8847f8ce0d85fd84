// aegis_lab.hip — microbenchmark of the AEGIS-128L chain (tools only, not the
// product path). Instantiates the production aegis_mac32 loop with different
// per-update step policies, times them on N 1-MiB messages with hipEvents and
// checks every variant's tags against the production step.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include aegis_lab.hip -o aegis_lab
#include "../tigerbeetle_amd/csrc/aegis.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace tbc {

// Table reads issued first; the round key (ds_bpermute) after them and
// folded in last.
struct StepLateKey {
    __device__ static __forceinline__ uint32_t step(const uint32_t *sT, const TableBase &tb, uint32_t key_src,
                                                    uint32_t x, uint32_t m) {
        const uint32_t a0 = __builtin_amdgcn_perm(x, tb.lo, 0x03020400u);
        const uint32_t a1 = __builtin_amdgcn_perm(x, tb.lo, 0x03020500u);
        const uint32_t a2 = __builtin_amdgcn_perm(x, tb.hi, 0x03020600u);
        const uint32_t a3 = __builtin_amdgcn_perm(x, tb.hi, 0x03020700u);
        const uint32_t t0 = lds_u32(sT, a0);
        const uint32_t t1 = lds_u32(sT, a1 + 128);
        const uint32_t t2 = lds_u32(sT, a2);
        const uint32_t t3 = lds_u32(sT, a3 + 128);
        const uint32_t key = bpermute(key_src, x);
        uint32_t r = t0 ^ m;
        r ^= quad_perm<1, 2, 3, 0>(t1);
        r ^= quad_perm<2, 3, 0, 1>(t2);
        r ^= quad_perm<3, 0, 1, 2>(t3);
        return r ^ key;
    }
};

// One message per 32-lane group; `per_wave` = 2 (production) or 1 (upper
// half duplicates the lower half's message).
template <class Step>
__global__ __launch_bounds__(1024) void k_lab(const uint8_t *base, uint32_t len, uint32_t count, uint32_t per_wave,
                                              uint8_t *out) {
    __shared__ uint32_t sT[kTableDwords];
    load_tables(sT);
    __syncthreads();
    const uint32_t wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint32_t half = (threadIdx.x >> 5) & 1;
    const uint32_t first = wave * per_wave;
    if (first >= count) return;
    uint32_t id = first + (per_wave == 2 ? half : 0);
    if (id >= count) id = count - 1;
    GlobalMsg m(base + ((size_t)id << 20), len);
    const uint32_t tag = aegis_mac32<GlobalMsg, Step>(sT, m);
    const uint32_t g = threadIdx.x & 31;
    if (g < 4 && (per_wave == 2 || half == 0)) gst<uint32_t>(out + 16 * (size_t)id + 4 * g, tag);
}

__global__ void k_fill(uint32_t *p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 0x9E3779B9u ^ seed;
        x ^= x >> 16;
        x *= 0x7feb352dU;
        x ^= x >> 15;
        x *= 0x846ca68bU;
        x ^= x >> 16;
        p[i] = x;
    }
}

} // namespace tbc

using namespace tbc;

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

template <class Step>
static float run(const char *name, const uint8_t *d_msgs, uint32_t count, uint32_t per_wave, uint8_t *d_out,
                 uint32_t len) {
    const uint32_t waves = (count + per_wave - 1) / per_wave;
    uint32_t wpb = (waves + 255) / 256;
    wpb = wpb < 1 ? 1 : (wpb > 16 ? 16 : wpb);
    const uint32_t blocks = (waves + wpb - 1) / wpb;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_lab<Step>, dim3(blocks), dim3(64 * wpb), 0, 0, d_msgs, len, count, per_wave, d_out);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 3; r++) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_lab<Step>, dim3(blocks), dim3(64 * wpb), 0, 0, d_msgs, len, count, per_wave, d_out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
    }
    const double updates = (len + 31) / 32 + 7;
    printf("%-16s count=%5u per_wave=%u waves=%5u wg=%4u x %2u  %8.3f ms  %6.1f ns/update  %7.1f GB/s\n", name,
           count, per_wave, waves, blocks, wpb, best, best * 1e6 / updates, (double)count * len / best / 1e6);
    fflush(stdout);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return best;
}

int main(int argc, char **argv) {
    const uint32_t nmax = argc > 1 ? (uint32_t)atoi(argv[1]) : 2072;
    const uint32_t len = 1048320; // one 1 MiB data block body (constants.zig:500)
    uint8_t *d_msgs, *d_out, *d_ref;
    CK(hipMalloc(&d_msgs, (size_t)nmax << 20));
    CK(hipMalloc(&d_out, 16ull * nmax));
    CK(hipMalloc(&d_ref, 16ull * nmax));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint32_t *)d_msgs, ((size_t)nmax << 20) / 4, 7u);
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> h_ref(16ull * nmax), h_out(16ull * nmax);
    const uint32_t counts[] = {2, 64, 2016, nmax};
    int bad = 0;
    for (uint32_t count : counts) {
        if (count > nmax) continue;
        run<StepBpermute>("bpermute", d_msgs, count, 2, d_ref, len);
        CK(hipMemcpy(h_ref.data(), d_ref, 16ull * count, hipMemcpyDeviceToHost));
        auto check = [&](const char *what) {
            CK(hipMemcpy(h_out.data(), d_out, 16ull * count, hipMemcpyDeviceToHost));
            if (memcmp(h_out.data(), h_ref.data(), 16ull * count)) {
                printf("  MISMATCH %s\n", what);
                bad++;
            }
        };
        CK(hipMemset(d_out, 0, 16ull * count));
        run<StepBpermute>("bpermute/1", d_msgs, count, 1, d_out, len);
        check("bpermute/1");
        CK(hipMemset(d_out, 0, 16ull * count));
        run<StepLateKey>("late-key", d_msgs, count, 2, d_out, len);
        check("late-key");
        CK(hipMemset(d_out, 0, 16ull * count));
        run<StepValuKey>("valu-key", d_msgs, count, 2, d_out, len);
        check("valu-key");

    }
    printf(bad ? "LAB FAILED (%d mismatches)\n" : "LAB OK\n", bad);
    return bad ? 1 : 0;
}
