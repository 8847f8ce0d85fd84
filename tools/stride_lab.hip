// Lab: what a key read costs when the key is 8 bytes of a 128-byte value
// (config 5's Account timestamps, config 1's object trees). Reads one key
// per record at a given offset over a 4 GiB table and compares the time with
// a full streaming read of the same table: if HBM delivers only the sector
// that holds the key, a key-only merge reads a fraction of R.
//
//   hipcc --offload-arch=gfx950 -O3 tools/stride_lab.hip -o tools/stride_lab
//   tools/stride_lab            (prints one JSON line)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Full streaming read: 16 B per lane, 8 loads in flight per lane.
__global__ __launch_bounds__(256) void k_stream(const u32x4 *p, size_t n16, uint32_t *out) {
    uint32_t acc = 0;
    const size_t stride = (size_t)gridDim.x * 256 * 8;
    for (size_t i = (size_t)blockIdx.x * 256 * 8 + threadIdx.x; i < n16; i += stride) {
        u32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = i + 256 * u < n16 ? p[i + 256 * u] : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < 8; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// One W-byte key per R-byte record at byte offset OFF, 8 records per lane in
// flight (lane-consecutive records).
template <int W>
__global__ __launch_bounds__(256) void k_keys(const uint8_t *p, size_t nrec, uint32_t rec, uint32_t off,
                                               uint32_t *out) {
    uint32_t acc = 0;
    const size_t stride = (size_t)gridDim.x * 256 * 8;
    for (size_t i = (size_t)blockIdx.x * 256 * 8 + threadIdx.x; i < nrec; i += stride) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const size_t r = i + 256 * u;
            if (r < nrec) {
                const uint8_t *q = p + r * rec + off;
                if (W == 8) {
                    const uint64_t k = *(const uint64_t *)q;
                    v[u] = (uint32_t)k ^ (uint32_t)(k >> 32);
                } else if (W == 16) {
                    const u32x4 k = *(const u32x4 *)q;
                    v[u] = k.x ^ k.y ^ k.z ^ k.w;
                } else {
                    v[u] = *(const uint32_t *)q;
                }
            } else {
                v[u] = 0;
            }
        }
#pragma unroll
        for (int u = 0; u < 8; u++) acc ^= v[u];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_fill(uint32_t *p, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (uint32_t)(i * 2654435761u);
}

int main() {
    const size_t bytes = 4ull << 30;
    uint8_t *buf;
    uint32_t *out;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&out, 64));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint32_t *)buf, bytes / 4);
    CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int grid = 256 * 8;
    auto time = [&](auto launch) {
        launch();
        hipDeviceSynchronize();
        float best = 1e9f;
        for (int r = 0; r < 5; r++) {
            hipEventRecord(e0, 0);
            launch();
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        return best;
    };
    printf("{");
    const float ts = time([&] { hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, 0, (const u32x4 *)buf, bytes / 16, out); });
    printf("\"stream_ms\": %.4f, \"stream_TBps\": %.3f", ts, bytes / ts / 1e9);
    struct Case { const char *name; uint32_t rec, off, w; };
    const Case cases[] = {{"k8_rec128_off120", 128, 120, 8}, {"k8_rec128_off0", 128, 0, 8},
                          {"k16_rec128_off0", 128, 0, 16}, {"k8_rec64_off0", 64, 0, 8},
                          {"k16_rec32_off0", 32, 0, 16}, {"k8_rec256_off0", 256, 0, 8},
                          {"k4_rec128_off124", 128, 124, 4}};
    for (const Case &c : cases) {
        const size_t nrec = bytes / c.rec;
        float t;
        if (c.w == 8)
            t = time([&] { hipLaunchKernelGGL(k_keys<8>, dim3(grid), dim3(256), 0, 0, buf, nrec, c.rec, c.off, out); });
        else if (c.w == 16)
            t = time([&] { hipLaunchKernelGGL(k_keys<16>, dim3(grid), dim3(256), 0, 0, buf, nrec, c.rec, c.off, out); });
        else
            t = time([&] { hipLaunchKernelGGL(k_keys<4>, dim3(grid), dim3(256), 0, 0, buf, nrec, c.rec, c.off, out); });
        printf(", \"%s_ms\": %.4f, \"%s_table_TBps\": %.3f", c.name, t, c.name, bytes / t / 1e9);
    }
    printf("}\n");
    CHECK(hipFree(buf));
    return 0;
}
