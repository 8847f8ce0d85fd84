// atomic_probe.hip — what k_sort_pack's end-of-tile histogram flush costs.
// 1,536 workgroups (config 3: 24 tables x 64 tiles), each adds nd x 256
// counters into its table's histogram, as device-scope atomics (k_sort_pack
// today) or as plain stores of a per-tile histogram (the alternative: the
// plan kernel reduces them). Timed with hipEvents over 20 launches each.
// Build: hipcc --offload-arch=gfx950 -O3 tools/atomic_probe.hip -o /tmp/atomic_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr uint32_t kTables = 24, kTilesPerTable = 64, kDigits = 5, kRadix = 256;

__global__ __launch_bounds__(256) void k_flush_atomic(uint32_t *hist) {
    const uint32_t table = blockIdx.x / kTilesPerTable, tid = threadIdx.x;
    uint32_t *h = hist + (size_t)table * kDigits * kRadix;
    for (uint32_t j = 0; j < kDigits; j++) atomicAdd(&h[j * kRadix + tid], (blockIdx.x * 7 + tid + j) & 15);
}

__global__ __launch_bounds__(256) void k_flush_store(uint32_t *tile_hist) {
    const uint32_t tid = threadIdx.x;
    uint32_t *h = tile_hist + (size_t)blockIdx.x * kDigits * kRadix;
    for (uint32_t j = 0; j < kDigits; j++) h[j * kRadix + tid] = (blockIdx.x * 7 + tid + j) & 15;
}

// One workgroup per table, a thread per (digit, pass): the sum over the table's tiles.
__global__ __launch_bounds__(256) void k_reduce(const uint32_t *tile_hist, uint32_t *hist) {
    const uint32_t table = blockIdx.x, tid = threadIdx.x;
    for (uint32_t j = 0; j < kDigits; j++) {
        uint32_t s = 0;
#pragma unroll 16
        for (uint32_t t = 0; t < kTilesPerTable; t++)
            s += tile_hist[((size_t)(table * kTilesPerTable + t) * kDigits + j) * kRadix + tid];
        hist[((size_t)table * kDigits + j) * kRadix + tid] = s;
    }
}

int main() {
    const uint32_t tiles = kTables * kTilesPerTable;
    uint32_t *hist, *tile_hist;
    if (hipMalloc(&hist, sizeof(uint32_t) * kTables * kDigits * kRadix) != hipSuccess ||
        hipMalloc(&tile_hist, sizeof(uint32_t) * tiles * kDigits * kRadix) != hipSuccess)
        return 1;
    hipMemset(hist, 0, sizeof(uint32_t) * kTables * kDigits * kRadix);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int reps = 20;
    float ms[3] = {0, 0, 0};
    for (int pass = 0; pass < 2; pass++) { // pass 0 warms up
        hipEventRecord(a, 0);
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_flush_atomic, dim3(tiles), dim3(256), 0, 0, hist);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms[0], a, b);
        hipEventRecord(a, 0);
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_flush_store, dim3(tiles), dim3(256), 0, 0, tile_hist);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms[1], a, b);
        hipEventRecord(a, 0);
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_reduce, dim3(kTables), dim3(256), 0, 0, tile_hist, hist);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms[2], a, b);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("{\"atomic_flush_us\": %.2f, \"store_flush_us\": %.2f, \"reduce_us\": %.2f, \"atomics\": %u}\n",
           1000 * ms[0] / reps, 1000 * ms[1] / reps, 1000 * ms[2] / reps, tiles * kDigits * kRadix);
    return 0;
}
