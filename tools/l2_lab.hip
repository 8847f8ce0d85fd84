// Lab: does a line written by plain vector stores stay in the XCD's L2 for a
// later read by the same workgroup? (the block kernel's chains
// miss L2 on bodies their producers wrote microseconds earlier.)
//
// Each workgroup owns a 16 KiB region of a 64 MiB buffer (4,096 workgroups):
//   k_write_read  writes its region with 16-byte stores, barrier, reads it back
//   k_read        reads a region written by an earlier kernel (baseline)
//   k_write       writes only
// Run under `rocprofv3 --pmc FETCH_SIZE`: FETCH_SIZE of k_write_read close to
// k_write's means the read-back hit L2; close to k_write + k_read means it
// missed.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/l2_lab.hip -o tools/l2_lab && tools/l2_lab
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                                          \
    do {                                                                                                               \
        hipError_t e_ = (x);                                                                                           \
        if (e_ != hipSuccess) {                                                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                                  \
            exit(1);                                                                                                   \
        }                                                                                                              \
    } while (0)

constexpr uint32_t kRegion = 16 << 10, kThreads = 256, kIters = kRegion / 16 / kThreads;

__global__ __launch_bounds__(kThreads) void k_write(uint4 *buf, uint32_t seed) {
    uint4 *r = buf + (size_t)blockIdx.x * (kRegion / 16);
    for (uint32_t i = 0; i < kIters; i++) {
        const uint32_t k = i * kThreads + threadIdx.x;
        r[k] = make_uint4(k ^ seed, k + seed, k * seed, blockIdx.x);
    }
}

__global__ __launch_bounds__(kThreads) void k_read(const uint4 *buf, uint32_t *out) {
    const uint4 *r = buf + (size_t)blockIdx.x * (kRegion / 16);
    uint32_t acc = 0;
    for (uint32_t i = 0; i < kIters; i++) {
        const uint4 v = r[i * kThreads + threadIdx.x];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    out[blockIdx.x * kThreads + threadIdx.x] = acc;
}

__global__ __launch_bounds__(kThreads) void k_write_read(uint4 *buf, uint32_t seed, uint32_t *out) {
    uint4 *r = buf + (size_t)blockIdx.x * (kRegion / 16);
    for (uint32_t i = 0; i < kIters; i++) {
        const uint32_t k = i * kThreads + threadIdx.x;
        r[k] = make_uint4(k ^ seed, k + seed, k * seed, blockIdx.x);
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    uint32_t acc = 0;
    for (uint32_t i = 0; i < kIters; i++) { // another thread's lines: not this lane's own stores
        const uint4 v = r[i * kThreads + (threadIdx.x + 64) % kThreads];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    out[blockIdx.x * kThreads + threadIdx.x] = acc;
}

int main() {
    const uint32_t blocks = 4096;
    uint4 *buf;
    uint32_t *out;
    CK(hipMalloc(&buf, (size_t)blocks * kRegion));
    CK(hipMalloc(&out, 4ull * blocks * kThreads));
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k_write, dim3(blocks), dim3(kThreads), 0, 0, buf, 7u + rep);
        hipLaunchKernelGGL(k_read, dim3(blocks), dim3(kThreads), 0, 0, buf, out);
        hipLaunchKernelGGL(k_write_read, dim3(blocks), dim3(kThreads), 0, 0, buf, 11u + rep, out);
        CK(hipDeviceSynchronize());
    }
    printf("{\"region_bytes\": %u, \"workgroups\": %u, \"buffer_bytes\": %llu}\n", kRegion, blocks,
           (unsigned long long)blocks * kRegion);
    return 0;
}
