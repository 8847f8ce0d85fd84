// sort.hip — TableMemory.sort (src/lsm/table_memory.zig:140-154) on gfx950.
//
// The reference sorts the mutable table's Values with std.mem.sort (Zig 0.11
// stable block sort) by key_from_value, only when puts arrived out of order
// (table_memory.zig:83-87). Stability is load-bearing: fill_immutable_values
// keeps the LAST of a run of equal keys (compaction.zig:519-522).
//
// Here: a stable LSD radix sort of (key limbs, original index) items with
// 4-bit digits, skipping every digit that is constant across the table (one
// probe pass computes OR/AND of all keys and the sortedness flag), then one
// gather of the Values by original index. Per pass:
//   hist    — per-tile digit counts (16 bins x tiles, digit-major);
//   scan    — exclusive scan of the digit-major counts (one workgroup);
//   scatter — each tile is staged through LDS so every thread owns 8
//             consecutive items, per-thread digit counts are scanned across
//             the tile in digit-major order, and items are written to
//             (tile offset of digit) + (rank among earlier same-digit items):
//             stable by construction.
#include <hip/hip_runtime.h>

#include "tbc_internal.h"

namespace tbc {

constexpr uint32_t kSortThreads = 256;
constexpr uint32_t kSortPer = 8;
constexpr uint32_t kSortTile = kSortThreads * kSortPer; // 2048 items per tile
constexpr uint32_t kDigitBits = 4;
constexpr uint32_t kBins = 1u << kDigitBits;

struct SortProbe {
    uint64_t or_[4];
    uint64_t and_[4];
    uint32_t unsorted;
    uint32_t pad[7];
};

__device__ __forceinline__ void key_of(uint32_t kind, const uint8_t *v, uint32_t ts_off, uint64_t k[3]) {
    k[1] = k[2] = 0;
    switch (kind) {
    case kKeyTimestamp: k[0] = gld<uint64_t>(v + ts_off) & ~kTombstoneBit; break;
    case kKeyIdU128: k[0] = gld<uint64_t>(v); k[1] = gld<uint64_t>(v + 8); break;
    case kKeyCompositeU64: k[0] = gld<uint64_t>(v + 8) & ~kTombstoneBit; k[1] = gld<uint64_t>(v); break;
    default: k[0] = gld<uint64_t>(v + 16) & ~kTombstoneBit; k[1] = gld<uint64_t>(v); k[2] = gld<uint64_t>(v + 8); break;
    }
}

// Extract keys (limb-major) and indices; OR/AND of all keys; sortedness.
__global__ __launch_bounds__(256) void k_sort_extract(uint32_t kind, uint32_t kl, const uint8_t *values, uint32_t n,
                                                      uint32_t vs, uint32_t ts_off, uint64_t *keys, uint32_t *idx,
                                                      SortProbe *probe) {
    __shared__ uint64_t s_or[3][4], s_and[3][4];
    __shared__ uint32_t s_uns;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_uns = 0;
    uint64_t o[3] = {0, 0, 0}, a[3] = {~0ull, ~0ull, ~0ull};
    uint32_t uns = 0;
    for (uint32_t i = blockIdx.x * 256 + tid; i < n; i += gridDim.x * 256) {
        uint64_t k[3], kn[3];
        key_of(kind, values + (size_t)i * vs, ts_off, k);
        for (uint32_t l = 0; l < kl; l++) {
            keys[(size_t)l * n + i] = k[l];
            o[l] |= k[l];
            a[l] &= k[l];
        }
        idx[i] = i;
        if (i + 1 < n) {
            key_of(kind, values + (size_t)(i + 1) * vs, ts_off, kn);
            // unsorted iff key[i] > key[i+1]
            bool gt = false, decided = false;
            for (int l = (int)kl - 1; l >= 0 && !decided; l--) {
                if (k[l] != kn[l]) {
                    gt = k[l] > kn[l];
                    decided = true;
                }
            }
            uns |= gt ? 1u : 0u;
        }
    }
    for (uint32_t l = 0; l < 3; l++) {
        for (int off = 32; off > 0; off >>= 1) {
            o[l] |= __shfl_xor(o[l], off, 64);
            a[l] &= __shfl_xor(a[l], off, 64);
        }
        if (lane == 0) {
            s_or[l][wave] = o[l];
            s_and[l][wave] = a[l];
        }
    }
    __syncthreads();
    if (uns) atomicOr(&s_uns, 1u);
    __syncthreads();
    if (tid == 0) {
        for (uint32_t l = 0; l < kl; l++) {
            uint64_t oo = 0, aa = ~0ull;
            for (int w = 0; w < 4; w++) {
                oo |= s_or[l][w];
                aa &= s_and[l][w];
            }
            atomicOr((unsigned long long *)&probe->or_[l], (unsigned long long)oo);
            atomicAnd((unsigned long long *)&probe->and_[l], (unsigned long long)aa);
        }
        if (s_uns) atomicOr(&probe->unsorted, 1u);
    }
}

__device__ __forceinline__ uint32_t digit_of(const uint64_t *keys, uint32_t n, uint32_t limb, uint32_t shift,
                                             uint32_t i) {
    return (uint32_t)(gld<uint64_t>(keys + (size_t)limb * n + i) >> shift) & (kBins - 1);
}

__global__ __launch_bounds__(kSortThreads) void k_sort_hist(const uint64_t *keys, uint32_t n, uint32_t limb,
                                                            uint32_t shift, uint32_t *hist, uint32_t ntiles) {
    __shared__ uint32_t cnt[kBins];
    const uint32_t tid = threadIdx.x;
    if (tid < kBins) cnt[tid] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * kSortTile;
    for (uint32_t r = 0; r < kSortPer; r++) {
        const uint32_t i = base + r * kSortThreads + tid;
        if (i < n) atomicAdd(&cnt[digit_of(keys, n, limb, shift, i)], 1u);
    }
    __syncthreads();
    if (tid < kBins) hist[tid * ntiles + blockIdx.x] = cnt[tid];
}

// Exclusive scan of m entries in place (one workgroup).
__global__ __launch_bounds__(1024) void k_sort_scan(uint32_t *hist, uint32_t m) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (uint32_t base = 0; base < m; base += 1024) {
        const uint32_t i = base + tid;
        const uint32_t v = i < m ? hist[i] : 0;
        uint32_t incl = v;
        for (int o = 1; o < 64; o <<= 1) {
            uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= (uint32_t)o) incl += y;
        }
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        uint32_t woff = 0;
        for (uint32_t w = 0; w < wave; w++) woff += wsum[w];
        const uint32_t c0 = carry;
        if (i < m) hist[i] = c0 + woff + incl - v;
        __syncthreads();
        if (tid == 1023) carry = c0 + woff + incl;
        __syncthreads();
    }
}

template <int KL>
__global__ __launch_bounds__(kSortThreads) void k_sort_scatter(const uint64_t *keys_in, const uint32_t *idx_in,
                                                               uint64_t *keys_out, uint32_t *idx_out, uint32_t n,
                                                               uint32_t limb, uint32_t shift, const uint32_t *hist,
                                                               uint32_t ntiles) {
    __shared__ uint64_t s_key[KL][kSortTile];
    __shared__ uint32_t s_idx[kSortTile];
    __shared__ uint32_t s_cnt[kBins][kSortThreads + 1]; // digit-major per-thread counts
    __shared__ uint32_t s_tot[kBins];
    const uint32_t tid = threadIdx.x;
    const uint32_t base = blockIdx.x * kSortTile;
    const uint32_t m = (n - base) < kSortTile ? (n - base) : kSortTile;
    // Coalesced load into LDS.
    for (uint32_t r = 0; r < kSortPer; r++) {
        const uint32_t e = r * kSortThreads + tid;
        if (e < m) {
#pragma unroll
            for (int l = 0; l < KL; l++) s_key[l][e] = gld<uint64_t>(keys_in + (size_t)l * n + base + e);
            s_idx[e] = gld<uint32_t>(idx_in + base + e);
        }
    }
    __syncthreads();
    // Thread tid owns items [tid*8, tid*8+8) in order.
    uint32_t dig[kSortPer];
    uint32_t c[kBins];
#pragma unroll
    for (uint32_t d = 0; d < kBins; d++) c[d] = 0;
#pragma unroll
    for (uint32_t k = 0; k < kSortPer; k++) {
        const uint32_t e = tid * kSortPer + k;
        dig[k] = e < m ? (uint32_t)(s_key[limb][e] >> shift) & (kBins - 1) : kBins; // kBins = none
#pragma unroll
        for (uint32_t d = 0; d < kBins; d++) c[d] += dig[k] == d ? 1u : 0u;
    }
#pragma unroll
    for (uint32_t d = 0; d < kBins; d++) s_cnt[d][tid] = c[d];
    __syncthreads();
    // Per digit, exclusive scan across threads (one wave per digit group).
    {
        const uint32_t wave = tid >> 6, lane = tid & 63;
        for (uint32_t d = wave; d < kBins; d += kSortThreads / 64) {
            uint32_t carry = 0;
            for (uint32_t b0 = 0; b0 < kSortThreads; b0 += 64) {
                const uint32_t v = s_cnt[d][b0 + lane];
                uint32_t incl = v;
                for (int o = 1; o < 64; o <<= 1) {
                    uint32_t y = __shfl_up(incl, o, 64);
                    if (lane >= (uint32_t)o) incl += y;
                }
                s_cnt[d][b0 + lane] = carry + incl - v;
                carry += __shfl(incl, 63, 64);
            }
            if (lane == 0) s_tot[d] = carry;
        }
    }
    __syncthreads();
    uint32_t run[kBins];
#pragma unroll
    for (uint32_t d = 0; d < kBins; d++) run[d] = hist[d * ntiles + blockIdx.x] + s_cnt[d][tid];
#pragma unroll
    for (uint32_t k = 0; k < kSortPer; k++) {
        const uint32_t e = tid * kSortPer + k;
        if (dig[k] < kBins) {
            uint32_t dst = 0;
#pragma unroll
            for (uint32_t d = 0; d < kBins; d++)
                if (dig[k] == d) dst = run[d]++;
#pragma unroll
            for (int l = 0; l < KL; l++) gst<uint64_t>(keys_out + (size_t)l * n + dst, s_key[l][e]);
            gst<uint32_t>(idx_out + dst, s_idx[e]);
        }
    }
}

// values_out[i] = values_in[idx[i]], 16 bytes per lane.
__global__ __launch_bounds__(256) void k_sort_gather(const uint8_t *values_in, uint8_t *values_out,
                                                     const uint32_t *idx, uint32_t n, uint32_t vs) {
    const uint32_t cpv = vs >> 4;
    const uint64_t chunks = (uint64_t)n * cpv;
    for (uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x; c < chunks; c += (uint64_t)gridDim.x * 256) {
        const uint32_t i = (uint32_t)(c / cpv), part = (uint32_t)(c % cpv);
        const uint32_t src = gld<uint32_t>(idx + i);
        gst<u32x4>(values_out + (size_t)i * vs + 16 * part, gld<u32x4>(values_in + (size_t)src * vs + 16 * part));
    }
}

static uint32_t key_limbs(uint32_t kind) {
    return kind == kKeyTimestamp ? 1 : kind == kKeyCompositeU128 ? 3 : 2;
}

uint64_t sort_scratch_bytes(uint32_t value_size, uint32_t n) {
    const uint64_t ntiles = (n + kSortTile - 1) / kSortTile;
    return 256                                       // probe
           + 2 * ((uint64_t)n * (3 * 8 + 4) + 256)   // two item buffers
           + 4 * kBins * ntiles + 256                // histogram
           + (uint64_t)n * value_size + 256;         // gathered values
}

int launch_sort(uint32_t kind, uint32_t vs, uint32_t ts_off, void *values, uint32_t n, void *scratch,
                uint64_t scratch_bytes, void *stream) {
    if (n < 2) return 0;
    if (scratch_bytes < sort_scratch_bytes(vs, n)) return -1;
    hipStream_t s = (hipStream_t)stream;
    const uint32_t kl = key_limbs(kind);
    const uint32_t ntiles = (n + kSortTile - 1) / kSortTile;
    uint8_t *p = (uint8_t *)scratch;
    SortProbe *probe = (SortProbe *)p;
    p += 256;
    uint64_t *keys[2];
    uint32_t *idx[2];
    for (int b = 0; b < 2; b++) {
        keys[b] = (uint64_t *)p;
        p += (uint64_t)n * 3 * 8;
        idx[b] = (uint32_t *)p;
        p += ((uint64_t)n * 4 + 255) / 256 * 256;
    }
    uint32_t *hist = (uint32_t *)p;
    p += ((uint64_t)4 * kBins * ntiles + 255) / 256 * 256;
    uint8_t *gathered = p;

    SortProbe init{};
    for (int l = 0; l < 4; l++) init.and_[l] = ~0ull;
    if (hipMemcpyAsync(probe, &init, sizeof init, hipMemcpyHostToDevice, s) != hipSuccess) return -1;
    const uint32_t eblocks = (n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048;
    hipLaunchKernelGGL(k_sort_extract, dim3(eblocks), dim3(256), 0, s, kind, kl, (const uint8_t *)values, n, vs,
                       ts_off, keys[0], idx[0], probe);
    // The digit plan needs the probe on the host (one small synchronous read).
    SortProbe host{};
    if (hipMemcpyAsync(&host, probe, sizeof host, hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
    if (hipStreamSynchronize(s) != hipSuccess) return -1;
    if (!host.unsorted) return 0; // table_memory.zig:141: already sorted, no-op
    int cur = 0;
    for (uint32_t limb = 0; limb < kl; limb++) {
        const uint64_t varies = host.or_[limb] ^ host.and_[limb];
        for (uint32_t shift = 0; shift < 64; shift += kDigitBits) {
            if (((varies >> shift) & (kBins - 1)) == 0) continue; // constant digit: order unchanged
            hipLaunchKernelGGL(k_sort_hist, dim3(ntiles), dim3(kSortThreads), 0, s, keys[cur], n, limb, shift, hist,
                               ntiles);
            hipLaunchKernelGGL(k_sort_scan, dim3(1), dim3(1024), 0, s, hist, kBins * ntiles);
            switch (kl) {
            case 1:
                hipLaunchKernelGGL(k_sort_scatter<1>, dim3(ntiles), dim3(kSortThreads), 0, s, keys[cur], idx[cur],
                                   keys[cur ^ 1], idx[cur ^ 1], n, limb, shift, hist, ntiles);
                break;
            case 2:
                hipLaunchKernelGGL(k_sort_scatter<2>, dim3(ntiles), dim3(kSortThreads), 0, s, keys[cur], idx[cur],
                                   keys[cur ^ 1], idx[cur ^ 1], n, limb, shift, hist, ntiles);
                break;
            default:
                hipLaunchKernelGGL(k_sort_scatter<3>, dim3(ntiles), dim3(kSortThreads), 0, s, keys[cur], idx[cur],
                                   keys[cur ^ 1], idx[cur ^ 1], n, limb, shift, hist, ntiles);
                break;
            }
            cur ^= 1;
        }
    }
    const uint64_t chunks = (uint64_t)n * (vs >> 4);
    const uint32_t gblocks = (uint32_t)((chunks + 255) / 256 < 4096 ? (chunks + 255) / 256 : 4096);
    hipLaunchKernelGGL(k_sort_gather, dim3(gblocks), dim3(256), 0, s, (const uint8_t *)values, gathered, idx[cur], n,
                       vs);
    if (hipMemcpyAsync(values, gathered, (size_t)n * vs, hipMemcpyDeviceToDevice, s) != hipSuccess) return -1;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace tbc
