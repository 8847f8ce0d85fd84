// grid.hip — the GPU-resident grid's side of a compaction batch.
//
// The reference reads a compaction's inputs through the grid
// (src/vsr/grid.zig:843-890): a cache hit is trusted once its header
// checksum equals the one the index block (or manifest) expects
// (read_block_from_cache, :802-841); a block read from storage is validated
// first (read_block_validate, :1059-1084). The table iterators then walk an
// input table's index block for its data blocks' addresses and checksums
// (table_data_iterator.zig, level_data_iterator.zig:142-224). Here the whole
// grid zone is resident in HBM, so a batch:
//   k_grid_resolve  finds every input data block through its table's index
//                   block (address, checksum) and fills the merge's segment
//                   table — the host only knows TableInfos, as Compaction does;
//   k_grid_expect   reads their expected checksums from the index blocks
//                   once the batches that wrote them have sealed them;
//   k_grid_check    applies read_block_from_cache's checks plus the header
//                   fields the iterators assert, to every input block (cheap);
//   k_grid_validate (aegis.hip) runs read_block_validate on the blocks staged
//                   from storage, on a second stream beside the compaction;
//   k_grid_mark     trusts the batch's outputs (written by the engine itself)
//                   once its input checks passed.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "tbc_internal.h"

namespace tbc {

__device__ __forceinline__ void grid_error(uint32_t *slot, uint32_t code) {
    uint32_t expected = 0;
    __hip_atomic_compare_exchange_strong(slot, &expected, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
}

// One thread per input data block: TableIndex.data_addresses[k] and
// data_checksums[k] (schema.zig:80-260) from the table's index block. An
// address outside the grid (a corrupt index block that slipped past its
// checks) is reported and replaced by the index block itself, so every later
// load stays inside the grid.
__global__ __launch_bounds__(256) void k_grid_resolve(const ResolveItem *items, uint32_t count, uint64_t *seg_ptr,
                                                      InputCheck *checks, const uint8_t *grid_base,
                                                      uint64_t grid_blocks, uint32_t block_size, JobResultDev *res) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    const ResolveItem it = items[i];
    const uint8_t *idx = (const uint8_t *)(uintptr_t)it.index_ptr;
    uint64_t address = gld<uint64_t>(idx + it.addr_off + 8 * it.k);
    uint64_t blk = (uint64_t)(uintptr_t)grid_base + (address - 1) * block_size;
    if (address == 0 || address > grid_blocks) {
        grid_error(&res[it.job].block_error, 7u);
        blk = it.index_ptr;
        address = 0; // k_grid_check / k_grid_validate skip it
    }
    seg_ptr[it.seg] = blk + kHeaderSize;
    InputCheck c;
    c.ptr = blk;
    c.address = address;
    c.checksum[0] = c.checksum[1] = 0; // k_grid_expect (the index block may not be sealed yet)
    c.value_count = it.value_count;
    c.job = it.job;
    c.kind = 5; // BlockType.data
    c.pad = 0;
    checks[it.check] = c;
}

// The expected checksum of every input data block, TableIndex.data_checksums[k]:
// read once the batches that wrote the index blocks have sealed them.
__global__ __launch_bounds__(256) void k_grid_expect(const ResolveItem *items, uint32_t count, InputCheck *checks) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    const ResolveItem it = items[i];
    const uint8_t *idx = (const uint8_t *)(uintptr_t)it.index_ptr;
    checks[it.check].checksum[0] = gld<uint64_t>(idx + it.cks_off + 32 * it.k);
    checks[it.check].checksum[1] = gld<uint64_t>(idx + it.cks_off + 32 * it.k + 8);
}

// One thread per trusted input block (index and data; blocks staged from
// storage are k_grid_validate's): read_block_from_cache's cache-hit test (the
// header checksum is the expected one; address and cluster match,
// grid.zig:818-835) and the header fields the compaction's iterators assert.
__global__ __launch_bounds__(256) void k_grid_check(const InputCheck *checks, uint32_t count, const uint8_t *verified,
                                                    const JobDesc *jobs, int njobs, JobResultDev *res,
                                                    uint32_t block_size) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    const InputCheck c = checks[i];
    if (c.address == 0 || !verified[c.address - 1]) return; // resolve reported it / the validation's
    const uint8_t *blk = (const uint8_t *)(uintptr_t)c.ptr;
    uint32_t r;
    if (gld<uint64_t>(blk) != c.checksum[0] || gld<uint64_t>(blk + 8) != c.checksum[1])
        r = 4; // not the block the index/manifest names (a cache miss in the reference)
    else if (gld<uint64_t>(blk + 224) != c.address)
        r = 5;
    else
        r = grid_header_check(job_of_result(jobs, njobs, c.job), c, block_size);
    if (r) grid_error(&res[c.job].block_error, r);
}

// Outputs of the batch's grid jobs are trusted from now on (every reserved
// address: unused ones are never named by an index block of this batch) —
// after the batch's input checks, and only for jobs that ended clean: blocks
// built from a corrupt input or by a job that hit an invariant stay
// unverified, so a later batch naming them validates them in full.
__global__ __launch_bounds__(256) void k_grid_mark(const JobDesc *jobs, int njobs, uint8_t *verified,
                                                   const JobResultDev *res) {
    const JobDesc &j = jobs[blockIdx.x];
    if (!j.grid_base) return;
    const JobResultDev &r = res[j.job_index];
    if (r.status || r.invariant || r.block_error) return;
    for (uint32_t a = threadIdx.x; a < j.address_count; a += 256) verified[gld<uint64_t>(j.addresses + a) - 1] = 1;
}

int launch_grid_resolve(const ResolveItem *d_items, uint32_t count, uint64_t *d_seg_ptr, InputCheck *d_checks,
                        const uint8_t *grid_base, uint64_t grid_blocks, uint32_t block_size, JobResultDev *d_results,
                        void *stream) {
    if (!count) return 0;
    hipLaunchKernelGGL(k_grid_resolve, dim3((count + 255) / 256), dim3(256), 0, (hipStream_t)stream, d_items, count,
                       d_seg_ptr, d_checks, grid_base, grid_blocks, block_size, d_results);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_grid_expect(const ResolveItem *d_items, uint32_t count, InputCheck *d_checks, void *stream) {
    if (!count) return 0;
    hipLaunchKernelGGL(k_grid_expect, dim3((count + 255) / 256), dim3(256), 0, (hipStream_t)stream, d_items, count,
                       d_checks);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_grid_checks(const InputCheck *d_checks, uint32_t count, const uint8_t *d_verified, const JobDesc *d_jobs,
                       int njobs, JobResultDev *d_results, uint32_t block_size, void *stream) {
    if (!count) return 0;
    hipLaunchKernelGGL(k_grid_check, dim3((count + 255) / 256), dim3(256), 0, (hipStream_t)stream, d_checks, count,
                       d_verified, d_jobs, njobs, d_results, block_size);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_grid_mark(const JobDesc *d_jobs, int njobs, uint8_t *d_verified, const JobResultDev *d_results,
                     void *stream) {
    if (!njobs) return 0;
    hipLaunchKernelGGL(k_grid_mark, dim3(njobs), dim3(256), 0, (hipStream_t)stream, d_jobs, njobs, d_verified,
                       d_results);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// One thread per address: the grid's `verified` byte of each block set to
// `value` (blocks staged from storage: 0, validated before they are trusted;
// blocks the engine wrote: 1), one launch for a whole list instead of one
// 1-byte fill per block.
__global__ __launch_bounds__(256) void k_grid_set_verified(const uint64_t *addresses, uint32_t count, uint8_t *verified,
                                                           uint8_t value) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < count) verified[addresses[i] - 1] = value;
}

int launch_grid_set_verified(const uint64_t *d_addresses, uint32_t count, uint8_t *d_verified, uint8_t value,
                             void *stream) {
    if (!count) return 0;
    hipLaunchKernelGGL(k_grid_set_verified, dim3((count + 255) / 256), dim3(256), 0, (hipStream_t)stream, d_addresses,
                       count, d_verified, value);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// tbc_copy_device_batch: many device-to-device copies (16-byte aligned,
// multiples of 16 bytes) in one launch. One workgroup per 64 KiB chunk:
// every lane's sixteen 16-byte loads are issued before its stores.
constexpr uint32_t kCopyChunk = 65536;

__global__ __launch_bounds__(256) void k_copy_batch(const CopyItem *items, uint32_t count) {
    uint32_t lo = 0, hi = count; // the copy whose chunk range holds this workgroup's chunk
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (items[mid].chunk0 <= blockIdx.x) lo = mid;
        else hi = mid;
    }
    const CopyItem it = items[lo];
    const uint64_t off = (uint64_t)(blockIdx.x - it.chunk0) * kCopyChunk;
    const uint64_t n = it.bytes - off < kCopyChunk ? it.bytes - off : kCopyChunk;
    const uint8_t *src = (const uint8_t *)it.src + off;
    uint8_t *dst = (uint8_t *)it.dst + off;
    u32x4 v[16];
#pragma unroll
    for (uint32_t r = 0; r < 16; r++) {
        const uint64_t o = 16 * ((uint64_t)threadIdx.x + 256 * r);
        if (o < n) v[r] = gld<u32x4>(src + o);
    }
#pragma unroll
    for (uint32_t r = 0; r < 16; r++) {
        const uint64_t o = 16 * ((uint64_t)threadIdx.x + 256 * r);
        if (o < n) gst<u32x4>(dst + o, v[r]);
    }
}

int launch_copy_batch(const CopyItem *d_items, uint32_t count, uint32_t chunks, void *stream) {
    if (!count || !chunks) return 0;
    hipLaunchKernelGGL(k_copy_batch, dim3(chunks), dim3(256), 0, (hipStream_t)stream, d_items, count);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
uint64_t copy_chunk_bytes() { return kCopyChunk; }

// Host-to-device upload of a pinned (device-mapped) host buffer by a compute
// kernel on the caller's stream: each batch's descriptor image, a sort's plan
// and a device-copy list are read over PCIe by the kernel itself instead of a
// DMA copy, so the engine stream never hands off to a copy engine between
// two half-bars (TBC_UPLOAD_COPY=1 restores hipMemcpyAsync, A/B only).
// The host rewrites a slot once the stream has passed its previous upload,
// so the source is read at system scope (no cache may hold the old bytes).
__global__ __launch_bounds__(256) void k_upload(uint64_t *dst, const uint64_t *src, uint64_t n8, uint8_t *dst_tail,
                                               const uint8_t *src_tail, uint32_t tail, uint64_t *zero, uint64_t zero8) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += stride)
        dst[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (blockIdx.x == 0 && threadIdx.x < tail)
        dst_tail[threadIdx.x] = __hip_atomic_load(src_tail + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < zero8; i += stride) zero[i] = 0;
}

int launch_upload(void *dst, const void *host_src, uint64_t bytes, void *stream, void *zero, uint64_t zero_bytes) {
    hipStream_t s = (hipStream_t)stream;
    if (zero_bytes && (((uintptr_t)zero | zero_bytes) & 7)) { // not whole words: a fill of its own
        if (hipMemsetAsync(zero, 0, zero_bytes, s) != hipSuccess) return -1;
        zero_bytes = 0;
    }
    if (!bytes && !zero_bytes) return 0;
    if (((uintptr_t)dst | (uintptr_t)host_src) & 7) {
        if (bytes && hipMemcpyAsync(dst, host_src, bytes, hipMemcpyHostToDevice, s) != hipSuccess) return -1;
        bytes = 0;
        if (!zero_bytes) return 0;
    }
    const uint64_t n8 = bytes / 8, z8 = zero_bytes / 8;
    const uint32_t tail = (uint32_t)(bytes - 8 * n8);
    const uint64_t blocks = ((n8 > z8 ? n8 : z8) + 255) / 256;
    hipLaunchKernelGGL(k_upload, dim3((uint32_t)(blocks < 512 ? (blocks ? blocks : 1) : 512)), dim3(256), 0, s,
                       (uint64_t *)dst, (const uint64_t *)host_src, n8, (uint8_t *)dst + 8 * n8,
                       (const uint8_t *)host_src + 8 * n8, tail, (uint64_t *)zero, z8);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) fprintf(stderr, "tbc: upload of %llu bytes: %s (%d)\n", (unsigned long long)bytes,
                                   hipGetErrorString(err), (int)err);
    return err == hipSuccess ? 0 : -1;
}

} // namespace tbc
