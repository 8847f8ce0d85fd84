// keys.h — key_from_value and key order on device, shared by the 2-way
// compaction merge (merge.hip) and the k-way scan merge (kway.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "tbc_internal.h"

namespace tbc {

template <int KIND> struct KeyLimbs { static constexpr int value = KIND == kKeyTimestamp ? 1 : KIND == kKeyCompositeU128 ? 3 : 2; };

template <int KL> struct Key {
    uint64_t l[KL];
};

template <int KL> __device__ __forceinline__ bool key_eq(const Key<KL> &a, const Key<KL> &b) {
    bool e = true;
#pragma unroll
    for (int i = 0; i < KL; i++) e &= a.l[i] == b.l[i];
    return e;
}

// a <= b (unsigned, most significant limb last)
template <int KL> __device__ __forceinline__ bool key_le(const Key<KL> &a, const Key<KL> &b) {
#pragma unroll
    for (int i = KL - 1; i > 0; i--)
        if (a.l[i] != b.l[i]) return a.l[i] < b.l[i];
    return a.l[0] <= b.l[0];
}

template <int KL> __device__ __forceinline__ bool key_lt(const Key<KL> &a, const Key<KL> &b) {
#pragma unroll
    for (int i = KL - 1; i > 0; i--)
        if (a.l[i] != b.l[i]) return a.l[i] < b.l[i];
    return a.l[0] < b.l[0];
}

__device__ __forceinline__ uint64_t ld64(const uint8_t *p) { return gld<uint64_t>(p); }

// key_from_value (composite_key.zig:48-50, groove.zig:27-29, 59-61).
template <int KIND>
__device__ __forceinline__ Key<KeyLimbs<KIND>::value> load_key(const uint8_t *v, uint32_t ts_off) {
    Key<KeyLimbs<KIND>::value> k;
    if constexpr (KIND == kKeyTimestamp) {
        k.l[0] = ld64(v + ts_off) & ~kTombstoneBit;
    } else if constexpr (KIND == kKeyIdU128) {
        k.l[0] = ld64(v);
        k.l[1] = ld64(v + 8);
    } else if constexpr (KIND == kKeyCompositeU64) {
        k.l[0] = ld64(v + 8) & ~kTombstoneBit;
        k.l[1] = ld64(v);
    } else {
        k.l[0] = ld64(v + 16) & ~kTombstoneBit;
        k.l[1] = ld64(v);
        k.l[2] = ld64(v + 8);
    }
    return k;
}

// Key of lane `src` (ds_bpermute of each 32-bit half; the whole wave active).
template <int KL> __device__ __forceinline__ Key<KL> key_of_lane(const Key<KL> &k, uint32_t src) {
    Key<KL> r;
    const int addr = (int)(src << 2);
#pragma unroll
    for (int l = 0; l < KL; l++) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)(uint32_t)k.l[l]);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)(uint32_t)(k.l[l] >> 32));
        r.l[l] = (uint64_t)hi << 32 | lo;
    }
    return r;
}

} // namespace tbc
