// Lab: one AES round per step, dependent chain, two ways.
//
//   table    production style: four T-table lookups from LDS per lane (one
//            per byte of the lane's column), a quad DPP exchange, XORs;
//   register no memory: ShiftRows by quad DPP, SubBytes by a v_perm_b32
//            nibble-pool S-box (32 pools of 8 S-box bytes, each v_perm looks
//            up 4 bytes at once by their low 3 bits, then a 5-level
//            byte-select tree by bits 3..7), MixColumns by xtime in-lane.
//
// Lane layout as aegis.hip: 4 lanes (a quad) hold one AES state, lane c
// column c. Both variants are checked against a CPU AES round chain, then
// timed at one wave (chain latency, the latency regime) and at 4 waves per
// SIMD on every CU (throughput). Prints JSON lines.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/sbox_lab.hip -o tools/sbox_lab && tools/sbox_lab
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                                                          \
    do {                                                                                                               \
        hipError_t e_ = (x);                                                                                           \
        if (e_ != hipSuccess) {                                                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                                  \
            exit(1);                                                                                                   \
        }                                                                                                              \
    } while (0)

static uint8_t g_sbox[256];
static uint32_t g_t0[256];

static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    for (int i = 0; i < 8; i++) {
        if (b & 1) p ^= a;
        const bool hi = a & 0x80;
        a <<= 1;
        if (hi) a ^= 0x1b;
        b >>= 1;
    }
    return p;
}

static void make_tables() {
    // S-box from the multiplicative inverse and the affine map (FIPS-197 5.1.1).
    for (int x = 0; x < 256; x++) {
        uint8_t inv = 0;
        for (int y = 1; y < 256 && x; y++)
            if (gmul((uint8_t)x, (uint8_t)y) == 1) inv = (uint8_t)y;
        uint8_t s = inv;
        for (int i = 1; i < 5; i++) s ^= (uint8_t)((inv << i) | (inv >> (8 - i)));
        g_sbox[x] = s ^ 0x63;
    }
    for (int x = 0; x < 256; x++) {
        const uint8_t s = g_sbox[x];
        g_t0[x] = (uint32_t)gmul(s, 2) | (uint32_t)s << 8 | (uint32_t)s << 16 | (uint32_t)gmul(s, 3) << 24;
    }
}

// CPU AES round on 4 columns (byte r of column c at bits 8r).
static void cpu_round(uint32_t col[4], const uint32_t key[4]) {
    uint8_t st[4][4], out[4][4];
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++) st[c][r] = (uint8_t)(col[c] >> (8 * r));
    for (int c = 0; c < 4; c++) {
        uint8_t a[4];
        for (int r = 0; r < 4; r++) a[r] = g_sbox[st[(c + r) & 3][r]];
        for (int r = 0; r < 4; r++)
            out[c][r] = gmul(a[r], 2) ^ gmul(a[(r + 1) & 3], 3) ^ a[(r + 2) & 3] ^ a[(r + 3) & 3];
    }
    for (int c = 0; c < 4; c++) {
        col[c] = 0;
        for (int r = 0; r < 4; r++) col[c] |= (uint32_t)out[c][r] << (8 * r);
        col[c] ^= key[c];
    }
}

struct Pools {
    uint32_t w[64]; // pool j = S[8j .. 8j+7]: lo word w[2j], hi word w[2j+1]
};

template <int SEL> __device__ __forceinline__ uint32_t quad(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, SEL, 0xf, 0xf, false);
}
// quad_perm [1,2,3,0] -> lane c reads lane c+1 (mod 4) etc.
constexpr int kQ1 = (1) | (2 << 2) | (3 << 4) | (0 << 6);
constexpr int kQ2 = (2) | (3 << 2) | (0 << 4) | (1 << 6);
constexpr int kQ3 = (3) | (0 << 2) | (1 << 4) | (2 << 6);

__device__ __forceinline__ uint32_t rotl(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }
__device__ __forceinline__ uint32_t rotr(uint32_t x, int s) { return (x >> s) | (x << (32 - s)); }

// Table round: lane c looks up its own column's bytes, the quad exchanges
// the looked-up words (what column c needs of row r comes from lane c + r).
__device__ __forceinline__ uint32_t round_table(const uint32_t *sT, uint32_t x, uint32_t key) {
    const uint32_t t0 = sT[x & 255];                            // row 0 of my column -> my output
    const uint32_t t1 = rotl(sT[(x >> 8) & 255], 8);            // row 1 -> lane c - 1
    const uint32_t t2 = rotl(sT[(x >> 16) & 255], 16);          // row 2 -> lane c - 2
    const uint32_t t3 = rotl(sT[x >> 24], 24);                  // row 3 -> lane c - 3
    return key ^ t0 ^ quad<kQ1>(t1) ^ quad<kQ2>(t2) ^ quad<kQ3>(t3);
}

__device__ __forceinline__ uint32_t sbox_perm(const Pools &P, uint32_t x) {
    const uint32_t lo3 = x & 0x07070707u;
    uint32_t r[32];
#pragma unroll
    for (int j = 0; j < 32; j++) r[j] = __builtin_amdgcn_perm(P.w[2 * j + 1], P.w[2 * j], lo3);
#pragma unroll
    for (int b = 3, n = 32; b < 8; b++, n >>= 1) {
        const uint32_t m = ((x >> b) & 0x01010101u) * 0xffu; // byte-wise mask of bit b
#pragma unroll
        for (int j = 0; j < n / 2; j++) r[j] = (r[2 * j + 1] & m) | (r[2 * j] & ~m);
    }
    return r[0];
}

__device__ __forceinline__ uint32_t xt(uint32_t y) {
    return ((y & 0x7f7f7f7fu) << 1) ^ (((y >> 7) & 0x01010101u) * 0x1bu);
}

// Register round: ShiftRows by DPP (row r of my new column is row r of
// column c + r), SubBytes by the perm S-box, MixColumns in-lane.
__device__ __forceinline__ uint32_t round_reg(const Pools &P, uint32_t x, uint32_t key) {
    const uint32_t x1 = quad<kQ1>(x), x2 = quad<kQ2>(x), x3 = quad<kQ3>(x);
    const uint32_t s = (x & 0x000000ffu) | (x1 & 0x0000ff00u) | (x2 & 0x00ff0000u) | (x3 & 0xff000000u);
    const uint32_t a = sbox_perm(P, s);
    const uint32_t r1 = rotr(a, 8), r2 = rotr(a, 16), r3 = rotr(a, 24);
    return xt(a ^ r1) ^ r1 ^ r2 ^ r3 ^ key;
}

template <bool Reg>
__global__ __launch_bounds__(256) void k_chain(const uint32_t *t0, Pools P, const uint32_t *init, uint32_t iters,
                                               uint32_t *out, uint64_t *ticks) {
    __shared__ uint32_t sT[256];
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) sT[i] = t0[i];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    uint32_t x = init[lane & 3] ^ (blockIdx.x * 0x9e3779b9u) ^ ((threadIdx.x >> 2) * 0x85ebca6bu);
    const uint32_t key = 0x01020304u * ((lane & 3) + 1);
    const uint64_t t_start = wall_clock64();
    for (uint32_t i = 0; i < iters; i++) x = Reg ? round_reg(P, x, key) : round_table(sT, x, key);
    const uint64_t t_end = wall_clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x == 0) ticks[blockIdx.x] = t_end - t_start;
}

int main() {
    make_tables();
    Pools P;
    for (int j = 0; j < 32; j++) {
        P.w[2 * j] = (uint32_t)g_sbox[8 * j] | (uint32_t)g_sbox[8 * j + 1] << 8 | (uint32_t)g_sbox[8 * j + 2] << 16 |
                     (uint32_t)g_sbox[8 * j + 3] << 24;
        P.w[2 * j + 1] = (uint32_t)g_sbox[8 * j + 4] | (uint32_t)g_sbox[8 * j + 5] << 8 |
                         (uint32_t)g_sbox[8 * j + 6] << 16 | (uint32_t)g_sbox[8 * j + 7] << 24;
    }
    const uint32_t init[4] = {0x00112233u, 0x44556677u, 0x8899aabbu, 0xccddeeffu};
    uint32_t *d_t0, *d_init, *d_out;
    uint64_t *d_ticks;
    const int max_blocks = 256 * 4; // 4 workgroups of 4 waves per CU: 4 waves per SIMD
    CK(hipMalloc(&d_t0, 1024));
    CK(hipMalloc(&d_init, 16));
    CK(hipMalloc(&d_out, 4ull * 256 * max_blocks));
    CK(hipMalloc(&d_ticks, 8ull * max_blocks));
    CK(hipMemcpy(d_t0, g_t0, 1024, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_init, init, 16, hipMemcpyHostToDevice));

    // Correctness: 64 rounds of block 0, wave 0, quad 0 against the CPU.
    bool ok = true;
    for (int v = 0; v < 2; v++) {
        const uint32_t iters = 64;
        if (v) hipLaunchKernelGGL(k_chain<true>, dim3(1), dim3(64), 0, 0, d_t0, P, d_init, iters, d_out, d_ticks);
        else hipLaunchKernelGGL(k_chain<false>, dim3(1), dim3(64), 0, 0, d_t0, P, d_init, iters, d_out, d_ticks);
        CK(hipDeviceSynchronize());
        uint32_t got[4];
        CK(hipMemcpy(got, d_out, 16, hipMemcpyDeviceToHost));
        uint32_t col[4], key[4];
        for (int c = 0; c < 4; c++) {
            col[c] = init[c];
            key[c] = 0x01020304u * (c + 1);
        }
        for (uint32_t i = 0; i < iters; i++) cpu_round(col, key);
        const bool eq = !memcmp(got, col, 16);
        ok = ok && eq;
        printf("{\"check\": \"%s\", \"bit_exact\": %s}\n", v ? "register" : "table", eq ? "true" : "false");
    }
    if (!ok) return 1;

    const uint32_t iters = 1u << 16;
    for (int v = 0; v < 2; v++) {
        for (int blocks : {1, max_blocks}) {
            const int threads = blocks == 1 ? 64 : 256;
            hipEvent_t a, b;
            CK(hipEventCreate(&a));
            CK(hipEventCreate(&b));
            float best = 1e30f;
            for (int r = 0; r < 3; r++) {
                CK(hipEventRecord(a));
                if (v) hipLaunchKernelGGL(k_chain<true>, dim3(blocks), dim3(threads), 0, 0, d_t0, P, d_init, iters, d_out,
                                          d_ticks);
                else hipLaunchKernelGGL(k_chain<false>, dim3(blocks), dim3(threads), 0, 0, d_t0, P, d_init, iters,
                                        d_out, d_ticks);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                best = ms < best ? ms : best;
            }
            uint64_t t0;
            CK(hipMemcpy(&t0, d_ticks, 8, hipMemcpyDeviceToHost));
            const double waves = (double)blocks * threads / 64;
            printf("{\"variant\": \"%s\", \"waves\": %.0f, \"ns_per_round_in_kernel\": %.2f, \"kernel_ms\": %.3f, "
                   "\"G_rounds_per_s_chip\": %.1f}\n",
                   v ? "register" : "table", waves, (double)t0 * 10.0 / iters, best,
                   waves * 64 / 4 * iters / (best * 1e-3) / 1e9);
            CK(hipEventDestroy(a));
            CK(hipEventDestroy(b));
        }
    }
    return 0;
}
