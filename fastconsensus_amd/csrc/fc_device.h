// fc_device.h -- host/device helpers shared by the HIP kernels: integer hashes, the
// bucketed random vertex order (Feistel permutation), Philox4x32-10, wave helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define FC_HD __host__ __device__ __forceinline__

namespace fc {

// 32-bit integer mixer (fmix32 of MurmurHash3).
FC_HD uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x85ebca6bu;
    x ^= x >> 13; x *= 0xc2b2ae35u;
    x ^= x >> 16;
    return x;
}
// hash32 is a bijection; its inverse recovers x from hash32(x)
FC_HD uint32_t hash32_inv(uint32_t x) {
    x ^= x >> 16; x *= 0x7ed1b41du;
    x ^= (x >> 13) ^ (x >> 26); x *= 0xa5cb9243u;
    x ^= x >> 16;
    return x;
}
FC_HD uint32_t hash2(uint32_t a, uint32_t b) { return hash32(a ^ hash32(b + 0x9e3779b9u)); }
FC_HD uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Per-(replica, iteration, sweep) stream key.  rg = GLOBAL replica index, so results do
// not depend on how replicas are sharded over GPUs.
FC_HD uint32_t stream_key(uint64_t seed, uint32_t rg, uint32_t iter, uint32_t sweep, uint32_t salt) {
    uint64_t z = mix64(seed ^ (0x9E3779B97F4A7C15ull * (1 + (uint64_t)rg)));
    z = mix64(z ^ ((uint64_t)iter << 32 | sweep) ^ ((uint64_t)salt << 56));
    return (uint32_t)(z ^ (z >> 32));
}
// Stream key of the visit order every replica of a batch shares (FC_OPT_CD_ENGINE 1 and 2:
// cd_rl.hip, and cd.hip's full sweeps in the hybrid; oracle TW_SHARED_RG).
constexpr uint32_t SHARED_RG = 0xffffffffu;

// Random bijection on [0, n): balanced 4-round Feistel network on 2*hb bits with cycle
// walking.  Sweep order of a replica = perm(0), perm(1), ...; bucket k of a sweep is the
// position range [k*S, (k+1)*S).
struct Perm {
    uint32_t n, hb, mask;
    uint32_t k0, k1, k2, k3;
    uint32_t off;   // chunked CD orders: shift of the chunk grid (cd.hip sweep_perm), else 0
};
FC_HD Perm make_perm(uint32_t n, uint32_t key) {
    Perm p;
    uint32_t bits = 1;
    while (bits < 32 && (1u << bits) < n) ++bits;
    uint32_t hb = (bits + 1) / 2;
    if (hb < 1) hb = 1;
    p.n = n; p.hb = hb; p.mask = (1u << hb) - 1u;
    p.k0 = hash2(key, 0x1234567u); p.k1 = hash2(key, 0x89abcdefu);
    p.k2 = hash2(key, 0x2468aceu); p.k3 = hash2(key, 0x13579bdu);
    p.off = 0;
    return p;
}
FC_HD uint32_t feistel_round(uint32_t x, const Perm& p) {
    uint32_t L = x >> p.hb, R = x & p.mask, t;
    t = R; R = L ^ (hash32(R ^ p.k0) & p.mask); L = t;
    t = R; R = L ^ (hash32(R ^ p.k1) & p.mask); L = t;
    t = R; R = L ^ (hash32(R ^ p.k2) & p.mask); L = t;
    t = R; R = L ^ (hash32(R ^ p.k3) & p.mask); L = t;
    return (L << p.hb) | R;
}
FC_HD uint32_t perm_apply(const Perm& p, uint32_t x) {
    do { x = feistel_round(x, p); } while (x >= p.n);
    return x;
}
// Inverse: position of element y (rounds undone in reverse; cycle walking backwards).
FC_HD uint32_t feistel_round_inv(uint32_t y, const Perm& p) {
    uint32_t L = y >> p.hb, R = y & p.mask, t;
    t = L; L = R ^ (hash32(L ^ p.k3) & p.mask); R = t;
    t = L; L = R ^ (hash32(L ^ p.k2) & p.mask); R = t;
    t = L; L = R ^ (hash32(L ^ p.k1) & p.mask); R = t;
    t = L; L = R ^ (hash32(L ^ p.k0) & p.mask); R = t;
    return (L << p.hb) | R;
}
FC_HD uint32_t perm_invert(const Perm& p, uint32_t y) {
    do { y = feistel_round_inv(y, p); } while (y >= p.n);
    return y;
}

// Philox4x32-10 (Salmon et al., SC'11): counter-based, so attempt t of iteration it draws
// the same numbers on every rank.
struct U4 { uint32_t x, y, z, w; };
FC_HD U4 philox(U4 c, uint32_t k0, uint32_t k1) {
    for (int i = 0; i < 10; ++i) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
        U4 n;
        n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
        n.y = (uint32_t)p1;
        n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
        n.w = (uint32_t)p0;
        c = n;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return c;
}
// uniform integer in [0, n) from a 32-bit draw (multiply-high; bias < n / 2^32).
FC_HD uint32_t below(uint32_t r, uint32_t n) { return (uint32_t)(((uint64_t)r * n) >> 32); }

// Sharded global counters [CSH][F]: a block adds into shard blockIdx % CSH, a one-block
// kernel (k_reduce_shards) folds them.  A single hot address would serialise every
// block's atomic (~12 ns each on MI355X).
constexpr int CSH = 256;
__device__ __forceinline__ unsigned long long* shard(unsigned long long* base, int F, int f) {
    return base + (size_t)(blockIdx.x & (CSH - 1)) * F + f;
}

}  // namespace fc
