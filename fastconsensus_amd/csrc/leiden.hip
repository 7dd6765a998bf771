// leiden.hip -- replica-batched Leiden on MI355X: the community detection of the reference's
// `leiden` branch, leidenalg.find_partition(graph, ModularityVertexPartition, weights='weight',
// seed=i, n_iterations=1) (fast_consensus.py:121-123, called n_p times at :210-211 and :386-387).
//
// leidenalg (not vendored, not installed; restated from its published algorithm, Traag,
// Waltman & van Eck 2019, and the package's documented defaults -- parity unpinned, see
// the oracle's restatement in oracle/fc_oracle.c) optimises one level at a time:
//   1. move nodes: a queue of every node in random order; a node moves to the neighbour (or
//      empty) community of largest modularity gain if that gain is positive, and its
//      neighbours outside the new community re-enter the queue;
//   2. refine: every node starts alone; in random order, a node that is still alone joins the
//      best (gain > 0) refined community among its neighbours inside its own step-1 community;
//   3. aggregate the graph by the refined communities, each aggregate node starting in the
//      step-1 community of its members; repeat from 1 while the refinement merged anything.
//
// MI355X layout.  All replicas of a level live in ONE union graph: replica r's aggregate
// nodes occupy a contiguous id range, so one launch serves every replica, and the replicas
// share 2M (aggregation preserves the total weight).  Level 0 is the input graph itself,
// addressed implicitly (union vertex x = r*N + v, row of v), and its move phase is the
// replica-batched Louvain local-moving engine (cd.hip) run to exhaustion (no 1e-7 cut).
// Levels >= 1 are explicit CSRs built here with LDS hash tables (global tables for long
// rows).  A sweep is B buckets: bucket(x) = hash(replica stream key, local id) mod B; a
// bucket's vertices decide against the state left by the earlier buckets, then apply.
// Integer weights: gains are exact int64 (w_vc*2M - k_v*Sigma_c).  Randomness is keyed by
// (seed, GLOBAL replica index, local vertex id), so results do not depend on the sharding.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <vector>

#include "fc_ctx.h"
#include "fc_device.h"
#include "fc_log2.h"

namespace fc {

template <class T> void exclusive_scan(Ctx& c, const T* in, T* out, int64_t n);

namespace {

constexpr int LTB = 256;          // threads per block (4 waves)
constexpr int LWS = 1024;         // LDS hash slots per wave (a table is sized to its row: 64..LWS)
constexpr int LIGHT = LWS / 2;    // rows / member-row sums above this go to the block-per-vertex kernels
constexpr int LWS_SMALL = 256;    // the short-row variant of k_lv_decide
constexpr int HLS = 8192;         // LDS slots of a block-per-vertex table
constexpr int HLIGHT = HLS / 2;   // longer rows use a global table
// Long rows are listed by length tier, each tier decided by a block-per-vertex kernel whose LDS
// table just fits it: <= 1024 entries in 2048 slots (16 KB: 8 blocks per CU), <= 2048 in 4096
// (32 KB: 5), <= 4096 in 8192 (64 KB: 2), longer rows in global tables.  One table size for a
// whole level (the longest row's) left a level of ~1000-entry rows with one 9576-entry row at 2
// blocks per CU.
constexpr int NTIER = 4;
__host__ __device__ constexpr int heavy_tier(int64_t d) { return d <= 1024 ? 0 : d <= 2048 ? 1 : d <= 4096 ? 2 : 3; }
constexpr int MODE_MOVE = 0, MODE_REFINE = 1, MODE_INFO = 2;   // Leiden move / refine; Infomap move
constexpr int MSH = 256;          // move-counter shards
constexpr int MAX_LEVELS = 64;
constexpr int UNR = 4;            // k_lv_heavy: entries / table slots per thread with their gathers in flight
                                  // (1 in k_lv_decide: its VGPRs cost more occupancy than the overlap gains)

inline unsigned nb(int64_t n, int tb = LTB) { return (unsigned)std::max<int64_t>(1, (n + tb - 1) / tb); }

// Level graph: explicit CSR over the union, or (IMPL) the input graph addressed per replica.
struct LvArgs {
    int64_t nU;               // union vertices
    int64_t N0;               // IMPL: vertices per replica
    const int64_t* rowptr;
    const int32_t* col;
    const int32_t* w;         // nullptr: unit weights
    const int64_t* kv;        // weighted degrees ([N0] when IMPL)
    const int32_t* rep;       // explicit: local replica of every union vertex
    const int32_t* roff;      // [n_r] first union id of each replica at this level
    const uint32_t* rkey;     // [n_r] stream key of this sweep per replica
    const uint8_t* done;      // [n_r] replica finished
    int64_t M2;
    int B;
    int32_t* P;               // move-phase community
    int32_t* R;               // refined community
    int64_t* tot;             // Sigma of the communities the mode works on (ptot or rtot)
    int32_t* rsize;           // refined community sizes
    uint8_t* act;             // move queue flags
    int32_t* blist;           // [nblk][LTB] movers of each decide block (vertex)
    int32_t* btgt;            // [nblk][LTB] their targets
    int32_t* bcnt;            // [nblk]
    int32_t* heavy;           // [NTIER][hcap] heavy vertices of this bucket, by length tier
    int32_t* heavy_cnt;       // [NTIER]
    int32_t* htgt;            // [NTIER][hcap] their decisions (-1: stay)
    int64_t hcap;
    int32_t* hkey;            // [LHB][hslots] global tables (kept cleared)
    int32_t* hval;
    int32_t* hlst;            // [LHB][hslots] created slots
    int64_t hslots;
    unsigned long long* moves;   // [MSH]
    unsigned long long* rmoves;  // Infomap: [n_r] moves of each replica in this pass
    const uint8_t* lvdone;       // Infomap: [n_r] replica's passes at this level are over (a pass moved nothing)
    const int32_t* ilist;        // Infomap: this bucket's vertices, compacted once per pass (k_info_lfill);
    int64_t icnt;                //   nullptr: every launch scans the union for its bucket (bmap below)
    const int32_t* bmap;         // Infomap, input-graph level: launch only the replicas still moving --
    int bpr;                     //   block b covers replica bmap[b / bpr], ids (b % bpr)*LTB.. of it
    int nact;                    //   replicas in bmap
    unsigned long long* mvt;     // [nU] move phase: (bucket stamp << 32) | target of this bucket's movers
    // Infomap (map equation): module exit weights, the replica's total exit weight, every
    // vertex's external weight (row sum; its weighted degree kv also counts internal edges),
    // the two adjacency weights a move changes, 1/2M
    int64_t* out;
    int64_t* mod;                // Infomap: per module {flow, exit weight} as one 16-byte record
    int64_t* qrep;
    const int64_t* sv;
    int32_t* mvo;                // [nU] Infomap: the old module of this bucket's movers (with mvt)
    double inv;
    unsigned long long* lvb;     // [2][MSH] algorithmic bytes of k_lv_decide / k_lv_heavy launches,
                                 // sharded by block: one hot address serialised every wave's atomic
};

// Algorithmic bytes (DESIGN.md "Leiden and Infomap"): the per-vertex records a decision
// reads and writes, per adjacency entry its column, weight and neighbour label(s), per
// candidate community its Sigma (int64) or Infomap module record (flow, exit: 16 B).
template <int MODE> __device__ __forceinline__ constexpr int lv_vertex_bytes() {
    return 16 /* rowptr */ + 4 /* own */ + 8 /* kv */ + (MODE == MODE_REFINE ? 4 : 0) /* P[x] */ +
           (MODE == MODE_INFO ? 8 + 16 + 8 : 0) /* sv, own module, qrep */;
}
template <int MODE> __device__ __forceinline__ constexpr int lv_mover_bytes() {
    return 4 + 4 + (MODE == MODE_REFINE ? 0 : 8) + (MODE == MODE_INFO ? 4 : 0);   // list, target, mvt, mvo
}
template <int MODE> __device__ __forceinline__ int lv_entry_bytes(bool weighted) {
    return 4 + (weighted ? 4 : 0) + (MODE == MODE_REFINE ? 8 : 4);
}
template <int MODE> __device__ __forceinline__ constexpr int lv_cand_bytes() { return MODE == MODE_INFO ? 16 : 8; }

__device__ __forceinline__ double plogp2(double p) { return p > 0.0 ? p * log2(p) : 0.0; }
// The decisions' terms use fc_log2 (~2 ulp, ~20 instructions, table in LDS) instead of the
// library's log2 (~0.5 ulp, 89 instructions): the map-equation deltas are sums of these terms
// compared against each other and against -1e-10, so ~1e-16 of error per term only matters for
// candidates within ~1e-15 of each other.  Reported codelengths (k_info_codelen) keep log2.
__constant__ Log2Entry c_log2[49] = FC_LOG2_TABLE;
__device__ __forceinline__ double plogp2f(double p, const Log2Entry* lt) { return p > 0.0 ? p * fc_log2(p, lt) : 0.0; }
// The map-equation change split into the part of the source module A (computed once per
// vertex) and the per-candidate part (module B and the total exit Q'), 5 logarithms each.
struct InfoA {
    long long dA;     // change of A's exit weight
    double termA;     // A's terms of delta-L
    double q0;        // plogp(Q)
};
__device__ __forceinline__ InfoA info_a(double inv, long long Q, long long oA, long long tA, long long kv, long long sv,
                                        long long wA, const Log2Entry* lt) {
    InfoA r;
    const long long oA2 = oA - sv + 2 * wA, tA2 = tA - kv;
    r.dA = oA2 - oA;
    r.termA = -2.0 * (plogp2f(oA2 * inv, lt) - plogp2f(oA * inv, lt)) +
              (plogp2f((oA2 + tA2) * inv, lt) - plogp2f((oA + tA) * inv, lt));
    r.q0 = plogp2f(Q * inv, lt);
    return r;
}
__device__ __forceinline__ double info_b(double inv, const InfoA& A, long long Q, long long oB, long long tB,
                                         long long kv, long long sv, long long wB, const Log2Entry* lt) {
    const long long oB2 = oB + sv - 2 * wB, tB2 = tB + kv;
    const long long Q2 = Q + A.dA + (oB2 - oB);
    return (plogp2f(Q2 * inv, lt) - A.q0) + A.termA - 2.0 * (plogp2f(oB2 * inv, lt) - plogp2f(oB * inv, lt)) +
           (plogp2f((oB2 + tB2) * inv, lt) - plogp2f((oB + tB) * inv, lt));
}
// smaller delta, then larger tie hash, then smaller id; c < 0 = none
__device__ __forceinline__ bool info_better(double d1, uint32_t h1, int32_t c1, double d2, uint32_t h2, int32_t c2) {
    if (c1 < 0) return false;
    if (c2 < 0) return true;
    if (d1 != d2) return d1 < d2;
    if (h1 != h2) return h1 > h2;
    return c1 < c2;
}
constexpr double INFO_MIN_GAIN = 1e-10;   // igraph's greedy core moves on a codelength decrease > 1e-10

template <bool IMPL> __device__ __forceinline__ int32_t rep_of(const LvArgs& a, int64_t x) {
    return IMPL ? (int32_t)(x / a.N0) : a.rep[x];
}
template <bool IMPL> __device__ __forceinline__ int64_t kv_of(const LvArgs& a, int64_t x) {
    return IMPL ? a.kv[x % a.N0] : a.kv[x];
}
template <bool IMPL> __device__ __forceinline__ int64_t sv_of(const LvArgs& a, int64_t x) {
    return IMPL ? a.sv[x % a.N0] : a.sv[x];
}
__device__ __forceinline__ int bucket_of(const LvArgs& a, int32_t r, int64_t x) {
    const uint32_t xl = (uint32_t)(x - a.roff[r]);
    return (int)(hash32(a.rkey[r] ^ hash32(xl)) % (uint32_t)a.B);
}
__device__ __forceinline__ bool in_bucket(const LvArgs& a, int32_t r, int64_t x, int bucket) {
    return bucket_of(a, r, x) == bucket;
}
__device__ __forceinline__ uint32_t tie_of(const LvArgs& a, int32_t r, int64_t x, int32_t c) {
    return hash32(hash32(a.rkey[r] ^ 0x5bd1e995u ^ (uint32_t)(x - a.roff[r])) ^ (uint32_t)(c - a.roff[r]));
}
// larger score, then larger tie hash, then smaller id; c < 0 = none
__device__ __forceinline__ bool lv_better(long long s1, uint32_t h1, int32_t c1, long long s2, uint32_t h2, int32_t c2) {
    if (c1 < 0) return false;
    if (c2 < 0) return true;
    if (s1 != s2) return s1 > s2;
    if (h1 != h2) return h1 > h2;
    return c1 < c2;
}
// Infomap candidate scan over table slots [0, ts) by a group of GL lanes (a power of two
// dividing 64, aligned): the most negative delta-L, reduced inside the group
__device__ __forceinline__ void wsync();
// The group's candidates (occupied slots other than the own module) are first compacted to the
// front of its table, in place (a slot's compacted index never exceeds it, and a pass reads its
// GL slots before any lane writes), so the map-equation terms -- five double logarithms per
// candidate, ~450 VALU instructions -- run on full lanes: a 64-slot table of a 27-entry row held
// ~10-27 candidates, and every lane paid for the slots of the busiest one.  The best candidate
// is a total order (delta, tie hash, id), so the evaluation order does not change it.
template <int GL = 64>
__device__ __forceinline__ void wave_scan_info(const LvArgs& a, int32_t* keys, int32_t* vals, uint32_t ts,
                                               int32_t own, long long kvx, long long svx, long long wown, int32_t r,
                                               int64_t x, double& bd, uint32_t& bh, int32_t& bc, int32_t& bw,
                                               int& ncand, const Log2Entry* lt) {
    const int lane = threadIdx.x & 63, gl = lane & (GL - 1);
    bd = 0.0; bh = 0; bc = -1; bw = 0;
    const long long Q = a.qrep[r];
    const longlong2 mo = *(const longlong2*)(a.mod + 2 * (int64_t)own);
    const InfoA A = info_a(a.inv, Q, mo.y, mo.x, kvx, svx, wown, lt);
    const unsigned long long gmask = GL == 64 ? ~0ull : (((1ull << GL) - 1) << (lane & ~(GL - 1)));
    const unsigned long long below = gmask & ((1ull << lane) - 1);
    uint32_t n = 0;
    for (uint32_t s0 = 0; s0 < ts; s0 += GL) {   // ts: a power of two >= 64 >= GL
        const int32_t k = keys[s0 + gl], v = vals[s0 + gl];
        const bool ok = k >= 0 && k != own;
        const unsigned long long b = __ballot(ok) & gmask;
        if (ok) {
            const uint32_t p = n + (uint32_t)__popcll(b & below);
            keys[p] = k;
            vals[p] = v;
        }
        n += (uint32_t)__popcll(b);
    }
    wsync();
    for (uint32_t ci = gl; ci < n; ci += GL) {
        const int32_t k = keys[ci], v = vals[ci];
        const longlong2 mk = *(const longlong2*)(a.mod + 2 * (int64_t)k);   // flow, exit
        ++ncand;
        const double d = info_b(a.inv, A, Q, mk.y, mk.x, kvx, svx, v, lt);
        const uint32_t h = tie_of(a, r, x, k);
        if (info_better(d, h, k, bd, bh, bc)) { bd = d; bh = h; bc = k; bw = v; }
    }
    for (int off = GL / 2; off; off >>= 1) {
        const double d2 = __shfl_xor(bd, off);
        const uint32_t h2 = __shfl_xor(bh, off);
        const int32_t c2 = __shfl_xor(bc, off);
        const int32_t w2 = __shfl_xor(bw, off);
        if (info_better(d2, h2, c2, bd, bh, bc)) { bd = d2; bh = h2; bc = c2; bw = w2; }
    }
}
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}
// insert (k, w); returns the slot if this call created it, else -1
__device__ __forceinline__ int tins(int32_t* keys, int32_t* vals, uint32_t nslots, bool pow2, int32_t k, int32_t w) {
    uint32_t h = hash32((uint32_t)k);
    h = pow2 ? (h & (nslots - 1)) : (h % nslots);
    while (true) {
        const int32_t prev = atomicCAS(&keys[h], -1, k);
        if (prev == -1) { atomicAdd(&vals[h], w); return (int)h; }
        if (prev == k) { atomicAdd(&vals[h], w); return -1; }
        h = (h + 1 == nslots) ? 0 : h + 1;
    }
}

// One row's entries j = j0, j0 + ST, ... < re into the table, UNR entries per thread in flight
// (columns and weights, then the label gathers, then the inserts: a thread's gathers overlap
// instead of forming a chain of UNR round trips).  Entries in the own community are summed
// into wl; refine only counts neighbours inside the move-phase community pc.  Global tables
// (lst != nullptr) list the slots they create.
template <int MODE, int UNR>
__device__ __forceinline__ void row_insert(const LvArgs& a, int64_t base, int64_t j0, int64_t re, int ST, int32_t own,
                                           int32_t pc, int32_t* keys, int32_t* vals, uint32_t ts, long long& wl,
                                           int32_t* lst, int* s_n) {
    for (int64_t j = j0; j < re; j += (int64_t)ST * UNR) {
        int64_t y[UNR];
        int32_t wy[UNR], cy[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const int64_t jj = j + (int64_t)u * ST;
            const bool ok = jj < re;
            y[u] = ok ? base + a.col[jj] : -1;
            wy[u] = ok ? (a.w ? a.w[jj] : 1) : 0;
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) cy[u] = y[u] >= 0 ? a.P[y[u]] : -1;
        if (MODE == MODE_REFINE) {
#pragma unroll
            for (int u = 0; u < UNR; ++u) cy[u] = (y[u] >= 0 && cy[u] == pc) ? a.R[y[u]] : -1;
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            if (y[u] < 0) continue;
            if (cy[u] < 0) continue;
            // entries in the own community are summed in registers, not inserted: on aggregated
            // levels they are a large share of a row, all on one LDS address
            if (cy[u] == own) { wl += wy[u]; continue; }
            const int sl = tins(keys, vals, ts, true, cy[u], wy[u]);
            if (lst && sl >= 0) lst[atomicAdd(s_n, 1)] = sl;
        }
    }
}

// Candidate evaluation shared by the light and heavy deciders.  Returns the target or -1.
// stay = w_v,own*2M - k_v*(Sigma_own - k_v); a candidate c scores w_vc*2M - k_v*Sigma_c.
// Move iff the best score beats stay; move phase only: an empty community (score 0, taken
// as v's own id when that community is empty) when both are negative (leidenalg considers
// the empty community, ModularityVertexPartition).
template <int MODE>
__device__ __forceinline__ int32_t lv_final(const LvArgs& a, int64_t x, int32_t own, long long kvx, long long wown,
                                            long long bs, int32_t bc) {
    const long long stay = wown * a.M2 - kvx * (a.tot[own] - kvx);
    int32_t t = -1;
    if (bc >= 0 && bs > stay) t = bc;
    if (MODE == MODE_MOVE && stay < 0 && (t < 0 || bs < 0) && own != (int32_t)x && a.tot[x] == 0) t = (int32_t)x;
    return t;
}

// Table size for a row of d entries: the power of two >= 2d, at least 64.
__device__ __forceinline__ uint32_t tsize(int64_t d) {
    uint32_t t = 64;
    while ((int64_t)t < 2 * d) t <<= 1;
    return t;
}

// Wave-level candidate scan over table slots [0, ts): best (score, tie, community) and the
// weight to the own community, reduced over the wave.  The occupied slots are packed to the
// front of the table first (as in wave_scan_info): a table of ts >= 2d slots is at least half
// empty, and each pass over GL slots is one dependent round trip (LDS read, Sigma gather).
template <int GL = 64>
__device__ __forceinline__ void wave_scan(const LvArgs& a, int32_t* keys, int32_t* vals, uint32_t ts,
                                          int32_t own, long long kvx, int32_t r, int64_t x, long long& bs,
                                          uint32_t& bh, int32_t& bc, long long& wown, int& ncand) {
    const int lane = threadIdx.x & 63, gl = lane & (GL - 1);
    bs = LLONG_MIN; bh = 0; bc = -1;   // wown: this lane's own-community weight (not in the table)
    const unsigned long long gmask = GL == 64 ? ~0ull : (((1ull << GL) - 1) << (lane & ~(GL - 1)));
    const unsigned long long below = gmask & ((1ull << lane) - 1);
    uint32_t n = 0;
    for (uint32_t s0 = 0; s0 < ts; s0 += GL) {   // ts: a power of two >= 64 >= GL
        const int32_t k = keys[s0 + gl], v = vals[s0 + gl];
        const bool ok = k >= 0;
        const unsigned long long b = __ballot(ok) & gmask;
        if (ok) {
            const uint32_t p = n + (uint32_t)__popcll(b & below);
            keys[p] = k;
            vals[p] = v;
        }
        n += (uint32_t)__popcll(b);
    }
    wsync();
    for (uint32_t ci = gl; ci < n; ci += GL) {
        const int32_t k = keys[ci];
        const long long val = vals[ci];
        const long long tk = a.tot[k];
        ++ncand;
        const long long sc = val * a.M2 - kvx * tk;
        const uint32_t h = tie_of(a, r, x, k);
        if (lv_better(sc, h, k, bs, bh, bc)) { bs = sc; bh = h; bc = k; }
    }
    (void)own;
    for (int off = GL / 2; off; off >>= 1) {
        const long long s2 = __shfl_xor(bs, off);
        const uint32_t h2 = __shfl_xor(bh, off);
        const int32_t c2 = __shfl_xor(bc, off);
        wown += __shfl_xor(wown, off);
        if (lv_better(s2, h2, c2, bs, bh, bc)) { bs = s2; bh = h2; bc = c2; }
    }
}

#ifndef FC_LV_XCD
#define FC_LV_XCD 1                     // XCD-contiguous chunks of the Infomap pass lists (A/B switch)
#endif
// Block b of a grid of nb -> chunk index, a bijection of [0, nb): the blocks of XCD x = b % 8
// (the hardware dispatches workgroups round-robin over the 8 XCDs) take the contiguous chunk
// range that starts at x * (nb / 8) + min(x, nb % 8).
__device__ __forceinline__ uint32_t xcd_chunk(uint32_t b, uint32_t nb) {
    const uint32_t x = b & 7, q = nb >> 3, rem = nb & 7;
    return x * q + min(x, rem) + (b >> 3);
}
// One bucket's decisions.  Each lane owns one union vertex; a wave ballots the eligible
// ones and decides them one at a time cooperatively: the row over the 64 lanes into an LDS
// table sized for it (64..LWS slots).  Rows longer than LIGHT go to k_lv_heavy.  Movers are
// listed per block and stamped in mvt (the apply kernel decides the neighbours' queue
// flags from the bucket's final state, so the result does not depend on thread timing).
// TS: LDS slots per wave -- LWS, or LWS_SMALL when every row of the level is short (the input
// graph: 8 KB of LDS per block instead of 32 KB, so 32 waves per CU instead of 20).
// G: vertices a wave decides at once (64/G lanes and TS/G slots each): G = 4 on short-row
// levels, where a 64-lane vertex left most lanes idle (LFR: 27 entries per row).
template <bool IMPL, int MODE, int TS, int G>
__global__ __launch_bounds__(LTB) void k_lv_decide(LvArgs a, int bucket, uint32_t stamp) {
    constexpr int GL = 64 / G, TSG = TS / G;
    __shared__ int32_t skey[LTB / 64][TS], sval[LTB / 64][TS];
    __shared__ int s_cnt;
    __shared__ uint32_t s_bytes;
    __shared__ Log2Entry s_lt[MODE == MODE_INFO ? 49 : 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x == 0) { s_cnt = 0; s_bytes = 0; }
    if (MODE == MODE_INFO && threadIdx.x < 49) s_lt[threadIdx.x] = c_log2[threadIdx.x];
    __syncthreads();
    // this lane's share of the algorithmic bytes (scanned / decided vertices, movers, entries,
    // candidates), ONE accumulator: five counters cost the Infomap instance an occupancy step
    // (88 -> 100 VGPRs, 5 -> 4 waves per SIMD: LFR-100k infomap 5.31 -> 5.82 s)
    uint32_t c_b = 0;
    const uint32_t eb = (uint32_t)lv_entry_bytes<MODE>(a.w != nullptr);
    int64_t x0 = (int64_t)blockIdx.x * LTB + threadIdx.x;
    const bool listed = MODE == MODE_INFO && a.ilist != nullptr;
    if (listed) {
        // the pass list is replica-major inside a bucket; XCD x (blocks b % 8 == x, round-robin
        // dispatch) takes one contiguous run of its chunks, so an XCD's L2 serves few replicas'
        // module and label rows at a time (decide block slots blist / bcnt stay by blockIdx)
        if (FC_LV_XCD) x0 = (int64_t)xcd_chunk(blockIdx.x, gridDim.x) * LTB + threadIdx.x;
        x0 = x0 < a.icnt ? (int64_t)a.ilist[x0] : a.nU;
    } else if (IMPL && a.bmap) {
        const int64_t loc = (int64_t)(blockIdx.x % a.bpr) * LTB + threadIdx.x;
        x0 = loc < a.N0 ? (int64_t)a.bmap[blockIdx.x / a.bpr] * a.N0 + loc : a.nU;
    }
    bool elig = false;
    if (listed) {
        // the pass list holds exactly this bucket's vertices of the replicas still moving
        elig = x0 < a.nU;
        c_b = elig ? 4u : 0u;
    } else if (x0 < a.nU) {
        // the eligibility scan: replica id (explicit levels), queue flag / refined size
        c_b = (IMPL ? 0 : 4) + (MODE == MODE_MOVE ? 1 : MODE == MODE_REFINE ? 8 : 0);
        const int32_t r = rep_of<IMPL>(a, x0);
        if (!a.done[r] && in_bucket(a, r, x0, bucket)) {
            if (MODE == MODE_MOVE) {
                elig = a.act[x0] != 0;
                if (elig) a.act[x0] = 0;   // popped from the queue
            } else if (MODE == MODE_REFINE) {
                elig = a.rsize[a.R[x0]] == 1;   // only nodes still alone in their refined community
            } else {
                elig = !a.lvdone[r];            // Infomap: full passes until the replica's pass moves nothing
            }
        }
    }
    // long rows go to k_lv_heavy, listed by length tier: one append per wave and tier (ballot +
    // one atomic)
    bool hv = false;
    int tier = -1;
    if (elig) {
        const int64_t xr0 = IMPL ? x0 % a.N0 : x0;
        const int64_t d0 = a.rowptr[xr0 + 1] - a.rowptr[xr0];
        hv = d0 > TS / G / 2;
        if (hv) tier = heavy_tier(d0);
    }
    if (__ballot(hv)) {
        for (int t = 0; t < NTIER; ++t) {
            const unsigned long long hmask = __ballot(tier == t);
            if (!hmask) continue;
            int hb = 0;
            if (lane == 0) hb = atomicAdd(a.heavy_cnt + t, __popcll(hmask));
            hb = __shfl(hb, 0);
            if (tier == t) a.heavy[t * a.hcap + hb + __popcll(hmask & ((1ull << lane) - 1))] = (int32_t)x0;
        }
    }
    unsigned long long mask = __ballot(elig && !hv);
    const int grp = lane / GL, gl = lane & (GL - 1);
    int32_t* keys = skey[wv] + grp * TSG;
    int32_t* vals = sval[wv] + grp * TSG;
    while (mask) {
        // group g takes the g-th remaining eligible lane (every lane computes the same split)
        int myl = -1;
        for (int g = 0; g < G; ++g) {
            if (!mask) break;
            const int l = __ffsll((long long)mask) - 1;
            mask &= mask - 1;
            if (g == grp) myl = l;
        }
        const int64_t x = __shfl(x0, myl < 0 ? 0 : myl);
        const bool valid = myl >= 0;
        const int64_t base = IMPL ? (x / a.N0) * a.N0 : 0;
        const int64_t xr = IMPL ? x - base : x;
        const int64_t rb = valid ? a.rowptr[xr] : 0, re = valid ? a.rowptr[xr + 1] : 0;
        const uint32_t ts = tsize(re - rb);
        for (uint32_t s = gl; s < ts; s += GL) { keys[s] = -1; vals[s] = 0; }
        wsync();
        const int32_t own = valid ? (MODE == MODE_REFINE ? a.R[x] : a.P[x]) : -1;
        const int32_t pc = valid ? a.P[x] : -1;
        long long wl = 0;   // Infomap: weight to the own module
        // the vertex's record and its row's entries, counted once by the group's first lane
        c_b += (valid && gl == 0) ? (uint32_t)lv_vertex_bytes<MODE>() + (uint32_t)(re - rb) * eb : 0u;
        row_insert<MODE, 1>(a, base, rb + gl, re, GL, own, pc, keys, vals, ts, wl, nullptr, nullptr);
        wsync();
        const long long kvx = valid ? kv_of<IMPL>(a, x) : 0;
        const int32_t rx = valid ? rep_of<IMPL>(a, x) : 0;
        long long bs, wown;
        uint32_t bh;
        int32_t bc, bw = 0;
        int ncand = 0;
        if (MODE == MODE_INFO) {
            for (int off = GL / 2; off; off >>= 1) wl += __shfl_xor(wl, off);
            wown = wl;
            double bd = 0.0;
            if (valid) {
                wave_scan_info<GL>(a, keys, vals, ts, own, kvx, sv_of<IMPL>(a, x), wown, rx, x, bd, bh, bc, bw, ncand,
                                   s_lt);
            } else {
                bc = -1;
            }
            if (!(bd < -INFO_MIN_GAIN)) bc = -1;
            bs = 0;
        } else {
            wown = wl;
            wave_scan<GL>(a, keys, vals, ts, own, kvx, rx, x, bs, bh, bc, wown, ncand);
        }
        c_b += valid ? (uint32_t)ncand * (uint32_t)lv_cand_bytes<MODE>() : 0u;
        if (valid && gl == 0) {
            const int32_t t = MODE == MODE_INFO ? bc : lv_final<MODE>(a, x, own, kvx, wown, bs, bc);
            if (t >= 0) {
                c_b += (uint32_t)lv_mover_bytes<MODE>();
                const int p = atomicAdd(&s_cnt, 1);
                const int64_t q = (int64_t)blockIdx.x * LTB + p;
                a.blist[q] = (int32_t)x;
                a.btgt[q] = t;
                if (MODE != MODE_REFINE) a.mvt[x] = ((unsigned long long)stamp << 32) | (uint32_t)t;
                if (MODE == MODE_INFO) a.mvo[x] = own;
            }
        }
        wsync();
    }
    // the block's bytes through one LDS word (a 64-bit wave reduction here cost the Infomap
    // instance 10 VGPRs: 90 -> 100, one occupancy step)
    if (c_b) atomicAdd(&s_bytes, c_b);
    __syncthreads();
    if (threadIdx.x == 0) {
        a.bcnt[blockIdx.x] = s_cnt;
        if (s_bytes) atomicAdd(a.lvb + (blockIdx.x & (MSH - 1)), (unsigned long long)s_bytes);
    }
}

// Block reduction of (score, tie, community) candidates; thread 0 ends with the best.
struct BRed {
    long long s[LTB / 64];
    uint32_t h[LTB / 64];
    int32_t c[LTB / 64];
    long long wown[LTB / 64];
};
__device__ __forceinline__ void block_best(BRed& red, long long& bs, uint32_t& bh, int32_t& bc, long long& wown) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int off = 32; off; off >>= 1) {
        const long long s2 = __shfl_xor(bs, off);
        const uint32_t h2 = __shfl_xor(bh, off);
        const int32_t c2 = __shfl_xor(bc, off);
        wown += __shfl_xor(wown, off);
        if (lv_better(s2, h2, c2, bs, bh, bc)) { bs = s2; bh = h2; bc = c2; }
    }
    if (lane == 0) { red.s[wv] = bs; red.h[wv] = bh; red.c[wv] = bc; red.wown[wv] = wown; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < LTB / 64; ++k) {
            wown += red.wown[k];
            if (lv_better(red.s[k], red.h[k], red.c[k], bs, bh, bc)) { bs = red.s[k]; bh = red.h[k]; bc = red.c[k]; }
        }
    }
    __syncthreads();
}

struct BRedI {
    double d[LTB / 64];
    uint32_t h[LTB / 64];
    int32_t c[LTB / 64];
    int32_t w[LTB / 64];
};
__device__ __forceinline__ void block_best_info(BRedI& red, double& bd, uint32_t& bh, int32_t& bc, int32_t& bw) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int off = 32; off; off >>= 1) {
        const double d2 = __shfl_xor(bd, off);
        const uint32_t h2 = __shfl_xor(bh, off);
        const int32_t c2 = __shfl_xor(bc, off);
        const int32_t w2 = __shfl_xor(bw, off);
        if (info_better(d2, h2, c2, bd, bh, bc)) { bd = d2; bh = h2; bc = c2; bw = w2; }
    }
    if (lane == 0) { red.d[wv] = bd; red.h[wv] = bh; red.c[wv] = bc; red.w[wv] = bw; }
    __syncthreads();
    if (threadIdx.x == 0)
        for (int k = 1; k < LTB / 64; ++k)
            if (info_better(red.d[k], red.h[k], red.c[k], bd, bh, bc)) {
                bd = red.d[k]; bh = red.h[k]; bc = red.c[k]; bw = red.w[k];
            }
    __syncthreads();
}

// Long rows: one block per vertex; an LDS table of up to HLS slots, or (rows > HLIGHT) a
// global table per block, cleared through the list of slots it created.
template <bool IMPL, int MODE, int HS>
__global__ __launch_bounds__(LTB) void k_lv_heavy(LvArgs a, uint32_t stamp, int tier) {
    // HS: LDS slots (HLS, or HLS/2 when no row of the level is longer than HLS/4: 32 KB instead
    // of 64 KB per block, so 4-5 blocks per CU instead of 2)
    __shared__ int32_t lkey[HS], lval[HS];
    __shared__ int s_n;
    __shared__ long long s_wown;
    __shared__ BRed red;
    __shared__ BRedI redi;
    __shared__ Log2Entry s_lt[MODE == MODE_INFO ? 49 : 1];
    if (MODE == MODE_INFO && threadIdx.x < 49) s_lt[threadIdx.x] = c_log2[threadIdx.x];   // (synced below)
    const int n = a.heavy_cnt[tier];
    const int32_t* hlist = a.heavy + tier * a.hcap;
    int32_t* htgt = a.htgt + tier * a.hcap;
    uint32_t c_b = 0;   // this thread's share of the algorithmic bytes
    const uint32_t eb = (uint32_t)lv_entry_bytes<MODE>(a.w != nullptr);
    int32_t* gkey = a.hkey + (int64_t)blockIdx.x * a.hslots;
    int32_t* gval = a.hval + (int64_t)blockIdx.x * a.hslots;
    int32_t* lst = a.hlst + (int64_t)blockIdx.x * a.hslots;
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        const int64_t x = hlist[i];
        const int64_t base = IMPL ? (x / a.N0) * a.N0 : 0;
        const int64_t xr = IMPL ? x - base : x;
        const int64_t rb = a.rowptr[xr], re = a.rowptr[xr + 1];
        const bool lds = re - rb <= HS / 2;
        const uint32_t ts = lds ? tsize(re - rb) : (uint32_t)a.hslots;
        int32_t* keys = lds ? lkey : gkey;
        int32_t* vals = lds ? lval : gval;
        if (threadIdx.x == 0) { s_n = 0; s_wown = 0; }
        if (lds)
            for (uint32_t s = threadIdx.x; s < ts; s += LTB) { lkey[s] = -1; lval[s] = 0; }
        __syncthreads();
        const int32_t own = MODE == MODE_REFINE ? a.R[x] : a.P[x];
        const int32_t pc = a.P[x];
        long long wl = 0;
        c_b += threadIdx.x == 0 ? (uint32_t)(lv_vertex_bytes<MODE>() + 4 /* heavy list */ + 4 /* htgt */) +
                                      (uint32_t)(re - rb) * eb : 0u;
        row_insert<MODE, UNR>(a, base, rb + threadIdx.x, re, LTB, own, pc, keys, vals, ts, wl, lds ? nullptr : lst,
                         &s_n);
        if (MODE == MODE_INFO && wl) atomicAdd((unsigned long long*)&s_wown, (unsigned long long)wl);
        __syncthreads();
        const long long kvx = kv_of<IMPL>(a, x);
        const int32_t r = rep_of<IMPL>(a, x);
        long long bs = LLONG_MIN, wown = MODE == MODE_INFO ? s_wown : wl;   // move/refine: summed by block_best
        double bd = 0.0;
        uint32_t bh = 0;
        int32_t bc = -1, bw = 0;
        const int cnt = lds ? (int)ts : s_n;
        InfoA IA{};
        if (MODE == MODE_INFO) {
            const longlong2 mo = *(const longlong2*)(a.mod + 2 * (int64_t)own);
            IA = info_a(a.inv, a.qrep[r], mo.y, mo.x, kvx, sv_of<IMPL>(a, x), wown, s_lt);
        }
        const long long qr = MODE == MODE_INFO ? a.qrep[r] : 0;
        const long long svx = MODE == MODE_INFO ? sv_of<IMPL>(a, x) : 0;
        for (int q0 = threadIdx.x; q0 < cnt; q0 += LTB * UNR) {   // UNR slots' gathers in flight
            int32_t k[UNR];
            long long val[UNR], tk[UNR], tk2[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                const int q = q0 + u * LTB;
                k[u] = -1; val[u] = 0;
                if (q < cnt) {
                    const int sl = lds ? q : lst[q];
                    k[u] = keys[sl];
                    val[u] = vals[sl];
                    if (!lds) { gkey[sl] = -1; gval[sl] = 0; }   // clear for the next vertex (read before)
                }
            }
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                tk[u] = tk2[u] = 0;
                if (k[u] < 0) continue;
                if (MODE == MODE_INFO) {
                    const longlong2 mk = *(const longlong2*)(a.mod + 2 * (int64_t)k[u]);
                    tk[u] = mk.x; tk2[u] = mk.y;
                } else {
                    tk[u] = a.tot[k[u]];
                }
            }
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                if (k[u] < 0) continue;
                c_b += (uint32_t)lv_cand_bytes<MODE>();
                const uint32_t h = tie_of(a, r, x, k[u]);
                if (MODE == MODE_INFO) {
                    const double d = info_b(a.inv, IA, qr, tk2[u], tk[u], kvx, svx, val[u], s_lt);
                    if (info_better(d, h, k[u], bd, bh, bc)) { bd = d; bh = h; bc = k[u]; bw = (int32_t)val[u]; }
                } else {
                    const long long sc = val[u] * a.M2 - kvx * tk[u];
                    if (lv_better(sc, h, k[u], bs, bh, bc)) { bs = sc; bh = h; bc = k[u]; }
                }
            }
        }
        if (MODE == MODE_INFO) {
            block_best_info(redi, bd, bh, bc, bw);
            if (threadIdx.x == 0) {
                const int32_t t = (bc >= 0 && bd < -INFO_MIN_GAIN) ? bc : -1;
                htgt[i] = t;
                if (t >= 0) { a.mvt[x] = ((unsigned long long)stamp << 32) | (uint32_t)t; a.mvo[x] = own; }
            }
        } else {
            block_best(red, bs, bh, bc, wown);
            if (threadIdx.x == 0) {
                const int32_t t = lv_final<MODE>(a, x, own, kvx, wown, bs, bc);
                htgt[i] = t;
                if (MODE == MODE_MOVE && t >= 0) a.mvt[x] = ((unsigned long long)stamp << 32) | (uint32_t)t;
            }
        }
        __syncthreads();
    }
    __shared__ uint32_t s_bytes;                      // the block's bytes through one LDS word (k_lv_decide)
    if (threadIdx.x == 0) s_bytes = 0;
    __syncthreads();
    if (c_b) atomicAdd(&s_bytes, c_b);
    __syncthreads();
    if (threadIdx.x == 0 && s_bytes) atomicAdd(a.lvb + MSH + (blockIdx.x & (MSH - 1)), (unsigned long long)s_bytes);
}

// Apply one bucket's moves, one wave per mover: blocks [0, nblk) take the decide blocks'
// lists, the rest the heavy decisions.  Lane 0 moves the vertex (move phase: P and Sigma;
// refine: R, Sigma and sizes); in the move phase the lanes then queue the neighbours whose
// community at the END of the bucket differs from the target (a neighbour that moves in
// this bucket is judged by its stamped target, the others by P, which this bucket leaves
// alone), so the queue flags do not depend on thread timing.
// GL lanes per mover (a power of two dividing 64): lane 0 of the group moves the vertex, the
// group walks its row.
template <bool IMPL, int MODE, int GL = 64>
__device__ __forceinline__ void lv_move(const LvArgs& a, int64_t x, int32_t t, uint32_t stamp, unsigned long long& mv) {
    const int lane = threadIdx.x & (GL - 1);
    if (lane == 0) {
        const long long kvx = kv_of<IMPL>(a, x);
        int32_t* lab = MODE == MODE_REFINE ? a.R : a.P;
        const int32_t old = lab[x];
        lab[x] = t;
        int64_t* tt = MODE == MODE_INFO ? a.mod + 2 * (int64_t)t : a.tot + t;
        int64_t* to = MODE == MODE_INFO ? a.mod + 2 * (int64_t)old : a.tot + old;
        atomicAdd((unsigned long long*)tt, (unsigned long long)kvx);
        atomicAdd((unsigned long long*)to, (unsigned long long)(-kvx));
        if (MODE == MODE_REFINE) {
            atomicAdd(&a.rsize[t], 1);
            atomicAdd(&a.rsize[old], -1);
        }
        ++mv;
    }
    if (MODE == MODE_INFO) {
        // exact module exit weights under simultaneous moves: every edge at a mover changes the
        // exits of its ends' modules from the bucket's before-labels to its after-labels (a
        // neighbour that moves in this bucket is read from its stamped records; an edge between
        // two movers is counted by the smaller id only)
        const int64_t base = IMPL ? (x / a.N0) * a.N0 : 0;
        const int64_t xr = IMPL ? x - base : x;
        const int32_t xo = a.mvo[x];
        const int64_t re = a.rowptr[xr + 1];
        long long dq = 0, sxo = 0, st = 0;   // this lane's deltas of xo's and t's exits
        for (int64_t j = a.rowptr[xr] + lane; j < re; j += GL) {
            const int64_t y = base + a.col[j];
            const long long w = a.w ? a.w[j] : 1;
            const unsigned long long my = a.mvt[y];
            int32_t yo, yn;
            if ((uint32_t)(my >> 32) == stamp) {
                if (y < x) continue;
                yo = a.mvo[y];
                yn = (int32_t)(uint32_t)my;
            } else {
                yo = yn = a.P[y];
            }
            // -w at xo and yo if the edge was cut, +w at t and yn if it is.  xo's and t's deltas
            // are summed over the row (two atomics per mover); y's modules take an atomic only when
            // they are neither (a neighbour staying in a third module: none, its -w and +w cancel)
            long long dyo = 0, dyn = 0;
            if (xo != yo) { sxo -= w; dyo -= w; dq -= 2 * w; }
            if (t != yn) { st += w; dyn += w; dq += 2 * w; }
            if (yo == yn) { dyo += dyn; dyn = 0; }
            if (yo == xo) { sxo += dyo; dyo = 0; } else if (yo == t) { st += dyo; dyo = 0; }
            if (yn == xo) { sxo += dyn; dyn = 0; } else if (yn == t) { st += dyn; dyn = 0; }
            if (dyo) atomicAdd((unsigned long long*)&a.mod[2 * (int64_t)yo + 1], (unsigned long long)dyo);
            if (dyn) atomicAdd((unsigned long long*)&a.mod[2 * (int64_t)yn + 1], (unsigned long long)dyn);
        }
        for (int off = GL / 2; off; off >>= 1) {
            dq += __shfl_xor(dq, off);
            sxo += __shfl_xor(sxo, off);
            st += __shfl_xor(st, off);
        }
        if (lane == 0) {
            if (sxo) atomicAdd((unsigned long long*)&a.mod[2 * (int64_t)xo + 1], (unsigned long long)sxo);
            if (st) atomicAdd((unsigned long long*)&a.mod[2 * (int64_t)t + 1], (unsigned long long)st);
            if (dq) atomicAdd((unsigned long long*)&a.qrep[rep_of<IMPL>(a, x)], (unsigned long long)dq);
        }
    }
    if (MODE == MODE_MOVE) {
        const int64_t base = IMPL ? (x / a.N0) * a.N0 : 0;
        const int64_t xr = IMPL ? x - base : x;
        const int64_t re = a.rowptr[xr + 1];
        for (int64_t j = a.rowptr[xr] + lane; j < re; j += GL) {
            const int64_t y = base + a.col[j];
            const unsigned long long my = a.mvt[y];
            const int32_t fin = (uint32_t)(my >> 32) == stamp ? (int32_t)(uint32_t)my : a.P[y];
            if (fin != t) a.act[y] = 1;
        }
    }
}
template <bool IMPL, int MODE>
__global__ __launch_bounds__(LTB) void k_lv_apply(LvArgs a, int nblk, int hblk, uint32_t stamp) {
    // Infomap: moves per replica (a decide block's 256 union ids span at most two replicas of the
    // input graph: LDS counters for those, global atomics otherwise)
    __shared__ unsigned long long s_rm[2];
    unsigned long long mv = 0;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int32_t r0 = 0;
    if (MODE == MODE_INFO) {
        if (threadIdx.x < 2) s_rm[threadIdx.x] = 0;
        if ((int)blockIdx.x < nblk) {
            if (a.ilist)   // a list block's vertices: mostly one replica, that of its first mover
                r0 = a.bcnt[blockIdx.x] ? rep_of<IMPL>(a, a.blist[(int64_t)blockIdx.x * LTB]) : 0;
            else
                r0 = (IMPL && a.bmap) ? a.bmap[blockIdx.x / a.bpr] : rep_of<IMPL>(a, (int64_t)blockIdx.x * LTB);
        }
        __syncthreads();
    }
    auto count_rep = [&](int64_t x, int gl) {
        if (MODE != MODE_INFO || gl != 0) return;
        const int32_t r = rep_of<IMPL>(a, x);
        if ((int)blockIdx.x < nblk && (uint32_t)(r - r0) < 2u) atomicAdd(&s_rm[r - r0], 1ull);
        else atomicAdd(&a.rmoves[r], 1ull);
    };
    if ((int)blockIdx.x < nblk) {
        // Infomap's input-graph level: 16 lanes per mover (rows of ~27 entries; a wave per mover
        // left most lanes idle through each row's chain of dependent gathers and atomics)
        constexpr int AG = (MODE == MODE_INFO && IMPL) ? 16 : 64;
        const int n = a.bcnt[blockIdx.x];
        for (int i = wv * (64 / AG) + lane / AG; i < n; i += (LTB / 64) * (64 / AG)) {
            const int64_t q = (int64_t)blockIdx.x * LTB + i;
            lv_move<IMPL, MODE, AG>(a, a.blist[q], a.btgt[q], stamp, mv);
            count_rep(a.blist[q], lane & (AG - 1));
        }
    } else {
        for (int tier = 0; tier < NTIER; ++tier) {
            const int n = a.heavy_cnt[tier];
            const int32_t* hl = a.heavy + tier * a.hcap;
            const int32_t* ht = a.htgt + tier * a.hcap;
            for (int i = (blockIdx.x - nblk) * (LTB / 64) + wv; i < n; i += hblk * (LTB / 64)) {
                const int32_t t = ht[i];
                if (t >= 0) {
                    lv_move<IMPL, MODE>(a, hl[i], t, stamp, mv);
                    count_rep(hl[i], lane);
                }
            }
        }
    }
    if (mv) atomicAdd(&a.moves[blockIdx.x & (MSH - 1)], mv);   // group leaders only
    if (MODE == MODE_INFO) {
        __syncthreads();
        if (threadIdx.x < 2 && s_rm[threadIdx.x]) atomicAdd(&a.rmoves[r0 + threadIdx.x], s_rm[threadIdx.x]);
    }
}

// ---------------------------------------------------------------- level bookkeeping kernels
__global__ void k_lv_init0(int64_t N, int n_r, const int32_t* lab, const int32_t* spos, int32_t* P, int32_t* R,
                           int64_t* rtot, int32_t* rsize, const int64_t* kdeg, int32_t* memb) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)n_r * N) return;
    const int64_t r = i / N, v = i - r * N;
    P[i] = (int32_t)(r * N + lab[r * N + spos[v]]);
    R[i] = (int32_t)i;
    rtot[i] = kdeg[v];
    rsize[i] = 1;
    memb[i] = (int32_t)i;
}
// singleton refined partition of an explicit level
__global__ void k_lv_rinit(int64_t nU, const int64_t* kv, int32_t* R, int64_t* rtot, int32_t* rsize) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nU) return;
    R[i] = (int32_t)i;
    rtot[i] = kv[i];
    rsize[i] = 1;
}
template <bool IMPL>
__global__ void k_ag_flags(LvArgs a, int32_t* flag) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c > a.nU) return;
    flag[c] = (c < a.nU && a.rsize[c] > 0 && !a.done[rep_of<IMPL>(a, c)]) ? 1 : 0;
}
// per replica: refined communities (from the scan) at the replica's first/last union id
__global__ void k_ag_counts(int n_r, const uint8_t* done, const int32_t* roff, const int32_t* rend, const int32_t* nid,
                            int32_t* out) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < n_r) out[r] = done[r] ? 0 : nid[rend[r]] - nid[roff[r]];   // finished: ranges are stale
}
template <bool IMPL>
__global__ void k_ag_nodes(LvArgs a, const int32_t* nid, int32_t* nrep, int64_t* nkv, int32_t* mcnt, int64_t* nsv) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.nU || nid[c + 1] == nid[c]) return;
    const int32_t xn = nid[c];
    nrep[xn] = rep_of<IMPL>(a, c);
    nkv[xn] = a.tot[c];   // rtot: the refined community's weighted degree
    mcnt[xn] = a.rsize[c];
    if (nsv) nsv[xn] = a.mod[2 * c + 1];   // Infomap: the module's exit weight = the new node's external weight
}
// pofR[R[x]] = P[x] (every member agrees: R refines P); prep[P] = min new id over members;
// ub[new id] += deg(x)
template <bool IMPL>
__global__ void k_ag_members(LvArgs a, const int32_t* nid, int32_t* pofR, int32_t* prep, int64_t* ub) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= a.nU) return;
    if (a.done[rep_of<IMPL>(a, x)]) return;
    const int32_t rc = a.R[x];
    pofR[rc] = a.P[x];
    const int32_t xn = nid[rc];
    atomicMin(&prep[a.P[x]], xn);
    const int64_t xr = IMPL ? x % a.N0 : x;
    atomicAdd((unsigned long long*)&ub[xn], (unsigned long long)(a.rowptr[xr + 1] - a.rowptr[xr]));
}
template <bool IMPL>
__global__ void k_ag_fill(LvArgs a, const int32_t* nid, const int32_t* moff, int32_t* mcur, int32_t* mlist) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= a.nU) return;
    if (a.done[rep_of<IMPL>(a, x)]) return;
    const int32_t xn = nid[a.R[x]];
    mlist[moff[xn] + atomicAdd(&mcur[xn], 1)] = (int32_t)x;
}
__global__ void k_ag_part(int64_t nU, const int32_t* nid, const int32_t* pofR, const int32_t* prep, int32_t* nP) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nU || nid[c + 1] == nid[c]) return;
    nP[nid[c]] = prep[pofR[c]];
}
__global__ void k_ag_ptot(int64_t nU, const int32_t* P, const int64_t* kv, int64_t* ptot) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x < nU) atomicAdd((unsigned long long*)&ptot[P[x]], (unsigned long long)kv[x]);
}
__global__ void k_ag_memb(int64_t total, int64_t N, const uint8_t* done, const int32_t* R, const int32_t* nid,
                          int32_t* memb) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total || done[i / N]) return;
    memb[i] = nid[R[memb[i]]];
}

// Lanes per member row when aggregating: the power of two >= the members' average row length,
// 4..cap (rows are walked by groups side by side; one group per member at a time)
__device__ __forceinline__ int ag_group(int64_t entries, int32_t members, int cap) {
    const int64_t avg = members > 0 ? (entries + members - 1) / members : 1;
    int g = 4;
    while (g < cap && g < avg) g <<= 1;
    return g;
}
// Aggregate rows: new vertex xn = refined community; its row = the members' rows mapped
// through nid[R[.]], self loops dropped, weights summed.  One wave per light new vertex
// (LDS table), heavy ones (member-row sum > LIGHT) are listed for k_ag_rows_heavy.  Rows
// are written at their upper-bound offsets ubo and compacted afterwards.
template <bool IMPL>
__global__ __launch_bounds__(LTB) void k_ag_rows(LvArgs a, int64_t nUn, const int32_t* nid, const int32_t* moff,
                                                 const int32_t* mlist, const int64_t* ubo, int32_t* ocol, int32_t* ow,
                                                 int32_t* olen, int32_t* hlist, int32_t* hcnt, int64_t hcap) {
    __shared__ int32_t skey[LTB / 64][LWS], sval[LTB / 64][LWS];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t xn = (int64_t)blockIdx.x * (LTB / 64) + wv;
    if (xn >= nUn) return;
    if (ubo[xn + 1] - ubo[xn] > LIGHT) {   // listed by length tier for k_ag_rows_heavy
        const int t = heavy_tier(ubo[xn + 1] - ubo[xn]);
        if (lane == 0) hlist[t * hcap + atomicAdd(hcnt + t, 1)] = (int32_t)xn;
        return;
    }
    int32_t* keys = skey[wv];
    int32_t* vals = sval[wv];
    const uint32_t ts = tsize(ubo[xn + 1] - ubo[xn]);
    for (uint32_t s = lane; s < ts; s += 64) { keys[s] = -1; vals[s] = 0; }
    wsync();
    // members side by side: groups of ga lanes (the member rows' average length, 4..64), so a
    // module of many short rows does not walk them one at a time
    const int ga = ag_group(ubo[xn + 1] - ubo[xn], moff[xn + 1] - moff[xn], 64);
    const int grp = lane / ga, gl = lane & (ga - 1);
    for (int32_t q = moff[xn] + grp; q < moff[xn + 1]; q += 64 / ga) {
        const int64_t x = mlist[q];
        const int64_t base = IMPL ? (x / a.N0) * a.N0 : 0;
        const int64_t xr = IMPL ? x - base : x;
        for (int64_t j = a.rowptr[xr] + gl; j < a.rowptr[xr + 1]; j += ga) {
            const int32_t yn = nid[a.R[base + a.col[j]]];
            if (yn != (int32_t)xn) tins(keys, vals, ts, true, yn, a.w ? a.w[j] : 1);
        }
    }
    wsync();
    int32_t cnt = 0;
    const int64_t o = ubo[xn];
    for (uint32_t s0 = 0; s0 < ts; s0 += 64) {
        const int32_t k = keys[s0 + lane];
        const unsigned long long bal = __ballot(k >= 0);
        if (k >= 0) {
            const int p = cnt + __popcll(bal & ((1ull << lane) - 1));
            ocol[o + p] = k;
            ow[o + p] = vals[s0 + lane];
        }
        cnt += __popcll(bal);
    }
    if (lane == 0) olen[xn] = cnt;
}
template <bool IMPL, int HS>
__global__ __launch_bounds__(LTB) void k_ag_rows_heavy(LvArgs a, const int32_t* nid, const int32_t* moff,
                                                       const int32_t* mlist, const int64_t* ubo, int32_t* ocol,
                                                       int32_t* ow, int32_t* olen, const int32_t* hlist_all,
                                                       const int32_t* hcnt, int64_t hcap, int tier) {
    __shared__ int32_t lkey[HS], lval[HS];   // sized for the tier's rows (tier 3: global tables)
    __shared__ int s_n;
    const int n = hcnt[tier];
    const int32_t* hlist = hlist_all + tier * hcap;
    int32_t* gkey = a.hkey + (int64_t)blockIdx.x * a.hslots;
    int32_t* gval = a.hval + (int64_t)blockIdx.x * a.hslots;
    int32_t* lst = a.hlst + (int64_t)blockIdx.x * a.hslots;
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        const int64_t xn = hlist[i];
        const int64_t ubn = ubo[xn + 1] - ubo[xn];
        const bool lds = ubn <= HS / 2;
        const uint32_t ts = lds ? tsize(ubn) : (uint32_t)a.hslots;
        int32_t* keys = lds ? lkey : gkey;
        int32_t* vals = lds ? lval : gval;
        if (threadIdx.x == 0) s_n = 0;
        if (lds)
            for (uint32_t s = threadIdx.x; s < ts; s += LTB) { lkey[s] = -1; lval[s] = 0; }
        __syncthreads();
        const int ga = ag_group(ubn, moff[xn + 1] - moff[xn], LTB);   // lanes per member (see k_ag_rows)
        const int grp = threadIdx.x / ga, gl = threadIdx.x & (ga - 1);
        for (int32_t q = moff[xn] + grp; q < moff[xn + 1]; q += LTB / ga) {
            const int64_t x = mlist[q];
            const int64_t base = IMPL ? (x / a.N0) * a.N0 : 0;
            const int64_t xr = IMPL ? x - base : x;
            for (int64_t j = a.rowptr[xr] + gl; j < a.rowptr[xr + 1]; j += ga) {
                const int32_t yn = nid[a.R[base + a.col[j]]];
                if (yn == (int32_t)xn) continue;
                const int s = tins(keys, vals, ts, true, yn, a.w ? a.w[j] : 1);
                if (!lds && s >= 0) lst[atomicAdd(&s_n, 1)] = s;
            }
        }
        __syncthreads();
        const int64_t o = ubo[xn];
        if (lds) {   // every slot of the LDS table; output positions from a block counter
            if (threadIdx.x == 0) s_n = 0;
            __syncthreads();
            for (uint32_t q = threadIdx.x; q < ts; q += LTB) {
                if (lkey[q] < 0) continue;
                const int p = atomicAdd(&s_n, 1);
                ocol[o + p] = lkey[q];
                ow[o + p] = lval[q];
            }
        } else {     // the global table through its created-slot list, cleared on the way
            for (int q = threadIdx.x; q < s_n; q += LTB) {
                const int s = lst[q];
                ocol[o + q] = gkey[s];
                ow[o + q] = gval[s];
                gkey[s] = -1; gval[s] = 0;
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) olen[xn] = s_n;
        __syncthreads();
    }
}
__global__ void k_ag_len64(int64_t n, const int32_t* len, int64_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= n) out[i] = i < n ? len[i] : 0;
}
// compact rows (entry order inside a row is the hash tables' and may vary between runs; no
// decision depends on it: table sums commute and candidates are ranked by a total order)
__global__ __launch_bounds__(LTB) void k_ag_compact(int64_t nUn, const int64_t* ubo, const int64_t* rp,
                                                    const int32_t* icol, const int32_t* iw, int32_t* ocol,
                                                    int32_t* ow) {
    const int lane = threadIdx.x & 63;
    const int64_t xn = (int64_t)blockIdx.x * (LTB / 64) + (threadIdx.x >> 6);
    if (xn >= nUn) return;
    const int64_t o = ubo[xn], d = rp[xn + 1] - rp[xn], q = rp[xn];
    for (int64_t k = lane; k < d; k += 64) { ocol[q + k] = icol[o + k]; ow[q + k] = iw[o + k]; }
}
__global__ void k_ag_roff(int64_t nU, const int32_t* rep, int32_t* roff, int32_t* rend) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= nU) return;
    if (x == 0 || rep[x - 1] != rep[x]) roff[rep[x]] = (int32_t)x;
    if (x == nU - 1 || rep[x + 1] != rep[x]) rend[rep[x]] = (int32_t)(x + 1);
}
// final labels of replica r (fin[r] = 1): lab[r][spos[v]] = P[memb[r*N+v]] - roff[r]
__global__ void k_lv_final(int64_t N, int n_r, const uint8_t* fin, const int32_t* memb, const int32_t* P,
                           const int32_t* roff, const int32_t* spos, int32_t* lab) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)n_r * N) return;
    const int64_t r = i / N, v = i - r * N;
    if (!fin[r]) return;
    lab[r * N + spos[v]] = P[memb[i]] - roff[r];
}
__global__ void k_lv_fill_i32(int64_t n, int32_t* p, int32_t v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}
__global__ void k_lv_fill_u8(int64_t n, uint8_t* p, const uint8_t* done, const int32_t* rep) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = done[rep[i]] ? 0 : 1;
}

// ---------------------------------------------------------------- Infomap bookkeeping
__global__ void k_degree(int64_t N, const int64_t* rowptr, int64_t* deg) {
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v < N) deg[v] = rowptr[v + 1] - rowptr[v];
}
// level 0: every vertex its own module (flow = degree, exit = degree)
__global__ void k_info_init0(int64_t N, int n_r, const int64_t* deg, int32_t* P, int64_t* mod, int32_t* memb) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)n_r * N) return;
    P[i] = (int32_t)i;
    mod[2 * i] = mod[2 * i + 1] = deg[i % N];
    memb[i] = (int32_t)i;
}
// explicit level: singleton modules of the aggregate nodes
__global__ void k_info_level(int64_t nU, const int64_t* kv, const int64_t* sv, int64_t* mod) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nU) return;
    mod[2 * i] = kv[i];
    mod[2 * i + 1] = sv[i];
}
// the modules play the refined communities' part in the aggregation: R = P, sizes, totals
__global__ void k_info_rclear(int64_t nU, const int64_t* mod, int32_t* rsize, int64_t* rtot) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nU) return;
    rsize[c] = 0;
    rtot[c] = mod[2 * c];
}
template <bool IMPL>
__global__ void k_info_modules(LvArgs a) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= a.nU || a.done[rep_of<IMPL>(a, x)]) return;
    const int32_t m = a.P[x];
    a.R[x] = m;
    atomicAdd(&a.rsize[m], 1);
}
// codelength (bits, without the constant node-entropy term) of replica r's modules: one
// block per finishing replica, fixed-order reduction (deterministic)
__global__ __launch_bounds__(LTB) void k_info_codelen(const uint8_t* fin, const int32_t* roff, const int32_t* rend,
                                                      const int64_t* mod, const int64_t* qrep,
                                                      double inv, double* cl) {
    __shared__ double sm[LTB];
    const int r = blockIdx.x;
    if (!fin[r]) return;
    double acc = 0.0;
    for (int64_t c = roff[r] + threadIdx.x; c < rend[r]; c += LTB)
        acc += -2.0 * plogp2(mod[2 * c + 1] * inv) + plogp2((mod[2 * c + 1] + mod[2 * c]) * inv);
    sm[threadIdx.x] = acc;
    __syncthreads();
    for (int k = LTB / 2; k > 0; k >>= 1) {
        if ((int)threadIdx.x < k) sm[threadIdx.x] += sm[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) cl[r] = plogp2(qrep[r] * inv) + sm[0];
}

// Infomap pass lists: every eligible vertex (replica neither finished nor done at this level)
// into the list of its bucket, once per pass.  Scanning the union in every bucket launch cost B
// scans per pass, and a wave then held ~64/B vertices of its bucket; a listed wave holds 64.
// Decisions within a bucket are pure functions of the state before it and the apply's updates
// are integer atomics, so the order inside a list does not change any result.
constexpr int ILIST_MAXB = 1024;
// The pass lists in two passes over contiguous ranges of the union (block k takes [k*span,
// (k+1)*span)): per-block bucket counts, an exclusive scan of them bucket-major, then each block
// writes its vertices at its own offsets -- a bucket's list stays in union (replica-major) order
// up to the order inside one block's range, and no global atomic is shared by the blocks (a
// block per 256 vertices with one atomic per bucket each was 1.7 ms per pass at LFR-100k:
// 250 k blocks on 32 hot counters).  cnt: [B][gridDim.x] (+1 for the scan).
template <bool IMPL>
__global__ __launch_bounds__(LTB) void k_info_lcount(LvArgs a, int64_t span, int32_t* cnt) {
    __shared__ int32_t h[ILIST_MAXB];
    for (int i = threadIdx.x; i < a.B; i += LTB) h[i] = 0;
    __syncthreads();
    const int64_t lo = (int64_t)blockIdx.x * span, hi = min(a.nU, lo + span);
    for (int64_t x = lo + threadIdx.x; x < hi; x += LTB) {
        const int32_t r = rep_of<IMPL>(a, x);
        if (!a.done[r] && !a.lvdone[r]) atomicAdd(&h[bucket_of(a, r, x)], 1);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < a.B; i += LTB) cnt[(int64_t)i * gridDim.x + blockIdx.x] = h[i];
}
// off: the exclusive scan of cnt; list: [sum cnt] bucket-major
template <bool IMPL>
__global__ __launch_bounds__(LTB) void k_info_lfill(LvArgs a, int64_t span, const int32_t* off, int32_t* list) {
    __shared__ int32_t base[ILIST_MAXB];
    for (int i = threadIdx.x; i < a.B; i += LTB) base[i] = off[(int64_t)i * gridDim.x + blockIdx.x];
    __syncthreads();
    const int64_t lo = (int64_t)blockIdx.x * span, hi = min(a.nU, lo + span);
    for (int64_t x = lo + threadIdx.x; x < hi; x += LTB) {
        const int32_t r = rep_of<IMPL>(a, x);
        if (!a.done[r] && !a.lvdone[r]) list[atomicAdd(&base[bucket_of(a, r, x)], 1)] = (int32_t)x;
    }
}
// the B bucket sizes (one host read per pass)
__global__ void k_info_lsizes(int B, int nblk, const int32_t* off, int32_t* icnt) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < B) icnt[b] = off[(int64_t)(b + 1) * nblk] - off[(int64_t)b * nblk];
}
constexpr int ILIST_BLOCKS = 2048;      // list-build blocks (ranges of the union)

// Buffers (Ctx::lv).
enum {
    B_P, B_R, B_RTOT, B_RSIZE, B_PTOT, B_ACT, B_BLIST, B_BTGT, B_BCNT, B_HEAVY, B_HCNT, B_HTGT, B_HKEY, B_HVAL,
    B_HLST, B_MOVES, B_MEMB, B_NID, B_ROFF, B_REND, B_DONE, B_RKEY, B_MISC, B_MVT,
    B_POUT, B_DEG, B_QREP, B_CL, B_BWA, B_BWB, B_HWA, B_HWB, B_TLAB, B_LVDONE, B_RMOVES, B_BMAP, B_LVB,
    B_ILC, B_ILL,   // Infomap pass lists: counts | cursors, the list
    // aggregation scratch
    B_FL, B_MCNT, B_MOFF, B_UB, B_UBO, B_MCUR, B_MLIST, B_TCOL, B_TW, B_OLEN, B_AGH, B_LEN64,
    // explicit level graphs, ping-pong: rowptr, col, w, kv, rep, sv (x2)
    B_G0, B_G1 = B_G0 + 6, B_END = B_G1 + 6
};
static_assert(B_END <= (int)(sizeof(((Ctx*)nullptr)->lv) / sizeof(DevBuf)), "Ctx::lv too small");

// device max of ubo[i+1]-ubo[i] (int64) or of len[i] (int32): one atomic per block
// Rows of [0, n) longer than thr entries (offsets ubo): what a level's heavy lists must hold.
__global__ void k_count_long(int64_t n, const int64_t* ubo, int64_t thr, unsigned long long* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long b = __ballot(i < n && ubo[i + 1] - ubo[i] > thr);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(out, (unsigned long long)__popcll(b));
}
__global__ void k_max_row(int64_t n, const int64_t* ubo, const int32_t* len, unsigned long long* out) {
    __shared__ unsigned long long sm[LTB / 64];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long v = 0;
    if (i < n) v = ubo ? (unsigned long long)(ubo[i + 1] - ubo[i]) : (unsigned long long)len[i];
    for (int off = 32; off; off >>= 1) { const unsigned long long o = __shfl_xor(v, off); v = o > v ? o : v; }
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < LTB / 64; ++k) v = sm[k] > v ? sm[k] : v;
        if (v) atomicMax(out, v);
    }
}

struct LvGraph {
    int64_t nU = 0, E = 0;
    int64_t* rowptr = nullptr;
    int32_t* col = nullptr;
    int32_t* w = nullptr;
    int64_t* kv = nullptr;
    int32_t* rep = nullptr;
    int64_t* sv = nullptr;
    int32_t max_deg = 0;
};

}  // namespace

// One multi-level run per local replica on the working graph c.g; labels -> lab_out (slot
// order, values in [0, N) per replica), exactly like cd_run leaves c.lab.
//   info = false: Leiden (level-0 move on the Louvain engine, refine, aggregate by R);
//   info = true:  `tu` Infomap trials per replica side by side in the union (union replica
//                 u = r*tu + j runs trial trial0 + j of replica r: the same random streams as
//                 running the trials one after the other); map-equation passes at every
//                 level, aggregation by the modules; cl_out[u] = its codelength (without the
//                 constant node-entropy term) for the best-of-trials choice.
static void multilevel(Ctx& c, bool info, int rbegin, int rcount, int n_p_total, int iteration, int tu, int trial0,
                       int32_t* lab_out, double* cl_out) {
    FC_REQUIRE(rcount >= 1 && rbegin >= 0 && rbegin + rcount <= n_p_total, FC_EINVAL, "bad replica range");
    FC_REQUIRE(c.N > 0 && c.g.rowptr.p, FC_ESTATE, "no graph loaded");
    const int64_t N = c.N;
    Graph& g = c.g;
    // Infomap runs on the topology (community_infomap() without weights, :268 / :390)
    const int64_t M2 = info ? 2 * g.m : g.M2;
    FC_REQUIRE(M2 < 0x7fffffffll, FC_ELIMIT, "leiden/infomap: total edge weight must stay below 2^30");
    FC_REQUIRE(tu >= 1 && (info || tu == 1), FC_EINVAL, "trials side by side are for Infomap");
    FC_REQUIRE((int64_t)rcount * tu * N < 0x7fffffffll, FC_ELIMIT,
               "leiden/infomap: replicas x trials x nodes must stay below 2^31");

    if (!info) {
        // ---- level 0, move phase: the replica-batched local-moving engine run to exhaustion
        const double mdq = c.cd_min_dq;
        c.cd_min_dq = 0.0;
        try {
            cd_run(c, FC_ALGO_LOUVAIN, rbegin, rcount, n_p_total, iteration);
        } catch (...) {
            c.cd_min_dq = mdq;
            throw;
        }
        c.cd_min_dq = mdq;
    }
    // lab_out == nullptr: c.lab, read only now (cd_run above may have (re)allocated it)
    if (!lab_out) lab_out = ensure<int32_t>(c.lab, (size_t)rcount * (size_t)N);
    const int sl0 = timer_begin(c);   // (cd_run timed itself) refinement, Infomap passes and the levels
    const char* name = info ? "infomap" : "leiden";

    const int n_r = rcount * tu;   // union replicas
    const int64_t nU0 = (int64_t)n_r * N;
    const int B = std::max(1, c.buckets > 0 ? c.buckets : CD_BUCKETS_LPA);   // refine / Infomap sweeps (level 0 Louvain: cd_buckets)
    auto I32 = [&](int k, int64_t n) { return ensure<int32_t>(c.lv[k], (size_t)std::max<int64_t>(n, 1)); };
    auto I64 = [&](int k, int64_t n) { return ensure<int64_t>(c.lv[k], (size_t)std::max<int64_t>(n, 1)); };
    auto U8 = [&](int k, int64_t n) { return ensure<uint8_t>(c.lv[k], (size_t)std::max<int64_t>(n, 1)); };

    int32_t* P = I32(B_P, nU0);
    int32_t* R = I32(B_R, nU0);
    int64_t* rtot = I64(B_RTOT, nU0);
    int32_t* rsize = I32(B_RSIZE, nU0);
    int32_t* memb = I32(B_MEMB, nU0);
    uint8_t* done = U8(B_DONE, n_r);
    int32_t* roff = I32(B_ROFF, n_r);
    int32_t* rend = I32(B_REND, n_r);
    uint32_t* rkey = (uint32_t*)I32(B_RKEY, n_r);
    unsigned long long* moves = (unsigned long long*)I64(B_MOVES, MSH);
    int32_t* hcnt = I32(B_HCNT, 4);
    // [n_r] refined-community counts | [n_r] finalize flags (u8 view) | 2 u64 maxima
    int32_t* misc = I32(B_MISC, 2 * (int64_t)n_r + 16);
    FC_HIP(hipMemsetAsync(done, 0, n_r, c.stream));
    int64_t* deg = nullptr;
    int64_t* ptot = nullptr;   // Leiden: move-phase community totals
    int64_t* mod = nullptr;    // Infomap: {flow, exit weight} per module
    int64_t* qrep = nullptr;
    double* dcl = nullptr;
    if (info) {
        deg = I64(B_DEG, N);
        mod = I64(B_POUT, 2 * nU0);
        qrep = I64(B_QREP, n_r);
        dcl = (double*)I64(B_CL, n_r);
        k_degree<<<nb(N), LTB, 0, c.stream>>>(N, g.rowptr.as<int64_t>(), deg);
        k_info_init0<<<nb(nU0), LTB, 0, c.stream>>>(N, n_r, deg, P, mod, memb);
        std::vector<int64_t> q0(n_r, M2);   // singletons: total exit weight = every edge end
        FC_HIP(hipMemcpyAsync(qrep, q0.data(), 8 * (size_t)n_r, hipMemcpyHostToDevice, c.stream));
        sync(c);
    } else {
        k_lv_init0<<<nb(nU0), LTB, 0, c.stream>>>(N, n_r, c.lab.as<int32_t>(), c.spos.as<int32_t>(), P, R, rtot,
                                                   rsize, g.kdeg.as<int64_t>(), memb);
    }
    std::vector<int32_t> h_roff(n_r), h_rend(n_r);
    for (int r = 0; r < n_r; ++r) { h_roff[r] = (int32_t)(r * N); h_rend[r] = (int32_t)((r + 1) * N); }
    FC_HIP(hipMemcpyAsync(roff, h_roff.data(), 4 * (size_t)n_r, hipMemcpyHostToDevice, c.stream));
    FC_HIP(hipMemcpyAsync(rend, h_rend.data(), 4 * (size_t)n_r, hipMemcpyHostToDevice, c.stream));
    std::vector<uint8_t> h_done(n_r, 0);
    uint32_t stamp_ctr = 0;
    std::vector<uint32_t> h_rkey(n_r);

    LvArgs a{};
    a.N0 = N; a.M2 = M2; a.B = B;
    a.inv = M2 > 0 ? 1.0 / (double)M2 : 0.0;
    a.mod = mod; a.qrep = qrep;
    a.roff = roff; a.rkey = rkey; a.done = done; a.moves = moves;
    a.heavy_cnt = hcnt;
    a.lvb = (unsigned long long*)I64(B_LVB, 2 * MSH);
    FC_HIP(hipMemsetAsync(a.lvb, 0, 16 * MSH, c.stream));
    a.mvt = (unsigned long long*)I64(B_MVT, nU0);
    FC_HIP(hipMemsetAsync(a.mvt, 0, 8 * (size_t)nU0, c.stream));

    LvGraph cur;            // explicit level (level >= 1)
    int pp = 0;             // ping-pong slot of the next explicit level
    int64_t nU = nU0;
    bool impl = true;
    int32_t max_deg = g.max_deg;

    auto set_keys = [&](int level, int sweep, uint32_t salt) {
        for (int r = 0; r < n_r; ++r)
            h_rkey[r] = stream_key(c.seed, (uint32_t)(rbegin + r / tu), (uint32_t)iteration,
                                   (uint32_t)(level * 4096 + sweep), 16 + salt + 8 * (uint32_t)(trial0 + r % tu));
        FC_HIP(hipMemcpyAsync(rkey, h_rkey.data(), 4 * (size_t)n_r, hipMemcpyHostToDevice, c.stream));
    };
    auto set_graph = [&]() {
        a.nU = nU;
        if (impl) {
            a.rowptr = g.rowptr.as<int64_t>(); a.col = g.col.as<int32_t>();
            a.w = (info || g.max_w == 1) ? nullptr : g.cw.as<int32_t>();
            a.kv = info ? deg : g.kdeg.as<int64_t>(); a.rep = nullptr;
            a.sv = deg;
        } else {
            a.rowptr = cur.rowptr; a.col = cur.col; a.w = cur.w; a.kv = cur.kv; a.rep = cur.rep; a.sv = cur.sv;
        }
        if (info) a.mvo = I32(B_BWA, nU);
        // block lists for scan grids, or (Infomap, input-graph level) per-replica grids of nb(N) blocks
        const int64_t nblk = std::max<int64_t>(nb(nU), impl ? (int64_t)nb(N) * n_r : 0);
        a.blist = I32(B_BLIST, nblk * LTB);
        a.btgt = I32(B_BTGT, nblk * LTB);
        a.bcnt = I32(B_BCNT, nblk);
        // each length tier's list holds at most the level's rows past the smallest heavy
        // threshold (64 entries, k_lv_decide<.., 512, 4>), not nU each
        {
            unsigned long long* dcnt = (unsigned long long*)(c.hpin + 48);
            unsigned long long* dd = (unsigned long long*)ensure<int64_t>(c.counters, 4);
            FC_HIP(hipMemsetAsync(dd, 0, 8, c.stream));
            const int64_t nrows = impl ? N : nU;
            if (max_deg > 64)
                k_count_long<<<nb(nrows), LTB, 0, c.stream>>>(nrows, impl ? g.rowptr.as<int64_t>() : cur.rowptr, 64, dd);
            FC_HIP(hipMemcpyAsync(dcnt, dd, 8, hipMemcpyDeviceToHost, c.stream));
            sync(c);
            a.hcap = std::max<int64_t>(1, (int64_t)*dcnt * (impl ? n_r : 1));
        }
        a.heavy = I32(B_HEAVY, NTIER * a.hcap);
        a.htgt = I32(B_HTGT, NTIER * a.hcap);
        int64_t hs = 64;   // global tables only for rows beyond the block's LDS table
        if (max_deg > HLIGHT)
            while (hs < 2 * (int64_t)max_deg) hs <<= 1;
        a.hslots = hs;
    };
    // heavy-kernel grid: one global table per block, bounded to ~2 GB of tables
    auto heavy_grid = [&](int64_t slots) {
        int64_t gr = std::min<int64_t>(1024, std::max<int64_t>(1, ((int64_t)2 << 30) / (12 * slots)));
        const size_t need = (size_t)(gr * slots);
        const bool grow = c.lv[B_HKEY].bytes < need * 4 + 16;
        a.hkey = I32(B_HKEY, gr * slots);
        a.hval = I32(B_HVAL, gr * slots);
        a.hlst = I32(B_HLST, gr * slots);
        if (grow) {   // tables are kept cleared by their users; a fresh allocation is cleared once
            FC_HIP(hipMemsetAsync(a.hkey, 0xff, c.lv[B_HKEY].bytes, c.stream));
            FC_HIP(hipMemsetAsync(a.hval, 0, c.lv[B_HVAL].bytes, c.stream));
        }
        return (int)gr;
    };

    // one bucketed sweep; returns moves
    // Infomap passes: compacted bucket lists (FC_INFO_LISTS=0: every bucket launch scans the union)
    static const bool info_lists = !getenv("FC_INFO_LISTS") || atoi(getenv("FC_INFO_LISTS")) != 0;
    // rows of 65..128 entries: two vertices per wave (256 slots each), not one per wave
    static const bool lv_g2 = !getenv("FC_LV_G2") || atoi(getenv("FC_LV_G2")) != 0;
    std::vector<int32_t> h_icnt;
    auto sweep = [&](int MODE, int level, int sw) -> unsigned long long {
        set_keys(level, sw, (uint32_t)MODE);
        FC_HIP(hipMemsetAsync(moves, 0, 8 * MSH, c.stream));
        int nblk = a.bmap ? a.bpr * a.nact : (int)nb(nU);
        const int hg = heavy_grid(a.hslots);
        const int hblk = 64;
        // Infomap: the pass's bucket lists (one host read of the B counts per pass)
        const bool listed = MODE == MODE_INFO && info_lists && a.B <= ILIST_MAXB;
        int32_t* ill = nullptr;
        a.ilist = nullptr;
        if (listed) {
            const int lblk = (int)std::min<int64_t>(ILIST_BLOCKS, nb(nU));
            const int64_t span = (nU + lblk - 1) / lblk;
            const int64_t nc = (int64_t)a.B * lblk;
            int32_t* ilc = I32(B_ILC, 2 * (nc + 1) + a.B);   // counts | their scan | bucket sizes
            int32_t* ioff = ilc + nc + 1;
            int32_t* isz = ioff + nc + 1;
            ill = I32(B_ILL, nU);
            if (impl) k_info_lcount<true><<<lblk, LTB, 0, c.stream>>>(a, span, ilc);
            else k_info_lcount<false><<<lblk, LTB, 0, c.stream>>>(a, span, ilc);
            FC_HIP(hipMemsetAsync(ilc + nc, 0, sizeof(int32_t), c.stream));
            exclusive_scan(c, (const int32_t*)ilc, ioff, nc + 1);
            if (impl) k_info_lfill<true><<<lblk, LTB, 0, c.stream>>>(a, span, ioff, ill);
            else k_info_lfill<false><<<lblk, LTB, 0, c.stream>>>(a, span, ioff, ill);
            k_info_lsizes<<<nb(a.B), LTB, 0, c.stream>>>(a.B, lblk, ioff, isz);
            h_icnt.resize(a.B);
            FC_HIP(hipMemcpyAsync(h_icnt.data(), isz, 4 * (size_t)a.B, hipMemcpyDeviceToHost, c.stream));
            sync(c);
        }
        int64_t ioff = 0;
        for (int b = 0; b < a.B; ++b) {
            if (listed) {
                a.ilist = ill + ioff;
                a.icnt = h_icnt[b];
                ioff += h_icnt[b];
                nblk = (int)nb(a.icnt);
            }
            // an empty bucket (coarse levels with one or two replicas still moving) has
            // nothing to decide, list as heavy or apply: no zero-block launches
            if (nblk == 0) continue;
            const uint32_t stamp = ++stamp_ctr;   // unique per bucket launch of this run (mvt)
            FC_HIP(hipMemsetAsync(hcnt, 0, 4 * NTIER, c.stream));
            // (timed per launch into spans 5 / 6 when timing is on: lv decide / lv heavy)
#define LV_LAUNCH(IM, MD)                                                                        \
    do {                                                                                         \
        const int t5 = timer_begin(c);                                                           \
        if (max_deg <= 64) k_lv_decide<IM, MD, 512, 4><<<nblk, LTB, 0, c.stream>>>(a, b, stamp);  \
        else if (max_deg <= 128 && lv_g2) k_lv_decide<IM, MD, 512, 2><<<nblk, LTB, 0, c.stream>>>(a, b, stamp); \
        else if (max_deg <= LWS_SMALL / 2) k_lv_decide<IM, MD, LWS_SMALL, 1><<<nblk, LTB, 0, c.stream>>>(a, b, stamp); \
        else k_lv_decide<IM, MD, LWS, 1><<<nblk, LTB, 0, c.stream>>>(a, b, stamp);               \
        timer_end(c, 5, t5);                                                                     \
        if (max_deg > LIGHT) {   /* tiers by row length (heavy_tier); tier 3: global tables */  \
            /* one timer span per kernel launch, as rocprofv3 counts them */                     \
            int t6 = timer_begin(c);                                                             \
            k_lv_heavy<IM, MD, 2048><<<2048, LTB, 0, c.stream>>>(a, stamp, 0);                   \
            timer_end(c, 6, t6);                                                                 \
            if (max_deg > 1024) {                                                                \
                t6 = timer_begin(c);                                                             \
                k_lv_heavy<IM, MD, 4096><<<1280, LTB, 0, c.stream>>>(a, stamp, 1);               \
                timer_end(c, 6, t6);                                                             \
            }                                                                                    \
            if (max_deg > 2048) {                                                                \
                t6 = timer_begin(c);                                                             \
                k_lv_heavy<IM, MD, HLS><<<512, LTB, 0, c.stream>>>(a, stamp, 2);                 \
                timer_end(c, 6, t6);                                                             \
            }                                                                                    \
            if (max_deg > 4096) {                                                                \
                t6 = timer_begin(c);                                                             \
                k_lv_heavy<IM, MD, 2048><<<hg, LTB, 0, c.stream>>>(a, stamp, 3);                 \
                timer_end(c, 6, t6);                                                             \
            }                                                                                    \
        }                                                                                        \
        k_lv_apply<IM, MD><<<nblk + (max_deg > LIGHT ? hblk : 0), LTB, 0, c.stream>>>(a, nblk, hblk, stamp); \
    } while (0)
            if (impl && MODE == MODE_MOVE) LV_LAUNCH(true, MODE_MOVE);
            else if (impl && MODE == MODE_REFINE) LV_LAUNCH(true, MODE_REFINE);
            else if (impl) LV_LAUNCH(true, MODE_INFO);
            else if (MODE == MODE_MOVE) LV_LAUNCH(false, MODE_MOVE);
            else if (MODE == MODE_REFINE) LV_LAUNCH(false, MODE_REFINE);
            else LV_LAUNCH(false, MODE_INFO);
#undef LV_LAUNCH
        }
        a.ilist = nullptr;
        std::vector<unsigned long long> hm(MSH);
        FC_HIP(hipMemcpyAsync(hm.data(), moves, 8 * MSH, hipMemcpyDeviceToHost, c.stream));
        sync(c);
        unsigned long long t = 0;
        for (auto v : hm) t += v;
        return t;
    };

    int level = 0;
    int64_t lv_sweeps = 0;
    for (;; ++level) {
        set_graph();
        if (info) {
            // ---- Infomap: greedy passes until one moves nothing (igraph: until the codelength
            // stops improving; its tune() every 10 passes only refreshes float flows), then the
            // modules are the units the level aggregates
            a.P = P; a.mod = mod; a.qrep = qrep;
            // a replica whose pass moved nothing is done at this level (re-sweeping it would
            // move nothing again), so the trials and replicas still moving run alone
            uint8_t* lvd = U8(B_LVDONE, n_r);
            unsigned long long* rmv = (unsigned long long*)I64(B_RMOVES, n_r);
            std::vector<uint8_t> h_lvd(h_done);
            std::vector<unsigned long long> h_rmv(n_r);
            FC_HIP(hipMemcpyAsync(lvd, h_lvd.data(), n_r, hipMemcpyHostToDevice, c.stream));
            a.lvdone = lvd; a.rmoves = rmv;
            a.bmap = nullptr;
            for (int sw = 0; sw < c.max_sweeps; ++sw) {
                ++lv_sweeps;
                FC_HIP(hipMemsetAsync(rmv, 0, 8 * (size_t)n_r, c.stream));
                if (c.trace && sw == 0) { sync(c); trace_dt_us(true); }
                const unsigned long long mvs = sweep(MODE_INFO, level, sw);   // syncs
                if (c.trace) {
                    int na = 0;
                    for (int r = 0; r < n_r; ++r) na += !h_lvd[r];
                    fprintf(stderr, "[fc] infomap level %d pass %d: %d replicas, %llu moves, %.0f us\n", level, sw, na,
                            mvs, trace_dt_us(false));
                }
                if (mvs == 0) break;
                FC_HIP(hipMemcpy(h_rmv.data(), rmv, 8 * (size_t)n_r, hipMemcpyDeviceToHost));
                for (int r = 0; r < n_r; ++r) h_lvd[r] |= h_rmv[r] == 0;
                FC_HIP(hipMemcpyAsync(lvd, h_lvd.data(), n_r, hipMemcpyHostToDevice, c.stream));
                if (impl) {   // the next passes launch blocks for the replicas still moving only
                    std::vector<int32_t> act;
                    for (int r = 0; r < n_r; ++r)
                        if (!h_lvd[r]) act.push_back(r);
                    if (act.empty()) { sync(c); break; }
                    int32_t* bm = I32(B_BMAP, n_r);
                    FC_HIP(hipMemcpyAsync(bm, act.data(), 4 * act.size(), hipMemcpyHostToDevice, c.stream));
                    a.bmap = bm; a.nact = (int)act.size(); a.bpr = (int)nb(N);
                    sync(c);   // `act` is pageable and local
                }
                sync(c);
            }
            a.bmap = nullptr;
            a.R = R; a.rsize = rsize;
            k_info_rclear<<<nb(nU), LTB, 0, c.stream>>>(nU, mod, rsize, rtot);
            if (impl) k_info_modules<true><<<nb(nU), LTB, 0, c.stream>>>(a);
            else k_info_modules<false><<<nb(nU), LTB, 0, c.stream>>>(a);
            a.tot = rtot;
        } else {
            // ---- refine: singletons inside the move-phase communities, one sweep
            if (!impl) k_lv_rinit<<<nb(nU), LTB, 0, c.stream>>>(nU, cur.kv, R, rtot, rsize);
            a.P = P; a.R = R; a.tot = rtot; a.rsize = rsize;
            sweep(MODE_REFINE, level, 0);
            ++lv_sweeps;
        }
        // ---- which replicas still aggregate: refined communities < level nodes
        int32_t* nid = I32(B_NID, nU + 1);
        int32_t* fl = I32(B_FL, nU + 1);
        if (impl) k_ag_flags<true><<<nb(nU + 1), LTB, 0, c.stream>>>(a, fl);
        else k_ag_flags<false><<<nb(nU + 1), LTB, 0, c.stream>>>(a, fl);
        exclusive_scan(c, fl, nid, nU + 1);
        k_ag_counts<<<nb(n_r), LTB, 0, c.stream>>>(n_r, done, roff, rend, nid, misc);
        std::vector<int32_t> rc(n_r);
        FC_HIP(hipMemcpyAsync(rc.data(), misc, 4 * (size_t)n_r, hipMemcpyDeviceToHost, c.stream));
        sync(c);
        std::vector<uint8_t> fin(n_r, 0);
        bool any_fin = false, any_left = false;
        for (int r = 0; r < n_r; ++r) {
            if (h_done[r]) continue;
            if (rc[r] == h_rend[r] - h_roff[r] || level + 1 >= MAX_LEVELS) { fin[r] = 1; any_fin = true; }
            else any_left = true;
        }
        if (any_fin) {
            uint8_t* dfin = (uint8_t*)(misc + n_r);
            FC_HIP(hipMemcpyAsync(dfin, fin.data(), n_r, hipMemcpyHostToDevice, c.stream));
            if (info) k_info_codelen<<<n_r, LTB, 0, c.stream>>>(dfin, roff, rend, mod, qrep, a.inv, dcl);
            k_lv_final<<<nb(nU0), LTB, 0, c.stream>>>(N, n_r, dfin, memb, P, roff, c.spos.as<int32_t>(), lab_out);
            for (int r = 0; r < n_r; ++r) h_done[r] |= fin[r];
            FC_HIP(hipMemcpyAsync(done, h_done.data(), n_r, hipMemcpyHostToDevice, c.stream));
            sync(c);
        }
        if (!any_left) break;
        if (any_fin) {   // drop the finished replicas from the next level
            if (impl) k_ag_flags<true><<<nb(nU + 1), LTB, 0, c.stream>>>(a, fl);
            else k_ag_flags<false><<<nb(nU + 1), LTB, 0, c.stream>>>(a, fl);
            exclusive_scan(c, fl, nid, nU + 1);
        }
        // ---- aggregate by the refined partition
        int64_t nUn = 0;
        {
            int32_t t32;
            FC_HIP(hipMemcpyAsync(&t32, nid + nU, 4, hipMemcpyDeviceToHost, c.stream));
            sync(c);
            nUn = t32;
        }
        const int gs = pp ? B_G1 : B_G0;
        LvGraph nx;
        nx.nU = nUn;
        nx.rowptr = I64(gs + 0, nUn + 1);
        nx.kv = I64(gs + 3, nUn);
        nx.rep = I32(gs + 4, nUn);
        nx.sv = info ? I64(gs + 5, nUn) : nullptr;
        int32_t* mcnt = I32(B_MCNT, nUn + 1);
        if (impl) k_ag_nodes<true><<<nb(nU), LTB, 0, c.stream>>>(a, nid, nx.rep, nx.kv, mcnt, nx.sv);
        else k_ag_nodes<false><<<nb(nU), LTB, 0, c.stream>>>(a, nid, nx.rep, nx.kv, mcnt, nx.sv);
        FC_HIP(hipMemsetAsync(mcnt + nUn, 0, 4, c.stream));
        int32_t* moff = I32(B_MOFF, nUn + 1);
        exclusive_scan(c, mcnt, moff, nUn + 1);
        int32_t* pofR = I32(B_HTGT, nU);   // free between sweeps
        int32_t* prep = I32(B_HEAVY, nU);
        int64_t* ub = I64(B_UB, nUn + 1);
        int64_t* ubo = I64(B_UBO, nUn + 1);
        k_lv_fill_i32<<<nb(nU), LTB, 0, c.stream>>>(nU, prep, INT_MAX);
        FC_HIP(hipMemsetAsync(ub, 0, 8 * ((size_t)nUn + 1), c.stream));
        if (impl) k_ag_members<true><<<nb(nU), LTB, 0, c.stream>>>(a, nid, pofR, prep, ub);
        else k_ag_members<false><<<nb(nU), LTB, 0, c.stream>>>(a, nid, pofR, prep, ub);
        exclusive_scan(c, ub, ubo, nUn + 1);
        int32_t* mcur = I32(B_MCUR, nUn + 1);
        int32_t* mlist = I32(B_MLIST, nU + 1);
        FC_HIP(hipMemsetAsync(mcur, 0, 4 * (size_t)nUn, c.stream));
        if (impl) k_ag_fill<true><<<nb(nU), LTB, 0, c.stream>>>(a, nid, moff, mcur, mlist);
        else k_ag_fill<false><<<nb(nU), LTB, 0, c.stream>>>(a, nid, moff, mcur, mlist);
        // [0] member-row sum total, [1] the longest one (bounds the heavy tables), [2] longest new row
        int64_t* hx = (int64_t*)c.hpin + 40;
        unsigned long long* dmax = (unsigned long long*)(misc + 2 * (int64_t)n_r + 2 + ((2 * n_r) & 1));
        FC_HIP(hipMemsetAsync(dmax, 0, 16, c.stream));
        unsigned long long* dlong = (unsigned long long*)ensure<int64_t>(c.counters, 4);
        FC_HIP(hipMemsetAsync(dlong, 0, 8, c.stream));
        k_max_row<<<nb(nUn), LTB, 0, c.stream>>>(nUn, ubo, nullptr, dmax);
        k_count_long<<<nb(nUn), LTB, 0, c.stream>>>(nUn, ubo, LIGHT, dlong);   // rows k_ag_rows lists as heavy
        FC_HIP(hipMemcpyAsync(hx, ubo + nUn, 8, hipMemcpyDeviceToHost, c.stream));
        FC_HIP(hipMemcpyAsync(hx + 1, dmax, 8, hipMemcpyDeviceToHost, c.stream));
        FC_HIP(hipMemcpyAsync(hx + 3, dlong, 8, hipMemcpyDeviceToHost, c.stream));
        sync(c);
        const int64_t ubtot = hx[0], ubmax = hx[1], nlong = hx[3];
        int32_t* tcol = I32(B_TCOL, ubtot + 1);
        int32_t* tw = I32(B_TW, ubtot + 1);
        int32_t* olen = I32(B_OLEN, nUn + 1);
        const int64_t ahc = std::max<int64_t>(1, nlong);   // per-tier capacity: the heavy rows
        int32_t* agh = I32(B_AGH, NTIER * ahc);
        FC_HIP(hipMemsetAsync(hcnt, 0, 4 * NTIER, c.stream));
        const unsigned agb = nb(nUn, LTB / 64);
        if (impl) k_ag_rows<true><<<agb, LTB, 0, c.stream>>>(a, nUn, nid, moff, mlist, ubo, tcol, tw, olen, agh, hcnt, ahc);
        else k_ag_rows<false><<<agb, LTB, 0, c.stream>>>(a, nUn, nid, moff, mlist, ubo, tcol, tw, olen, agh, hcnt, ahc);
        if (ubmax > LIGHT) {
            int64_t hs = 64;
            if (ubmax > HLIGHT)
                while (hs < 2 * ubmax) hs <<= 1;
            a.hslots = hs;
            const int hg = heavy_grid(hs);
            // by length tier (heavy_tier): LDS tables sized for the tier, global tables past 4096
#define AG_HEAVY(IM)                                                                                              \
    do {                                                                                                          \
        k_ag_rows_heavy<IM, 2048><<<2048, LTB, 0, c.stream>>>(a, nid, moff, mlist, ubo, tcol, tw, olen, agh, hcnt, ahc, 0); \
        if (ubmax > 1024) k_ag_rows_heavy<IM, 4096><<<1280, LTB, 0, c.stream>>>(a, nid, moff, mlist, ubo, tcol, tw, olen, agh, hcnt, ahc, 1); \
        if (ubmax > 2048) k_ag_rows_heavy<IM, HLS><<<512, LTB, 0, c.stream>>>(a, nid, moff, mlist, ubo, tcol, tw, olen, agh, hcnt, ahc, 2); \
        if (ubmax > 4096) k_ag_rows_heavy<IM, 2048><<<hg, LTB, 0, c.stream>>>(a, nid, moff, mlist, ubo, tcol, tw, olen, agh, hcnt, ahc, 3); \
    } while (0)
            if (impl) AG_HEAVY(true);
            else AG_HEAVY(false);
#undef AG_HEAVY
        }
        int64_t* len64 = I64(B_LEN64, nUn + 1);
        k_ag_len64<<<nb(nUn + 1), LTB, 0, c.stream>>>(nUn, olen, len64);
        exclusive_scan(c, len64, nx.rowptr, nUn + 1);
        k_max_row<<<nb(nUn), LTB, 0, c.stream>>>(nUn, nullptr, olen, dmax + 1);
        FC_HIP(hipMemcpyAsync(hx, nx.rowptr + nUn, 8, hipMemcpyDeviceToHost, c.stream));
        FC_HIP(hipMemcpyAsync(hx + 2, dmax + 1, 8, hipMemcpyDeviceToHost, c.stream));
        sync(c);
        nx.E = hx[0];
        nx.max_deg = (int32_t)hx[2];
        nx.col = I32(gs + 1, nx.E);
        nx.w = I32(gs + 2, nx.E);
        k_ag_compact<<<agb, LTB, 0, c.stream>>>(nUn, ubo, nx.rowptr, tcol, tw, nx.col, nx.w);
        // P of the new level: each new vertex starts in its members' move-phase community
        int32_t* nP = I32(B_PTOT, nUn);   // staged in the (free) ptot buffer, then swapped into P
        k_ag_part<<<nb(nU), LTB, 0, c.stream>>>(nU, nid, pofR, prep, nP);
        k_ag_memb<<<nb(nU0), LTB, 0, c.stream>>>(nU0, N, done, R, nid, memb);
        std::swap(c.lv[B_P], c.lv[B_PTOT]);
        P = c.lv[B_P].as<int32_t>();
        // replica ranges of the new level
        k_ag_roff<<<nb(nUn), LTB, 0, c.stream>>>(nUn, nx.rep, roff, rend);
        FC_HIP(hipMemcpyAsync(h_roff.data(), roff, 4 * (size_t)n_r, hipMemcpyDeviceToHost, c.stream));
        FC_HIP(hipMemcpyAsync(h_rend.data(), rend, 4 * (size_t)n_r, hipMemcpyDeviceToHost, c.stream));
        sync(c);
        cur = nx;
        pp ^= 1;
        impl = false;
        nU = nUn;
        max_deg = nx.max_deg;
        if (info) {   // singleton modules of the aggregate nodes; the next loop trip optimises them
            mod = I64(B_POUT, 2 * nU);
            R = I32(B_R, nU); rtot = I64(B_RTOT, nU); rsize = I32(B_RSIZE, nU);
            k_info_level<<<nb(nU), LTB, 0, c.stream>>>(nU, cur.kv, cur.sv, mod);
            if (c.trace) {
                sync(c);
                fprintf(stderr, "[fc] infomap level %d: %lld union vertices, %lld entries, max degree %d\n", level + 1,
                        (long long)nU, (long long)cur.E, max_deg);
            }
            continue;
        }
        // ---- move phase on the new level, from the inherited partition, until no move
        ptot = I64(B_PTOT, nU);
        R = I32(B_R, nU); rtot = I64(B_RTOT, nU); rsize = I32(B_RSIZE, nU);
        FC_HIP(hipMemsetAsync(ptot, 0, 8 * (size_t)nU, c.stream));
        k_ag_ptot<<<nb(nU), LTB, 0, c.stream>>>(nU, P, cur.kv, ptot);
        uint8_t* act = U8(B_ACT, nU);
        k_lv_fill_u8<<<nb(nU), LTB, 0, c.stream>>>(nU, act, done, cur.rep);
        set_graph();
        a.P = P; a.R = R; a.tot = ptot; a.rsize = rsize; a.act = act;
        // aggregate levels: lv_level_b buckets per move sweep (default 4, not level 0's 32).  The
        // dense levels run tens of sweeps whose queues are a few re-queued vertices per replica;
        // a bucket is a launch chain (decide, heavy tiers, apply) of ~100 us whatever it holds,
        // and more simultaneous deciders did not cost sweeps or modularity (LFR-1M: 2.37 s with
        // 32 buckets, 2.11 s with 16, 1.97 s with 8, 1.92 s with 4; modularity 0.46515 /
        // 0.46517 / 0.46517 at 32 / 8 / 4, LFR-100k 0.46454 / 0.46457 / 0.46457;
        // profiles/r04_leiden_buckets.txt).  FC_LV_DENSE_DIV (off): more buckets on dense levels,
        // buckets >= average degree / div, up to 1024 -- measured slower (DESIGN).
        const int64_t avgdeg = cur.E / std::max<int64_t>(nU, 1);
        int Bl = (c.buckets == 0 && c.lv_level_b > 0) ? c.lv_level_b : B;   // FC_OPT_BUCKETS wins
        if (c.lv_dense_div > 0)
            while (Bl < 1024 && (int64_t)Bl * c.lv_dense_div < avgdeg) Bl <<= 1;
        a.B = Bl;
        int sw = 0;
        for (; sw < c.max_sweeps; ++sw) {
            ++lv_sweeps;
            const auto t_sw = std::chrono::steady_clock::now();
            const unsigned long long mvs = sweep(MODE_MOVE, level + 1, sw + 1);
            if (c.trace) {
                // algorithmic bytes of the decide / heavy launches so far (the work the sweep did)
                std::vector<unsigned long long> hb(2 * MSH);
                FC_HIP(hipMemcpy(hb.data(), a.lvb, 16 * MSH, hipMemcpyDeviceToHost));
                unsigned long long bd = 0, bh = 0;
                for (int k = 0; k < MSH; ++k) { bd += hb[k]; bh += hb[MSH + k]; }
                static unsigned long long pd = 0, ph = 0;
                if (bd < pd || bh < ph) pd = ph = 0;
                fprintf(stderr, "[fc] leiden level %d sweep %d: %llu moves, %.2f ms, decide %.1f MB, heavy %.1f MB\n",
                        level + 1, sw, mvs,
                        1e-3 * (double)std::chrono::duration_cast<std::chrono::microseconds>(
                                   std::chrono::steady_clock::now() - t_sw).count(), (bd - pd) / 1e6, (bh - ph) / 1e6);
                pd = bd; ph = bh;
            }
            if (mvs == 0) break;
        }
        a.B = B;
        if (c.trace) {
            sync(c);
            fprintf(stderr, "[fc] leiden level %d: %lld union vertices, %lld entries, max degree %d, %d move sweeps, "
                    "%.1f ms since the previous level\n", level + 1, (long long)nU, (long long)cur.E, max_deg, sw + 1,
                    1e-3 * trace_dt_us());
        }
    }
    if (c.trace) fprintf(stderr, "[fc] %s it=%d: %d levels, %lld level sweeps\n", name, iteration, level + 1,
                         (long long)lv_sweeps);
    if (info) FC_HIP(hipMemcpyAsync(cl_out, dcl, 8 * (size_t)n_r, hipMemcpyDeviceToHost, c.stream));
    std::vector<unsigned long long> lvb(2 * MSH);
    FC_HIP(hipMemcpyAsync(lvb.data(), a.lvb, 16 * MSH, hipMemcpyDeviceToHost, c.stream));
    sync(c);
    unsigned long long lvd = 0, lvh = 0;
    for (int k = 0; k < MSH; ++k) { lvd += lvb[k]; lvh += lvb[MSH + k]; }
    for (fc_stats* st : {&c.acc, &c.prof}) {
        st->cd_sweeps += lv_sweeps * n_r;
        st->lv_decide_bytes += (int64_t)lvd;
        st->lv_heavy_bytes += (int64_t)lvh;
    }
    c.n_r = rcount; c.rbase = rbegin; c.n_p_total = n_p_total;
    c.labT_valid = false;
    timer_end(c, 0, sl0);
    sync(c);
}

void leiden_run(Ctx& c, int rbegin, int rcount, int n_p_total, int iteration) {
    multilevel(c, false, rbegin, rcount, n_p_total, iteration, 1, 0, nullptr, nullptr);   // -> c.lab
}

// igraph community_infomap(trials=10) (fast_consensus.py:268, :390): the best of `trials`
// independent runs per replica, by codelength.  The trials run side by side in one union
// (as many as fit: int32 union ids, ~2^29 union vertices), so the small upper levels are
// one launch sequence for all of them instead of one per trial.
void infomap_run(Ctx& c, int rbegin, int rcount, int n_p_total, int iteration) {
    const int64_t N = std::max<int64_t>(c.N, 1);
    const int T = std::max(1, c.infomap_trials);
    const int64_t per = (int64_t)rcount * N;
    int tu = T;
    while (tu > 1 && per * tu > ((int64_t)1 << 29)) --tu;
    int32_t* lab = ensure<int32_t>(c.lab, (size_t)per);
    int32_t* tlab = ensure<int32_t>(c.lv[B_TLAB], (size_t)(per * tu));
    std::vector<double> best(rcount, 1e300), cl((size_t)rcount * tu);
    for (int t0 = 0; t0 < T; t0 += tu) {
        const int k = std::min(tu, T - t0);
        multilevel(c, true, rbegin, rcount, n_p_total, iteration, k, t0, tlab, cl.data());
        for (int r = 0; r < rcount; ++r)
            for (int j = 0; j < k; ++j) {   // trial order: the earliest of equal codelengths wins
                const size_t u = (size_t)r * k + j;
                if (c.trace && r < 4)
                    fprintf(stderr, "[fc] infomap trial %d replica %d codelength %.6f (best %.6f)\n", t0 + j, r, cl[u],
                            best[r]);
                if (!(cl[u] < best[r])) continue;
                best[r] = cl[u];
                FC_HIP(hipMemcpyAsync(lab + (size_t)r * N, tlab + u * N, 4 * (size_t)N, hipMemcpyDeviceToDevice,
                                      c.stream));
            }
        sync(c);
    }
    c.n_r = rcount; c.rbase = rbegin; c.n_p_total = n_p_total;
    c.labT_valid = false;
}

}  // namespace fc
