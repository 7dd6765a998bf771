// cd.hip -- replica-batched community detection on the device-resident CSR:
//   * Louvain level-0 local moving (python-louvain 0.15 `__one_level`, the only level the
//     reference consumes: partition_at_level(..., 0) at fast_consensus.py:148, :384);
//   * label propagation (igraph 0.9.7 community_label_propagation(), unweighted as called
//     at fast_consensus.py:270, :392).
//
// Sequential asynchronous order -> bucketed rounds.  Each replica visits its vertices in
// a per-(replica, iteration, sweep) random order (Feistel bijection); a sweep is split
// into B buckets of that order; vertices of a bucket decide simultaneously against the
// state left by the previous buckets, then their moves are applied (integer atomics:
// deterministic).  Gains use exact int64 arithmetic on the integer edge weights:
//     G_c = (k_v,c - k_v,own) * 2M + k_v * ((tot_own - k_v) - tot_c)      (= incr * 2M)
// move iff max_c G_c > 0 (python-louvain's strict `incr > best_increase` from 0); ties
// broken uniformly at random by a hash (python-louvain shuffles neighbour communities).
// A sweep ends the run when its predicted modularity gain < 1e-7 (python-louvain __MIN)
// or nothing moved.  LPA: random dominant label; stop after a sweep in which every
// visited vertex already held a dominant label (igraph 0.9 `running` flag).
//
// Memory layout: replica-major state (lab/tot [n_r][N]), shared read-only CSR.
// One 16-lane tile per vertex with a 128-slot LDS hash table (degree <= 64); larger
// rows go to a workgroup-per-vertex kernel (LDS table up to 4096 slots, else global).
#include <hipcub/hipcub.hpp>

#include <chrono>

#include "fc_ctx.h"
#include "fc_device.h"

namespace fc {

template <class T> void exclusive_scan(Ctx& c, const T* in, T* out, int64_t n);
template <class K, class V>
void sort_pairs_public(Ctx& c, const K* kin, K* kout, const V* vin, V* vout, int64_t n, int end_bit);

static constexpr int TB = 256;
// Sweep order: vertices, or chunks of CHUNK consecutive vertices (chunk = 0 or CHUNK,
// FC_OPT_CHUNK), in a random order; position p of vertex v is the inverse permutation
// (k_list_build).  Positions fit 32 bits since N < 2^31.
static constexpr int CHUNK = 16;

static constexpr int TILE = 16;         // lanes per decision in k_apply's row scatter
#ifndef FC_ATB
#define FC_ATB 256
#endif
static constexpr int ATB = FC_ATB;      // threads per k_apply block
static constexpr int TILES = ATB / TILE;
#ifndef FC_WNT
#define FC_WNT 8
#endif
static constexpr int WNT = FC_WNT;      // vertices per wave in the light decide (rows flattened over 64 lanes;
                                        // LFR-1M 254 ms at 8, 308 ms at 4)
#ifndef FC_DTB
#define FC_DTB 64
#endif
static constexpr int DTB = FC_DTB;      // threads per k_decide_light block: one wave (LFR-1M 257.9 ms at 256,
                                        // 255.6 at 128, 254.1 at 64; 266.5 at 512)
static constexpr int LNT = WNT * (DTB / 64);  // vertices per k_decide_light block (one item)
static constexpr int HCAP = 64;         // slots per tile table (>= LIGHT_MAX_DEG: every insert finds a slot)
static constexpr int LIGHT_MAX_DEG = 64;
static constexpr int HEAVY_LDS_SLOTS = 4096;
static constexpr int HEAVY_GRID = 256;
static constexpr double DQ_SCALE = 1099511627776.0;  // 2^40 fixed point for predicted dQ
static constexpr int NSH = 16;          // counter shards per replica
static constexpr int RF = 8;            // fields: 0 dq, 1 unstable, 2 moves, 3 verts, 4 entries, 5 cands
static constexpr int RR_FULL = 1, RR_PUSH = 2, RR_TRANS = 4;   // round-record flags


static inline unsigned nblk(int64_t n, int tb = TB) {
    int64_t b = (n + tb - 1) / tb;
    if (b < 1) b = 1;
    return (unsigned)b;
}

struct CDArgs {
    int64_t N;
    int64_t S;          // bucket size (positions per bucket)
    int64_t PN;         // positions per sweep (N, or N rounded up to whole chunks)
    int chunk;          // 0: vertex-level random order; else order over chunks of `chunk` vertices
    uint32_t perm_n;    // permutation domain: N, or the number of chunks
    int n_r, rbase;
    uint32_t iter;
    uint64_t seed;
    const int64_t* rowptr;
    const int32_t* col;
    const int32_t* colp;         // storage slot of col[j] (label gathers: lab rows are in slot order)
    const int32_t* spos;         // storage slot of vertex v in every lab row (Ctx::spos)
    const int4* vrec;            // per vertex: row start (uint32), degree, k_v (int32 totals only), slot
    const int32_t* cw;
    const int64_t* kdeg;
    int64_t M2;
    int32_t* lab;
    int32_t* nlab;               // [n_r][m2]: label of the neighbour behind adjacency entry j
    const int32_t* rev;          // reverse adjacency entry of j
    int64_t m2;                  // 2m (adjacency entries)
    void* tot;                   // int32 [n_r][N] when 2M < 2^31, else int64
    int4* dec;                   // [n_r][dstride] (target community or -1, vertex, own label, k_v when 2M < 2^31):
                                 // the move needs no random read of the old label or the degree
    int32_t* active;
    // Sharded per-replica counters [n_r][NSH][RF]: one hot address per replica would
    // serialise every block's atomic (~12 ns each, MI355X_MICROARCH.md "fanin").
    unsigned long long* red;
    // pruning (list mode): per sweep >= 1 only vertices whose neighbour moved are visited
    uint32_t* aff;               // [n_r][aw] affected bits, bit v & 31 of word v >> 5 (set by moves,
                                 // read + cleared by the list build): N/8 bytes per replica
    int64_t aw;                  // words per replica
    int own_bal;                 // 1: own-label entries of weight w0 summed by wave ballots, not inserted in the LDS table
    int w0;                      // that weight: 1 on unit-weight graphs, n_p on consensus graphs (their typical weight)
    int wbits;                   // bits of the largest edge weight (LPA: 1)
    int track_div, push_div;     // pruning starts after a sweep moving < N/track_div; pull -> push after < N/push_div (0: never)
    int unitw;                   // every weight is 1: no weight loads
    int32_t* track;              // [n_r] moves mark neighbours affected this sweep; [n_r..2n_r) list filters;
                                 // [2n_r..3n_r) push mode: nlab is current (else decide gathers lab[col]);
                                 // [3n_r..4n_r) transition sweep: decide writes the nlab rows it gathers,
                                 // moves push (every vertex is visited), push mode from the next sweep
    int prune;
    // Leiden-style marking (FC_OPT_PRUNE_MARK, weighted Louvain graphs): tracking starts at
    // sweep 1, and a tracked sweep's movers mark, at the sweep's end, only the neighbours
    // whose label differs from theirs (k_mark_lm); k_apply just flags the movers in mvf
    int lm;
    uint8_t* mvf;                // [n_r][N] moved this (tracked) sweep
    const int32_t* list;         // [n_r][PN] vertices to visit, grouped by round (offsets loff)
    const int32_t* loff;         // [n_r][B+1] round offsets into a replica's list
    int B;                       // buckets per sweep
    int coarsen;                 // FC_OPT_COARSEN: 0, or the largest g (filtered sweeps in rounds of g buckets)
    int64_t hcap;                // heavy-row slots per replica and round (heavy vertices in the graph)
    int64_t dstride;             // decision slots per replica (PN: a coarse round may exceed S)
    const int32_t* lcnt;         // [B][n_r] list lengths
    // [B][n_r] per round and replica (k_list_plan): x first position (implicit list) or list
    // offset, y entries, z flags RR_*; one scalar load gives a decide block all it needs
    const int4* rrec;
    int32_t* heavy;              // (r, dec index, position) triples
    int32_t* heavy_cnt;
    int32_t* heavy_scratch;      // global tables when rows exceed the LDS table
    int64_t heavy_slots;         // slots per global table (power of 2)
    unsigned long long* sacc;    // [n_r][4] light-kernel vertices / entries / candidates, summed by k_sweep_end
    double min_dq;               // Louvain stop: a sweep gaining < min_dq (python-louvain __MIN 1e-7; Leiden's
                                 // move phase 0: run until a sweep moves nothing)
    int shared_full;             // FC_OPT_CD_ENGINE=2: a replica's full sweeps visit the batch's SHARED order
                                 // (SHARED_RG), its filtered sweeps its own (oracle tw_replica shared = 2)
    const int32_t* vcnt;         // hybrid: [n_r] affected flags at this sweep's start (the filtered list's
                                 // size); a list of >= N/dense_div ("dense") keeps the shared order and 1-bucket rounds
    int dense_div;
};

// Sweep order of replica rg: a random permutation of the vertices, or of chunks of CHUNK
// consecutive vertices whose grid is shifted by a per-(replica, sweep) offset in [0, CHUNK):
// with a fixed grid, two vertices closer than CHUNK would share a chunk -- and so decide
// simultaneously -- in every sweep (a dyad whose ends each join the other's singleton then
// swaps forever; LFR-1M final pass: 200 sweeps).  The chunk domain has room for the shift
// (cd_run: NC = (N + 2*CHUNK - 2) / CHUNK).  oracle/fc_oracle.c tw_pos_vertex restates it.
__device__ __forceinline__ Perm sweep_perm(const CDArgs& a, int rg, int sweep) {
    Perm P = make_perm(a.perm_n, stream_key(a.seed, (uint32_t)rg, a.iter, (uint32_t)sweep, 1));
    if (a.chunk) P.off = stream_key(a.seed, (uint32_t)rg, a.iter, (uint32_t)sweep, 3) & (CHUNK - 1);
    return P;
}
// Key of replica r's visit order this sweep: its own, or the shared one while its sweeps are
// full in the hybrid (the replica-lane engine runs those sweeps when the batch is wide enough;
// this engine runs them for narrow batches and for replicas still full after the hand-off).
__device__ __forceinline__ bool rep_full(const CDArgs& a, int r);
__device__ __forceinline__ int order_rg(const CDArgs& a, int r, bool shared) {
    return (a.shared_full && shared) ? (int)SHARED_RG : a.rbase + r;
}
// hybrid: replica r's filtered sweep still visits >= N/dense_div vertices -- the shared order, no coarse rounds
__device__ __forceinline__ bool rep_dense(const CDArgs& a, int r) {
    return a.shared_full && a.vcnt && !rep_full(a, r) && (int64_t)a.dense_div * a.vcnt[r] >= a.N;
}
// Vertex at sweep position p, or -1 for a padding slot.
__device__ __forceinline__ int32_t pos_vertex(const CDArgs& a, const Perm& P, int64_t p) {
    const uint32_t p32 = (uint32_t)p;
    if (!a.chunk) return (int32_t)perm_apply(P, p32);
    const int64_t w = (int64_t)perm_apply(P, p32 / CHUNK) * CHUNK + (p32 % CHUNK) - (int64_t)P.off;
    return (w >= 0 && w < a.N) ? (int32_t)w : -1;
}
// Sweep position of vertex v (inverse of pos_vertex).
__device__ __forceinline__ uint32_t vertex_pos(const CDArgs& a, const Perm& P, uint32_t v) {
    if (!a.chunk) return perm_invert(P, v);
    const uint32_t w = v + P.off;
    return perm_invert(P, w / CHUNK) * CHUNK + w % CHUNK;
}
// Replica r's sweep visits every position (no pruning filter yet): its "list" is implicit,
// entry di of bucket k = position k*S + di.
__device__ __forceinline__ bool rep_full(const CDArgs& a, int r) { return !(a.prune && a.track[a.n_r + r]); }
// Rounds of a filtered sweep of V vertices: g consecutive buckets per round, g the largest
// power of two <= B with V*g <= N (oracle/fc_oracle.c tw_coarse restates it).
__device__ __forceinline__ int coarse_factor(int64_t N, int64_t V, int B, int gmax) {
    int g = 1;
    while (2 * g <= B && 2 * g <= gmax && V * 2 * (int64_t)g <= N) g *= 2;
    return g;
}



__device__ __forceinline__ unsigned long long* red_slot(const CDArgs& a, int r, int f) {
    return a.red + ((size_t)r * NSH + (blockIdx.x & (NSH - 1))) * RF + f;
}

// Block -> (replica, chunk) with all chunks of a replica on as few XCDs as possible
// (blocks b and b+8 share an XCD under round-robin dispatch; speed only).
__device__ __forceinline__ void xcd_remap(int64_t b, int64_t total, int64_t per, int* r, int64_t* chunk) {
    const int64_t xcd = b & 7, q = total >> 3, rem = total & 7;
    const int64_t w = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (b >> 3);
    *r = (int)(w / per);
    *chunk = w % per;
}

__device__ __forceinline__ void tbl_insert(int32_t* keys, int32_t* vals, uint32_t mask, int32_t c, int32_t w) {
    uint32_t h = hash32((uint32_t)c) & mask;
    while (true) {
        const int32_t prev = atomicCAS(&keys[h], -1, c);
        if (prev == -1 || prev == c) { atomicAdd(&vals[h], w); return; }
        h = (h + 1) & mask;
    }
}
// Same, but returns the slot when THIS lane created it (the slot's owner evaluates it).
__device__ __forceinline__ int tbl_insert_owner(int32_t* keys, int32_t* vals, uint32_t mask, int32_t c, int32_t w) {
    uint32_t h = hash32((uint32_t)c) & mask;
    while (true) {
        const int32_t prev = atomicCAS(&keys[h], -1, c);
        if (prev == -1) { atomicAdd(&vals[h], w); return (int)h; }
        if (prev == c) { atomicAdd(&vals[h], w); return -1; }
        h = (h + 1) & mask;
    }
}

// Lexicographic best: larger score, then larger random tie key, then smaller id.
__device__ __forceinline__ bool better(long long s1, uint32_t h1, int32_t c1, long long s2, uint32_t h2, int32_t c2) {
    if (s1 != s2) return s1 > s2;
    if (h1 != h2) return h1 > h2;
    return c1 < c2;
}
__device__ __forceinline__ uint32_t tie_hash(uint32_t tbk, int32_t v, int32_t c) {
    return hash32(hash32(tbk ^ (uint32_t)v) ^ (uint32_t)c);
}

// Affected bits: one atomic OR per flag (a moved vertex's neighbour); 8x less memory than a
// byte per vertex, so a replica's flags (N/8 bytes) stay cache-resident between the movers
// that set them and the next sweep's list build
__device__ __forceinline__ void aff_set(uint32_t* affr, int32_t v) { atomicOr(affr + (v >> 5), 1u << (v & 31)); }
__device__ __forceinline__ bool aff_get(const uint32_t* affr, int64_t v) { return (affr[v >> 5] >> (v & 31)) & 1u; }
// Final decision shared by the light and heavy kernels (runs on one lane).
// Returns the target community or -1; writes predicted dQ (fixed point) / unstable flag.
template <bool LOUV, typename TT>
__device__ __forceinline__ int32_t decide_final(const CDArgs& a, int r, int32_t v, int32_t own, long long best_s,
                                                int32_t best_c, long long kown, int have_best,
                                                unsigned long long* dq_out, int* unstable_out) {
    *dq_out = 0;
    *unstable_out = 0;
    if (LOUV) {
        if (!have_best) return -1;
        const int64_t kv = a.kdeg[v];
        const int64_t tot_own = ((const TT*)a.tot)[(int64_t)r * a.N + own];
        const long long G = best_s - kown * a.M2 + kv * (tot_own - kv);
        if (G <= 0) return -1;
        const double dq = (double)G * 2.0 / ((double)a.M2 * (double)a.M2);
        *dq_out = (unsigned long long)llrint(dq * DQ_SCALE);
        return best_c;
    } else {
        if (!have_best) return -1;  // isolated vertex keeps its label
        *unstable_out = (kown != best_s);   // own label not dominant
        return best_c != own ? best_c : -1;
    }
}

// Result of one vertex visit (decide_wave, heavy_visit).  Louvain: move iff the best gain
// is > 0; LPA: the most frequent label.
struct Visit {
    int32_t dcs;               // target community, or -1
    unsigned long long dq;     // predicted modularity gain (fixed point, Louvain)
    int unst;                  // LPA: own label not dominant
    int ncand;                 // Sigma gathers (Louvain) / candidates (LPA)
    int64_t d;                 // degree
    int32_t own, kvw;          // own label and k_v (int32 when 2M < 2^31) for the decision record
    bool work, heavy;
    bool tied;                 // LPA: >= 2 dominant labels (the vertex redraws at every visit)
};
#ifdef FC_PHASE_PROF
// Diagnostic build only: cycles per phase of decide_wave, sampled on 1/64 of the blocks.
__device__ unsigned long long g_phase[16];
#define PST(i)                                                                          \
    do {                                                                                \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                     \
        const unsigned long long _t = __builtin_amdgcn_s_memtime();                     \
        if (_samp && lane == 0) atomicAdd(&g_phase[i], _t - _tp);                       \
        _tp = _t;                                                                       \
    } while (0)
#else
#define PST(i) do { } while (0)
#endif

// LDS of one wave: 8 vertex tables + per-vertex scratch.
struct WaveShared {
    int32_t key[WNT * HCAP];
    int32_t val[WNT * HCAP];
    long long best2[WNT];        // best exact score among lower-val candidates (rare path)
    long long tmin[WNT];         // min Sigma among the max-val candidates
    unsigned long long tb[WNT];  // int32 Sigma: best max-val candidate, (Sigma << 32) | ~tie hash (min wins)
    long long b1[WNT];           // int32 Sigma: score of that candidate
    unsigned long long k2[WNT];
    long long kv[WNT];
    int32_t vm[WNT], own[WNT], kown[WNT];
    uint32_t tvh[WNT];
    int32_t hope[WNT];           // Louvain: some candidate may gain (else no Sigma is gathered)
    int32_t ntie[WNT];           // LPA: labels at the largest count
};

__device__ __forceinline__ void wave_sync() {
    // one wave's LDS operations execute in order; only the compiler must not reorder
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// One wave decides 8 vertices (lane t < 8 brings vertex t; every lane of the wave calls).
// The 8 adjacency rows are FLATTENED over the 64 lanes (entry e of their concatenation goes
// to lane e % 64), so every lane loads and inserts useful entries (a 27-entry row on an
// 8-lane tile left most lanes idle and every entry behind its own branch).  Rows stream
// from nlab (push mode) or are gathered through lab[col] (pull); each vertex gets a 64-slot
// LDS hash table and the lane whose CAS creates a slot owns that candidate.  Per vertex,
// through LDS atomics: the max val over foreign communities; Sigma gathered only for the
// candidates of maximal val (score = val*2M - k_v*Sigma <= val*2M, so a lower one cannot
// win unless its bound still reaches the best exact score -- checked, rare); the best
// score; the best tie key among equal scores.  Python-louvain's rule: move iff the gain
// of the best community > 0; LPA: the most frequent label (own label competing).
// Returns vertex t's visit in lane t (< 8); ncand is per lane (sum it over the wave).
template <bool LOUV, typename TT>
__device__ __forceinline__ Visit decide_wave(const CDArgs& a, int r, int rg, int sweep, bool valid, int32_t v,
                                             bool push, bool trans, WaveShared& ws) {
    const int lane = threadIdx.x & 63;
    const int32_t* labr = a.lab + (int64_t)r * a.N;
    const TT* totr = (const TT*)a.tot + (int64_t)r * a.N;
    const int32_t* nlr = a.nlab + (int64_t)r * a.m2;
#ifdef FC_PHASE_PROF
    const bool _samp = (blockIdx.x & 63) == 0;
    unsigned long long _tp = __builtin_amdgcn_s_memtime();
#endif
    // ---- per-vertex state, lanes 0..7
    const bool vl = lane < WNT && valid;
    int64_t rb = 0, d = 0, kv = 0;
    int32_t own = -1;
    TT tot_own = 0;
    if (vl) {
        const int4 vr = a.vrec[v];               // one 16-byte load: row, degree, k_v, slot
        rb = (int64_t)(uint32_t)vr.x;
        d = vr.y;
        own = labr[vr.w];
        if (LOUV) kv = sizeof(TT) == 4 ? (int64_t)vr.z : a.kdeg[v];
    }
    PST(0);
    const bool heavy = vl && d > LIGHT_MAX_DEG;
    const bool work = vl && !heavy && d > 0;
    if (LOUV && work) tot_own = totr[own];       // in flight with the row loads below
    const int de = work ? (int)d : 0;
    int inc = de;                                // inclusive scan of the row lengths (lanes 0..7)
#pragma unroll
    for (int off = 1; off < WNT; off <<= 1) {
        const int y = __shfl_up(inc, off, WNT);
        if ((lane & (WNT - 1)) >= off) inc += y;
    }
    const int ex = inc - de;
    const long long jb = (long long)rb - ex;     // entry e of vertex t is adjacency entry jb_t + e
    {   // clear the 8 tables (16-byte stores) and the per-vertex scratch
        int4* k4 = reinterpret_cast<int4*>(ws.key);
        int4* v4 = reinterpret_cast<int4*>(ws.val);
#pragma unroll
        for (int s = lane; s < WNT * HCAP / 4; s += 64) { k4[s] = make_int4(-1, -1, -1, -1); v4[s] = make_int4(0, 0, 0, 0); }
        if (lane < WNT) {
            ws.best2[lane] = LLONG_MIN; ws.tmin[lane] = LLONG_MAX; ws.tb[lane] = ~0ull; ws.k2[lane] = 0; ws.vm[lane] = INT_MIN; ws.kown[lane] = 0;
            ws.ntie[lane] = 0;
            ws.own[lane] = work ? own : -1;
            ws.kv[lane] = kv;
            ws.tvh[lane] = hash32(stream_key(a.seed, rg, a.iter, sweep, 2) ^ (uint32_t)v);
        }
    }
    int o[WNT];
#pragma unroll
    for (int s = 0; s < WNT; ++s) o[s] = __shfl(ex, s);
    const int E = __shfl(inc, WNT - 1);
    // loads of 64 entries the wave holds (scalar): every loop over loads / owned slots stops
    // there instead of walking all 8 with per-lane exec masks (a consensus-graph wave has 3)
    const int nl = __builtin_amdgcn_readfirstlane((E + 63) >> 6);
    wave_sync();
    PST(1);
    // own labels of the 8 vertices (wave-uniform) and, on lane t, vertex t's own-label weight
    int32_t own_s[WNT];
#pragma unroll
    for (int q = 0; q < WNT; ++q) own_s[q] = __builtin_amdgcn_readlane(work ? own : -1, q);
    int kacc = 0;
    // ---- flattened rows: at most 2 chunks of 4 x 64 entries (8 rows of <= 64)
    int rec[8];                                  // owned slots: (t << 8) | slot, or -1
#pragma unroll
    for (int it = 0; it < 8; ++it) rec[it] = -1;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        if (c * 256 >= E) break;                 // wave-uniform
        int32_t kq[4], wq[4], tq[4];
        long long jq[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = c * 256 + u * 64 + lane;
            int t = 0;
#pragma unroll
            for (int s = 1; s < WNT; ++s) t += (e >= o[s]) ? 1 : 0;
            jq[u] = __shfl(jb, t) + e;
            const bool ok = e < E;
            kq[u] = ok ? (push ? nlr[jq[u]] : a.colp[jq[u]]) : -1;   // pull: a label slot
            wq[u] = ok ? ((LOUV && !a.unitw) ? a.cw[jq[u]] : 1) : 0;
            tq[u] = t;
        }
        PST(2);
        if (!push) {
#pragma unroll
            for (int u = 0; u < 4; ++u) kq[u] = kq[u] >= 0 ? labr[kq[u]] : -1;
            if (trans) {                         // transition sweep: these nlab entries, as seen now
                int32_t* nlw = a.nlab + (int64_t)r * a.m2;
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (kq[u] >= 0) nlw[jq[u]] = kq[u];
            }
        }
        if (a.own_bal) {                         // wave-uniform
            // Entries carrying their vertex's OWN label skip the table: in a settled pull sweep
            // about half of a row does (its in-community neighbours; nearly all of it on a
            // consensus graph), and those same-address LDS atomics serialise.  Those of weight
            // w0 (1 on unit graphs -- LPA, the input graph -- n_p on consensus graphs, where
            // agreement made most weights n_p) sum to w0 * count: lane t (< 8) counts its
            // lanes [ex - base, inc - base) of each load in one ballot.  Own entries of any
            // other weight still go to the table; kown adds both.
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                int32_t ow = own_s[0];
#pragma unroll
                for (int q = 1; q < WNT; ++q) ow = tq[u] == q ? own_s[q] : ow;
                const bool isown = kq[u] >= 0 && kq[u] == ow && wq[u] == a.w0;
                if (isown) kq[u] = -2;
                const int base = c * 256 + u * 64;
                const int lo = min(max(ex - base, 0), 64), hi = min(max(inc - base, 0), 64);
                const unsigned long long msk = (hi == 64 ? ~0ull : ((1ull << hi) - 1ull)) &
                                               ~(lo == 64 ? ~0ull : ((1ull << lo) - 1ull));
                const unsigned long long bal = __ballot(isown);
                if (bal && lane < WNT) kacc += (int)__popcll(bal & msk);
            }
        }
        PST(3);
        // insert: first probes back to back (one LDS round trip; a wave's LDS operations
        // execute in order, so entries of one key agree on its slot), then linear probing
        uint32_t hq[4];
        int32_t pv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            hq[u] = hash32((uint32_t)kq[u]) & (HCAP - 1);
            pv[u] = kq[u] >= 0 ? atomicCAS(&ws.key[tq[u] * HCAP + hq[u]], -1, kq[u]) : kq[u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (kq[u] < 0) continue;
            while (pv[u] != -1 && pv[u] != kq[u]) {
                hq[u] = (hq[u] + 1) & (HCAP - 1);
                pv[u] = atomicCAS(&ws.key[tq[u] * HCAP + hq[u]], -1, kq[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (kq[u] < 0) continue;
            atomicAdd(&ws.val[tq[u] * HCAP + hq[u]], wq[u]);
            if (pv[u] == -1) rec[c * 4 + u] = (tq[u] << 8) | (int)hq[u];
        }
        PST(4);
    }
    if (a.own_bal && lane < WNT) ws.kown[lane] = kacc * a.w0;   // the table's own slot adds to it below
    wave_sync();
    // ---- candidates: own-community weight; max val over the foreign ones (Louvain) or over
    // all labels (LPA)
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        if (it >= nl) break;                     // scalar: slots past the wave's loads are empty
        if (rec[it] < 0) continue;
        const int t = rec[it] >> 8, sl = t * HCAP + (rec[it] & 255);
        const int32_t key = ws.key[sl], val = ws.val[sl];
        if (key == ws.own[t]) {
            ws.kown[t] += val;                   // one owner per slot; the ballot sum landed before the barrier
            if (LOUV) { rec[it] = -1; continue; }   // LPA: the own label competes
        }
        if (LOUV) atomicMax(&ws.vm[t], val);
        // LPA: count and tie key in one packed max, (count << 32) | hash (the hash is a
        // bijection of the label: no id tie remains; the winner is recovered by inversion)
        else atomicMax(&ws.k2[t], ((unsigned long long)(uint32_t)val << 32) | hash32(ws.tvh[t] ^ (uint32_t)key));
    }
    wave_sync();
    if (!LOUV && a.own_bal && lane < WNT && kacc > 0) {   // LPA: the own label competes
        const unsigned long long ko = ((unsigned long long)(uint32_t)kacc << 32) | hash32(ws.tvh[lane] ^ (uint32_t)own);
        if (ko > ws.k2[lane]) ws.k2[lane] = ko;   // every other lane's max landed before the barrier
    }
    if (!LOUV && lane < WNT && ws.k2[lane]) ws.vm[lane] = (int32_t)(ws.k2[lane] >> 32);   // read by this lane only
    bool tied = false;
    if (!LOUV) {
        // ties at the top count: the table's labels at vm, plus the own label (counted by the
        // ballots, never in the table) when its count is vm too
        wave_sync();
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            if (it >= nl) break;
            if (rec[it] < 0) continue;
            const int t = rec[it] >> 8, sl = t * HCAP + (rec[it] & 255);
            if (ws.val[sl] == ws.vm[t]) atomicAdd(&ws.ntie[t], 1);
        }
        wave_sync();
        if (lane < WNT && ws.vm[lane] != INT_MIN)
            tied = ws.ntie[lane] + ((a.own_bal && kacc > 0 && kacc == ws.vm[lane]) ? 1 : 0) >= 2;
    }
    if (LOUV) {
        // no candidate can gain when even weight vm at Sigma = 0 cannot: (vm - k_own)*2M +
        // k_v*(Sigma_own - k_v) <= 0 (score_c <= vm*2M for every c) -- then the vertex stays and
        // no Sigma is gathered (most vertices of a settled sweep)
        if (lane < WNT)
            ws.hope[lane] = (work && ws.vm[lane] != INT_MIN &&
                             ((long long)ws.vm[lane] - ws.kown[lane]) * a.M2 + kv * ((long long)tot_own - kv) > 0) ? 1 : 0;
        wave_sync();
    }
    PST(5);
    int ncand = 0;
    auto score = [&](int32_t val, long long tt, long long kvt) -> long long {
        if constexpr (sizeof(TT) == 4)          // 2M < 2^31: k_v and Sigma fit 32 bits
            return (long long)val * (int32_t)a.M2 - (long long)(int32_t)kvt * (int32_t)tt;
        else
            return (long long)val * a.M2 - kvt * tt;
    };
    // best score of vertex t: Louvain max(vm*2M - k_v*min Sigma, rare lower-val best); LPA vm
    auto best_of = [&](int t) -> long long {
        if (!LOUV) return (long long)ws.vm[t];
        const long long b1 = score(ws.vm[t], ws.tmin[t], ws.kv[t]);
        return max(b1, ws.best2[t]);
    };
    TT tg[8];                                    // gathered Sigma (-1: not evaluated)
#pragma unroll
    for (int it = 0; it < 8; ++it) tg[it] = (TT)-1;
    // int32 Sigma (Louvain): among the max-val candidates score = vm*2M - k_v*Sigma, so the
    // best one and its tie key come from ONE packed atomicMin per candidate,
    // (Sigma << 32) | ~hash (smallest Sigma, then largest hash; Sigma taken as 0 when k_v = 0,
    // where they all tie); the hash is a bijection of the id, so no id tie remains and the
    // winner's id is recovered by inverting it.  The separate tie pass runs only when a
    // lower-val candidate may still reach the best score (rare).
    constexpr bool PK = LOUV && sizeof(TT) == 4;
    bool slow = LOUV && !PK;                     // wave-uniform: generic tie pass (k2)
    if (LOUV) {
        // among the max-val candidates the score is vm*2M - k_v*Sigma: the smallest Sigma wins
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            if (it >= nl) break;
            if (rec[it] < 0) continue;
            const int t = rec[it] >> 8, sl = t * HCAP + (rec[it] & 255);
            if (ws.val[sl] == ws.vm[t] && ws.hope[t]) tg[it] = totr[ws.key[sl]];
        }
        if constexpr (PK) {
#pragma unroll
            for (int it = 0; it < 8; ++it) {
                if (it >= nl) break;
                if (tg[it] < 0) continue;
                ++ncand;
                const int t = rec[it] >> 8, sl = t * HCAP + (rec[it] & 255);
                const uint32_t h = hash32(ws.tvh[t] ^ (uint32_t)ws.key[sl]);
                const uint32_t sg = ws.kv[t] ? (uint32_t)tg[it] : 0u;
                atomicMin(&ws.tb[t], ((unsigned long long)sg << 32) | (uint32_t)~h);
            }
            wave_sync();
            if (lane < WNT && ws.vm[lane] != INT_MIN) {
                ws.tmin[lane] = (long long)(ws.tb[lane] >> 32);
                ws.b1[lane] = score(ws.vm[lane], ws.tmin[lane], ws.kv[lane]);
            }
            wave_sync();
        } else {
#pragma unroll
            for (int it = 0; it < 8; ++it) {
                if (it >= nl) break;
                if (tg[it] >= 0) { ++ncand; atomicMin(&ws.tmin[rec[it] >> 8], (long long)tg[it]); }
            }
            wave_sync();
        }
        // a lower val whose bound val*2M still reaches that score (rare: k_v*Sigma >= 2M)
        bool need = false;
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            if (it >= nl) break;
            if (rec[it] < 0 || tg[it] >= 0) continue;
            const int t = rec[it] >> 8;
            if (!ws.hope[t]) continue;
            const long long b1 = PK ? ws.b1[t] : score(ws.vm[t], ws.tmin[t], ws.kv[t]);
            need |= (long long)ws.val[t * HCAP + (rec[it] & 255)] * a.M2 >= b1;
        }
        if (__any(need)) {                       // wave-uniform
            slow = true;
#pragma unroll
            for (int it = 0; it < 8; ++it) {
                if (it >= nl) break;
                if (rec[it] < 0 || tg[it] >= 0) continue;
                const int t = rec[it] >> 8, sl = t * HCAP + (rec[it] & 255);
                if (!ws.hope[t]) continue;
                const int32_t val = ws.val[sl];
                if ((long long)val * a.M2 < score(ws.vm[t], ws.tmin[t], ws.kv[t])) continue;
                tg[it] = totr[ws.key[sl]];
                ++ncand;
                atomicMax(&ws.best2[t], score(val, tg[it], ws.kv[t]));
            }
            wave_sync();
        }
    } else {
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            if (it >= nl) break;
            if (rec[it] >= 0) { tg[it] = 0; ++ncand; }
        }
    }
    PST(6);
    // tie key among the candidates at the best score: larger hash, then smaller id
    if (slow) {                                  // wave-uniform
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            if (it >= nl) break;
            if (tg[it] < 0) continue;
            const int t = rec[it] >> 8, sl = t * HCAP + (rec[it] & 255);
            const int32_t key = ws.key[sl], val = ws.val[sl];
            const long long sc = LOUV ? score(val, tg[it], ws.kv[t]) : (long long)val;
            if (sc != best_of(t)) continue;
            atomicMax(&ws.k2[t], ((unsigned long long)hash32(ws.tvh[t] ^ (uint32_t)key) << 32) | (uint32_t)~key);
        }
        wave_sync();
    }
    PST(7);
    // ---- the decision, lanes 0..7
    Visit out;
    out.dcs = -1; out.dq = 0; out.unst = 0; out.ncand = ncand; out.d = d; out.work = work; out.heavy = heavy;
    out.tied = tied && work;
    out.own = own; out.kvw = (int32_t)kv;
    if (work && ws.vm[lane] != INT_MIN && (!LOUV || ws.hope[lane])) {   // a candidate that may gain (Louvain)
        const long long best_s = best_of(lane);
        {
            const int32_t best_c = !LOUV ? (int32_t)(hash32_inv((uint32_t)ws.k2[lane]) ^ ws.tvh[lane])
                                 : slow ? (int32_t)~(uint32_t)ws.k2[lane]
                                        : (int32_t)(hash32_inv(~(uint32_t)ws.tb[lane]) ^ ws.tvh[lane]);
            const TT kown = (TT)ws.kown[lane];
            if (LOUV) {
                const long long G = best_s - (long long)kown * a.M2 + kv * ((long long)tot_own - kv);
                if (G > 0) {
                    const double dqd = (double)G * 2.0 / ((double)a.M2 * (double)a.M2);
                    out.dq = (unsigned long long)llrint(dqd * DQ_SCALE);
                    out.dcs = best_c;
                }
            } else {
                out.unst = (long long)kown != best_s;   // own label not dominant
                out.dcs = best_c != own ? best_c : -1;
            }
        }
    }
    PST(8);
    return out;
}

template <bool LOUV, typename TT>
__global__ __launch_bounds__(DTB) __attribute__((amdgpu_waves_per_eu(8))) void k_decide_light(CDArgs a, int bucket, int sweep,
                                                                                         int X) {
    __shared__ WaveShared s_ws[DTB / 64];
    __shared__ unsigned long long s_red[2][DTB / 64][5];   // by item parity (no second barrier)
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // One item (LNT list entries of one replica) per block.  Every replica owns X item slots
    // (X = the sweep's largest per-replica round, from the host's one read per sweep); slots
    // past a replica's entries return at once.  XCD x (blocks b with b % 8 == x, round-robin
    // dispatch) takes the contiguous slots [x*q, (x+1)*q), so a replica's items share an L2.
    const uint32_t W = (uint32_t)a.n_r * (uint32_t)X, q = (W + 7) / 8;
    const uint32_t w = (blockIdx.x & 7) * q + (blockIdx.x >> 3);
    if ((blockIdx.x >> 3) >= q || w >= W) return;                       // block-uniform
    const int r = (int)(w / (uint32_t)X);
    const int i = (int)(w - (uint32_t)r * (uint32_t)X);
    const int4 rr = a.rrec[(int64_t)bucket * a.n_r + r];                // one scalar load
    const int cnt = rr.y - i * LNT;
    if (cnt <= 0) return;                                                // block-uniform
    auto item = [&](int par) {
    const int slot = wv * WNT + lane;
    const int64_t di = (int64_t)i * LNT + slot;                          // decision slot (lane < 8)
    const bool in_range = lane < WNT && slot < cnt;
    const int rg = a.rbase + r;
    int32_t v = -1;
    if (in_range) {
        if (rr.z & RR_FULL) v = pos_vertex(a, sweep_perm(a, order_rg(a, r, true), sweep),
                                           (int64_t)rr.x + di);
        else v = a.list[(int64_t)r * a.PN + rr.x + di];                  // vertex ids
    }
    const bool valid = in_range && v >= 0;
    const Visit vis = decide_wave<LOUV, TT>(a, r, rg, sweep, valid, v, (rr.z & RR_PUSH) != 0, (rr.z & RR_TRANS) != 0,
                                            s_ws[wv]);
    if (in_range) {
        // LPA, tracked sweep: a vertex with several dominant labels is revisited next sweep
        if (!LOUV && vis.tied && a.track[r]) aff_set(a.aff + (int64_t)r * a.aw, v);
        a.dec[(int64_t)r * a.dstride + di] = make_int4(v >= 0 ? vis.dcs : -1, v, vis.own, vis.kvw);   // heavy: .x later
        if (vis.heavy) {
            const int hq = atomicAdd(a.heavy_cnt, 1);
            a.heavy[3 * hq] = r;
            a.heavy[3 * hq + 1] = (int32_t)di;
            a.heavy[3 * hq + 2] = v;
        }
    }
    // ---- block counters: per-vertex fields on lanes 0..7, candidates on every lane
    unsigned long long f0 = lane < WNT ? vis.dq : 0;
    unsigned f1 = lane < WNT ? (unsigned)vis.unst : 0u, f2 = (lane < WNT && vis.work) ? 1u : 0u;
    unsigned f3 = (lane < WNT && vis.work) ? (unsigned)vis.d : 0u, f4 = (unsigned)vis.ncand;
#pragma unroll
    for (int off = WNT / 2; off > 0; off >>= 1) {
        f0 += __shfl_xor(f0, off, WNT); f1 += __shfl_xor(f1, off, WNT); f2 += __shfl_xor(f2, off, WNT);
        f3 += __shfl_xor(f3, off, WNT);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) f4 += __shfl_xor(f4, off);
    if (lane == 0) {
        s_red[par][wv][0] = f0; s_red[par][wv][1] = f1; s_red[par][wv][2] = f2; s_red[par][wv][3] = f3;
        s_red[par][wv][4] = f4;
    }
    __syncthreads();
    if (threadIdx.x < 5) {
        unsigned long long sm = 0;
        for (int k = 0; k < DTB / 64; ++k) sm += s_red[par][k][threadIdx.x];
        // fields: s_red 0 dq -> 0, 1 unstable -> 1, 2 verts -> 3, 3 entries -> 4, 4 cands -> 5
        if (sm) atomicAdd(red_slot(a, r, threadIdx.x < 2 ? threadIdx.x : threadIdx.x + 1), sm);
    }
    };   // item
    item(0);
}

// A high-degree vertex decided by a whole 256-thread block (every thread calls it).  Table
// in LDS when it fits, else the block's global slice `scratch`.  Returns the decision on
// thread 0 (dq / unstable through the pointers).
template <int NTH>
struct HeavyShared {
    int32_t key[HEAVY_LDS_SLOTS];
    int32_t val[HEAVY_LDS_SLOTS];
    long long s[NTH];
    uint32_t h[NTH];
    int32_t c[NTH];
    int have[NTH];
    long long kown[NTH];
};
template <bool LOUV, typename TT, int NTH>
__device__ int32_t heavy_visit(const CDArgs& a, int r, int sweep, int32_t v, HeavyShared<NTH>& sh, int32_t* scratch,
                               unsigned long long* dq_out, int* unst_out, bool* tied_out = nullptr) {
    const int rg = a.rbase + r;
    const uint32_t tbk = stream_key(a.seed, rg, a.iter, sweep, 2);
    const int64_t rb = a.rowptr[v], d = a.rowptr[v + 1] - rb;
    uint32_t slots = 1;
    while (slots < 2 * (uint32_t)d) slots <<= 1;
    int32_t* keys;
    int32_t* vals;
    if (slots <= HEAVY_LDS_SLOTS) { keys = sh.key; vals = sh.val; }
    else {
        slots = (uint32_t)a.heavy_slots;
        keys = scratch;
        vals = keys + slots;
    }
    for (uint32_t s = threadIdx.x; s < slots; s += NTH) { keys[s] = -1; vals[s] = 0; }
    __syncthreads();
    const int32_t* labr = a.lab + (int64_t)r * a.N;
    const int32_t* nlr = a.nlab + (int64_t)r * a.m2;
    const bool push = a.track[2 * a.n_r + r] != 0, trans = a.track[3 * a.n_r + r] != 0;
    for (int64_t j = rb + threadIdx.x; j < rb + d; j += NTH) {
        const int32_t lj = push ? nlr[j] : labr[a.colp[j]];
        if (trans) a.nlab[(int64_t)r * a.m2 + j] = lj;   // transition sweep (see decide_wave)
        tbl_insert(keys, vals, slots - 1, lj, LOUV ? a.cw[j] : 1);
    }
    __syncthreads();
    const int32_t own = labr[a.spos[v]];
    const int64_t kv = a.kdeg[v];
    const TT* totr = (const TT*)a.tot + (int64_t)r * a.N;
    long long best_s = LLONG_MIN, kown = 0;
    uint32_t best_h = 0;
    int32_t best_c = 0x7fffffff;
    int have = 0;
    for (uint32_t s = threadIdx.x; s < slots; s += NTH) {
        const int32_t key = keys[s];
        if (key < 0) continue;
        const int32_t val = vals[s];
        if (key == own) kown = val;
        long long sc;
        if (LOUV) {
            if (key == own) continue;
            sc = (long long)val * a.M2 - kv * (long long)totr[key];
        } else {
            sc = val;
        }
        const uint32_t h = tie_hash(tbk, v, key);
        if (!have || better(sc, h, key, best_s, best_h, best_c)) { best_s = sc; best_h = h; best_c = key; have = 1; }
    }
    sh.s[threadIdx.x] = best_s; sh.h[threadIdx.x] = best_h; sh.c[threadIdx.x] = best_c;
    sh.have[threadIdx.x] = have; sh.kown[threadIdx.x] = kown;
    __syncthreads();
    for (int o = NTH / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            const int t2 = threadIdx.x + o;
            if (sh.have[t2] && (!sh.have[threadIdx.x] ||
                                better(sh.s[t2], sh.h[t2], sh.c[t2], sh.s[threadIdx.x], sh.h[threadIdx.x], sh.c[threadIdx.x]))) {
                sh.s[threadIdx.x] = sh.s[t2]; sh.h[threadIdx.x] = sh.h[t2]; sh.c[threadIdx.x] = sh.c[t2];
                sh.have[threadIdx.x] = 1;
            }
            sh.kown[threadIdx.x] += sh.kown[t2];
        }
        __syncthreads();
    }
    int32_t dcs = -1;
    if (!LOUV) {   // LPA: labels at the top count (ties redraw at every visit: revisited while tracking)
        const long long top = sh.s[0];
        const int hv0 = sh.have[0];
        __syncthreads();                         // every thread has read the reduction's result
        if (threadIdx.x == 0) sh.have[0] = 0;
        __syncthreads();
        int nt = 0;
        if (hv0)
            for (uint32_t s = threadIdx.x; s < slots; s += NTH) nt += (keys[s] >= 0 && (long long)vals[s] == top) ? 1 : 0;
        if (nt) atomicAdd(&sh.have[0], nt);
        __syncthreads();
        if (threadIdx.x == 0) {
            if (tied_out) *tied_out = sh.have[0] >= 2;
            sh.have[0] = hv0;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        dcs = decide_final<LOUV, TT>(a, r, v, own, sh.s[0], sh.c[0], sh.kown[0], sh.have[0], dq_out, unst_out);
    __syncthreads();
    return dcs;
}

// Workgroup per high-degree vertex of the bucket (listed by k_decide_light).
template <bool LOUV, typename TT>
__global__ __launch_bounds__(256) void k_decide_heavy(CDArgs a, int bucket, int sweep) {
    __shared__ HeavyShared<TB> sh;
    const int cnt = *a.heavy_cnt;
    for (int item = blockIdx.x; item < cnt; item += gridDim.x) {
        const int r = a.heavy[3 * item];
        const int64_t di = a.heavy[3 * item + 1];
        const int32_t v = a.heavy[3 * item + 2];
        unsigned long long dq = 0;
        int unst = 0;
        bool tied = false;
        const int32_t dcs = heavy_visit<LOUV, TT, TB>(a, r, sweep, v, sh, a.heavy_scratch + (int64_t)blockIdx.x * 2 * a.heavy_slots,
                                                  &dq, &unst, &tied);
        if (threadIdx.x == 0) {
            if (!LOUV && tied && a.track[r]) aff_set(a.aff + (int64_t)r * a.aw, v);
            a.dec[(int64_t)r * a.dstride + di].x = dcs;   // the light kernel wrote v, own, k_v
            if (dq) atomicAdd(red_slot(a, r, 0), dq);
            if (unst) atomicAdd(red_slot(a, r, 1), 1ull);
        }
    }
}

// Apply a bucket's decisions (fixed grid: blockIdx.y = replica, blocks stride over the
// replica's list).  Label + community totals only (the replica neither pushes nor tracks
// this sweep): one thread per decision slot.  Otherwise one 16-lane tile per slot: lane 0
// updates the label and the totals, the tile scatters the new label into the reverse
// adjacency entries (nlab) and, while tracking, flags the neighbours for the next sweep.
template <bool LOUV, typename TT>
__device__ __forceinline__ void apply_move(const CDArgs& a, int r, const int4& dv, int32_t slot) {
    const int32_t d = dv.x, v = dv.y, old = dv.z;
    a.lab[(int64_t)r * a.N + slot] = d;
    if (LOUV) {
        TT* tot = (TT*)a.tot + (int64_t)r * a.N;
        const TT kv = sizeof(TT) == 4 ? (TT)dv.w : (TT)a.kdeg[v];
        if constexpr (sizeof(TT) == 8) {
            atomicAdd((unsigned long long*)&tot[old], (unsigned long long)(-(long long)kv));
            atomicAdd((unsigned long long*)&tot[d], (unsigned long long)kv);
        } else {
            atomicAdd((int*)&tot[old], -(int)kv);
            atomicAdd((int*)&tot[d], (int)kv);
        }
    }
}
template <bool LOUV, typename TT>
__global__ __launch_bounds__(ATB) void k_apply(CDArgs a, int bucket) {
    const int r = blockIdx.y;
    // the round's heavy list was consumed by k_decide_heavy: empty it for the next round
    // (one store here instead of a memset launch per round)
    if (blockIdx.x == 0 && r == 0 && threadIdx.x == 0) *a.heavy_cnt = 0;
    if (!a.active[r]) return;
    const int64_t seg = (int64_t)bucket * a.n_r + r;
    const int64_t len = a.lcnt[seg];
    const int4* decr = a.dec + (int64_t)r * a.dstride;
    const bool push = a.track[2 * a.n_r + r] != 0 || a.track[3 * a.n_r + r] != 0, trk = a.track[r] != 0;
    int moved = 0;
    if (!push && (!trk || a.lm)) {               // lm: a tracked move only flags the mover
        uint8_t* mv = a.mvf + (int64_t)r * a.N;
        for (int64_t di = (int64_t)blockIdx.x * ATB + threadIdx.x; di < len; di += (int64_t)gridDim.x * ATB) {
            const int4 dv = decr[di];
            if (dv.x >= 0) {
                apply_move<LOUV, TT>(a, r, dv, a.spos[dv.y]);
                ++moved;
                if (trk) mv[dv.y] = 1;
            }
        }
    } else {
        const int tile = threadIdx.x / TILE, lane = threadIdx.x % TILE;
        int32_t* nlr = a.nlab + (int64_t)r * a.m2;
        uint32_t* aff = a.aff + (int64_t)r * a.aw;
        for (int64_t di = (int64_t)blockIdx.x * TILES + tile; di < len; di += (int64_t)gridDim.x * TILES) {
            const int4 dv = decr[di];
            const int32_t d = dv.x, v = dv.y;
            if (d < 0) continue;
            const int4 vr = a.vrec[v];
            if (lane == 0) { apply_move<LOUV, TT>(a, r, dv, vr.w); ++moved; }
            const int64_t rb = (int64_t)(uint32_t)vr.x, re = rb + vr.y;
            if (push && trk) {
                for (int64_t j = rb + lane; j < re; j += TILE) {
                    nlr[a.rev[j]] = d;     // neighbours now see v's new community
                    aff_set(aff, a.col[j]);   // ... and are revisited next sweep (pruning)
                }
            } else if (push) {
                for (int64_t j = rb + lane; j < re; j += TILE) nlr[a.rev[j]] = d;
            } else {
                for (int64_t j = rb + lane; j < re; j += TILE) aff_set(aff, a.col[j]);
            }
        }
    }
    __shared__ int s_mv;
    if (threadIdx.x == 0) s_mv = 0;
    __syncthreads();
    if (moved) atomicAdd(&s_mv, moved);
    __syncthreads();
    if (threadIdx.x == 0 && s_mv) atomicAdd(red_slot(a, r, 2), (unsigned long long)s_mv);
}

// End of a tracked sweep in lm mode: each mover v marks the neighbours whose label now
// differs from v's (Traag et al.'s fast local moving rule: a neighbour that ended in v's
// community is not revisited), comparing the labels the sweep left -- deterministic, unlike a
// mark at move time, which would race with the round's other moves.
// A wave takes its 64 vertices' movers one at a time and walks each mover's row with all 64
// lanes (one row = one round of independent gathers), instead of one thread walking a row
// while the wave's non-movers idle.
__global__ __launch_bounds__(256) void k_mark_lm(CDArgs a) {
    const int r = blockIdx.y;
    if (!a.active[r] || !a.track[r]) return;     // block-uniform: this sweep was not tracked
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint8_t* mv = a.mvf + (int64_t)r * a.N;
    const bool moved = v < a.N && mv[v];         // no early exit: every lane walks the rows
    if (moved) mv[v] = 0;
    unsigned long long m = __ballot(moved);
    const int lane = threadIdx.x & 63;
    const int64_t v0 = v - lane;
    const int32_t* labr = a.lab + (int64_t)r * a.N;
    uint32_t* aff = a.aff + (int64_t)r * a.aw;
    // four movers at a time, 16 lanes each (rows of ~20-30 entries left most of a 64-lane wave
    // idle through each mover's chain of loads); the flags are ORs, so the order is free
    const int grp = lane >> 4, gl = lane & 15;
    while (m) {
        int b = -1;
        for (int g = 0; g < 4 && m; ++g) {        // group g takes the g-th remaining mover
            const int l = __ffsll((long long)m) - 1;
            m &= m - 1;
            if (g == grp) b = l;
        }
        if (b < 0) continue;
        const int4 vr = a.vrec[v0 + b];
        const int32_t d = labr[vr.w];
        const int64_t rb = (int64_t)(uint32_t)vr.x, re = rb + vr.y;
        for (int64_t j = rb + gl; j < re; j += 16)
            if (labr[a.colp[j]] != d) aff_set(aff, a.col[j]);
    }
}

// End of sweep: python-louvain stops a level when the pass gained < 1e-7 modularity or
// moved nothing; igraph LPA stops when no visited vertex was unstable.
template <bool LOUV>
__global__ void k_sweep_end(CDArgs a, int32_t* n_active_out) {
    __shared__ int cnt, cnt0;
    __shared__ unsigned long long mv, vis;
    if (threadIdx.x == 0) { cnt = 0; cnt0 = 0; mv = 0; vis = 0; }
    __syncthreads();
    for (int r = threadIdx.x; r < a.n_r; r += blockDim.x) {
        unsigned long long f[RF] = {0, 0, 0, 0, 0, 0, 0, 0};
        unsigned long long* base = a.red + (size_t)r * NSH * RF;
        for (int sh = 0; sh < NSH; ++sh)
            for (int k = 0; k < RF; ++k) { f[k] += base[sh * RF + k]; base[sh * RF + k] = 0; }
        a.sacc[4 * r + 0] += f[3]; a.sacc[4 * r + 1] += f[4]; a.sacc[4 * r + 2] += f[5];
        atomicAdd(&mv, f[2]);
        atomicAdd(&vis, f[3]);
        if (a.prune) {   // lists filter next sweep iff moves were tracked this sweep
            a.track[a.n_r + r] = a.track[r];
            if (a.lm || f[2] * (unsigned long long)a.track_div < (unsigned long long)a.N) a.track[r] = 1;
        }
        // pull -> push once a sweep moved < N/4 vertices (push pays d writes per MOVE,
        // pull d gathers per VISIT), through one transition sweep that builds nlab
        if (a.track[3 * a.n_r + r]) { a.track[3 * a.n_r + r] = 0; a.track[2 * a.n_r + r] = 1; }
        // (only into an UNFILTERED sweep: the transition writes the nlab row of every vertex it
        // visits, so it must visit them all; a replica already filtering stays in pull mode)
        else if (a.push_div && !a.track[2 * a.n_r + r] && !a.track[a.n_r + r] &&
                 f[2] * (unsigned long long)a.push_div < (unsigned long long)a.N)
            a.track[3 * a.n_r + r] = 1;
        if (a.active[r]) {
            atomicAdd(&cnt0, 1);
            bool stop;
            if (LOUV) stop = f[2] == 0 || ((double)f[0] / DQ_SCALE) < a.min_dq;
            else stop = f[1] == 0;
            if (stop) a.active[r] = 0;
            else atomicAdd(&cnt, 1);
        }
    }
    __syncthreads();
    // n_active_out: [0] active after, [2..3] u64 moves, [4..5] u64 replica-sweeps so far,
    // [6..7] u64 light-kernel visits of this sweep
    if (threadIdx.x == 0) {
        n_active_out[0] = cnt;
        *(unsigned long long*)(n_active_out + 2) = mv;
        *(unsigned long long*)(n_active_out + 4) += (unsigned long long)cnt0;
        *(unsigned long long*)(n_active_out + 6) = vis;
    }
}

// Singletons: label row in slot order (slot i holds vertex sinv[i]), totals in vertex order.
template <typename TT>
__global__ void k_cd_init(int64_t n, int n_r, const int64_t* kdeg, const int32_t* sinv, int32_t* lab, TT* tot,
                          int louv) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int r = blockIdx.y;
    if (i >= n) return;
    lab[(int64_t)r * n + i] = sinv[i];
    if (louv) tot[(int64_t)r * n + i] = (TT)kdeg[i];
}

// ------------------------------------------------------------------ tail sweeps
// Once pruning has shrunk the sweeps to a few thousand visits per replica, a multi-kernel
// sweep is bound by its ~100 launches, not by work.  k_cd_tail then runs every remaining
// sweep of one replica inside one workgroup, with exactly the semantics of the
// multi-kernel path (same visit sets, buckets, decisions, pruning and mode bookkeeping):
//   * the visit list of the next sweep is a worklist: a move's neighbours are appended
//     when their mark (int32 epoch stamp, tailmark[r][N]) is raised to this sweep -- the
//     set the aff flags would hold -- so no pass over all N vertices;
//   * the worklist is bucketed by inverse permutation (counting sort in LDS);
//   * per bucket: light decisions (8-lane tiles, 32 per pass), heavy rows (whole block),
//     barrier, moves applied, barrier.
// The first sweep's visit list is the one k_list_fill built for it (bucketed, flags cleared).
static constexpr int TAIL_MAXB = 256;
#ifndef FC_TAIL_TB
#define FC_TAIL_TB 1024
#endif
static constexpr int TAIL_TB = FC_TAIL_TB;   // threads per replica workgroup in k_cd_tail
template <bool LOUV, typename TT, int NTH>
__global__ __launch_bounds__(NTH) void k_cd_tail(CDArgs a, int sweep0, int max_sweeps, int32_t* tbuf,
                                                 int32_t* tmark, unsigned long long* tail_acc, int32_t* n_active_out) {
    const int B = a.B;
    __shared__ WaveShared s_ws[NTH / 64];
    __shared__ HeavyShared<NTH> sh;
    __shared__ int s_off[TAIL_MAXB + 1], s_cur[TAIL_MAXB];
    __shared__ int s_n, s_nnext, s_nheavy, s_stop, s_nmv;
    __shared__ unsigned long long s_acc[6];   // dq, unstable, moves, verts, entries, cands
    const int r = blockIdx.x;
    if (!a.active[r]) return;                 // block-uniform
    const int rg = a.rbase + r;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int32_t* wl = tbuf + (int64_t)r * 3 * a.N;
    int32_t* wl2 = wl + a.N;
    int32_t* bl = wl2 + a.N;
    int32_t* mark = tmark + (int64_t)r * a.N;
    int4* decr = a.dec + (int64_t)r * a.dstride;
    int32_t* hv = a.heavy + (int64_t)r * a.hcap;
    int32_t* scratch = a.heavy_scratch ? a.heavy_scratch + (int64_t)blockIdx.x * 2 * a.heavy_slots : nullptr;
    const int32_t* lo0 = a.loff + (int64_t)r * (B + 1);
    if (threadIdx.x == 0) s_n = lo0[B];       // the first sweep's list (k_list_fill), when filtered
    __syncthreads();
    bool first = true;
    for (int sweep = sweep0; sweep < max_sweeps; ++sweep) {
        const bool full = rep_full(a, r);
        const bool push = a.track[2 * a.n_r + r] != 0 || a.track[3 * a.n_r + r] != 0, trk = a.track[r] != 0;
        const bool dpush = a.track[2 * a.n_r + r] != 0, dtrans = a.track[3 * a.n_r + r] != 0;
        const int n = s_n;                    // this sweep's list (when filtered)
        const bool dense = a.shared_full && a.dense_div && !full && (int64_t)a.dense_div * n >= a.N;   // rep_dense, from the list
        const Perm P = sweep_perm(a, order_rg(a, r, full || dense), sweep);
        const int32_t stamp = sweep + 1;
        __syncthreads();                      // every thread has read s_n
        for (int k = threadIdx.x; k <= B; k += NTH) s_off[k] = 0;
        if (threadIdx.x < 6) s_acc[threadIdx.x] = 0;
        if (threadIdx.x == 0) { s_nnext = 0; s_stop = 0; s_nheavy = 0; s_nmv = 0; }
        __syncthreads();
        const int32_t* blp = bl;
        if (!full && first) {                 // rounds as k_list_plan laid them out: round j = buckets [j*g, (j+1)*g)
            const int g0 = (a.coarsen && !dense) ? coarse_factor(a.N, (int64_t)n, B, a.coarsen) : 1;
            for (int k = threadIdx.x; k <= B; k += NTH) s_off[k] = lo0[(k + g0 - 1) / g0];
            blp = a.list + (int64_t)r * a.PN;
            __syncthreads();
        } else if (!full) {                   // bucket the worklist (order inside a bucket is immaterial)
            for (int i = threadIdx.x; i < n; i += NTH) {
                const uint32_t v = (uint32_t)wl[i];
                const uint32_t pos = vertex_pos(a, P, v);
                atomicAdd(&s_off[pos / (uint32_t)a.S + 1], 1);
            }
            __syncthreads();
            if (threadIdx.x == 0)
                for (int k = 0; k < B; ++k) { s_off[k + 1] += s_off[k]; s_cur[k] = s_off[k]; }
            __syncthreads();
            for (int i = threadIdx.x; i < n; i += NTH) {
                const uint32_t v = (uint32_t)wl[i];
                const uint32_t pos = vertex_pos(a, P, v);
                bl[atomicAdd(&s_cur[pos / (uint32_t)a.S], 1)] = (int32_t)v;
            }
            __syncthreads();
        }
        // rounds: one bucket each, or g consecutive buckets of a filtered sweep (k_list_plan)
        const int g = (!full && !dense && a.coarsen) ? coarse_factor(a.N, (int64_t)n, B, a.coarsen) : 1;
        for (int k = 0; k < B; k += g) {
            const int k1 = min(B, k + g);
            const int64_t nk = full ? min(a.S, a.PN - (int64_t)k * a.S) : (int64_t)(s_off[k1] - s_off[k]);
            // (s_nheavy was zeroed before the previous bucket's last barrier, or before the sweep's)
            for (int64_t base = wv * WNT; base < nk; base += WNT * (NTH / 64)) {   // wave-uniform (waves are independent)
                const int64_t idx = base + lane;
                const bool in = lane < WNT && idx < nk;
                int32_t v = -1;
                if (in) v = full ? pos_vertex(a, P, (int64_t)k * a.S + idx) : blp[s_off[k] + idx];
                const Visit vis = decide_wave<LOUV, TT>(a, r, rg, sweep, in && v >= 0, v, dpush, dtrans, s_ws[wv]);
                unsigned nc = (unsigned)vis.ncand;
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) nc += __shfl_xor(nc, off);
                if (lane == 0 && nc) atomicAdd(&s_acc[5], (unsigned long long)nc);
                if (in) {
                    decr[idx] = make_int4(v >= 0 ? vis.dcs : -1, v, vis.own, vis.kvw);
                    // LPA, tracked: a tied vertex joins the next worklist itself
                    if (!LOUV && vis.tied && trk && atomicMax(&mark[v], stamp) < stamp) wl2[atomicAdd(&s_nnext, 1)] = v;
                    if (vis.heavy) hv[atomicAdd(&s_nheavy, 1)] = (int32_t)idx;
                    if (vis.dq) atomicAdd(&s_acc[0], vis.dq);
                    if (vis.unst) atomicAdd(&s_acc[1], 1ull);
                    if (vis.work) {
                        atomicAdd(&s_acc[3], 1ull);
                        atomicAdd(&s_acc[4], (unsigned long long)vis.d);
                    }
                }
            }
            __syncthreads();
            const int nh = s_nheavy;
            for (int h = 0; h < nh; ++h) {    // block-uniform (heavy_visit holds block barriers)
                const int32_t idx = hv[h];
                const int32_t v = decr[idx].y;
                unsigned long long dq = 0;
                int unst = 0;
                bool tied = false;
                const int32_t dcs = heavy_visit<LOUV, TT, NTH>(a, r, sweep, v, sh, scratch, &dq, &unst, &tied);
                if (threadIdx.x == 0) {
                    if (!LOUV && tied && trk && atomicMax(&mark[v], stamp) < stamp) wl2[atomicAdd(&s_nnext, 1)] = v;
                    decr[idx].x = dcs;
                    if (dq) atomicAdd(&s_acc[0], dq);
                    if (unst) atomicAdd(&s_acc[1], 1ull);
                }
            }
            if (nh) __syncthreads();          // block-uniform: heavy decisions land before the moves
            if (threadIdx.x == 0) s_nheavy = 0;   // read above; next bucket's decide appends after the barrier below
            // apply the bucket's moves; while tracking, neighbours join the next worklist
            int moved = 0;
            if (!push && (!trk || a.lm)) {       // lm: a tracked move joins the sweep's mover list
                for (int64_t di = threadIdx.x; di < nk; di += NTH) {
                    const int4 dv = decr[di];
                    if (dv.x >= 0) {
                        apply_move<LOUV, TT>(a, r, dv, a.spos[dv.y]);
                        ++moved;
                        // wl (this sweep's unbucketed worklist) is free once bucketed
                        if (trk) wl[atomicAdd(&s_nmv, 1)] = dv.y;
                    }
                }
            } else {
                const int t16 = threadIdx.x / TILE, l16 = threadIdx.x % TILE;
                int32_t* nlr = a.nlab + (int64_t)r * a.m2;
                for (int64_t di = t16; di < nk; di += NTH / TILE) {
                    const int4 dv = decr[di];
                    const int32_t d = dv.x, v = dv.y;
                    if (d < 0) continue;
                    const int4 vr = a.vrec[v];
                    if (l16 == 0) { apply_move<LOUV, TT>(a, r, dv, vr.w); ++moved; }
                    const int64_t rb = (int64_t)(uint32_t)vr.x, re = rb + vr.y;
                    for (int64_t j = rb + l16; j < re; j += TILE) {
                        if (push) nlr[a.rev[j]] = d;
                        if (trk) {
                            const int32_t u = a.col[j];
                            if (atomicMax(&mark[u], stamp) < stamp) wl2[atomicAdd(&s_nnext, 1)] = u;
                        }
                    }
                }
            }
            if (moved) atomicAdd(&s_acc[2], (unsigned long long)moved);
            __syncthreads();
        }
        if (trk && a.lm) {                       // block-uniform: k_mark_lm for this replica
            const int t16 = threadIdx.x / TILE, l16 = threadIdx.x % TILE;
            const int32_t* labr = a.lab + (int64_t)r * a.N;
            const int nmv = s_nmv;
            for (int i = t16; i < nmv; i += NTH / TILE) {
                const int4 vr = a.vrec[wl[i]];
                const int32_t d = labr[vr.w];
                const int64_t rb = (int64_t)(uint32_t)vr.x, re = rb + vr.y;
                for (int64_t j = rb + l16; j < re; j += TILE) {
                    if (labr[a.colp[j]] == d) continue;
                    const int32_t u = a.col[j];
                    if (atomicMax(&mark[u], stamp) < stamp) wl2[atomicAdd(&s_nnext, 1)] = u;
                }
            }
            __syncthreads();
        }
        // end of sweep: the same bookkeeping as k_sweep_end, for this replica
        if (threadIdx.x == 0) {
            const unsigned long long moves = s_acc[2];
            tail_acc[4 * r + 0] += s_acc[3]; tail_acc[4 * r + 1] += s_acc[4]; tail_acc[4 * r + 2] += s_acc[5];
            atomicAdd((unsigned long long*)(n_active_out + 4), 1ull);
            if (a.prune) {
                a.track[a.n_r + r] = a.track[r];
                if (a.lm || moves * (unsigned long long)a.track_div < (unsigned long long)a.N) a.track[r] = 1;
            }
            if (a.track[3 * a.n_r + r]) { a.track[3 * a.n_r + r] = 0; a.track[2 * a.n_r + r] = 1; }
            else if (a.push_div && !a.track[2 * a.n_r + r] && !a.track[a.n_r + r] &&
                     moves * (unsigned long long)a.push_div < (unsigned long long)a.N)
                a.track[3 * a.n_r + r] = 1;
            bool stop;
            if (LOUV) stop = moves == 0 || ((double)s_acc[0] / DQ_SCALE) < a.min_dq;
            else stop = s_acc[1] == 0;
            if (stop) { a.active[r] = 0; s_stop = 1; }
            s_n = s_nnext;
        }
        __syncthreads();
        if (s_stop) break;
        first = false;
        int32_t* t = wl; wl = wl2; wl2 = t;
    }
}

// Visit lists of one sweep, per replica: every vertex (sweeps before tracking starts, or
// pruning off; the list stays implicit: entry di of bucket k is position k*S + di), or
// those flagged affected by the previous sweep's moves -- bucketed by the vertex's position
// in this sweep's random order (inverse permutation).  A filtered sweep of V vertices runs
// its buckets in ROUNDS of g consecutive buckets, g the largest power of two <= B with
// V*g <= N (k_list_plan), so a round holds about as many decisions as a bucket of a full
// sweep -- not 32 latency-bound launches of a few hundred visits each.  The order inside a
// round is immaterial: its decisions all read the state the earlier rounds left, and its
// moves commute (distinct vertices, integer atomics), so entries land in any order.
// Pass 1 counts the flagged vertices per bucket, the plan sizes the rounds, pass 2 fills the
// per-replica lists [n_r][PN] and clears the flags.  Dynamic LDS: 2 * B ints.
__device__ __forceinline__ uint32_t vertex_bucket(const CDArgs& a, const Perm& P, uint32_t v) {
    const uint32_t pos = vertex_pos(a, P, v);
    return pos / (uint32_t)a.S;
}
// The flag scans take one 32-bit word (32 vertices) per thread and walk its set bits: in a
// late filtered sweep almost every word is zero (C5's LPA tie regime: ~0.8 % of the vertices
// flagged), and a thread per vertex paid a load, a test and a branch for each of them
// (k_list_count + k_list_fill were 86 ms of a C5 step).
// Hybrid: each filtered replica's affected flags (its list size this sweep, rep_dense).
__global__ __launch_bounds__(256) void k_aff_count(CDArgs a, int32_t* vcnt) {
    const int r = blockIdx.y;
    if (!a.active[r] || rep_full(a, r)) return;   // block-uniform
    const uint32_t* aff = a.aff + (int64_t)r * a.aw;
    const int64_t w = (int64_t)blockIdx.x * TB + threadIdx.x;
    int c = w < a.aw ? __popc(aff[w]) : 0;
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(vcnt + r, c);
}
__global__ __launch_bounds__(256) void k_list_count(CDArgs a, int sweep, int32_t* cntfine) {
    extern __shared__ int s_lb[];
    const int r = blockIdx.y, B = a.B;
    if (!a.active[r] || rep_full(a, r)) return;   // block-uniform
    for (int k = threadIdx.x; k < B; k += TB) s_lb[k] = 0;
    __syncthreads();
    const Perm P = sweep_perm(a, order_rg(a, r, rep_dense(a, r)), sweep);
    const uint32_t* aff = a.aff + (int64_t)r * a.aw;
    const int64_t w = (int64_t)blockIdx.x * TB + threadIdx.x;
    uint32_t bits = w < a.aw ? aff[w] : 0u;
    while (bits) {
        const int64_t v = w * 32 + (__ffs(bits) - 1);
        bits &= bits - 1;
        if (v < a.N) atomicAdd(&s_lb[vertex_bucket(a, P, (uint32_t)v)], 1);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < B; k += TB)
        if (s_lb[k]) atomicAdd(&cntfine[(int64_t)r * B + k], s_lb[k]);
}
// Rounds per replica: lcnt[k][r] (entries of round k), loff[r][k] (offsets into the
// replica's list), fill cursors, coarsening g; info[0] = max rounds, info[2..3] = visits,
// info[4] = the largest replica's visits.
// One block.  It also resets what the sweep's bookkeeping accumulates -- info (zeroed before
// the atomics below) and cntfine (each replica's row, once read: the next sweep's k_list_count
// finds it zero) -- and copies the active count left by the previous sweep into info[6], so a
// sweep costs one host read and no memset launches.
__global__ void k_list_plan(CDArgs a, int32_t* cntfine, int32_t* loff, int32_t* cursor, int32_t* gco,
                            int32_t* lcnt, int4* rrec, int32_t* info, const int32_t* n_active) {
    const int B = a.B;
    if (threadIdx.x == 0) {
        for (int i = 0; i < 8; ++i) info[i] = 0;
        info[6] = n_active[0];
    }
    __syncthreads();
    for (int r = threadIdx.x; r < a.n_r; r += blockDim.x) {
        int32_t* lo = loff + (int64_t)r * (B + 1);
        if (!a.active[r]) {
            for (int k = 0; k < B; ++k) {
                lcnt[(int64_t)k * a.n_r + r] = 0;
                rrec[(int64_t)k * a.n_r + r] = make_int4(0, 0, 0, 0);
            }
            gco[r] = 1;
            continue;
        }
        const int fl = (a.track[2 * a.n_r + r] ? RR_PUSH : 0) | (a.track[3 * a.n_r + r] ? RR_TRANS : 0);
        int32_t cmax = 0;                        // largest round: decide item slots per replica
        if (rep_full(a, r)) {
            int64_t tot = 0;
            for (int k = 0; k < B; ++k) {
                const int32_t c = (int32_t)max((int64_t)0, min(a.S, a.PN - (int64_t)k * a.S));
                lcnt[(int64_t)k * a.n_r + r] = c;
                rrec[(int64_t)k * a.n_r + r] = make_int4((int32_t)((int64_t)k * a.S), c, fl | RR_FULL, 0);
                cmax = max(cmax, c);
                tot += c;
            }
            atomicMax(info + 1, (cmax + LNT - 1) / LNT);
            gco[r] = 1;
            atomicMax(info, B);
            atomicAdd((unsigned long long*)(info + 2), (unsigned long long)tot);
            atomicMax(info + 4, (int)min(tot, (int64_t)INT_MAX));
            continue;
        }
        int32_t* cf = cntfine + (int64_t)r * B;
        int64_t V = 0;
        for (int k = 0; k < B; ++k) V += cf[k];
        const int g = (a.coarsen && !rep_dense(a, r)) ? coarse_factor(a.N, V, B, a.coarsen) : 1;
        const int rounds = (B + g - 1) / g;
        int32_t acc = 0;
        for (int k = 0; k < B; ++k) {
            int32_t c = 0;
            if (k < rounds)
                for (int f = k * g; f < min(B, (k + 1) * g); ++f) c += cf[f];
            lo[k] = acc;
            cursor[(int64_t)r * B + k] = acc;
            lcnt[(int64_t)k * a.n_r + r] = c;
            rrec[(int64_t)k * a.n_r + r] = make_int4(acc, c, fl, 0);
            cmax = max(cmax, c);
            acc += c;
        }
        lo[B] = acc;
        for (int k = 0; k < B; ++k) cf[k] = 0;   // consumed: zero for the next sweep
        gco[r] = g;
        atomicMax(info + 1, (cmax + LNT - 1) / LNT);
        atomicMax(info, rounds);
        atomicAdd((unsigned long long*)(info + 2), (unsigned long long)V);
        atomicMax(info + 4, (int)V);
    }
}
__global__ __launch_bounds__(256) void k_list_fill(CDArgs a, int sweep, const int32_t* gco, int32_t* cursor,
                                                   int32_t* list) {
    extern __shared__ int s_lb[];
    const int r = blockIdx.y, B = a.B;
    int* s_cnt = s_lb;
    int* s_base = s_lb + B;
    if (!a.active[r] || rep_full(a, r)) return;   // block-uniform
    for (int k = threadIdx.x; k < B; k += TB) s_cnt[k] = 0;
    __syncthreads();
    const int g = gco[r];
    const Perm P = sweep_perm(a, order_rg(a, r, rep_dense(a, r)), sweep);
    uint32_t* aff = a.aff + (int64_t)r * a.aw;
    const int64_t w = (int64_t)blockIdx.x * TB + threadIdx.x;   // one word: 32 vertices
    const uint32_t word = w < a.aw ? aff[w] : 0u;
    // pass 1: the block's count per round; pass 2 (after the block's bases are reserved) places
    // the entries -- entries within a round may land in any order (see above)
    for (uint32_t bits = word; bits; bits &= bits - 1) {
        const int64_t v = w * 32 + (__ffs(bits) - 1);
        if (v < a.N) atomicAdd(&s_cnt[(int)vertex_bucket(a, P, (uint32_t)v) / g], 1);
    }
    if (word) aff[w] = 0u;   // flags consumed (filter: vertices whose neighbour moved last sweep)
    __syncthreads();
    for (int k = threadIdx.x; k < B; k += TB) {
        s_base[k] = s_cnt[k] ? atomicAdd(&cursor[(int64_t)r * B + k], s_cnt[k]) : 0;
        s_cnt[k] = 0;
    }
    __syncthreads();
    int32_t* lr = list + (int64_t)r * a.PN;
    for (uint32_t bits = word; bits; bits &= bits - 1) {
        const int64_t v = w * 32 + (__ffs(bits) - 1);
        if (v >= a.N) continue;
        const int k = (int)vertex_bucket(a, P, (uint32_t)v) / g;
        lr[s_base[k] + atomicAdd(&s_cnt[k], 1)] = (int32_t)v;
    }
}
// One bucket: decide (light + heavy rows) against the state left by earlier buckets, apply.
// Every grid is fixed and every size is read on the device, so a sweep never waits on
// the host.
template <bool LOUV, typename TT>
static void sub_round(Ctx& c, const CDArgs& a, int k, int sweep, bool any_heavy, int X) {
    (void)any_heavy;   // heavy_cnt: zeroed at cd_run start, then by each round's k_apply
    const int ev = timer_begin(c);
    // one item per block: X item slots per replica, rounded up to whole XCD groups of 8
    const int64_t grid = (((int64_t)a.n_r * X + 7) / 8) * 8;
    k_decide_light<LOUV, TT><<<(unsigned)grid, DTB, 0, c.stream>>>(a, k, sweep, X);
    timer_end(c, 4, ev);
    if (any_heavy) k_decide_heavy<LOUV, TT><<<HEAVY_GRID, TB, 0, c.stream>>>(a, k, sweep);
    // apply: FC_APPLY_BLOCKS blocks per replica, more when few replicas share the GPU (a
    // push/tracking move is a dependent row walk, so the chip needs ~2K resident blocks), but
    // no more than the round's decisions fill (16-lane tiles)
    const int64_t ab = std::min<int64_t>(std::max<int64_t>(c.apply_blocks, (2048 + a.n_r - 1) / a.n_r),
                                         std::max<int64_t>(1, ((int64_t)X * LNT + TILES - 1) / TILES));
    k_apply<LOUV, TT><<<dim3((unsigned)ab, a.n_r), ATB, 0, c.stream>>>(a, k);
}

__global__ void k_count_heavy(int64_t n, const int64_t* rowptr, int64_t thr, unsigned long long* out) {
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool h = v < n && rowptr[v + 1] - rowptr[v] > thr;
    const unsigned long long b = __ballot(h);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(out, (unsigned long long)__popcll(b));
}
// Vertices whose row exceeds thr entries (heavy rows of the working graph).
static int64_t count_heavy(Ctx& c, int64_t thr) {
    unsigned long long* d = (unsigned long long*)ensure<int64_t>(c.counters, 4);
    FC_HIP(hipMemsetAsync(d, 0, 8, c.stream));
    k_count_heavy<<<nblk(c.N), TB, 0, c.stream>>>(c.N, c.g.rowptr.as<int64_t>(), thr, d);
    FC_HIP(hipMemcpyAsync(c.hpin, d, 8, hipMemcpyDeviceToHost, c.stream));
    sync(c);
    return c.hpin[0];
}

void cd_run(Ctx& c, int algo, int rbegin, int rcount, int n_p_total, int iteration, int shared_full,
            const CDHandoff* h) {
    FC_REQUIRE(rcount >= 1 && rbegin >= 0 && rbegin + rcount <= n_p_total, FC_EINVAL, "bad replica range");
    FC_REQUIRE(c.N > 0 && c.g.rowptr.p, FC_ESTATE, "no graph loaded");
    const int sl0 = timer_begin(c);
    const bool louv = is_louvain(algo);
    const int64_t N = c.N;
    Graph& g = c.g;
    c.n_r = rcount; c.rbase = rbegin; c.n_p_total = n_p_total;
    c.labT_valid = false;
    // sweep positions: vertices in a random order, or whole chunks of CHUNK consecutive
    // vertices in a random chunk order (coalesced per-vertex accesses)
    const int CH = c.chunk;
    const int64_t NC = CH ? (N + 2 * CH - 2) / CH : N;   // room for the chunk-grid shift (sweep_perm)
    const int B = (int)std::min<int64_t>(cd_buckets(c, algo), NC);
    const int64_t S = CH ? ((NC + B - 1) / B) * CH : (N + B - 1) / B;
    int32_t* lab = ensure<int32_t>(c.lab, (size_t)rcount * N);
    // tot in int32 whenever every community total fits (all <= 2M < 2^31): half the gathers
    const bool tot32 = g.M2 <= 0x7fffffffll && !c.order_pass;
    void* tot = louv ? (void*)ensure<int64_t>(c.tot, (size_t)rcount * N) : nullptr;
    const int64_t PN = CH ? NC * CH : N;
    int4* dec = ensure<int4>(c.dec, (size_t)rcount * PN);   // a coarse round may hold up to PN decisions
    const int64_t m2 = 2 * g.m;
    int32_t* nlab = ensure<int32_t>(c.nlab, (size_t)rcount * (m2 > 0 ? m2 : 1));
    // per-replica state: active i32 [n_r] | red u64 [n_r][NSH][RF] | sacc u64 [n_r][4] | n_active
    char* rs = (char*)ensure<char>(c.rep_state, (size_t)rcount * (4 + 8 * NSH * RF + 64) + 256);
    int32_t* active = (int32_t*)rs;
    unsigned long long* red = (unsigned long long*)(rs + (((size_t)rcount * 4 + 255) & ~size_t(255)));
    unsigned long long* sacc = red + (size_t)rcount * NSH * RF;
    int32_t* n_active = (int32_t*)(sacc + 4 * (size_t)rcount);   // see k_sweep_end
    unsigned long long* tail_acc = (unsigned long long*)(n_active + 8);   // [n_r][4] k_cd_tail visits
    const size_t zero_bytes = (char*)(tail_acc + 4 * (size_t)rcount) - (char*)red;
    // heavy rows (degree > LIGHT_MAX_DEG): at most one entry per heavy vertex and replica per round
    int64_t n_heavy = 0;
    if (g.max_deg > LIGHT_MAX_DEG) n_heavy = count_heavy(c, LIGHT_MAX_DEG);
    int32_t* heavy = ensure<int32_t>(c.heavy_list, 3 * (size_t)rcount * (size_t)std::max<int64_t>(n_heavy, 1) + 3);
    const int64_t aw = (N + 31) / 32;
    uint32_t* aff = ensure<uint32_t>(c.aff, (size_t)rcount * aw);
    int32_t* track = ensure<int32_t>(c.track, 4 * (size_t)rcount);
    if (!h) {
        FC_HIP(hipMemsetAsync(aff, 0, 4 * (size_t)rcount * aw, c.stream));
        FC_HIP(hipMemsetAsync(track, 0, 16 * (size_t)rcount, c.stream));   // pull mode, no tracking
    }
    int32_t* list = ensure<int32_t>(c.vlist, (size_t)rcount * PN);
    // rrec int4 [B][n_r] | lcnt [B][n_r] | cntfine [n_r][B] | loff [n_r][B+1] | cursor [n_r][B] | gco [n_r] | info [8]
    const size_t plan_ints = 4 * (size_t)B * rcount + (size_t)B * rcount + (size_t)rcount * B +
                             (size_t)rcount * (B + 1) + (size_t)rcount * B + rcount + 1 + 8;
    int4* rrec = (int4*)ensure<int32_t>(c.vcnt, plan_ints);
    int32_t* lcnt = (int32_t*)(rrec + (size_t)B * rcount);
    int32_t* cntfine = lcnt + (size_t)B * rcount;
    int32_t* loff = cntfine + (size_t)rcount * B;
    int32_t* cursor = loff + (size_t)rcount * (B + 1);
    int32_t* gco = cursor + (size_t)rcount * B;
    // [0] max rounds, [1] decide item slots per replica (its largest round), [2..3] u64 visits
    // (8-byte aligned: 64-bit atomics), [4] the largest replica's visits
    int32_t* info = gco + rcount;
    if ((uintptr_t)info & 7) ++info;
    int32_t* heavy_cnt = ensure<int32_t>(c.heavy_cnt, 4);
    FC_HIP(hipMemsetAsync(heavy_cnt, 0, sizeof(int32_t), c.stream));
    int64_t heavy_slots = 1;
    while (heavy_slots < 2 * (int64_t)g.max_deg) heavy_slots <<= 1;
    int32_t* hscr = nullptr;
    if (heavy_slots > HEAVY_LDS_SLOTS)   // one slice per heavy-kernel block, or per tail-kernel block (replica)
        hscr = ensure<int32_t>(c.heavy_scratch, (size_t)std::max(HEAVY_GRID, rcount) * 2 * heavy_slots);

    if (!h) {
        std::vector<int32_t> ones(rcount, (g.M2 > 0) ? 1 : 0);
        FC_HIP(hipMemcpyAsync(active, ones.data(), sizeof(int32_t) * rcount, hipMemcpyHostToDevice, c.stream));
        sync(c);  // `ones` is pageable host memory
    }
    FC_HIP(hipMemsetAsync(red, 0, zero_bytes, c.stream));
    dim3 ig(nblk(N), rcount);
    const int32_t* spos = c.spos.as<int32_t>();
    const int32_t* sinv = c.sinv.as<int32_t>();
    if (h) {   // a hybrid batch from its first filtered sweep: the replica-lane engine's state
        FC_REQUIRE(tot32 || !louv, FC_ESTATE, "hybrid hand-off needs int32 totals");
        h->fill(c, h->user, lab, (int32_t*)tot, aff, track, active, nlab);
    } else if (tot32) {
        k_cd_init<int32_t><<<ig, TB, 0, c.stream>>>(N, rcount, g.kdeg.as<int64_t>(), sinv, lab, (int32_t*)tot, louv ? 1 : 0);
    } else {
        k_cd_init<int64_t><<<ig, TB, 0, c.stream>>>(N, rcount, g.kdeg.as<int64_t>(), sinv, lab, (int64_t*)tot, louv ? 1 : 0);
    }
    FC_REQUIRE(!louv || (double)g.max_kdeg * (double)g.M2 < 4.0e18, FC_ELIMIT,
               "edge weights too large for exact int64 modularity gains");

    CDArgs a;
    a.N = N; a.S = S; a.PN = PN; a.B = B; a.dstride = PN; a.coarsen = louv ? c.coarsen : 0; a.chunk = CH; a.perm_n = (uint32_t)NC; a.n_r = rcount; a.rbase = rbegin; a.iter = (uint32_t)iteration; a.seed = c.seed;
    a.rowptr = g.rowptr.as<int64_t>(); a.col = g.col.as<int32_t>(); a.cw = g.cw.as<int32_t>();
    a.colp = g.colp.as<int32_t>(); a.spos = spos; a.vrec = g.vrec.as<int4>();
    a.kdeg = g.kdeg.as<int64_t>(); a.M2 = g.M2;
    a.lab = lab; a.tot = tot; a.dec = dec; a.active = active;
    a.nlab = nlab; a.rev = g.crev.as<int32_t>(); a.m2 = m2;
    a.red = red; a.sacc = sacc;
    a.min_dq = c.cd_min_dq;
    a.shared_full = shared_full;
    // hybrid: per-replica list sizes of the filtered sweeps (dense lists keep the shared order)
    int32_t* vcnt = (shared_full && c.prune && c.dense_div) ? ensure<int32_t>(c.aff_cnt, (size_t)rcount) : nullptr;
    a.vcnt = vcnt;
    a.dense_div = c.dense_div;
    a.heavy = heavy; a.heavy_cnt = heavy_cnt; a.heavy_scratch = hscr; a.heavy_slots = heavy_slots;
    a.aff = aff; a.aw = aw; a.list = list; a.loff = loff; a.lcnt = lcnt; a.rrec = rrec; a.track = track; a.prune = c.prune;
    a.hcap = std::max<int64_t>(n_heavy, 1);
    a.track_div = c.track_div;
    // push mode only on unit-weight graphs: on consensus graphs the pull sweeps measured
    // faster (LFR-1M weighted CD batch 46.1 vs 47.1 ms; input graph 125.7 vs 129.6 with push);
    // the mode never changes a decision
    a.push_div = (louv && g.max_w > 1) ? 0 : c.push_div;
    // Leiden-style marking on consensus graphs (weights > 1; LPA ignores them but runs on the
    // same strongly clustered graph): after the first sweep few vertices move, and nearly all
    // the later movers have a neighbour that ended in another community (LFR-100k consensus
    // graph: 1.5 % of the vertices marked after sweep 1, covering 99.6-100 % of sweep 2's
    // movers, against 85 % marked by "every neighbour of a mover").  Sweep 2 is already
    // filtered, so no unfiltered sweep is left for the pull -> push transition: lm is pull-only.
    a.lm = ((g.max_w > 1 || c.prune_mark == 2) && c.prune && c.prune_mark >= 1) ? 1 : 0;
    if (a.lm) a.push_div = 0;
    a.mvf = nullptr;
    if (a.lm) {
        a.mvf = ensure<uint8_t>(c.mvf, (size_t)rcount * N);
        FC_HIP(hipMemsetAsync(a.mvf, 0, (size_t)rcount * N, c.stream));
    }
    a.unitw = (!louv || (g.max_w == 1 && g.M2 == 2 * g.m)) ? 1 : 0;
    a.wbits = 1;
    if (louv) while (a.wbits < 31 && (g.max_w >> a.wbits) != 0) ++a.wbits;
    // own-label register sums (one ballot per load) for the entries of the graph's typical
    // weight w0; the rest of a weighted row keeps the table (a full wave scan of weighted own
    // sums measured slower: LFR-1M consensus graph decide 32.7 vs 29.0 ms per batch)
    a.own_bal = c.own_ballot ? 1 : 0;
    a.w0 = a.wbits == 1 ? 1 : std::max(1, n_p_total);

    // One host round trip per sweep, after the visit lists are planned: it returns the number
    // of rounds (coarse buckets) and the largest per-replica round (decide item slots), so
    // every launch is sized exactly, plus the active count left by the previous sweep.
    const bool hv = g.max_deg > LIGHT_MAX_DEG;
    const unsigned lb_grid = (unsigned)((aw + TB - 1) / TB);   // flag scans: one 32-vertex word per thread
    int32_t* hinfo = (int32_t*)(c.hpin + 8);   // info[0..4] | n_active[0] at [6]
    const int sweep0 = h ? h->sweep0 : 0;
    int sweep = sweep0;
    if (c.trace && !h) { sync(c); trace_dt_us(true); }   // a hand-off's first sweep includes the conversion
    FC_HIP(hipMemsetAsync(cntfine, 0, sizeof(int32_t) * (size_t)rcount * B, c.stream));   // then kept zero by k_list_plan
    for (; sweep < c.max_sweeps && g.M2 > 0; ++sweep) {
        if (vcnt && sweep > 0) {
            FC_HIP(hipMemsetAsync(vcnt, 0, sizeof(int32_t) * (size_t)rcount, c.stream));
            k_aff_count<<<dim3(lb_grid, rcount), TB, 0, c.stream>>>(a, vcnt);
        }
        k_list_count<<<dim3(lb_grid, rcount), TB, sizeof(int) * B, c.stream>>>(a, sweep, cntfine);
        k_list_plan<<<1, TB, 0, c.stream>>>(a, cntfine, loff, cursor, gco, lcnt, rrec, info, n_active);
        FC_HIP(hipMemcpyAsync(hinfo, info, 28, hipMemcpyDeviceToHost, c.stream));
        sync(c);
        const int rounds = hinfo[0];
        const unsigned long long visits = *(unsigned long long*)(hinfo + 2);
        if (rounds == 0 || (sweep > sweep0 && hinfo[6] == 0)) break;   // every replica has stopped
        // small sweeps (every replica visits <= tail_visits vertices): hand every remaining
        // sweep to the per-replica tail kernel (it takes the flags as its first worklist)
        const int64_t tail_thr = c.tail_visits >= 0 ? c.tail_visits : (louv ? 1024 : 4096);
        if (tail_thr > 0 && (int64_t)hinfo[4] <= tail_thr && B <= TAIL_MAXB) {
            int32_t* tbuf = ensure<int32_t>(c.tailbuf, (size_t)rcount * 3 * N);
            int32_t* tmark = ensure<int32_t>(c.tailmark, (size_t)rcount * N);
            FC_HIP(hipMemsetAsync(tmark, 0, 4 * (size_t)rcount * N, c.stream));
            if (c.trace) fprintf(stderr, "[fc] cd it=%d tail kernel from sweep %d\n", iteration, sweep);
            k_list_fill<<<dim3(lb_grid, rcount), TB, 2 * sizeof(int) * B, c.stream>>>(a, sweep, gco, cursor, list);
            if (!louv)
                k_cd_tail<false, int32_t, TAIL_TB><<<rcount, TAIL_TB, 0, c.stream>>>(a, sweep, c.max_sweeps, tbuf, tmark, tail_acc, n_active);
            else if (tot32)
                k_cd_tail<true, int32_t, TAIL_TB><<<rcount, TAIL_TB, 0, c.stream>>>(a, sweep, c.max_sweeps, tbuf, tmark, tail_acc, n_active);
            else
                k_cd_tail<true, int64_t, TAIL_TB><<<rcount, TAIL_TB, 0, c.stream>>>(a, sweep, c.max_sweeps, tbuf, tmark, tail_acc, n_active);
            if (c.trace) {
                sync(c);
                fprintf(stderr, "[fc] cd it=%d tail kernel dt_us=%.0f\n", iteration, trace_dt_us());
            }
            break;
        }
        k_list_fill<<<dim3(lb_grid, rcount), TB, 2 * sizeof(int) * B, c.stream>>>(a, sweep, gco, cursor, list);
        const int X = std::max(hinfo[1], 1);
        for (int k = 0; k < rounds; ++k) {
            if (!louv) sub_round<false, int32_t>(c, a, k, sweep, hv, X);
            else if (tot32) sub_round<true, int32_t>(c, a, k, sweep, hv, X);
            else sub_round<true, int64_t>(c, a, k, sweep, hv, X);
        }
        if (a.lm) k_mark_lm<<<ig, TB, 0, c.stream>>>(a);
        if (louv) k_sweep_end<true><<<1, TB, 0, c.stream>>>(a, n_active);
        else k_sweep_end<false><<<1, TB, 0, c.stream>>>(a, n_active);
        if (c.trace) {
            sync(c);
            int32_t st4[4];   // n_active[0] active, [2..3] moves of this sweep (all replicas)
            FC_HIP(hipMemcpy(st4, n_active, sizeof(st4), hipMemcpyDeviceToHost));
            fprintf(stderr, "[fc] cd it=%d sweep=%d rounds=%d visits=%llu moves=%llu active=%d dt_us=%.0f\n", iteration,
                    sweep, rounds, visits, *(unsigned long long*)(st4 + 2), st4[0], trace_dt_us());
        }
    }
    // replica-sweeps and light-kernel traffic counters for the roofline model
    std::vector<unsigned long long> sa(8 * (size_t)rcount + 4);   // sacc | n_active | tail_acc
    FC_HIP(hipMemcpyAsync(sa.data(), sacc, sa.size() * 8, hipMemcpyDeviceToHost, c.stream));
    sync(c);
    const unsigned long long rep_sweeps = sa[4 * (size_t)rcount + 2];   // n_active[4..5]
    if (c.trace)
        fprintf(stderr, "[fc] cd it=%d done: %d multi-kernel sweeps, %.2f sweeps per replica\n", iteration, sweep,
                (double)rep_sweeps / rcount);
    if (!c.order_pass) {
        c.acc.cd_sweeps += (int64_t)rep_sweeps;
        c.prof.cd_sweeps += (int64_t)rep_sweeps;
    }
    c.hpin[0] = c.hpin[1] = c.hpin[2] = 0;
    int64_t tv = 0, te = 0;
    for (int r = 0; r < rcount; ++r) {
        c.hpin[0] += sa[4 * r]; c.hpin[1] += sa[4 * r + 1]; c.hpin[2] += sa[4 * r + 2];
        tv += sa[4 * (size_t)rcount + 4 + 4 * r]; te += sa[4 * (size_t)rcount + 4 + 4 * r + 1];
    }
    // algorithmic bytes of the light decide kernel: per vertex rowptr 16 + kdeg 8 + own
    // label 4 + own tot (4|8) + decision 8 + list entry 4; per adjacency entry neighbour
    // label 4 + weight 4; per Sigma gathered (candidates of maximal val) its tot (4|8)
    // (louvain).  LPA: no kdeg/tot/weights.
    const int64_t tsz = tot32 ? 4 : 8;
    const int64_t db = louv ? c.hpin[0] * (40 + tsz) + c.hpin[1] * 8 + c.hpin[2] * tsz
                            : c.hpin[0] * 32 + c.hpin[1] * 4;
    for (fc_stats* s : {&c.acc, &c.prof}) {
        if (c.order_pass) break;                 // load-time ordering run (store_order)
        s->cd_vertex_visits += c.hpin[0] + tv;   // light kernel + tail kernel
        s->cd_edge_visits += c.hpin[1] + te;
        s->decide_bytes += db;                   // light kernel only (its time is decide_ms)
    }
    timer_end(c, 0, sl0);
#ifdef FC_PHASE_PROF
    {
        unsigned long long hp[16];
        FC_HIP(hipMemcpyFromSymbol(hp, HIP_SYMBOL(g_phase), sizeof(hp)));
        fprintf(stderr, "[fc] phase cycles (cumulative, sampled):");
        for (int i = 0; i < 9; ++i) fprintf(stderr, " %llu", hp[i]);
        fprintf(stderr, "\n");
    }
#endif
}

// ------------------------------------------------------------------ transpose / renumber
// lab [n_r][N] (slot order) -> labT [N][ldT] (vertex rows): 64 slots x 64 replicas per tile
// through LDS; rows read coalesced, each vertex's 64 labels written as one 256-byte run
__global__ __launch_bounds__(256) void k_transpose(int64_t N, int n_r, int ldT, const int32_t* lab, const int32_t* sinv,
                                                  int32_t* labT) {
    __shared__ int32_t t[64][65];
    __shared__ int32_t sv[64];
    const int64_t s0 = (int64_t)blockIdx.x * 64;
    const int r0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
    if (ty == 0) sv[tx] = s0 + tx < N ? sinv[s0 + tx] : -1;
    for (int rr = ty; rr < 64; rr += 4) {
        const int r = r0 + rr;
        const int64_t s = s0 + tx;
        if (r < n_r && s < N) t[rr][tx] = lab[(int64_t)r * N + s];
    }
    __syncthreads();
    for (int ss = ty; ss < 64; ss += 4) {
        const int32_t v = sv[ss];
        const int r = r0 + tx;
        if (v >= 0 && r < n_r) labT[(int64_t)v * ldT + r] = t[tx][ss];
    }
}
void labels_transpose(Ctx& c) {
    FC_REQUIRE(c.n_r > 0, FC_ESTATE, "no labelings");
    c.ldT = (c.n_r + 3) & ~3;
    int32_t* labT = ensure<int32_t>(c.labT, (size_t)c.N * c.ldT);
    dim3 grid(nblk(c.N, 64), (c.n_r + 63) / 64);
    k_transpose<<<grid, TB, 0, c.stream>>>(c.N, c.n_r, c.ldT, c.lab.as<int32_t>(), c.sinv.as<int32_t>(), labT);
    c.labT_valid = true;
}

__global__ void k_first_init(int64_t total, int32_t* first) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < total) first[i] = 0x7fffffff;
}
// first[r][c] = earliest NODE position of community c.  A block takes FM_SPAN consecutive
// slots of one row -- slot order is community order at load, so they hold few distinct
// labels -- folds them into an LDS table (label -> min position), and issues one global
// atomic per distinct label.  Labels overflowing the table (more distinct labels than
// FM_SLOTS / 2 in a span) go straight to global memory.
static constexpr int FM_SPAN = 2048, FM_SLOTS = 1024;
__global__ __launch_bounds__(256) void k_first_min(int64_t N, const int32_t* lab, const int32_t* snpos, int32_t* first) {
    __shared__ int32_t key[FM_SLOTS], val[FM_SLOTS];
    const int r = blockIdx.y;
    const int64_t s0 = (int64_t)blockIdx.x * FM_SPAN;
    const int32_t* labr = lab + (int64_t)r * N;
    int32_t* fr = first + (int64_t)r * N;
    for (int k = threadIdx.x; k < FM_SLOTS; k += 256) { key[k] = -1; val[k] = 0x7fffffff; }
    __syncthreads();
    for (int k = threadIdx.x; k < FM_SPAN; k += 256) {
        const int64_t s = s0 + k;
        if (s >= N) break;
        const int32_t c = labr[s], t = snpos[s];
        uint32_t h = hash32((uint32_t)c) & (FM_SLOTS - 1);
        bool done = false;
        for (int probe = 0; probe < 16 && !done; ++probe) {   // bounded probing, then global
            const int32_t prev = atomicCAS(&key[h], -1, c);
            if (prev == -1 || prev == c) { atomicMin(&val[h], t); done = true; }
            else h = (h + 1) & (FM_SLOTS - 1);
        }
        if (!done) atomicMin(&fr[c], t);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < FM_SLOTS; k += 256)
        if (key[k] >= 0) atomicMin(&fr[key[k]], val[k]);
}
// over node order t: out[r][t] = raw label of node t; flag = t opens its community
__global__ void k_node_order(int64_t N, int64_t total, const int32_t* lab, const int32_t* tpos,
                             const int32_t* first, int32_t* out, int32_t* flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > total) return;
    if (i == total) { if (flag) flag[i] = 0; return; }
    const int64_t r = i / N, t = i % N;
    const int32_t c = lab[r * N + tpos[t]];
    out[i] = c;
    if (flag) flag[i] = first[r * N + c] == (int32_t)t ? 1 : 0;
}
// flag[r][t] = 1 where node position t opens a community of row r: one scattered store per
// community (first[r][c] != INT_MAX), the rest of the row left at the memset's 0
__global__ void k_open_flags(int64_t N, const int32_t* first, int32_t* flag) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= N) return;
    const int64_t base = (int64_t)blockIdx.y * N;
    const int32_t f = first[base + c];
    if (f != 0x7fffffff) flag[base + f] = 1;
}
// renumbered labels written in SLOT order (the label row and the first-node table read
// coalesced: slots are stored in community order), scattered to their node positions:
// out[r][t] = rank of the community's first node among the row's opening nodes
__global__ void k_relabel_slots(int64_t N, const int32_t* lab, const int32_t* snpos, const int32_t* first,
                                const int32_t* rank, int32_t* out) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= N) return;
    const int64_t base = (int64_t)blockIdx.y * N;
    const int32_t c = lab[base + s];
    out[base + snpos[s]] = rank[base + first[base + c]] - rank[base];
}
// Local labelings -> host in NODE order; renumber: community ids 0..k-1 by first node.
// Renumbered: first-node table (k_first_min), opening flags from it, their scan, then one
// slot-order pass (k_relabel_slots) -- two random reads per label fewer than a node-order
// gather followed by a relabel pass (LFR-1M run 103.4 -> 102.6 ms, SBM-4M 744.7 -> 742.8 ms).
void labels_to_host(Ctx& c, int32_t* host, bool renumber) {
    const int64_t N = c.N, total = (int64_t)c.n_r * N;
    FC_REQUIRE(total < (int64_t(1) << 31), FC_ELIMIT, "n_p * n too large for one labelling export");
    int32_t* out = ensure<int32_t>(c.st_lab, total + 1);
    if (renumber) {
        int32_t* first = ensure<int32_t>(c.dec, total + 1);   // CD scratch is free now
        int32_t* flag = ensure<int32_t>(c.wnew, total + 1);
        int32_t* rank = ensure<int32_t>(c.hit, total + 1);
        const dim3 rows((unsigned)nblk(N), (unsigned)c.n_r);
        k_first_init<<<nblk(total), TB, 0, c.stream>>>(total, first);
        k_first_min<<<dim3((unsigned)((N + FM_SPAN - 1) / FM_SPAN), c.n_r), 256, 0, c.stream>>>(
            N, c.lab.as<int32_t>(), c.snpos.as<int32_t>(), first);
        FC_HIP(hipMemsetAsync(flag, 0, sizeof(int32_t) * (size_t)(total + 1), c.stream));
        k_open_flags<<<rows, TB, 0, c.stream>>>(N, first, flag);
        exclusive_scan(c, flag, rank, total + 1);
        k_relabel_slots<<<rows, TB, 0, c.stream>>>(N, c.lab.as<int32_t>(), c.snpos.as<int32_t>(), first, rank, out);
    } else {
        k_node_order<<<nblk(total + 1), TB, 0, c.stream>>>(N, total, c.lab.as<int32_t>(), c.tpos.as<int32_t>(), nullptr,
                                                           out, nullptr);
    }
    // hipMemcpyDefault: `host` may be host memory or a device buffer (distributed gather)
    FC_HIP(hipMemcpyAsync(host, out, 4 * (size_t)total, hipMemcpyDefault, c.stream));
    sync(c);
}
__global__ void k_from_node_order(int64_t N, int64_t total, const int32_t* in, const int32_t* tpos, int32_t* lab) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int64_t r = i / N, t = i % N;
    lab[r * N + tpos[t]] = in[i];   // label values only matter through equality
}
// Host labelings in node order -> local replicas (replay).
void labels_from_host(Ctx& c, int count, const int32_t* host) {
    const int64_t N = c.N, total = (int64_t)count * N;
    int32_t* in = ensure<int32_t>(c.st_lab, total + 1);
    FC_HIP(hipMemcpyAsync(in, host, 4 * (size_t)total, hipMemcpyHostToDevice, c.stream));
    int32_t* lab = ensure<int32_t>(c.lab, (size_t)total);
    k_from_node_order<<<nblk(total), TB, 0, c.stream>>>(N, total, in, c.tpos.as<int32_t>(), lab);
    sync(c);
}

// ------------------------------------------------------------------ label storage order
// Ctx::spos: every replica's label row is stored in COMMUNITY order, so the neighbour-label
// gathers of a sweep (lab[colp[j]]) land on few lines.  The order comes from one Louvain
// replica run on the input graph at load (the same engine, any seed: only locality
// matters); vertices sorted by (community, id).  Storage only -- label VALUES, visit order
// and every decision are unchanged, so results are identical with or without it.
__global__ void k_store_keys(int64_t N, const int32_t* lab, uint32_t* key, int32_t* idx) {
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= N) return;
    key[v] = (uint32_t)lab[v];   // spos is the identity while this runs
    idx[v] = (int32_t)v;
}
__global__ void k_store_slots(int64_t N, const int32_t* order, int32_t* spos) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) spos[order[i]] = (int32_t)i;
}
void store_order(Ctx& c) {
    const int64_t N = c.N;
    // int64 totals: the pass runs the k_decide_light<true, long> instance, so kernel
    // statistics of the int32 instance cover the consensus runs alone
    // and it is load-time work: neither its kernels nor its counters enter the run statistics
    struct Pass {
        Ctx& c;
        bool timer_on;
        explicit Pass(Ctx& x) : c(x), timer_on(x.timer.on) { c.order_pass = true; c.timer.on = false; }
        ~Pass() { c.order_pass = false; c.timer.on = timer_on; }
    } pass(c);
    // The first sweeps place almost every vertex (LFR-1M: 89 % and 52 % of the vertices move
    // in sweeps 0 and 1, < 6 % from sweep 3 on), so a few sweeps give the storage order; the
    // remaining one-replica sweeps would only pay latency (FC_ORDER_SWEEPS, default 3; profiles/r06_ab.txt).
    const int ms = c.max_sweeps, mb = c.buckets;
    c.max_sweeps = std::max(1, std::min(ms, c.order_sweeps));
    c.buckets = std::max(1, c.order_buckets);
    try {
        cd_run(c, FC_ALGO_LOUVAIN, 0, 1, 1, 0x3fffffff);
    } catch (...) {
        c.max_sweeps = ms;
        c.buckets = mb;
        throw;
    }
    c.max_sweeps = ms;
    c.buckets = mb;
    uint32_t* k1 = (uint32_t*)ensure<uint64_t>(c.mkey, N);
    uint32_t* k2 = (uint32_t*)ensure<uint64_t>(c.mkey2, N);
    int32_t* i1 = (int32_t*)ensure<int64_t>(c.midx, N);
    int32_t* i2 = (int32_t*)ensure<int64_t>(c.midx2, N);
    k_store_keys<<<nblk(N), TB, 0, c.stream>>>(N, c.lab.as<int32_t>(), k1, i1);
    sort_pairs_public(c, (const uint32_t*)k1, k2, (const int32_t*)i1, i2, N, c.key_bits);
    k_store_slots<<<nblk(N), TB, 0, c.stream>>>(N, i2, c.spos.as<int32_t>());
    c.n_r = 0;
    sync(c);
}
__global__ void k_slot_maps(int64_t N, const int32_t* spos, const int32_t* npos, int32_t* sinv, int32_t* tpos,
                            int32_t* snpos) {
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= N) return;
    const int32_t s = spos[v], t = npos[v];
    sinv[s] = (int32_t)v;
    snpos[s] = t;
    tpos[t] = s;        // sigma[t] == v
}
void slot_maps(Ctx& c) {
    const int64_t N = c.N;
    int32_t* sinv = ensure<int32_t>(c.sinv, N);
    int32_t* tpos = ensure<int32_t>(c.tpos, N);
    int32_t* snpos = ensure<int32_t>(c.snpos, N);
    k_slot_maps<<<nblk(N), TB, 0, c.stream>>>(N, c.spos.as<int32_t>(), c.npos.as<int32_t>(), sinv, tpos, snpos);
}

}  // namespace fc
