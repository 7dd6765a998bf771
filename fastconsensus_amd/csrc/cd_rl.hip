// cd_rl.hip -- replica-lane community detection: the default engine for the louvain and lpm
// CD batches (python-louvain level 0, fast_consensus.py:148 / :384; igraph LPA, :270 / :392).
//
// The classic engine (cd.hip) gives every replica its own random visit order, so a bucket of
// one replica and a bucket of another hold different vertices: every neighbour-label gather
// is a random 4-byte read of that replica's label row, one 128-byte line each.  Here every
// replica of a CD batch visits the vertices in the SAME per-(iteration, sweep) random order
// (replicas still differ: ties are broken by per-replica hashes, and each replica keeps its
// own pruning state and stop).  A bucket is then one vertex set for all replicas, and labels
// are stored node-major, labT[v][ldT] (one replica per lane): deciding vertex v for up to 64
// replicas costs ONE row walk and, per neighbour u, ONE coalesced 256-byte read of u's labels
// for all of them -- 2 lines per neighbour for 64 visits instead of 64 lines.  Community
// totals are node-major too (totT[c][ldT]); with shared orders the replicas mostly agree on
// community names, so Sigma reads coalesce as well.
//
// Statistical effect of the shared order (CPU engine model, tests/test_engine_semantics.py):
// LFR-1k louvain consensus NMI 0.917 +- 0.03 (per-replica orders 0.906; reference loop 0.905),
// lpm recovery 24/30 (20/30; reference 14/30), LFR-100k louvain 0.971 (0.968; reference-
// semantics loop 0.968).  Every decision is exactly the classic rule; the CPU twin
// (oracle/fc_oracle.c tw_replica, shared = 1, coarsen = 0) reproduces the engine bit for bit.
//
// Lanes: a wave holds VPW = 64 / LG vertices ("sub-groups") x LG replica lanes, LG the
// smallest power of two >= the local replica count (at least 8, at most 64); more than 64
// local replicas form banks of 64 (one unit = one vertex of one bank).  Per unit, light rows
// (degree <= DM): the row's labels are staged in LDS as L[j][lane] (conflict-free columns),
// equal labels are merged per lane by a triangular scan (duplicates marked), the candidates of
// maximal weight compacted in place, and only their Sigma gathered (score = w*2M - k_v*Sigma
// <= w*2M: a lighter candidate can only win if k_v*Sigma >= 2M, handled exactly by a rare
// per-lane fallback).  Longer rows: one workgroup per unit (k_rl_exact).
#include <hipcub/hipcub.hpp>

#include <chrono>

#include "fc_ctx.h"
#include "fc_device.h"

namespace fc {

template <class T> void exclusive_scan(Ctx& c, const T* in, T* out, int64_t n);

namespace {

constexpr int RTB = 64;                 // decide / apply / mark blocks: one wave
constexpr int DM = 64;                  // light rows: degree <= DM
constexpr int VPWMAX = 8;               // sub-groups per wave (lane groups of >= 8 replicas)
constexpr int RL_CHUNK = 16;            // = cd.hip CHUNK (chunked visit orders)
// slow-visit and visit-mode list entries pack the local replica in 14 bits ((e << 14) | rr)
constexpr int RL_MAX_REPLICAS = 16384;
// Narrower sorting networks for short rows inside one decide launch (A/B switch bits): one unit
// per wave -- 4: 16 keys and 1: 24 keys in the 32-key kernel, 2: 48 keys in the 64-key one; per-lane
// rows (by the wave's longest) -- 8: 16 keys in the 32-key kernel, 16: 48 keys in the 64-key one
#ifndef FC_RL_SPLIT
#define FC_RL_SPLIT 30
#endif
#ifndef FC_LPA_TIES
#define FC_LPA_TIES 1                   // LPA tie revisits under pruning (oracle tw_replica); 0: bisect builds only
#endif

constexpr int32_t DONE = -1;            // merged / own / empty table entry (labels are >= 0)
constexpr int NSH = 16;                 // counter shards per replica
constexpr int RF = 8;                   // fields: 0 dq, 1 unstable, 2 moves, 3 visits, 4 entries, 5 cands, 6 units
constexpr double DQ_SCALE = 1099511627776.0;   // 2^40 fixed point for predicted dQ (as cd.hip)
constexpr int HWSLOTS = 1024;           // heavy rows: LDS table slots per wave (rows <= 512 entries)
constexpr int HTB = 256;
constexpr int HEAVY_GRID = 2048;       // k_rl_exact blocks at most (HTB / 64 visits each)
constexpr int SLOW_GRID = 256;         // k_rl_exact blocks for the slow visits (their count stays on the device)
constexpr int LTB = 256;                // list kernels
constexpr int LPER = 8;                 // vertices per thread in the list kernels
// Degree classes of a bucket's entries (the list is bucket-major, class-minor): rows of <= 16,
// <= 24, <= 32, <= 48, <= DM entries are decided by sorting networks of that width (24 and 48:
// the 32- and 64-input odd-even merge networks without the comparators past the width, 132 and
// 384 compare-exchanges against 191 and 543), longer ones by k_rl_exact.  LFR-1M (tau1 = 3,
// degrees ~19..50): ~44 % of the rows have 19..24 entries and ~23 % 33..48.
constexpr int NCLS = 6;
__host__ __device__ __forceinline__ int rl_class(int d) {
    return d <= 16 ? 0 : d <= 24 ? 1 : d <= 32 ? 2 : d <= 48 ? 3 : d <= DM ? 4 : 5;
}

struct RL {
    int64_t N, S, PN;
    int chunk;
    uint32_t perm_n;
    int B;
    int n_r, rbase, LG, VPW, banks, ldT;
    int lgs;                     // log2(LG)
    uint32_t iter;
    uint64_t seed;
    const int64_t* rowptr;
    const int32_t* col;
    const int32_t* cw;
    const int4* vrec;            // row start, degree, k_v (int32: 2M < 2^31), slot
    const int64_t* kdeg;
    int64_t M2;
    int unitw;
    int wbits;                   // bits of the largest edge weight (key packing)
    const int32_t* colw;         // weighted graphs with weights < 256: (col << wbits) | weight per entry
    int32_t* lab;                // labT [N][ldT]
    int32_t* tot;                // totT [N][ldT] (louvain)
    int32_t* dec;                // [PN][ldT]: target community or -1, per list entry and replica
    // visits whose best max-weight candidate does not settle the decision (a lighter community
    // may still score higher: k_v * Sigma >= 2M), decided exactly by k_rl_exact: (entry << 14) |
    // local replica; slow_cnt is reset by the bucket's k_rl_apply
    int64_t* slow;
    int32_t* slow_cnt;
    int4* list;                  // [PN] the sweep's entries, bucket-major: vertex, row start, degree, k_v
                                 // (the vertex record travels with the entry: no dependent vrec read)
    uint64_t* lmask;             // [PN][banks] visiting replicas of each entry
    uint64_t* vmask;             // [N][banks] list-build scratch
    int32_t* boff;               // [B*NCLS+1] segment offsets (segment = bucket * NCLS + degree class)
    int32_t* cursor;             // [B*NCLS] fill cursors
    // visit mode (sparse sweeps): one lane per (entry, replica) visit instead of one wave per
    // entry; visits of segment s are voff[s]..voff[s+1] in vlist (entry << 7 | local replica)
    int32_t* voff;               // [B*NCLS+1]
    int32_t* vcursor;            // [B*NCLS]
    int64_t* vlist;
    uint64_t* aff;               // [banks][N] affected flags (pruning), one bit per replica
    uint64_t* mvf;               // [banks][N] movers of a tracked sweep (lm)
    int32_t* active;             // [n_r]
    int32_t* track;              // [n_r] moves tracked this sweep | [n_r..2n_r) this sweep's list filters
    int prune, lm, track_div;
    unsigned long long* red;     // [n_r][NSH][RF]
    unsigned long long* sacc;    // [n_r][4] visits / entries / cands / units over the run
    int32_t* hscratch;           // global tables for rows past the LDS table
    int64_t hslots;
    double min_dq;
    int hybrid;                  // FC_OPT_CD_ENGINE=2: stop before the first sweep in which a replica's
                                 // filtered list is sparse (< N/4; cd.hip takes over: cd_run_hybrid)
    const int32_t* acnt;         // hybrid: [n_r] affected bits per replica at the sweep's start
    int dense_div;               // hybrid: a filtered list of >= N/dense_div stays here (0: none does)
};
// hybrid: replica r runs a filtered sweep whose list holds < N/dense_div vertices (its own order on cd.hip)
__device__ __forceinline__ bool rl_sparse(const RL& a, int r) {
    return a.hybrid && a.active[r] && a.prune && a.track[a.n_r + r] && (int64_t)a.dense_div * a.acnt[r] < a.N;
}

__device__ __forceinline__ Perm rl_perm(const RL& a, int sweep) {
    Perm P = make_perm(a.perm_n, stream_key(a.seed, SHARED_RG, a.iter, (uint32_t)sweep, 1));
    if (a.chunk) P.off = stream_key(a.seed, SHARED_RG, a.iter, (uint32_t)sweep, 3) & (RL_CHUNK - 1);
    return P;
}
__device__ __forceinline__ uint32_t rl_bucket(const RL& a, const Perm& P, uint32_t v) {
    uint32_t pos;
    if (!a.chunk) pos = perm_invert(P, v);
    else {
        const uint32_t w = v + P.off;
        pos = perm_invert(P, w / RL_CHUNK) * RL_CHUNK + w % RL_CHUNK;
    }
    return pos / (uint32_t)a.S;
}
__device__ __forceinline__ unsigned long long* rl_red(const RL& a, int r, int f) {
    return a.red + ((size_t)r * NSH + (blockIdx.x & (NSH - 1))) * RF + f;
}
__device__ __forceinline__ bool rl_better(long long s1, uint32_t h1, int32_t c1, long long s2, uint32_t h2,
                                          int32_t c2) {
    if (s1 != s2) return s1 > s2;
    if (h1 != h2) return h1 > h2;
    return c1 < c2;
}
// base[i] through a 32-bit byte offset (global_load saddr + voffset: one VGPR per address;
// every node-major table here is < 4 GiB)
__device__ __forceinline__ int32_t ld_off(const int32_t* base, uint32_t i) {
    return *reinterpret_cast<const int32_t*>(reinterpret_cast<const char*>(base) + (i << 2));
}
__device__ __forceinline__ int wave_max(int x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x = max(x, __shfl_xor(x, off));
    return x;
}
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// LPA, tracked sweep: a visit with several dominant labels flags its own vertex for the next
// sweep (igraph redraws among them at every visit; oracle tw_replica) -- one lane's bit
__device__ __forceinline__ void rl_tie_flag(const RL& a, int rr, int32_t v) {
    atomicOr((unsigned long long*)&a.aff[(int64_t)(rr >> 6) * a.N + v], 1ull << (rr & 63));
}

// ------------------------------------------------------------------ init / export
__global__ void k_rl_init(int64_t N, int ldT, const int64_t* kdeg, int32_t* lab, int32_t* tot) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N * ldT) return;
    const int64_t v = i / ldT;
    lab[i] = (int32_t)v;
    if (tot) tot[i] = (int32_t)kdeg[v];
}
// labT [N][ldT] -> lab [n_r][N] in slot order (what labels_to_host and the Leiden code read):
// 64 slots x 64 replicas per tile through LDS, label rows read and slot rows written as whole
// 256-byte runs (the inverse of cd.hip k_transpose).  sinv = nullptr: vertex order (the hybrid
// hands totT [N][ldT] over as cd.hip's tot [n_r][N] this way).
__global__ __launch_bounds__(256) void k_rl_export(int64_t N, int n_r, int ldT, const int32_t* labT, const int32_t* sinv,
                                                   int32_t* lab) {
    __shared__ int32_t t[64][65];
    __shared__ int32_t sv[64];
    const int64_t s0 = (int64_t)blockIdx.x * 64;
    const int r0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 64 x 4
    if (ty == 0) sv[tx] = s0 + tx < N ? (sinv ? sinv[s0 + tx] : (int32_t)(s0 + tx)) : -1;
    __syncthreads();
    for (int ss = ty; ss < 64; ss += 4) {
        const int32_t v = sv[ss];
        const int r = r0 + tx;
        if (v >= 0 && r < n_r) t[ss][tx] = labT[(int64_t)v * ldT + r];
    }
    __syncthreads();
    for (int rr = ty; rr < 64; rr += 4) {
        const int r = r0 + rr;
        if (r < n_r && s0 + tx < N) lab[(int64_t)r * N + s0 + tx] = t[tx][rr];
    }
}

// ------------------------------------------------------------------ visit lists
// Per vertex and bank: the replicas visiting it this sweep -- active ones in a full sweep,
// plus filtered ones whose affected bit is set (every neighbour of a tracked mover, or with
// lm the neighbours that ended in another community).  A listed sweep (prune, sweep > 0)
// consumes the flags (oracle tw_replica clears them at the sweep start).  Dynamic LDS:
// B ints + 2 * banks u64.
__global__ __launch_bounds__(LTB) void k_rl_list_count(RL a, int sweep, int listed, int32_t* bcnt, int32_t* vcnt) {
    extern __shared__ unsigned long long s_dyn[];
    uint64_t* s_act = (uint64_t*)s_dyn;
    uint64_t* s_flt = s_act + a.banks;
    int* s_b = (int*)(s_flt + a.banks);
    int* s_v = s_b + a.B * NCLS;
    for (int k = threadIdx.x; k < a.B * NCLS; k += LTB) { s_b[k] = 0; s_v[k] = 0; }
    for (int b = threadIdx.x; b < a.banks; b += LTB) { s_act[b] = 0; s_flt[b] = 0; }
    __syncthreads();
    for (int r = threadIdx.x; r < a.n_r; r += LTB) {
        if (!a.active[r]) continue;
        atomicOr((unsigned long long*)&s_act[r >> 6], 1ull << (r & 63));
        if (a.prune && a.track[a.n_r + r]) atomicOr((unsigned long long*)&s_flt[r >> 6], 1ull << (r & 63));
    }
    __syncthreads();
    if (a.hybrid && listed) {   // a sparse filtered list: cd.hip takes over, the flags stay for it (block-uniform)
        bool any = false;
        for (int r = 0; r < a.n_r && !any; ++r) any = rl_sparse(a, r);
        if (any) return;
    }
    const Perm P = rl_perm(a, sweep);
    const int64_t v0 = (int64_t)blockIdx.x * LTB * LPER + threadIdx.x;
#pragma unroll
    for (int i = 0; i < LPER; ++i) {
        const int64_t v = v0 + (int64_t)i * LTB;
        if (v >= a.N) break;
        int nv = 0;
        for (int b = 0; b < a.banks; ++b) {
            uint64_t f = a.aff[(int64_t)b * a.N + v];
            if (listed && f) a.aff[(int64_t)b * a.N + v] = 0;
            const uint64_t m = s_act[b] & (~s_flt[b] | f);
            a.vmask[v * a.banks + b] = m;
            nv += __popcll(m);
        }
        if (nv) {
            const int sg = rl_bucket(a, P, (uint32_t)v) * NCLS + rl_class(a.vrec[v].y);
            atomicAdd(&s_b[sg], 1);
            atomicAdd(&s_v[sg], nv);
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < a.B * NCLS; k += LTB) {
        if (s_b[k]) atomicAdd(&bcnt[k], s_b[k]);
        if (s_v[k]) atomicAdd(&vcnt[k], s_v[k]);
    }
}
// Offsets of the sweep's segments; the counts are zeroed once read (the next sweep's
// k_rl_list_count finds them zero: no memset launches per sweep) and the active counts the
// previous sweep left are copied behind voff, so boff | voff | n_active[0..1] is ONE host read.
__global__ void k_rl_list_plan(int nseg, int32_t* bcnt, int32_t* boff, int32_t* cursor, int32_t* vcnt,
                               int32_t* voff, int32_t* vcursor, const int32_t* n_active) {
    if (threadIdx.x != 0) return;
    int32_t acc = 0, vacc = 0;
    for (int k = 0; k < nseg; ++k) {
        boff[k] = acc; cursor[k] = acc; acc += bcnt[k];
        voff[k] = vacc; vcursor[k] = vacc; vacc += vcnt[k];
        bcnt[k] = 0; vcnt[k] = 0;
    }
    boff[nseg] = acc;
    voff[nseg] = vacc;
    voff[nseg + 1] = n_active[0];
    voff[nseg + 2] = n_active[1];
}
// Visit mode: each listed entry's replicas as (entry, replica) pairs.  The entries are
// segment-major, so an exclusive scan of the per-entry visit counts lays the visits out
// segment-major too (segment s starts at the scan value of its first entry, = voff[s]).
__global__ __launch_bounds__(LTB) void k_rl_visits_count(RL a, int64_t n_entries, int32_t* nv) {
    const int64_t e = (int64_t)blockIdx.x * LTB + threadIdx.x;
    if (e >= n_entries) return;
    int c = 0;
    for (int b = 0; b < a.banks; ++b) c += __popcll(a.lmask[e * a.banks + b]);
    nv[e] = c;
}
__global__ __launch_bounds__(LTB) void k_rl_visits_fill(RL a, int64_t n_entries, const int32_t* vpos) {
    const int64_t e = (int64_t)blockIdx.x * LTB + threadIdx.x;
    if (e >= n_entries) return;
    int64_t pos = vpos[e];
    for (int b = 0; b < a.banks; ++b) {
        uint64_t m = a.lmask[e * a.banks + b];
        while (m) {
            const int bit = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            a.vlist[pos++] = (e << 14) | (int64_t)(b * 64 + bit);
        }
    }
}

__global__ __launch_bounds__(LTB) void k_rl_list_fill(RL a, int sweep) {
    extern __shared__ int s_lb[];
    int* s_cnt = s_lb;
    int* s_base = s_lb + a.B * NCLS;
    for (int k = threadIdx.x; k < a.B * NCLS; k += LTB) s_cnt[k] = 0;
    __syncthreads();
    const Perm P = rl_perm(a, sweep);
    int bk[LPER], loc[LPER];
    const int64_t v0 = (int64_t)blockIdx.x * LTB * LPER + threadIdx.x;
#pragma unroll
    for (int i = 0; i < LPER; ++i) {
        const int64_t v = v0 + (int64_t)i * LTB;
        bk[i] = -1;
        if (v >= a.N) continue;
        bool any = false;
        for (int b = 0; b < a.banks; ++b) any |= a.vmask[v * a.banks + b] != 0;
        if (!any) continue;
        bk[i] = (int)rl_bucket(a, P, (uint32_t)v) * NCLS + rl_class(a.vrec[v].y);
        loc[i] = atomicAdd(&s_cnt[bk[i]], 1);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < a.B * NCLS; k += LTB) s_base[k] = s_cnt[k] ? atomicAdd(&a.cursor[k], s_cnt[k]) : 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < LPER; ++i) {
        if (bk[i] < 0) continue;
        const int64_t v = v0 + (int64_t)i * LTB;
        const int64_t e = s_base[bk[i]] + loc[i];
        const int4 vr = a.vrec[v];
        a.list[e] = make_int4((int32_t)v, vr.x, vr.y, vr.z);
        for (int b = 0; b < a.banks; ++b) a.lmask[e * a.banks + b] = a.vmask[v * a.banks + b];
    }
}

// ------------------------------------------------------------------ unit mapping
// Wave item w of a bucket whose entries are [e0, e1): one bank -> VPW consecutive entries
// (sub-group s takes entry e0 + w*VPW + s); several banks -> entry e0 + w / banks, bank w % banks.
struct Unit {
    int64_t e;
    int bank, s, rl, r;
    bool valid;
};
__device__ __forceinline__ Unit rl_unit(const RL& a, int64_t e0, int64_t e1, int64_t w) {
    Unit u;
    const int lane = threadIdx.x & 63;
    u.s = lane >> a.lgs;
    u.rl = lane & (a.LG - 1);
    if (a.banks == 1) { u.e = e0 + (w << (6 - a.lgs)) + u.s; u.bank = 0; }
    else { u.e = e0 + w / a.banks; u.bank = (int)(w % a.banks); }
    u.r = u.bank * 64 + u.rl;
    u.valid = u.e < e1 && u.s < a.VPW;
    return u;
}
__device__ __forceinline__ int64_t rl_items(const RL& a, int64_t n) {
    return a.banks == 1 ? (n + a.VPW - 1) / a.VPW : n * a.banks;
}

// ------------------------------------------------------------------ decide (light rows)
// Per unit the lanes' header: the entry's vertex, the lane's replica bit, the row.  Rows
// longer than DM are listed for k_rl_exact (one entry per unit, by the sub-group's lane 0).
struct Hdr {
    int32_t v;
    uint64_t msk;
    int64_t rb;
    int d, kvi, ds, rr;
    bool on, heavy, work;
};
// The entry record and replica mask of a unit (prefetched one item ahead by the decide kernel).
struct Rec {
    int4 e;
    uint64_t msk;
};
__device__ __forceinline__ Rec rl_fetch(const RL& a, const Unit& u) {
    Rec r;
    r.e = make_int4(-1, 0, 0, 0);
    r.msk = 0;
    if (u.valid) {
        r.e = a.list[u.e];
        r.msk = a.lmask[u.e * a.banks + u.bank];
    }
    return r;
}
__device__ __forceinline__ Hdr rl_header(const RL& a, const Unit& u, const Rec& rec) {
    Hdr h;
    h.rr = u.bank * 64 + u.rl;
    h.v = rec.e.x;
    h.msk = rec.msk;
    h.rb = (int64_t)(uint32_t)rec.e.y;
    h.d = rec.e.z;
    h.kvi = rec.e.w;
    h.on = u.valid && h.rr < a.n_r && ((h.msk >> u.rl) & 1ull);
    h.heavy = u.valid && h.d > DM;
    h.work = h.on && !h.heavy && h.d > 0;
    h.ds = (u.valid && !h.heavy && h.msk) ? h.d : 0;
    return h;
}

// Ascending sort of K keys held in registers: Batcher's odd-even merge sort (K = 2^k; 63 / 191 /
// 543 compare-exchanges at K = 16 / 32 / 64 against a bitonic network's 80 / 240 / 672; every
// index is a compile-time constant, 2 VALU per compare-exchange).
template <int K>
__device__ __forceinline__ void oem_sort(int32_t (&x)[K]) {
#pragma unroll
    for (int p = 1; p < K; p <<= 1)
#pragma unroll
        for (int k = p; k >= 1; k >>= 1)
#pragma unroll
            for (int j = k % p; j + k < K; j += 2 * k)
#pragma unroll
                for (int i = 0; i < k; ++i)
                    if ((i + j) / (2 * p) == (i + j + k) / (2 * p) && i + j + k < K) {
                        const int32_t a = x[i + j], b = x[i + j + k];
                        x[i + j] = min(a, b);
                        x[i + j + k] = max(a, b);
                    }
}

// One lane's decision from its row (K >= the wave's longest light row).  Keys are
// (label << wb) | weight (wb = 0 on unit graphs), -1 for empty and (louvain) own-community
// entries; sorted, a run of equal labels is one neighbour community with its summed weight.
// Pass A: the largest weight vm (louvain: foreign communities only; LPA: own included).
// Pass B: the runs of weight vm are the candidates; their Sigma is gathered (16 positions per
// batch, batches without a candidate skipped wave-wide) and the best score wins (score =
// vm*2M - k_v*Sigma, ties by the replica's hash, then the smaller id).  A lighter run scores
// <= (vm - 1)*2M: only when that still reaches the best are the lighter runs evaluated.
// WM: the row's weights -- WM_UNIT none (every weight 1), WM_W8 read with the neighbour id from
// colw and kept 4 per register while the label gathers are in flight (weights < 256), WM_WIDE a
// separate cw row (one register per entry)
constexpr int WM_WIDE = 0, WM_UNIT = 1, WM_W8 = 2;
#ifndef FC_RL_SB
#define FC_RL_SB 16
#endif
constexpr int SB = FC_RL_SB;            // Sigma gathers per batch in rl_runs
// FC_RL_LPA_OWN (A/B switch, default on): LPA keeps its own-label entries out of the keys too
// (counted in k_own; the own label a candidate when k_own is the largest count), so a wave whose
// lanes are all settled (2 k_own > d: own is the unique majority) skips like Louvain's, and the
// sort networks hold fewer live keys (LPA K = 32: 146 -> 126 VGPRs, 3 -> 4 waves per SIMD)
#ifndef FC_RL_LPA_OWN
#define FC_RL_LPA_OWN 1
#endif
// The decision from a lane's K keys ((label << wbits) | weight, -1 for empty and own-label
// entries -- LPA's too under FC_RL_LPA_OWN): sort, runs, candidates (rl_sorted's second half).
template <bool LOUV, int K, int WM>
__device__ __forceinline__ int32_t rl_runs(const RL& a, const Hdr& h, int sweep, int32_t (&x)[K], int32_t own,
                                           long long kown, int32_t tot_own, uint32_t home, unsigned long long& c_dq,
                                           uint32_t& c_unst, uint32_t& c_cand, bool& slow_out) {
    constexpr bool UNITW = WM == WM_UNIT;
    const uint32_t rr = (uint32_t)h.rr, ldT = (uint32_t)a.ldT;
    const int wb = UNITW ? 0 : a.wbits;
    const int32_t wm = (1 << wb) - 1;
    const bool wk = h.work;
    oem_sort<K>(x);
    // run ends and summed weights: e = bit q set when the run of equal labels ends at q
    // pass A: the largest weight vm
    int vm = INT_MIN;
    {
        int acc = 0;
        int32_t kl = (int32_t)kown;
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const int32_t l = x[q] >> wb;
            const int w = UNITW ? 1 : (x[q] & wm);
            acc = (q > 0 && l == (x[q - 1] >> wb)) ? acc + w : w;
            const bool end = x[q] >= 0 && (q == K - 1 || (x[q + 1] >> wb) != l);
            vm = end ? max(vm, acc) : vm;
            if (!LOUV && !FC_RL_LPA_OWN) kl = (end && l == own) ? acc : kl;
        }
        if (!LOUV && !FC_RL_LPA_OWN) kown = kl;
        if (!LOUV && FC_RL_LPA_OWN) vm = max(vm, (int)kown);  // the own label's count is a run too
    }
    // Louvain: no candidate can gain when even weight vm at Sigma = 0 cannot, i.e. when
    // (vm - k_own)*2M + k_v*(Sigma_own - k_v) <= 0 (score_c <= vm*2M for every c): then no
    // Sigma is gathered and the vertex stays (in settled sweeps most vertices)
    bool hope = true;
    if (LOUV) hope = wk && ((long long)vm - kown) * a.M2 + (long long)h.kvi * ((long long)tot_own - h.kvi) > 0;
    // pass B: candidate runs (the runs of weight vm), as bits of cm
    uint32_t cm_lo = 0, cm_hi = 0;
    if (hope) {
        int acc = 0;
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const int32_t l = x[q] >> wb;
            const int w = UNITW ? 1 : (x[q] & wm);
            acc = (q > 0 && l == (x[q - 1] >> wb)) ? acc + w : w;
            const bool cand = x[q] >= 0 && (q == K - 1 || (x[q + 1] >> wb) != l) && acc == vm;
            if (q < 32) cm_lo |= (uint32_t)cand << (q & 31);
            else cm_hi |= (uint32_t)cand << (q & 31);
        }
    }
    // LPA, own entries out of the keys: the own label is a candidate when its count is the largest
    const bool own_cand = !LOUV && FC_RL_LPA_OWN && wk && kown > 0 && kown == (long long)vm;
    const int ncand = __popc(cm_lo) + __popc(cm_hi) + (own_cand ? 1 : 0);
    if (wk) c_cand += (uint32_t)ncand;
    const uint32_t tvh = hash32(stream_key(a.seed, (uint32_t)(a.rbase + h.rr), a.iter, (uint32_t)sweep, 2) ^ (uint32_t)h.v);
    int32_t dcs = -1;
    if (LOUV) {
        const long long kv = h.kvi;
        // among the candidates (all of weight vm) score = vm*2M - k_v*Sigma: the best is the
        // smallest Sigma (every Sigma taken as 0 when k_v = 0), then the largest hash -- one
        // unsigned 64-bit minimum of (Sigma << 32) | ~hash; the hash is a bijection of the id
        // (no id tie is left), inverted for the winner
        uint64_t bkey = ~0ull;
        // SB positions per batch: FC_RL_SB (default 16; 8 holds 8 fewer VGPRs live)
#pragma unroll
        for (int c0 = 0; c0 < K; c0 += SB) {
            const uint32_t bits = ((c0 < 32 ? cm_lo : cm_hi) >> (c0 & 31)) & ((1u << SB) - 1u);
            if (__ballot(bits != 0) == 0) continue;             // wave-uniform
            int32_t tq[SB];
#pragma unroll
            for (int i = 0; i < SB; ++i) {                     // non-candidates read the lane's own slot (a hit)
                if (c0 + i >= K) break;                        // K = 24: the last batch is half
                const bool b = (bits >> i) & 1u;
                tq[i] = ld_off(a.tot, b ? (uint32_t)(x[c0 + i] >> wb) * ldT + rr : home);
            }
#pragma unroll
            for (int i = 0; i < SB; ++i) {
                if (c0 + i >= K) break;
                const bool b = (bits >> i) & 1u;
                const uint32_t hh = hash32(tvh ^ (uint32_t)(x[c0 + i] >> wb));
                const uint64_t key = ((uint64_t)(kv ? (uint32_t)tq[i] : 0u) << 32) | (uint32_t)~hh;
                bkey = (b && key < bkey) ? key : bkey;
            }
        }
        long long best_s = LLONG_MIN;
        uint32_t best_h = 0;
        int32_t best_c = INT_MAX;
        if (ncand != 0) {
            best_h = ~(uint32_t)bkey;
            best_c = (int32_t)(hash32_inv(best_h) ^ tvh);
            best_s = (long long)vm * a.M2 - kv * (long long)(uint32_t)(bkey >> 32);
        }
        // a lighter run (weight <= vm - 1) scores <= weight * 2M: it can still reach the best
        // only when k_v * Sigma_best >= 2M -- rare on large graphs, common on small weighted
        // consensus graphs (2M small against k_v * Sigma).  Such a visit is handed to
        // k_rl_exact (a wave and an LDS table per visit) instead of being finished here.
        slow_out = wk && ncand != 0 && (long long)(vm - 1) * a.M2 >= best_s;
        if (wk && ncand != 0 && !slow_out) {
            const long long G = best_s - kown * a.M2 + kv * ((long long)tot_own - kv);
            if (G > 0) {
                const double dqd = (double)G * 2.0 / ((double)a.M2 * (double)a.M2);
                c_dq += (unsigned long long)llrint(dqd * DQ_SCALE);
                dcs = best_c;
            }
        }
    } else {
        uint32_t best_h = 0;
        int32_t best_c = -1;
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const bool b = ((q < 32 ? cm_lo : cm_hi) >> (q & 31)) & 1u;
            const uint32_t hh = hash32(tvh ^ (uint32_t)x[q]);
            const bool take = b && (best_c < 0 || hh > best_h);
            best_h = take ? hh : best_h;
            best_c = take ? x[q] : best_c;
        }
        if (own_cand) {
            const uint32_t hh = hash32(tvh ^ (uint32_t)own);
            if (best_c < 0 || hh > best_h) { best_h = hh; best_c = own; }
        }
        if (wk && ncand != 0) {
            c_unst += (kown != (long long)vm) ? 1 : 0;
            dcs = best_c != own ? best_c : -1;
        }
    }
    return dcs;
}

template <bool LOUV, int K, int WM>
__device__ __forceinline__ int32_t rl_sorted(const RL& a, const Hdr& h, int sweep, unsigned long long& c_dq,
                                             uint32_t& c_unst, uint32_t& c_cand, bool& slow_out) {
    constexpr bool UNITW = WM == WM_UNIT;
    slow_out = false;
    const uint32_t rr = (uint32_t)h.rr, ldT = (uint32_t)a.ldT;
    const int wb = UNITW ? 0 : a.wbits;
    const int32_t wm = (1 << wb) - 1;
    const bool wk = h.work;
    // padding / idle lanes read a slot of their own vertex's row (cached, distinct per wave)
    // instead of branching; never a shared row, which every wave would hit on one L2 channel
    const uint32_t home = (h.v >= 0 ? (uint32_t)h.v : 0u) * ldT + rr;
    const int32_t own0 = ld_off(a.lab, home);
    const int32_t own = wk ? own0 : -1;
    // entry j of the lane's row is live iff j < dsw: the selects below test that, not the
    // loaded values, so a neighbour id is dead once its label load is issued (one register
    // per entry)
    const int dsw = wk ? h.ds : 0;
    int32_t x[K];
#pragma unroll
    for (int j = 0; j < K; ++j)                                 // idle / padding lanes read col[rb] (a hit)
        x[j] = ld_off(WM == WM_W8 ? a.colw : a.col, (uint32_t)h.rb + (uint32_t)(j < dsw ? j : 0));
    int32_t tot_own = 0;
    if (LOUV) {
        const int32_t t0 = ld_off(a.tot, wk ? (uint32_t)own * ldT + rr : home);
        tot_own = wk ? t0 : 0;
    }
    long long kown = 0;
    if constexpr (UNITW) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const int32_t lj = ld_off(a.lab, j < dsw ? (uint32_t)x[j] * ldT + rr : home);
            x[j] = j < dsw ? lj : -1;
        }
        if (LOUV || FC_RL_LPA_OWN) {
            int ko = 0;
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const bool mine = x[j] == own && x[j] >= 0;
                ko += mine ? 1 : 0;
                x[j] = mine ? -1 : x[j];
            }
            kown = ko;
        }
    } else if constexpr (WM == WM_W8) {
        uint32_t wpk[(K + 3) / 4];                              // 4 weights per register
#pragma unroll
        for (int i = 0; i < (K + 3) / 4; ++i) wpk[i] = 0;
#pragma unroll
        for (int j = 0; j < K; ++j) wpk[j >> 2] |= (uint32_t)(x[j] & wm) << (8 * (j & 3));
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const int32_t lj = ld_off(a.lab, j < dsw ? (uint32_t)(x[j] >> wb) * ldT + rr : home);
            x[j] = j < dsw ? lj : -1;
        }
        int ko = 0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const int32_t wj = (int32_t)((wpk[j >> 2] >> (8 * (j & 3))) & 0xffu);
            const bool mine = LOUV && x[j] == own && x[j] >= 0;
            ko += mine ? wj : 0;
            x[j] = (mine || x[j] < 0) ? -1 : ((x[j] << wb) | wj);
        }
        kown = ko;
    } else {
        int32_t wv[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const int32_t wj = ld_off(a.cw, (uint32_t)h.rb + (uint32_t)(j < dsw ? j : 0));
            wv[j] = j < dsw ? wj : 0;
        }
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const int32_t lj = ld_off(a.lab, j < dsw ? (uint32_t)x[j] * ldT + rr : home);
            x[j] = j < dsw ? lj : -1;
        }
        int ko = 0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const bool mine = LOUV && x[j] == own && x[j] >= 0;
            ko += mine ? wv[j] : 0;
            x[j] = (mine || x[j] < 0) ? -1 : ((x[j] << wb) | wv[j]);
        }
        kown = ko;
    }
    // Louvain, settled vertex: every foreign community weighs at most k_v - k_own, so no move can
    // gain when (k_v - 2 k_own)*2M + k_v*(Sigma_own - k_v) <= 0.  When that holds on every lane
    // (the vertex is settled in all the wave's replicas -- most of a consensus graph), the sort
    // and the passes are skipped.
    if (LOUV) {
        const long long kvl = h.kvi;
        const bool settled = !wk || (kvl - 2 * kown) * a.M2 + kvl * ((long long)tot_own - kvl) <= 0;
        if (__ballot(!settled) == 0) return -1;                 // wave-uniform
    } else if (FC_RL_LPA_OWN) {
        // LPA: the own label holds more than half the row -- the unique largest count, no move
        // and a stable vertex -- on every lane: nothing to sort
        const bool settled = !wk || 2 * kown > (long long)dsw;
        if (__ballot(!settled) == 0) {
            if (wk) c_cand += 1u;                               // the own label, the one candidate
            return -1;
        }
    }
    // per-lane rows (several vertices per wave): the wave's longest row picks the network (a
    // bucket's list is class-minor, so a wave's rows mostly share their class), which lets one
    // launch serve the rows of <= 32 and one those of 33..64 (FC_RL_SPLIT bits 8 / 16)
    constexpr int KN = (K == 32 && (FC_RL_SPLIT & 8)) ? 16 : (K == 64 && (FC_RL_SPLIT & 16)) ? 48 : K;
    if constexpr (KN < K) {
        if (__builtin_amdgcn_readfirstlane(wave_max(dsw)) <= KN) {
            int32_t y[KN];
#pragma unroll
            for (int j = 0; j < KN; ++j) y[j] = x[j];
            return rl_runs<LOUV, KN, WM>(a, h, sweep, y, own, kown, tot_own, home, c_dq, c_unst, c_cand, slow_out);
        }
    }
    return rl_runs<LOUV, K, WM>(a, h, sweep, x, own, kown, tot_own, home, c_dq, c_unst, c_cand, slow_out);
}

// ---- one unit per wave (LG = 64: every lane deciding the same vertex, VPW = 1; C4 / C5) ----
// The unit's record and row are wave-uniform, so the row is not K per-lane broadcast loads:
// lane j holds entry j of the NEXT item's row (one coalesced load issued an item ahead, in
// flight while this item sorts), and the label gathers take each neighbour id with a
// readlane -- a scalar row base (saddr) plus the lane's replica offset, no per-entry address
// arithmetic and the neighbour-id stage off the item's dependent chain.  Same decisions.
struct RowPre {
    int32_t col;                 // lane j: entry j's neighbour id (colw: id << wbits | weight)
    int32_t w;                   // WM_WIDE: entry j's weight
    int32_t own;                 // this lane's label of the unit's vertex
};
__device__ __forceinline__ Rec rl_fetch_u(const RL& a, const Unit& u) {
    Rec r = rl_fetch(a, u);      // every lane fetched the same record: make that visible
    r.e.x = __builtin_amdgcn_readfirstlane(r.e.x);
    r.e.y = __builtin_amdgcn_readfirstlane(r.e.y);
    r.e.z = __builtin_amdgcn_readfirstlane(r.e.z);
    r.e.w = __builtin_amdgcn_readfirstlane(r.e.w);
    r.msk = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(r.msk >> 32)) << 32) |
            (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)r.msk);
    return r;
}
template <int WM>
__device__ __forceinline__ RowPre rl_row_pre(const RL& a, const Unit& u, const Rec& r) {
    RowPre p;
    p.col = 0; p.w = 0; p.own = 0;
    const uint32_t lane = threadIdx.x & 63;
    if (r.e.x >= 0) {            // u.valid (uniform)
        const int d = r.e.z;
        if (d > 0 && d <= DM) {  // lanes past the row repeat entry 0 (same line; masked by the decide)
            const uint32_t j = lane < (uint32_t)d ? lane : 0u;
            p.col = ld_off(WM == WM_W8 ? a.colw : a.col, (uint32_t)r.e.y + j);
            if (WM == WM_WIDE) p.w = ld_off(a.cw, (uint32_t)r.e.y + j);
        }
        p.own = ld_off(a.lab, (uint32_t)r.e.x * (uint32_t)a.ldT + (uint32_t)(u.bank * 64) + lane);
    }
    return p;
}
template <bool LOUV, int K, int WM>
__device__ __forceinline__ int32_t rl_sorted_u1(const RL& a, const Hdr& h, int sweep, const RowPre& pre,
                                                unsigned long long& c_dq, uint32_t& c_unst, uint32_t& c_cand,
                                                bool& slow_out) {
    constexpr bool UNITW = WM == WM_UNIT;
    slow_out = false;
    const uint32_t rr = (uint32_t)h.rr, ldT = (uint32_t)a.ldT;
    const int wb = UNITW ? 0 : a.wbits;
    const int32_t wm = (1 << wb) - 1;
    const bool wk = h.work;
    const int ds = h.ds;                                        // wave-uniform: the row's length or 0
    if (ds == 0) return -1;                                     // past the list, heavy, idle unit, empty row
    const uint32_t home = (uint32_t)h.v * ldT + rr;
    const int32_t own = wk ? pre.own : -1;
    int32_t x[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        // entries past the row repeat entry 0 (same line, a hit) and are masked below
        const int32_t cj = __builtin_amdgcn_readlane(pre.col, j);
        const uint32_t id = (uint32_t)(WM == WM_W8 ? (cj >> wb) : cj);
        x[j] = ld_off(a.lab, id * ldT + rr);                    // id * ldT scalar: one VALU add per entry
    }
    int32_t tot_own = 0;
    if (LOUV) {
        const int32_t t0 = ld_off(a.tot, wk ? (uint32_t)own * ldT + rr : home);
        tot_own = wk ? t0 : 0;
    }
    long long kown = 0;
    int ko = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const bool live = wk && j < ds;
        int32_t wj = 1;
        if (WM == WM_W8) wj = __builtin_amdgcn_readlane(pre.col, j) & wm;
        else if (WM == WM_WIDE) wj = __builtin_amdgcn_readlane(pre.w, j);
        const bool mine = (LOUV || FC_RL_LPA_OWN) && live && x[j] == own;
        ko += mine ? wj : 0;
        x[j] = (mine || !live) ? -1 : (UNITW ? x[j] : ((x[j] << wb) | wj));
    }
    kown = ko;
    if (LOUV) {
        const long long kvl = h.kvi;
        const bool settled = !wk || (kvl - 2 * kown) * a.M2 + kvl * ((long long)tot_own - kvl) <= 0;
        if (__ballot(!settled) == 0) return -1;                 // wave-uniform
    } else if (FC_RL_LPA_OWN) {
        const bool settled = !wk || 2 * kown > (long long)ds;
        if (__ballot(!settled) == 0) {
            if (wk) c_cand += 1u;                               // the own label, the one candidate
            return -1;
        }
    }
    // The row length is wave-uniform here, so a row of <= 3K/4 entries is sorted by the narrower
    // network (24 keys in the 32-key kernel, 48 in the 64-key one: the truncated odd-even merge
    // networks, 132 / 384 compare-exchanges against 191 / 543) without a launch of its own; the
    // keys past the row are empty (-1) and empty keys never form a run, so dropping them changes
    // no decision.  LFR-1M: ~57 % of the 17..32-entry rows have <= 24, ~96 % of the 33..64 ones
    // <= 48.
    constexpr int KS1 = (K == 32 && (FC_RL_SPLIT & 4)) ? 16 : K;   // 16-entry rows in the 32-key kernel
    if constexpr (KS1 < K) {
        if (__builtin_amdgcn_readfirstlane(ds) <= KS1) {
            int32_t y[KS1];
#pragma unroll
            for (int j = 0; j < KS1; ++j) y[j] = x[j];
            return rl_runs<LOUV, KS1, WM>(a, h, sweep, y, own, kown, tot_own, home, c_dq, c_unst, c_cand, slow_out);
        }
    }
    constexpr int KS = (K == 32 && (FC_RL_SPLIT & 1)) ? 24 : (K == 64 && (FC_RL_SPLIT & 2)) ? 48 : K;
    if constexpr (KS < K) {
        if (__builtin_amdgcn_readfirstlane(ds) <= KS) {
            int32_t y[KS];
#pragma unroll
            for (int j = 0; j < KS; ++j) y[j] = x[j];
            return rl_runs<LOUV, KS, WM>(a, h, sweep, y, own, kown, tot_own, home, c_dq, c_unst, c_cand, slow_out);
        }
    }
    return rl_runs<LOUV, K, WM>(a, h, sweep, x, own, kown, tot_own, home, c_dq, c_unst, c_cand, slow_out);
}

// Light rows with sortable keys (label and weight fit 31 bits): no LDS, one sorting network
// per lane, K chosen per wave from its longest row.
// Append the wave's slow visits to the exact kernel's list (one atomic per wave).
__device__ __forceinline__ void rl_push_slow(const RL& a, bool slow, int64_t e, int rr) {
    const uint64_t m = __ballot(slow);
    if (!m) return;                                             // wave-uniform
    const int lane = threadIdx.x & 63;
    int base = 0;
    if (lane == 0) base = atomicAdd(a.slow_cnt, __popcll(m));
    base = __shfl(base, 0);
    if (slow) a.slow[base + __popcll(m & ((1ull << lane) - 1))] = (e << 14) | (int64_t)rr;
}

// Occupancy bounds per key width (waves per SIMD; 1 = the compiler's choice): A/B switches
#ifndef FC_RLW16
#define FC_RLW16 1
#endif
#ifndef FC_RLW32
#define FC_RLW32 1
#endif
template <bool LOUV, int K, int WM, bool U1>
#ifndef FC_RLW32U
#define FC_RLW32U 4
#endif
#ifndef FC_RLW24U
#define FC_RLW24U 4
#endif
__global__ __launch_bounds__(RTB)
__attribute__((amdgpu_waves_per_eu(K <= 16 ? FC_RLW16 : K <= 24 ? (U1 ? FC_RLW24U : FC_RLW32) :
                                   K <= 32 ? (U1 ? FC_RLW32U : FC_RLW32) : 1)))
void k_rl_decide(RL a, int seg, int ns, int sweep) {
    const int lane = threadIdx.x & 63;
    const int64_t e0 = a.boff[seg], e1 = a.boff[seg + ns];   // degree classes seg .. seg + ns - 1
    const int64_t items = rl_items(a, e1 - e0);
    const int LG = a.LG;
    unsigned long long c_dq = 0;                                // 32-bit counts: one block's items
    uint32_t c_unst = 0, c_vis = 0, c_ent = 0, c_cand = 0, c_units = 0;
    int last_r = -1;
    auto flush = [&](int r) {
        if (r < 0) return;
        for (int off = LG; off < 64; off <<= 1) {
            c_dq += __shfl_xor(c_dq, off); c_unst += __shfl_xor(c_unst, off); c_vis += __shfl_xor(c_vis, off);
            c_ent += __shfl_xor(c_ent, off); c_cand += __shfl_xor(c_cand, off); c_units += __shfl_xor(c_units, off);
        }
        if (lane < LG && r < a.n_r) {
            if (c_dq) atomicAdd(rl_red(a, r, 0), c_dq);
            if (c_unst) atomicAdd(rl_red(a, r, 1), (unsigned long long)c_unst);
            if (c_vis) atomicAdd(rl_red(a, r, 3), (unsigned long long)c_vis);
            if (c_ent) atomicAdd(rl_red(a, r, 4), (unsigned long long)c_ent);
            if (c_cand) atomicAdd(rl_red(a, r, 5), (unsigned long long)c_cand);
            if (c_units) atomicAdd(rl_red(a, r, 6), (unsigned long long)c_units);
        }
        c_dq = 0;
        c_unst = c_vis = c_ent = c_cand = c_units = 0;
    };
    // records two items ahead; U1: the next item's row and own labels one item ahead
    Rec nxt = U1 ? rl_fetch_u(a, rl_unit(a, e0, e1, blockIdx.x)) : rl_fetch(a, rl_unit(a, e0, e1, blockIdx.x));
    Rec nx2 = nxt;
    RowPre pre;
    pre.col = pre.w = pre.own = 0;
    if constexpr (U1) {
        pre = rl_row_pre<WM>(a, rl_unit(a, e0, e1, blockIdx.x), nxt);
        nx2 = rl_fetch_u(a, rl_unit(a, e0, e1, (int64_t)blockIdx.x + gridDim.x));
    }
    for (int64_t w = blockIdx.x; w < items; w += gridDim.x) {
        const Unit u = rl_unit(a, e0, e1, w);
        if (a.banks > 1 && u.r != last_r) flush(last_r);
        last_r = a.banks > 1 ? u.r : (lane & (LG - 1));
        const Rec cur = nxt;
        RowPre pc = pre;
        if constexpr (U1) {
            nxt = nx2;
            pre = rl_row_pre<WM>(a, rl_unit(a, e0, e1, w + gridDim.x), nxt);   // in flight while this item runs
            nx2 = rl_fetch_u(a, rl_unit(a, e0, e1, w + 2 * (int64_t)gridDim.x));
        } else {
            nxt = rl_fetch(a, rl_unit(a, e0, e1, w + gridDim.x));   // in flight while this item runs
        }
        const Hdr h = rl_header(a, u, cur);
        bool slow;
        const uint32_t cc0 = c_cand;
        const int32_t dcs = U1 ? rl_sorted_u1<LOUV, K, WM>(a, h, sweep, pc, c_dq, c_unst, c_cand, slow)
                               : rl_sorted<LOUV, K, WM>(a, h, sweep, c_dq, c_unst, c_cand, slow);
        rl_push_slow(a, slow, u.e, h.rr);
        // LPA: the visit's candidates are the labels at the top count (rl_runs adds them to
        // c_cand; a settled lane adds 1), so >= 2 of them is a tie.  Read off the counter rather
        // than returned: one more live value through rl_runs changed the K = 64 kernel's code
        // (205 VGPRs, ~180 SGPR spills) into one that departed from the twin in sweep 0.
        const bool tied = !LOUV && c_cand - cc0 >= 2u;
        if (!LOUV && FC_LPA_TIES) {                             // LPA ties of tracked replicas: one OR per sub-group
            const uint64_t tb = __ballot(tied && a.track[h.rr]);
            const uint64_t ts = (tb >> (u.s * LG)) & (LG == 64 ? ~0ull : ((1ull << LG) - 1ull));
            if (u.valid && u.rl == 0 && ts) atomicOr((unsigned long long*)&a.aff[(int64_t)u.bank * a.N + h.v], (unsigned long long)ts);
        }
        if (h.work) { c_vis += 1; c_ent += (uint32_t)h.d; }
        if (u.valid && u.rl == 0 && h.msk) c_units += 1;
        if (u.valid && h.rr < a.n_r) a.dec[u.e * a.ldT + h.rr] = h.work ? dcs : -1;
    }
    flush(last_r);
}

// Visit mode: lane = one (entry, replica) visit -- rows are per lane (no sharing), for the
// sparse sweeps where most replicas of an entry are idle and a wave per entry would run mostly
// empty lanes.  Same decision code; counters go straight to the per-replica shards.
template <bool LOUV, int K, int WM>
__global__ __launch_bounds__(RTB) void k_rl_decide_v(RL a, int seg, int ns, int sweep) {
    const int64_t v0 = a.voff[seg], v1 = a.voff[seg + ns];
    for (int64_t base = (int64_t)blockIdx.x * 64; base < v1 - v0; base += (int64_t)gridDim.x * 64) {
        const int64_t i = base + (threadIdx.x & 63);
        const bool valid = i < v1 - v0;
        int64_t vp = 0;
        if (valid) vp = a.vlist[v0 + i];
        const int64_t e = vp >> 14;
        Hdr h;
        h.rr = (int)(vp & 16383);
        const int4 er = valid ? a.list[e] : make_int4(-1, 0, 0, 0);
        h.v = er.x;
        h.rb = (int64_t)(uint32_t)er.y;
        h.d = er.z;
        h.kvi = er.w;
        h.msk = 0;
        h.on = valid;
        h.heavy = false;
        h.work = valid && h.d > 0;
        h.ds = valid ? h.d : 0;
        unsigned long long c_dq = 0;
        uint32_t c_unst = 0, c_cand = 0;
        bool slow;
        const int32_t dcs = rl_sorted<LOUV, K, WM>(a, h, sweep, c_dq, c_unst, c_cand, slow);
        rl_push_slow(a, slow, e, h.rr);
        const bool tied = !LOUV && c_cand >= 2u;                 // this visit's candidates (see k_rl_decide)
        if (!LOUV && FC_LPA_TIES && valid && tied && a.track[h.rr]) rl_tie_flag(a, h.rr, h.v);
        if (valid) {
            a.dec[e * a.ldT + h.rr] = h.work ? dcs : -1;
            if (c_dq) atomicAdd(rl_red(a, h.rr, 0), c_dq);
            if (c_unst) atomicAdd(rl_red(a, h.rr, 1), (unsigned long long)c_unst);
            if (h.work) {
                atomicAdd(rl_red(a, h.rr, 3), 1ull);
                atomicAdd(rl_red(a, h.rr, 4), (unsigned long long)h.d);
            }
            if (c_cand) atomicAdd(rl_red(a, h.rr, 5), (unsigned long long)c_cand);
        }
    }
}

// Resident waves of a decide instantiation on this device (occupancy x CUs), once per
// instantiation: Louvain's grid is sized to them (c.rl_grid_mul x) instead of up to 8192 blocks,
// so a launch's blocks split its items evenly in one generation -- 8192 blocks ran ~2.7
// generations of 4-5 items, the last one on two thirds of the SIMDs.  LPA keeps the 8192 cap:
// its items' cost varies more (most waves settled, a few sorting) and the extra blocks balance
// it (SBM-4M 687 vs 695 ms).
template <bool LOUV, int K, int WM, bool U1>
static int64_t rl_decide_slots() {
    static int64_t slots = 0;
    if (!slots) {
        int nb = 0, dev = 0;
        FC_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)k_rl_decide<LOUV, K, WM, U1>, RTB, 0));
        FC_HIP(hipGetDevice(&dev));
        int cus = 0;
        FC_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        slots = (int64_t)std::max(1, nb) * std::max(1, cus);
    }
    return slots;
}

// Fallback for keys that do not pack into 31 bits (huge graphs or weights): the row's labels
// staged in LDS as L[j][lane], equal labels merged per lane by a triangular scan.
struct RLShared {
    int32_t L[DM][64];           // row labels per lane; merged / own entries DONE; then the candidates
    int32_t C[VPWMAX][DM];       // the sub-groups' rows (neighbour ids)
    int32_t W[VPWMAX][DM];       // their weights (weighted graphs)
};
template <bool LOUV>
__global__ __launch_bounds__(RTB) void k_rl_decide_lds(RL a, int k, int sweep) {
    __shared__ RLShared sh;
    const int lane = threadIdx.x & 63;
    const int64_t e0 = a.boff[k * NCLS], e1 = a.boff[k * NCLS + NCLS - 1];   // the light classes
    const int64_t items = rl_items(a, e1 - e0);
    const int LG = a.LG, VPW = a.VPW;
    // per-lane counters, flushed once per wave
    unsigned long long c_dq = 0, c_unst = 0, c_vis = 0, c_ent = 0, c_cand = 0, c_units = 0;
    int last_r = -1;
    auto flush = [&](int r) {
        if (r < 0) return;
        // lanes with the same replica (one per sub-group) are folded first
        for (int off = LG; off < 64; off <<= 1) {
            c_dq += __shfl_xor(c_dq, off); c_unst += __shfl_xor(c_unst, off); c_vis += __shfl_xor(c_vis, off);
            c_ent += __shfl_xor(c_ent, off); c_cand += __shfl_xor(c_cand, off); c_units += __shfl_xor(c_units, off);
        }
        if (lane < LG && r < a.n_r) {
            if (c_dq) atomicAdd(rl_red(a, r, 0), c_dq);
            if (c_unst) atomicAdd(rl_red(a, r, 1), c_unst);
            if (c_vis) atomicAdd(rl_red(a, r, 3), c_vis);
            if (c_ent) atomicAdd(rl_red(a, r, 4), c_ent);
            if (c_cand) atomicAdd(rl_red(a, r, 5), c_cand);
            if (c_units) atomicAdd(rl_red(a, r, 6), c_units);
        }
        c_dq = c_unst = c_vis = c_ent = c_cand = c_units = 0;
    };
    for (int64_t w = blockIdx.x; w < items; w += gridDim.x) {
        const Unit u = rl_unit(a, e0, e1, w);
        if (a.banks > 1 && u.r != last_r) { flush(last_r); }
        last_r = a.banks > 1 ? u.r : (lane & (LG - 1));
        const int rr = u.bank * 64 + u.rl;                      // local replica of this lane
        int32_t v = -1;
        uint64_t msk = 0;
        int4 er = make_int4(-1, 0, 0, 0);
        if (u.valid) {
            er = a.list[u.e];
            v = er.x;
            msk = a.lmask[u.e * a.banks + u.bank];
        }
        const bool on = u.valid && rr < a.n_r && ((msk >> u.rl) & 1ull);
        const int64_t rb = (int64_t)(uint32_t)er.y;
        const int d = er.z, kvi = er.w;
        const bool heavy = u.valid && d > DM;
        const bool work = on && !heavy && d > 0;
        const int ds = (u.valid && !heavy && msk) ? d : 0;     // the sub-group's staged row length
        const int64_t lrow = (int64_t)v * a.ldT + rr;
        int32_t own = -1;
        int32_t tot_own = 0;
        if (work) own = a.lab[lrow];
        // sub-group rows, flattened over the wave: prefix of the row lengths
        int o[VPWMAX], dsub[VPWMAX];
        int E = 0, dmax = 0;
#pragma unroll
        for (int t = 0; t < VPWMAX; ++t) {
            dsub[t] = t < VPW ? __shfl(ds, t * LG) : 0;
            o[t] = E;
            E += dsub[t];
            dmax = max(dmax, dsub[t]);
        }
        if (E == 0) {                                           // wave-uniform: nothing light here
            if (u.valid && rr < a.n_r) a.dec[u.e * a.ldT + rr] = -1;
            continue;
        }
        // row starts of the sub-groups, read while every lane is active (a shuffle from a
        // lane that has left the loop below would read garbage)
        int64_t rbs[VPWMAX];
#pragma unroll
        for (int t = 0; t < VPWMAX; ++t) rbs[t] = t < VPW ? __shfl(rb, t * LG) : 0;
        for (int f = lane; f < E; f += 64) {
            int t = 0;
#pragma unroll
            for (int q = 1; q < VPWMAX; ++q) t += (q < VPW && f >= o[q]) ? 1 : 0;
            int64_t rbt = rbs[0];
            int ot = o[0];
#pragma unroll
            for (int q = 1; q < VPWMAX; ++q)
                if (t == q) { rbt = rbs[q]; ot = o[q]; }
            const int j = f - ot;
            sh.C[t][j] = a.col[rbt + j];
            if (!a.unitw) sh.W[t][j] = a.cw[rbt + j];
        }
        if (LOUV && work) tot_own = a.tot[(int64_t)own * a.ldT + rr];
        wsync();
        // stage the labels: 32 gathers in flight per lane, own-community entries summed (louvain)
        long long kown = 0;
        for (int j0 = 0; j0 < dmax; j0 += 32) {
            int32_t lb[32];
#pragma unroll
            for (int q = 0; q < 32; ++q) {
                const int j = j0 + q;
                lb[q] = (work && j < ds) ? a.lab[(int64_t)sh.C[u.s][j] * a.ldT + rr] : DONE;
            }
#pragma unroll
            for (int q = 0; q < 32; ++q) {
                const int j = j0 + q;
                if (j >= dmax) break;
                int32_t c = lb[q];
                if (LOUV && c >= 0 && c == own) {
                    kown += a.unitw ? 1 : sh.W[u.s][j];
                    c = DONE;
                }
                sh.L[j][lane] = c;
            }
        }
        wsync();
        // merge equal labels: the first occurrence sums its duplicates and marks them; the
        // candidates of maximal weight are compacted into L[0..nc)
        int vm = INT_MIN, nc = 0;
        for (int j1 = 0; j1 < dmax; ++j1) {
            const int32_t c1 = sh.L[j1][lane];
            if (__ballot(c1 >= 0) == 0) continue;               // wave-uniform
            int acc = 0;
            if (c1 >= 0) {
                acc = a.unitw ? 1 : sh.W[u.s][j1];
                for (int j2 = j1 + 1; j2 < dmax; ++j2) {
                    if (sh.L[j2][lane] == c1) {
                        acc += a.unitw ? 1 : sh.W[u.s][j2];
                        sh.L[j2][lane] = DONE;
                    }
                }
                if (!LOUV && c1 == own) kown = acc;
                if (acc > vm) { vm = acc; nc = 0; }
                if (acc == vm) { sh.L[nc][lane] = c1; ++nc; }
            }
        }
        wsync();
        const uint32_t tvh = hash32(stream_key(a.seed, (uint32_t)(a.rbase + rr), a.iter, (uint32_t)sweep, 2) ^ (uint32_t)v);
        int32_t dcs = -1;
        if (LOUV) {
            // Sigma of the maximal-weight candidates, 8 gathers in flight per lane
            long long best_s = LLONG_MIN;
            uint32_t best_h = 0;
            int32_t best_c = INT_MAX;
            const long long kv = kvi;
            const int ncm = wave_max(work ? nc : 0);
            for (int i0 = 0; i0 < ncm; i0 += 8) {
                int32_t cq[8], tq[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    cq[q] = (work && i0 + q < nc) ? sh.L[i0 + q][lane] : -1;
                    tq[q] = cq[q] >= 0 ? a.tot[(int64_t)cq[q] * a.ldT + rr] : 0;
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    if (cq[q] < 0) continue;
                    const long long sc = (long long)vm * a.M2 - kv * (long long)tq[q];
                    const uint32_t h = hash32(tvh ^ (uint32_t)cq[q]);
                    if (best_c == INT_MAX || rl_better(sc, h, cq[q], best_s, best_h, best_c)) {
                        best_s = sc; best_h = h; best_c = cq[q];
                    }
                }
            }
            if (work) c_cand += (unsigned long long)nc;
            // a lighter candidate scores <= (vm - 1) * 2M: it can only reach the best when
            // k_v * Sigma_min >= 2M (rare) -- then the lane re-evaluates every candidate
            const bool slow = work && nc > 0 && (long long)(vm - 1) * a.M2 >= best_s;
            if (__ballot(slow)) {                               // wave-uniform
                if (slow) {
                    for (int j1 = 0; j1 < d; ++j1) {
                        const int32_t c1 = a.lab[(int64_t)a.col[rb + j1] * a.ldT + rr];
                        if (c1 == own) continue;
                        bool dup = false;
                        for (int j2 = 0; j2 < j1 && !dup; ++j2) dup = a.lab[(int64_t)a.col[rb + j2] * a.ldT + rr] == c1;
                        if (dup) continue;
                        long long val = 0;
                        for (int j2 = j1; j2 < d; ++j2)
                            if (a.lab[(int64_t)a.col[rb + j2] * a.ldT + rr] == c1) val += a.unitw ? 1 : a.cw[rb + j2];
                        if (val >= vm) continue;                // evaluated above
                        const long long sc = val * a.M2 - kv * (long long)a.tot[(int64_t)c1 * a.ldT + rr];
                        const uint32_t h = hash32(tvh ^ (uint32_t)c1);
                        ++c_cand;
                        if (rl_better(sc, h, c1, best_s, best_h, best_c)) { best_s = sc; best_h = h; best_c = c1; }
                    }
                }
            }
            if (work && nc > 0) {
                const long long G = best_s - kown * a.M2 + kv * ((long long)tot_own - kv);
                if (G > 0) {
                    const double dqd = (double)G * 2.0 / ((double)a.M2 * (double)a.M2);
                    c_dq += (unsigned long long)llrint(dqd * DQ_SCALE);
                    dcs = best_c;
                }
            }
        } else {
            // LPA: the most frequent label (own included), ties by the replica's hash
            uint32_t best_h = 0;
            int32_t best_c = -1;
            for (int i = 0; i < nc; ++i) {
                const int32_t c = sh.L[i][lane];
                const uint32_t h = hash32(tvh ^ (uint32_t)c);
                if (best_c < 0 || h > best_h) { best_h = h; best_c = c; }
            }
            if (work) {
                c_cand += (unsigned long long)nc;
                if (nc > 0) {
                    c_unst += (kown != (long long)vm) ? 1 : 0;
                    dcs = best_c != own ? best_c : -1;
                }
                if (FC_LPA_TIES && nc >= 2 && a.track[rr]) rl_tie_flag(a, rr, v);
            }
        }
        if (work) { c_vis += 1; c_ent += (unsigned long long)d; }
        if (u.valid && u.rl == 0 && msk && !heavy) c_units += 1;
        if (u.valid && rr < a.n_r) a.dec[u.e * a.ldT + rr] = work ? dcs : -1;
        wsync();                                                // L is reused by the next item
    }
    flush(last_r);
}

// ------------------------------------------------------------------ decide (exact, by table)
// Visits the sorting networks do not finish: the heavy class's rows (degree > DM) for every
// visiting replica, and the slow visits k_rl_decide listed.  One WAVE per visit, four per block:
// a wave's LDS table (HWSLOTS slots, rows <= HWSLOTS / 2; longer rows a global table of the
// wave's own) is cleared, filled and scanned by its 64 lanes with no block barrier (a wave's LDS
// operations execute in order), and the best candidate over EVERY neighbour community is a wave
// reduction.  (One block per vertex deciding its replicas one after the other paid four block
// barriers per replica; the slow visits used to re-read their row O(d^2) times per lane.)
template <bool LOUV>
__global__ __launch_bounds__(HTB) void k_rl_exact(RL a, int k, int sweep) {
    __shared__ int32_t key[HTB / 64][HWSLOTS], val[HTB / 64][HWSLOTS];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t h0 = a.boff[k * NCLS + NCLS - 1], h1 = a.boff[k * NCLS + NCLS];   // the heavy class
    const int64_t ch = (h1 - h0) * a.n_r;
    const int64_t cnt = ch + (LOUV ? *a.slow_cnt : 0);
    const int64_t gw = (int64_t)blockIdx.x * (HTB / 64) + wv, nw = (int64_t)gridDim.x * (HTB / 64);
    for (int64_t item = gw; item < cnt; item += nw) {      // wave-uniform
        int64_t e;
        int rr;
        const bool heavy = item < ch;
        if (heavy) {
            e = h0 + item / a.n_r;
            rr = (int)(item % a.n_r);
            const uint64_t msk = a.lmask[e * a.banks + (rr >> 6)];
            if (!((msk >> (rr & 63)) & 1ull)) continue;
        } else {                                            // k_rl_decide counted the visit itself
            const int64_t p = a.slow[item - ch];
            e = p >> 14;
            rr = (int)(p & 16383);
        }
        const int32_t v = a.list[e].x;
        const int64_t rb = a.rowptr[v], d = a.rowptr[v + 1] - rb;
        uint32_t slots = 64;
        while (slots < 2 * (uint32_t)d) slots <<= 1;
        int32_t* keys = key[wv];
        int32_t* vals = val[wv];
        if (slots > HWSLOTS) {
            slots = (uint32_t)a.hslots;
            keys = a.hscratch + gw * 2 * a.hslots;
            vals = keys + slots;
        }
        for (uint32_t q = lane; q < slots; q += 64) { keys[q] = -1; vals[q] = 0; }
        wsync();
        for (int64_t j = rb + lane; j < rb + d; j += 64) {
            const int32_t c = a.lab[(int64_t)a.col[j] * a.ldT + rr];
            const int32_t w = a.unitw ? 1 : a.cw[j];
            uint32_t h = hash32((uint32_t)c) & (slots - 1);
            while (true) {
                const int32_t prev = atomicCAS(&keys[h], -1, c);
                if (prev == -1 || prev == c) { atomicAdd(&vals[h], w); break; }
                h = (h + 1) & (slots - 1);
            }
        }
        wsync();
        const int32_t own = a.lab[(int64_t)v * a.ldT + rr];
        const long long kv = a.kdeg[v];
        const uint32_t tvh = hash32(stream_key(a.seed, (uint32_t)(a.rbase + rr), a.iter, (uint32_t)sweep, 2) ^ (uint32_t)v);
        long long best_s = LLONG_MIN, kown = 0;
        uint32_t best_h = 0;
        int32_t best_c = INT_MAX;
        int ncand = 0;
        int ntop = 0;                                         // LPA: labels at this lane's top count
        for (uint32_t q = lane; q < slots; q += 64) {
            const int32_t c = keys[q];
            if (c < 0) continue;
            const long long w = vals[q];
            if (c == own) kown = w;
            long long sc;
            if (LOUV) {
                if (c == own) continue;
                sc = w * a.M2 - kv * (long long)a.tot[(int64_t)c * a.ldT + rr];
            } else {
                sc = w;
                ntop = (best_c == INT_MAX || w > best_s) ? 1 : (w == best_s ? ntop + 1 : ntop);
            }
            ++ncand;
            const uint32_t h = hash32(tvh ^ (uint32_t)c);
            if (best_c == INT_MAX || rl_better(sc, h, c, best_s, best_h, best_c)) { best_s = sc; best_h = h; best_c = c; }
        }
        wsync();                                              // the table is reused by the next visit
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const long long s2 = __shfl_xor(best_s, off);
            const uint32_t hh2 = __shfl_xor(best_h, off);
            const int32_t c2 = __shfl_xor(best_c, off);
            if (!LOUV) {                                      // LPA: how many labels reach the top count
                const int n2 = __shfl_xor(ntop, off);
                if (c2 != INT_MAX) ntop = (best_c == INT_MAX || s2 > best_s) ? n2 : (s2 == best_s ? ntop + n2 : ntop);
            }
            if (c2 != INT_MAX && (best_c == INT_MAX || rl_better(s2, hh2, c2, best_s, best_h, best_c))) {
                best_s = s2; best_h = hh2; best_c = c2;
            }
            kown += __shfl_xor(kown, off);
            ncand += __shfl_xor(ncand, off);
        }
        // LPA ties of a tracked replica, counted in the reduction above (a second pass over the
        // table here made the compiler's k_rl_exact<false> depart from the twin in untracked
        // sweeps too: tools/debug_rl_lpa.py, round 5)
        if (!LOUV && FC_LPA_TIES && lane == 0 && ntop >= 2 && a.track[rr]) rl_tie_flag(a, rr, v);
        if (lane == 0) {
            int32_t dcs = -1;
            if (best_c != INT_MAX) {
                if (LOUV) {
                    const long long tot_own = a.tot[(int64_t)own * a.ldT + rr];
                    const long long G = best_s - kown * a.M2 + kv * (tot_own - kv);
                    if (G > 0) {
                        const double dqd = (double)G * 2.0 / ((double)a.M2 * (double)a.M2);
                        atomicAdd(rl_red(a, rr, 0), (unsigned long long)llrint(dqd * DQ_SCALE));
                        dcs = best_c;
                    }
                } else {
                    if (kown != best_s) atomicAdd(rl_red(a, rr, 1), 1ull);
                    dcs = best_c != own ? best_c : -1;
                }
            }
            a.dec[e * a.ldT + rr] = dcs;
            if (heavy) {                                      // slow visits: k_rl_decide counted them
                if (ncand) atomicAdd(rl_red(a, rr, 5), (unsigned long long)ncand);
                atomicAdd(rl_red(a, rr, 3), 1ull);
                atomicAdd(rl_red(a, rr, 4), (unsigned long long)d);
            }
        }
    }
}

// ------------------------------------------------------------------ apply
// A bucket's moves: label, community totals (int32 atomics, order-free), and while tracking
// either every neighbour flagged (one 64-bit OR per neighbour for all the sub-group's movers)
// or, with lm, the movers listed for k_rl_mark_lm.
template <bool LOUV>
__global__ __launch_bounds__(RTB) void k_rl_apply(RL a, int k) {
    const int lane = threadIdx.x & 63;
    // k_rl_exact consumed the bucket's slow list: empty it for the next bucket
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.slow_cnt = 0;
    const int64_t e0 = a.boff[k * NCLS], e1 = a.boff[k * NCLS + NCLS];
    const int64_t items = rl_items(a, e1 - e0);
    const int LG = a.LG;
    unsigned long long moves = 0;
    int last_r = -1;
    auto flush = [&](int r) {
        if (r < 0) return;
        for (int off = LG; off < 64; off <<= 1) moves += __shfl_xor(moves, off);
        if (lane < LG && r < a.n_r && moves) atomicAdd(rl_red(a, r, 2), moves);
        moves = 0;
    };
    const uint64_t gmask = LG == 64 ? ~0ull : ((1ull << LG) - 1ull);
    // items pipelined: entry record and decision two items ahead, the mover's old label one
    // ahead (a wave's items were a chain list -> decision -> label -> atomics each)
    struct Ap {
        int4 er;
        uint64_t msk;
        int32_t t;
    };
    auto fetch = [&](int64_t w) {
        Ap p;
        p.er = make_int4(-1, 0, 0, 0);
        p.msk = 0;
        p.t = -1;
        const Unit u = rl_unit(a, e0, e1, w);
        if (u.valid) {
            p.er = a.list[u.e];
            p.msk = a.lmask[u.e * a.banks + u.bank];
            if (u.r < a.n_r) p.t = a.dec[u.e * a.ldT + u.r];   // every visit slot was written (-1: none)
        }
        return p;
    };
    auto old_of = [&](const Ap& p, int64_t w) -> int32_t {
        const Unit u = rl_unit(a, e0, e1, w);
        const bool mv = u.valid && ((p.msk >> u.rl) & 1ull) && p.t >= 0;
        return mv ? a.lab[(int64_t)p.er.x * a.ldT + u.r] : -1;
    };
    const int64_t G = gridDim.x;
    Ap p1 = fetch(blockIdx.x), p2 = fetch(blockIdx.x + G);
    int32_t o1 = old_of(p1, blockIdx.x);
    for (int64_t w = blockIdx.x; w < items; w += G) {
        const Unit u = rl_unit(a, e0, e1, w);
        if (a.banks > 1 && u.r != last_r) flush(last_r);
        last_r = a.banks > 1 ? u.r : (lane & (LG - 1));
        const int rr = u.r;
        const Ap cur = p1;
        const int32_t old = o1;
        p1 = p2;
        o1 = old_of(p1, w + G);
        p2 = fetch(w + 2 * G);
        const int4 er = cur.er;
        const int32_t v = er.x, kvr = er.w;
        const int32_t t = (u.valid && ((cur.msk >> u.rl) & 1ull)) ? cur.t : -1;
        const bool moved = t >= 0;
        if (moved) {
            a.lab[(int64_t)v * a.ldT + rr] = t;
            if (LOUV) {
                atomicAdd(&a.tot[(int64_t)old * a.ldT + rr], -kvr);
                atomicAdd(&a.tot[(int64_t)t * a.ldT + rr], kvr);
            }
            ++moves;
        }
        const bool trk = moved && a.track[rr];
        const uint64_t bal = __ballot(trk);
        const uint64_t ms = (bal >> (u.s * LG)) & gmask;        // the sub-group's tracked movers
        if (!bal) continue;                                     // wave-uniform
        if (a.lm) {
            if (u.valid && u.rl == 0 && ms) a.mvf[(int64_t)u.bank * a.N + v] = ms;
        } else if (u.valid && ms) {
            const int64_t rb = (int64_t)(uint32_t)er.y;
            for (int j = u.rl; j < er.z; j += LG)
                atomicOr((unsigned long long*)&a.aff[(int64_t)u.bank * a.N + a.col[rb + j]], (unsigned long long)ms);
        }
    }
    flush(last_r);
}

// End of a tracked lm sweep: each mover marks the neighbours whose label now differs from its
// own (oracle tw_replica; cd.hip k_mark_lm), comparing the labels the sweep left.
__global__ __launch_bounds__(RTB) void k_rl_mark_lm(RL a) {
    const int lane = threadIdx.x & 63;
    const int LG = a.LG, VPW = a.VPW;
    const int s = lane / LG, rl = lane - s * LG;
    const int64_t per = a.banks == 1 ? VPW : 1;
    const int64_t items = a.banks == 1 ? (a.N + VPW - 1) / VPW : a.N * a.banks;
    const uint64_t gmask = LG == 64 ? ~0ull : ((1ull << LG) - 1ull);
    for (int64_t w = blockIdx.x; w < items; w += gridDim.x) {
        int64_t v;
        int bank;
        if (a.banks == 1) { v = w * per + s; bank = 0; }
        else { v = w / a.banks; bank = (int)(w % a.banks); }
        const bool valid = s < VPW && v < a.N;
        uint64_t m = valid ? a.mvf[(int64_t)bank * a.N + v] : 0;
        if (__ballot(m != 0) == 0) continue;                    // wave-uniform
        if (valid && rl == 0 && m) a.mvf[(int64_t)bank * a.N + v] = 0;
        const int rr = bank * 64 + rl;
        const bool mine = valid && ((m >> rl) & 1ull);
        const int32_t dl = mine ? a.lab[v * a.ldT + rr] : -1;
        int d = 0;
        int64_t rb = 0;
        if (valid && m) {
            const int4 vr = a.vrec[v];
            rb = (int64_t)(uint32_t)vr.x;
            d = vr.y;
        }
        // four entries' column and label loads in flight at a time (a row walk one entry per
        // iteration was a chain of dependent round trips: 13 ms per call at C5)
        const int dmax = wave_max(d);
        for (int j0 = 0; j0 < dmax; j0 += 4) {
            int32_t nb[4], lb[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) nb[u] = j0 + u < d ? a.col[rb + j0 + u] : -1;
#pragma unroll
            for (int u = 0; u < 4; ++u) lb[u] = (mine && nb[u] >= 0) ? a.lab[(int64_t)nb[u] * a.ldT + rr] : dl;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint64_t bs = (__ballot(lb[u] != dl) >> (s * LG)) & gmask;
                if (nb[u] >= 0 && rl == 0 && bs)
                    atomicOr((unsigned long long*)&a.aff[(int64_t)bank * a.N + nb[u]], (unsigned long long)bs);
            }
        }
    }
}

// End of a sweep, per replica (cd.hip k_sweep_end without the push / transition modes):
// python-louvain stops a level when the pass gained < min_dq or moved nothing; igraph LPA
// when no visited vertex was unstable.  n_active_out: [0] active after, [1] (k_rl_hand) replicas
// whose filtered list is sparse this sweep, [2..3] u64 moves,
// [4..5] u64 replica-sweeps so far, [6..7] u64 visits of this sweep.
template <bool LOUV>
__global__ void k_rl_sweep_end(RL a, int32_t* n_active_out) {
    __shared__ int cnt, cnt0;
    __shared__ unsigned long long mv, vis;
    if (threadIdx.x == 0) { cnt = 0; cnt0 = 0; mv = 0; vis = 0; }
    __syncthreads();
    for (int r = threadIdx.x; r < a.n_r; r += blockDim.x) {
        unsigned long long f[RF] = {0, 0, 0, 0, 0, 0, 0, 0};
        unsigned long long* base = a.red + (size_t)r * NSH * RF;
        for (int sh = 0; sh < NSH; ++sh)
            for (int q = 0; q < RF; ++q) { f[q] += base[sh * RF + q]; base[sh * RF + q] = 0; }
        a.sacc[4 * r + 0] += f[3]; a.sacc[4 * r + 1] += f[4]; a.sacc[4 * r + 2] += f[5]; a.sacc[4 * r + 3] += f[6];
        atomicAdd(&mv, f[2]);
        atomicAdd(&vis, f[3]);
        if (a.prune) {   // lists filter next sweep iff moves were tracked this sweep
            a.track[a.n_r + r] = a.track[r];
            if (a.lm || f[2] * (unsigned long long)a.track_div < (unsigned long long)a.N) a.track[r] = 1;
        }
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
    if (threadIdx.x == 0) {
        n_active_out[0] = cnt;
        *(unsigned long long*)(n_active_out + 2) = mv;
        *(unsigned long long*)(n_active_out + 4) += (unsigned long long)cnt0;
        *(unsigned long long*)(n_active_out + 6) = vis;
    }
}

inline unsigned nb(int64_t n, int tb) {
    int64_t b = (n + tb - 1) / tb;
    return (unsigned)(b < 1 ? 1 : b);
}

// Hybrid: affected bits per replica at a listed sweep's start (a wave turns its 64 words per bank
// into 64 per-replica counts with one ballot per bit).  Dynamic LDS: banks * 64 ints.
__global__ __launch_bounds__(LTB) void k_rl_aff_count(RL a, int32_t* cnt) {
    extern __shared__ int s_c[];
    for (int k = threadIdx.x; k < a.banks * 64; k += LTB) s_c[k] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    for (int64_t v0 = (int64_t)blockIdx.x * LTB * LPER; v0 < min(a.N, (int64_t)(blockIdx.x + 1) * LTB * LPER); v0 += LTB) {
        const int64_t v = v0 + threadIdx.x;
        for (int b = 0; b < a.banks; ++b) {
            const uint64_t w = v < a.N ? a.aff[(int64_t)b * a.N + v] : 0;
            if (__ballot(w != 0) == 0) continue;                // wave-uniform
            int mine = 0;
#pragma unroll 8
            for (int q = 0; q < 64; ++q) {
                const int c = __popcll(__ballot((w >> q) & 1ull));
                mine = lane == q ? c : mine;
            }
            if (mine) atomicAdd(&s_c[b * 64 + lane], mine);
        }
    }
    __syncthreads();
    for (int r = threadIdx.x; r < a.n_r; r += LTB)
        if (s_c[r]) atomicAdd(cnt + r, s_c[r]);
}
// Hybrid: the replicas whose filtered list is sparse this sweep (any: hand over to cd.hip).
__global__ void k_rl_hand(RL a, int32_t* n_active_out) {
    __shared__ int n;
    if (threadIdx.x == 0) n = 0;
    __syncthreads();
    for (int r = threadIdx.x; r < a.n_r; r += blockDim.x)
        if (rl_sparse(a, r)) atomicAdd(&n, 1);
    __syncthreads();
    if (threadIdx.x == 0) n_active_out[1] = n;
}

// (col << wb) | weight per adjacency entry (WM_W8: one load brings both)
__global__ __launch_bounds__(256) void k_rl_colw(int64_t n, const int32_t* col, const int32_t* cw, int wb, int32_t* out) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j < n) out[j] = (col[j] << wb) | cw[j];
}

// Hybrid hand-off into push mode: nlab[r][j] = the label of neighbour col[j] in replica r, for
// 64 CSR entries x 64 replicas per block through LDS (labT rows read, nlab rows written as
// whole 256-byte runs)
__global__ __launch_bounds__(256) void k_rl_nlab(int64_t m2, int n_r, int ldT, const int32_t* col, const int32_t* labT,
                                                 int32_t* nlab) {
    __shared__ int32_t t[64][65];
    __shared__ int32_t sc[64];
    const int64_t j0 = (int64_t)blockIdx.x * 64;
    const int r0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 64 x 4
    if (ty == 0) sc[tx] = j0 + tx < m2 ? col[j0 + tx] : -1;
    __syncthreads();
    for (int jj = ty; jj < 64; jj += 4) {
        const int32_t u = sc[jj];
        if (u >= 0 && r0 + tx < n_r) t[jj][tx] = labT[(int64_t)u * ldT + r0 + tx];
    }
    __syncthreads();
    for (int rr = ty; rr < 64; rr += 4) {
        const int r = r0 + rr;
        if (r < n_r && j0 + tx < m2) nlab[(int64_t)r * m2 + j0 + tx] = t[tx][rr];
    }
}
__global__ void k_rl_fill_i32(int64_t n, int32_t* p, int32_t v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

// Hybrid hand-off: the affected bits [banks][N] as cd.hip's per-replica bit words [n_r][aw]
// (aw = (N+31)/32; vertex v is bit v & 31 of word v >> 5):
// the bank's 64-bit replica masks per vertex -> cd.hip's per-replica bit words (word v >> 5 of
// replica r, aw words per replica): a wave takes 64 vertices of one bank and turns them, one
// ballot per replica, into that replica's two words
__global__ __launch_bounds__(256) void k_rl_aff_export(int64_t N, int n_r, const uint64_t* aff, int64_t aw, uint32_t* out) {
    const int lane = threadIdx.x & 63;
    const int64_t v0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;
    const int bank = blockIdx.y;
    if (v0 >= N) return;                                        // wave-uniform
    const int64_t v = v0 + lane;
    const uint64_t m = v < N ? aff[(int64_t)bank * N + v] : 0ull;
    uint64_t mine = 0;
#pragma unroll 8
    for (int q = 0; q < 64; ++q) {
        const uint64_t b = __ballot((m >> q) & 1ull);
        mine = lane == q ? b : mine;
    }
    const int r = bank * 64 + lane;
    if (r < n_r) {
        uint32_t* o = out + (int64_t)r * aw + (v0 >> 5);
        o[0] = (uint32_t)mine;
        if ((v0 >> 5) + 1 < aw) o[1] = (uint32_t)(mine >> 32);
    }
}

// CDHandoff::fill: the batch's state in cd.hip's layout (labels in slot order, int32 totals by
// community, affected flags, tracked / filtered flags with pull mode, active flags)
void rl_handoff_fill(Ctx& c, const void* user, int32_t* lab, int32_t* tot, uint32_t* aff, int32_t* track,
                     int32_t* active, int32_t* nlab) {
    const RL& a = *(const RL*)user;
    const dim3 tg(nb(a.N, 64), (a.n_r + 63) / 64);
    k_rl_export<<<tg, 256, 0, c.stream>>>(a.N, a.n_r, a.ldT, a.lab, c.sinv.as<int32_t>(), lab);
    if (tot) k_rl_export<<<tg, 256, 0, c.stream>>>(a.N, a.n_r, a.ldT, a.tot, nullptr, tot);
    k_rl_aff_export<<<dim3(nb(a.N, 256), a.banks), 256, 0, c.stream>>>(a.N, a.n_r, a.aff, (a.N + 31) / 32, aff);
    FC_HIP(hipMemcpyAsync(track, a.track, 8 * (size_t)a.n_r, hipMemcpyDeviceToDevice, c.stream));
    FC_HIP(hipMemsetAsync(track + 2 * a.n_r, 0, 8 * (size_t)a.n_r, c.stream));
    FC_HIP(hipMemcpyAsync(active, a.active, 4 * (size_t)a.n_r, hipMemcpyDeviceToDevice, c.stream));
    // Push from the first filtered sweep on (unit weights, no Leiden-style marks: cd_run's own
    // push rule): a filtered sweep of pull visits gathers one random line per neighbour label
    // (SBM-4M: 14.5x the algorithmic bytes), a push visit streams its row of nlab.  The rows
    // are written here from labT (one coalesced 256-byte label row per CSR entry, read through
    // L2 by its row's other entries).  cd_run never switches a filtering replica to push (its
    // transition sweep must visit every vertex), so without this the hand-off ran pull-only.
    // Measured (MI355X, bench lines): SBM-4M lpm 878 -> 834 ms (LPA's tie revisits keep ~30
    // filtered sweeps of many visits and few moves going); LFR-1M louvain 119.4 -> 126.8 ms (the
    // row fill and the push writes of its movers cost more than the gathers saved).  So LPA only
    // by default (FC_RL_HANDOFF_PUSH: 0 never, 1 LPA, 2 every unit-weight batch).
    const int64_t m2 = 2 * c.g.m;
    const bool lpa = a.tot == nullptr;
    if (c.push_div > 0 && !a.lm && a.unitw && m2 > 0 && (c.rl_handoff_push == 2 || (c.rl_handoff_push == 1 && lpa))) {
        k_rl_nlab<<<dim3(nb(m2, 64), a.banks), 256, 0, c.stream>>>(m2, a.n_r, a.ldT, a.col, a.lab, nlab);
        k_rl_fill_i32<<<nb(a.n_r, 256), 256, 0, c.stream>>>(a.n_r, track + 2 * a.n_r, 1);
    }
}

}  // namespace

// Replica-lane layout of a batch of n_r local replicas: lane group LG (power of two, 8..64),
// vertices per wave 64 / LG, banks of 64 past 64 replicas; label rows of ldT int32.
void rl_layout(int n_r, int* LG, int* VPW, int* banks, int* ldT) {
    int lg = 8;
    while (lg < n_r && lg < 64) lg <<= 1;
    *LG = lg;
    *VPW = 64 / lg;
    *banks = (n_r + 63) / 64;
    *ldT = n_r > 64 ? 64 * *banks : lg;
}

// the graph and options the replica-lane kernels handle (int32 totals, 32-bit row offsets)
static bool cd_rl_fits(const Ctx& c, int algo) {
    // int32 community totals (louvain only: LPA ignores the weights, so a heavily weighted
    // consensus graph -- 2M past 2^31 at SBM-4M, n_p = 128 -- still fits its label propagation);
    // the sweep record (boff | voff | n_active, one pinned DMA per sweep) must fit the pinned
    // scratch: B * NCLS segments, i.e. B <= 339 buckets -- more go to cd.hip (same semantics)
    const int64_t nseg = (int64_t)cd_buckets(c, algo) * NCLS;
    return !c.order_pass && (is_louvain(algo) || algo == FC_ALGO_LPM) && (!is_louvain(algo) || c.g.M2 <= 0x7fffffffll) &&
           c.g.m < (int64_t(1) << 31) && (c.chunk == 0 || c.chunk == RL_CHUNK) &&
           16 + 2 * (nseg + 1) + 2 <= 2 * (int64_t)FC_HPIN_I64;
}
bool cd_rl_supported(const Ctx& c, int algo) { return c.cd_engine == 1 && cd_rl_fits(c, algo); }

// FC_OPT_CD_ENGINE=2.  Semantics (oracle tw_replica shared = 2): a replica's sweeps visit the
// batch's shared order while they are full, and its own order from its first filtered sweep.
// The replica-lane engine runs the full sweeps -- one row walk and one coalesced label read per
// neighbour for every replica of a wave -- and cd.hip runs the rest, where per-replica lists,
// coarse rounds and the tail kernel pay.  A batch too narrow for replica lanes runs on cd.hip
// throughout, with the same semantics (its full sweeps use the shared order too), so results
// never depend on how replicas are sharded over GPUs.
void cd_run_hybrid(Ctx& c, int algo, int rbegin, int rcount, int n_p_total, int iteration) {
    if (cd_rl_fits(c, algo) && (int64_t)rcount >= c.rl_min_replicas && rcount <= RL_MAX_REPLICAS &&
        c.N >= c.rl_min_vertices)
        cd_run_rl(c, algo, rbegin, rcount, n_p_total, iteration, true);
    else
        cd_run(c, algo, rbegin, rcount, n_p_total, iteration, 1);
}

void cd_run_rl(Ctx& c, int algo, int rbegin, int rcount, int n_p_total, int iteration, bool hybrid) {
    FC_REQUIRE(rcount >= 1 && rbegin >= 0 && rbegin + rcount <= n_p_total, FC_EINVAL, "bad replica range");
    FC_REQUIRE(rcount <= RL_MAX_REPLICAS, FC_ELIMIT, "replica-lane engine: more than 16384 replicas per GPU");
    FC_REQUIRE(c.N > 0 && c.g.rowptr.p, FC_ESTATE, "no graph loaded");
    const int sl0 = timer_begin(c);
    const bool louv = is_louvain(algo);
    const int64_t N = c.N;
    Graph& g = c.g;
    c.n_r = rcount; c.rbase = rbegin; c.n_p_total = n_p_total;
    int LG, VPW, banks, ldT;
    rl_layout(rcount, &LG, &VPW, &banks, &ldT);
    const int CH = c.chunk;
    const int64_t NC = CH ? (N + 2 * CH - 2) / CH : N;   // room for the chunk-grid shift (as cd.hip)
    const int B = (int)std::min<int64_t>(cd_buckets(c, algo), NC);
    const int64_t S = CH ? ((NC + B - 1) / B) * CH : (N + B - 1) / B;
    const int64_t PN = CH ? NC * CH : N;

    RL a;
    a.N = N; a.S = S; a.PN = PN; a.chunk = CH; a.perm_n = (uint32_t)NC; a.B = B;
    a.n_r = rcount; a.rbase = rbegin; a.LG = LG; a.VPW = VPW; a.banks = banks; a.ldT = ldT;
    a.lgs = 0;
    while ((1 << a.lgs) < LG) ++a.lgs;
    a.iter = (uint32_t)iteration; a.seed = c.seed;
    a.rowptr = g.rowptr.as<int64_t>(); a.col = g.col.as<int32_t>(); a.cw = g.cw.as<int32_t>();
    a.vrec = g.vrec.as<int4>(); a.kdeg = g.kdeg.as<int64_t>(); a.M2 = g.M2;
    a.unitw = (!louv || (g.max_w == 1 && g.M2 == 2 * g.m)) ? 1 : 0;
    a.wbits = 0;
    while (a.wbits < 31 && ((int64_t)g.max_w >> a.wbits) != 0) ++a.wbits;
    // sortable keys (label << wbits | weight) need N << wbits < 2^31; else the LDS merge
    const bool pack = ((int64_t)(N - 1) << (a.unitw ? 0 : a.wbits)) < (int64_t(1) << 31);
    a.colw = nullptr;
    if (pack && louv && !a.unitw && a.wbits <= 8 && g.m > 0) {
        int32_t* cwp = ensure<int32_t>(c.rl_colw, 2 * (size_t)g.m);
        k_rl_colw<<<nb(2 * g.m, 256), 256, 0, c.stream>>>(2 * g.m, g.col.as<int32_t>(), g.cw.as<int32_t>(), a.wbits, cwp);
        a.colw = cwp;
    }
    a.lab = ensure<int32_t>(c.labT, (size_t)N * ldT);
    a.tot = louv ? ensure<int32_t>(c.rl_tot, (size_t)N * ldT) : nullptr;
    a.dec = ensure<int32_t>(c.dec, (size_t)PN * ldT);
    // slow visits of one bucket: at most its entries (<= S) times the local replicas
    a.slow = ensure<int64_t>(c.rl_slow, (size_t)S * ldT + 1);
    a.slow_cnt = ensure<int32_t>(c.rl_slow_cnt, 4);
    FC_HIP(hipMemsetAsync(a.slow_cnt, 0, 4, c.stream));
    a.list = (int4*)ensure<int4>(c.vlist, (size_t)PN);
    a.lmask = (uint64_t*)ensure<uint64_t>(c.rl_lmask, (size_t)PN * banks);
    a.vmask = (uint64_t*)ensure<uint64_t>(c.rl_vmask, (size_t)N * banks);
    const int nseg = B * NCLS;
    // boff [nseg+1] | voff [nseg+1] | n_active copy [2] | bcnt | cursor | vcnt | vcursor
    int32_t* plan = ensure<int32_t>(c.vcnt, 6 * (size_t)nseg + 16);
    a.boff = plan;
    a.voff = a.boff + nseg + 1;
    int32_t* bcnt = a.voff + nseg + 3;
    a.cursor = bcnt + nseg;
    int32_t* vcnt = a.cursor + nseg;
    a.vcursor = vcnt + nseg;
    FC_REQUIRE(16 + 2 * (nseg + 1) + 2 <= 2 * FC_HPIN_I64, FC_ELIMIT, "too many CD buckets for the pinned sweep record");
    FC_HIP(hipMemsetAsync(bcnt, 0, sizeof(int32_t) * nseg, c.stream));   // kept zero by k_rl_list_plan
    FC_HIP(hipMemsetAsync(vcnt, 0, sizeof(int32_t) * nseg, c.stream));
    a.vlist = nullptr;
    a.aff = (uint64_t*)ensure<uint64_t>(c.rl_aff, (size_t)banks * N);
    a.mvf = (uint64_t*)ensure<uint64_t>(c.rl_mvf, (size_t)banks * N);
    FC_HIP(hipMemsetAsync(a.aff, 0, 8 * (size_t)banks * N, c.stream));
    FC_HIP(hipMemsetAsync(a.mvf, 0, 8 * (size_t)banks * N, c.stream));
    a.prune = c.prune;
    a.track_div = c.track_div;
    // Leiden-style marks (cd.hip): consensus graphs, or every graph with prune_mark = 2
    a.lm = ((g.max_w > 1 || c.prune_mark == 2) && c.prune && c.prune_mark >= 1) ? 1 : 0;
    a.min_dq = c.cd_min_dq;
    a.hybrid = hybrid ? 1 : 0;
    int32_t* acnt = hybrid ? ensure<int32_t>(c.aff_cnt, (size_t)rcount) : nullptr;
    a.acnt = acnt;
    a.dense_div = c.dense_div;
    // per-replica state: active i32 [n_r] | track i32 [2 n_r] | red u64 [n_r][NSH][RF] | sacc u64 [n_r][4] | n_active [8]
    char* rs = (char*)ensure<char>(c.rl_state, (size_t)rcount * (12 + 8 * NSH * RF + 32) + 512);
    a.active = (int32_t*)rs;
    a.track = a.active + rcount;
    a.red = (unsigned long long*)(rs + (((size_t)rcount * 12 + 255) & ~size_t(255)));
    a.sacc = a.red + (size_t)rcount * NSH * RF;
    int32_t* n_active = (int32_t*)(a.sacc + 4 * (size_t)rcount);
    const size_t zero_bytes = (char*)(n_active + 8) - (char*)a.red;
    FC_HIP(hipMemsetAsync(a.track, 0, 8 * (size_t)rcount, c.stream));
    FC_HIP(hipMemsetAsync(a.red, 0, zero_bytes, c.stream));
    {
        std::vector<int32_t> ones(rcount, (g.M2 > 0) ? 1 : 0);
        FC_HIP(hipMemcpyAsync(a.active, ones.data(), sizeof(int32_t) * rcount, hipMemcpyHostToDevice, c.stream));
        sync(c);   // `ones` is pageable host memory
    }
    a.hslots = 1;
    while (a.hslots < 2 * (int64_t)g.max_deg) a.hslots <<= 1;
    a.hscratch = nullptr;
    // global tables (rows past HWSLOTS / 2): one per wave of at most hblocks blocks, <= 1 GiB in all
    int64_t hblocks = HEAVY_GRID;
    if (a.hslots > HWSLOTS) {
        hblocks = std::max<int64_t>(1, std::min<int64_t>(HEAVY_GRID, (int64_t(1) << 30) / ((HTB / 64) * 2 * a.hslots * 4)));
        a.hscratch = ensure<int32_t>(c.heavy_scratch, (size_t)hblocks * (HTB / 64) * 2 * a.hslots);
    }

    k_rl_init<<<nb(N * ldT, 256), 256, 0, c.stream>>>(N, ldT, g.kdeg.as<int64_t>(), a.lab, a.tot);

    int32_t* hb = (int32_t*)(c.hpin + 8);   // boff | voff | n_active[0..1] (pinned: one DMA per sweep)
    int32_t* hinfo = hb + 2 * (nseg + 1);
    const unsigned lgrid = nb(N, LTB * LPER);
    const size_t lcount_lds = sizeof(unsigned long long) * 2 * banks + 2 * sizeof(int) * nseg;
    int sweep = 0, handoff = -1;
    if (c.trace) { sync(c); trace_dt_us(true); }
    for (; sweep < c.max_sweeps && g.M2 > 0; ++sweep) {
        const int listed = (c.prune && sweep > 0) ? 1 : 0;
        if (hybrid && listed) {   // per-replica list sizes: a sparse one hands the batch to cd.hip
            FC_HIP(hipMemsetAsync(acnt, 0, sizeof(int32_t) * (size_t)rcount, c.stream));
            if (a.dense_div) k_rl_aff_count<<<lgrid, LTB, sizeof(int) * 64 * banks, c.stream>>>(a, acnt);
            k_rl_hand<<<1, 256, 0, c.stream>>>(a, n_active);
        }
        k_rl_list_count<<<lgrid, LTB, lcount_lds, c.stream>>>(a, sweep, listed, bcnt, vcnt);
        k_rl_list_plan<<<1, 64, 0, c.stream>>>(nseg, bcnt, a.boff, a.cursor, vcnt, a.voff, a.vcursor, n_active);
        FC_HIP(hipMemcpyAsync(hb, a.boff, sizeof(int32_t) * (2 * (nseg + 1) + 2), hipMemcpyDeviceToHost, c.stream));
        sync(c);
        if (sweep > 0 && hinfo[0] == 0) break;                      // every replica has stopped
        if (hybrid && listed && hinfo[1] > 0) { handoff = sweep; break; }   // a sparse filtered list: cd.hip
        if (hb[nseg] == 0) break;
        k_rl_list_fill<<<lgrid, LTB, 2 * sizeof(int) * nseg, c.stream>>>(a, sweep);
        // visit mode when the replicas of an entry are mostly idle (few visits per listed entry):
        // a wave per entry would run mostly empty lanes
        const int64_t n_ent = hb[nseg], n_vis = hb[2 * nseg + 1];
        const bool vmode = pack && c.rl_visit_div > 0 && n_vis * c.rl_visit_div < n_ent * (int64_t)std::min(rcount, 64);
        if (vmode) {
            a.vlist = ensure<int64_t>(c.rl_vlist, (size_t)n_vis + 1);
            int32_t* nvv = ensure<int32_t>(c.rl_vcount, 2 * (size_t)n_ent + 2);
            k_rl_visits_count<<<nb(n_ent, LTB), LTB, 0, c.stream>>>(a, n_ent, nvv);
            exclusive_scan(c, (const int32_t*)nvv, nvv + n_ent + 1, n_ent);
            k_rl_visits_fill<<<nb(n_ent, LTB), LTB, 0, c.stream>>>(a, n_ent, nvv + n_ent + 1);
        }
        // one unit per wave: rows read as wave-uniform, an item ahead (rl_sorted_u1)
        const bool u1 = VPW == 1 && c.rl_u1;
        // degree classes -> decide launches (sorting-network widths): every class on its own,
        // or neighbouring classes merged into the wider network (fewer, larger launches)
        struct ClsGroup { int c0, c1, K; };
        static const ClsGroup G2[] = {{0, 3, 32}, {3, 5, 64}};   // one unit per wave only (in-kernel widths)
        static const ClsGroup G3[] = {{0, 1, 16}, {1, 3, 32}, {3, 5, 64}};
        static const ClsGroup G4[] = {{0, 1, 16}, {1, 3, 32}, {3, 4, 48}, {4, 5, 64}};
        static const ClsGroup G5[] = {{0, 1, 16}, {1, 2, 24}, {2, 3, 32}, {3, 4, 48}, {4, 5, 64}};
        const int gsel = louv ? c.rl_groups_louv : c.rl_groups_lpa;
        const bool g2 = gsel == 2 && (u1 || (FC_RL_SPLIT & 24) == 24);
        const ClsGroup* groups = g2 ? G2 : gsel <= 3 ? G3 : gsel == 4 ? G4 : G5;
        const int ngroups = g2 ? 2 : gsel <= 3 ? 3 : gsel == 4 ? 4 : 5;
        auto grid_of = [&](int64_t n) {
            const int64_t items = banks == 1 ? (n + VPW - 1) / VPW : n * banks;
            return (unsigned)std::max<int64_t>(1, std::min<int64_t>(items, 8192));
        };
        for (int k = 0; k < B; ++k) {
            const int64_t nb_all = hb[(k + 1) * NCLS] - hb[k * NCLS];
            if (nb_all <= 0) continue;
            // each decide launch timed on its own (span 7: one span per launch, as rocprofv3 counts them)
            if (pack && vmode) {
                for (int gi = 0; gi < ngroups; ++gi) {
                    const int seg = k * NCLS + groups[gi].c0, ns = groups[gi].c1 - groups[gi].c0, KG = groups[gi].K;
                    const int64_t n = hb[nseg + 1 + seg + ns] - hb[nseg + 1 + seg];
                    if (n <= 0) continue;
                    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 63) / 64, 8192));
#define RL_LAUNCH(L, KK, U) do { const int ev = timer_begin(c); k_rl_decide_v<L, KK, U><<<grid, RTB, 0, c.stream>>>(a, seg, ns, sweep); timer_end(c, 7, ev); } while (0)
#define RL_LAUNCH_K(L, U)                                                                            \
    do {                                                                                             \
        if (KG == 16) RL_LAUNCH(L, 16, U); else if (KG == 24) RL_LAUNCH(L, 24, U);                   \
        else if (KG == 32) RL_LAUNCH(L, 32, U); else if (KG == 48) RL_LAUNCH(L, 48, U);              \
        else RL_LAUNCH(L, 64, U);                                                                    \
    } while (0)
                    if (louv && a.unitw) RL_LAUNCH_K(true, WM_UNIT);
                    else if (louv && a.colw) RL_LAUNCH_K(true, WM_W8);
                    else if (louv) RL_LAUNCH_K(true, WM_WIDE);
                    else RL_LAUNCH_K(false, WM_UNIT);
#undef RL_LAUNCH_K
#undef RL_LAUNCH
                }
            } else if (pack) {
                // a bucket's decide launches follow each other with nothing between them: the end
                // event of one is the start event of the next (one event record per launch)
                int chain_ev = -1;
                for (int gi = 0; gi < ngroups; ++gi) {
                    const int seg = k * NCLS + groups[gi].c0, ns = groups[gi].c1 - groups[gi].c0, KG = groups[gi].K;
                    const int64_t n = hb[seg + ns] - hb[seg];
                    if (n <= 0) continue;
                    const int64_t items = banks == 1 ? (n + VPW - 1) / VPW : n * banks;
#define RL_LAUNCH_1(L, KK, U, U1)                                                                                  \
    do {                                                                                                           \
        const unsigned grid = (c.rl_grid_mul > 0 && L)                                                             \
            ? (unsigned)std::max<int64_t>(1, std::min<int64_t>(items, rl_decide_slots<L, KK, U, U1>() * c.rl_grid_mul)) \
            : grid_of(n);                                                                                          \
        const int ev = chain_ev >= 0 ? chain_ev : timer_begin(c);                                                  \
        k_rl_decide<L, KK, U, U1><<<grid, RTB, 0, c.stream>>>(a, seg, ns, sweep);                                  \
        const int ee = timer_end_ev(c, 7, ev);                                                                     \
        if (c.timer_chain) chain_ev = ee;                                                                          \
    } while (0)
#define RL_LAUNCH(L, KK, U) do { if (u1) RL_LAUNCH_1(L, KK, U, true); else RL_LAUNCH_1(L, KK, U, false); } while (0)
#define RL_LAUNCH_K(L, U)                                                                            \
    do {                                                                                             \
        if (KG == 16) RL_LAUNCH(L, 16, U); else if (KG == 24) RL_LAUNCH(L, 24, U);                   \
        else if (KG == 32) RL_LAUNCH(L, 32, U); else if (KG == 48) RL_LAUNCH(L, 48, U);              \
        else RL_LAUNCH(L, 64, U);                                                                    \
    } while (0)
                    if (louv && a.unitw) RL_LAUNCH_K(true, WM_UNIT);
                    else if (louv && a.colw) RL_LAUNCH_K(true, WM_W8);
                    else if (louv) RL_LAUNCH_K(true, WM_WIDE);
                    else RL_LAUNCH_K(false, WM_UNIT);
#undef RL_LAUNCH_K
#undef RL_LAUNCH
#undef RL_LAUNCH_1
                }
            } else {
                const int64_t n = hb[k * NCLS + NCLS - 1] - hb[k * NCLS];
                if (n > 0) {
                    const int ev = timer_begin(c);
                    if (louv) k_rl_decide_lds<true><<<grid_of(n), RTB, 0, c.stream>>>(a, k, sweep);
                    else k_rl_decide_lds<false><<<grid_of(n), RTB, 0, c.stream>>>(a, k, sweep);
                    timer_end(c, 7, ev);
                }
            }
            // exact decisions: the heavy rows (one wave per (entry, replica) visit, HTB / 64 per
            // block) and, louvain, the slow visits the decide launches listed (count on the device:
            // a floor of SLOW_GRID blocks, idle ones return at once)
            {
                const int64_t hv = (int64_t)(hb[(k + 1) * NCLS] - hb[k * NCLS + NCLS - 1]) * rcount;
                const int64_t want = (hv + HTB / 64 - 1) / (HTB / 64) + (louv && pack ? SLOW_GRID : 0);
                const unsigned hgrid = (unsigned)std::min<int64_t>(hblocks, want);
                if (hgrid > 0) {
                    if (louv) k_rl_exact<true><<<hgrid, HTB, 0, c.stream>>>(a, k, sweep);
                    else k_rl_exact<false><<<hgrid, HTB, 0, c.stream>>>(a, k, sweep);
                }
            }
            if (louv) k_rl_apply<true><<<grid_of(nb_all), RTB, 0, c.stream>>>(a, k);
            else k_rl_apply<false><<<grid_of(nb_all), RTB, 0, c.stream>>>(a, k);
        }
        if (a.lm) {
            const int64_t items = banks == 1 ? (N + VPW - 1) / VPW : N * banks;
            k_rl_mark_lm<<<(unsigned)std::min<int64_t>(items, 8192), RTB, 0, c.stream>>>(a);
        }
        if (louv) k_rl_sweep_end<true><<<1, 256, 0, c.stream>>>(a, n_active);
        else k_rl_sweep_end<false><<<1, 256, 0, c.stream>>>(a, n_active);
        if (c.trace) {
            sync(c);
            int32_t st8[8];
            FC_HIP(hipMemcpy(st8, n_active, sizeof(st8), hipMemcpyDeviceToHost));
            fprintf(stderr, "[fc] rl it=%d sweep=%d entries=%d visits=%llu moves=%llu active=%d dt_us=%.0f\n", iteration,
                    sweep, hb[nseg], *(unsigned long long*)(st8 + 6), *(unsigned long long*)(st8 + 2), st8[0],
                    trace_dt_us());
        }
    }
    if (handoff < 0) {
        // labels for the consensus kernels (labT, native) and the slot-order rows everything else reads
        int32_t* lab = ensure<int32_t>(c.lab, (size_t)rcount * N);
        k_rl_export<<<dim3(nb(N, 64), (rcount + 63) / 64), 256, 0, c.stream>>>(N, rcount, ldT, a.lab, c.sinv.as<int32_t>(), lab);
        c.ldT = ldT;
        c.labT_valid = true;
    }
    // statistics: replica-sweeps, visits, and the decide kernel's algorithmic bytes
    std::vector<unsigned long long> sa(4 * (size_t)rcount + 4);
    FC_HIP(hipMemcpyAsync(sa.data(), a.sacc, sa.size() * 8, hipMemcpyDeviceToHost, c.stream));
    sync(c);
    const unsigned long long rep_sweeps = sa[4 * (size_t)rcount + 2];
    unsigned long long vis = 0, ent = 0, cand = 0, units = 0;
    for (int r = 0; r < rcount; ++r) { vis += sa[4 * r]; ent += sa[4 * r + 1]; cand += sa[4 * r + 2]; units += sa[4 * r + 3]; }
    if (c.trace)
        fprintf(stderr, "[fc] rl it=%d done: %d sweeps, %.2f sweeps per replica, %llu visits in %llu units\n", iteration,
                sweep, (double)rep_sweeps / rcount, vis, units);
    // algorithmic bytes of the light decide kernel: per unit (vertex x bank) its record 16 B
    // and row (col 4 B, weight 4 B unless unit) per entry -- read once for every replica of
    // the unit; per visit (vertex x replica) its own label 4 + own total 4 + decision 4, the
    // neighbour labels 4 B per entry, and per Sigma gathered 4 B (louvain)
    const unsigned long long rowb = a.unitw ? 4 : 8;
    const unsigned long long db = louv ? units * 16 + (ent / std::max<unsigned long long>(1, vis)) * units * rowb +
                                             vis * 12 + ent * 4 + cand * 4
                                       : units * 16 + (ent / std::max<unsigned long long>(1, vis)) * units * rowb +
                                             vis * 8 + ent * 4;
    for (fc_stats* s : {&c.acc, &c.prof}) {
        s->cd_sweeps += (int64_t)rep_sweeps;
        s->cd_vertex_visits += (int64_t)vis;
        s->cd_edge_visits += (int64_t)ent;
        s->rl_decide_bytes += (int64_t)db;
    }
    timer_end(c, 0, sl0);
    if (handoff >= 0) {
        if (c.trace) fprintf(stderr, "[fc] rl it=%d hands over to cd.hip at sweep %d\n", iteration, handoff);
        const CDHandoff h{handoff, rl_handoff_fill, &a};
        cd_run(c, algo, rbegin, rcount, n_p_total, iteration, 1, &h);
    }
}

}  // namespace fc
