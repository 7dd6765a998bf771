// fc_ctx.h -- engine context: device-resident graph, replica state and scratch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <chrono>
#include <string>
#include <vector>

#include "../../include/fastconsensus_amd.h"

namespace fc {

// FC_TRACE: microseconds since the previous trace mark -- one clock shared by every engine
// (cd.hip, cd_rl.hip, leiden.hip), so a line's dt is the work since the line before it;
// reset = true marks a batch start (returns 0)
inline double trace_dt_us(bool reset = false) {
    static std::chrono::steady_clock::time_point last = std::chrono::steady_clock::now();
    const auto now = std::chrono::steady_clock::now();
    const double dt = 1e-3 * (double)std::chrono::duration_cast<std::chrono::nanoseconds>(now - last).count();
    last = now;
    return reset ? 0.0 : dt;
}

void set_error(const std::string& msg);

// Louvain community detection + louvain consensus loop (closure counts, isolate repair,
// check #1): FC_ALGO_LOUVAIN and its new_consensus.py weight-rule variant.
inline bool is_louvain(int algo) { return algo == FC_ALGO_LOUVAIN || algo == FC_ALGO_LOUVAIN_NC; }

struct FcError {
    int code;
    std::string msg;
};

#define FC_HIP(call)                                                                       \
    do {                                                                                   \
        hipError_t _e = (call);                                                            \
        if (_e != hipSuccess) {                                                            \
            (void)hipGetLastError(); /* clear it: library calls (hipcub) re-check it later */ \
            throw ::fc::FcError{FC_EHIP, std::string(#call) + ": " + hipGetErrorString(_e)}; \
        }                                                                                  \
    } while (0)
#define FC_REQUIRE(cond, code, msg)                      \
    do {                                                 \
        if (!(cond)) throw ::fc::FcError{(code), (msg)}; \
    } while (0)

// Growable device buffer (never shrinks; grows by 1.5x).
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    template <class T> T* as() const { return static_cast<T*>(p); }
    void ensure(size_t need) {
        if (need <= bytes) return;
        size_t nb = bytes ? bytes + bytes / 2 : 0;
        if (nb < need) nb = need;
        nb = (nb + 255) & ~size_t(255);
        if (p) {
            FC_HIP(hipDeviceSynchronize());  // queued kernels may still use the old buffer
            FC_HIP(hipFree(p));
        }
        p = nullptr;
        FC_HIP(hipMalloc(&p, nb));
        bytes = nb;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

// Canonical edge list (u < v in node order, sorted by (u,v)) + symmetric CSR with
// every row sorted ascending.
struct Graph {
    int64_t m = 0;
    DevBuf eu, ev, ew, eage;        // int32, int32, int32, int64  [m]
    DevBuf rowptr, col, cw, ceid;   // int64 [N+1], int32 [2m] x3
    DevBuf crev;                    // int32 [2m]: index of the reverse entry (v->u for u->v)
    DevBuf colp;                    // int32 [2m]: storage slot (Ctx::spos) of col[j]: label gathers
    DevBuf vrec;                    // int4 [N]: row start (m < 2^31), degree, k_v (valid when 2M < 2^31), slot
    DevBuf kdeg;                    // int64 [N] weighted degree
    int64_t M2 = 0;                 // sum of kdeg = 2 * total weight
    int32_t max_deg = 0;
    int64_t max_kdeg = 0;
    int32_t max_w = 0;              // largest edge weight (unit-weight graphs skip the weight loads)
    void release() {
        DevBuf* b[] = {&eu, &ev, &ew, &eage, &rowptr, &col, &cw, &ceid, &crev, &colp, &vrec, &kdeg};
        for (auto* x : b) x->release();
    }
};

struct Timer {
    bool on = false;
    std::vector<hipEvent_t> pool;
    // cd, consensus, closure, rebuild, decide, lv decide, lv heavy, rl decide
    std::vector<std::pair<int, int>> spans[8];
    size_t next = 0;
};

struct Ctx {
    int device = 0;
    uint64_t seed = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    int64_t N = 0, m_original = 0;
    // internal vertex numbering: internal = sigma[node], node = npos[internal] (a seeded
    // random permutation, or the identity): engine behaviour is independent of input order
    DevBuf sigma, npos;             // int32 [N]
    // label storage maps (int32 [N], slot_maps()): sinv slot -> internal vertex, tpos node
    // position -> slot, snpos slot -> node position; label-row passes walk rows in slot order
    DevBuf sinv, tpos, snpos;
    std::vector<int32_t> h_sigma;
    DevBuf st_u, st_v, st_w, st_age, st_lab;   // host-facing staging (node space)
    int key_bits = 1;               // bits to hold a node id (N <= 2^key_bits)
    Graph g;                        // `graph` (fast_consensus.py:131)
    Graph g0;                       // pristine G as loaded (never modified, like the caller's G)
    // replica state (replica-major [n_r][N])
    int n_r = 0, rbase = 0, n_p_total = 0;
    DevBuf lab, tot, dec, labT;     // int32 [n_r][N], int64 [n_r][N], int32 [n_r][S], int32 [N][ldT]
    DevBuf nlab;                    // int32 [n_r][2m]: label of each adjacency entry's neighbour
    DevBuf aff, vlist, vcnt, track; // pruning: affected flags, per-sweep visit lists, list lengths, modes
    DevBuf mvf;                     // movers of a tracked sweep (prune_mark = 1 on weighted Louvain graphs)
    DevBuf aff_cnt;                 // hybrid: per-replica affected-flag counts at a sweep's start
    // replica-lane engine (cd_rl.hip): per-entry replica masks, list-build scratch, affected /
    // mover bits [banks][N]; labels and totals node-major in labT / tot ([N][ldT])
    DevBuf rl_lmask, rl_vmask, rl_aff, rl_mvf, rl_vlist, rl_vcount;
    // visit mode for sparse sweeps: when visits * rl_visit_div < entries * min(n_r, 64) (0: never)
    int rl_visit_div = getenv("FC_RL_VISIT_DIV") ? atoi(getenv("FC_RL_VISIT_DIV")) : 4;
    // hybrid hand-off into push mode: 0 never, 1 LPA batches (default), 2 every unit-weight batch
    int rl_handoff_push = getenv("FC_RL_HANDOFF_PUSH") ? atoi(getenv("FC_RL_HANDOFF_PUSH")) : 1;
    int cd_engine = 2;              // FC_OPT_CD_ENGINE: 0 classic (cd.hip), 1 replica-lane (cd_rl.hip), 2 hybrid (default)
    // hybrid: the replica-lane engine runs a batch's full sweeps only when it holds this many
    // replicas (8 lanes per vertex at 8: LFR-1M n_p = 8 run 40.3 vs 42.9 ms on cd.hip since the
    // 16-bucket / resident-grid changes; 51.3 vs 46.2 before them)
    int64_t rl_min_replicas = getenv("FC_RL_MIN_REPLICAS") ? atoll(getenv("FC_RL_MIN_REPLICAS")) : 8;
    // ... and the graph this many vertices (a bucket of a smaller graph is too few waves for the
    // replica-lane kernels: LFR-100k louvain 45.9 vs 31.2 ms, LFR-1M 175.8 vs 211 ms; at the
    // round-4 end LFR-100k louvain 33.0 vs 26.5, lpm 24.2 vs 16.6 ms)
    int64_t rl_min_vertices = getenv("FC_RL_MIN_VERTICES") ? atoll(getenv("FC_RL_MIN_VERTICES")) : 262144;
    // hybrid semantics: a filtered sweep visiting >= N/dense_div vertices keeps the shared order
    // (without coarse rounds); 0 = never (FC_OPT_DENSE_DIV).  Measured no gain: LFR-1M 175.9 /
    // 177.7 / 176.7 ms at 0 / 2 / 4, SBM-4M 712 / 759 / 722 ms (profiles/r04_dense_ab.txt)
    int dense_div = 0;
    DevBuf rl_tot, rl_state;        // replica-lane totals [N][ldT] and per-replica state (kept apart from cd.hip's)
    DevBuf rl_colw;                 // replica-lane: (col << wbits) | weight per adjacency entry (weights < 256)
    DevBuf rl_slow, rl_slow_cnt;    // replica-lane: one bucket's visits left to the exact kernel
    int ldT = 0;
    bool labT_valid = false;
    DevBuf rep_state;               // per replica: active flag, dq accum, moves, unstable
    DevBuf heavy_list, heavy_cnt, heavy_scratch;
    // consensus / kept graph
    DevBuf wnew, flag, pos;         // int32 [m] (flag/pos also reused for 2m CSR compaction)
    int64_t kept_m = 0;
    DevBuf ku, kv, kw, kage;        // kept canonical list
    DevBuf krowptr, kcol;           // kept CSR (sorted rows)
    DevBuf counters;                // int64 scratch counters
    DevBuf hcounters;               // (pinned host) mirror
    // closure / repair / merge
    int64_t n_cand = 0;
    DevBuf ckey, cval, ckey2, cval2;  // uint64 keys + int64 sample index
    DevBuf cu, cv, cw2, cage;       // closure edges
    DevBuf deg_next, iso, isoflag, target, tw, active, active2, hit;
    int64_t n_iso = 0;
    DevBuf mkey, mkey2, midx, midx2;  // merge sort
    // closure over closure_rounds blocks of attempts (closure_sample): candidate table (uint64
    // key, u64 first attempt), listed slots and their count, accumulated candidates (key,
    // first attempt), the C graph of the earlier blocks' closure edges (CSR rowptr int64
    // [N+1] / col int32, ping-pong), a block's new entries (int32 row offsets + cursors, cols)
    DevBuf clo_rec;                 // closure: per node {kept row start, length, C row start, length}
    // closure sampler reads the packed node records (0: krowptr / crowptr, the path of graphs past
    // 2^31 entries; FC_CLO_PACK=0 lets the tests run it at small sizes)
    int clo_pack = getenv("FC_CLO_PACK") ? atoi(getenv("FC_CLO_PACK")) : 1;
    DevBuf clo_hkey, clo_hval, clo_list, clo_cnt, clo_akey, clo_aval, clo_rowptr, clo_col, clo_rowptr2, clo_col2,
        clo_nrow, clo_ncol, clo_own, clo_own2;
    int closure_rounds = 0;         // FC_OPT_CLOSURE_ROUNDS; 0 = per algorithm (closure_blocks below)
    int clo_algo = 0;               // algorithm of the last consensus_apply (the kept graph the closure samples)
    // sharded closure (fc_closure_begin / _block_sample / _block_add / _finish): the run's
    // attempts and block count, the next block to add (blocks go in order), -1 = not begun
    int64_t clo_attempts = 0;
    int clo_R = 0, clo_next = -1, clo_iter = 0;
    int prune_mark = 1;             // FC_OPT_PRUNE_MARK: 1 Leiden-style marks on consensus graphs, 2 on every graph, 0 every neighbour
    DevBuf sort_tmp;                // hipcub temporary storage
    DevBuf nodetmp, nodetmp2, nodetmp3;  // int64 [N+1] scratch
    DevBuf part, ccount;            // consensus partial / closure counts (single-GPU driver)
    // params
    int buckets = 0, max_sweeps = 200, max_iters = 1000;   // buckets 0: cd_buckets' default per algorithm
    int chunk = 16;                 // CD order granularity (0 = per vertex), FC_OPT_CHUNK
    int relabel = 1;                // FC_OPT_RELABEL (applies at the next fc_load_graph)
    int64_t apply_blocks = getenv("FC_APPLY_BLOCKS") ? atoll(getenv("FC_APPLY_BLOCKS")) : 32;   // per replica
    std::vector<hipEvent_t> sweep_ev;   // per-sweep completion ring (cd_run)
    DevBuf tailbuf, tailmark;       // CD tail kernel: worklists [n_r][3N], epoch marks [n_r][N]
    // per replica; 0 = off; -1 (default) = per algorithm: 1024 for Louvain (n_p = 8 share 45.5 ->
    // 44.4 ms against 4096), 4096 for LPA (C3 lpm 24.1 -> 22.2 ms against 1024; profiles/r05_tail_ab.txt)
    int64_t tail_visits = getenv("FC_TAIL_VISITS") ? atoll(getenv("FC_TAIL_VISITS")) : -1;
    bool order_pass = false;        // store_order()'s CD run (int64 totals, see there)
    int store_order = 1;            // FC_OPT_STORE: label rows in community order (slot spos[v])
    int order_sweeps = getenv("FC_ORDER_SWEEPS") ? atoi(getenv("FC_ORDER_SWEEPS")) : 3;   // sweeps of that pass (4 until round 6: LFR-1M load -0.37 ms at 3, same run time)
    // its buckets per sweep: the pass only permutes label storage (results are identical), and
    // 4 big launches per sweep beat 32 small ones (LFR-1M load 9.9 -> 8.0 ms, tools/r03_ordb.sh)
    int order_buckets = getenv("FC_ORDER_BUCKETS") ? atoi(getenv("FC_ORDER_BUCKETS")) : 4;
    DevBuf spos;                    // int32 [N]: storage slot of internal vertex v in every lab row
    int coarsen = 8;                // FC_OPT_COARSEN: 0 off, else the largest g (filtered sweeps in rounds of g buckets)
    double cd_min_dq = 1e-7;        // Louvain sweeps stop below this predicted gain (Leiden's move phase: 0)
    DevBuf lv[64];                  // Leiden level state (leiden.hip)
    int infomap_trials = 10;        // FC_OPT_INFOMAP_TRIALS (igraph community_infomap default)
    int lv_dense_div = getenv("FC_LV_DENSE_DIV") ? atoi(getenv("FC_LV_DENSE_DIV")) : 0;   // leiden.hip level buckets
    // leiden.hip aggregate levels: buckets per move sweep (0: B, the level-0 count)
    int lv_level_b = getenv("FC_LV_LEVEL_B") ? atoi(getenv("FC_LV_LEVEL_B")) : 4;
    // cd_rl.hip Louvain decide grid: resident waves x rl_grid_mul (0: up to 8192 blocks, as LPA)
    int rl_grid_mul = getenv("FC_RL_GRID_MUL") ? atoi(getenv("FC_RL_GRID_MUL")) : 1;
    int prune = 1;                  // FC_OPT_PRUNE: visit only vertices whose neighbour moved (once moves < N/4)
    // CD kernel variant that leaves every decision unchanged (A/B switch, default on):
    // own-label entries summed in registers (ballots / wave scan) instead of the LDS table
    int own_ballot = getenv("FC_OWN_BALLOT") ? atoi(getenv("FC_OWN_BALLOT")) : 1;
    // sweep-mode thresholds (experiment switches): tracking/pruning after a sweep moving
    // < N/track_div vertices, pull -> push after < N/push_div (0: stay in pull mode)
    int track_div = getenv("FC_TRACK_DIV") ? atoi(getenv("FC_TRACK_DIV")) : 4;
    int push_div = getenv("FC_PUSH_DIV") ? atoi(getenv("FC_PUSH_DIV")) : 4;
    bool trace = getenv("FC_TRACE") && *getenv("FC_TRACE") && *getenv("FC_TRACE") != '0';  // per-sweep stderr
    Timer timer;
    fc_stats acc{};                 // accumulated during a run (fc_run)
    fc_stats prof{};                // accumulated since the last fc_collect_timing
    int64_t* hpin = nullptr;        // pinned host scratch (FC_HPIN_I64 int64)
    // cd_rl.hip decide with one unit per wave (64 local replicas or more): the row as one
    // coalesced load an item ahead, neighbour ids by readlane (A/B switch; same decisions)
    int rl_u1 = getenv("FC_RL_U1") ? atoi(getenv("FC_RL_U1")) : 1;
    // timed decide launches of one bucket share their boundary events (FC_TIMER_CHAIN=0: two each)
    int timer_chain = getenv("FC_TIMER_CHAIN") ? atoi(getenv("FC_TIMER_CHAIN")) : 1;
    // replica-lane decide launches per bucket: 3 (networks of 16 / 32 / 64 keys), 4 (+48) or 5
    // (+24 and 48) -- per algorithm (cd_rl.hip, degree classes); 2: one launch for the rows of
    // <= 32 and one for 33..64, the one-unit-per-wave kernels picking the network per row
    // (FC_RL_SPLIT; other layouts run 3)
    int rl_groups_louv = getenv("FC_RL_GROUPS_LOUV") ? atoi(getenv("FC_RL_GROUPS_LOUV")) : 2;
    int rl_groups_lpa = getenv("FC_RL_GROUPS_LPA") ? atoi(getenv("FC_RL_GROUPS_LPA")) : 2;
};

struct Ctx;
constexpr int FC_HPIN_I64 = 2048;   // pinned host scratch: per-sweep records (cd_rl.hip: boff | voff | n_active)
// State the replica-lane engine hands to cd_run at the first filtered sweep of a hybrid batch
// (FC_OPT_CD_ENGINE=2, cd_rl.hip): fill() writes it in cd.hip's layout on c.stream -- labels
// [n_r][N] in slot order, int32 totals [n_r][N], affected flags as bit words uint32
// [n_r][aw] (aw = (N+31)/32 words per replica; vertex v is bit v & 31 of word v >> 5), track int32
// [4][n_r] (tracked, filtered, push, transition) and active [n_r] -- and the sweeps go on from
// sweep0.  On unit-weight graphs without Leiden-style marks it also writes every neighbour-label
// row nlab [n_r][2m] and starts the replicas in push mode (cd.hip streams the rows instead of
// gathering labels).
struct CDHandoff {
    int sweep0;
    void (*fill)(Ctx& c, const void* user, int32_t* lab, int32_t* tot, uint32_t* aff, int32_t* track, int32_t* active,
                 int32_t* nlab);
    const void* user;
};

// CD buckets per sweep: FC_OPT_BUCKETS when set, else 16 for Louvain (louvain, louvain_nc and
// Leiden's level-0 move phase) and 32 for LPA.  16 buckets (twice the simultaneous deciders)
// cut LFR-1M louvain from 149 to 121 ms with the CPU model's consensus NMI within the reference
// loop's spread (0.912 vs 0.917, reference 0.905 +- 0.035); LPA keeps 32: at its detectability
// edge its bucketed batches must stay within 0.25 of sequential LPA's structured fraction
// (tests/test_gpu_cd_parity.py), and 16 buckets measured 0.28 off (profiles/r04_buckets_ab.txt)
constexpr int CD_BUCKETS_LOUVAIN = 16, CD_BUCKETS_LPA = 32;
// Closure blocks per algorithm (DESIGN, "Triadic closure"): the reference's sampler sees every
// earlier attempt's edge; a block sees only the earlier blocks'.  Louvain's closure edges carry
// co-membership weights and 4 blocks keep its consensus at or above the reference loop's
// (C2 / C3 gates); lpm's (and infomap's) weight-0 closure edges are topology for the next LPA,
// and 4 blocks (+1.7 % candidates vs sequential on the sparse C3 graph) cost 0.0008 consensus
// NMI there -- 16 blocks (+0.5 %) match the reference loop (tools/lpm_ablate.py).
constexpr int CLOSURE_ROUNDS_LOUVAIN = 4, CLOSURE_ROUNDS_LPM = 16;
inline int closure_blocks(const Ctx& c) {
    return c.closure_rounds > 0 ? c.closure_rounds
                                : (is_louvain(c.clo_algo) ? CLOSURE_ROUNDS_LOUVAIN : CLOSURE_ROUNDS_LPM);
}
inline int cd_buckets(const Ctx& c, int algo) {
    return c.buckets > 0 ? c.buckets : (is_louvain(algo) ? CD_BUCKETS_LOUVAIN : CD_BUCKETS_LPA);
}

// graph.cpp
void graph_load(Ctx& c, int64_t n, int64_t m, const int32_t* u, const int32_t* v);
void graph_build_csr(Ctx& c, Graph& g);
void graph_merge_next(Ctx& c, int64_t n_added);
void graph_copy(Ctx& c, Graph& dst, const Graph& src);
// cd.cpp
// shared_full: full sweeps in the batch's shared order (the hybrid's semantics); h: resume a
// hybrid batch handed over by the replica-lane engine
void cd_run(Ctx& c, int algo, int rbegin, int rcount, int n_p_total, int iteration, int shared_full = 0,
            const CDHandoff* h = nullptr);
// cd_rl.hip: the replica-lane engine (louvain / lpm batches when cd_rl_supported)
bool cd_rl_supported(const Ctx& c, int algo);
void cd_run_rl(Ctx& c, int algo, int rbegin, int rcount, int n_p_total, int iteration, bool hybrid = false);
// FC_OPT_CD_ENGINE=2: full sweeps in one shared order (on the replica-lane engine when the batch
// holds >= rl_min_replicas and the graph fits it), filtered sweeps on cd.hip in per-replica orders
void cd_run_hybrid(Ctx& c, int algo, int rbegin, int rcount, int n_p_total, int iteration);
void store_order(Ctx& c);             // Ctx::spos from a one-replica Louvain run (FC_OPT_STORE)
void slot_maps(Ctx& c);               // Ctx::sinv / tpos / snpos from spos
void graph_slots(Ctx& c, Graph& g);   // g.colp = spos[g.col]
void labels_transpose(Ctx& c);
void labels_to_host(Ctx& c, int32_t* out, bool renumber);   // node order [n_r][N]
void labels_from_host(Ctx& c, int count, const int32_t* in);
void graph_to_host(Ctx& c, int64_t m, const int32_t* u, const int32_t* v, const int32_t* w, const int64_t* age,
                   int32_t* ou, int32_t* ov, int32_t* ow, int64_t* oage);
// leiden.hip: replica-batched Leiden (leidenalg ModularityVertexPartition, n_iterations=1)
void leiden_run(Ctx& c, int rbegin, int rcount, int n_p_total, int iteration);
// igraph Infomap core (two-level map equation, best of `trials`), same layout
void infomap_run(Ctx& c, int rbegin, int rcount, int n_p_total, int iteration);
// consensus.cpp
void consensus_partial(Ctx& c, int algo, int32_t* out);
void consensus_apply(Ctx& c, int algo, int n_p, double tau, const int32_t* partial, int64_t* kept,
                     int64_t* unconv);
void closure_sample(Ctx& c, int64_t attempts, int iteration);
int closure_begin(Ctx& c, int64_t attempts, int iteration);
int64_t closure_block_sample(Ctx& c, int block, int64_t t_lo, int64_t t_hi, int64_t* out, int64_t capacity);
void closure_block_add(Ctx& c, int block, const int64_t* in, int64_t count);
int64_t closure_finish(Ctx& c);
void closure_from_pairs(Ctx& c, int64_t npairs, const int32_t* pairs, int iteration);
void closure_partial(Ctx& c, int32_t* out);
void closure_apply(Ctx& c, int algo, int n_p, const int32_t* counts, int iteration);
int64_t count_unconverged(Ctx& c, const int32_t* w, int64_t m, int n_p);
// timing helpers
int timer_begin(Ctx& c);
void timer_end(Ctx& c, int slot, int begin_ev);
int timer_end_ev(Ctx& c, int slot, int begin_ev);   // timer_end, returning the end event (-1: off)
void timer_collect(Ctx& c, fc_stats* st);
// scratch helpers
template <class T> inline T* ensure(DevBuf& b, size_t count) {
    b.ensure(count * sizeof(T) + 16);
    return b.as<T>();
}
void sync(Ctx& c);
// zero / fold sharded counters (CSH x F u64 in c.counters); max_mask bit f: max instead of sum
unsigned long long* shards_begin(Ctx& c, int F);
void shards_fold(Ctx& c, int F, unsigned max_mask, int64_t* host_out);
int64_t read_i64(Ctx& c, const int64_t* dev);

constexpr int64_t AGE_ITER_SHIFT = 40;
constexpr int64_t AGE_REPAIR_OFFSET = int64_t(1) << 39;

}  // namespace fc
