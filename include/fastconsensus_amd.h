/*
 * fastconsensus_amd.h -- C-ABI of the MI355X-native fast-consensus engine.
 *
 * The reference (ytabatabaee/fastconsensus, fast_consensus.py) is a Python script with
 * no FFI; its hot path is the while-loop of fast_consensus() (fast_consensus.py:129-411)
 * plus the community-detection calls it makes.  Each entry point below replaces a span
 * of that loop; the replaced reference lines are cited per function.  A host binds this
 * with ctypes (see fastconsensus_amd/_lib.py and INTEGRATION.md).
 *
 * Conventions
 *   - Plain pointers + sizes; no torch or HIP types in signatures (streams are void*).
 *   - Node ids are 0..n-1 in NODE ORDER (first appearance, as networkx read_edgelist
 *     orders nodes); the host keeps the label<->id map.
 *   - Every function returns 0 on success, a negative FC_E* code on error; the message
 *     is in fc_last_error() (thread-local).  There is no CPU fallback: without a usable
 *     gfx950 device fc_create fails with FC_ENODEV.
 *   - One context per host thread; a context is bound to one GPU and is not thread-safe.
 *   - Host arrays are caller-owned and copied; device buffers are context-owned, except
 *     buffers passed as `void* dev_*` which the caller owns (e.g. torch tensors used as
 *     RCCL all-reduce buffers).
 */
#ifndef FASTCONSENSUS_AMD_H
#define FASTCONSENSUS_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FC_OK 0
#define FC_EINVAL -1      /* bad argument */
#define FC_ENODEV -2      /* no HIP device / not gfx950 */
#define FC_EHIP -3        /* HIP runtime error */
#define FC_ESTATE -4      /* call out of order (e.g. no graph loaded) */
#define FC_ELIMIT -5      /* a size limit was exceeded */

#define FC_ALGO_LOUVAIN 0 /* fast_consensus.py:141-202 (+ final pass :383-384) */
#define FC_ALGO_LPM 1     /* fast_consensus.py:260-310 (+ final pass :391-392) */
#define FC_ALGO_LOUVAIN_NC 2 /* louvain with new_consensus.py's weight rule (:155-163): an edge of
                                weight w not in {0,n_p} gets the plain co-membership count,
                                others keep w; everything else as FC_ALGO_LOUVAIN */
#define FC_ALGO_LEIDEN 3  /* fast_consensus.py:204-258 (+ final pass :385-388): n_p Leiden runs
                             (leidenalg ModularityVertexPartition, n_iterations=1, :121-123).  On the
                             integer-labelled graphs the CLI reads (:434) the loop's membership
                             lookups are keyed by str(vertex) (:97) and never match an int node
                             (:217), so every consensus weight stays 0, :223-227 removes every
                             edge and check #1 (:229) converges on the empty graph: the result is
                             the final pass on G.  fc_run reports that one iteration (exit 1)
                             without running its discarded CD batch.   */
#define FC_ALGO_INFOMAP 4 /* fast_consensus.py:260-310 with the infomap CD (:267-268, final pass
                             :389-390): the lpm loop (co-membership count, threshold, weight-0
                             closure, check after closure) around igraph community_infomap()
                             (unweighted, trials=10): the two-level map-equation core, best of
                             FC_OPT_INFOMAP_TRIALS runs.   */

typedef struct fc_ctx fc_ctx;

typedef struct fc_stats {
    int32_t iterations;       /* consensus iterations executed (while-loop trips)          */
    int32_t exit_check;       /* 1: louvain check #1 (:172-173); 2: check after closure     */
    int32_t hit_iter_cap;     /* 1 if max_iters stopped the loop (the reference never stops) */
    int32_t n_p;
    int64_t m_final;          /* edges of the graph the final pass ran on                  */
    int64_t partition_edges;  /* sum_iter n_p*m_iter + n_p*m_final                           */
    int64_t cd_sweeps;        /* local-moving / LPA sweeps, summed over replicas            */
    int64_t cd_vertex_visits; /* vertices processed by CD kernels, summed over replicas     */
    int64_t cd_edge_visits;   /* adjacency entries scanned by CD kernels                    */
    double cd_ms;             /* device time per phase (filled when timing is enabled)      */
    double consensus_ms;
    double closure_ms;
    double rebuild_ms;
    double decide_ms;         /* light local-moving kernel (the dominant kernel)            */
    int64_t decide_launches;
    int64_t decide_bytes;     /* algorithmic bytes of those launches */
    /* Leiden / Infomap (leiden.hip): the move/refine decide kernel (k_lv_decide) and the
     * block-per-vertex kernel for long rows (k_lv_heavy), timed per launch like decide_ms;
     * bytes per the model in DESIGN.md (counted on the device) */
    double lv_decide_ms;
    int64_t lv_decide_launches;
    int64_t lv_decide_bytes;
    double lv_heavy_ms;
    int64_t lv_heavy_launches;
    int64_t lv_heavy_bytes;
    /* replica-lane decide kernels (cd_rl.hip k_rl_decide*: the full sweeps of the hybrid,
     * FC_OPT_CD_ENGINE=2, and every sweep at 1); decide_* above covers cd.hip's k_decide_light */
    double rl_decide_ms;
    int64_t rl_decide_launches;
    int64_t rl_decide_bytes;
} fc_stats;

/* ---- lifecycle ---------------------------------------------------------------- */
const char* fc_last_error(void);
const char* fc_version(void);
/* Provenance: the 16-hex hash of the sources, header, compile flags and target the library was
 * compiled from (fastconsensus_amd/build.py source_hash, embedded at compile time). */
const char* fc_build_hash(void);
/* device: HIP ordinal; seed: drives every random choice (CD order/ties, closure). */
int fc_create(int device, uint64_t seed, fc_ctx** out);
void fc_destroy(fc_ctx* ctx);
/* Run all work on an external stream (e.g. torch.cuda.current_stream().cuda_stream).
 * NULL restores the context's own stream. */
int fc_set_stream(fc_ctx* ctx, void* hip_stream);
/* Wait for the context's queued work (device buffers written by the step API are then
 * safe to read from another stream). */
int fc_synchronize(fc_ctx* ctx);
/* 0/1: record HIP events around kernels and fill the *_ms fields of fc_stats. */
int fc_set_timing(fc_ctx* ctx, int enable);
/* Fill *stats with everything accumulated since the last call: the *_ms fields and
 * decide_launches from the recorded HIP events (synchronises the stream) and the CD
 * counters (sweeps, visits, decide_bytes) of every fc_run / fc_cd; then reset both. */
int fc_collect_timing(fc_ctx* ctx, fc_stats* stats);
/* Tunables (0 = default): buckets per sweep, max sweeps per CD run, max iterations. */
int fc_set_params(fc_ctx* ctx, int buckets, int max_sweeps, int max_iters);
#define FC_OPT_BUCKETS 1     /* rounds per CD sweep; 0 (default) = per algorithm: 16 for louvain,
                                louvain_nc and Leiden's level-0 move; 32 for lpm (LPA), Infomap
                                and Leiden's refinement; 4 for Leiden's aggregate-level moves.
                                A value >= 1 applies to all of them.                          */
#define FC_OPT_MAX_SWEEPS 2  /* cap on sweeps per CD run (default 200)                      */
#define FC_OPT_MAX_ITERS 3   /* cap on consensus iterations (default 1000)                  */
#define FC_OPT_CHUNK 4       /* CD visit order granularity: 0 per vertex, 16 (default) chunks */
#define FC_OPT_RELABEL 6     /* 1 (default): engine-internal random vertex numbering (set it
                                before fc_load_graph); results are reported in node order.
                                2: numbered in community order (a one-replica Louvain run at
                                load), for infomap runs, whose union levels gather neighbour
                                state by internal id (louvain / lpm need the random numbering:
                                their visit orders are chunks of consecutive ids).  0: identity */
#define FC_OPT_PRUNE 5       /* 1 (default): once a sweep moves < n/4 vertices, later sweeps visit only vertices with a moved
                                neighbour (GVE-Louvain-style pruning); 0: every vertex       */
#define FC_OPT_TAIL_VISITS 7 /* once no replica visits more than this many vertices in a sweep,
                                the remaining sweeps run in one workgroup per replica (-1, the
                                default: per algorithm, 1024 for Louvain, 4096 for LPA; 0 = off).
                                Same results either way.                                          */
#define FC_OPT_COARSEN 8    /* gmax (default 8; 0 = off): a filtered sweep of V vertices runs its buckets in
                                rounds of g (the largest power of two <= gmax, <= buckets, with V*g <= n),
                                so a small sweep is not 32 latency-bound rounds.  Measured neutral on
                                quality (LFR-100k CD modularity/NMI equal at 0/4/8; LFR-1k consensus NMI
                                0.9035 vs 0.9034 at 0/8) and -18 ms on the LFR-1M run.              */
#define FC_OPT_STORE 9       /* label storage order (set it before fc_load_graph).  1 (default): the
                                replicas' label rows are stored in community order (a one-replica
                                Louvain run at load orders the vertices), so the neighbour-label
                                gathers of a sweep hit nearby lines; 0: internal-id order.  Storage
                                only: results are identical either way.                         */
#define FC_OPT_SEED 10       /* replace the seed fc_create took; everything random after the call
                                (the next fc_load_graph's numbering, CD, closure) follows it     */
#define FC_OPT_CLOSURE_ROUNDS 11  /* triadic closure (:175-190, :292-304) samples from a GROWING graph; the
                                L attempts run in this many consecutive blocks, each drawing from the
                                post-threshold graph plus the earlier blocks' closure edges.  0 (the
                                default): per algorithm -- 4 for louvain / louvain_nc, 16 for lpm and
                                infomap (whose weight-0 closure edges shape the next LPA's topology);
                                1 = every attempt from the post-threshold graph only.             */
#define FC_OPT_PRUNE_MARK 12 /* which neighbours a tracked move marks for the next (filtered) sweep.
                                1 (default): on consensus graphs (weights > 1; Louvain and LPA)
                                tracking starts at sweep 1 and, at each tracked sweep's end, a
                                mover marks only the neighbours whose label differs from its own
                                (fast local moving, Traag et al. 2019); unit-weight graphs keep
                                0.  2: the same marks on every graph (the input graph too).
                                0: every neighbour of a mover, tracking from the first sweep
                                that moves < n/4 vertices.                                       */
#define FC_OPT_INFOMAP_TRIALS 13 /* independent Infomap runs per replica, the smallest codelength kept
                                    (default 10, igraph community_infomap's trials)              */
#define FC_OPT_CD_ENGINE 14  /* louvain / lpm CD batches.  0: the classic engine, a random
                                visit order per replica (FC_OPT_COARSEN / FC_OPT_TAIL_VISITS
                                apply).  1: the replica-lane engine (cd_rl.hip) -- every replica of
                                a batch visits the vertices in ONE shared random order per sweep
                                (ties broken per replica), labels node-major, one wave deciding a
                                vertex for up to 64 replicas; no coarse rounds or tail kernel.
                                2 (default): the hybrid -- a replica's sweeps visit the batch's shared order
                                while they are full and its own order from its first filtered
                                (pruned) sweep on; the replica-lane engine runs the full sweeps of a
                                batch of >= FC_OPT_RL_MIN_REPLICAS replicas, cd.hip everything else.
                                All three are bit-exact against oracle/fc_oracle.c orc_engine_cd
                                (shared = 0 / 1 / 2).                                            */
#define FC_OPT_RL_MIN_REPLICAS 15 /* hybrid: the smallest batch whose full sweeps run on the
                                replica-lane engine (default 8).  Speed only: same results.      */
#define FC_OPT_RL_MIN_VERTICES 16 /* hybrid: ... and the smallest graph (default 262144 vertices;
                                below it cd.hip runs the full sweeps too).  Speed only.          */
#define FC_OPT_DENSE_DIV 17  /* hybrid semantics: a filtered sweep that still visits >= n/dense_div
                                vertices keeps the shared order (single-bucket rounds); default 0
                                = the shared order for full sweeps only (twin: dense_div)        */
int fc_set_option(fc_ctx* ctx, int option, int64_t value);

/* ---- graph (replaces nx.read_edgelist + G.copy() + weight reset, :131-136, :434) ---- */
/* Edge list in input order (ids 0..n-1).  Self loops are dropped, duplicates keep their
 * first occurrence (its position defines the edge's networkx adjacency age); all weights
 * are set to 1 (fast_consensus.py:135-136). */
int fc_load_graph(fc_ctx* ctx, int64_t n, int64_t m, const int32_t* u, const int32_t* v);
int fc_graph_info(fc_ctx* ctx, int64_t* n, int64_t* m, int64_t* m_original);
/* The engine's internal vertex numbering: sigma[node id] = internal id (testing aid). */
int fc_get_node_map(fc_ctx* ctx, int32_t* sigma);
/* graph <- the loaded G (device-to-device; fc_run does this itself, like graph = G.copy()
 * at fast_consensus.py:131).  The step API calls it before a new run. */
int fc_reset_graph(fc_ctx* ctx);
/* Copy the working graph `graph` out: canonical (u<v) sorted by (u,v); any pointer may
 * be NULL. */
int fc_get_graph(fc_ctx* ctx, int32_t* u, int32_t* v, int32_t* w, int64_t* age);

/* Copy out the post-threshold `nextgraph` left by fc_consensus_apply (what the reference
 * passes to check #1, fast_consensus.py:172): canonical, sorted, consensus weights. */
int fc_get_nextgraph(fc_ctx* ctx, int64_t* m, int32_t* u, int32_t* v, int32_t* w, int64_t* age);

/* ---- one-shot driver: fast_consensus(G, algorithm, n_p, thresh, delta) (:129-411) --- */
/* Starts from the loaded G every call (G itself is never modified).  labels_out: [n_p][n] final partitions (community ids renumbered 0..k-1 in node
 * order), may be NULL (then fc_get_labels can fetch them). */
int fc_run(fc_ctx* ctx, int algo, int n_p, double tau, double delta, int32_t* labels_out,
           fc_stats* stats);

/* ---- fine-grained steps (distributed driver; parity tests) ------------------------ */
/* Community detection on the working graph for replicas [replica_begin,
 * replica_begin+replica_count) of n_p_total (:148 / :384 louvain level 0, :270 / :392 LPA,
 * :210-211 / :386-387 Leiden, :268 / :390 Infomap).
 * Randomness depends on (seed, global replica index, iteration), not on the sharding. */
int fc_cd(fc_ctx* ctx, int algo, int replica_begin, int replica_count, int n_p_total,
          int iteration);
/* Replay: install host labelings [count][n] as the local replicas (begin = 0).  Every label
 * must lie in [0, n) (community ids are vertex-sized indices on the device); FC_EINVAL
 * otherwise -- a host with arbitrary ids (1-based, sparse, negative) compacts them first
 * (fastconsensus_amd.Engine.set_labels does). */
int fc_set_labels(fc_ctx* ctx, int count, const int32_t* labels);
/* The local replica range the next fc_get_labels exports: count (n_r), first global index
 * and the run's n_p.  count = 0 before any fc_cd / fc_set_labels. */
int fc_replica_info(fc_ctx* ctx, int* count, int* replica_begin, int* n_p_total);
/* Download local labelings [count][n] (in node order) into host memory or a device buffer of
 * the context's GPU; renumber != 0 -> ids 0..k-1 by first node.  capacity: int32 elements
 * the caller's buffer holds; FC_EINVAL if it is below count * n (nothing is written). */
int fc_get_labels(fc_ctx* ctx, int32_t* labels, int64_t capacity, int renumber);
/* Per-edge partial over the local replicas into caller device buffer dev_out (int32[m]):
 * louvain -> largest global replica index whose labels split the edge, or -1
 * (reduce with MAX); lpm and louvain_nc -> number of local replicas co-clustering it
 * (reduce with SUM). */
int fc_consensus_partial(fc_ctx* ctx, int algo, void* dev_out);
/* Apply the reduced partial: consensus weight rule (:150-159 / :273-280), threshold
 * (:163-168 / :284-288) and, for louvain, check #1 (:172).  kept_out/unconv_out: counts. */
int fc_consensus_apply(fc_ctx* ctx, int algo, int n_p, double tau, double delta,
                       const void* dev_partial, int* converged, int64_t* kept_out,
                       int64_t* unconverged_out);
/* Closure candidates: L attempts drawn on the device (:175-184 / :292-300), or recorded
 * pairs (replay, int32[npairs][2]).  n_cand: new distinct absent edges. */
int fc_closure_sample(fc_ctx* ctx, int64_t attempts, int iteration, int64_t* n_cand);
int fc_closure_set_pairs(fc_ctx* ctx, int64_t npairs, const int32_t* pairs, int iteration,
                         int64_t* n_cand);
/* The same device closure (fast_consensus.py:175-184 / :292-300, the growing nextgraph) with
 * each block's attempts split over ranks (multi-GPU: no rank draws all L attempts).
 * fc_closure_begin returns the block count; block b covers attempts
 * [L*b/blocks, L*(b+1)/blocks).  For b = 0, 1, ... in order: every rank draws its sub-range
 * [t_lo, t_hi) with fc_closure_block_sample -> `count` int64 (key, first attempt) pairs in
 * dev_out (FC_EINVAL if more than `capacity`); the ranks' lists are concatenated (any order)
 * and handed to fc_closure_block_add on every rank.  fc_closure_finish then leaves exactly
 * the candidates fc_closure_sample(L) gives, on every rank. */
int fc_closure_begin(fc_ctx* ctx, int64_t attempts, int iteration, int* blocks);
int fc_closure_block_sample(fc_ctx* ctx, int block, int64_t t_lo, int64_t t_hi, void* dev_out,
                            int64_t capacity, int64_t* count);
int fc_closure_block_add(fc_ctx* ctx, int block, const void* dev_in, int64_t count);
int fc_closure_finish(fc_ctx* ctx, int64_t* n_cand);
/* Per-candidate count of local replicas co-clustering it into dev_out (int32[n_cand]). */
int fc_closure_partial(fc_ctx* ctx, void* dev_out);
/* Add closure edges (louvain weight = reduced count (:186-190); lpm weight 0 (:302-304)),
 * isolate repair for louvain (:193-195), swap graph <- nextgraph (:198 / :307) and run
 * the check (:201 / :309). dev_counts may be NULL for lpm. */
int fc_closure_apply(fc_ctx* ctx, int algo, int n_p, double delta, const void* dev_counts,
                     int iteration, int* converged, int64_t* m_out);

/* ---- synthetic inputs for benchmarks (host C++, not on the hot path) ---------------- */
/* LFR-like benchmark graph (power-law degrees tau1, community sizes tau2, mixing mu).
 * Writes at most m_cap edges into u/v and the planted community of every node. */
int fc_generate_lfr(int64_t n, double tau1, double tau2, double mu, double avg_deg,
                    int32_t max_deg, int32_t min_comm, int32_t max_comm, uint64_t seed,
                    int64_t m_cap, int32_t* u, int32_t* v, int64_t* m_out, int32_t* planted);
/* Planted-partition SBM: n/block_size blocks, expected internal/external degree. */
int fc_generate_sbm(int64_t n, int32_t block_size, double deg_in, double deg_out,
                    uint64_t seed, int64_t m_cap, int32_t* u, int32_t* v, int64_t* m_out);
/* Edge-list text parser (2+ whitespace-separated int columns; extra columns ignored).
 * Returns labels in node order (first appearance) and edges as ids. Two-phase: call with
 * NULL outputs to get sizes. */
int fc_read_edgelist(const char* path, int64_t* n_out, int64_t* m_out, int64_t* labels,
                     int32_t* u, int32_t* v);

#ifdef __cplusplus
}
#endif
#endif /* FASTCONSENSUS_AMD_H */
