// gdist_internal.hpp — shared host/device definitions of libgdist.so.
//
// Everything here is gfx950 (MI355X) only: 64-lane waves, 160 KiB LDS per CU,
// 8 XCDs of 32 CUs. No CUDA compatibility layer, no dual paths.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <climits>
#include <functional>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/gdist.h"

namespace gdist {

// ---------------------------------------------------------------------------
// errors: every C-ABI entry point converts an Error into its status code and
// stores the message in a thread-local string (gdist_last_error()).
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string& msg);

#define GD_HIP(x)                                                                        \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess)                                                            \
            throw ::gdist::Error(e_ == hipErrorOutOfMemory ? GDIST_ENOMEM : GDIST_EDEVICE, \
                                 std::string(#x) + ": " + hipGetErrorString(e_));       \
    } while (0)

#define GD_REQUIRE(cond, msg)                                                            \
    do {                                                                                 \
        if (!(cond)) throw ::gdist::Error(GDIST_EINVAL, msg);                            \
    } while (0)

// ---------------------------------------------------------------------------
// device buffers.
//
// Blocks come from a per-device caching allocator: a released block goes
// back to a free list keyed by its size class once its stream has drained,
// and later requests of that class reuse it without calling hipMalloc. On
// gfx950 / ROCm 7.2 a large hipMalloc that misses the runtime's reuse can
// stall for seconds (a fresh 16 GiB block: 3 s, scripts/diag/alloc_churn.py),
// which made the chunked setup paths (pack, dictionary, bitsets) spend 90 % of
// their time allocating. Reuse only after the owning stream has drained is
// the same ordering guarantee hipFree gives (the stream-ordered pool,
// hipMallocAsync/hipFreeAsync, was intermittently unsafe here: DESIGN.md §8).
void* cache_alloc(int device, size_t bytes, size_t* cls_out);
void cache_free(int device, void* p, size_t cls);
void cache_trim(int device);     // hipFree every cached block of the device
// fresh hipMallocs of the caching allocator (count, bytes, wall ms) and cache
// trims: the trace prints them at the end of a build
struct AllocStats {
    int64_t fresh = 0, trims = 0;
    double fresh_bytes = 0, fresh_ms = 0;
};
AllocStats& alloc_stats();

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    size_t cls = 0;               // size class actually held
    int device = 0;
    hipStream_t stream = nullptr;
    DevBuf() = default;
    DevBuf(size_t n, hipStream_t s) { alloc(n, s); }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept { *this = std::move(o); }
    DevBuf& operator=(DevBuf&& o) noexcept {
        release();
        p = o.p; bytes = o.bytes; cls = o.cls; device = o.device; stream = o.stream;
        o.p = nullptr; o.bytes = 0; o.cls = 0;
        return *this;
    }
    ~DevBuf() { release(); }
    void alloc(size_t n, hipStream_t s) {
        release();
        stream = s;
        bytes = n;
        if (n) {
            GD_HIP(hipGetDevice(&device));
            p = cache_alloc(device, n, &cls);
        }
    }
    void release() noexcept {
        if (p) {
            (void)hipStreamSynchronize(stream);
            cache_free(device, p, cls);
        }
        p = nullptr;
        bytes = 0;
        cls = 0;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

// Host <-> device copies are host-blocking and ordered on the stream: the
// stream is drained, then a synchronous copy. Pageable-source
// hipMemcpyAsync was observed (ROCm 7.2, gfx950) to let the next kernel on
// the stream read partly stale bytes, and its host buffer may die before a
// deferred copy runs; every host<->device transfer goes through these two.
inline void h2d(void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (!bytes) return;
    GD_HIP(hipStreamSynchronize(s));
    GD_HIP(hipMemcpyWithStream(dst, src, bytes, hipMemcpyHostToDevice, s));
    GD_HIP(hipStreamSynchronize(s));
}
inline void d2h(void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (!bytes) return;
    GD_HIP(hipStreamSynchronize(s));
    GD_HIP(hipMemcpyWithStream(dst, src, bytes, hipMemcpyDeviceToHost, s));
    GD_HIP(hipStreamSynchronize(s));
}

// Launch plan of one bitset_matrix region, cached on the collection: the
// tile lists live on the device and the sparse chunk partials stay
// allocated, so repeated calls over one region (the bench steps, row-block
// loops) upload nothing and never wait on the host before their launches.
struct SparseScratch {
    bool ready = false;
    DevBuf tiles, part;   // tile list, per-chunk counters
    DevBuf bounds;        // int32 [nchunks + 1]: first sparse word of each chunk (cost-balanced)
    // the rare tier's pairs are recounted every step by the sparse tile
    // launch's leading workgroups into a per-tile slab the chunk reduce adds
    // (sparse.hip rare_slab_row): the region's (row block, column block) ->
    // tile map and the slab (uint32 [ntiles][128 x 128], written each step)
    DevBuf rare_tile, rare_slab;
    int64_t rare_ab0 = 0, rare_nbc = 0;
    bool rare_in = false;
    int nchunks = 0;
    bool use_part = false;   // chunks store partials (else flush with atomics)
    int64_t ntiles = 0;
};
// One captured step: zero counts, the tile / sparse / rare launches on both
// streams, the epilogue (gdist_intersect_matrix, option graph)
struct StepGraph {
    hipGraphExec_t exec = nullptr;
    int calls = 0;          // uncaptured calls so far (the first builds the launch plans)
    bool failed = false;    // capture refused: this key runs uncaptured
    ~StepGraph() { if (exec) (void)hipGraphExecDestroy(exec); }
};
struct MatrixPlan {
    DevBuf tiles;                    // the four launch groups' tiles
    DevBuf mtiles;                   // the MFMA tiles (256 x 256) of the region (option bitset_mfma)
    int64_t nmt = 0;
    size_t at[5] = {0, 0, 0, 0, 0};  // group bounds
    int64_t corg = 0;
    int rr = 8;
    bool part = false;
    SparseScratch sparse;
};

// ---------------------------------------------------------------------------
// NaN: the call recorded no timing events (a graph-replayed step without
// option step_timing, or no kernel time of its own)
struct Timing {
    double kernel_ms = __builtin_nan(""), call_ms = __builtin_nan("");
    int64_t launches = 0;
};

// Tuning options of a context (gdist_ctx_set_option). These are the A/B
// switches of DESIGN.md §5; each defaults to the measured best. The library
// never reads the environment: a JNI host whose environment differs gets the
// same kernels as the tests, and callers that share a context
// (MethodTableProcessor.java:275, concurrent getDistance) share its options.
// Every option preserves results: each only picks among exact kernels,
// tilings, thresholds or setup paths, and the parity tests run each non-default
// value against the oracle (tests/test_gpu_parity.py, test_gpu_options.py).
#define GDIST_OPTIONS(X)                                                                                       \
    X(TRACE, "trace")                         /* 1: setup stage timings and plans on stderr */                 \
    X(RARE_T, "rare_t")                       /* rare-tier threshold T (default: histogram cost model) */      \
    X(RARE_DEDUP, "rare_dedup")               /* 0: one posting list per rare kmer */                          \
    X(RARE_KERNEL, "rare_kernel")             /* 0 list-major / 1 row-major (default: cost model per call) */  \
    X(RARE_OVERLAP, "rare_overlap")           /* 0: list-major rare kernel in line */                          \
    X(BITSET_DIAG, "bitset_diag")             /* 0: no separate trimmed launch for diagonal tiles */           \
    X(BITSET_PARTIAL_RR, "bitset_partial_rr") /* largest RR whose partial row tile gets its own launches */    \
    X(BITSET_WG_PER_CU, "bitset_wg_per_cu")   /* K-split target (default 16) */                                \
    X(BITSET_MIN_CHUNKS, "bitset_min_chunks") /* fewest 8-word chunks per K-split workgroup (default 16) */     \
    X(REPS_BLOCK, "reps_block")               /* greedy-reps row block (default: by memory) */                 \
    X(LOCUS_ORDER, "locus_order")             /* 0: dense ranks in code order */                               \
    X(SPARSE, "sparse")                       /* 0: no sparse words */                                         \
    X(SPARSE_ZMAX, "sparse_zmax")             /* words with z_w <= ZMAX are sparse (forces the split) */       \
    X(SPARSE_WG_PER_CU, "sparse_wg_per_cu")   /* chunking target of the sparse tiles (default 4) */            \
    X(SPARSE_SUN, "sparse_sun")               /* slots per lane in flight: 2 / 3 / 4 (default 4) */            \
    X(SPARSE_DYN, "sparse_dyn")               /* 1 (default): a tile workgroup's waves claim word batches in turn; 0: equal runs */ \
    X(SPARSE_DIAG22, "sparse_diag22")         /* 1 (default): diagonal tiles in 2 x 2 micro-tiles too (sparse_mt 2) */ \
    X(SPARSE_RPART22, "sparse_rpart22")       /* 1 (default): row-trimmed sparse tiles in 2 x 2 micro-tiles too */ \
    X(SPARSE_MT, "sparse_mt")                 /* off-diagonal micro-tiles: 1 (1 x 2) / 2 (2 x 2, default) */   \
    X(SKETCH_K, "sketch_k")                   /* sketch merge window (1 / 2 / 4 / 6, default 2) */             \
    X(SKETCH_TILE, "sketch_tile")             /* 16: force the 16x16 sketch tile */                            \
    X(SKETCH_V2, "sketch_v2")                 /* 0: the round-2 lane map and checked merge loop */             \
    X(SKETCH_PHASE, "sketch_phase")           /* 0: whole sketches in LDS (V2 / windows), not the ring kernel */ \
    X(SKETCH_CAP, "sketch_cap")               /* ring kernel: merge steps per phase (default 160) */           \
    X(SKETCH_RING, "sketch_ring")             /* ring kernel slots per sketch (default 256) */                 \
    X(SKETCH_WAIT, "sketch_wait")             /* 1: ring pairs without room wait (global reads only if stuck) */ \
    X(SPARSE_PART_BUDGET, "sparse_part_budget") /* bytes of sparse chunk partials one region may hold */       \
    X(GUIDES, "guides")                       /* guide sequences keyed at pack time (default kGuides) */       \
    X(FORCE_EXCHANGE, "force_exchange")       /* 1: a one-rank communicator runs every collective (tests) */   \
    X(SPARSE_CHUNKS, "sparse_chunks")         /* chunks of the sparse words per tile (tests) */                \
    X(GRAPH, "graph")                         /* 0: no hipGraph replay of repeated matrix calls */             \
    X(TIME_KERNELS, "time_kernels")           /* 1: HIP events around each kernel family's launches (no replay) */ \
    X(STEP_TIMING, "step_timing")             /* 1: graph-replayed steps record timing events too */           \
    X(SPARSE_RARE, "sparse_rare")             /* 0: the rare pairs by the rare kernel, not the chunk reduce */ \
    X(SPARSE_FUSED, "sparse_fused")           /* 0: zeroing, rare kernel and epilogue as their own launches */ \
    X(SPARSE_FOLD, "sparse_fold")             /* most (padded) dense words counted in the sparse tile kernel */\
    X(FILL_SORT, "fill_sort")                 /* bitset fill: 0/3 windows, 1 sort, 2 atomics, 4 hash, 5 one-wave windows (default: by size) */\
    X(PACK_SORT, "pack_sort")                 /* 1: two (code, set) pair sorts instead of packed keys */       \
    X(PACK_SUMMARY, "pack_summary")           /* 0: set|code pack keys, the bitset build re-sorts codes */     \
    X(PACK_CODE_SORT, "pack_code_sort")       /* 1 (default): the code-major sort on the code bits when no window was skipped */ \
    X(PACK_OVERLAP, "pack_overlap")           /* 0: upload first / 1: overlapped host thread / 2: registered */\
    X(PACK_CHUNK, "pack_chunk")               /* kmer windows per pack chunk (default 2^28) */                 \
    X(EXCHANGE_BUDGET, "exchange_budget")     /* device bytes an exchange may use (default 0.8 x HBM) */    \
    X(PACK_CODES_BUDGET, "pack_codes_budget") /* bytes of the one-buffer pack (default 1/4 HBM; past it: grown) */\
    X(SPARSE_GROUPS, "sparse_groups")         /* 0: no group tier (clade patterns) in the sparse words */       \
    X(SPARSE_XCD, "sparse_xcd")               /* 1: chunk c of every sparse tile on XCD c mod 8 */           \
    X(RARE_U16, "rare_u16")                   /* 0: 4-byte list members in the row-major rare walk */        \
    X(RARE_ROWS_THREADS, "rare_rows_threads") /* row-major rare walk: threads a workgroup (256/512/1024; default by LDS) */ \
    X(RARE_DIRECT, "rare_direct")             /* row-major rare walk: 1 every record once, members added to I by atomics; 0 LDS column chunks (default: direct past one chunk) */ \
    X(BITSET_MFMA, "bitset_mfma")             /* 0: dense tiles by AND+popcount instead of FP4 MFMA */       \
    X(BITSET_MFMA_RAW, "bitset_mfma_raw")     /* MFMA tiles: 1 (default) stages of the bitsets, nibbles in registers; 0 the FP4 operand */ \
    X(BITSET_MFMA_KM, "bitset_mfma_km")       /* MFMA tiles: words per stage (4 default, 2: 64 KiB of LDS) */ \
    X(BITSET_MFMA_NS, "bitset_mfma_ns")       /* MFMA tiles with 2-word stages: stages in the ring (2..4) */    \
    X(BITSET_MFMA_SPLITS, "bitset_mfma_splits") /* MFMA tiles: K splits a tile (default: ~4 rounds of the chip) */ \
    X(BITSET_MFMA_GROUP, "bitset_mfma_group") /* MFMA tiles: G x 2G tile blocks in launch order (0: row-major) */ \
    X(BITSET_MFMA_STORE, "bitset_mfma_store") /* MFMA tiles: 1 one K split storing its counts, the side families after it; 0 atomics */ \
    X(BITSET_MFMA_SCHED, "bitset_mfma_sched") /* raw MFMA tiles: 1 (default) next stage's DMA between the MFMAs, 0 round 5 */ \
    X(SKETCH_PERM, "sketch_perm")             /* ring kernel, 256 slots: 1 (default) slot addresses by one v_perm_b32, 0 AND + shift-add */ \
    X(BITSET_MFMA_PLANE, "bitset_mfma_plane") /* raw MFMA tiles: 1 (default) bit-plane operands under per-step scales, 0 nibbles of one dword */ \
    X(SORT_RADIX, "sort_radix")               /* 10: onesweep radix sorts of u64 keys in 10-bit passes (A/B) */\
    X(VARIANT, "variant")                     /* variant tier: 1 force, 0 off (default: by the dictionary) */ \
    X(VARIANT_DMIN, "variant_dmin")           /* sets holding a dense-tier kmer (default N / 20; N / 10 before round 6) */            \
    X(RANGE_SUMMARY, "range_summary")         /* 1: the code-range dictionary whatever the size, 0: never */  \
    X(RARE_C16, "rare_c16")                   /* row-major rare walk: 1 (default) 16-bit LDS counters when every row's rare weight < 2^16, 0 32-bit */ \
    X(VARIANT_C16, "variant_c16")             /* variant walk: 1 (default) 16-bit counters in 32,768-column chunks, 0 32-bit in 16,384 */ \
    X(VARIANT_SPLIT, "variant_split")         /* variant walk: workgroups a row (default: ~8 a CU over the rows) */ \
    X(RARE_GROUP, "rare_group")               /* 1: the rare kmers as 16-kmer variant words (short-list walk), 2: the same unless keyless kmers are most of them, 0 never (default: as 2 for 4,096..65,536 sets with guides) */ \
    X(VARIANT_SHORT, "variant_short")         /* packed variant entries: 1 (default) the lane-per-entry walk / 8-byte members, 0 the wave-per-entry walk over the 4 + 8-byte arrays */ \
    X(EPILOGUE_ROWS, "epilogue_rows")         /* distance epilogue: 1 (default) a block a row, 0 the flat kernel */ \
    X(VARIANT_PACK_KEYLESS, "variant_pack_keyless") /* 1 (default): keyless variant kmers packed a word-width at a time in code order; 0 a word each */ \
    X(VARIANT_KEY2, "variant_key2")           /* 1 (default): second-level variant keys (a keyless kmer keyed by the pair of sites of its keyed variant neighbours); 0 first level only */ \
    X(VARIANT_KEYLESS_RARE, "variant_keyless_rare") /* 1: keyless kmers of the 47 / 64-kmer variant tier as rare posting lists instead of packed words (default off) */ \
    X(VARIANT_BITS, "variant_bits")           /* kmers a variant word: 64 or 47 (default 47: < 2^17 sets, k x strands <= 47) */ \
    X(DENSE_FIRST, "dense_first")             /* the dense tiles issued before the side stream's launches (default: without sparse words) */ \
    X(REPS_SPLIT, "reps_split")               /* greedy reps of a gathered collection: 1 (default) columns sharded over the ranks, 0 every rank all */ \
    X(SERIAL_STEP, "serial_step")             /* 1: the side stream's kernel families on the main stream, in turn (timing) */ \
    X(SPLIT_BUILD, "split_build")             /* gathered collection on R ranks: each builds 1/R and all-gathers (default); 0 every rank all; k >= 2 without peers: k shares in turn here */

enum Opt : int {
#define GDIST_OPT_ENUM(id, name) OPT_##id,
    GDIST_OPTIONS(GDIST_OPT_ENUM)
#undef GDIST_OPT_ENUM
    OPT_COUNT
};
extern const char* const kOptNames[OPT_COUNT];
constexpr int64_t kOptUnset = INT64_MIN;

// Stage timer for setup paths: option "trace" = 1 prints "gdist: <stage> <ms>"
// to stderr after synchronising the stream (off: no synchronisation, no cost).
struct Trace {
    bool on;
    hipStream_t st;
    std::chrono::steady_clock::time_point t;
    Trace(hipStream_t s, bool enabled) : on(enabled), st(s), t(std::chrono::steady_clock::now()) {}
    void mark(const char* stage) {
        if (!on) return;
        (void)hipStreamSynchronize(st);
        const auto n = std::chrono::steady_clock::now();
        fprintf(stderr, "gdist: %-28s %9.1f ms\n", stage, std::chrono::duration<double, std::milli>(n - t).count());
        t = n;
    }
};

// Dictionary summary: sorted distinct codes + the number of sets holding each
// (bitset.hip; pack.hip keeps one per pack chunk, gdist_sets::pack_sum)
struct Summary {
    DevBuf codes;    // uint64 [n]
    DevBuf counts;   // uint32 [n]
    int64_t n = 0;
};

}  // namespace gdist

struct gdist_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::recursive_mutex mu;
    hipEvent_t ev_call0 = nullptr, ev_call1 = nullptr, ev_k0 = nullptr, ev_k1 = nullptr;
    hipStream_t side = nullptr;                          // concurrent rare-tier launches
    void* pinned = nullptr;                              // host staging for host outputs (2 halves)
    size_t pinned_bytes = 0;
    hipEvent_t ev_stage[2] = {nullptr, nullptr};
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // option time_kernels: each kernel family's launches alone (uncaptured
    // calls), by family (GDIST_KERNEL_SPARSE / RARE / DENSE / SORTED)
    static constexpr int kFamilies = 5;
    hipEvent_t ev_kf0[kFamilies] = {}, ev_kf1[kFamilies] = {};
    bool kf_timed[kFamilies] = {};
    gdist::Timing last;
    int cus = 256;
    // RCCL communicator (multi-GPU row sharding)
    ncclComm_t comm = nullptr;
    gdist_allgather_fn host_ag = nullptr;   // host-staged transport (gdist_comm_init_host)
    void* host_user = nullptr;
    int nranks = 1, rank = 0;
    // tuning options (gdist_ctx_set_option), kOptUnset = the default
    int64_t opt[gdist::OPT_COUNT];
    bool capturing = false;                  // a step is being captured into a hipGraph
    // kernel-time events of the recent matrix calls (a ring): ev_k0 / ev_k1
    // point at the current call's pair; calls into device outputs return
    // without waiting, their times are read later (gdist_ctx_recent_timings)
    static constexpr int kTimingRing = 256;
    hipEvent_t ring0[kTimingRing] = {}, ring1[kTimingRing] = {};
    int64_t ring_n = 0;                      // calls whose kernel events were recorded
    bool pending = false;                    // the last call's times are not read yet
    bool last_kernel = false;
    gdist_ctx() { for (auto& o : opt) o = gdist::kOptUnset; }
    int64_t option(gdist::Opt o, int64_t dflt) const { return opt[o] == gdist::kOptUnset ? dflt : opt[o]; }
    bool has_option(gdist::Opt o) const { return opt[o] != gdist::kOptUnset; }
    bool trace() const { return option(gdist::OPT_TRACE, 0) != 0; }
};

// A collection of kmer sets resident in HBM.
//   codes:  CSR of sorted unique uint64 codes (kind DNA / PROT)
//   sigs:   CSR of sorted int32 signatures (kind SKETCH)
//   bits:   optional dictionary-rank bitsets, [nsets][W] uint64 row-major
//   segoff: optional value-range segment index for the sorted path,
//           [nsets][nseg+1] absolute positions into codes
struct gdist_sets {
    gdist_ctx* ctx = nullptr;
    int kind = GDIST_DNA;
    int k = 0;
    unsigned flags = 0;
    int width = 0;                        // sketches
    int64_t nsets = 0, total = 0;
    std::vector<int64_t> h_off;           // nsets+1, host mirror (sizes)
    gdist::DevBuf off;                    // int64 [nsets+1]
    gdist::DevBuf codes;                  // uint64 [total] or int32 [total] for sketches
    // bitset representation
    gdist::DevBuf bits;                   // uint64 [nsets][W]
    int64_t W = 0, dict_size = 0;
    bool bits_keep_singletons = false;
    // segment index of the sorted path
    gdist::DevBuf segoff;                 // int64 [nsets][nseg+1]
    gdist::DevBuf seg_split;              // its nseg - 1 splitters (kept: appended sets are indexed by them)
    int nseg = 0;
    int64_t max_seg = 0;
    bool has_codes = true;                // false for all-gathered bitset-only collections
    bool replicated = false;              // every rank of the communicator holds this same collection
                                          // (the code all-gather's result): its build is split by rank
    // the last bitset build: wall time, the split stages' time per share
    // (summary ranges + fill sets; one rank's projection = the rest + the largest share)
    double build_ms = 0, build_split_ms = 0, build_share_max_ms = 0;
    int build_shares = 0;
    // rare tier of the dictionary: kmers held by 2..rare_T-1 sets as posting lists
    gdist::DevBuf post_off;               // int64 [n_rare+1]
    gdist::DevBuf post_sets;              // uint32 [rare_records], ascending within a list
    gdist::DevBuf post_sets16;            // uint16 copy for the row-major walk (nsets <= 65,536; else empty)
    int64_t n_rare = 0, rare_T = 0, rare_records = 0;
    int64_t rare_incs = 0;                // sum over rare lists of m(m-1)/2 pair increments
    int64_t rare_max_list = 0;            // longest rare posting list
    int64_t rare_incs_long = 0;           // pair increments of lists with kLongList+ sets
    int64_t rare_row_wmax = 0;            // max over sets of their rare lists' weights (16-bit row counters below 2^16)
    gdist::DevBuf srare_off;              // int64 [nsets+1]: set -> its rare kmers (CSR)
    gdist::DevBuf srare_ent;              // uint64 [rare_records]: the set's rare lists as
                                          // (list start << 24 | list length), by rare rank
    // Kmers whose posting lists are identical (every kmer covering one shared
    // variant has the same holders) are one list of weight = their number:
    // post_w[list], and srare_w[] aligned with srare_ent.
    gdist::DevBuf post_w;                 // uint32 [n_rare]
    gdist::DevBuf srare_w;                // uint32 [rare_records]
    gdist::DevBuf srare_skip;             // uint16 [rare_records]: 1 + the set's position in the list (0: none)
    int64_t rare_kmers = 0;               // rare dictionary entries before identical lists merge
    // locus guides (pack time, sparse.hip): the kmers of the first kGuides
    // sequences with the position of their first window (window * strands +
    // strand, guides in order), sorted by code
    gdist::DevBuf guide_codes;            // uint64 [n_guide]
    gdist::DevBuf guide_keys;             // uint64 [n_guide]
    int64_t n_guide = 0;
    // complement-sparse words of the dense tier (sparse.hip)
    bool sparse = false;
    gdist::DevBuf dbits;                  // uint64 [nsets][Wd]: the dense words only (tile kernels)
    gdist::DevBuf fp4;                    // the dense tile operand as FP4 nibbles [nsets][32 fp4_W] (MFMA tiles)
    int64_t fp4_W = 0;
    int64_t Wd = 0;                       // dense words, padded to 16 (0: none)
    int64_t Ws = 0;                       // sparse words
    gdist::DevBuf sp_off;                 // int64 [ceil(nsets/128) * Ws + 1]: (set block, sparse word) -> entries
    gdist::DevBuf sp_ent;                 // 16-byte records {row code, word, column code} [sp_entries + 4]
    gdist::DevBuf sp_nc;                  // int32 [nsets]: complement bits over the sparse words
    int64_t sp_entries = 0, sp_U = 0;     // entries; valid bits of the sparse words
    int64_t sp_pos_words = 0;             // sparse words counted from their set bits (positive-sparse)
    bool sp_fold_dense = false;           // the dense words are counted by the sparse tile kernel (no tile launch),
    int sp_fold_slabs = 0;                // 8 words per chunk in the first sp_fold_slabs chunks
    // group tier (sparse.hip): words whose heavy entries are one group's
    // pattern keep per member only the residual; the group part of pair
    // (i, j) is T[gi][gj] + V[gi][j] + V[gj][i], evaluated by the flush /
    // reduce from the set -> group map, V (int32 [groups][nsets]) and T
    // (int32 [groups][groups])
    gdist::DevBuf sp_grp, sp_V, sp_T;
    int64_t sp_groups = 0, sp_group_words = 0;
    std::vector<int32_t> sp_bucket_bits;  // [nsets][sp_nbk]: complement bits per set and 1024 sparse words
    int64_t sp_nbk = 0;
    // summaries of the pack chunks (option pack_summary): the code-major pack
    // sort leaves each chunk's codes in code order, so their runs are that
    // chunk's summary; local_summary merges them instead of re-sorting codes
    std::vector<gdist::Summary> pack_sum;
    double sp_products = 0, sp_items = 0; // whole-triangle products / (tile, word) visits (cost model)
    double sp_pairs = 0;                  // sum over the sparse words of z (z - 1) / 2: the walk's products
    // variant tier (variant.hip): kmers held by T .. Dmin - 1 sets in 64-kmer
    // words grouped by substitution; per word a list of (set, mask) entries,
    // sets ascending; the set -> entry CSR for the row walk
    bool variant = false;
    int64_t vw_words = 0, vw_entries = 0, vw_kmers = 0, vw_dmin = 0, vw_max_list = 0;
    double vw_products = 0;               // sum over words of z (z - 1) / 2
    gdist::DevBuf vw_set;                 // uint32 [E] (grouped by word, ascending set)
    gdist::DevBuf vw_mask;                // uint64 [E]
    gdist::DevBuf vw_beg, vw_end;         // uint32 [E]: the entry's word list
    gdist::DevBuf vs_off;                 // int64 [nsets + 1]
    gdist::DevBuf vs_ent;                 // uint32 [E]: entries by set
    int vw_bits = 64;                     // kmers a variant word (64, 47: packed 8-byte members, 16: grouped rare tier)
    gdist::DevBuf vw_pack;                // uint32 [E] (16-kmer words, <= 65,536 sets): set | mask << 16
    gdist::DevBuf vw_pk64;                // uint64 [E] (47-kmer words, < 2^17 sets): set << 47 | mask
    gdist::DevBuf vs_pent;                // uint64 [E] by set: entry | (end - entry) << 31 | (entry - beg) << 48
    int64_t vw_row_wmax = 0;              // max over sets of their entries' popcounts
    bool auto_sorted = false;             // METHOD_AUTO measured the sorted join cheaper
    // bitset_matrix launch plans by (region, kernel switches); cleared with the bitsets
    mutable std::map<std::vector<int64_t>, std::unique_ptr<gdist::MatrixPlan>> plans;
    // captured steady-state steps (gdist_intersect_matrix into device outputs):
    // a region's launches replayed as one hipGraph; cleared with the plans
    mutable std::map<std::vector<int64_t>, std::unique_ptr<gdist::StepGraph>> graphs;
};

// LSH index of a sketch collection (lsh.hip)
struct gdist_lsh {
    gdist_ctx* ctx = nullptr;
    const gdist_sets* sk = nullptr;       // the indexed sketches (must outlive the index)
    int stages = 0, buckets = 0;
    uint64_t seed = 0;
    gdist::DevBuf salts;                  // uint64 [stages]
    gdist::DevBuf off;                    // int64 [stages * buckets + 1]: bucket -> members
    gdist::DevBuf members;                // int32 [nsets * stages], by (stage, bucket), ascending set
};

namespace gdist {

// pack.hip
// h_seqs (optional): the bytes are still on the host; d_seqs is then the
// caller's device buffer of the same extent, filled chunk by chunk during the pack
void pack_sets(gdist_ctx* ctx, int kind, int k, unsigned flags, const char* d_seqs,
               const int64_t* d_seq_off, const std::vector<int64_t>& h_seq_off, gdist_sets* out,
               const char* h_seqs = nullptr);
void sort_pairs_u64_i32(gdist_ctx* ctx, uint64_t*& keys, uint64_t*& keys_alt, int32_t*& vals,
                        int32_t*& vals_alt, size_t n, int begin_bit, int end_bit);
void sort_keys_u64(gdist_ctx* ctx, uint64_t*& keys, uint64_t*& keys_alt, size_t n, int begin_bit,
                   int end_bit);
void exclusive_scan_i64(gdist_ctx* ctx, const int64_t* in, int64_t* out, size_t n);
void exclusive_scan_i32_to_i64(gdist_ctx* ctx, const int32_t* in, int64_t* out, size_t n);
int code_bits(int kind, int k, unsigned flags);

// bitset.hip — dictionary summaries (struct Summary above gdist_sets)
struct SummaryView {
    const uint64_t* codes;
    const uint32_t* counts;
    int64_t n;
};
void local_summary(gdist_ctx* ctx, const gdist_sets* s, Summary& out);
// T (in/out): rare-tier threshold; T < 0 picks the cost-optimal one for a
// collection of nsets sets from the histogram of kmer counts
// dcounts (optional): the number of sets holding each dense dictionary kmer
void dictionary_from(gdist_ctx* ctx, const std::vector<SummaryView>& parts, bool keep, int64_t& T, int64_t nsets,
                     DevBuf& dict, int64_t& U, DevBuf& rare, int64_t& Ur, int64_t& rare_mass,
                     DevBuf* dcounts = nullptr);
int64_t bitset_words(int64_t dict_size);
int64_t local_rare_mass(gdist_ctx* ctx, const Summary& local, const uint64_t* rare, int64_t Ur);
int64_t auto_rare_threshold(int64_t nsets);
// cost-optimal rare threshold from hist[c] = number of kmers held by c sets
// (c = 0..nsets); the chosen T is reported by gdist_sets_rare_info
int64_t choose_rare_threshold(const std::vector<uint64_t>& hist, int64_t nsets);
// perm (optional): bit position of each dense rank (locus order)
// hook (optional, default fill only): called per chunk of sets [s0, s1)
// with the chunk's position array (u32 per code from code `base`; ~0 outside
// the dictionary) before it is released (variant.hip: the variant records)
using FillHook = std::function<void(const uint32_t* pos, int64_t s0, int64_t s1, int64_t base)>;
// the bits of sets [s0, s1) from their codes' positions (pos from code `base`;
// positions past the W words and ~0 are skipped): LDS row slices, no atomics
void bits_from_positions(gdist_ctx* ctx, const gdist_sets* s, const uint32_t* pos, int64_t s0, int64_t s1,
                         int64_t base, int64_t W, unsigned long long* bits);
// sets [sa, sb) (sb < 0: to the end): their rows of bits, their rare records
void hash_fill(gdist_ctx* ctx, const gdist_sets* s, const uint64_t* dict, int64_t U, const uint32_t* perm,
               const uint64_t* rare, int64_t Ur, int64_t W, unsigned long long* bits, int64_t id_base,
               unsigned long long* rare_out, int64_t rare_cap, int64_t* rare_written, const FillHook& hook,
               int64_t sa = 0, int64_t sb = -1);
void fill_bits(gdist_ctx* ctx, const gdist_sets* s, const uint64_t* dict, int64_t U, int64_t W,
               unsigned long long* bits, const uint64_t* rare, int64_t Ur, int64_t id_base,
               unsigned long long* rare_out, int64_t rare_cap, int64_t* rare_written,
               const uint32_t* perm = nullptr, const FillHook& hook = FillHook(), int64_t sa = 0, int64_t sb = -1);
void build_postings(gdist_ctx* ctx, gdist_sets* s, unsigned long long* recs, int64_t n, int64_t Ur);
// Cost model (seconds), calibrated on MI355X from per-kernel rocprofv3
// averages (scripts/calib_rare.sh; profiles/r01/rare_model): bitset = dense
// AND+popcount tiles + the rare tier; sorted = streaming hash join. Used by
// METHOD_AUTO, the rare-threshold choice, the per-call rare kernel choice and
// the cost-balanced row partition (gdist_sets_block_cost).
constexpr double kDenseWordPairsPerS = 8.6e12;   // launched tile area; 0.87 of the measured and+bcnt ceiling (C2)
constexpr double kDiagTileShare = 0.59;          // a DIAG-launch tile vs an off-diagonal one (C2)
constexpr int kLongList = 64;                    // rare lists of this many sets are walked by a wave
constexpr double kRareListIncsPerS = 2.6e10;     // list-major: pair increments in the block (lane-walked lists)
constexpr double kRareLongIncsPerS = 8.5e9;      // list-major: pair increments of wave-walked long lists
constexpr double kRareListScanPerS = 1.85e11;    // list-major: every list is opened once per call
constexpr double kRareRowPerS = 7.5e10;          // row-major: (incs + records) x the block's share of rows
constexpr double kRareOverlapExposed = 0.6;      // list-major beside the dense launch: the share not hidden
// rare-tier totals the model reads
struct RareTier {
    double incs = 0, incs_long = 0, records = 0, lists = 0;
};
struct RareChoice {
    double list_s = 0, row_s = 0;   // modelled kernel times for the block
    bool row_major = false;
    double cost() const { return row_major ? row_s : list_s * kRareOverlapExposed; }
};
// f_area: the block's share of the tier's pair increments (pairs in the
// block / all pairs); f_rows: its share of the sets as rows. The list-major
// kernel opens every list but walks pairs only from its rows; the row-major
// kernel walks every list of each of its rows. The list-major kernel runs on
// the side stream beside the dense tiles, so its exposed share is compared.
inline RareChoice rare_choice(const RareTier& t, double f_area, double f_rows) {
    RareChoice c;
    if (t.lists <= 0) return c;
    c.list_s = f_area * ((t.incs - t.incs_long) / kRareListIncsPerS + t.incs_long / kRareLongIncsPerS) +
               t.lists / kRareListScanPerS;
    c.row_s = f_rows * (t.incs + t.records) / kRareRowPerS;
    c.row_major = c.row_s < c.list_s * kRareOverlapExposed;
    return c;
}
RareTier rare_tier(const gdist_sets* s);
// pairs of the block rows [r0, r1) x cols [c0, c1) (upper: only j > i)
double block_pairs(int64_t r0, int64_t r1, int64_t c0, int64_t c1, bool upper);
// modelled seconds of bitset_matrix on the block (dense + the rare kernel it picks)
double bitset_block_cost_s(const gdist_sets* s, int64_t r0, int64_t r1, int64_t c0, int64_t c1, bool upper,
                           bool* rare_row_major);
constexpr double kSortedBytesPerS = 6.0e12;      // sorted_join_kernel streaming, C3
double bitset_cost_s(const gdist_sets* s, double pairs);
double sorted_cost_s(const gdist_sets* s, double pairs);
void free_bitsets(gdist_sets* s);
void build_bitsets(gdist_ctx* ctx, gdist_sets* s, unsigned flags, int64_t rare_threshold = -1);
void bitset_matrix(gdist_ctx* ctx, const gdist_sets* s, int64_t r0, int64_t r1, int64_t c0,
                   int64_t c1, bool upper, int32_t* d_I, int64_t ldI);
// the fused sparse step (sparse tiles + reduce storing I and D): true when it
// ran, false when the region needs zeroing + bitset_matrix + epilogue
bool bitset_matrix_fused(gdist_ctx* ctx, const gdist_sets* s, int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                         bool upper, unsigned flags, int32_t* d_I, int64_t ldI, double* d_D, int64_t ldD);

// sparse.hip — locus order of the dense dictionary, complement-sparse words
constexpr int kGuides = 8;                       // guide sequences per packed collection (C2-realistic, 8
                                                 // clades: 2 -> 8 guides took the step 4.60 -> 3.25 ms; C2 and
                                                 // pack time unchanged, profiles/r02/realistic/guides.txt)
constexpr double kSparseProductsPerS = 6.5e11;   // sparse tiles (v6): complement-word products (C2)
constexpr double kSparseItemsPerS = 1.0e11;      // sparse tiles (v6): (tile, sparse word) visits (C2)
bool locus_order_enabled(const gdist_ctx* ctx);  // option locus_order = 0 keeps code order (A/B)
// key[r] = tag | guide position of dense rank r; kmers no guide holds sort
// after every guide key by the number of sets holding them (dcounts)
void locus_keys(gdist_ctx* ctx, const gdist_sets* s, const uint64_t* dict, const uint32_t* dcounts, int64_t U,
                uint64_t tag, DevBuf& key);
// key[r] = min over R ranks' keys (all[q * stride_r + r])
void locus_keys_min(gdist_ctx* ctx, const uint64_t* all, int64_t U, int64_t stride_r, int R, DevBuf& key);
// perm[r] = bit position of dense rank r: ascending key, ties in rank order
void locus_perm(gdist_ctx* ctx, DevBuf& key, int64_t U, DevBuf& perm);
void build_sparse_words(gdist_ctx* ctx, gdist_sets* s);
void free_sparse(gdist_sets* s);
double sparse_block_cost_s(const gdist_sets* s, double f_area, double tiles);
// Fused epilogue of a sparse step (bitset_matrix_fused): the chunk reduce
// stores I (no zeroing) and writes D, the rare pairs come with it
struct SparseEpilogue {
    double* D = nullptr;
    int64_t ldD = 0;
    const int64_t* off = nullptr;         // set offsets: sizes n_i
    int empty_nan = 0;
};
void sparse_plan(gdist_ctx* ctx, const gdist_sets* s, int64_t r0, int64_t r1, int64_t c0, int64_t c1, bool upper,
                 hipStream_t st, SparseScratch& sc);
// returns true when the rare tier's pairs were added with the sparse words
bool sparse_matrix(gdist_ctx* ctx, const gdist_sets* s, int64_t r0, int64_t r1, int64_t c0, int64_t c1, bool upper,
                   int32_t* d_I, int64_t ldI, hipStream_t st, SparseScratch& sc, const SparseEpilogue* ep = nullptr);

// The bitset build of a replicated collection split by rank (option
// split_build): share r counts the code ranges [Pe r / R, Pe (r + 1) / R) of
// the summary and fills the sets [r m, (r + 1) m), m = ceil(N / R); the
// summary, bits, rare records and variant entries are all-gathered. Without
// peers (real = false) every share runs here in turn (option split_build = k:
// the one-rank timing and parity of the split).
struct BuildSplit {
    int R = 1, me = 0;
    bool real = false;
    std::vector<double> share_ms;         // per share: the split stages' time
    int first() const { return real ? me : 0; }
    int last() const { return real ? me + 1 : R; }
    int64_t set_lo(int r, int64_t n) const { return std::min<int64_t>(n, (int64_t)r * ceil_div_h(n, R)); }
    int64_t set_hi(int r, int64_t n) const { return std::min<int64_t>(n, (int64_t)(r + 1) * ceil_div_h(n, R)); }
    static int64_t ceil_div_h(int64_t a, int64_t b) { return (a + b - 1) / b; }
};
BuildSplit build_split(const gdist_ctx* ctx, const gdist_sets* s);
// wall time of one share's stage (synchronises the stream at both ends)
struct ShareClock {
    BuildSplit& sp;
    int r;
    hipStream_t st;
    std::chrono::steady_clock::time_point t;
    ShareClock(BuildSplit& b, int share, hipStream_t s) : sp(b), r(share), st(s) {
        GD_HIP(hipStreamSynchronize(st));
        t = std::chrono::steady_clock::now();
    }
    ~ShareClock() {
        (void)hipStreamSynchronize(st);
        sp.share_ms[r] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    }
};
// communicator (gdist_api.hip): true with peers (RCCL or the host transport)
bool comm_active(const gdist_ctx* ctx);
void comm_allgather_inplace(gdist_ctx* ctx, void* d_buf, size_t bytes);
void comm_allgather(gdist_ctx* ctx, const void* d_send, void* d_recv, size_t bytes);
// every rank's n elements of es bytes (buf) concatenated in rank order into
// buf; returns the total (one all-gather of the counts, one padded in place)
int64_t allgather_concat(gdist_ctx* ctx, DevBuf& buf, int64_t n, size_t es);
// variant.hip — the variant tier
constexpr double kVariantProductsPerS = 2.0e10;  // variant_rows_kernel: popc products (estimate)
constexpr int64_t kVariantMaxT = 32;             // rare threshold of a variant build (unless given)
constexpr int64_t kVariantMinSets = 4096;        // collections the variant tier is considered for by default
constexpr int64_t kRangeSummaryMin = int64_t(1) << 31;   // codes past which an unsummarised collection counts by range
constexpr double kVariantVisitsPerS = 2.0e9;     // ... (entry, column chunk) visits with their list search
int64_t variant_dmin(const gdist_ctx* ctx, int64_t nsets);
bool variant_wanted(const gdist_ctx* ctx, int64_t nsets, int64_t mid_kmers, int64_t dict_kmers);
// summary entries held by lo <= count < hi sets
int64_t count_in_range(gdist_ctx* ctx, const uint32_t* counts, int64_t n, int64_t lo, int64_t hi);
// builds bits (dense tier), the rare postings and the variant tier from the
// dictionary (dict: codes held by >= T sets, dcounts their holders)
// (dmin_in > 0: the dense tier's threshold, else variant_dmin; wb: kmers a
// variant word, 64, 47 (8-byte packed members) or 16 (the packed entries of
// the short-list walk))
// probe: a grouped rare tier chosen by default — false (nothing built or
// changed) when keyless kmers are most of the tier
bool build_variant_bitsets(gdist_ctx* ctx, gdist_sets* s, DevBuf& dict, DevBuf& dcounts, int64_t U, DevBuf& rare,
                           int64_t Ur, int64_t mass, int64_t T, BuildSplit& sp, int64_t dmin_in = -1, int wb = 64,
                           bool probe = false);
void free_variant(gdist_sets* s);
void variant_matrix(gdist_ctx* ctx, const gdist_sets* s, int64_t r0, int64_t r1, int64_t c0, int64_t c1, bool upper,
                    int32_t* d_I, int64_t ldI, hipStream_t rs);
void variant_query(gdist_ctx* ctx, const gdist_sets* s, int64_t q, int32_t* cnt);
// Summary of the codes held by >= min_count sets by ranges of the code space
// (workspace: one range, not the collection: huge gathered collections);
// the ranges of this rank's shares, all-gathered when split
void range_summary(gdist_ctx* ctx, const gdist_sets* s, int min_count, Summary& out, BuildSplit& sp);

// sorted.hip
void build_segments(gdist_ctx* ctx, gdist_sets* s);
// the segment index rows of sets [n_old, nsets) appended to an indexed collection (same splitters)
void extend_segments(gdist_ctx* ctx, gdist_sets* s, int64_t n_old);
void sorted_matrix(gdist_ctx* ctx, const gdist_sets* s, int64_t r0, int64_t r1, int64_t c0,
                   int64_t c1, bool upper, int32_t* d_I, int64_t ldI);
void sorted_row(gdist_ctx* ctx, const gdist_sets* s, int64_t q, const int64_t* d_cols, int64_t ncols,
                int32_t* d_I);

void bitset_row(gdist_ctx* ctx, const gdist_sets* s, int64_t q, const int64_t* d_cols, int64_t ncols,
                int32_t* d_I);
void row_epilogue(gdist_ctx* ctx, const gdist_sets* s, int64_t q, const int64_t* d_cols, int64_t ncols,
                  unsigned flags, const int32_t* d_I, double* d_D);

// epilogue (bitset.hip): D from I and set sizes, Java expression, fp64
void greedy_reps(gdist_ctx* ctx, gdist_sets* s, int method, double t, const int64_t* tie_rank, int32_t* is_rep,
                 int64_t* rep_of, double* rep_dist, int64_t* nreps);
// zero I over the region, only entries with j > i when upper (the others
// belong to the caller: gdist.h, GDIST_UPPER_TRIANGLE)
void zero_counts(gdist_ctx* ctx, int64_t r0, int64_t r1, int64_t c0, int64_t c1, bool upper, int32_t* d_I,
                 int64_t ldI);
void distance_epilogue(gdist_ctx* ctx, const gdist_sets* s, int64_t r0, int64_t r1, int64_t c0,
                       int64_t c1, bool upper, unsigned flags, const int32_t* d_I, int64_t ldI,
                       double* d_D, int64_t ldD);

// lsh.hip
void lsh_build(gdist_ctx* ctx, const gdist_sets* sk, int stages, int buckets, uint64_t seed, gdist_lsh* L);
void lsh_closest(gdist_ctx* ctx, const gdist_lsh* L, const gdist_sets* qs, int nbest, double max_dist,
                 int64_t* idx_out, double* d_out, int32_t* count_out);

// sketch.hip
void sketch_build(gdist_ctx* ctx, const gdist_sets* s, int width, gdist_sets* out);
void sketch_matrix(gdist_ctx* ctx, const gdist_sets* sk, int64_t r0, int64_t r1, int64_t c0,
                   int64_t c1, unsigned flags, int32_t* d_common, double* d_D, int64_t ld);

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// HIP events around one kernel family's launches on stream st (option
// time_kernels, calls not captured): gdist_ctx_kernel_ms reads them
struct FamilyTimer {
    gdist_ctx* ctx;
    int fam;
    hipStream_t st;
    bool on;
    FamilyTimer(gdist_ctx* c, int f, hipStream_t s)
        : ctx(c), fam(f), st(s), on(c->option(OPT_TIME_KERNELS, 0) != 0 && !c->capturing) {
        if (on) GD_HIP(hipEventRecord(ctx->ev_kf0[fam], st));
    }
    void end() {
        if (!on) return;
        GD_HIP(hipEventRecord(ctx->ev_kf1[fam], st));
        ctx->kf_timed[fam] = true;
        on = false;
    }
};

}  // namespace gdist
