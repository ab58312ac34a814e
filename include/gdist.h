/*
 * gdist.h — C-ABI of the MI355X-native pairwise kmer-distance hot path of
 * SEEDtk genome.distance (libgdist.so).
 *
 * Plain C types only: pointers, sizes and status codes. No torch, no C++.
 * Every entry point returns GDIST_OK (0) or a negative GDIST_E* code; the
 * message of the last failure on the calling thread is gdist_last_error().
 *
 * What each entry point replaces in the reference (paths relative to the
 * reference root /root/reference; the kmer classes live in the un-vendored
 * org.theseed:sequence:1.0.0 module, pom.xml:46-49, so their behaviour is
 * taken from the in-repo call sites):
 *
 *   gdist_sets_pack        KmerType.createKmers(seq, K)          FastaDistanceProcessor.java:153,184
 *                          new GenomeKmers(genome)               GenomeProcessor.java:109,139
 *                          new ProteinKmers(seq)                 ProteinKmerReader.java:101
 *   gdist_sets_sizes       SequenceKmers.size()                  (used by distance())
 *   gdist_intersect_matrix SequenceKmers.distance(other) over the
 *                          N×N upper triangle                    FastaDistanceProcessor.java:177-186
 *                          M×N rectangle                         GenomeProcessor.java:140
 *                          group all-pairs                       WidthProcessor.java:159-165
 *   gdist_row_query        anyMatch(d <= maxDist)                DistanceRepsProcessor.java:190
 *                          reduce(NULL_RESULT, merge) argmin     DistanceRepsProcessor.java:238-239
 *                          sequential early exit                 FastaDistanceRepsProcessor.java:117-128
 *   gdist_sketch_build     SequenceKmers.hashSet(width)          SketchProcessor.java:88, WidthProcessor.java:178
 *   gdist_sketch_matrix    Sketch.distance(other) all-pairs      WidthProcessor.java:183-185, TuningProcessor.java:131-133
 *   gdist_sets_allgather   (new) RCCL all-gather of packed sets for row-sharded N×N
 *
 * Kmer code spec (shared by the device packer, the CPU oracle in oracle/ and
 * the Python restatement; see DESIGN.md "Packing spec"). A kmer is k
 * consecutive characters of the sequence after case folding; its code is an
 * order-preserving (code order == Java String order) injective uint64:
 *   DNA, AMBIG_SKIP (default): 2-bit A0 C1 G2 T3, first char most significant,
 *        k <= 32; kmers holding any other char are skipped.
 *   DNA, AMBIG_KEEP: 3-bit A0 C1 G2 N3 R4 T5 Y6, k <= 21; any other char -> EINVAL.
 *   PROT, k <= 8: the k ASCII bytes big-endian (any byte value).
 *   PROT, 8 < k <= 12: 5-bit '*'0 'A'..'Z' 1..26; any other char -> EINVAL.
 *   PROT, AMBIG_SKIP: kmers holding a char outside ACDEFGHIKLMNPQRSTVWY skipped.
 * Byte 0x00 is a sequence separator in every mode: no kmer spans it (used to
 * pack the contigs of one genome, or the proteins of one group, as one set).
 * DNA strand modes: FWD (forward only), BOTH (forward kmers ∪ reverse-
 * complement kmers, the default), CANON (per-position min(fwd, rc)).
 * Distance: d = (I > 0) ? 1.0 - (double)I / (double)(|A|+|B|-I) : 1.0
 * (GDIST_EMPTY_NAN turns the I == 0 && |A|+|B| == 0 case into NaN), fp64,
 * no contraction: bit-identical to the Java expression.
 */
#ifndef GDIST_H
#define GDIST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GDIST_ABI_VERSION 1

/* status codes */
#define GDIST_OK        0
#define GDIST_EINVAL   -1   /* bad argument / unencodable input        -> IllegalArgumentException */
#define GDIST_ENOMEM   -2   /* host or device allocation failed         -> OutOfMemoryError */
#define GDIST_EDEVICE  -3   /* HIP runtime / kernel failure             -> IllegalStateException */
#define GDIST_ECOMM    -4   /* RCCL failure                             -> IllegalStateException */

/* set kinds (KmerType) */
#define GDIST_DNA     0
#define GDIST_PROT    1
#define GDIST_SKETCH  2

/* pack flags */
#define GDIST_STRAND_BOTH   0x0u   /* default for DNA */
#define GDIST_STRAND_FWD    0x1u
#define GDIST_STRAND_CANON  0x2u
#define GDIST_STRAND_MASK   0x3u
#define GDIST_AMBIG_DEFAULT 0x0u   /* DNA: skip, PROT: keep */
#define GDIST_AMBIG_SKIP    0x4u
#define GDIST_AMBIG_KEEP    0x8u
#define GDIST_AMBIG_MASK    0xCu
#define GDIST_NO_CASE_FOLD  0x10u  /* PROT only; DNA always folds to upper case */

/* distance / matrix flags */
#define GDIST_UPPER_TRIANGLE 0x100u /* only pairs with global col > global row */
#define GDIST_OUT_DEVICE     0x200u /* I_out / D_out are device pointers (gdist_dev_alloc); the call
                                       returns once its work is queued on the context's stream:
                                       gdist_ctx_synchronize, gdist_memcpy_d2h or the next call that
                                       reads results waits for it */
#define GDIST_EMPTY_NAN      0x400u /* |A|+|B| == 0 -> NaN instead of 1.0 */
#define GDIST_SKETCH_JACCARD 0x800u /* sketch distance: plain Jaccard of the two signatures
                                       (default: Mash bottom-s of the union) */

/* intersection methods */
#define GDIST_METHOD_AUTO    0   /* bitsets if built; when the sorted join's estimate for the
                                    region exceeds ~20 ms, build the two-tier dictionary and
                                    keep it when its cost estimate beats the sorted join */
#define GDIST_METHOD_SORTED  1   /* sorted uint64 sets: LDS hash-join tiles */
#define GDIST_METHOD_BITSET  2   /* dictionary-rank bitsets: AND + popcount tiles */

/* bitset build flags */
#define GDIST_BITSET_KEEP_SINGLETONS 0x1u /* keep kmers present in only one set
                                             (default prunes them: they never intersect) */

/* row-query modes */
#define GDIST_QUERY_ALL     0
#define GDIST_QUERY_ANY_LE  1
#define GDIST_QUERY_ARGMIN  2

typedef struct gdist_ctx  gdist_ctx;
typedef struct gdist_sets gdist_sets;
typedef struct gdist_lsh  gdist_lsh;

/* ---- library / context ---------------------------------------------- */
const char* gdist_version(void);
/* sha256 prefix (16 hex) of the sources the library was built from
 * (csrc/ *.hip in name order, csrc/gdist_internal.hpp, include/gdist.h):
 * a stale build is detectable against the tree it runs from. */
const char* gdist_source_hash(void);
int  gdist_abi_version(void);
const char* gdist_last_error(void);                 /* thread-local */
int  gdist_device_count(int* n);
int  gdist_ctx_create(int device, gdist_ctx** out);
int  gdist_ctx_destroy(gdist_ctx* ctx);
int  gdist_ctx_synchronize(gdist_ctx* ctx);
/* HIP-event time of the last intersect/sketch matrix call's main kernel(s)
 * and of the whole call, in ms (recorded on the stream they run on); NaN when
 * the call recorded none (a graph-replayed step into device outputs records
 * no events unless option "step_timing" = 1; a call without a kernel of its
 * own has no kernel time). */
int  gdist_ctx_last_timing(gdist_ctx* ctx, double* kernel_ms, double* call_ms, int64_t* launches);
/* Kernel times (ms, HIP events on the stream they ran on) of the last
 * min(max, 256) matrix calls, oldest first, *count of them; waits for them. */
int  gdist_ctx_recent_timings(gdist_ctx* ctx, int max, double* kernel_ms, int* count);
/* HIP-event time (ms) of one kernel family's launches alone, on the stream
 * they ran on, in the last matrix call made with option "time_kernels" = 1
 * (such calls are not graph-replayed); -1 when that family was not timed.
 * Waits for it. Families: the sparse tile launch (with the rare rows it
 * carries), the rare-tier kernel (list- or row-major), the dense tile
 * launches, the sorted join. */
#define GDIST_KERNEL_SPARSE 0
#define GDIST_KERNEL_RARE   1
#define GDIST_KERNEL_DENSE  2
#define GDIST_KERNEL_SORTED 3
#define GDIST_KERNEL_VARIANT 4
int  gdist_ctx_kernel_ms(gdist_ctx* ctx, int family, double* ms);
/* Tuning options of a context: the A/B switches of DESIGN.md §5 by name
 * ("rare_t", "bitset_diag", "sparse", "sparse_zmax", "sketch_k", ...;
 * gdist_ctx_option_name enumerates them, EINVAL past the last). Every option
 * defaults to the measured best; GDIST_OPTION_DEFAULT restores it. No option
 * changes a result: each picks among exact kernels, tilings, thresholds or
 * setup paths, and the parity tests run every non-default value against the
 * oracle; an unknown name is EINVAL. The
 * library never reads the environment, so every host (JNI, ctypes) sharing a
 * context gets the same kernels (concurrent getDistance callers,
 * MethodTableProcessor.java:275). Options read at build time (rare_t,
 * rare_dedup, locus_order, sparse, sparse_zmax, guides) apply to collections
 * packed or built after the call. */
#define GDIST_OPTION_DEFAULT INT64_MIN
int  gdist_ctx_set_option(gdist_ctx* ctx, const char* name, int64_t value);
int  gdist_ctx_get_option(gdist_ctx* ctx, const char* name, int64_t* value, int* is_set);
int  gdist_ctx_option_name(int index, const char** name);
int  gdist_dev_alloc(gdist_ctx* ctx, int64_t bytes, void** dptr);
int  gdist_dev_free(gdist_ctx* ctx, void* dptr);
int  gdist_memcpy_d2h(gdist_ctx* ctx, void* dst, const void* src, int64_t bytes);
int  gdist_memcpy_h2d(gdist_ctx* ctx, void* dst, const void* src, int64_t bytes);
/* Page-locked host memory for sequence bytes (a FASTA reader fills it in
 * place): gdist_sets_pack uploads such a buffer with one DMA per pack chunk
 * at the link's rate instead of the runtime's staged pageable copies. */
int  gdist_host_alloc(int64_t bytes, void** hptr);
/* Return the library's cached device blocks of `device` (freed buffers it
 * keeps for reuse) to the driver, e.g. before another process takes the
 * GPU. Blocks in use are untouched. */
int  gdist_release_cache(int device);
int  gdist_host_free(void* hptr);

/* ---- kmer sets ------------------------------------------------------- */
/* Build kmer sets of nseqs sequences on the device. seqs is the byte
 * concatenation, sequence s = seqs[seq_off[s] .. seq_off[s+1]). The call
 * is synchronous; inside it a short-lived host thread of the library
 * uploads the bytes of pack chunk c + 1 while chunk c is packed (option
 * "pack_overlap"), so seqs is read until the call returns. */
/* seqs in a gdist_host_alloc buffer: one DMA per chunk (detected). */
int  gdist_sets_pack(gdist_ctx* ctx, int kind, int k, unsigned flags,
                     const char* seqs, const int64_t* seq_off, int64_t nseqs,
                     gdist_sets** out);
/* Same, but the sequences are already in device memory (no H2D). */
int  gdist_sets_pack_device(gdist_ctx* ctx, int kind, int k, unsigned flags,
                            const char* d_seqs, const int64_t* d_seq_off, int64_t nseqs,
                            int64_t total_bytes, gdist_sets** out);
/* Pack nseqs more sequences with the collection's kmer spec (kind, k, flags)
 * and append them as sets nsets .. nsets + nseqs - 1 (*first = the old nsets).
 * Replaces `new GenomeKmers(genome)` for a genome seen for the first time by
 * a cache that packs each genome once (MethodTableProcessor.java:261-275 via
 * jni/GpuKmerMethod.java). Every derived representation (bitsets, tiers,
 * plans, the sorted join's index) is dropped and rebuilt on the next call;
 * the codes grow in place, doubling when full. */
int  gdist_sets_append(gdist_ctx* ctx, gdist_sets* sets, const char* seqs, const int64_t* seq_off,
                       int64_t nseqs, int64_t* first);
/* Adopt caller-packed sets: CSR of sorted, unique codes (host arrays, copied). */
int  gdist_sets_upload(gdist_ctx* ctx, int kind, int k, int64_t nsets,
                       const int64_t* offsets, const uint64_t* codes, gdist_sets** out);
int  gdist_sets_free(gdist_sets* sets);
int  gdist_sets_info(const gdist_sets* sets, int* kind, int* k, int64_t* nsets, int64_t* total_codes);
int  gdist_sets_sizes(const gdist_sets* sets, int64_t* sizes);           /* nsets values */
int  gdist_sets_download(const gdist_sets* sets, int64_t* offsets, uint64_t* codes);
/* Build the dictionary-rank bitset representation (kept with the sets).
 * Two exact tiers: kmers held by >= T sets are bit columns of the dense
 * bitsets (AND + popcount tiles); kmers held by 2..T-1 sets are posting lists
 * whose m(m-1)/2 pairs are counted directly. _ex sets T (-1 = automatic,
 * 0..2 = dense only); KEEP_SINGLETONS forces a dense-only dictionary of
 * every distinct kmer. */
int  gdist_sets_build_bitsets(gdist_sets* sets, unsigned flags);
int  gdist_sets_build_bitsets_ex(gdist_sets* sets, unsigned flags, int64_t rare_threshold);
/* A collection the code all-gather returned (gdist_sets_allgather_ex) is the
 * same on every rank; its bitset build is then collective and split by rank
 * (option "split_build", default on): rank r counts 1/R of the code ranges
 * of the dictionary summary and fills the tiers of sets [r m, (r + 1) m),
 * m = ceil(N / R); the summary, bitset rows, rare records and variant entries
 * are all-gathered, and every rank holds the whole representation (the same
 * on every rank as a one-rank build). Every rank must make the build call
 * (build_bitsets, prepare, or a BITSET/AUTO matrix call that builds; AUTO
 * builds on every rank when any rank's region asks for it). The setup step of
 * FastaDistanceProcessor.java:150-155 (the reference builds every batch's
 * kmer sets on one host). */
/* Release the codes of a collection whose bitsets are built (the C4 code
 * all-gather's 160 GB per rank): the collection keeps its bitset tiers and
 * sizes and answers METHOD_BITSET / AUTO calls; the sorted join, sketches, a
 * rebuild and appends need codes and refuse it (EINVAL). */
int  gdist_sets_release_codes(gdist_sets* sets);
/* The last bitset build: wall time (ms), the time of its split stages (the
 * summary's code ranges and the fill's sets, all shares) and of the largest
 * share, and the shares (1: not split). One rank of a split build ran one
 * share; option "split_build" = k on one rank runs k shares in turn, so that
 * build_ms - split_ms + share_max_ms is one rank's build of 1/k of the sets. */
int  gdist_sets_build_timing(const gdist_sets* sets, double* build_ms, double* split_ms, double* share_max_ms,
                             int* shares);
/* Rare tier: threshold T, distinct posting lists and their member records.
 * Kmers with identical posting lists (e.g. every kmer covering one shared
 * variant) are one list weighted by their number (option "rare_dedup" = 0: one
 * list per kmer); gdist_sets_rare_kmers gives the kmers before merging. */
int  gdist_sets_rare_info(const gdist_sets* sets, int64_t* threshold, int64_t* lists, int64_t* records);
int  gdist_sets_rare_kmers(const gdist_sets* sets, int64_t* kmers);
/* Rare-tier statistics behind the cost model: pair increments (sum of
 * m(m-1)/2 over the posting lists) and the longest list. */
int  gdist_sets_rare_stats(const gdist_sets* sets, int64_t* pair_incs, int64_t* max_list);
int  gdist_sets_bitset_info(const gdist_sets* sets, int64_t* dict_size, int64_t* words_per_set);
/* Complement-sparse words of the dense tier: the dense
 * dictionary is ranked in locus order (the kmer's window in the collection's
 * first sequences), and each bitset word that few sets lack anything in is
 * counted from the sets' complement words instead of the AND+popcount tiles.
 * Reports the sparse words, the dense words left to the tiles (padded) and
 * the complement entries (0s when the split was not worth building).
 * Options "sparse" = 0 / "locus_order" = 0 switch it off (A/B). */
int  gdist_sets_sparse_info(const gdist_sets* sets, int64_t* sparse_words, int64_t* dense_words, int64_t* entries);
/* The variant tier: kmers held by T .. Dmin - 1 sets (Dmin:
 * option "variant_dmin", default N / 10) grouped by the substitution that
 * made them into 64-kmer words, each a list of (set, 64-bit mask) entries;
 * a pair adds popc(mask_i & mask_j) per shared word. Built by the bitset
 * build when those kmers dominate the dictionary (option "variant": 1
 * forces, 0 never). Reports the kmers, words, entries and the walk's
 * products (sum over words of z(z-1)/2); zeros without the tier. */
int  gdist_sets_variant_info(const gdist_sets* sets, int64_t* kmers, int64_t* words, int64_t* entries,
                             double* products);
/* The variant tier's layout: kmers a word (47 or 64, option variant_bits;
 * 16 for the grouped rare tier, option rare_group), the bytes of a list
 * member the walk reads (4: set | mask << 16 of the short-list walk, 16-kmer
 * words of <= 65,536 sets; 8: set << 47 | mask, 47-kmer words of < 2^17
 * sets; 12: the 4-byte set and 8-byte mask arrays), and the largest sum of a
 * set's entry popcounts (16-bit counters below 2^16; 4-byte layout only).
 * Zeros without a variant tier. Diagnostics (bench roofline). */
int  gdist_sets_variant_layout(const gdist_sets* sets, int* word_kmers, int* member_bytes, int64_t* row_weight_max);
/* The sparse words by side: counted from the sets' complement words (sets
 * lacking a commonly held kmer) or from their words (sets holding a rarely
 * held one: positive-sparse). */
int  gdist_sets_sparse_sides(const gdist_sets* sets, int64_t* complement_words, int64_t* positive_words);
/* The sparse tile kernel's products over the whole collection: the sum over
 * the sparse words of z (z - 1) / 2 (z = the word's entries), each pair of a
 * word's entries once (0 without the split). Diagnostics: the bench line's
 * VALU per 64 products. */
int  gdist_sets_sparse_pairs(const gdist_sets* sets, double* pairs);
/* The group tier of the sparse words: groups of sets (e.g.
 * the clades of a structured collection) whose members all carry the same
 * pattern in a word; those words keep per member only the residual entries
 * and the group part of a pair is evaluated from per-group tables (T, V)
 * with the pair's constant part. Reports the groups used
 * and the sparse words factorised by one (0s without the tier; option
 * "sparse_groups" = 0 switches it off). */
int  gdist_sets_group_info(const gdist_sets* sets, int64_t* groups, int64_t* grouped_words);
/* Copy the bitsets (nsets x words_per_set uint64, row-major) to the host. */
int  gdist_sets_bitset_download(const gdist_sets* sets, uint64_t* bits);
/* Concatenate two collections (e.g. base genomes + comparison genomes). */
int  gdist_sets_concat(const gdist_sets* a, const gdist_sets* b, gdist_sets** out);

/* ---- distances ------------------------------------------------------- */
/* Prepare the representation `method` needs for a region of `pairs` pairs
 * (pairs < 0: the whole N(N-1)/2 triangle) and report the method a later
 * gdist_intersect_matrix(method) call will run (*chosen: SORTED or BITSET).
 * With METHOD_AUTO this is where the two-tier dictionary is built and costed;
 * *cost_bitset_s / *cost_sorted_s (may be NULL) return the model's estimates
 * (-1 when no bitsets are held). The setup step of FastaDistanceProcessor.java:150-155
 * (a batch's kmer sets are built and cached before its pair loop). */
int  gdist_sets_prepare(gdist_ctx* ctx, gdist_sets* sets, int method, double pairs, int* chosen,
                        double* cost_bitset_s, double* cost_sorted_s);
/* Pairs (i, j), r0 <= i < r1, c0 <= j < c1 (global set indices of `sets`).
 * I_out[(i-r0)*ld + (j-c0)] = |A_i ∩ A_j|, D_out[...] = distance; either
 * output may be NULL. With GDIST_UPPER_TRIANGLE, entries with j <= i are
 * left untouched. */
int  gdist_intersect_matrix(gdist_ctx* ctx, const gdist_sets* sets,
                            int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                            int method, unsigned flags,
                            int32_t* I_out, double* D_out, int64_t ld);
/* Greedy representatives over the whole collection, on the device.
 * Pass 1 (DistanceRepsProcessor.java:185-200, FastaDistanceRepsProcessor.java:
 * 117-144): sets in index order; set k becomes a representative unless an
 * earlier representative lies within max_dist (d <= max_dist); is_rep[k] =
 * 1 / 0, *nreps = their number. Keys are assumed unique (the reference's
 * repMap.put would replace a representative with the same id).
 * Pass 2, when rep_of or rep_dist is non-NULL (DistanceRepsProcessor.java:
 * 227-237): every set's closest representative, ties to the lowest
 * tie_rank (NULL: index), d < 1.0 only (NULL_RESULT identity); a
 * representative maps to itself at 0.0; -1 / 1.0 when none. */
int  gdist_greedy_reps(gdist_ctx* ctx, const gdist_sets* sets, int method, double max_dist,
                       const int64_t* tie_rank, int32_t* is_rep, int64_t* rep_of, double* rep_dist,
                       int64_t* nreps);
/* One query set q against ncols sets (indices cols[]):
 *  ALL:    D_out[c] for every c
 *  ANY_LE: *hit = 1 if any distance <= t (D_out may be NULL)
 *  ARGMIN: *best_idx = position in cols[] of the smallest distance (ties ->
 *          lowest position), *best_d = that distance; -1 / 1.0 when no
 *          distance is below 1.0 (the reference's NULL_RESULT identity wins
 *          ties at 1.0, DistanceRepsProcessor.java:108-122). */
int  gdist_row_query(gdist_ctx* ctx, const gdist_sets* sets, int64_t q,
                     const int64_t* cols, int64_t ncols, int mode, double t,
                     double* D_out, int32_t* hit, int64_t* best_idx, double* best_d);

/* ---- MinHash sketches ------------------------------------------------ */
/* Bottom-`width` signature per set: the width smallest distinct
 * murmur3_x86_32(seed 0) hashes (signed int order) of the kmer strings. */
int  gdist_sketch_build(gdist_ctx* ctx, const gdist_sets* sets, int width, gdist_sets** out);
int  gdist_sketch_upload(gdist_ctx* ctx, int width, int64_t nsets, const int64_t* offsets,
                         const int32_t* sigs, gdist_sets** out);
int  gdist_sketch_download(const gdist_sets* sk, int64_t* offsets, int32_t* sigs);
int  gdist_sketch_matrix(gdist_ctx* ctx, const gdist_sets* sk,
                         int64_t r0, int64_t r1, int64_t c0, int64_t c1, unsigned flags,
                         int32_t* common_out, double* D_out, int64_t ld);

/* ---- LSH bucket query (MashProcessor / FindProcessor) ------------------ */
/* Index of a sketch collection: new LSHMemSeqHash(width, stages, buckets)
 * + add() per subject (MashProcessor.java:110,130; BuildProcessor.java:131,148).
 * Stage t files a sketch in bucket (min over its signature of a salted
 * splitmix64 mix) mod buckets; seed picks the salts. The sketches must
 * outlive the index. (Restated: the LSH classes are un-vendored.) */
int  gdist_lsh_build(gdist_ctx* ctx, const gdist_sets* sketches, int stages, int buckets, uint64_t seed,
                     gdist_lsh** out);
int  gdist_lsh_free(gdist_lsh* lsh);
/* getClosest(kmers, n, maxDist) for every query sketch (MashProcessor.java:150,
 * FindProcessor.java:110): among the indexed sets sharing a bucket with the
 * query in any stage, those at sketch distance <= max_dist, nearest first
 * (ties by index), at most n: idx_out[q*n + r], d_out[q*n + r], count_out[q]. */
int  gdist_lsh_closest(gdist_ctx* ctx, const gdist_lsh* lsh, const gdist_sets* queries, int n, double max_dist,
                       int64_t* idx_out, double* d_out, int32_t* count_out);

/* ---- multi-GPU (RCCL over xGMI) -------------------------------------- */
#define GDIST_UNIQUE_ID_BYTES 128
int  gdist_comm_unique_id(char id[GDIST_UNIQUE_ID_BYTES]);
int  gdist_comm_init(gdist_ctx* ctx, const char id[GDIST_UNIQUE_ID_BYTES], int nranks, int rank);
/* Host-staged communicator: every collective of the library becomes one
 * all-gather of host buffers through `fn`, which must place the `bytes` of
 * every rank, in rank order, into recv (nranks * bytes) and return 0. For
 * ranks that share one GPU (rehearsing the multi-rank path; RCCL refuses two
 * ranks on one device) or hosts without RCCL peer access; RCCL
 * (gdist_comm_init) is the transport of a multi-GPU node. */
typedef int (*gdist_allgather_fn)(const void* send, void* recv, int64_t bytes, void* user);
int  gdist_comm_init_host(gdist_ctx* ctx, int nranks, int rank, gdist_allgather_fn fn, void* user);
int  gdist_comm_destroy(gdist_ctx* ctx);
/* Every rank passes its local shard; every rank receives the concatenation
 * in rank order (one all-gather of offsets and one, in place, of codes). */
int  gdist_sets_allgather(gdist_ctx* ctx, const gdist_sets* local, gdist_sets** out);
/* The same; with GDIST_ALLGATHER_CONSUME the library releases `local`'s
 * device data once its codes are in the gather buffer (local keeps its sizes
 * and can still be freed; it can no longer be used for distances). Peak
 * device bytes per rank: (ranks + 1) x the largest shard's codes. The local
 * data is released BEFORE the collective runs: if the all-gather itself
 * fails (GDIST_ECOMM, or the host transport's callback), `local` stays
 * unusable and no result is returned; the caller re-packs its shard. */
#define GDIST_ALLGATHER_CONSUME 0x1u
int  gdist_sets_allgather_ex(gdist_ctx* ctx, gdist_sets* local, unsigned flags, gdist_sets** out);
/* Which exchange a row-sharded N×N over this communicator should use
 * (collective: every rank calls it with its local shard and gets the same
 * answer). *chosen = GDIST_METHOD_BITSET: the dictionary exchange
 * (gdist_sets_allgather_bitsets); GDIST_METHOD_SORTED: the code all-gather
 * (gdist_sets_allgather_ex) for the sorted join. METHOD_AUTO takes the
 * dictionary exchange when its per-rank estimate fits the budget (option
 * "exchange_budget", default 0.8 x the device memory), else the codes; the
 * estimates (bytes per rank; the codes' assume the shard is consumed) are
 * returned. ENOMEM when neither fits.
 * (C4 = 100,000 x 100 kbp on 8 GPUs takes the codes.) */
int  gdist_sets_exchange_plan(gdist_ctx* ctx, const gdist_sets* local, int method, int* chosen,
                              double* bytes_bitsets, double* bytes_codes);
/* Dictionary-rank bitsets of the concatenation (in rank order) of every
 * rank's local sets: one all-gather of the local dictionary summaries
 * (distinct codes + counts), one of the local bitsets. The result holds the
 * bitsets and sizes of all sets but no codes: use it with
 * GDIST_METHOD_BITSET (or AUTO). Memory per rank ~ N * W words instead of
 * every rank's codes. */
int  gdist_sets_allgather_bitsets(gdist_ctx* ctx, const gdist_sets* local, unsigned flags, gdist_sets** out);
/* Scalar max-reduction and barrier over the communicator (timing only). */
int  gdist_comm_allreduce_max(gdist_ctx* ctx, double* value);

/* The cost model's estimate (seconds) of one intersect-matrix call on the
 * block rows [r0, r1) x columns [c0, c1) (upper: pairs j > i only): with
 * bitsets built, dense tiles + the rare kernel the call would pick
 * (*rare_kernel = 0 list-major, 1 row-major, -1 no rare tier); otherwise the
 * sorted join (*rare_kernel = -1). For row partitions that balance modelled
 * time rather than area (gdist.shard.balanced_bounds). */
int  gdist_sets_block_cost(const gdist_sets* sets, int64_t r0, int64_t r1, int64_t c0, int64_t c1, int upper,
                           double* seconds, int* rare_kernel);

/* Row partition with equal upper-triangle area:
 * r_g = N (1 - sqrt(1 - g/G)), rounded to multiples of `align`. */
int  gdist_triangle_partition(int64_t n, int nparts, int64_t align, int64_t* bounds /* nparts+1 */);

#ifdef __cplusplus
}
#endif
#endif /* GDIST_H */
