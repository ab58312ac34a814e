// variant.hip — the variant tier of the two-tier dictionary: kmers held by
// many sets but far from all (C4: 100,000 genomes of one 100 kbp ancestor at
// up to 5 % substitutions, where every single-substitution kmer is shared by
// ~500 genomes).
//
// Why a third tier. The dense tier costs every pair one AND+popcount per
// 64-kmer word whether or not the pair holds any of the word's kmers; the
// rare tier costs m(m-1)/2 increments per posting list of m sets. C4's
// 12.6 M single-substitution kmers are neither: as dense words they would be
// 200 K words a pair (1e15 word pairs on the triangle), as posting lists of
// ~500 sets 1e12 increments. Grouped by the substitution that made them (a
// substitution at one site makes the k windows covering it, on both strands,
// 2k kmers held by nearly the same genomes), 64 to a word, each word is a
// list of (set, 64-bit mask) entries, and a pair sharing the word adds
// popc(mask_i & mask_j): the kmers of one substitution cost one product, not
// 2k increments.
//
// Grouping needs no positions: a variant kmer's substitution shows as its
// Hamming-1 neighbour in the dense tier (the ancestral kmer at the same
// window), whose locus the guide sequences give (pack time, sparse.hip
// locus_keys); (neighbour window + offset of the differing symbol, the
// symbol) names the site and the letter on the forward strand, so both
// strands' kmers of one substitution get one key. Kmers with no dense
// neighbour get a second-level key when a keyed VARIANT neighbour exists
// (round 6: the unordered pair of the two substitution sites, see
// variant_key2_kernel); the rest (no guide, three substitutions in a
// window) keep code order after the keyed ones. Any grouping is exact; it
// only decides how many products the walk does.
//
// Tiers by the number of sets c holding a kmer: dense c >= Dmin (default
// N / 20 since round 6, was N / 10: bit columns of the tile kernels),
// variant T <= c < Dmin, rare 2 <= c < T (posting lists), singletons
// dropped (they never intersect). Dmin prices a kmer as a bit column of
// every pair (N^2 / 2 bit-products on the matrix cores, ~4e-16 s each) or as
// a share of a variant word (~c^2 / (2 x 47) products of the walk, ~4e-12 s
// each): the break-even holder count is ~0.07 N for kmers grouped 47 to a
// word. The C4-realistic slice (clade-specific kmers held by ~7.5 K of
// 100 K genomes) measured 68.5 ms at N / 10 with first-level keys, 31.1 ms
// with second-level keys, 21.0 ms at N / 20; C4 (nothing held by 5-10 % of
// the genomes) is the same at both (profiles/r06/s8, s9).
//
// Build (build_variant_bitsets, one GPU, from codes; C4 on 8 GPUs runs it on
// every rank after the one code all-gather): a code-range dictionary
// (range_summary: per range of the code space every set's codes of that
// range gathered, sorted, counted, singletons dropped: the workspace is one
// range, not the collection), the tiers, the variant keys and word order, one
// fill pass over every set's codes (fill_bits with a hook: dense codes set
// bits, variant codes emit (word, set, bit) records that are sorted and
// OR-merged per set chunk), then the word lists and the set -> entry CSR.
//
// Walk (variant_rows_kernel, bitset_matrix): one workgroup per row (or a
// slice of its entries); a wave takes one of the row's entries and its 64
// lanes stream the entry's word list (sets ascending, coalesced 4 + 8 bytes
// per member) from the row's own position (upper triangle), adding
// popc(mask_i & mask_j) into LDS counters of one column chunk at a time; each
// entry's list position stays in LDS from chunk to chunk, so every list is
// read once; each chunk's counters are added to I's row once.
#include <algorithm>
#include <cstring>
#include <vector>

#include "gdist_internal.hpp"

namespace gdist {
namespace {

inline int grid_for(int64_t n, int block = 256, int64_t cap = 256 * 32) {
    int64_t g = ceil_div(n, block);
    return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

__device__ __forceinline__ int64_t lower_bound_u64(const uint64_t* __restrict__ a, int64_t lo, int64_t hi, uint64_t k) {
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] < k) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// ---- code-range dictionary ----------------------------------------------
// splitter positions: spos[i * (P + 1) + p] = lower bound of splitter p in
// set i's codes (p = 0: the set's start, p = P: its end)
__global__ void range_pos_kernel(const uint64_t* __restrict__ codes, const int64_t* __restrict__ off, int64_t nsets,
                                 const uint64_t* __restrict__ split, int P, int64_t* __restrict__ spos) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nsets * (P + 1)) return;
    const int64_t i = t / (P + 1);
    const int p = (int)(t % (P + 1));
    const int64_t b = off[i], e = off[i + 1];
    spos[t] = p == 0 ? b : p == P ? e : lower_bound_u64(codes, b, e, split[p - 1]);
}

// the sizes of range p per set -> cnt[i]
__global__ void range_sizes_kernel(const int64_t* __restrict__ spos, int64_t nsets, int P, int p,
                                   int64_t* __restrict__ cnt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nsets) cnt[i] = spos[i * (P + 1) + p + 1] - spos[i * (P + 1) + p];
}

// gather range p of every set: one workgroup per set
__global__ __launch_bounds__(256) void range_gather_kernel(const uint64_t* __restrict__ codes,
                                                           const int64_t* __restrict__ spos, int P, int p,
                                                           const int64_t* __restrict__ at, uint64_t* __restrict__ out) {
    const int64_t i = blockIdx.x;
    const int64_t b = spos[i * (P + 1) + p], e = spos[i * (P + 1) + p + 1];
    uint64_t* o = out + at[i] - b;
    for (int64_t x = b + threadIdx.x; x < e; x += 256) o[x] = codes[x];
}

__global__ void sample_kernel(const uint64_t* __restrict__ codes, int64_t first, int64_t stride, int64_t n,
                              uint64_t* __restrict__ out) {
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gs) out[i] = codes[first + i * stride];
}

// heads of runs in sorted keys
__global__ void heads_kernel(const uint64_t* __restrict__ k, int64_t n, int32_t* __restrict__ flag) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        flag[i] = (i == 0 || k[i] != k[i - 1]) ? 1 : 0;
}

// runs of >= min_count: (code, count) compacted; keep[] = 1 for kept heads
__global__ void run_keep_kernel(const uint64_t* __restrict__ k, int64_t n, const int32_t* __restrict__ flag,
                                int min_count, int32_t* __restrict__ keep, uint32_t* __restrict__ len) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        int32_t kp = 0;
        uint32_t c = 0;
        if (flag[i]) {
            int64_t e = i + 1;
            while (e < n && k[e] == k[i]) e++;
            c = (uint32_t)(e - i);
            kp = (int64_t)c >= min_count ? 1 : 0;
        }
        keep[i] = kp;
        len[i] = c;
    }
}

__global__ void run_emit_kernel(const uint64_t* __restrict__ k, const int32_t* __restrict__ keep,
                                const uint32_t* __restrict__ len, const int64_t* __restrict__ pos, int64_t n,
                                uint64_t* __restrict__ oc, uint32_t* __restrict__ on) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        if (keep[i]) { oc[pos[i]] = k[i]; on[pos[i]] = len[i]; }
}

// ---- tiers and the variant order -----------------------------------------
__global__ void tier_flags_kernel(const uint32_t* __restrict__ cnt, int64_t n, uint32_t dmin,
                                  int32_t* __restrict__ dense, int32_t* __restrict__ mid) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        dense[i] = cnt[i] >= dmin ? 1 : 0;
        mid[i] = cnt[i] >= dmin ? 0 : 1;
    }
}

__global__ void split_codes_kernel(const uint64_t* __restrict__ dict, const uint32_t* __restrict__ cnt, int64_t n,
                                   const int32_t* __restrict__ dense, const int64_t* __restrict__ dpos,
                                   const int64_t* __restrict__ mpos, uint64_t* __restrict__ dcodes,
                                   uint32_t* __restrict__ dcnt, uint64_t* __restrict__ mcodes) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (dense[i]) { dcodes[dpos[i]] = dict[i]; dcnt[dpos[i]] = cnt[i]; }
        else mcodes[mpos[i]] = dict[i];
    }
}

// guide entry of every dense code (-1: no guide holds it): the locus
__global__ void dense_entry_kernel(const uint64_t* __restrict__ dcodes, int64_t Ud,
                                   const uint64_t* __restrict__ gcodes, const uint64_t* __restrict__ gkeys, int64_t ng,
                                   int64_t* __restrict__ entry) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < Ud; r += stride) {
        const int64_t g = lower_bound_u64(gcodes, 0, ng, dcodes[r]);
        entry[r] = (g < ng && gcodes[g] == dcodes[r]) ? (int64_t)gkeys[g] : -1;
    }
}

// Code geometry of a collection for the neighbour search: symbols of `bits`
// bits, first symbol most significant; alphabet (the symbols a kmer can
// hold) and the complement map of DNA.
struct CodeGeom {
    int k = 0, bits = 0, strands = 1;
    int nalpha = 0;
    uint8_t alpha[32] = {};
    int8_t comp[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
};

// Variant key of every variant-tier kmer: min over its Hamming-1 neighbours
// in the dense tier that a guide holds of (site << 8 | forward letter), with
// site = the neighbour's window + the offset of the differing symbol
// (reversed on the reverse strand, whose letter is complemented); ~0 when no
// keyed neighbour exists.
// (site << 8 | forward letter) of a kmer's symbol j when its window is the
// guide entry e (window << 1 | strand for two strands)
__device__ __forceinline__ uint64_t site_key(const CodeGeom& g, int64_t e, int j, uint64_t cur) {
    const int64_t w = e / g.strands, strand = e % g.strands;
    int64_t site;
    uint64_t letter;
    if (strand == 0) { site = w + j; letter = cur; }
    else { site = w + (g.k - 1 - j); letter = (uint64_t)(g.comp[cur] < 0 ? cur : g.comp[cur]); }
    return ((uint64_t)site << 8) | letter;
}
__global__ __launch_bounds__(256) void variant_key_kernel(const uint64_t* __restrict__ mcodes, int64_t Um,
                                                          const uint64_t* __restrict__ dcodes, int64_t Ud,
                                                          const int64_t* __restrict__ dentry, CodeGeom g,
                                                          uint64_t* __restrict__ vkey, int64_t* __restrict__ went) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const uint64_t smask = (1ull << g.bits) - 1ull;
    for (int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; m < Um; m += stride) {
        const uint64_t c = mcodes[m];
        uint64_t best = ~0ull;
        int64_t be = -1;
        for (int j = 0; j < g.k; j++) {
            const int sh = (g.k - 1 - j) * g.bits;          // symbol j (0 = first, most significant)
            const uint64_t cur = (c >> sh) & smask;
            for (int a = 0; a < g.nalpha; a++) {
                const uint64_t s = g.alpha[a];
                if (s == cur) continue;
                const uint64_t nb = (c & ~(smask << sh)) | (s << sh);
                const int64_t r = lower_bound_u64(dcodes, 0, Ud, nb);
                if (r >= Ud || dcodes[r] != nb || dentry[r] < 0) continue;
                const uint64_t key = site_key(g, dentry[r], j, cur);
                if (key < best) { best = key; be = dentry[r]; }
            }
        }
        vkey[m] = best;
        if (went) went[m] = be;          // the window (guide entry) the key was read in
    }
}

// Round 6: second-level keys of the keyless variant kmers (a substitution
// inside a window that a first-level variant already changed: C4-realistic's
// clade-specific kmers are held by ~7.5 K of 100 K genomes, below Dmin, so an
// individual substitution next to a clade substitution has no dense
// neighbour). Such a kmer x has keyed variant neighbours: y (x with the
// individual substitution reverted; y's key is the clade site C, its window
// known) and x' (the clade substitution reverted; key I). Through y, x's
// differing symbol in y's window names I; through x', C — so the unordered
// pair {C, I} keys every window that holds both substitutions, and they share
// a word (their holders: one clade's genomes with that substitution). The
// key is a 63-bit mix of the pair with the top bit set (first-level keys
// have it clear; ~0 stays "keyless"); any grouping is exact.
__device__ __forceinline__ uint64_t pair_key(uint64_t a, uint64_t b) {
    const uint64_t lo = a < b ? a : b, hi = a < b ? b : a;
    uint64_t z = lo * 0x9E3779B97F4A7C15ull ^ (hi + 0x632BE59BD9B4E019ull);
    z ^= z >> 31; z *= 0xBF58476D1CE4E5B9ull; z ^= z >> 29; z *= 0x94D049BB133111EBull; z ^= z >> 32;
    const uint64_t k = (1ull << 63) | (z >> 1);
    return k == ~0ull ? k - 1 : k;
}
__global__ __launch_bounds__(256) void variant_key2_kernel(const uint64_t* __restrict__ mcodes, int64_t Um,
                                                           const uint64_t* __restrict__ vkey,
                                                           const int64_t* __restrict__ went, CodeGeom g,
                                                           uint64_t* __restrict__ vkey2) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const uint64_t smask = (1ull << g.bits) - 1ull;
    for (int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; m < Um; m += stride) {
        uint64_t best = vkey[m];
        if (best == ~0ull) {
            const uint64_t c = mcodes[m];
            for (int j = 0; j < g.k; j++) {
                const int sh = (g.k - 1 - j) * g.bits;
                const uint64_t cur = (c >> sh) & smask;
                for (int a = 0; a < g.nalpha; a++) {
                    const uint64_t s = g.alpha[a];
                    if (s == cur) continue;
                    const uint64_t nb = (c & ~(smask << sh)) | (s << sh);
                    const int64_t r = lower_bound_u64(mcodes, 0, Um, nb);
                    if (r >= Um || mcodes[r] != nb || went[r] < 0) continue;
                    const uint64_t key = pair_key(vkey[r], site_key(g, went[r], j, cur));
                    best = key < best ? key : best;
                }
            }
        }
        vkey2[m] = best;
    }
}

// group heads of the sorted keys (a keyless kmer is a group of its own) ->
// words of the group: ceil(len / wb), each group starting a new word (wb:
// kmers a word, 64, or 16 for the short-list walk's packed entries)
// (pack = 0: every keyless kmer a word of its own — unrelated kmers never
// share a word's entry list)
__global__ void group_words_kernel(const uint64_t* __restrict__ k, int64_t n, int wb, int pack,
                                   int32_t* __restrict__ head, int64_t* __restrict__ words) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const bool h = i == 0 || k[i] != k[i - 1] || k[i] == ~0ull;
        head[i] = h ? 1 : 0;
        int64_t wn = 0;
        if (h) {
            int64_t e = i + 1;
            if (k[i] == ~0ull) e = pack ? n : i + 1;         // the keyless kmers: one group, packed
            else while (e < n && k[e] == k[i]) e++;
            wn = ceil_div(e - i, wb);
            if (pack && k[i] == ~0ull && i > 0 && k[i - 1] == ~0ull) wn = 0;
        }
        words[i] = wn;
    }
}

// the variant position of every variant kmer (sorted index q -> word of its
// group + offset): perm over the combined dictionary's variant ranks
__global__ void group_pos_kernel(const uint64_t* __restrict__ k, const int32_t* __restrict__ order, int64_t n,
                                 const int64_t* __restrict__ wstart, int wb, int pack, uint32_t base,
                                 uint32_t* __restrict__ mpos) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        // the group's head: the first index with the same key (keyless: the first keyless)
        int64_t lo = 0, hi = i;
        const uint64_t key = k[i];
        if (!pack && key == ~0ull) {                         // a keyless kmer's own word
            mpos[order[i]] = base + (uint32_t)(wstart[i] * wb);
            continue;
        }
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (k[mid] < key) lo = mid + 1; else hi = mid;
        }
        mpos[order[i]] = base + (uint32_t)(wstart[lo] * wb + (i - lo));
    }
}

// combined perm over the dictionary (dense + variant ranks in code order)
__global__ void combine_perm_kernel(const int32_t* __restrict__ dense, const int64_t* __restrict__ dpos,
                                    const int64_t* __restrict__ mpos_idx, int64_t n,
                                    const uint32_t* __restrict__ dperm, const uint32_t* __restrict__ mperm,
                                    uint32_t* __restrict__ perm) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += stride)
        perm[r] = dense[r] ? (dperm ? dperm[dpos[r]] : (uint32_t)dpos[r]) : mperm[mpos_idx[r]];
}

// ---- the hash fill --------------------------------------------------------
// The windowed fill (bitset.hip fill_pos_kernel) stages a stretch of the
// sorted dictionary per segment of a set's codes: made for dictionaries about
// the size of a set (C2: 4 M each). C4's dictionary of kmers held by >= 2
// sets is 377 M codes against 200 K per set, so every segment's windows spill
// to global walks (25 s). Here every code of the dictionary goes into an
// open-addressing table (linear probing, load <= 1/2, 16-byte slots
// {code, tagged value}) and each set's codes probe it: one or two lines per
// code, coalesced reads of the codes. Values: kPosTag | bit position (dense
// or variant), kRareTag | rare rank.
constexpr unsigned long long kHashEmpty = ~0ull;
constexpr unsigned long long kPosTag = 1ull << 62, kRareTag = 2ull << 62, kTagMask = 3ull << 62;

__device__ __forceinline__ unsigned long long hmix(unsigned long long x) {
    x ^= x >> 33;
    x *= 0xFF51AFD7ED558CCDull;
    x ^= x >> 33;
    x *= 0xC4CEB9FE1A85EC53ull;
    x ^= x >> 33;
    return x;
}

// inserts codes[0, n) with values tag | (perm ? perm[i] : i). The code ~0
// (64-bit codes: DNA k = 32's poly-T, 8-bit protein k = 8) is the empty
// marker, so it lives out of band: tab[2 (mask + 1)] = 1 when present,
// tab[2 (mask + 1) + 1] = its value
__global__ void hash_insert_kernel(const uint64_t* __restrict__ codes, int64_t n, const uint32_t* __restrict__ perm,
                                   unsigned long long tag, unsigned long long* __restrict__ tab,
                                   unsigned long long mask) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const unsigned long long code = codes[i];
        const unsigned long long val = tag | (perm ? (unsigned long long)perm[i] : (unsigned long long)i);
        if (code == kHashEmpty) {
            tab[2 * (mask + 1) + 1] = val;
            tab[2 * (mask + 1)] = 1ull;
            continue;
        }
        unsigned long long slot = hmix(code) & mask;
        for (;;) {
            const unsigned long long prev = atomicCAS(tab + 2 * slot, kHashEmpty, code);
            if (prev == kHashEmpty || prev == code) {
                tab[2 * slot + 1] = val;
                break;
            }
            slot = (slot + 1) & mask;
        }
    }
}

// one workgroup per set of the chunk: every code probes the table; positions
// go to pos (u32, ~0: not dense / variant), rare codes append their record
// (rare rank << 32 | set + id_base), staged in LDS and appended with one
// atomic per kProbeBuf records (C3: one atomic per wave and round on a single
// counter was 5 M same-address atomics, ~60 ms)
constexpr int kProbeBuf = 2048;
__device__ __forceinline__ void probe_flush(unsigned long long* s_rb, unsigned* s_n, unsigned long long* s_g,
                                            unsigned long long* __restrict__ rare_out,
                                            unsigned long long* __restrict__ rare_cnt, int64_t rare_cap) {
    const unsigned n = *s_n;                                   // uniform: read after a barrier
    if (!n) return;
    if (threadIdx.x == 0) *s_g = atomicAdd(rare_cnt, (unsigned long long)n);
    __syncthreads();
    const unsigned long long g = *s_g;
    for (unsigned j = threadIdx.x; j < n; j += blockDim.x)
        if ((int64_t)(g + j) < rare_cap) rare_out[g + j] = s_rb[j];
    __syncthreads();
    if (threadIdx.x == 0) *s_n = 0;
    __syncthreads();
}

__global__ __launch_bounds__(256) void hash_probe_kernel(const uint64_t* __restrict__ codes,
                                                         const int64_t* __restrict__ off, int64_t s0, int64_t base,
                                                         const unsigned long long* __restrict__ tab,
                                                         unsigned long long mask, uint32_t* __restrict__ pos,
                                                         int64_t id_base, unsigned long long* __restrict__ rare_out,
                                                         unsigned long long* __restrict__ rare_cnt, int64_t rare_cap) {
    __shared__ unsigned long long s_rb[kProbeBuf];
    __shared__ unsigned s_n;
    __shared__ unsigned long long s_g;
    const int64_t set = s0 + blockIdx.x;
    const int lane = threadIdx.x & 63;
    const int64_t b = off[set], e = off[set + 1];
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    for (int64_t x0 = b; x0 < e; x0 += 256) {
        const int64_t x = x0 + threadIdx.x;
        unsigned long long val = kHashEmpty;
        if (x < e) {
            const unsigned long long code = codes[x];
            if (code == kHashEmpty) {                          // out of band (hash_insert_kernel)
                if (tab[2 * (mask + 1)] == 1ull) val = tab[2 * (mask + 1) + 1];
            } else {
                unsigned long long slot = hmix(code) & mask;
                for (;;) {
                    const ulonglong2 kv = *reinterpret_cast<const ulonglong2*>(tab + 2 * slot);
                    if (kv.x == code) { val = kv.y; break; }
                    if (kv.x == kHashEmpty) break;
                    slot = (slot + 1) & mask;
                }
            }
            pos[x - base] = (val != kHashEmpty && (val & kTagMask) == kPosTag) ? (uint32_t)(val & 0xFFFFFFFFull) : ~0u;
        }
        const bool rhit = val != kHashEmpty && (val & kTagMask) == kRareTag;
        const unsigned long long m = __ballot(rhit);
        if (m) {
            unsigned b0 = 0;
            if (lane == __ffsll((long long)m) - 1) b0 = atomicAdd(&s_n, (unsigned)__popcll(m));
            b0 = (unsigned)__shfl((int)b0, __ffsll((long long)m) - 1, 64);
            if (rhit)
                s_rb[b0 + __popcll(m & ((1ull << lane) - 1))] =
                    ((val & 0xFFFFFFFFull) << 32) | (unsigned long long)(uint32_t)(set + id_base);
        }
        __syncthreads();
        if (s_n > (unsigned)(kProbeBuf - 256)) probe_flush(s_rb, &s_n, &s_g, rare_out, rare_cnt, rare_cap);
    }
    probe_flush(s_rb, &s_n, &s_g, rare_out, rare_cnt, rare_cap);
}

// ---- variant records of one fill chunk -----------------------------------
// per set of the chunk: its variant positions (>= vbase) counted, then
// written as keys (word << (sbits + 6) | set << 6 | bit), word = q / wb and
// bit = q mod wb for words of wb kmers (shifts when wb = 2^lg, lg >= 0)
__global__ __launch_bounds__(256) void vrec_count_kernel(const uint32_t* __restrict__ pos,
                                                         const int64_t* __restrict__ off, int64_t s0, int64_t base,
                                                         uint32_t vbase, int64_t* __restrict__ cnt) {
    __shared__ int64_t red[256];
    const int64_t i = s0 + blockIdx.x;
    int64_t c = 0;
    for (int64_t x = off[i] - base + threadIdx.x; x < off[i + 1] - base; x += 256) {
        const uint32_t p = pos[x];
        c += p != ~0u && p >= vbase;
    }
    red[threadIdx.x] = c;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) cnt[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(256) void vrec_write_kernel(const uint32_t* __restrict__ pos,
                                                         const int64_t* __restrict__ off, int64_t s0, int64_t base,
                                                         uint32_t vbase, int sbits, int lg, uint32_t wb,
                                                         const int64_t* __restrict__ at, uint64_t* __restrict__ out) {
    __shared__ int64_t wbase;
    const int64_t i = s0 + blockIdx.x;
    const int lane = threadIdx.x & 63;
    if (threadIdx.x == 0) wbase = at[blockIdx.x];
    __syncthreads();
    const int64_t b = off[i] - base, e = off[i + 1] - base;
    for (int64_t x0 = b; x0 < e; x0 += 256) {
        const int64_t x = x0 + threadIdx.x;
        const uint32_t p = x < e ? pos[x] : ~0u;
        const bool hit = p != ~0u && p >= vbase;
        const unsigned long long m = __ballot(hit);
        int64_t slot = 0;
        if (m) {
            if (lane == __ffsll((long long)m) - 1)
                slot = (int64_t)atomicAdd(reinterpret_cast<unsigned long long*>(&wbase), (unsigned long long)__popcll(m));
            slot = (int64_t)__shfl((long long)slot, __ffsll((long long)m) - 1, 64);
        }
        if (hit) {
            const uint64_t q = p - vbase;
            out[slot + __popcll(m & ((1ull << lane) - 1))] =
                (lg >= 0 ? ((q >> lg) << (sbits + 6)) | ((uint64_t)i << 6) | (q & ((1u << lg) - 1))
                         : ((q / wb) << (sbits + 6)) | ((uint64_t)i << 6) | (q % wb));
        }
        __syncthreads();
    }
}

// OR the bits of each (word, set) run of sorted records: (word << sbits | set, mask)
__global__ void vrec_heads_kernel(const uint64_t* __restrict__ k, int64_t n, int32_t* __restrict__ flag) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        flag[i] = (i == 0 || (k[i] >> 6) != (k[i - 1] >> 6)) ? 1 : 0;
}

__global__ void vrec_or_kernel(const uint64_t* __restrict__ k, int64_t n, const int32_t* __restrict__ flag,
                               const int64_t* __restrict__ pos, uint64_t* __restrict__ ekey,
                               unsigned long long* __restrict__ emask) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (!flag[i]) continue;
        const uint64_t h = k[i] >> 6;
        unsigned long long m = 0;
        for (int64_t e = i; e < n && (k[e] >> 6) == h; e++) m |= 1ull << (k[e] & 63);
        ekey[pos[i]] = h;
        emask[pos[i]] = m;
    }
}

// ---- entries -> word lists and the set side ------------------------------
__global__ void entry_fields_kernel(const uint64_t* __restrict__ key, const int32_t* __restrict__ idx, int64_t E,
                                    int sbits, const unsigned long long* __restrict__ mask_in,
                                    uint32_t* __restrict__ vset, unsigned long long* __restrict__ vmask) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += stride) {
        const uint32_t set = (uint32_t)(key[e] & ((1ull << sbits) - 1));
        vset[e] = set;
        vmask[e] = mask_in[idx[e]];
    }
}

// set-side keys (set, entry)
__global__ void set_keys_kernel(const uint32_t* __restrict__ vset, int64_t E, uint64_t* __restrict__ skey) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += stride)
        skey[e] = ((uint64_t)vset[e] << 32) | (uint64_t)e;
}

// word w's list = entries [woff[w], woff[w + 1])
__global__ void word_offsets_kernel(const uint64_t* __restrict__ key, int64_t E, int sbits, int64_t nw,
                                    int64_t* __restrict__ woff) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w <= nw; w += stride) {
        int64_t lo = 0, hi = E;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if ((int64_t)(key[mid] >> sbits) < w) lo = mid + 1; else hi = mid;
        }
        woff[w] = lo;
    }
}

__global__ void entry_bounds_kernel(const uint64_t* __restrict__ key, int64_t E, int sbits,
                                    const int64_t* __restrict__ woff, uint32_t* __restrict__ beg,
                                    uint32_t* __restrict__ end) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += stride) {
        const int64_t w = (int64_t)(key[e] >> sbits);
        beg[e] = (uint32_t)woff[w];
        end[e] = (uint32_t)woff[w + 1];
    }
}

__global__ void set_offsets_kernel(const uint64_t* __restrict__ skey, int64_t E, int64_t nsets, int sh,
                                   int64_t* __restrict__ soff, uint32_t* __restrict__ sent) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= nsets; i += stride) {
        int64_t lo = 0, hi = E;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if ((int64_t)(skey[mid] >> sh) < i) lo = mid + 1; else hi = mid;
        }
        soff[i] = lo;
    }
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += stride) sent[e] = (uint32_t)(skey[e] & 0x7FFFFFFFull);
}

// products of the tier: sum over words of z (z - 1) / 2, and the longest list
__global__ void word_products_kernel(const int64_t* __restrict__ woff, int64_t nw,
                                     unsigned long long* __restrict__ out) {
    unsigned long long acc = 0, mx = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) {
        const unsigned long long z = (unsigned long long)(woff[w + 1] - woff[w]);
        acc += z * (z - (z ? 1 : 0)) / 2;
        mx = z > mx ? z : mx;
    }
    for (int o = 32; o > 0; o >>= 1) {
        acc += __shfl_xor(acc, o, 64);
        const unsigned long long v = __shfl_xor(mx, o, 64);
        mx = v > mx ? v : mx;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(out, acc);
        atomicMax(out + 1, mx);
    }
}

// (set | mask << 16) of every entry of a 16-kmer-word tier of <= 65,536 sets
__global__ void pack_entries_kernel(const uint32_t* __restrict__ vset, const unsigned long long* __restrict__ vmask,
                                    int64_t E, uint32_t* __restrict__ pack) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += stride)
        pack[e] = (vset[e] & 0xFFFFu) | ((uint32_t)(vmask[e] & 0xFFFFull) << 16);
}

// 47-kmer words of < 2^17 sets: every entry in one 8-byte member (set << 47
// | mask) for the wave-per-entry walk (C4: 12 -> 8 bytes a product)
__global__ void pack64_entries_kernel(const uint32_t* __restrict__ vset, const unsigned long long* __restrict__ vmask,
                                      int64_t E, unsigned long long* __restrict__ pk) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += stride)
        pk[e] = ((unsigned long long)vset[e] << 47) | (vmask[e] & ((1ull << 47) - 1));
}

// the short walk's set-side records, coalesced by the set's position: entry
// e (31 bits) | the members after it, end - e (17 bits) | its position in its
// list, e - beg (16 bits): a row reads no random bounds (lists of <= 65,536
// sets)
__global__ void pack_set_side_kernel(const uint32_t* __restrict__ sent, const uint32_t* __restrict__ beg,
                                     const uint32_t* __restrict__ end, int64_t E, uint64_t* __restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < E; x += stride) {
        const uint64_t e = sent[x];
        out[x] = e | ((uint64_t)(end[e] - e) << 31) | ((uint64_t)(e - beg[e]) << 48);
    }
}

// max over sets of the popcounts of their entries' masks
__global__ void row_vweight_kernel(const int64_t* __restrict__ soff, const uint32_t* __restrict__ sent,
                                   const unsigned long long* __restrict__ vmask, int64_t nsets,
                                   unsigned long long* __restrict__ out) {
    unsigned long long mx = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nsets; i += stride) {
        unsigned long long w = 0;
        for (int64_t x = soff[i]; x < soff[i + 1]; x++) w += (unsigned long long)__popcll(vmask[sent[x]]);
        mx = w > mx ? w : mx;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long v = __shfl_xor(mx, o, 64);
        mx = v > mx ? v : mx;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(out, mx);
}

}  // namespace

// ---- the walk --------------------------------------------------------------
constexpr int VCH = 16384;   // columns per LDS chunk (64 KiB of counters)

namespace {
// grid = rows x nsplit slices of the row's entries. A workgroup takes its
// entries in batches of VBATCH and walks the column chunks in order; each
// entry's list position is kept in LDS between chunks (lists are sorted by
// set), so a list is read once across all chunks and no chunk searches it.
constexpr int VBATCH = 2048;
// C16 (round 5, option variant_c16, default): 16-bit counters, two to a dword, so a
// chunk is 32,768 columns (C4's 100,000 in 4 chunks instead of 7: fewer
// (entry, chunk) visits, fuller 64-member steps); a batch then holds at most
// 1,023 entries, so a pair's count in it is at most 1,023 x 64 < 2^16 (a
// set holds one entry per word, and each entry adds at most 64).
// PK (round 5): members packed as set << 47 | mask (47-kmer words of < 2^17
// sets, vw_pk64): one 8-byte load a member instead of 4 + 8
template <bool C16, bool PK = false>
__global__ __launch_bounds__(1024) void variant_rows_kernel(const int64_t* __restrict__ soff,
                                                           const uint32_t* __restrict__ sent,
                                                           const uint32_t* __restrict__ vset,
                                                           const unsigned long long* __restrict__ vmask,
                                                           const unsigned long long* __restrict__ vpk,
                                                           const uint32_t* __restrict__ vbeg,
                                                           const uint32_t* __restrict__ vend, int64_t r0, int64_t r1,
                                                           int64_t c0, int64_t c1, int nsplit, int upper,
                                                           int32_t* __restrict__ I, int64_t ldI) {
    constexpr int CH = C16 ? 2 * VCH : VCH, VB = C16 ? 1023 : VBATCH;
    __shared__ int32_t cnt[VCH];
    __shared__ uint32_t ypos[VB];
    const int64_t i = r0 + blockIdx.x / nsplit;
    const int split = blockIdx.x % nsplit;
    if (i >= r1) return;
    const int64_t lo = upper && i + 1 > c0 ? i + 1 : c0;      // first column of the row
    if (lo >= c1) return;
    const int64_t rb = soff[i], re = soff[i + 1];
    const int64_t per = (re - rb + nsplit - 1) / nsplit;
    const int64_t xb = rb + per * split;
    const int64_t xe = xb + per < re ? xb + per : re;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, nwv = (int)(blockDim.x >> 6);
    int32_t* row = I + (i - r0) * ldI - c0;                   // row[j] for column j
    for (int64_t bb = xb; bb < xe; bb += VB) {
        const int nb = (int)(xe - bb < VB ? xe - bb : VB);
        // each entry's first list position at or past the row's first column
        // (upper: the members after the row's own entry)
        for (int t = wv; t < nb; t += nwv) {
            const uint32_t e = sent[bb + t];
            int64_t y = upper ? (int64_t)e + 1 : (int64_t)vbeg[e];
            const int64_t ye = vend[e];
            if (!upper || lo > i + 1) {                        // columns below lo: one search
                int64_t a = y, z = ye;
                while (a < z) {
                    const int64_t mid = (a + z) >> 1;
                    const int64_t js = PK ? (int64_t)(vpk[mid] >> 47) : (int64_t)vset[mid];
                    if (js < lo) a = mid + 1; else z = mid;
                }
                y = a;
            }
            if (lane == 0) ypos[t] = (uint32_t)y;
        }
        for (int64_t cb = lo - ((lo - c0) % CH); cb < c1; cb += CH) {
            const int64_t ce = cb + CH < c1 ? cb + CH : c1;
            const int n = (int)(ce - cb);
            __syncthreads();                                   // ypos written; previous chunk flushed
            for (int t = threadIdx.x; t < (C16 ? (n + 1) >> 1 : n); t += blockDim.x) cnt[t] = 0;
            __syncthreads();
            for (int t = wv; t < nb; t += nwv) {                 // a wave per entry
                const uint32_t e = sent[bb + t];
                constexpr unsigned long long M47 = (1ull << 47) - 1;
                const unsigned long long mi = PK ? (vpk[e] & M47) : vmask[e];
                const int64_t ye = vend[e];
                int64_t y = ypos[t];
                // member y: (set, mask) from one packed load or two
                auto member = [&](int64_t yy, uint32_t& jj, unsigned long long& mm) {
                    if (PK) {
                        const unsigned long long p = yy < ye ? vpk[yy] : ~0ull;
                        jj = yy < ye ? (uint32_t)(p >> 47) : 0xFFFFFFFFu;
                        mm = p & M47;
                    } else {
                        jj = yy < ye ? vset[yy] : 0xFFFFFFFFu;
                        mm = yy < ye ? vmask[yy] : 0ull;
                    }
                };
                if (y < ye) {
                    // the next 64 members are loaded before this step's are
                    // counted (two steps of loads in flight a wave; round 5:
                    // the walk waited out one load round trip per 64 members)
                    int64_t yy = y + lane;
                    uint32_t j;
                    unsigned long long mj;
                    member(yy, j, mj);
                    for (;;) {
                        const bool in = yy < ye && (int64_t)j < ce;
                        const int64_t yn = yy + 64;
                        uint32_t jn;
                        unsigned long long mn;
                        member(yn, jn, mn);
                        if (in && (int64_t)j != i) {
                            const int v = __popcll(mi & mj);
                            if (v) {
                                if (C16) atomicAdd(&cnt[(j - cb) >> 1], v << (((j - cb) & 1) << 4));
                                else atomicAdd(&cnt[j - cb], v);
                            }
                        }
                        const unsigned long long m = __ballot(in);
                        y += __popcll(m);                      // lists ascend: the in-chunk members come first
                        if (m != ~0ull) break;
                        yy = yn;
                        j = jn;
                        mj = mn;
                    }
                }
                if (lane == 0) ypos[t] = (uint32_t)y;
            }
            __syncthreads();
            for (int t = threadIdx.x; t < n; t += blockDim.x) {
                const int v = C16 ? (int)(((uint32_t)cnt[t >> 1] >> ((t & 1) << 4)) & 0xFFFFu) : cnt[t];
                if (v && cb + t >= lo) atomicAdd(row + cb + t, v);
            }
        }
    }
}

// one query set q against every set: cnt[t] += shared variant kmers (global atomics)
__global__ __launch_bounds__(256) void variant_query_kernel(const int64_t* __restrict__ soff,
                                                            const uint32_t* __restrict__ sent,
                                                            const uint32_t* __restrict__ vset,
                                                            const unsigned long long* __restrict__ vmask,
                                                            const uint32_t* __restrict__ vbeg,
                                                            const uint32_t* __restrict__ vend, int64_t q,
                                                            int32_t* __restrict__ cnt) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t x = soff[q] + wave; x < soff[q + 1]; x += waves) {
        const uint32_t e = sent[x];
        const unsigned long long mi = vmask[e];
        for (int64_t y = (int64_t)vbeg[e] + lane; y < (int64_t)vend[e]; y += 64) {
            const uint32_t j = vset[y];
            const int v = __popcll(mi & vmask[y]);
            if ((int64_t)j != q && v) atomicAdd(cnt + j, v);
        }
    }
}
// Short-list walk of a grouped rare tier (round 5; C3: 22.7 M entries whose
// word lists hold ~20 sets). The wave-per-entry walk above leaves most of a
// wave's 64 lanes idle on such lists; here, as in the rare tier's row walk
// (bitset.hip rare_rows_kernel), a thread takes one entry of the row and
// walks its list from the row's own position (upper triangle) four packed
// members (set | mask << 16) a 16-byte load, adding popc(mask_i & mask_j)
// into LDS counters of one column chunk; lists of kLongList+ entries are
// walked by the whole wave. Grid: rows x column chunks x nsplit slices of the
// row's entries; the chunk's counters are added to I's row once (atomics:
// the other families add beside it). C16: two 16-bit counters a dword
// (vw_row_wmax < 2^16 bounds every pair's count).
constexpr int VSCH = 16384;   // columns per LDS chunk
template <int NT, bool C16>
__global__ __launch_bounds__(NT) void variant_short_kernel(const int64_t* __restrict__ soff,
                                                           const uint64_t* __restrict__ spent,
                                                           const uint32_t* __restrict__ vpack, int64_t r0, int64_t r1,
                                                           int64_t c0, int64_t c1, int nch, int nsplit, int upper,
                                                           int32_t* __restrict__ I, int64_t ldI) {
    extern __shared__ int32_t vcnt[];
    const int64_t unit = blockIdx.x / nsplit;
    const int split = blockIdx.x % nsplit;
    const int64_t i = r0 + unit / nch;
    const int ch = (int)(unit % nch);
    const int64_t cb = c0 + (int64_t)ch * VSCH;
    const int64_t ce = cb + VSCH < c1 ? cb + VSCH : c1;
    if (i >= r1 || cb >= ce || (upper && ce - 1 <= i)) return;
    const int n = (int)(ce - cb);
    const int nw = C16 ? (n + 1) >> 1 : n;
    for (int t = threadIdx.x; t < nw; t += NT) vcnt[t] = 0;
    __syncthreads();
    auto add = [&](int64_t t, int32_t v) {
        if (C16) atomicAdd(&vcnt[(t - cb) >> 1], v << (((t - cb) & 1) << 4));
        else atomicAdd(&vcnt[t - cb], v);
    };
    const int64_t lo = upper && i + 1 > cb ? i + 1 : cb;
    const int64_t rb = soff[i], re = soff[i + 1];
    const int64_t per = (re - rb + nsplit - 1) / nsplit;
    const int64_t xb = rb + per * split;
    const int64_t xe = xb + per < re ? xb + per : re;
    const int lane = threadIdx.x & 63;
    // an entry's (list start, end, own mask) from its set-side record
    auto decode = [&](uint64_t r, int64_t& b, int64_t& ee) -> int64_t {
        const int64_t e = (int64_t)(r & 0x7FFFFFFFull);
        b = upper ? e + 1 : e - (int64_t)(r >> 48);
        ee = e + (int64_t)((r >> 31) & 0x1FFFFull);
        return e;
    };
    auto count4 = [&](const uint32_t* mem, int64_t y, int64_t ee, uint32_t mi) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int64_t t = mem[u] & 0xFFFFu;
            const int v = __popc(mi & (mem[u] >> 16));
            if (y + u < ee && v && t >= lo && t < ce && t != i) add(t, v);
        }
    };
    auto long_lists = [&](int64_t b, int64_t ee, uint32_t mi) {        // the wave walks them
        const bool lng = ee - b >= kLongList;
        for (unsigned long long m = __ballot(lng); m; m &= m - 1) {
            const int l = __ffsll((long long)m) - 1;
            const int64_t lb = __shfl((long long)b, l, 64), le = __shfl((long long)ee, l, 64);
            const uint32_t lm = (uint32_t)__shfl((int)mi, l, 64);
            for (int64_t y = lb + lane; y < le; y += 64) {
                const uint32_t p = vpack[y];
                const int64_t t = p & 0xFFFFu;
                const int v = __popc(lm & (p >> 16));
                if (v && t >= lo && t < ce && t != i) add(t, v);
            }
        }
        return lng;
    };
    for (int64_t xbase = xb; xbase < xe; xbase += NT) {          // wave-uniform trip count
        const int64_t x = xbase + threadIdx.x;
        int64_t b = 0, ee = 0;
        uint32_t mi = 0;
        if (x < xe) {
            // (entry, members after it, position in its list): coalesced; the
            // entry's own mask shares a line with its list's next members
            const int64_t e = decode(spent[x], b, ee);
            mi = vpack[e] >> 16;
        }
        if (long_lists(b, ee, mi)) continue;
#pragma unroll 2
        for (int64_t y = b; y < ee; y += 4) {
            uint32_t mem[4];
            __builtin_memcpy(mem, vpack + y, 16);                 // the array is padded past its end
            count4(mem, y, ee, mi);
        }
    }
    __syncthreads();
    int32_t* row = I + (i - r0) * ldI + (cb - c0);
    for (int t = threadIdx.x; t < n; t += NT) {
        const int v = C16 ? (int)(((uint32_t)vcnt[t >> 1] >> ((t & 1) << 4)) & 0xFFFFu) : vcnt[t];
        if (v && cb + t >= lo) atomicAdd(row + t, v);
    }
}

// the first index of a sorted key array holding ~0 (n if none): one thread
__global__ void first_keyless_kernel(const uint64_t* __restrict__ k, int64_t n, int64_t* __restrict__ out) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (k[mid] != ~0ull) lo = mid + 1; else hi = mid;
    }
    *out = lo;
}

// Keyless variant kmers routed to the rare tier (round 6, option
// variant_keyless_rare): flag[idx[t]] = 1 for the routed variant indices
__global__ void mark_idx_kernel(const int32_t* __restrict__ idx, int64_t n, int32_t* __restrict__ flag) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += stride) flag[idx[t]] = 1;
}
// g[i] = 1 for the dictionary codes that are routed variant kmers
__global__ void routed_flags_kernel(const int32_t* __restrict__ fm, const int64_t* __restrict__ pm,
                                    const int32_t* __restrict__ kl, int64_t U, int32_t* __restrict__ g) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < U; i += stride)
        g[i] = fm[i] && kl[pm[i]] ? 1 : 0;
}
// the routed codes appended to the rare codes (ranks Ur + gp[i]) and their
// holders counted (the rare records they will write): a sum per wave, one
// atomic a wave
__global__ __launch_bounds__(256) void routed_emit_kernel(const uint64_t* __restrict__ dict,
                                                          const uint32_t* __restrict__ dcnt,
                                                          const int32_t* __restrict__ g, const int64_t* __restrict__ gp,
                                                          int64_t U, uint64_t* __restrict__ out,
                                                          unsigned long long* __restrict__ msum) {
    unsigned long long c = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < U; i += stride)
        if (g[i]) {
            out[gp[i]] = dict[i];
            c += dcnt[i];
        }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(msum, c);
}

__global__ void viota_kernel(int32_t* __restrict__ p, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = (int32_t)i;
}
}  // namespace

// ---- host --------------------------------------------------------------------

// Summary of the collection's codes held by >= min_count sets, by ranges of
// the code space (P splitters from a sample of every set's codes): one range
// of every set gathered, sorted, counted at a time.
void range_summary(gdist_ctx* ctx, const gdist_sets* s, int min_count, Summary& out, BuildSplit& sp) {
    hipStream_t st = ctx->stream;
    Trace tr(st, ctx->trace());
    const int cbits = std::min(64, code_bits(s->kind, s->k, s->flags));
    const int64_t N = s->nsets, total = s->total;
    // ranges of at most ~2^28 codes (about 4 GiB of sort buffers), at least
    // one per share of a split build; the sample and so the splitters are the
    // same on every rank (the same codes)
    const int64_t target = int64_t(1) << 28;
    const int P = (int)std::max<int64_t>(sp.R, std::min<int64_t>(4096, ceil_div(total, target)));
    std::vector<uint64_t> split;
    if (P > 1) {
        // sample: the codes at a stride (every set's codes are sorted, so
        // the sample spans each set's range), sorted on the host
        const int64_t want = std::min<int64_t>(total, (int64_t)P * 256);
        const int64_t stride = std::max<int64_t>(1, total / std::max<int64_t>(1, want));
        const int64_t ns = ceil_div(total - stride / 2, stride);
        DevBuf dsm(ns * 8 + 8, st);
        sample_kernel<<<grid_for(ns), 256, 0, st>>>(s->codes.as<uint64_t>(), stride / 2, stride, ns,
                                                    dsm.as<uint64_t>());
        GD_HIP(hipGetLastError());
        std::vector<uint64_t> smp(ns);
        d2h(smp.data(), dsm.p, ns * 8, st);
        std::sort(smp.begin(), smp.end());
        for (int p = 1; p < P; p++) {
            const uint64_t v = smp.empty() ? 0 : smp[std::min<size_t>(smp.size() - 1, smp.size() * p / P)];
            if (split.empty() || v > split.back()) split.push_back(v);
        }
    }
    const int Pe = (int)split.size() + 1;
    DevBuf dsplit(std::max<size_t>(1, split.size()) * 8, st), spos((size_t)N * (Pe + 1) * 8, st);
    if (!split.empty()) h2d(dsplit.p, split.data(), split.size() * 8, st);
    range_pos_kernel<<<(unsigned)ceil_div(N * (Pe + 1), 256), 256, 0, st>>>(
        s->codes.as<uint64_t>(), s->off.as<int64_t>(), N, dsplit.as<uint64_t>(), Pe, spos.as<int64_t>());
    GD_HIP(hipGetLastError());
    std::vector<Summary> parts;
    DevBuf cnt((N + 1) * 8, st), at((N + 1) * 8, st);
    int64_t kept = 0;
    // one code range of every set gathered, sorted, counted, the kept runs emitted
    auto count_range = [&](int p) {
        range_sizes_kernel<<<(unsigned)ceil_div(N, 256), 256, 0, st>>>(spos.as<int64_t>(), N, Pe, p,
                                                                       cnt.as<int64_t>());
        GD_HIP(hipMemsetAsync(cnt.as<int64_t>() + N, 0, 8, st));
        exclusive_scan_i64(ctx, cnt.as<int64_t>(), at.as<int64_t>(), (size_t)(N + 1));
        int64_t n = 0;
        d2h(&n, at.as<int64_t>() + N, 8, st);
        Summary part;
        if (n > 0) {
            DevBuf kA(n * 8 + 8, st), kB(n * 8 + 8, st);
            range_gather_kernel<<<(unsigned)N, 256, 0, st>>>(s->codes.as<uint64_t>(), spos.as<int64_t>(), Pe, p,
                                                             at.as<int64_t>(), kA.as<uint64_t>());
            GD_HIP(hipGetLastError());
            uint64_t* keys = kA.as<uint64_t>(); uint64_t* alt = kB.as<uint64_t>();
            sort_keys_u64(ctx, keys, alt, (size_t)n, 0, cbits);
            DevBuf flag(n * 4 + 4, st), keep(n * 4 + 4, st), len(n * 4 + 4, st), pos(n * 8 + 8, st);
            heads_kernel<<<grid_for(n), 256, 0, st>>>(keys, n, flag.as<int32_t>());
            run_keep_kernel<<<grid_for(n), 256, 0, st>>>(keys, n, flag.as<int32_t>(), min_count, keep.as<int32_t>(),
                                                         len.as<uint32_t>());
            GD_HIP(hipGetLastError());
            exclusive_scan_i32_to_i64(ctx, keep.as<int32_t>(), pos.as<int64_t>(), (size_t)n);
            int64_t last = 0;
            int32_t lf = 0;
            d2h(&last, pos.as<int64_t>() + n - 1, 8, st);
            d2h(&lf, keep.as<int32_t>() + n - 1, 4, st);
            part.n = last + lf;
            part.codes.alloc(part.n * 8 + 8, st);
            part.counts.alloc(part.n * 4 + 4, st);
            run_emit_kernel<<<grid_for(n), 256, 0, st>>>(keys, keep.as<int32_t>(), len.as<uint32_t>(),
                                                         pos.as<int64_t>(), n, part.codes.as<uint64_t>(),
                                                         part.counts.as<uint32_t>());
            GD_HIP(hipGetLastError());
            GD_HIP(hipStreamSynchronize(st));
        }
        kept += part.n;
        parts.push_back(std::move(part));
    };
    for (int r = sp.first(); r < sp.last(); r++) {
        ShareClock clk(sp, r, st);
        for (int p = (int)((int64_t)Pe * r / sp.R); p < (int)((int64_t)Pe * (r + 1) / sp.R); p++) count_range(p);
    }
    // ranges ascend (shares too): the parts concatenate in code order
    out.n = kept;
    out.codes.alloc(kept * 8 + 8, st);
    out.counts.alloc(kept * 4 + 4, st);
    int64_t o = 0;
    for (auto& pt : parts) {
        if (pt.n) {
            GD_HIP(hipMemcpyAsync(out.codes.as<uint64_t>() + o, pt.codes.p, pt.n * 8, hipMemcpyDeviceToDevice, st));
            GD_HIP(hipMemcpyAsync(out.counts.as<uint32_t>() + o, pt.counts.p, pt.n * 4, hipMemcpyDeviceToDevice, st));
        }
        o += pt.n;
    }
    parts.clear();
    if (sp.real) {
        // the shares of every rank, in rank order: the whole summary
        const int64_t mine = kept;
        kept = allgather_concat(ctx, out.codes, mine, 8);
        allgather_concat(ctx, out.counts, mine, 4);
        out.n = kept;
    }
    GD_HIP(hipStreamSynchronize(st));
    if (ctx->trace())
        fprintf(stderr, "gdist: range summary: %d code ranges in %d shares, %lld codes held by >= %d sets\n", Pe, sp.R,
                (long long)kept, min_count);
    tr.mark("variant: range summary");
}

static CodeGeom code_geom(const gdist_sets* s) {
    CodeGeom g;
    g.k = s->k;
    const unsigned am = s->flags & GDIST_AMBIG_MASK;
    if (s->kind == GDIST_DNA) {
        const bool keep = am == GDIST_AMBIG_KEEP;
        g.bits = keep ? 3 : 2;
        g.strands = (s->flags & GDIST_STRAND_MASK) == GDIST_STRAND_BOTH ? 2 : 1;
        if (keep) {   // A0 C1 G2 N3 R4 T5 Y6
            const uint8_t a[7] = {0, 1, 2, 3, 4, 5, 6};
            const int8_t c[7] = {5, 2, 1, 3, 6, 0, 4};
            g.nalpha = 7;
            memcpy(g.alpha, a, 7);
            memcpy(g.comp, c, 7);
        } else {      // A0 C1 G2 T3
            const uint8_t a[4] = {0, 1, 2, 3};
            const int8_t c[4] = {3, 2, 1, 0};
            g.nalpha = 4;
            memcpy(g.alpha, a, 4);
            memcpy(g.comp, c, 4);
        }
    } else {
        g.strands = 1;
        if (s->k <= 8) {   // raw bytes: the 20 standard residues
            g.bits = 8;
            const char* aa = "ACDEFGHIKLMNPQRSTVWY";
            g.nalpha = 20;
            for (int i = 0; i < 20; i++) g.alpha[i] = (uint8_t)aa[i];
        } else {           // 5-bit: * 0, A..Z 1..26
            g.bits = 5;
            const char* aa = "ACDEFGHIKLMNPQRSTVWY";
            g.nalpha = 20;
            for (int i = 0; i < 20; i++) g.alpha[i] = (uint8_t)(aa[i] - 'A' + 1);
        }
    }
    return g;
}

// The fill by hash probes (above): dense bits, rare records (rank << 32 |
// set + id_base) and, through the hook, the variant records of every chunk of
// sets. The variant build's fill, and the two-tier build's when the sets are
// sparse against the dictionary (bitset.hip fill_bits: C3)
void hash_fill(gdist_ctx* ctx, const gdist_sets* s, const uint64_t* dict, int64_t U, const uint32_t* perm,
               const uint64_t* rare, int64_t Ur, int64_t W, unsigned long long* bits, int64_t id_base,
               unsigned long long* rare_out, int64_t rare_cap, int64_t* rare_written, const FillHook& hook,
               int64_t sa, int64_t sb) {
    hipStream_t st = ctx->stream;
    Trace tr(st, ctx->trace());
    if (sb < 0) sb = s->nsets;
    GD_REQUIRE(0 <= sa && sa <= sb && sb <= s->nsets, "fill set range outside the collection");
    GD_REQUIRE(Ur < (int64_t(1) << 32) && U < (int64_t(1) << 32), "dictionary too large for the hash fill");
    GD_HIP(hipMemsetAsync(bits + (size_t)sa * W, 0, (size_t)(sb - sa) * W * 8, st));
    int64_t cap = 2;
    while (cap < 2 * (U + Ur)) cap <<= 1;                   // load <= 1/2
    DevBuf tab((size_t)cap * 16 + 16, st), rcnt(8, st);                // + the out-of-band slot of code ~0
    GD_HIP(hipMemsetAsync(tab.p, 0xFF, (size_t)cap * 16 + 16, st));
    GD_HIP(hipMemsetAsync(rcnt.p, 0, 8, st));
    const unsigned long long mask = (unsigned long long)cap - 1;
    if (U) hash_insert_kernel<<<grid_for(U, 256, 256 * 64), 256, 0, st>>>(dict, U, perm, kPosTag,
                                                                           tab.as<unsigned long long>(), mask);
    if (Ur) hash_insert_kernel<<<grid_for(Ur, 256, 256 * 64), 256, 0, st>>>(rare, Ur, nullptr, kRareTag,
                                                                             tab.as<unsigned long long>(), mask);
    GD_HIP(hipGetLastError());
    tr.mark("fill: hash table");
    int64_t s0 = sa;
    while (s0 < sb) {
        int64_t s1 = s0 + 1;
        // chunks of <= 2^28 codes: their 1 GiB position buffer and record
        // sorts reuse the code-range summary's cached blocks (fresh device
        // memory costs ~0.2 s a GB: C4's first 2^30-code chunk took 2.8 s)
        while (s1 < sb && s->h_off[s1 + 1] - s->h_off[s0] <= (int64_t(1) << 28)) s1++;
        const int64_t base = s->h_off[s0], n = s->h_off[s1] - base;
        DevBuf pos(std::max<int64_t>(1, n) * 4 + 16, st);
        hash_probe_kernel<<<(unsigned)(s1 - s0), 256, 0, st>>>(s->codes.as<uint64_t>(), s->off.as<int64_t>(), s0, base,
                                                               tab.as<unsigned long long>(), mask, pos.as<uint32_t>(),
                                                               id_base, rare_out, rcnt.as<unsigned long long>(), rare_cap);
        GD_HIP(hipGetLastError());
        if (hook) hook(pos.as<uint32_t>(), s0, s1, base);
        bits_from_positions(ctx, s, pos.as<uint32_t>(), s0, s1, base, W, bits);
        GD_HIP(hipStreamSynchronize(st));
        tr.mark("fill: probes + bits + variant records");
        s0 = s1;
    }
    unsigned long long w = 0;
    d2h(&w, rcnt.p, 8, st);
    GD_REQUIRE((int64_t)w <= rare_cap, "rare-tier record count exceeds its reservation");
    *rare_written = (int64_t)w;
}

int64_t variant_dmin(const gdist_ctx* ctx, int64_t nsets) {
    return ctx->has_option(OPT_VARIANT_DMIN) ? std::max<int64_t>(2, ctx->option(OPT_VARIANT_DMIN, 2))
                                             : std::max<int64_t>(2, nsets / 20);
}

void free_variant(gdist_sets* s) {
    s->variant = false;
    s->vw_pack.release();
    s->vw_pk64.release();
    s->vs_pent.release();
    s->vw_row_wmax = 0;
    s->vw_bits = 64;
    s->vw_words = s->vw_entries = s->vw_kmers = s->vw_dmin = 0;
    s->vw_products = 0.0;
    s->vw_max_list = 0;
    s->vw_set.release();
    s->vw_mask.release();
    s->vw_beg.release();
    s->vw_end.release();
    s->vs_off.release();
    s->vs_ent.release();
}

bool build_variant_bitsets(gdist_ctx* ctx, gdist_sets* s, DevBuf& dict, DevBuf& dcnt, int64_t U, DevBuf& rare,
                           int64_t Ur, int64_t mass, int64_t T, BuildSplit& sp, int64_t dmin_in, int wb, bool probe) {
    hipStream_t st = ctx->stream;
    Trace tr(st, ctx->trace());
    const int64_t N = s->nsets;
    GD_REQUIRE(N < (int64_t(1) << 31), "too many sets for the variant tier");
    GD_REQUIRE(wb == 16 || wb == 47 || wb == 64, "variant words hold 16, 47 or 64 kmers");
    const int lg = wb == 16 ? 4 : wb == 64 ? 6 : -1;
    // keyless kmers (no keyed dense neighbour: two substitutions in a window,
    // or no guide) packed wb to a word in code order (option
    // variant_pack_keyless, default), or each in a word of its own
    // (16-kmer words of the grouped rare tier: packed only while keyless
    // kmers are <= 1/4 of the tier — C3 ~9 % — so that unrelated kmers never
    // make one long list; without locus keys, packed, C3 took 15.1 ms a step)
    int pack = ctx->option(OPT_VARIANT_PACK_KEYLESS, 1) != 0 ? 1 : 0;
    // 2. tiers: dense (>= Dmin) and variant (T .. Dmin - 1), in code order within the dictionary
    const int64_t dmin = dmin_in > 0 ? dmin_in : variant_dmin(ctx, N);
    DevBuf fd(U * 4 + 4, st), fm(U * 4 + 4, st), pd(U * 8 + 8, st), pm(U * 8 + 8, st);
    int64_t Ud = 0, Um = 0;
    if (U) {
        tier_flags_kernel<<<grid_for(U), 256, 0, st>>>(dcnt.as<uint32_t>(), U, (uint32_t)dmin, fd.as<int32_t>(),
                                                       fm.as<int32_t>());
        GD_HIP(hipGetLastError());
        exclusive_scan_i32_to_i64(ctx, fd.as<int32_t>(), pd.as<int64_t>(), (size_t)U);
        exclusive_scan_i32_to_i64(ctx, fm.as<int32_t>(), pm.as<int64_t>(), (size_t)U);
        int64_t h[2];
        int32_t hf[2];
        d2h(&h[0], pd.as<int64_t>() + U - 1, 8, st);
        d2h(&h[1], pm.as<int64_t>() + U - 1, 8, st);
        d2h(&hf[0], fd.as<int32_t>() + U - 1, 4, st);
        d2h(&hf[1], fm.as<int32_t>() + U - 1, 4, st);
        Ud = h[0] + hf[0];
        Um = h[1] + hf[1];
    }
    DevBuf dcodes(Ud * 8 + 8, st), dcounts(Ud * 4 + 4, st), mcodes(Um * 8 + 8, st);
    if (U)
        split_codes_kernel<<<grid_for(U), 256, 0, st>>>(dict.as<uint64_t>(), dcnt.as<uint32_t>(), U, fd.as<int32_t>(),
                                                        pd.as<int64_t>(), pm.as<int64_t>(), dcodes.as<uint64_t>(),
                                                        dcounts.as<uint32_t>(), mcodes.as<uint64_t>());
    GD_HIP(hipGetLastError());
    // 3. dense positions: locus order of the guides (as build_bitsets)
    DevBuf dperm;
    if (s->n_guide > 0 && locus_order_enabled(ctx) && Ud > 0) {
        DevBuf key;
        locus_keys(ctx, s, dcodes.as<uint64_t>(), dcounts.as<uint32_t>(), Ud, 0, key);
        locus_perm(ctx, key, Ud, dperm);
    }
    const int64_t Wd = bitset_words(Ud);
    const uint32_t vbase = (uint32_t)(Wd * 64);
    tr.mark("variant: tiers + dense locus order");
    // 4. variant order: keys from the dense neighbours, groups, words
    DevBuf mperm(Um * 4 + 4, st);
    int64_t vwords = 0;
    if (Um > 0) {
        DevBuf dentry(Ud * 8 + 8, st), vkey(Um * 8 + 8, st), vkalt(Um * 8 + 8, st), ord(Um * 4 + 4, st),
            oalt(Um * 4 + 4, st);
        if (Ud > 0) {
            if (s->n_guide > 0)
                dense_entry_kernel<<<grid_for(Ud), 256, 0, st>>>(dcodes.as<uint64_t>(), Ud, s->guide_codes.as<uint64_t>(),
                                                                 s->guide_keys.as<uint64_t>(), s->n_guide,
                                                                 dentry.as<int64_t>());
            else
                GD_HIP(hipMemsetAsync(dentry.p, 0xFF, Ud * 8, st));
        }
        // option variant_key2 (round 6, default 1): second-level keys for the
        // kmers the first level leaves keyless
        const bool key2 = ctx->option(OPT_VARIANT_KEY2, 1) != 0;
        DevBuf went(key2 ? Um * 8 + 8 : 8, st);
        variant_key_kernel<<<grid_for(Um, 256, 256 * 64), 256, 0, st>>>(mcodes.as<uint64_t>(), Um,
                                                                         dcodes.as<uint64_t>(), Ud,
                                                                         dentry.as<int64_t>(), code_geom(s),
                                                                         key2 ? vkalt.as<uint64_t>() : vkey.as<uint64_t>(),
                                                                         key2 ? went.as<int64_t>() : nullptr);
        GD_HIP(hipGetLastError());
        if (key2) {
            variant_key2_kernel<<<grid_for(Um, 256, 256 * 64), 256, 0, st>>>(mcodes.as<uint64_t>(), Um,
                                                                              vkalt.as<uint64_t>(),
                                                                              went.as<int64_t>(), code_geom(s),
                                                                              vkey.as<uint64_t>());
            GD_HIP(hipGetLastError());
        }
        // iota values: the variant index; stable sort by key keeps code order within a group
        viota_kernel<<<grid_for(Um), 256, 0, st>>>(ord.as<int32_t>(), Um);
        uint64_t* k = vkey.as<uint64_t>(); uint64_t* ka = vkalt.as<uint64_t>();
        int32_t* v = ord.as<int32_t>(); int32_t* va = oalt.as<int32_t>();
        sort_pairs_u64_i32(ctx, k, ka, v, va, (size_t)Um, 0, 64);
        if (wb == 16) {
            // keyless kmers sort last (key ~0): their share decides the packing,
            // and a probing build (the grouped rare tier chosen by default)
            // gives up when they are most of the tier: the grouping would not
            // pay (C3 without locus keys: 3.59 ms a step, the two tiers 2.28)
            DevBuf fk(8, st);
            first_keyless_kernel<<<1, 1, 0, st>>>(k, Um, fk.as<int64_t>());
            GD_HIP(hipGetLastError());
            int64_t first = Um;
            d2h(&first, fk.p, 8, st);
            const int64_t keyless = Um - first;
            if (!ctx->has_option(OPT_VARIANT_PACK_KEYLESS)) pack = 4 * keyless <= Um ? 1 : 0;
            if (probe && 2 * keyless > Um) {
                if (ctx->trace())
                    fprintf(stderr, "gdist: grouped rare tier: %lld of %lld kmers keyless, two tiers instead\n",
                            (long long)keyless, (long long)Um);
                return false;
            }
        }
        // Round 6 (option variant_keyless_rare = 1): keyless kmers of the 47 /
        // 64-kmer tier go to the rare posting lists instead of words, on the
        // premise that they are segment-move junctions (~40 a junction, held
        // by the same genomes that share the move): packed wb to a word in
        // code order a word joins unrelated kmers and its list the union of
        // their holders (C4-realistic slice: 855 M entries, 1.3e12 products,
        // 61 ms a step). As posting lists kmers of one junction have identical
        // holders and merge into one weighted list (option rare_dedup). Off
        // by default: measured on the C4-realistic slice the routed kmers
        // were not junctions but the clade-context substitutions the
        // second-level keys now group (their lists barely merged: 7.7 M
        // kmers in 3.7 M lists; the direct rare walk 52 ms, the step 76 vs
        // 68.5 ms). The hash fill only: the windowed fill looks codes up in
        // the sorted rare codes.
        int64_t Ug = Um;
        if (wb != 16) {
            DevBuf fk(8, st);
            first_keyless_kernel<<<1, 1, 0, st>>>(k, Um, fk.as<int64_t>());
            GD_HIP(hipGetLastError());
            int64_t first = Um;
            d2h(&first, fk.p, 8, st);
            const int64_t keyless = Um - first;
            const int64_t kr = ctx->option(OPT_VARIANT_KEYLESS_RARE, -1);
            const bool route = keyless > 0 && ctx->option(OPT_FILL_SORT, 0) != 3 && kr > 0;
            if (ctx->trace())
                fprintf(stderr, "gdist: variant tier: %lld of %lld kmers keyless%s\n", (long long)keyless,
                        (long long)Um, route ? ", to the rare tier" : "");
            if (route) {
                DevBuf kl(Um * 4 + 4, st), g(U * 4 + 4, st), gp(U * 8 + 8, st), msum(8, st);
                GD_HIP(hipMemsetAsync(kl.p, 0, Um * 4 + 4, st));
                mark_idx_kernel<<<grid_for(keyless), 256, 0, st>>>(v + first, keyless, kl.as<int32_t>());
                routed_flags_kernel<<<grid_for(U), 256, 0, st>>>(fm.as<int32_t>(), pm.as<int64_t>(), kl.as<int32_t>(),
                                                                 U, g.as<int32_t>());
                GD_HIP(hipGetLastError());
                exclusive_scan_i32_to_i64(ctx, g.as<int32_t>(), gp.as<int64_t>(), (size_t)U);
                DevBuf r2((Ur + keyless) * 8 + 8, st);
                if (Ur) GD_HIP(hipMemcpyAsync(r2.p, rare.p, Ur * 8, hipMemcpyDeviceToDevice, st));
                GD_HIP(hipMemsetAsync(msum.p, 0, 8, st));
                routed_emit_kernel<<<grid_for(U), 256, 0, st>>>(dict.as<uint64_t>(), dcnt.as<uint32_t>(),
                                                                g.as<int32_t>(), gp.as<int64_t>(), U,
                                                                r2.as<uint64_t>() + Ur, msum.as<unsigned long long>());
                GD_HIP(hipGetLastError());
                unsigned long long hm = 0;
                d2h(&hm, msum.p, 8, st);
                GD_HIP(hipStreamSynchronize(st));
                rare = std::move(r2);
                Ur += keyless;
                mass += (int64_t)hm;
                Ug = first;
                // the routed kmers keep no bit position (the rare tag the hash
                // fill inserts after the dictionary's replaces theirs)
                GD_HIP(hipMemsetAsync(mperm.p, 0xFF, Um * 4 + 4, st));
            }
        }
        if (Ug > 0) {
            DevBuf head(Ug * 4 + 4, st), wn(Ug * 8 + 8, st), wst(Ug * 8 + 8, st);
            group_words_kernel<<<grid_for(Ug), 256, 0, st>>>(k, Ug, wb, pack, head.as<int32_t>(), wn.as<int64_t>());
            GD_HIP(hipGetLastError());
            exclusive_scan_i64(ctx, wn.as<int64_t>(), wst.as<int64_t>(), (size_t)Ug);
            int64_t h[2];
            d2h(&h[0], wst.as<int64_t>() + Ug - 1, 8, st);
            d2h(&h[1], wn.as<int64_t>() + Ug - 1, 8, st);
            vwords = h[0] + h[1];
            GD_REQUIRE((double)vbase + (double)vwords * wb < 4294967295.0, "variant tier too large for u32 positions");
            group_pos_kernel<<<grid_for(Ug), 256, 0, st>>>(k, v, Ug, wst.as<int64_t>(), wb, pack, vbase,
                                                           mperm.as<uint32_t>());
            GD_HIP(hipGetLastError());
        }
        Um = Ug;
    }
    DevBuf perm(U * 4 + 4, st);
    if (U)
        combine_perm_kernel<<<grid_for(U), 256, 0, st>>>(fd.as<int32_t>(), pd.as<int64_t>(), pm.as<int64_t>(), U,
                                                         dperm.p ? dperm.as<uint32_t>() : nullptr,
                                                         mperm.as<uint32_t>(), perm.as<uint32_t>());
    GD_HIP(hipGetLastError());
    tr.mark("variant: word order");
    // 5. one fill pass: dense bits, rare records, and per chunk the variant
    //    records sorted and OR-merged into (word, set, mask) entries
    int sbits = 1;
    while ((int64_t(1) << sbits) < N) sbits++;
    int wbits = 1;
    while ((int64_t(1) << wbits) < std::max<int64_t>(1, vwords)) wbits++;
    GD_REQUIRE(wbits + sbits + 6 <= 64, "variant tier too large for packed record keys");
    std::vector<DevBuf> ekeys, emasks;
    std::vector<int64_t> en;
    auto hook = [&](const uint32_t* pos, int64_t s0, int64_t s1, int64_t base) {
        if (Um == 0 || s1 <= s0) return;
        const int64_t ns = s1 - s0;
        DevBuf c((ns + 1) * 8, st), a((ns + 1) * 8, st);
        vrec_count_kernel<<<(unsigned)ns, 256, 0, st>>>(pos, s->off.as<int64_t>(), s0, base, vbase, c.as<int64_t>());
        GD_HIP(hipGetLastError());
        GD_HIP(hipMemsetAsync(c.as<int64_t>() + ns, 0, 8, st));
        exclusive_scan_i64(ctx, c.as<int64_t>(), a.as<int64_t>(), (size_t)(ns + 1));
        int64_t n = 0;
        d2h(&n, a.as<int64_t>() + ns, 8, st);
        if (n == 0) return;
        DevBuf rA(n * 8 + 8, st), rB(n * 8 + 8, st);
        vrec_write_kernel<<<(unsigned)ns, 256, 0, st>>>(pos, s->off.as<int64_t>(), s0, base, vbase, sbits, lg,
                                                        (uint32_t)wb,
                                                        a.as<int64_t>(), rA.as<uint64_t>());
        GD_HIP(hipGetLastError());
        uint64_t* rk = rA.as<uint64_t>(); uint64_t* ra = rB.as<uint64_t>();
        sort_keys_u64(ctx, rk, ra, (size_t)n, 0, wbits + sbits + 6);
        DevBuf flag(n * 4 + 4, st), fpos(n * 8 + 8, st);
        vrec_heads_kernel<<<grid_for(n), 256, 0, st>>>(rk, n, flag.as<int32_t>());
        GD_HIP(hipGetLastError());
        exclusive_scan_i32_to_i64(ctx, flag.as<int32_t>(), fpos.as<int64_t>(), (size_t)n);
        int64_t last = 0;
        int32_t lf = 0;
        d2h(&last, fpos.as<int64_t>() + n - 1, 8, st);
        d2h(&lf, flag.as<int32_t>() + n - 1, 4, st);
        const int64_t ne = last + lf;
        DevBuf ek(ne * 8 + 8, st), em(ne * 8 + 8, st);
        vrec_or_kernel<<<grid_for(n), 256, 0, st>>>(rk, n, flag.as<int32_t>(), fpos.as<int64_t>(), ek.as<uint64_t>(),
                                                    em.as<unsigned long long>());
        GD_HIP(hipGetLastError());
        GD_HIP(hipStreamSynchronize(st));
        ekeys.push_back(std::move(ek));
        emasks.push_back(std::move(em));
        en.push_back(ne);
    };
    s->fp4.release();                    // the MFMA operand expanded the old bits
    s->fp4_W = 0;
    // rows of R equal shares (m = ceil(N / R) sets, the last padded): share r's
    // rows are slot r of the in-place all-gather
    const int64_t mrows = BuildSplit::ceil_div_h(N, sp.R);
    s->bits.alloc((size_t)sp.R * mrows * Wd * 8 + 8, st);
    DevBuf recs(mass * 8 + 8, st);
    int64_t written = 0;
    for (int r = sp.first(); r < sp.last(); r++) {
        ShareClock clk(sp, r, st);
        const int64_t sa = sp.set_lo(r, N), sb = sp.set_hi(r, N);
        int64_t w = 0;
        // the hash fill (default) or the windowed fill of the two-tier build
        // (option fill_sort = 3 selects the windowed one: A/B, parity)
        if (ctx->option(OPT_FILL_SORT, 0) == 3)
            fill_bits(ctx, s, dict.as<uint64_t>(), U, Wd, s->bits.as<unsigned long long>(), rare.as<uint64_t>(), Ur, 0,
                      recs.as<unsigned long long>() + written, mass - written, &w, perm.as<uint32_t>(), hook, sa, sb);
        else
            hash_fill(ctx, s, dict.as<uint64_t>(), U, perm.as<uint32_t>(), rare.as<uint64_t>(), Ur, Wd,
                      s->bits.as<unsigned long long>(), 0, recs.as<unsigned long long>() + written, mass - written, &w,
                      hook, sa, sb);
        written += w;
    }
    if (sp.real) {
        // every rank's rows and rare records
        comm_allgather_inplace(ctx, s->bits.p, (size_t)mrows * Wd * 8);
        written = allgather_concat(ctx, recs, written, 8);
    }
    GD_REQUIRE(written == mass, "rare-tier record count mismatch");
    tr.mark("variant: fill (dense bits, rare and variant records)");
    build_postings(ctx, s, recs.as<unsigned long long>(), written, Ur);
    recs.release();
    tr.mark("variant: rare postings");
    // 6. entries of every chunk (every rank's: keys are unique, (word, set),
    //    and sorted next) -> one list per word (sets ascending) + the set side
    int64_t E = 0;
    for (int64_t n : en) E += n;
    DevBuf kA(E * 8 + 8, st), mall(E * 8 + 8, st);
    {
        int64_t o = 0;
        for (size_t c = 0; c < en.size(); c++) {
            GD_HIP(hipMemcpyAsync(kA.as<uint64_t>() + o, ekeys[c].p, en[c] * 8, hipMemcpyDeviceToDevice, st));
            GD_HIP(hipMemcpyAsync(mall.as<uint64_t>() + o, emasks[c].p, en[c] * 8, hipMemcpyDeviceToDevice, st));
            o += en[c];
        }
        GD_HIP(hipStreamSynchronize(st));
        ekeys.clear();
        emasks.clear();
    }
    if (sp.real) {
        const int64_t mine = E;
        E = allgather_concat(ctx, kA, mine, 8);
        allgather_concat(ctx, mall, mine, 8);
    }
    tr.mark("variant: entries (gathered)");
    GD_REQUIRE(E < (int64_t(1) << 31), "variant tier: too many entries");
    free_variant(s);
    if (E > 0) {
        DevBuf kB(E * 8 + 8, st), iA(E * 4 + 4, st), iB(E * 4 + 4, st);
        viota_kernel<<<grid_for(E), 256, 0, st>>>(iA.as<int32_t>(), E);
        uint64_t* k = kA.as<uint64_t>(); uint64_t* ka = kB.as<uint64_t>();
        int32_t* v = iA.as<int32_t>(); int32_t* va = iB.as<int32_t>();
        sort_pairs_u64_i32(ctx, k, ka, v, va, (size_t)E, 0, wbits + sbits);
        tr.mark("variant: entries sorted by (word, set)");
        s->vw_set.alloc(E * 4 + 16, st);
        s->vw_mask.alloc(E * 8 + 16, st);
        DevBuf skey(E * 8 + 8, st), skalt(E * 8 + 8, st);
        entry_fields_kernel<<<grid_for(E), 256, 0, st>>>(k, v, E, sbits, mall.as<unsigned long long>(),
                                                         s->vw_set.as<uint32_t>(), s->vw_mask.as<unsigned long long>());
        GD_HIP(hipGetLastError());
        DevBuf woff((vwords + 1) * 8 + 8, st);
        word_offsets_kernel<<<grid_for(vwords + 1), 256, 0, st>>>(k, E, sbits, vwords, woff.as<int64_t>());
        s->vw_beg.alloc(E * 4 + 4, st);
        s->vw_end.alloc(E * 4 + 4, st);
        entry_bounds_kernel<<<grid_for(E), 256, 0, st>>>(k, E, sbits, woff.as<int64_t>(), s->vw_beg.as<uint32_t>(),
                                                         s->vw_end.as<uint32_t>());
        GD_HIP(hipGetLastError());
        set_keys_kernel<<<grid_for(E), 256, 0, st>>>(s->vw_set.as<uint32_t>(), E, skey.as<uint64_t>());
        GD_HIP(hipGetLastError());
        uint64_t* sk = skey.as<uint64_t>(); uint64_t* ska = skalt.as<uint64_t>();
        sort_keys_u64(ctx, sk, ska, (size_t)E, 0, 32 + sbits);
        tr.mark("variant: set side sorted");
        s->vs_off.alloc((N + 1) * 8, st);
        s->vs_ent.alloc(E * 4 + 4, st);
        set_offsets_kernel<<<grid_for(std::max<int64_t>(E, N + 1)), 256, 0, st>>>(sk, E, N, 32,
                                                                                  s->vs_off.as<int64_t>(),
                                                                                  s->vs_ent.as<uint32_t>());
        GD_HIP(hipGetLastError());
        DevBuf prod(16, st);
        GD_HIP(hipMemsetAsync(prod.p, 0, 16, st));
        word_products_kernel<<<grid_for(vwords, 256, 4096), 256, 0, st>>>(woff.as<int64_t>(), vwords,
                                                                          prod.as<unsigned long long>());
        GD_HIP(hipGetLastError());
        unsigned long long hp[2] = {0, 0};
        d2h(hp, prod.p, 16, st);
        s->vw_products = (double)hp[0];
        s->vw_max_list = (int64_t)hp[1];
        s->variant = true;
        // 16-kmer words of at most 65,536 sets: every entry packed in one
        // dword (set | mask << 16) for the short-list walk, and the largest
        // row weight (sum of its entries' popcounts: a bound on any pair's
        // count, so 16-bit LDS counters hold it when below 2^16)
        if (wb == 16 && N <= 65536) {
            s->vw_pack.alloc(E * 4 + 64, st);
            GD_HIP(hipMemsetAsync(s->vw_pack.p, 0, E * 4 + 64, st));   // padded: 16-byte loads past a list's end
            pack_entries_kernel<<<grid_for(E), 256, 0, st>>>(s->vw_set.as<uint32_t>(),
                                                             s->vw_mask.as<unsigned long long>(), E,
                                                             s->vw_pack.as<uint32_t>());
            GD_HIP(hipGetLastError());
            s->vs_pent.alloc(E * 8 + 8, st);
            pack_set_side_kernel<<<grid_for(E), 256, 0, st>>>(s->vs_ent.as<uint32_t>(), s->vw_beg.as<uint32_t>(),
                                                              s->vw_end.as<uint32_t>(), E, s->vs_pent.as<uint64_t>());
            GD_HIP(hipGetLastError());
            DevBuf wmax(8, st);
            GD_HIP(hipMemsetAsync(wmax.p, 0, 8, st));
            row_vweight_kernel<<<grid_for(N), 256, 0, st>>>(s->vs_off.as<int64_t>(), s->vs_ent.as<uint32_t>(),
                                                            s->vw_mask.as<unsigned long long>(), N,
                                                            wmax.as<unsigned long long>());
            GD_HIP(hipGetLastError());
            unsigned long long hw = 0;
            d2h(&hw, wmax.p, 8, st);
            s->vw_row_wmax = (int64_t)hw;
        }
        if (wb == 47 && N < (int64_t(1) << 17)) {
            s->vw_pk64.alloc(E * 8 + 64, st);
            pack64_entries_kernel<<<grid_for(E), 256, 0, st>>>(s->vw_set.as<uint32_t>(),
                                                               s->vw_mask.as<unsigned long long>(), E,
                                                               s->vw_pk64.as<unsigned long long>());
            GD_HIP(hipGetLastError());
        }
    }
    GD_HIP(hipStreamSynchronize(st));
    s->vw_words = vwords;
    s->vw_entries = E;
    s->vw_kmers = Um;
    s->vw_dmin = dmin;
    s->vw_bits = wb;
    s->W = Wd;
    s->dict_size = Ud;
    s->rare_T = T;
    s->bits_keep_singletons = false;
    tr.mark("variant: word lists + set side");
    if (ctx->trace())
        fprintf(stderr, "gdist: variant tier: T %lld, Dmin %lld: dense %lld kmers (%lld words), variant %lld kmers in "
                        "%lld words of %d, %lld entries, %.3g products, longest list %lld%s; rare %lld kmers\n",
                (long long)T, (long long)dmin, (long long)Ud, (long long)Wd, (long long)Um, (long long)vwords, wb,
                (long long)E, s->vw_products, (long long)s->vw_max_list,
                s->vw_pack.p ? " (packed 4 B)" : s->vw_pk64.p ? " (packed 8 B)" : "",
                (long long)Ur);
    build_sparse_words(ctx, s);
    return true;
}

// Decides after the dictionary of build_bitsets whether the collection takes
// the variant tier: option variant = 1 forces it, 0 keeps the two tiers;
// by default for large collections (>= kVariantMinSets sets: smaller ones
// keep the measured two-tier paths) whose kmers held by T .. Dmin - 1 sets
// are many (>= 4096) and at least a quarter of the dictionary (C4: 12.6 M of
// 12.8 M).
bool variant_wanted(const gdist_ctx* ctx, int64_t nsets, int64_t mid_kmers, int64_t dict_kmers) {
    const int64_t opt = ctx->option(OPT_VARIANT, -1);
    if (opt == 0) return false;
    if (opt > 0) return mid_kmers > 0;
    return nsets >= kVariantMinSets && mid_kmers >= 4096 && 4 * mid_kmers >= dict_kmers;
}

namespace {
__global__ void range_count_kernel(const uint32_t* __restrict__ cnt, int64_t n, int64_t lo, int64_t hi,
                                   unsigned long long* __restrict__ out) {
    unsigned long long c = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        c += (int64_t)cnt[i] >= lo && (int64_t)cnt[i] < hi;
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}
}  // namespace

int64_t count_in_range(gdist_ctx* ctx, const uint32_t* counts, int64_t n, int64_t lo, int64_t hi) {
    hipStream_t st = ctx->stream;
    if (n == 0) return 0;
    DevBuf o(8, st);
    GD_HIP(hipMemsetAsync(o.p, 0, 8, st));
    range_count_kernel<<<grid_for(n, 256, 4096), 256, 0, st>>>(counts, n, lo, hi, o.as<unsigned long long>());
    GD_HIP(hipGetLastError());
    unsigned long long h = 0;
    d2h(&h, o.p, 8, st);
    return (int64_t)h;
}

// the variant tier's counts of rows [r0, r1) x cols [c0, c1) added into I (atomics)
void variant_matrix(gdist_ctx* ctx, const gdist_sets* s, int64_t r0, int64_t r1, int64_t c0, int64_t c1, bool upper,
                    int32_t* d_I, int64_t ldI, hipStream_t rs) {
    if (!s->variant || r1 <= r0 || c1 <= c0) return;
    const int64_t units = r1 - r0;
    if (s->vw_pack.p && ctx->option(OPT_VARIANT_SHORT, 1) != 0) {
        // packed 16-kmer words: a thread an entry (the short-list walk)
        const int64_t nc = c1 - c0;
        const int nch = (int)ceil_div(nc, VSCH);
        const int64_t su = units * nch;
        // slices a row: ~8 workgroups a CU over few rows, else ~1,536 of a
        // row's entries a slice (C3: 2,266 a row; walk alone 0.81 ms with 2
        // slices, 0.85 with 3, 0.88 with 1: profiles/r05/s21)
        // (round 6: one slice a row past ~8 workgroups a CU — beside the
        // round-6 MFMA tiles C3's step is 1.376 vs 1.406 ms with 1 slice
        // against 2, C3-realistic 1.494 vs 1.541; profiles/r06/s24)
        const int nsplit = ctx->has_option(OPT_VARIANT_SPLIT)
                               ? (int)std::max<int64_t>(1, std::min<int64_t>(64, ctx->option(OPT_VARIANT_SPLIT, 1)))
                               : (int)std::max<int64_t>(1, std::min<int64_t>(16, ceil_div((int64_t)ctx->cus * 8, su)));
        const int64_t grid = su * nsplit;
        GD_REQUIRE(grid < (int64_t(1) << 31), "variant-tier grid too large");
        const bool c16 = s->vw_row_wmax < 65536 && ctx->option(OPT_VARIANT_C16, 1) != 0;
        const int64_t cols = std::min<int64_t>(nc, VSCH);
        const size_t lds = c16 ? (size_t)((cols + 1) / 2) * 4 : (size_t)cols * 4;
        FamilyTimer ft(ctx, GDIST_KERNEL_VARIANT, rs);
        auto go = [&](auto kern, int nt) {
            kern<<<(unsigned)grid, nt, lds, rs>>>(s->vs_off.as<int64_t>(), s->vs_pent.as<uint64_t>(),
                                                  s->vw_pack.as<uint32_t>(), r0, r1, c0, c1, nch, nsplit,
                                                  upper ? 1 : 0, d_I, ldI);
        };
        // (round 5: the next entry's record and first members loaded a trip
        // ahead measured slower, 0.86 vs 0.81 ms alone, profiles/r05/s27)
        if (c16) go(variant_short_kernel<512, true>, 512);
        else go(variant_short_kernel<512, false>, 512);
        GD_HIP(hipGetLastError());
        ft.end();
        return;
    }
    // few rows: slice each row's entries over several workgroups
    // (option variant_split: a given number of slices a row)
    // (~16 workgroups a CU over few rows: the C4 slice's 1,024 rows in 4
    // slices, walk alone 7.35 vs 7.5 ms with 2, 8.2 with 1; profiles/r05/s35)
    // (round 6: 16 slices a row measured 13.52 vs 13.96 ms on the C4 slice
    // beside the round-6 MFMA tiles, 8: 13.66 (profiles/r06/s24), but the
    // C4-realistic slice took 23.0 vs 19.3-19.5 ms with 16 (profiles/r06/
    // final6): kept at ~16 workgroups a CU)
    const int nsplit = ctx->has_option(OPT_VARIANT_SPLIT)
                           ? (int)std::max<int64_t>(1, std::min<int64_t>(64, ctx->option(OPT_VARIANT_SPLIT, 1)))
                           : (int)std::max<int64_t>(1, std::min<int64_t>(64, ceil_div((int64_t)ctx->cus * 16, units)));
    const int64_t grid = units * nsplit;
    GD_REQUIRE(grid < (int64_t(1) << 31), "variant-tier grid too large");
    FamilyTimer ft(ctx, GDIST_KERNEL_VARIANT, rs);
    // 1,024 threads: the walk is latency-bound and its 72 KiB of LDS allow two
    // workgroups a CU, so 16 waves each fill the CU's 32 wave slots
    // option variant_c16 (default 1): 16-bit counters, 32,768-column chunks
    // (a workgroup of 32 KiB that fits beside an MFMA tile workgroup, 512
    // threads and 14,336-column chunks: 12.4 vs 8.6 ms alone, step 20.3 vs
    // 16.0 ms, profiles/r05/s10/ab_c4.txt; dropped)
    // packed 8-byte members (47-kmer words of < 2^17 sets; option variant_short 0 reads the two arrays)
    const bool pk = s->vw_pk64.p && ctx->option(OPT_VARIANT_SHORT, 1) != 0;
    const bool c16 = ctx->option(OPT_VARIANT_C16, 1) != 0;
    auto* kern = c16 ? (pk ? variant_rows_kernel<true, true> : variant_rows_kernel<true, false>)
                     : (pk ? variant_rows_kernel<false, true> : variant_rows_kernel<false, false>);
    kern<<<(unsigned)grid, 1024, 0, rs>>>(s->vs_off.as<int64_t>(), s->vs_ent.as<uint32_t>(),
                                          s->vw_set.as<uint32_t>(), s->vw_mask.as<unsigned long long>(),
                                          s->vw_pk64.as<unsigned long long>(),
                                          s->vw_beg.as<uint32_t>(), s->vw_end.as<uint32_t>(), r0, r1, c0,
                                          c1, nsplit, upper ? 1 : 0, d_I, ldI);
    GD_HIP(hipGetLastError());
    ft.end();
}

// one query row's variant-tier counts against every set (cnt: int32 [nsets], added)
void variant_query(gdist_ctx* ctx, const gdist_sets* s, int64_t q, int32_t* cnt) {
    if (!s->variant) return;
    variant_query_kernel<<<256, 256, 0, ctx->stream>>>(s->vs_off.as<int64_t>(), s->vs_ent.as<uint32_t>(),
                                                       s->vw_set.as<uint32_t>(), s->vw_mask.as<unsigned long long>(),
                                                       s->vw_beg.as<uint32_t>(), s->vw_end.as<uint32_t>(), q, cnt);
    GD_HIP(hipGetLastError());
}

}  // namespace gdist
