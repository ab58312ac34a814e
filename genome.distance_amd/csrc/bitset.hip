// bitset.hip — dictionary-rank bitsets and the tiled AND+popcount N×N kernel.
//
// Replaces the SequenceKmers.distance(other) loop over many pairs
// (FastaDistanceProcessor.java:177-186, GenomeProcessor.java:140,
// WidthProcessor.java:159-165): |A∩B| = Σ_w popcount(a_w & b_w) over
// per-set bitsets indexed by the rank of each kmer in a global dictionary.
//
// Dictionary: all codes of all sets, radix-sorted with their set id; a run of
// equal codes is one dictionary entry. Kmers present in only one set can
// never contribute to any intersection, so by default they are left out of
// the dictionary (|A| still counts them: it comes from the CSR sizes). The
// result is exact either way (tests check both).
//
// Kernel (bitset_tile_kernel): a 256-thread workgroup owns a 128×128 tile of
// (row set, column set) pairs and a K-slice of the bitset words; each thread
// keeps an 8×8 register tile of popcount accumulators. Per 16-word chunk the
// row and column tiles are staged into LDS (XOR-swizzled 128-B rows, read as
// ds_read_b128 without bank conflicts); the inner step is 2×v_and_b32 +
// 2×v_bcnt_u32_b32 (accumulating) per 64-bit word pair — pure VALU integer
// work, no MFMA. K-slices are summed with exact int32 atomics.
#include <cstring>
#include <rocprim/rocprim.hpp>

#include <algorithm>

#include "gdist_internal.hpp"

namespace gdist {
namespace {

inline int grid_for(int64_t n, int block = 256, int64_t cap = 256 * 32) {
    int64_t g = ceil_div(n, block);
    return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

__global__ void set_ids_kernel(const int64_t* __restrict__ off, int64_t s0, int64_t s1, int32_t* __restrict__ ids) {
    const int64_t base = off[s0];
    const int64_t n = off[s1] - base;
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
        const int64_t i = base + e;
        int64_t lo = s0, hi = s1;   // upper_bound(off, i) - 1
        while (hi - lo > 1) {
            int64_t mid = (lo + hi) >> 1;
            if (off[mid] <= i) lo = mid; else hi = mid;
        }
        ids[e] = (int32_t)lo;
    }
}

__global__ void head_flags_u64(const uint64_t* __restrict__ keys, int64_t n, int32_t* __restrict__ flag) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        flag[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
}

// run heads -> unique code and run start
__global__ void run_heads_kernel(const uint64_t* __restrict__ keys, const int32_t* __restrict__ flag,
                                 const int64_t* __restrict__ pos, int64_t n, uint64_t* __restrict__ uniq,
                                 int64_t* __restrict__ start) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        if (flag[i]) { uniq[pos[i]] = keys[i]; start[pos[i]] = i; }
}

// total weight per run: weights given (prefix sums cw over elements) or 1 per element
__global__ void run_totals_kernel(const int64_t* __restrict__ start, int64_t nruns, int64_t n,
                                  const int64_t* __restrict__ cw, uint32_t* __restrict__ total) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nruns) return;
    const int64_t b = start[r], e = (r + 1 < nruns) ? start[r + 1] : n;
    const int64_t t = cw ? (cw[e] - cw[b]) : (e - b);
    total[r] = (uint32_t)(t > 0xFFFFFFFFll ? 0xFFFFFFFFll : t);
}


__global__ void compact_u64_kernel(const uint64_t* __restrict__ v, const int32_t* __restrict__ flag,
                                   const int64_t* __restrict__ pos, int64_t n, uint64_t* __restrict__ out) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        if (flag[i]) out[pos[i]] = v[i];
}

__global__ void compact_u32_kernel(const uint32_t* __restrict__ v, const int32_t* __restrict__ flag,
                                   const int64_t* __restrict__ pos, int64_t n, uint32_t* __restrict__ out) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        if (flag[i]) out[pos[i]] = v[i];
}

__global__ void widen_u32_kernel(const uint32_t* __restrict__ in, int64_t n, int64_t* __restrict__ out) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = in[i];
}

// rank of each run's code: r >= 0 in the dense dictionary, -(r + 2) in the
// rare dictionary, -1 in neither
__global__ void run_rank_kernel(const uint64_t* __restrict__ keys, const int64_t* __restrict__ start, int64_t nruns,
                                const uint64_t* __restrict__ dict, int64_t U, const uint64_t* __restrict__ rare,
                                int64_t Ur, int64_t* __restrict__ rank) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nruns) return;
    const uint64_t k = keys[start[r]];
    int64_t lo = 0, hi = U;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (dict[mid] < k) lo = mid + 1; else hi = mid;
    }
    if (lo < U && dict[lo] == k) { rank[r] = lo; return; }
    lo = 0; hi = Ur;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (rare[mid] < k) lo = mid + 1; else hi = mid;
    }
    rank[r] = (lo < Ur && rare[lo] == k) ? -(lo + 2) : -1;
}

// dense ranks -> bits; rare ranks -> (rare rank << 32 | global set id) records
__global__ void scatter_bits_kernel(const int32_t* __restrict__ ids, const int32_t* __restrict__ flag,
                                    const int64_t* __restrict__ pos, const int64_t* __restrict__ rank, int64_t n,
                                    int64_t W, unsigned long long* __restrict__ bits, int64_t id_base,
                                    unsigned long long* __restrict__ rare_out, unsigned long long* __restrict__ rare_cnt,
                                    int64_t rare_cap, const uint32_t* __restrict__ perm) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t run = pos[i] + flag[i] - 1;       // inclusive run index
        const int64_t r = rank[run];
        if (r >= 0) {
            const int64_t b = perm ? (int64_t)perm[r] : r;   // bit position (locus order)
            atomicOr(bits + (int64_t)ids[i] * W + (b >> 6), 1ull << (b & 63));
        } else if (r <= -2) {
            const unsigned long long slot = atomicAdd(rare_cnt, 1ull);
            if ((int64_t)slot < rare_cap)
                rare_out[slot] = ((unsigned long long)(-r - 2) << 32) | (unsigned long long)(uint32_t)(ids[i] + id_base);
        }
    }
}

// posting offsets: first record of each rare rank
__global__ void posting_offsets_kernel(const uint64_t* __restrict__ recs, int64_t n, int64_t nposts,
                                       int64_t* __restrict__ off) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p > nposts) return;
    const uint64_t v = (uint64_t)p << 32;
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (recs[mid] < v) lo = mid + 1; else hi = mid;
    }
    off[p] = lo;
}

__global__ void posting_sets_kernel(const uint64_t* __restrict__ recs, int64_t n, uint32_t* __restrict__ sets) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) sets[i] = (uint32_t)recs[i];
}

// Lists of kLongList+ sets (gdist_internal.hpp) are walked by a whole wave
// (lanes stride the members) instead of one lane: a lane-serial walk of an
// m-member list is an O(m) (row-major) or O(m^2) (list-major) tail the rest
// of the wave idles on.

// pairs (s = psets[x], t = psets[y]) for y in [y0, e) step dy, s < t
__device__ __forceinline__ void rare_pair_walk(const uint32_t* __restrict__ psets, int64_t x, int64_t y0, int64_t e,
                                               int dy, int64_t r0, int64_t r1, int64_t c0, int64_t c1, int upper,
                                               int32_t w, int32_t* __restrict__ I, int64_t ldI) {
    const int64_t s = psets[x];
    const bool srow = s >= r0 && s < r1, scol = s >= c0 && s < c1;
    if (!srow && (upper || !scol)) return;
    for (int64_t y = y0; y < e; y += dy) {
        const int64_t t = psets[y];                  // t > s
        if (srow && t >= c0 && t < c1) atomicAdd(I + (s - r0) * ldI + (t - c0), w);
        if (!upper && scol && t >= r0 && t < r1) atomicAdd(I + (t - r0) * ldI + (s - c0), w);
    }
}

// Rare tier: every posting list (ascending set ids) adds its weight (the
// number of kmers sharing it) to each of its m(m-1)/2 pairs that fall in the
// region. One lane per list; lists of kLongList+ members are taken by the
// wave (trip counts are wave-uniform).
__global__ __launch_bounds__(256) void rare_pairs_kernel(const int64_t* __restrict__ poff,
                                                         const uint32_t* __restrict__ psets,
                                                         const uint32_t* __restrict__ pw, int64_t nposts,
                                                         int64_t r0, int64_t r1, int64_t c0, int64_t c1, int upper,
                                                         int32_t* __restrict__ I, int64_t ldI) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int lane = threadIdx.x & 63;
    for (int64_t pb = (int64_t)blockIdx.x * blockDim.x; pb < nposts; pb += stride) {
        const int64_t p = pb + threadIdx.x;
        int64_t b = 0, e = 0;
        int32_t w = 0;
        if (p < nposts) { b = poff[p]; e = poff[p + 1]; w = (int32_t)pw[p]; }
        const bool lng = e - b >= kLongList;
        for (unsigned long long m = __ballot(lng); m; m &= m - 1) {
            const int l = __ffsll((long long)m) - 1;
            const int64_t lb = __shfl((long long)b, l, 64), le = __shfl((long long)e, l, 64);
            const int32_t lw = __shfl(w, l, 64);
            for (int64_t x = lb; x < le - 1; x++)
                rare_pair_walk(psets, x, x + 1 + lane, le, 64, r0, r1, c0, c1, upper, lw, I, ldI);
        }
        if (!lng)
            for (int64_t x = b; x < e - 1; x++)
                rare_pair_walk(psets, x, x + 1, e, 1, r0, r1, c0, c1, upper, w, I, ldI);
    }
}

// Rare tier, row-major: one workgroup per (row set i, chunk of RCH columns).
// The row's rare kmers (set -> rare CSR) are walked by the threads; each
// member j of their posting lists adds 1 to an LDS counter; the counters are
// then added to I's row once, coalesced. No global atomics, and each (i, j)
// is owned by exactly one workgroup (the dense kernel ran before, in stream
// order).
constexpr int RCH = 16384;   // max columns per LDS chunk (64 KiB of counters)

// grid = nr rows x nch column chunks x nsplit slices of the row's rare kmers;
// counters live in dynamic LDS sized to the chunk. With nsplit > 1 several
// workgroups share a row chunk and flush with global atomics.
// Member = uint32 (post_sets) or uint16 (post_sets16, collections of at most
// 65,536 sets): the walk's scattered list reads are whole lines from HBM or
// the Infinity Cache, and 2-byte members halve the lines a list spans and
// let C3's lists (72 M members: 287 MB as uint32) sit in the 256 MiB cache.
// NT threads a workgroup (option rare_rows_threads: 512 default, 256): the
// walk is latency-bound (each record's members are a dependent load after its
// record's), and the 40 KiB of counters of a C3 row allow 4 workgroups a CU:
// 512 threads make that the full 32 waves a CU instead of 16
// C16 (round 5): 16-bit counters, two to an LDS dword, when no row's rare
// kmers weigh 65,536 or more (rare_row_wmax, build time: a count never
// carries into its neighbour) — C3's 10,000 columns take 20 KiB instead of
// 40, so a workgroup fits on a CU beside an MFMA dense-tile workgroup.
template <typename M, int NT, bool C16 = false>
__global__ __launch_bounds__(NT) void rare_rows_kernel(const int64_t* __restrict__ soff,
                                                        const uint64_t* __restrict__ sent,
                                                        const uint32_t* __restrict__ sw,
                                                        const uint16_t* __restrict__ sskip,
                                                        const M* __restrict__ psets, int64_t r0, int64_t r1,
                                                        int64_t c0, int64_t c1, int nch, int nsplit, int upper,
                                                        int atomic_flush, int32_t* __restrict__ I, int64_t ldI) {
    constexpr int PER = 16 / (int)sizeof(M);     // members per 16-byte load
    extern __shared__ int32_t cnt[];
    const int64_t unit = blockIdx.x / nsplit;
    const int split = blockIdx.x % nsplit;
    const int64_t i = r0 + unit / nch;
    const int ch = (int)(unit % nch);
    const int64_t cb = c0 + (int64_t)ch * RCH;
    const int64_t ce = cb + RCH < c1 ? cb + RCH : c1;
    if (i >= r1 || cb >= ce || (upper && ce - 1 <= i)) return;
    const int n = (int)(ce - cb);
    const int nw = C16 ? (n + 1) >> 1 : n;
    for (int t = threadIdx.x; t < nw; t += blockDim.x) cnt[t] = 0;
    __syncthreads();
    auto add = [&](int64_t t, int32_t v) {
        if (C16) atomicAdd(&cnt[(t - cb) >> 1], v << (((t - cb) & 1) << 4));
        else atomicAdd(&cnt[t - cb], v);
    };
    const int64_t lo = upper && i + 1 > cb ? i + 1 : cb;
    const int64_t rb = soff[i], re = soff[i + 1];
    const int64_t per = (re - rb + nsplit - 1) / nsplit;
    const int64_t xb = rb + per * split;
    const int64_t xe = xb + per < re ? xb + per : re;
    const int lane = threadIdx.x & 63;
    for (int64_t xbase = xb; xbase < xe; xbase += blockDim.x) {   // wave-uniform trip count
        const int64_t x = xbase + threadIdx.x;
        const uint64_t ent = x < xe ? sent[x] : 0ull;  // coalesced: no random bounds lookup
        const int32_t w = x < xe ? (int32_t)sw[x] : 0;
        const int64_t b0 = (int64_t)(ent >> 24), e = b0 + (int64_t)(ent & 0xFFFFFFu);
        // upper triangle: only the members after the row's own set (ascending lists)
        const int64_t b = upper && x < xe ? b0 + sskip[x] : b0;
        const bool lng = e - b >= kLongList;
        for (unsigned long long m = __ballot(lng); m; m &= m - 1) {   // long lists: the wave walks them
            const int l = __ffsll((long long)m) - 1;
            const int64_t lb = __shfl((long long)b, l, 64), le = __shfl((long long)e, l, 64);
            const int32_t lw = __shfl(w, l, 64);
            for (int64_t y = lb + lane; y < le; y += 64) {
                const int64_t t = psets[y];
                if (t >= lo && t < ce && t != i) add(t, lw);
            }
        }
        if (lng) continue;
        // PER members per 16-byte load (global_load_dwordx4 when the list
        // start is dword-aligned; post_sets / post_sets16 are padded past the
        // last list)
#pragma unroll 2
        for (int64_t y = b; y < e; y += PER) {
            M mem[PER];
            __builtin_memcpy(mem, psets + y, 16);
#pragma unroll
            for (int u = 0; u < PER; u++) {
                const int64_t t = mem[u];
                if (y + u < e && t >= lo && t < ce && t != i) add(t, w);
            }
        }
    }
    __syncthreads();
    int32_t* row = I + (i - r0) * ldI + (cb - c0);
    for (int t = threadIdx.x; t < n; t += blockDim.x) {
        const int v = C16 ? (int)(((uint32_t)cnt[t >> 1] >> ((t & 1) << 4)) & 0xFFFFu) : cnt[t];
        if (v && cb + t >= lo) {
            if (nsplit > 1 || atomic_flush) atomicAdd(row + t, v);
            else row[t] += v;
        }
    }
}

// Rare tier, row-major over a wide column range (round 5; C4's 100,000
// columns would need 7 LDS chunks, and rare_rows_kernel walks every list of
// the row once PER CHUNK, filtering its members to the chunk: 10.2 ms on the
// C4 slice for 0.9 GB of algorithmic bytes). Here each (set, list) record of
// the row is walked ONCE and every member in [lo, c1) adds the list's weight
// straight into I's row with a device-scope atomic (the dense tiles and the
// variant walk beside it add atomically too). A thread takes one record
// (16-byte member loads, as rare_rows_kernel); long lists go to the whole
// wave. Grid: rows x nsplit slices of the row's records.
template <typename M>
__global__ __launch_bounds__(256) void rare_rows_direct_kernel(const int64_t* __restrict__ soff,
                                                               const uint64_t* __restrict__ sent,
                                                               const uint32_t* __restrict__ sw,
                                                               const uint16_t* __restrict__ sskip,
                                                               const M* __restrict__ psets, int64_t r0, int64_t r1,
                                                               int64_t c0, int64_t c1, int nsplit, int upper,
                                                               int32_t* __restrict__ I, int64_t ldI) {
    constexpr int PER = 16 / (int)sizeof(M);
    const int64_t i = r0 + blockIdx.x / nsplit;
    const int split = blockIdx.x % nsplit;
    if (i >= r1) return;
    const int64_t lo = upper && i + 1 > c0 ? i + 1 : c0;
    if (lo >= c1) return;
    int32_t* row = I + (i - r0) * ldI - c0;                 // row[t] for column t
    const int64_t rb = soff[i], re = soff[i + 1];
    const int64_t per = (re - rb + nsplit - 1) / nsplit;
    const int64_t xb = rb + per * split;
    const int64_t xe = xb + per < re ? xb + per : re;
    const int lane = threadIdx.x & 63;
    for (int64_t xbase = xb; xbase < xe; xbase += blockDim.x) {   // wave-uniform trip count
        const int64_t x = xbase + threadIdx.x;
        const uint64_t ent = x < xe ? sent[x] : 0ull;
        const int32_t w = x < xe ? (int32_t)sw[x] : 0;
        const int64_t b0 = (int64_t)(ent >> 24), e = b0 + (int64_t)(ent & 0xFFFFFFu);
        const int64_t b = upper && x < xe ? b0 + sskip[x] : b0;
        const bool lng = e - b >= kLongList;
        for (unsigned long long m = __ballot(lng); m; m &= m - 1) {
            const int l = __ffsll((long long)m) - 1;
            const int64_t lb = __shfl((long long)b, l, 64), le = __shfl((long long)e, l, 64);
            const int32_t lw = __shfl(w, l, 64);
            for (int64_t y = lb + lane; y < le; y += 64) {
                const int64_t t = psets[y];
                if (t >= lo && t < c1 && t != i) atomicAdd(row + t, lw);
            }
        }
        if (lng) continue;
#pragma unroll 2
        for (int64_t y = b; y < e; y += PER) {
            M mem[PER];
            __builtin_memcpy(mem, psets + y, 16);
#pragma unroll
            for (int u = 0; u < PER; u++) {
                const int64_t t = mem[u];
                if (y + u < e && t >= lo && t < c1 && t != i) atomicAdd(row + t, w);
            }
        }
    }
}

// Rare tier of one query set q: cnt[t] += shared rare kmers of q and t
// (global atomics, one row's worth); gather_add adds cnt[cols[c]] to I[c]
// for every requested column position (duplicates included).
__global__ __launch_bounds__(256) void rare_query_kernel(const int64_t* __restrict__ soff,
                                                         const uint64_t* __restrict__ sent,
                                                         const uint32_t* __restrict__ sw,
                                                         const uint32_t* __restrict__ psets, int64_t q,
                                                         int32_t* __restrict__ cnt) {
    const int64_t xb = soff[q], xe = soff[q + 1];
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int lane = threadIdx.x & 63;
    for (int64_t xbase = xb + (int64_t)blockIdx.x * blockDim.x; xbase < xe; xbase += stride) {
        const int64_t x = xbase + threadIdx.x;
        const uint64_t ent = x < xe ? sent[x] : 0ull;
        const int32_t w = x < xe ? (int32_t)sw[x] : 0;
        const int64_t b = (int64_t)(ent >> 24), e = b + (int64_t)(ent & 0xFFFFFFu);
        const bool lng = e - b >= kLongList;
        for (unsigned long long m = __ballot(lng); m; m &= m - 1) {
            const int l = __ffsll((long long)m) - 1;
            const int64_t lb = __shfl((long long)b, l, 64), le = __shfl((long long)e, l, 64);
            const int32_t lw = __shfl(w, l, 64);
            for (int64_t y = lb + lane; y < le; y += 64) {
                const int64_t t = psets[y];
                if (t != q) atomicAdd(cnt + t, lw);
            }
        }
        if (lng) continue;
        for (int64_t y = b; y < e; y++) {
            const int64_t t = psets[y];
            if (t != q) atomicAdd(cnt + t, w);
        }
    }
}

__global__ void gather_add_kernel(const int64_t* __restrict__ cols, int64_t ncols, const int32_t* __restrict__ cnt,
                                  int32_t* __restrict__ I) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c < ncols) I[c] += cnt[cols[c]];
}

// set-side entries: rare rank -> (list start << 24 | list length)
__global__ void rare_entries_kernel(const uint64_t* __restrict__ keys, int64_t n, const int64_t* __restrict__ poff,
                                    uint64_t* __restrict__ ent) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t r = (uint32_t)keys[i];
        const int64_t b = poff[r];
        ent[i] = ((uint64_t)b << 24) | (uint64_t)(poff[r + 1] - b);
    }
}

// per (set, list) record: one past the set's position in its list (the
// members an upper-triangle row walk starts at; lists are ascending), 0
// past 65534 members (the walk then starts at the list's first member)
__global__ void rare_skip_kernel(const uint64_t* __restrict__ keys, int64_t n, const int64_t* __restrict__ poff,
                                 const uint32_t* __restrict__ psets, uint16_t* __restrict__ skip) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t set = (uint32_t)(keys[i] >> 32), r = (uint32_t)keys[i];
        int64_t lo = poff[r], hi = poff[r + 1];
        const int64_t b = lo;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (psets[mid] < set) lo = mid + 1; else hi = mid;
        }
        const int64_t k = lo - b + 1;
        skip[i] = k < 65535 ? (uint16_t)k : (uint16_t)0;
    }
}

// set -> rare CSR: records (rare << 32 | set) become (set << 32 | rare)
__global__ void swap_halves_kernel(const uint64_t* __restrict__ in, int64_t n, uint64_t* __restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = (in[i] << 32) | (in[i] >> 32);
}

// rare-tier mass: count of records each rare dictionary entry will produce
__global__ void rare_flag_kernel(const uint32_t* __restrict__ cnt, int64_t n, int64_t T, int keep,
                                 int32_t* __restrict__ dflag, int32_t* __restrict__ rflag, int64_t* __restrict__ rmass) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t c = cnt[i];
        const bool dense = keep || (c >= 2 && (int64_t)c >= T);
        const bool rare = !keep && c >= 2 && (int64_t)c < T;
        dflag[i] = dense ? 1 : 0;
        rflag[i] = rare ? 1 : 0;
        rmass[i] = rare ? (int64_t)c : 0;
    }
}

constexpr int BT = 128;                 // tile edge (sets)
// A block's last row tile holding RR <= kPartialMaxRR sixteen-row groups gets
// its own launches with RR accumulator rows (RR = 7 saves less than the two
// launches cost: C2, 104 rows, 4.51 vs 4.27 ms)
constexpr int kPartialMaxRR = 6;
constexpr int KC = 16;                  // bitsets are padded to whole multiples of KC words
constexpr int NT = 256;

// v_bcnt_u32_b32 d, x, acc = popcount(x) + acc. Written as asm because hipcc
// otherwise reassociates the sums into extra v_add3_u32 (10 VALU ops per
// 4 dwords instead of 8).
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}

// ---- dense tiles: LDS-DMA double buffering, split-major XCD-aware order ----
// 256 threads own a 128×128 tile, 8×8 counts per thread;
//  * chunks of KC2 = 8 words are moved HBM/L2 -> LDS by global_load_lds_dwordx4
//    (no register staging, so ≤ 128 VGPRs and 4 waves per SIMD), double
//    buffered: chunk k+1 is in flight while chunk k is computed;
//  * the LDS image swizzle (slot q of row g at q ^ ((g >> 2) & 3)) is applied on
//    the DMA source address (the destination of one DMA instruction is linear);
//  * blocks are ordered split-major and remapped so one XCD runs consecutive
//    units: concurrently resident blocks work on the same K-range of every set,
//    which stays in the L2 / Infinity Cache while all tiles consume it.
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

constexpr int KC2 = 8;                        // words per chunk
constexpr int ROW2 = KC2 * 8;                 // 64 B per set row
constexpr int OPB2 = BT * ROW2;               // 8 KiB per operand per stage
constexpr int STAGE2 = 2 * OPB2;              // A + B

__device__ __forceinline__ int lds_off2(int g, int q) { return g * ROW2 + ((q ^ ((g >> 2) & 3)) << 4); }

// one operand's chunk: 8 DMA instructions of 1 KiB (16 rows), 2 per wave
__device__ __forceinline__ void dma_chunk(const unsigned long long* __restrict__ bits, int64_t W, int64_t set0,
                                          int64_t lo, int64_t lim, int64_t kc, unsigned char* lds_op, int wave,
                                          int lane) {
#pragma unroll
    for (int i = 0; i < 2; i++) {
        const int rbase = (wave * 2 + i) * 16;
        const int g = rbase + (lane >> 2);
        const int p = lane & 3;
        const int q = p ^ ((g >> 2) & 3);
        int64_t set = set0 + g;
        set = set < lim ? set : lim - 1;              // clamp: rows outside [lo, lim) are masked at the end
        set = set >= lo ? set : lo;
        const unsigned long long* src = bits + set * W + kc * KC2 + q * 2;
        __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(lds_op + rbase * ROW2), 16, 0, 0);
    }
}

// One staged chunk (KC2 words of 128 row sets and 128 column sets) into the
// thread's 8x8 accumulators, two column fragments at once, dword-outer, so
// consecutive v_and/v_bcnt pairs belong to 16 different accumulators and no
// instruction waits on its predecessor. DIAG: the tile sits on the diagonal of an
// upper-triangle region, where accumulator (r, c) holds pairs with j > i only
// when c >= r (rows ty + 16r, columns tx + 16c): the c < r ones (28 of 64) are
// never computed. RR: only accumulator rows r < RR hold rows of the block (a
// partial row tile at a block's end); the others are never computed.
template <bool DIAG, int RR = 8>
__device__ __forceinline__ void chunk_pairs(const unsigned char* A, const unsigned char* B, int ty, int tx,
                                            uint32_t (&acc)[8][8]) {
#pragma unroll 1
    for (int q = 0; q < KC2 / 2; q++) {
        uint4 a[8];
#pragma unroll
        for (int r = 0; r < RR; r++) a[r] = *reinterpret_cast<const uint4*>(A + lds_off2(ty + 16 * r, q));
#pragma unroll
        for (int c = 0; c < 8; c += 2) {
            const uint4 b0 = *reinterpret_cast<const uint4*>(B + lds_off2(tx + 16 * c, q));
            const uint4 b1 = *reinterpret_cast<const uint4*>(B + lds_off2(tx + 16 * (c + 1), q));
            const uint32_t bw0[4] = {b0.x, b0.y, b0.z, b0.w};
            const uint32_t bw1[4] = {b1.x, b1.y, b1.z, b1.w};
#pragma unroll
            for (int d = 0; d < 4; d++) {
#pragma unroll
                for (int r = 0; r < RR; r++) {
                    const uint32_t ad = d == 0 ? a[r].x : d == 1 ? a[r].y : d == 2 ? a[r].z : a[r].w;
                    if (!DIAG || c >= r) acc[r][c] = bcnt_acc(ad & bw0[d], acc[r][c]);
                    if (!DIAG || c + 1 >= r) acc[r][c + 1] = bcnt_acc(ad & bw1[d], acc[r][c + 1]);
                }
            }
        }
    }
}

// DIAG: every tile of the launch sits on the diagonal of an upper-triangle
// region (bitset_matrix launches those tiles separately). RR < 8: every tile
// of the launch is the partial last row tile of the block, with at most 16 RR
// rows (rows ty + 16r with r >= RR are past r1 for every thread).
template <bool DIAG, int RR = 8>
__global__ __launch_bounds__(NT, 4) void bitset_tile_kernel2(
    const unsigned long long* __restrict__ bits, int64_t W, const int2* __restrict__ tiles, int ntiles, int splits,
    int64_t nchunks, int64_t r0, int64_t r1, int64_t c0, int64_t c1, int64_t corg, int upper,
    int32_t* __restrict__ I, int64_t ldI) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[2 * STAGE2];

    // XCD-aware bijective remap, then split-major unit order
    const int64_t G = gridDim.x, blk = blockIdx.x;
    const int64_t xcd = blk & 7, kq = blk >> 3, qg = G >> 3, rem = G & 7;
    const int64_t u = xcd * qg + (xcd < rem ? xcd : rem) + kq;
    const int split = (int)(u / ntiles);
    const int tile = (int)(u - (int64_t)split * ntiles);
    const int2 t = tiles[tile];
    if (split >= splits || t.x < 0 || t.y < 0) return;
    const int64_t row0 = r0 + (int64_t)t.x * BT;
    const int64_t col0 = corg + (int64_t)t.y * BT;     // column tiles start at corg <= c0 (see bitset_matrix)
    const int64_t kc_per = ceil_div(nchunks, splits);
    const int64_t kc0 = (int64_t)split * kc_per;
    const int64_t kc1 = kc0 + kc_per < nchunks ? kc0 + kc_per : nchunks;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int tx = tid & 15, ty = tid >> 4;

    uint32_t acc[8][8];
#pragma unroll
    for (int r = 0; r < 8; r++)
#pragma unroll
        for (int c = 0; c < 8; c++) acc[r][c] = 0;

    if (kc0 < kc1) {
        dma_chunk(bits, W, row0, r0, r1, kc0, lds, wave, lane);
        dma_chunk(bits, W, col0, c0, c1, kc0, lds + OPB2, wave, lane);
    }
    for (int64_t kc = kc0; kc < kc1; kc++) {
        const int st = (int)((kc - kc0) & 1);
        unsigned char* A = lds + st * STAGE2;
        unsigned char* B = A + OPB2;
        if (kc + 1 < kc1) {
            unsigned char* An = lds + (st ^ 1) * STAGE2;
            dma_chunk(bits, W, row0, r0, r1, kc + 1, An, wave, lane);
            dma_chunk(bits, W, col0, c0, c1, kc + 1, An + OPB2, wave, lane);
            asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");   // chunk kc landed everywhere
        } else {
            asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        }
        chunk_pairs<DIAG, RR>(A, B, ty, tx, acc);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // stage free for the next DMA
    }

#pragma unroll
    for (int r = 0; r < 8; r++) {
        const int64_t i = row0 + ty + 16 * r;
        if (i >= r1) continue;
#pragma unroll
        for (int c = 0; c < 8; c++) {
            const int64_t j = col0 + tx + 16 * c;
            if (j < c0 || j >= c1 || (upper && j <= i)) continue;
            if (acc[r][c]) atomicAdd(I + (i - r0) * ldI + (j - c0), (int32_t)acc[r][c]);
        }
    }
}

// ---- dense tiles on the matrix cores (round 4) ------------------------------
// |A ∩ B| over the dense words is a bit-matrix product: I = Σ_k a_ik b_jk over
// the dictionary bits. The block-scaled MFMA v_mfma_scale_f32_32x32x64_f8f6f4
// takes FP4 (e2m1) operands, where the codes 0x0 and 0x2 are 0.0 and 1.0:
// with every bit stored as one nibble, one instruction is a 32 x 32 block of
// pairs over 64 bits (one word), products and f32 sums exact (a count <=
// 64 W < 2^24). The FP4 rate is 4x the BF16 MFMA rate, 5 P products/s
// dense; the AND + popcount tiles are capped at 0.63 P bit-pairs/s by the
// half-rate v_bcnt. Operand map (scripts/microbench/fp4_probe.hip, checked
// against the CPU): lane r + 32 h holds row r's bits [32 h, 32 h + 32) of the
// word as 16 bytes of nibbles, low nibble first; D: column lane & 31, row
// (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5).
// F = the dense bits expanded once per collection, [N][32 W] bytes (4x the
// bitsets). A workgroup of 8 waves owns a 256 x 256 tile of pairs and a range
// of words, each wave 64 rows x 128 columns (2 x 4 MFMA blocks, 128 f32
// accumulators a lane); stages of KM words of both operands (256 rows x
// 32 KM bytes each) are moved by global_load_lds, double buffered, with the
// 16-byte chunk c of row g stored at c ^ ((g >> 1) & 7) (conflict-free
// fragment reads); units split-major and XCD-remapped as the VALU tiles.
constexpr int MT = 256;                       // tile edge (sets)
constexpr int64_t kMfmaMinWords = 64;         // dense words from which the MFMA tiles run (option bitset_mfma)
constexpr int MNT = 512;                      // threads
// f32 is exact for integers <= 2^24: one K split's count of shared bits is
// <= 64 x its words, so a split spans at most 2^18 words
constexpr int64_t kMfmaMaxSplitWords = int64_t(1) << 18;
// the fewest K splits (of nst stages of km words) that keep every split's
// count exact in f32
static inline int64_t mfma_min_splits(int64_t nst, int km) {
    const int64_t per_max = kMfmaMaxSplitWords / km;                 // stages a split may span
    return nst <= per_max ? 1 : (nst + per_max - 1) / per_max;
}
// KM words per stage (4: 2 x 32 KiB a stage, 128 KiB double-buffered; 2:
// 64 KiB, so a row-major rare workgroup fits beside it on a CU: option
// bitset_mfma_km)
template <int KM> constexpr int mrow() { return KM * 32; }          // bytes per row per stage
template <int KM> constexpr int mopb() { return MT * mrow<KM>(); }  // one operand's stage
typedef int v8i_t __attribute__((ext_vector_type(8)));
typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef float v16f_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t bits_to_nibbles(uint32_t byte) {   // 8 bits -> 8 nibbles 0x0 / 0x2
    uint32_t t = (byte & 0x0Fu) | ((byte & 0xF0u) << 12);
    t = (t | (t << 6)) & 0x03030303u;
    t = (t | (t << 3)) & 0x11111111u;
    return t << 1;
}

// F[i][32 w + q] for one (set, word) per thread: 32 bytes of nibbles
__global__ void fp4_expand_kernel(const unsigned long long* __restrict__ bits, int64_t n, uint4* __restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += stride) {
        const unsigned long long w = bits[t];
        const uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
        out[2 * t] = make_uint4(bits_to_nibbles(lo & 0xFF), bits_to_nibbles((lo >> 8) & 0xFF),
                                bits_to_nibbles((lo >> 16) & 0xFF), bits_to_nibbles(lo >> 24));
        out[2 * t + 1] = make_uint4(bits_to_nibbles(hi & 0xFF), bits_to_nibbles((hi >> 8) & 0xFF),
                                    bits_to_nibbles((hi >> 16) & 0xFF), bits_to_nibbles(hi >> 24));
    }
}

// chunk c (16 B) of row g: KM = 4 rows of 8 chunks, c ^ ((g >> 1) & 7); KM =
// 2 rows of 4 chunks, c ^ ((g >> 2) & 3) (conflict-free ds_read_b128 either way)
template <int KM> __device__ __forceinline__ int mslot(int g, int c) {
    return KM == 4 ? (c ^ ((g >> 1) & 7)) : (c ^ ((g >> 2) & 3));
}
template <int KM> __device__ __forceinline__ int mlds(int g, int c) { return g * mrow<KM>() + (mslot<KM>(g, c) << 4); }

// one operand's stage: 16-byte chunks, KM per thread (lane-linear LDS, the
// swizzle applied on the source address)
template <int KM, int NT = MNT>
__device__ __forceinline__ void mfma_stage(const unsigned char* __restrict__ F, int64_t rowbytes, int64_t set0,
                                           int64_t lo, int64_t lim, int64_t w0, unsigned char* lds_op, int tid) {
    constexpr int CPR = 2 * KM;                       // chunks per row
#pragma unroll
    for (int i = 0; i < KM * (MNT / NT); i++) {
        const int q = i * NT + tid;                   // 16-byte slot of the stage
        const int g = q / CPR, sl = q % CPR;
        const int c = mslot<KM>(g, sl);               // the chunk this slot holds (the swizzle is an involution)
        int64_t set = set0 + g;
        set = set < lim ? set : lim - 1;              // rows outside [lo, lim): clamped, masked at the end
        set = set >= lo ? set : lo;
        const unsigned char* src = F + set * rowbytes + w0 * 32 + c * 16;
        __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(lds_op + (i * NT + (tid & ~63)) * 16), 16,
                                         0, 0);
    }
}

// piece i (0 .. KM - 1) of one operand's stage: the i-th iteration of
// mfma_stage, so that a stage's DMA can be spread between MFMAs
template <int KM>
__device__ __forceinline__ void mfma_piece(const unsigned char* __restrict__ F, int64_t rowbytes, int64_t set0,
                                           int64_t lo, int64_t lim, int64_t w0, unsigned char* lds_op, int tid,
                                           int i) {
    constexpr int CPR = 2 * KM;
    const int q = i * MNT + tid;
    const int g = q / CPR, sl = q % CPR;
    const int c = mslot<KM>(g, sl);
    int64_t set = set0 + g;
    set = set < lim ? set : lim - 1;
    set = set >= lo ? set : lo;
    const unsigned char* src = F + set * rowbytes + w0 * 32 + c * 16;
    __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(lds_op + (i * MNT + (tid & ~63)) * 16), 16, 0,
                                     0);
}

// the wait at the top of a stage: every stage still in flight after it may stay
// (g = glds per stage per thread: 2 KM); a counted vmcnt keeps the later stages'
// DMAs going across the barrier (raw s_barrier, never __syncthreads, whose
// fence would drain them)
template <int G>
__device__ __forceinline__ void mfma_wait(int later) {
    switch (later) {
        case 0: asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(G) : "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(2 * G) : "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(3 * G) : "memory"); break;
    }
}

// Round 5 (RAW): the operand is the bitsets themselves, not the nibbles. A
// stage of the same 128 bytes per row holds 16 words instead of 4, so a tile
// moves a quarter of the bytes global -> LDS (C4: 80 -> 20 GB a 1,024-row
// step; the nibble operand was 4x the bitsets in HBM and in every L2), and
// each lane expands its fragment in registers: MFMA step m of a stage takes
// lane (r, h)'s dword 4 q + m of its half h of row r (chunk 4 h + q), and
// nibble j of fragment dword k holds bit 4 j + k of that dword as 0x0 / 0x2
// (x << 1, x, x >> 1, x >> 2 under 0x22222222: 7 VALU per dword). Any
// assignment of bits to K positions is exact as long as both operands use
// the same one.
__device__ __forceinline__ v4i_t raw_nibbles(uint32_t x) {
    const v4i_t f = {(int)((x << 1) & 0x22222222u), (int)(x & 0x22222222u), (int)((x >> 1) & 0x22222222u),
                     (int)((x >> 2) & 0x22222222u)};
    return f;
}

// NS stages in a ring (2: double buffering; 4 with KM = 2 in the same 128
// KiB: three stages in flight while one is computed; option bitset_mfma_km)
// STORE (round 5, option bitset_mfma_store): one K split, every pair of the
// tile STORED (the tile is its only writer; the other families add after it
// in stream order) instead of 64 K device atomics a tile
// SPREAD (round 6, raw KM = 4 double-buffered only; option bitset_mfma_sched,
// default 1): the next stage's DMA spread between the current stage's MFMAs
// (one piece after each MFMA step of its first two fragment reads) with ONE
// barrier a stage — the barrier at the top of stage ks says both that stage
// ks landed and that every wave is done with stage ks - 1's buffer, which the
// pieces of stage ks + 1 then overwrite. Before, every wave issued its 8
// pieces at the top of the stage, where the CU's 64 KiB of requests held
// the MFMA pipe (tiles alone: C4 slice 7.45 vs 7.98 ms, C3 0.72 vs 0.79;
// profiles/r06/s12)
// PLANE (round 6, with SPREAD; option bitset_mfma_plane): MFMA step m takes
// bit m of every nibble of the chunk's four dwords (x & 0x11111111 << m;
// plane 3, the sign bit, shifted into bit 2) instead of the four bits of
// dword m moved to bit 1: 5 VALU a dword instead of 7. The planes' nibbles
// are the e2m1 codes 0x1 / 0x2 / 0x4 = 0.5 / 1.0 / 2.0, each step under the
// e8m0 scale (both operands) that makes them 1.0 (128 / 127 / 126), so every
// product is still 0 or 1 (scripts/microbench/fp4_scale_probe.hip)
__device__ __forceinline__ int bit_plane(uint32_t x, int m) {
    return (int)(m < 3 ? (x & (0x11111111u << m)) : ((x >> 1) & 0x44444444u));
}
template <int KM, int NS, bool RAW = false, bool STORE = false, bool SPREAD = false, bool PLANE = false>
__global__ __launch_bounds__(MNT, 2) void bitset_mfma_kernel(
    const unsigned char* __restrict__ F, int64_t W, const int2* __restrict__ tiles, int ntiles, int splits,
    int64_t nstages, int64_t r0, int64_t r1, int64_t c0, int64_t c1, int upper, int32_t* __restrict__ I,
    int64_t ldI) {
    static_assert(NS >= 2 && NS <= 4, "stage ring of 2..4");
    extern __shared__ __attribute__((aligned(16))) unsigned char mlds_buf[];     // NS stages x (A, B)
    constexpr int MOPB = mopb<KM>();
    const int64_t G = gridDim.x, blk = blockIdx.x;
    const int64_t xcd = blk & 7, kq = blk >> 3, qg = G >> 3, rem = G & 7;
    const int64_t u = xcd * qg + (xcd < rem ? xcd : rem) + kq;
    const int split = (int)(u / ntiles);
    const int tile = (int)(u - (int64_t)split * ntiles);
    if (split >= splits) return;
    const int2 t = tiles[tile];
    const int64_t row0 = r0 + (int64_t)t.x * MT, col0 = c0 + (int64_t)t.y * MT;
    const int64_t per = ceil_div(nstages, splits);
    const int64_t ks0 = (int64_t)split * per, ks1 = ks0 + per < nstages ? ks0 + per : nstages;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;          // 4 x 2 waves of 64 rows x 128 columns
    const int r = lane & 31, h = lane >> 5;
    const int64_t rowbytes = RAW ? W * 8 : W * 32;
    v16f_t acc[2][4];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 4; b++)
#pragma unroll
            for (int q = 0; q < 16; q++) acc[a][b][q] = 0.0f;
    if constexpr (SPREAD) {
        static_assert(RAW && KM == 4 && NS == 2 && !STORE, "the spread DMA: raw 16-word stages, double buffered");
        // piece pc of stage ks: operand A's slots 0 .. KM - 1, then B's
        // (into the buffer of stage ks, the bytes of stage kd: the last stage
        // re-reads its own bytes into the free buffer, so that the pieces
        // need no branch between the MFMAs)
        auto piece = [&](int64_t ks, int64_t kd, int pc) {
            unsigned char* An = mlds_buf + (int)((ks - ks0) & 1) * (2 * MOPB);
            if (pc < KM) mfma_piece<KM>(F, rowbytes, row0, r0, r1, kd * KM, An, tid, pc);
            else mfma_piece<KM>(F, rowbytes, col0, c0, c1, kd * KM, An + MOPB, tid, pc - KM);
        };
        if (ks0 < ks1)
            for (int pc = 0; pc < 2 * KM; pc++) piece(ks0, ks0, pc);
        for (int64_t ks = ks0; ks < ks1; ks++) {
            // stage ks landed everywhere, and stage ks - 1's buffer is free
            asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
            const int64_t kd = ks + 1 < ks1 ? ks + 1 : ks;
            const unsigned char* A = mlds_buf + (int)((ks - ks0) & 1) * (2 * MOPB);
            const unsigned char* B = A + MOPB;
#pragma unroll
            for (int q = 0; q < KM; q++) {
                v4i_t af[2], bf[4];
#pragma unroll
                for (int a = 0; a < 2; a++)
                    af[a] = *reinterpret_cast<const v4i_t*>(A + mlds<KM>(wr * 64 + a * 32 + r, KM * h + q));
#pragma unroll
                for (int b = 0; b < 4; b++)
                    bf[b] = *reinterpret_cast<const v4i_t*>(B + mlds<KM>(wc * 128 + b * 32 + r, KM * h + q));
#pragma unroll
                for (int m = 0; m < 4; m++) {
                    v4i_t an[2], bn[4];
                    if constexpr (PLANE) {
#pragma unroll
                        for (int a = 0; a < 2; a++)
                            an[a] = v4i_t{bit_plane((uint32_t)af[a][0], m), bit_plane((uint32_t)af[a][1], m),
                                          bit_plane((uint32_t)af[a][2], m), bit_plane((uint32_t)af[a][3], m)};
#pragma unroll
                        for (int b = 0; b < 4; b++)
                            bn[b] = v4i_t{bit_plane((uint32_t)bf[b][0], m), bit_plane((uint32_t)bf[b][1], m),
                                          bit_plane((uint32_t)bf[b][2], m), bit_plane((uint32_t)bf[b][3], m)};
                    } else {
#pragma unroll
                        for (int a = 0; a < 2; a++) an[a] = raw_nibbles((uint32_t)af[a][m]);
#pragma unroll
                        for (int b = 0; b < 4; b++) bn[b] = raw_nibbles((uint32_t)bf[b][m]);
                    }
                    // plane m's nibbles are 0.5 / 1.0 / 2.0 / 2.0: scales 2, 1, 1/2, 1/2 a side
                    constexpr int kPlaneScale[4] = {128, 127, 126, 126};
                    const int sc = PLANE ? kPlaneScale[m] : 0;
#pragma unroll
                    for (int a = 0; a < 2; a++)
#pragma unroll
                        for (int b = 0; b < 4; b++) {
                            const v8i_t av = {an[a][0], an[a][1], an[a][2], an[a][3], 0, 0, 0, 0};
                            const v8i_t bv = {bn[b][0], bn[b][1], bn[b][2], bn[b][3], 0, 0, 0, 0};
                            acc[a][b] =
                                __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, acc[a][b], 4, 4, 0, sc, 0, sc);
                        }
                    if (q * 4 + m < 2 * KM) piece(ks + 1, kd, q * 4 + m);
                }
            }
        }
    } else {
    auto issue = [&](int64_t ks) {
        unsigned char* An = mlds_buf + (int)((ks - ks0) % NS) * (2 * MOPB);
        mfma_stage<KM>(F, rowbytes, row0, r0, r1, ks * KM, An, tid);
        mfma_stage<KM>(F, rowbytes, col0, c0, c1, ks * KM, An + MOPB, tid);
    };
    for (int64_t k = ks0; k < ks1 && k < ks0 + NS - 1; k++) issue(k);
    for (int64_t ks = ks0; ks < ks1; ks++) {
        const unsigned char* A = mlds_buf + (int)((ks - ks0) % NS) * (2 * MOPB);
        const unsigned char* B = A + MOPB;
        if (ks + NS - 1 < ks1) issue(ks + NS - 1);
        // stages issued after ks: min(NS - 1, ks1 - 1 - ks)
        const int64_t later = ks1 - 1 - ks < NS - 1 ? ks1 - 1 - ks : NS - 1;
        mfma_wait<2 * KM>((int)later);               // stage ks landed everywhere
        if constexpr (RAW) {
            // KM = 4: 128-byte rows (16 words a stage); KM = 2: 64-byte rows
            // (8 words), a 64 KiB double-buffered ring (option bitset_mfma_km 2)
            // lane half h takes chunks KM h .. KM h + KM - 1 of its row
#pragma unroll
            for (int q = 0; q < KM; q++) {
                v4i_t af[2], bf[4];
#pragma unroll
                for (int a = 0; a < 2; a++)
                    af[a] = *reinterpret_cast<const v4i_t*>(A + mlds<KM>(wr * 64 + a * 32 + r, KM * h + q));
#pragma unroll
                for (int b = 0; b < 4; b++)
                    bf[b] = *reinterpret_cast<const v4i_t*>(B + mlds<KM>(wc * 128 + b * 32 + r, KM * h + q));
#pragma unroll
                for (int m = 0; m < 4; m++) {
                    v4i_t an[2], bn[4];
#pragma unroll
                    for (int a = 0; a < 2; a++) an[a] = raw_nibbles((uint32_t)af[a][m]);
#pragma unroll
                    for (int b = 0; b < 4; b++) bn[b] = raw_nibbles((uint32_t)bf[b][m]);
#pragma unroll
                    for (int a = 0; a < 2; a++)
#pragma unroll
                        for (int b = 0; b < 4; b++) {
                            const v8i_t av = {an[a][0], an[a][1], an[a][2], an[a][3], 0, 0, 0, 0};
                            const v8i_t bv = {bn[b][0], bn[b][1], bn[b][2], bn[b][3], 0, 0, 0, 0};
                            acc[a][b] =
                                __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, acc[a][b], 4, 4, 0, 0, 0, 0);
                        }
                }
            }
        } else
#pragma unroll
        for (int kk = 0; kk < KM; kk++) {
            v4i_t af[2], bf[4];
#pragma unroll
            for (int a = 0; a < 2; a++)
                af[a] = *reinterpret_cast<const v4i_t*>(A + mlds<KM>(wr * 64 + a * 32 + r, 2 * kk + h));
#pragma unroll
            for (int b = 0; b < 4; b++)
                bf[b] = *reinterpret_cast<const v4i_t*>(B + mlds<KM>(wc * 128 + b * 32 + r, 2 * kk + h));
#pragma unroll
            for (int a = 0; a < 2; a++)
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const v8i_t av = {af[a][0], af[a][1], af[a][2], af[a][3], 0, 0, 0, 0};
                    const v8i_t bv = {bf[b][0], bf[b][1], bf[b][2], bf[b][3], 0, 0, 0, 0};
                    acc[a][b] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, acc[a][b], 4, 4, 0, 0, 0, 0);
                }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // stage free for the next DMA
    }
    }
    // D of block (a, b): row (q & 3) + 8 (q >> 2) + 4 h of the block, column r
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 4; b++)
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const int64_t i = row0 + wr * 64 + a * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
                const int64_t j = col0 + wc * 128 + b * 32 + r;
                const int v = (int)acc[a][b][q];
                if (STORE) {
                    if (i < r1 && j < c1 && !(upper && j <= i)) I[(i - r0) * ldI + (j - c0)] = v;
                } else if (v && i < r1 && j < c1 && !(upper && j <= i)) {
                    atomicAdd(I + (i - r0) * ldI + (j - c0), v);
                }
            }
}

// Self pairs: |A ∩ A| = |A|. The pruned dictionary drops kmers held by one
// set only, so the bitset count of a self pair misses them; take |A|.
__global__ void self_pairs_kernel(const int64_t* __restrict__ off, int64_t lo, int64_t hi, int64_t r0, int64_t c0,
                                  int32_t* __restrict__ I, int64_t ldI) {
    const int64_t i = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= hi) return;
    I[(i - r0) * ldI + (i - c0)] = (int32_t)(off[i + 1] - off[i]);
}

// Java expression of SequenceKmers.distance, fp64 with contraction off:
// d = I > 0 ? 1.0 - (double)I / (double)(nA + nB - I) : 1.0
__global__ void epilogue_kernel(const int64_t* __restrict__ off, int64_t r0, int64_t r1, int64_t c0,
                                int64_t c1, int upper, int empty_nan, const int32_t* __restrict__ I,
                                int64_t ldI, double* __restrict__ D, int64_t ldD) {
#pragma clang fp contract(off)
    const int64_t ncol = c1 - c0;
    const int64_t n = (r1 - r0) * ncol;
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
        const int64_t ri = e / ncol, cj = e - ri * ncol;
        const int64_t i = r0 + ri, j = c0 + cj;
        if (upper && j <= i) continue;
        const int64_t inter = I[ri * ldI + cj];
        const int64_t na = off[i + 1] - off[i], nb = off[j + 1] - off[j];
        double d;
        if (inter > 0) {
            const double uni = (double)(na + nb - inter);
            d = 1.0 - (double)inter / uni;
        } else {
            d = (empty_nan && na + nb == 0) ? __builtin_nan("") : 1.0;
        }
        D[ri * ldD + cj] = d;
    }
}

// The epilogue by rows: block row a (set i = r0 + a), its columns [lo, nc)
// (upper: j > i) strided over the blocks of the row; the same expression as
// epilogue_kernel
__global__ __launch_bounds__(256) void epilogue_rows_kernel(const int64_t* __restrict__ off, int64_t r0, int64_t c0,
                                                            int64_t nc, int upper, int empty_nan,
                                                            const int32_t* __restrict__ I, int64_t ldI,
                                                            double* __restrict__ D, int64_t ldD) {
#pragma clang fp contract(off)
    const int64_t a = blockIdx.y, i = r0 + a;
    const int64_t l0 = upper ? i + 1 - c0 : 0;
    const int64_t lo = l0 > 0 ? l0 : 0;
    const int64_t na = off[i + 1] - off[i];
    const int32_t* Ir = I + a * ldI;
    double* Dr = D + a * ldD;
    for (int64_t b = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nc; b += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = c0 + b;
        const int64_t inter = Ir[b];
        const int64_t nb = off[j + 1] - off[j];
        double d;
        if (inter > 0) {
            const double uni = (double)(na + nb - inter);
            d = 1.0 - (double)inter / uni;
        } else {
            d = (empty_nan && na + nb == 0) ? __builtin_nan("") : 1.0;
        }
        Dr[b] = d;
    }
}

// one query row against a column list: one wave per column, streaming
__global__ __launch_bounds__(256) void bitset_row_kernel(const unsigned long long* __restrict__ bits, int64_t W,
                                                         int64_t q, const int64_t* __restrict__ cols,
                                                         int64_t ncols, int32_t* __restrict__ I) {
    const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (c >= ncols) return;
    const unsigned long long* a = bits + q * W;
    const unsigned long long* b = bits + cols[c] * W;
    uint32_t acc = 0;
    for (int64_t w = lane; w < W; w += 64) acc += __popcll(a[w] & b[w]);
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) I[c] = (cols[c] == q) ? -1 : (int32_t)acc;   // -1: self pair, fixed by the epilogue
}

__global__ void row_epilogue_kernel(const int64_t* __restrict__ off, int64_t q, const int64_t* __restrict__ cols,
                                    int64_t ncols, int empty_nan, const int32_t* __restrict__ I,
                                    double* __restrict__ D) {
#pragma clang fp contract(off)
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= ncols) return;
    const int64_t j = cols[c];
    const int64_t na = off[q + 1] - off[q], nb = off[j + 1] - off[j];
    const int64_t inter = (j == q) ? na : I[c];
    double d;
    if (inter > 0) {
        const double uni = (double)(na + nb - inter);
        d = 1.0 - (double)inter / uni;
    } else {
        d = (empty_nan && na + nb == 0) ? __builtin_nan("") : 1.0;
    }
    D[c] = d;
}

}  // namespace

void bitset_row(gdist_ctx* ctx, const gdist_sets* s, int64_t q, const int64_t* d_cols, int64_t ncols,
                int32_t* d_I) {
    if (ncols <= 0) return;
    bitset_row_kernel<<<(unsigned)ceil_div(ncols, 4), 256, 0, ctx->stream>>>(s->bits.as<unsigned long long>(), s->W,
                                                                             q, d_cols, ncols, d_I);
    GD_HIP(hipGetLastError());
    if (s->n_rare > 0 || s->variant) {
        DevBuf cnt(s->nsets * 4 + 4, ctx->stream);
        GD_HIP(hipMemsetAsync(cnt.p, 0, s->nsets * 4, ctx->stream));
        if (s->n_rare > 0)
            rare_query_kernel<<<256, 256, 0, ctx->stream>>>(s->srare_off.as<int64_t>(), s->srare_ent.as<uint64_t>(),
                                                            s->srare_w.as<uint32_t>(), s->post_sets.as<uint32_t>(), q,
                                                            cnt.as<int32_t>());
        variant_query(ctx, s, q, cnt.as<int32_t>());
        gather_add_kernel<<<(unsigned)ceil_div(ncols, 256), 256, 0, ctx->stream>>>(d_cols, ncols, cnt.as<int32_t>(),
                                                                                   d_I);
        GD_HIP(hipGetLastError());
        GD_HIP(hipStreamSynchronize(ctx->stream));
    }
}

void row_epilogue(gdist_ctx* ctx, const gdist_sets* s, int64_t q, const int64_t* d_cols, int64_t ncols,
                  unsigned flags, const int32_t* d_I, double* d_D) {
    if (ncols <= 0) return;
    row_epilogue_kernel<<<(unsigned)ceil_div(ncols, 256), 256, 0, ctx->stream>>>(
        s->off.as<int64_t>(), q, d_cols, ncols, (flags & GDIST_EMPTY_NAN) ? 1 : 0, d_I, d_D);
    GD_HIP(hipGetLastError());
}

// ---- dictionary construction ------------------------------------------
// A Summary is a sorted array of distinct codes with the number of sets
// holding each. Summaries of disjoint set ranges merge by summing counts; the
// dictionary is the codes with count >= 2 (or all codes, keep_singletons).

namespace {

constexpr int64_t kBitsChunk = int64_t(1) << 30;   // codes per working chunk

// (keys sorted) -> runs: unique codes, run starts, run count
void runs_of(gdist_ctx* ctx, const uint64_t* keys, int64_t n, DevBuf& flag, DevBuf& pos, DevBuf& uniq,
             DevBuf& start, int64_t& nruns) {
    hipStream_t st = ctx->stream;
    flag.alloc(n * 4 + 4, st);
    pos.alloc(n * 8 + 8, st);
    nruns = 0;
    if (n == 0) { uniq.alloc(8, st); start.alloc(8, st); return; }
    head_flags_u64<<<grid_for(n), 256, 0, st>>>(keys, n, flag.as<int32_t>());
    GD_HIP(hipGetLastError());
    exclusive_scan_i32_to_i64(ctx, flag.as<int32_t>(), pos.as<int64_t>(), (size_t)n);
    int64_t last = 0;
    int32_t lf = 0;
    d2h(&last, pos.as<int64_t>() + n - 1, 8, st);
    d2h(&lf, flag.as<int32_t>() + n - 1, 4, st);
    GD_HIP(hipStreamSynchronize(st));
    nruns = last + lf;
    uniq.alloc(nruns * 8 + 8, st);
    start.alloc(nruns * 8 + 8, st);
    run_heads_kernel<<<grid_for(n), 256, 0, st>>>(keys, flag.as<int32_t>(), pos.as<int64_t>(), n,
                                                   uniq.as<uint64_t>(), start.as<int64_t>());
    GD_HIP(hipGetLastError());
}

// merge (codes, counts) parts into one summary
void merge_parts(gdist_ctx* ctx, const std::vector<SummaryView>& parts, Summary& out, int end_bit = 64) {
    hipStream_t st = ctx->stream;
    int64_t m = 0;
    for (auto& p : parts) m += p.n;
    DevBuf kA(m * 8 + 8, st), kB(m * 8 + 8, st), vA(m * 4 + 4, st), vB(m * 4 + 4, st);
    int64_t at = 0;
    for (auto& p : parts) {
        if (p.n) {
            GD_HIP(hipMemcpyAsync(kA.as<uint64_t>() + at, p.codes, p.n * 8, hipMemcpyDeviceToDevice, st));
            GD_HIP(hipMemcpyAsync(vA.as<uint32_t>() + at, p.counts, p.n * 4, hipMemcpyDeviceToDevice, st));
        }
        at += p.n;
    }
    uint64_t* keys = kA.as<uint64_t>(); uint64_t* kalt = kB.as<uint64_t>();
    int32_t* vals = vA.as<int32_t>(); int32_t* valt = vB.as<int32_t>();
    if (parts.size() > 1) sort_pairs_u64_i32(ctx, keys, kalt, vals, valt, (size_t)m, 0, end_bit);
    DevBuf flag, pos, start;
    runs_of(ctx, keys, m, flag, pos, out.codes, start, out.n);
    // per-run sum of counts via prefix sums of the counts
    DevBuf wide((m + 1) * 8, st), cw((m + 1) * 8, st);
    if (m) {
        widen_u32_kernel<<<grid_for(m), 256, 0, st>>>(reinterpret_cast<const uint32_t*>(vals), m, wide.as<int64_t>());
        GD_HIP(hipGetLastError());
    }
    GD_HIP(hipMemsetAsync(wide.as<int64_t>() + m, 0, 8, st));
    exclusive_scan_i64(ctx, wide.as<int64_t>(), cw.as<int64_t>(), (size_t)(m + 1));
    out.counts.alloc(out.n * 4 + 4, st);
    if (out.n) {
        run_totals_kernel<<<(int)ceil_div(out.n, 256), 256, 0, st>>>(start.as<int64_t>(), out.n, m, cw.as<int64_t>(),
                                                                      out.counts.as<uint32_t>());
        GD_HIP(hipGetLastError());
    }
    GD_HIP(hipStreamSynchronize(st));
}

}  // namespace

// Summary of sets [0, nsets): chunked sort + run-length, then merge.
void local_summary(gdist_ctx* ctx, const gdist_sets* s, Summary& out) {
    hipStream_t st = ctx->stream;
    const int cbits = std::min(64, code_bits(s->kind, s->k, s->flags));
    if (!s->pack_sum.empty()) {
        // the pack's chunk summaries (code-major pack sort): merge, no code sort
        if (s->pack_sum.size() == 1) {
            const Summary& p = s->pack_sum[0];
            out.n = p.n;
            out.codes.alloc(p.n * 8 + 8, st);
            out.counts.alloc(p.n * 4 + 4, st);
            if (p.n) {
                GD_HIP(hipMemcpyAsync(out.codes.p, p.codes.p, p.n * 8, hipMemcpyDeviceToDevice, st));
                GD_HIP(hipMemcpyAsync(out.counts.p, p.counts.p, p.n * 4, hipMemcpyDeviceToDevice, st));
            }
            GD_HIP(hipStreamSynchronize(st));
            return;
        }
        std::vector<SummaryView> parts;
        for (auto& p : s->pack_sum) parts.push_back({p.codes.as<uint64_t>(), p.counts.as<uint32_t>(), p.n});
        merge_parts(ctx, parts, out, cbits);
        return;
    }
    std::vector<Summary> chunks;
    int64_t s0 = 0;
    while (s0 < s->nsets) {
        int64_t s1 = s0 + 1;
        while (s1 < s->nsets && s->h_off[s1 + 1] - s->h_off[s0] <= kBitsChunk) s1++;
        const int64_t b = s->h_off[s0], n = s->h_off[s1] - b;
        DevBuf kA(n * 8 + 8, st), kB(n * 8 + 8, st);
        if (n) GD_HIP(hipMemcpyAsync(kA.p, s->codes.as<uint64_t>() + b, n * 8, hipMemcpyDeviceToDevice, st));
        uint64_t* keys = kA.as<uint64_t>(); uint64_t* alt = kB.as<uint64_t>();
        sort_keys_u64(ctx, keys, alt, (size_t)n, 0, cbits);
        Summary c;
        DevBuf flag, pos, start;
        runs_of(ctx, keys, n, flag, pos, c.codes, start, c.n);
        c.counts.alloc(c.n * 4 + 4, st);
        if (c.n) {   // codes are unique per set: run length = number of sets
            run_totals_kernel<<<(int)ceil_div(c.n, 256), 256, 0, st>>>(start.as<int64_t>(), c.n, n, nullptr,
                                                                        c.counts.as<uint32_t>());
            GD_HIP(hipGetLastError());
        }
        GD_HIP(hipStreamSynchronize(st));
        chunks.push_back(std::move(c));
        s0 = s1;
    }
    if (chunks.size() == 1) {
        out.codes = std::move(chunks[0].codes);
        out.counts = std::move(chunks[0].counts);
        out.n = chunks[0].n;
        return;
    }
    std::vector<SummaryView> parts;
    for (auto& c : chunks) parts.push_back({c.codes.as<uint64_t>(), c.counts.as<uint32_t>(), c.n});
    merge_parts(ctx, parts, out);
}

namespace {
// hist[c] += number of summary entries with count c (c <= nsets); small
// counts (the singletons dominate) go through an LDS histogram first
constexpr int kHistLds = 4096;
__global__ void count_hist_kernel(const uint32_t* __restrict__ cnt, int64_t n, int64_t nsets,
                                  unsigned long long* __restrict__ hist) {
    __shared__ unsigned int h[kHistLds];
    for (int t = threadIdx.x; t < kHistLds; t += blockDim.x) h[t] = 0;
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t c = cnt[i] < (uint32_t)nsets ? (int64_t)cnt[i] : nsets;
        if (c < kHistLds) atomicAdd(&h[c], 1u);
        else atomicAdd(&hist[c], 1ull);
    }
    __syncthreads();
    for (int t = threadIdx.x; t < kHistLds && t <= nsets; t += blockDim.x)
        if (h[t]) atomicAdd(&hist[t], (unsigned long long)h[t]);
}

}  // namespace

// Dictionary tiers from merged summaries: dense = codes held by >= T sets
// (all codes with keep_singletons), rare = codes held by 2..T-1 sets.
// rare_mass = number of (code, set) records the rare tier will produce.
void dictionary_from(gdist_ctx* ctx, const std::vector<SummaryView>& parts, bool keep, int64_t& T, int64_t nsets,
                     DevBuf& dict, int64_t& U, DevBuf& rare, int64_t& Ur, int64_t& rare_mass, DevBuf* dcounts) {
    hipStream_t st = ctx->stream;
    Summary all;
    SummaryView m = parts.size() == 1 ? parts[0] : SummaryView{nullptr, nullptr, 0};
    if (parts.size() != 1) {
        merge_parts(ctx, parts, all);
        m = {all.codes.as<uint64_t>(), all.counts.as<uint32_t>(), all.n};
    }
    const int64_t n = m.n;
    if (keep) T = 0;
    if (T < 0) {
        if (ctx->has_option(OPT_RARE_T)) {
            T = ctx->option(OPT_RARE_T, -1);
        } else {
            DevBuf dh((nsets + 1) * 8, st);
            GD_HIP(hipMemsetAsync(dh.p, 0, (nsets + 1) * 8, st));
            if (n) {
                count_hist_kernel<<<grid_for(n, 256, 256 * 16), 256, 0, st>>>(m.counts, n, nsets,
                                                                             dh.as<unsigned long long>());
                GD_HIP(hipGetLastError());
            }
            std::vector<uint64_t> hist(nsets + 1);
            d2h(hist.data(), dh.p, (nsets + 1) * 8, st);
            GD_HIP(hipStreamSynchronize(st));
            T = choose_rare_threshold(hist, nsets);
        }
    }
    U = Ur = rare_mass = 0;
    DevBuf df(n * 4 + 4, st), rf(n * 4 + 4, st), dpos(n * 8 + 8, st), rpos(n * 8 + 8, st), mass(n * 8 + 8, st),
        cmass(n * 8 + 8, st);
    if (n) {
        rare_flag_kernel<<<grid_for(n), 256, 0, st>>>(m.counts, n, T, keep ? 1 : 0, df.as<int32_t>(), rf.as<int32_t>(),
                                                      mass.as<int64_t>());
        GD_HIP(hipGetLastError());
        exclusive_scan_i32_to_i64(ctx, df.as<int32_t>(), dpos.as<int64_t>(), (size_t)n);
        exclusive_scan_i32_to_i64(ctx, rf.as<int32_t>(), rpos.as<int64_t>(), (size_t)n);
        exclusive_scan_i64(ctx, mass.as<int64_t>(), cmass.as<int64_t>(), (size_t)n);
        int64_t h[6];
        int32_t hf[2];
        d2h(&h[0], dpos.as<int64_t>() + n - 1, 8, st);
        d2h(&h[1], rpos.as<int64_t>() + n - 1, 8, st);
        d2h(&h[2], cmass.as<int64_t>() + n - 1, 8, st);
        d2h(&h[3], mass.as<int64_t>() + n - 1, 8, st);
        d2h(&hf[0], df.as<int32_t>() + n - 1, 4, st);
        d2h(&hf[1], rf.as<int32_t>() + n - 1, 4, st);
        U = h[0] + hf[0];
        Ur = h[1] + hf[1];
        rare_mass = h[2] + h[3];
    }
    dict.alloc(U * 8 + 8, st);
    rare.alloc(Ur * 8 + 8, st);
    if (dcounts) dcounts->alloc(U * 4 + 4, st);
    if (n) {
        compact_u64_kernel<<<grid_for(n), 256, 0, st>>>(m.codes, df.as<int32_t>(), dpos.as<int64_t>(), n,
                                                        dict.as<uint64_t>());
        if (dcounts)
            compact_u32_kernel<<<grid_for(n), 256, 0, st>>>(m.counts, df.as<int32_t>(), dpos.as<int64_t>(), n,
                                                            dcounts->as<uint32_t>());
        compact_u64_kernel<<<grid_for(n), 256, 0, st>>>(m.codes, rf.as<int32_t>(), rpos.as<int64_t>(), n,
                                                        rare.as<uint64_t>());
        GD_HIP(hipGetLastError());
    }
    GD_HIP(hipStreamSynchronize(st));
}

namespace {
__global__ void local_mass_kernel(const uint64_t* __restrict__ codes, const uint32_t* __restrict__ cnt, int64_t n,
                                  const uint64_t* __restrict__ rare, int64_t Ur, unsigned long long* __restrict__ out) {
    unsigned long long acc = 0;
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t k = codes[i];
        int64_t lo = 0, hi = Ur;
        while (lo < hi) {
            int64_t mid = (lo + hi) >> 1;
            if (rare[mid] < k) lo = mid + 1; else hi = mid;
        }
        if (lo < Ur && rare[lo] == k) acc += cnt[i];
    }
    if (acc) atomicAdd(out, acc);
}

// over the posting lists: sum of m(m-1)/2 (the rare tier's pair increments)
// -> out[0], the longest list -> out[1], the increments of kLongList+ lists
// -> out[2]. One atomic of each kind per workgroup.
__global__ __launch_bounds__(256) void rare_incs_kernel(const int64_t* __restrict__ post_off, int64_t n,
                                                        unsigned long long* __restrict__ out) {
    __shared__ unsigned long long part[3][4];
    unsigned long long acc = 0, mx = 0, lng = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; l < n; l += stride) {
        const unsigned long long m = (unsigned long long)(post_off[l + 1] - post_off[l]);
        const unsigned long long inc = m * (m - 1) / 2;
        acc += inc;
        if (m >= (unsigned long long)kLongList) lng += inc;
        mx = m > mx ? m : mx;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        acc += __shfl_xor(acc, o, 64);
        lng += __shfl_xor(lng, o, 64);
        const unsigned long long om = __shfl_xor(mx, o, 64);
        mx = om > mx ? om : mx;
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { part[0][w] = acc; part[1][w] = mx; part[2][w] = lng; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int v = 1; v < (int)(blockDim.x >> 6); v++) {
            acc += part[0][v]; lng += part[2][v];
            mx = part[1][v] > mx ? part[1][v] : mx;
        }
        if (acc) atomicAdd(out, acc);
        if (mx) atomicMax(out + 1, mx);
        if (lng) atomicAdd(out + 2, lng);
    }
}

}  // namespace

// records the local sets contribute to the rare tier (local counts of rare codes)
int64_t local_rare_mass(gdist_ctx* ctx, const Summary& local, const uint64_t* rare, int64_t Ur) {
    hipStream_t st = ctx->stream;
    if (Ur == 0 || local.n == 0) return 0;
    DevBuf c(8, st);
    GD_HIP(hipMemsetAsync(c.p, 0, 8, st));
    local_mass_kernel<<<grid_for(local.n), 256, 0, st>>>(local.codes.as<uint64_t>(), local.counts.as<uint32_t>(),
                                                         local.n, rare, Ur, c.as<unsigned long long>());
    GD_HIP(hipGetLastError());
    int64_t h = 0;
    d2h(&h, c.p, 8, st);
    return h;
}

int64_t bitset_words(int64_t dict_size) {
    return std::max<int64_t>(KC, ceil_div(ceil_div(dict_size, 64), KC) * KC);
}

int64_t auto_rare_threshold(int64_t nsets) {
    // Fixed heuristic (before the histogram model): a dense entry costs one
    // bit column over all N^2/2 pairs, a rare entry held by m sets m(m-1)/2
    // pair increments; ~N/80 balances them for C2-like collections.
    return std::max<int64_t>(2, nsets / 80);
}

int64_t choose_rare_threshold(const std::vector<uint64_t>& hist, int64_t nsets) {
    // cost(T) = pairs * W(dense kmers with count >= T) / dense rate
    //         + the cheaper rare kernel on the lists of kmers with 2 <= count < T
    // over the whole triangle, for every T in [2, nsets+1]; T = 2 is dense-only.
    const double pairs = 0.5 * (double)nsets * (double)(nsets - 1);
    const int64_t top = (int64_t)hist.size() - 1;
    std::vector<double> dense_ge(top + 2, 0.0);
    for (int64_t c = top; c >= 2; c--) dense_ge[c] = dense_ge[c + 1] + (double)hist[c];
    RareTier t;
    double best = -1.0;
    int64_t bestT = 2;
    for (int64_t T = 2; T <= top + 1; T++) {
        if (T > 2) {
            const double c = (double)(T - 1), h = (double)hist[T - 1], inc = h * c * (c - 1.0) / 2.0;
            t.incs += inc;
            if (T - 1 >= kLongList) t.incs_long += inc;
            t.records += h * c;
            t.lists += h;
        }
        const double U = T <= top ? dense_ge[T] : 0.0;
        const double cost = pairs * (double)bitset_words((int64_t)U) / kDenseWordPairsPerS + rare_choice(t, 1.0, 1.0).cost();
        if (best < 0 || cost < best) { best = cost; bestT = T; }
    }
    return bestT;
}

// The fill without a sort: each set's codes are sorted (pack), and so are
// the dense dictionary and the rare codes, so a wave takes a segment of
// kFillSeg consecutive codes of ONE set, finds the segment's window in the
// dictionary and in the rare codes (four binary searches, one lane each),
// and each lane then searches its codes inside those windows (L1-resident).
// Dense codes set their bit (locus position through perm), rare codes append
// a (rare rank << 32 | set) record; singletons are skipped. Segments that
// straddle a set boundary are cut there, so a window is always monotone.
constexpr int kFillSeg = 2048;
__device__ __forceinline__ int64_t lower_bound_u64(const uint64_t* __restrict__ a, int64_t lo, int64_t hi, uint64_t k) {
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] < k) lo = mid + 1; else hi = mid;
    }
    return lo;
}
__global__ __launch_bounds__(256) void fill_search_kernel(
    const uint64_t* __restrict__ codes, const int64_t* __restrict__ off, const int64_t* __restrict__ seg,
    int64_t nseg, const uint64_t* __restrict__ dict, int64_t U, const uint64_t* __restrict__ rare, int64_t Ur,
    int64_t W, unsigned long long* __restrict__ bits, int64_t id_base, unsigned long long* __restrict__ rare_out,
    unsigned long long* __restrict__ rare_cnt, int64_t rare_cap, const uint32_t* __restrict__ perm) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (wave >= nseg) return;
    // segment: (set << 40 | first code index) packed, its end the next segment's start or its set's end
    const uint64_t sd = (uint64_t)seg[wave];
    const int64_t set = (int64_t)(sd >> 40), b = (int64_t)(sd & ((1ull << 40) - 1));
    const int64_t e = std::min<int64_t>(b + kFillSeg, off[set + 1]);
    if (e <= b) return;
    const uint64_t kfirst = codes[b], klast = codes[e - 1];
    // lanes 0-3: the windows [lower_bound(first), upper_bound(last)) in dict and rare
    int64_t w = 0;
    if (lane == 0) w = lower_bound_u64(dict, 0, U, kfirst);
    else if (lane == 1) w = lower_bound_u64(dict, 0, U, klast + 1 == 0 ? klast : klast + 1) + (klast == ~0ull);
    else if (lane == 2) w = lower_bound_u64(rare, 0, Ur, kfirst);
    else if (lane == 3) w = lower_bound_u64(rare, 0, Ur, klast + 1 == 0 ? klast : klast + 1) + (klast == ~0ull);
    const int64_t dlo = __shfl((long long)w, 0, 64), dhi = std::min<int64_t>(U, __shfl((long long)w, 1, 64));
    const int64_t rlo = __shfl((long long)w, 2, 64), rhi = std::min<int64_t>(Ur, __shfl((long long)w, 3, 64));
    unsigned long long* row = bits + set * W;
    for (int64_t i = b + lane; i < e; i += 64) {
        const uint64_t k = codes[i];
        const int64_t r = lower_bound_u64(dict, dlo, dhi, k);
        if (r < dhi && dict[r] == k) {
            const int64_t pos = perm ? (int64_t)perm[r] : r;     // bit position (locus order)
            atomicOr(row + (pos >> 6), 1ull << (pos & 63));
            continue;
        }
        const int64_t q = lower_bound_u64(rare, rlo, rhi, k);
        if (q < rhi && rare[q] == k) {
            const unsigned long long slot = atomicAdd(rare_cnt, 1ull);
            if ((int64_t)slot < rare_cap)
                rare_out[slot] = ((unsigned long long)q << 32) | (unsigned long long)(uint32_t)(set + id_base);
        }
    }
}

// The default fill, in two passes so that no bit is set by a global atomic
// (a wave's 64 atomicOr land in 64 different rows' cache lines, the slow
// case of the L2 atomic unit: the one-pass fill above spends 0.27 s of C2's
// setup on them).
// Pass 1 (fill_window_kernel + fill_pos_kernel): segments of up to kPosSeg
// consecutive codes of one set (shorter for sets much smaller than the
// dictionary, so that a segment's window fits in LDS). One thread per
// (segment, bound) finds the segment's windows [dlo, dhi) in the dense codes
// and [rlo, rhi) in the rare codes and writes them beside the segment's
// bounds - independent searches, instead of a dependent chain inside the
// wave that uses them. A wave (one per block) then stages its dense window in
// LDS with coalesced loads (codes and their bit positions perm[]), loads its
// codes up front, and each lane binary-searches its codes in LDS. Misses
// (about 1 code in 100 on C2) are listed in LDS and looked up together after
// the dense pass: a search over LDS fences (every 8th rare code of the
// window) and one 64-byte load of the 8-code bucket, so a segment waits on
// one global latency for its rare codes, not one per round. Each code's bit
// position (u32; ~0 outside the dense tier) goes to a position array
// parallel to the codes; rare-tier codes append their records (one atomic
// per wave and round). A window over the LDS caps (a set sparse against the
// dictionary) falls back to a wave walk over global memory.
// (The one-pass fill's per-lane binary searches in global memory chain ~20
// dependent loads per code: it is latency-bound at 0.27 s for C2.)
// Pass 2 (pos_bits_kernel): a workgroup owns one set's row slice of
// kPosSlice 32-bit words in LDS, streams the set's positions, ORs the ones in
// its slice into LDS (ds_or) and stores the slice whole: every row word is
// written once, coalesced, and the row needs no memset.
constexpr int kPosSeg = 512;       // codes per segment (at most)
constexpr int kWinDense = 768;     // LDS dense-window cap (entries)
constexpr int kRareBucket = 8;     // rare codes per LDS fence
constexpr int kRareFences = 256;   // LDS fence cap (a rare window of up to 2048 codes)
constexpr int kPosSlice = 32768;   // 32-bit row words per workgroup (128 KiB of LDS)
constexpr int64_t kFillPosChunk = int64_t(1) << 30;   // codes per position-array chunk (4 GiB)

__device__ __forceinline__ int64_t upper_bound_u64(const uint64_t* __restrict__ a, int64_t lo, int64_t hi, uint64_t k) {
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] <= k) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// per segment 8 int64: dlo, dhi, rlo, rhi, (set << 40 | b), e
__global__ __launch_bounds__(256) void fill_window_kernel(const uint64_t* __restrict__ codes,
                                                          const int64_t* __restrict__ off, const int64_t* __restrict__ seg,
                                                          int64_t ns, const uint64_t* __restrict__ dict, int64_t U,
                                                          const uint64_t* __restrict__ rare, int64_t Ur,
                                                          int64_t* __restrict__ win) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ns * 4) return;
    const int64_t sg = t >> 2;
    const uint64_t sd = (uint64_t)seg[sg];
    const int64_t set = (int64_t)(sd >> 40), b = (int64_t)(sd & ((1ull << 40) - 1));
    int64_t e = off[set + 1];   // the next segment's start within the set
    if (sg + 1 < ns) {
        const uint64_t nx = (uint64_t)seg[sg + 1];
        if ((int64_t)(nx >> 40) == set) e = (int64_t)(nx & ((1ull << 40) - 1));
    }
    const int which = (int)(t & 3);
    const uint64_t* a = which < 2 ? dict : rare;
    const int64_t n = which < 2 ? U : Ur;
    win[sg * 8 + which] = (which & 1) ? upper_bound_u64(a, 0, n, codes[e - 1]) : lower_bound_u64(a, 0, n, codes[b]);
    if (which == 0) {
        win[sg * 8 + 4] = (int64_t)sd;
        win[sg * 8 + 5] = e;
    }
}

// Ranks of the active lanes' codes k (sorted across lanes) in a[P, hi) of
// global memory (the fallback walk): rk = lower bound, hit = a[rk] == k. P is
// uniform and only moves forward; on return it is the largest active rank.
__device__ __forceinline__ void wave_rank(const uint64_t* __restrict__ a, int64_t& P, int64_t hi, uint64_t k,
                                          bool active, int64_t& rk, bool& hit) {
    const int lane = threadIdx.x & 63;
    bool pend = active;
    rk = hi;
    hit = false;
    for (int round = 0; __ballot(pend); round++) {
        const int nb = (int)std::min<int64_t>(64, hi - P);
        if (nb <= 0) break;   // pending lanes: past the end (rk = hi, no hit)
        const uint64_t B = lane < nb ? a[P + lane] : ~0ull;
        int c = 0;   // # block codes < k
#pragma unroll
        for (int st = 32; st >= 1; st >>= 1) {
            const uint64_t v = (uint64_t)__shfl((long long)B, c + st - 1, 64);
            if (c + st <= nb && v < k) c += st;
        }
        const uint64_t v = (uint64_t)__shfl((long long)B, c & 63, 64);
        if (c < nb && v < k) c++;
        const uint64_t m = (uint64_t)__shfl((long long)B, c & 63, 64);
        if (pend && (c < nb || P + nb >= hi)) {
            rk = P + c;
            hit = c < nb && m == k;
            pend = false;
        }
        const unsigned long long left = __ballot(pend);
        if (!left) break;
        const uint64_t kmin = (uint64_t)__shfl((long long)k, __ffsll((long long)left) - 1, 64);
        P += nb;
        if (round >= 1) P = lower_bound_u64(a, P, hi, kmin);   // uniform: a gap, search it
    }
    const unsigned long long act = __ballot(active);
    if (act) P = __shfl((long long)rk, 63 - __clzll((long long)act), 64);
}

// lower bound of k in LDS a[0, n)
__device__ __forceinline__ int lds_lower_bound(const uint64_t* a, int n, uint64_t k) {
    int lo = 0;
    for (int len = n; len > 0;) {
        const int half = len >> 1;
        if (a[lo + half] < k) { lo += half + 1; len -= half + 1; } else len = half;
    }
    return lo;
}

// Rare-tier records of a one-wave block, staged in LDS and appended to the
// output with ONE atomic per kRareBuf records: C2's fill appended ~17 records
// a segment with one atomic each on a single counter (2 M per launch), and
// same-address atomics run at ~0.1 G/s — 84 of the fill's 112 ms.
constexpr int kRareBuf = 256;
struct WaveRareBuf {
    unsigned long long* buf;              // LDS [cap]
    int n;                                // records staged (wave-uniform)
    int cap;
};
__device__ __forceinline__ void rare_flush(WaveRareBuf& rb, unsigned long long* __restrict__ rare_out,
                                           unsigned long long* __restrict__ rare_cnt, int64_t rare_cap) {
    if (!rb.n) return;
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const int lane = threadIdx.x & 63;
    unsigned long long g = 0;
    if (lane == 0) g = atomicAdd(rare_cnt, (unsigned long long)rb.n);
    g = (unsigned long long)__shfl((long long)g, 0, 64);
    for (int j = lane; j < rb.n; j += 64)
        if ((int64_t)(g + j) < rare_cap) rare_out[g + j] = rb.buf[j];
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    rb.n = 0;
}
__device__ __forceinline__ void append_rare(bool rhit, int64_t q, int64_t set, int64_t id_base, WaveRareBuf& rb,
                                            unsigned long long* __restrict__ rare_out,
                                            unsigned long long* __restrict__ rare_cnt, int64_t rare_cap) {
    const unsigned long long m = __ballot(rhit);
    if (!m) return;
    const int c = __popcll(m);
    if (rb.n + c > rb.cap) rare_flush(rb, rare_out, rare_cnt, rare_cap);
    if (rhit) {
        const int lane = threadIdx.x & 63;
        rb.buf[rb.n + __popcll(m & ((1ull << lane) - 1))] =
            ((unsigned long long)q << 32) | (unsigned long long)(uint32_t)(set + id_base);
    }
    rb.n += c;
}

// one wave per block; the blocks take the segments in turn (their rare
// records staged across segments, above)
__global__ __launch_bounds__(64) void fill_pos_kernel(
    const uint64_t* __restrict__ codes, const int64_t* __restrict__ win, int64_t ns, const uint64_t* __restrict__ dict,
    const uint64_t* __restrict__ rare, int64_t base, uint32_t* __restrict__ pos_out, int64_t id_base,
    unsigned long long* __restrict__ rare_out, unsigned long long* __restrict__ rare_cnt, int64_t rare_cap,
    const uint32_t* __restrict__ perm) {
    __shared__ uint64_t s_d[kWinDense];
    __shared__ uint32_t s_p[kWinDense];
    __shared__ uint64_t s_f[kRareFences];
    __shared__ uint64_t s_mk[kPosSeg];
    __shared__ unsigned long long s_rb[kRareBuf];
    const int lane = threadIdx.x;
    WaveRareBuf rb{s_rb, 0, kRareBuf};
    for (int64_t sg = blockIdx.x; sg < ns; sg += gridDim.x) {
    __syncthreads();                                      // the previous segment's LDS reads are done
    const int64_t wv = lane < 6 ? win[sg * 8 + lane] : 0;
    int64_t dlo = __shfl((long long)wv, 0, 64), dhi = __shfl((long long)wv, 1, 64);
    int64_t rlo = __shfl((long long)wv, 2, 64), rhi = __shfl((long long)wv, 3, 64);
    const uint64_t sd = (uint64_t)__shfl((long long)wv, 4, 64);
    const int64_t e = __shfl((long long)wv, 5, 64);
    const int64_t set = (int64_t)(sd >> 40), b = (int64_t)(sd & ((1ull << 40) - 1));
    const int64_t nd = dhi - dlo, nr = rhi - rlo, nf = (nr + kRareBucket - 1) / kRareBucket;
    if (nd <= kWinDense && nf <= kRareFences) {
        // lane l takes the segment's codes [8 l, 8 l + 8): one binary search
        // for the first, then (codes ascending) a short forward walk per code
        // from the previous code's rank
        constexpr int PL = kPosSeg / 64;
        const int64_t i0 = b + (int64_t)PL * lane;
        uint64_t kk[PL];
#pragma unroll
        for (int j = 0; j < PL; j++) kk[j] = i0 + j < e ? codes[i0 + j] : 0;
        for (int j = lane; j < nd; j += 64) {
            s_d[j] = dict[dlo + j];
            s_p[j] = perm ? perm[dlo + j] : (uint32_t)(dlo + j);
        }
        for (int j = lane; j < nf; j += 64) s_f[j] = rare[rlo + (int64_t)j * kRareBucket];
        __syncthreads();
        int nm = 0;   // misses listed (uniform)
        int r = i0 < e ? lds_lower_bound(s_d, (int)nd, kk[0]) : (int)nd;
#pragma unroll
        for (int j = 0; j < PL; j++) {
            const int64_t i = i0 + j;
            const bool valid = i < e;
            bool miss = false;
            if (valid) {
                const uint64_t k = kk[j];
                // forward from the previous rank: two steps, then a search of the rest
                if (r < nd && s_d[r] < k) {
                    r++;
                    if (r < nd && s_d[r] < k) r = r + 1 + lds_lower_bound(s_d + r + 1, (int)nd - r - 1, k);
                }
                const bool hit = r < nd && s_d[r] == k;
                pos_out[i - base] = hit ? s_p[r] : ~0u;
                miss = !hit;
            }
            const unsigned long long m = __ballot(miss);
            if (miss) s_mk[nm + __popcll(m & ((1ull << lane) - 1))] = kk[j];
            nm += __popcll(m);
        }
        __syncthreads();
        for (int t0 = 0; t0 < nm; t0 += 64) {
            bool rhit = false;
            int64_t q = 0;
            if (t0 + lane < nm && nf > 0) {
                const uint64_t k = s_mk[t0 + lane];
                const int g = lds_lower_bound(s_f, (int)nf, k + 1) - 1;   // last fence <= k (k = ~0: the last fence)
                if (g >= 0 || k == ~0ull) {
                    const int gg = g >= 0 ? g : (int)nf - 1;
                    const int64_t q0 = rlo + (int64_t)gg * kRareBucket;
                    uint64_t v[kRareBucket];
#pragma unroll
                    for (int u = 0; u < kRareBucket; u++) v[u] = q0 + u < rhi ? rare[q0 + u] : 0;
#pragma unroll
                    for (int u = 0; u < kRareBucket; u++)
                        if (q0 + u < rhi && v[u] == k) { rhit = true; q = q0 + u; }
                }
            }
            append_rare(rhit, q, set, id_base, rb, rare_out, rare_cnt, rare_cap);
        }
        continue;
    }
    // fallback: walk the windows in global memory
    for (int64_t i0 = b; i0 < e; i0 += 64) {
        const int64_t i = i0 + lane;
        const bool valid = i < e;
        const uint64_t k = valid ? codes[i] : 0;
        int64_t r;
        bool hit;
        wave_rank(dict, dlo, dhi, k, valid, r, hit);
        if (valid) pos_out[i - base] = hit ? (perm ? perm[r] : (uint32_t)r) : ~0u;
        const bool miss = valid && !hit;
        if (__ballot(miss) && rlo < rhi) {
            int64_t q;
            bool rhit;
            wave_rank(rare, rlo, rhi, k, miss, q, rhit);
            append_rare(rhit, q, set, id_base, rb, rare_out, rare_cnt, rare_cap);
        }
    }
    }
    rare_flush(rb, rare_out, rare_cnt, rare_cap);
}

// The default pass 1 (round 4): a 256-thread workgroup per segment of up to
// kMSeg codes. fill_pos_kernel above runs one wave with 17 KiB of LDS, so a
// CU holds ~9 waves and each waits out its own global and LDS latency chains
// (C2: 21 ms per 2^30 codes). Here four waves share one staged window: the
// dense window (padded one entry in 8 so that lanes whose ranks sit ~8 apart
// spread over the banks instead of 16 to a bank) and the rare fences; a
// thread takes 8 consecutive codes (one search, then the forward walk), its
// bit positions are gathered from perm[] in global memory (8 independent
// loads, no LDS copy), and each wave lists its misses as 16-bit offsets
// (one list per wave: it cannot overflow) and stages its rare records in its
// own buffer. ~37 KiB a workgroup: four workgroups, 16 waves, per CU.
constexpr int kMNT = 256;
constexpr int kMPT = 8;
constexpr int kMSeg = kMNT * kMPT;           // 2048 codes
constexpr int kMWin = 2560;                  // dense window cap
constexpr int kMFences = 1024;               // rare window cap kMFences x kRareBucket
constexpr int kMWaveRare = 128;              // rare records staged per wave
__device__ __forceinline__ int mpad(int r) { return r + (r >> 3); }
__device__ __forceinline__ int lds_lower_bound_pad(const uint64_t* a, int lo, int n, uint64_t k) {
    for (int len = n - lo; len > 0;) {
        const int half = len >> 1;
        if (a[mpad(lo + half)] < k) { lo += half + 1; len -= half + 1; } else len = half;
    }
    return lo;
}
__global__ __launch_bounds__(kMNT) void fill_merge_kernel(
    const uint64_t* __restrict__ codes, const int64_t* __restrict__ win, int64_t ns, const uint64_t* __restrict__ dict,
    const uint64_t* __restrict__ rare, int64_t base, uint32_t* __restrict__ pos_out, int64_t id_base,
    unsigned long long* __restrict__ rare_out, unsigned long long* __restrict__ rare_cnt, int64_t rare_cap,
    const uint32_t* __restrict__ perm) {
    constexpr int NW = kMNT / 64, WC = kMSeg / NW;
    __shared__ uint64_t s_d[kMWin + kMWin / 8];
    __shared__ uint64_t s_f[kMFences];
    __shared__ uint16_t s_mi[NW][WC];
    __shared__ unsigned long long s_rb[NW][kMWaveRare];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    WaveRareBuf rb{s_rb[wv], 0, kMWaveRare};
    for (int64_t sg = blockIdx.x; sg < ns; sg += gridDim.x) {
        const int64_t* w = win + sg * 8;
        const int64_t dlo = w[0], dhi = w[1], rlo = w[2], rhi = w[3];
        const uint64_t sd = (uint64_t)w[4];
        const int64_t e = w[5];
        const int64_t set = (int64_t)(sd >> 40), b = (int64_t)(sd & ((1ull << 40) - 1));
        const int64_t nd = dhi - dlo, nr = rhi - rlo, nf = (nr + kRareBucket - 1) / kRareBucket;
        __syncthreads();                                  // the previous segment's LDS reads are done
        if (nd <= kMWin && nf <= kMFences && e - b <= kMSeg) {
            const int64_t i0 = b + (int64_t)kMPT * threadIdx.x;
            uint64_t kk[kMPT];
#pragma unroll
            for (int j = 0; j < kMPT; j++) kk[j] = i0 + j < e ? codes[i0 + j] : 0;
            for (int j = threadIdx.x; j < nd; j += kMNT) s_d[mpad(j)] = dict[dlo + j];
            for (int j = threadIdx.x; j < nf; j += kMNT) s_f[j] = rare[rlo + (int64_t)j * kRareBucket];
            __syncthreads();
            const int n = (int)nd;
            int r = i0 < e ? lds_lower_bound_pad(s_d, 0, n, kk[0]) : n;
            int nm = 0;                                   // the wave's misses (uniform)
            int rk[kMPT];
            bool hit[kMPT];
#pragma unroll
            for (int j = 0; j < kMPT; j++) {
                const bool valid = i0 + j < e;
                hit[j] = false;
                if (valid) {
                    const uint64_t k = kk[j];
                    if (r < n && s_d[mpad(r)] < k) {
                        r++;
                        if (r < n && s_d[mpad(r)] < k) r = lds_lower_bound_pad(s_d, r + 1, n, k);
                    }
                    hit[j] = r < n && s_d[mpad(r)] == k;
                }
                rk[j] = r;
                const bool miss = valid && !hit[j];
                const unsigned long long m = __ballot(miss);
                if (miss) s_mi[wv][nm + __popcll(m & ((1ull << lane) - 1))] = (uint16_t)(i0 + j - b);
                nm += __popcll(m);
            }
            uint32_t pv[kMPT];
#pragma unroll
            for (int j = 0; j < kMPT; j++)
                pv[j] = hit[j] ? (perm ? perm[dlo + rk[j]] : (uint32_t)(dlo + rk[j])) : ~0u;
#pragma unroll
            for (int j = 0; j < kMPT; j++)
                if (i0 + j < e) pos_out[i0 + j - base] = pv[j];
            __builtin_amdgcn_wave_barrier();
            __atomic_signal_fence(__ATOMIC_SEQ_CST);
            for (int t0 = 0; t0 < nm; t0 += 64) {
                bool rhit = false;
                int64_t q = 0;
                if (t0 + lane < nm && nf > 0) {
                    const uint64_t k = codes[b + s_mi[wv][t0 + lane]];
                    const int g = lds_lower_bound(s_f, (int)nf, k + 1) - 1;   // last fence <= k (k = ~0: the last fence)
                    if (g >= 0 || k == ~0ull) {
                        const int gg = g >= 0 ? g : (int)nf - 1;
                        const int64_t q0 = rlo + (int64_t)gg * kRareBucket;
                        uint64_t v[kRareBucket];
#pragma unroll
                        for (int u = 0; u < kRareBucket; u++) v[u] = q0 + u < rhi ? rare[q0 + u] : 0;
#pragma unroll
                        for (int u = 0; u < kRareBucket; u++)
                            if (q0 + u < rhi && v[u] == k) { rhit = true; q = q0 + u; }
                    }
                }
                append_rare(rhit, q, set, id_base, rb, rare_out, rare_cnt, rare_cap);
            }
            continue;
        }
        // fallback: each wave walks its share of the codes over the windows in global memory
        int64_t dp = dlo, rp = rlo;
        for (int64_t c0 = b + 64 * wv; c0 < e; c0 += kMNT) {
            const int64_t i = c0 + lane;
            const bool valid = i < e;
            const uint64_t k = valid ? codes[i] : 0;
            int64_t r;
            bool hit;
            wave_rank(dict, dp, dhi, k, valid, r, hit);
            if (valid) pos_out[i - base] = hit ? (perm ? perm[r] : (uint32_t)r) : ~0u;
            const bool miss = valid && !hit;
            if (__ballot(miss) && rp < rhi) {
                int64_t q;
                bool rhit;
                wave_rank(rare, rp, rhi, k, miss, q, rhit);
                append_rare(rhit, q, set, id_base, rb, rare_out, rare_cnt, rare_cap);
            }
        }
    }
    rare_flush(rb, rare_out, rare_cnt, rare_cap);
}

__device__ __forceinline__ void pos_or(uint32_t* lds, uint32_t p, uint32_t sb) {
    const uint32_t x = (p >> 5) - sb;   // ~0 positions and other slices wrap to >= kPosSlice
    if (x < (uint32_t)kPosSlice) atomicOr(lds + x, 1u << (p & 31));
}

// grid (slices, sets of the chunk); block 1024
__global__ __launch_bounds__(1024) void pos_bits_kernel(const uint32_t* __restrict__ pos, const int64_t* __restrict__ off,
                                                        int64_t s0, int64_t base, int64_t W, uint32_t* __restrict__ bits) {
    __shared__ uint32_t lds[kPosSlice];
    const int64_t set = s0 + blockIdx.y;
    const int64_t words = 2 * W;
    const uint32_t sb = blockIdx.x * (uint32_t)kPosSlice;
    const int n32 = (int)std::min<int64_t>(kPosSlice, words - sb);
    for (int j = threadIdx.x; j < kPosSlice; j += 1024) lds[j] = 0;
    __syncthreads();
    int64_t ob = off[set] - base;
    const int64_t oe = off[set + 1] - base;
    // head up to a 16-byte boundary, then 4 x uint4 per thread per pass, then the tail
    const int64_t ha = std::min<int64_t>(oe, (ob + 3) & ~int64_t(3));
    if (ob + threadIdx.x < ha) pos_or(lds, pos[ob + threadIdx.x], sb);
    ob = ha;
    const int64_t nv = (oe - ob) >> 2;   // whole uint4 in [ob, oe)
    const uint4* v = reinterpret_cast<const uint4*>(pos + ob);
    int64_t j = threadIdx.x;
    for (; j + 3 * 1024 < nv; j += 4 * 1024) {
        uint4 a[4];
#pragma unroll
        for (int u = 0; u < 4; u++) a[u] = v[j + u * 1024];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            pos_or(lds, a[u].x, sb); pos_or(lds, a[u].y, sb); pos_or(lds, a[u].z, sb); pos_or(lds, a[u].w, sb);
        }
    }
    for (; j < nv; j += 1024) {
        const uint4 a = v[j];
        pos_or(lds, a.x, sb); pos_or(lds, a.y, sb); pos_or(lds, a.z, sb); pos_or(lds, a.w, sb);
    }
    const int64_t t = ob + nv * 4 + threadIdx.x;
    if (t < oe) pos_or(lds, pos[t], sb);
    __syncthreads();
    uint32_t* row = bits + set * words + sb;
    for (int x = threadIdx.x; x < n32; x += 1024) row[x] = lds[x];
}

// bits of sets [0, nsets) against the dense dictionary (default: merged
// positions + LDS slices; option fill_sort 1: the chunked pairs sort + run
// ranks + scatter; 2: the one-pass windowed searches with global atomics);
// rare-tier records appended to rare_out (capacity cap)
void bits_from_positions(gdist_ctx* ctx, const gdist_sets* s, const uint32_t* pos, int64_t s0, int64_t s1,
                         int64_t base, int64_t W, unsigned long long* bits) {
    const unsigned nslice = (unsigned)ceil_div(2 * W, kPosSlice);
    if (W == 0) return;
    for (int64_t c0 = s0; c0 < s1; c0 += 65535) {
        const unsigned ny = (unsigned)std::min<int64_t>(65535, s1 - c0);
        pos_bits_kernel<<<dim3(nslice, ny), 1024, 0, ctx->stream>>>(pos, s->off.as<int64_t>(), c0, base, W,
                                                                     reinterpret_cast<uint32_t*>(bits));
        GD_HIP(hipGetLastError());
    }
}

void fill_bits(gdist_ctx* ctx, const gdist_sets* s, const uint64_t* dict, int64_t U, int64_t W,
               unsigned long long* bits, const uint64_t* rare, int64_t Ur, int64_t id_base,
               unsigned long long* rare_out, int64_t rare_cap, int64_t* rare_written, const uint32_t* perm,
               const FillHook& hook, int64_t sa, int64_t sb) {
    hipStream_t st = ctx->stream;
    if (sb < 0) sb = s->nsets;
    GD_REQUIRE(0 <= sa && sa <= sb && sb <= s->nsets, "fill set range outside the collection");
    // Sets sparse against the dictionary (C3: 33 K codes a set against tens of
    // millions) give the windowed fill's segments windows past its LDS caps
    // even at 64 codes (dictionary entries per code of a set >= 12 dense or
    // >= 32 rare): every segment would walk global memory. The hash fill
    // probes a table of the dictionary instead. Option fill_sort: 0 or 3 the
    // windows, 1 the sort, 2 the atomics, 4 the hash, 5 the windows one wave a
    // segment (round 3's pass 1).
    const int64_t total = s->h_off[s->nsets];
    const double per_set = (double)total / (double)std::max<int64_t>(1, s->nsets);
    const bool sparse_sets = (double)U > 12.0 * per_set || (double)Ur > 32.0 * per_set;
    const int64_t opt = ctx->option(OPT_FILL_SORT, -1);
    if (U + Ur > 0 && (opt == 4 || (opt < 0 && sparse_sets))) {
        hash_fill(ctx, s, dict, U, perm, rare, Ur, W, bits, id_base, rare_out, rare_cap, rare_written, hook, sa, sb);
        return;
    }
    const int cbits = std::min(64, code_bits(s->kind, s->k, s->flags));
    Trace tr(st, ctx->trace());
    GD_HIP(hipMemsetAsync(bits + (size_t)sa * W, 0, (size_t)(sb - sa) * W * 8, st));
    DevBuf rcnt(8, st);
    GD_HIP(hipMemsetAsync(rcnt.p, 0, 8, st));
    // the hook needs the position arrays; option 5: pass 1 by fill_pos_kernel (one wave a segment)
    const int64_t mode = hook || opt == 3 || opt == 5 || opt < 0 ? 0 : opt;
    const bool wave_fill = opt == 5;
    if (U + Ur > 0 && mode == 0) {
        GD_REQUIRE(s->nsets < (int64_t(1) << 23) && s->h_off[s->nsets] < (int64_t(1) << 40),
                   "collection too large for packed fill segments");
        GD_REQUIRE(U <= (int64_t(1) << 31), "dense tier too large for u32 positions");   // keeps ~0 out of every row
        // segment length per set: its windows should fit the LDS caps (window ~ length x dictionary / set size)
        std::vector<int64_t> seg, first(s->nsets + 1, 0);
        for (int64_t i = sa; i < sb; i++) {
            first[i] = (int64_t)seg.size();
            const double ni = (double)(s->h_off[i + 1] - s->h_off[i]);
            const double wd = wave_fill ? kWinDense : kMWin, wf = wave_fill ? kRareFences : kMFences;
            const double fit = 0.8 * std::min(wd * ni / (double)std::max<int64_t>(1, U),
                                              wf * kRareBucket * ni / (double)std::max<int64_t>(1, Ur));
            const int64_t L = std::max<int64_t>(64, std::min<int64_t>(wave_fill ? kPosSeg : kMSeg, (int64_t)(fit / 64) * 64));
            for (int64_t b = s->h_off[i]; b < s->h_off[i + 1]; b += L) seg.push_back((i << 40) | b);
        }
        first[sb] = (int64_t)seg.size();
        DevBuf dseg(std::max<int64_t>(1, (int64_t)seg.size()) * 8, st);
        if (!seg.empty()) h2d(dseg.p, seg.data(), seg.size() * 8, st);
        const unsigned nslice = (unsigned)ceil_div(2 * W, kPosSlice);
        int64_t s0 = sa;
        while (s0 < sb) {
            int64_t s1 = s0 + 1;
            while (s1 < sb && s->h_off[s1 + 1] - s->h_off[s0] <= kFillPosChunk) s1++;
            const int64_t base = s->h_off[s0], n = s->h_off[s1] - base, ns = first[s1] - first[s0];
            // sized like the summary's per-chunk key buffers (8 B a code) so that the caching
            // allocator hands back one of those blocks: a fresh 4 GiB block costs ~25 ms
            DevBuf pos(std::max<int64_t>(1, n) * 8 + 8, st);
            if (ns) {
                const int64_t* sg = dseg.as<int64_t>() + first[s0];
                DevBuf win(ns * 8 * 8, st);
                fill_window_kernel<<<(unsigned)ceil_div(ns * 4, 256), 256, 0, st>>>(
                    s->codes.as<uint64_t>(), s->off.as<int64_t>(), sg, ns, dict, U, rare, Ur, win.as<int64_t>());
                GD_HIP(hipGetLastError());
                GD_REQUIRE(ns < (int64_t(1) << 31), "too many fill segments in one chunk");
                // blocks take the segments in turn (a block's rare records staged across them)
                if (wave_fill) {
                    const int64_t nblk = std::min<int64_t>(ns, (int64_t)ctx->cus * 32);
                    fill_pos_kernel<<<(unsigned)nblk, 64, 0, st>>>(s->codes.as<uint64_t>(), win.as<int64_t>(), ns,
                                                                 dict, rare, base, pos.as<uint32_t>(), id_base,
                                                                 rare_out, rcnt.as<unsigned long long>(), rare_cap,
                                                                 perm);
                } else {
                    // persistent: exactly the resident workgroups (a block that only
                    // starts when a resident one exits would run its share at the end)
                    static int per_cu = 0;
                    if (!per_cu) {
                        GD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fill_merge_kernel, kMNT, 0));
                        per_cu = std::max(1, per_cu);
                    }
                    const int64_t nblk = std::min<int64_t>(ns, (int64_t)ctx->cus * per_cu);
                    fill_merge_kernel<<<(unsigned)nblk, kMNT, 0, st>>>(s->codes.as<uint64_t>(), win.as<int64_t>(),
                                                                       ns, dict, rare, base, pos.as<uint32_t>(),
                                                                       id_base, rare_out,
                                                                       rcnt.as<unsigned long long>(), rare_cap, perm);
                }
                GD_HIP(hipGetLastError());
            }
            tr.mark("fill: merged positions");
            if (hook) hook(pos.as<uint32_t>(), s0, s1, base);
            for (int64_t c0 = s0; c0 < s1; c0 += 65535) {
                const unsigned ny = (unsigned)std::min<int64_t>(65535, s1 - c0);
                pos_bits_kernel<<<dim3(nslice, ny), 1024, 0, st>>>(pos.as<uint32_t>(), s->off.as<int64_t>(), c0, base,
                                                                    W, reinterpret_cast<uint32_t*>(bits));
                GD_HIP(hipGetLastError());
            }
            GD_HIP(hipStreamSynchronize(st));
            tr.mark("fill: LDS row slices");
            s0 = s1;
        }
    } else if (U + Ur > 0 && mode == 2) {
        // segments of <= kFillSeg codes inside one set, built on the host from the offsets
        GD_REQUIRE(s->nsets < (int64_t(1) << 23) && s->h_off[s->nsets] < (int64_t(1) << 40),
                   "collection too large for packed fill segments");
        std::vector<int64_t> seg;
        for (int64_t i = sa; i < sb; i++)
            for (int64_t b = s->h_off[i]; b < s->h_off[i + 1]; b += kFillSeg) seg.push_back((i << 40) | b);
        const int64_t nseg = (int64_t)seg.size();
        if (nseg) {
            DevBuf dseg(nseg * 8, st);
            h2d(dseg.p, seg.data(), nseg * 8, st);
            const int64_t threads = nseg * 64;
            fill_search_kernel<<<(unsigned)ceil_div(threads, 256), 256, 0, st>>>(
                s->codes.as<uint64_t>(), s->off.as<int64_t>(), dseg.as<int64_t>(), nseg, dict, U, rare, Ur, W, bits,
                id_base, rare_out, rcnt.as<unsigned long long>(), rare_cap, perm);
            GD_HIP(hipGetLastError());
            GD_HIP(hipStreamSynchronize(st));
        }
        tr.mark("fill: windowed searches + scatter");
    } else if (U + Ur > 0) {
        int64_t s0 = sa;
        while (s0 < sb) {
            int64_t s1 = s0 + 1;
            while (s1 < sb && s->h_off[s1 + 1] - s->h_off[s0] <= kBitsChunk) s1++;
            const int64_t b = s->h_off[s0], n = s->h_off[s1] - b;
            if (n) {
                DevBuf kA(n * 8, st), kB(n * 8, st), vA(n * 4, st), vB(n * 4, st);
                GD_HIP(hipMemcpyAsync(kA.p, s->codes.as<uint64_t>() + b, n * 8, hipMemcpyDeviceToDevice, st));
                set_ids_kernel<<<grid_for(n), 256, 0, st>>>(s->off.as<int64_t>(), s0, s1, vA.as<int32_t>());
                GD_HIP(hipGetLastError());
                uint64_t* keys = kA.as<uint64_t>(); uint64_t* kalt = kB.as<uint64_t>();
                int32_t* ids = vA.as<int32_t>(); int32_t* ialt = vB.as<int32_t>();
                sort_pairs_u64_i32(ctx, keys, kalt, ids, ialt, (size_t)n, 0, cbits);
                DevBuf flag, pos, uniq, start;
                int64_t nruns = 0;
                runs_of(ctx, keys, n, flag, pos, uniq, start, nruns);
                DevBuf rank(nruns * 8 + 8, st);
                run_rank_kernel<<<(int)ceil_div(nruns, 256), 256, 0, st>>>(keys, start.as<int64_t>(), nruns, dict, U,
                                                                           rare, Ur, rank.as<int64_t>());
                GD_HIP(hipGetLastError());
                tr.mark("fill: copy+sort+runs+rank");
                scatter_bits_kernel<<<grid_for(n), 256, 0, st>>>(ids, flag.as<int32_t>(), pos.as<int64_t>(),
                                                                 rank.as<int64_t>(), n, W, bits, id_base, rare_out,
                                                                 rcnt.as<unsigned long long>(), rare_cap, perm);
                GD_HIP(hipGetLastError());
                GD_HIP(hipStreamSynchronize(st));
                tr.mark("fill: scatter");
            }
            s0 = s1;
        }
    }
    int64_t w = 0;
    d2h(&w, rcnt.p, 8, st);
    GD_REQUIRE(w <= rare_cap, "rare-tier record count exceeds its reservation");
    *rare_written = w;
}

// ---- identical posting lists ------------------------------------------
// Every kmer covering one variant that several sets share has the same
// holders, so the rare tier is full of identical posting lists (C2: 42 per
// shared substitution, 21 windows x 2 strands). Such lists are merged into
// one list whose weight is their number: the kernels add the weight instead
// of 1, and do the work of one list. Lists are grouped by a 64-bit content
// hash and merged only after a member-by-member comparison with the group's
// first list, so a hash collision costs compression, never exactness.
namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void list_hash_kernel(const int64_t* __restrict__ poff, const uint32_t* __restrict__ psets, int64_t nl,
                                 uint64_t* __restrict__ h, int32_t* __restrict__ ids) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; l < nl; l += stride) {
        const int64_t b = poff[l], e = poff[l + 1];
        uint64_t x = mix64(0x9E3779B97F4A7C15ull * (uint64_t)(e - b + 1));
        for (int64_t y = b; y < e; y++) x = mix64(x ^ (0x632BE59BD9B4E019ull + psets[y]));
        h[l] = x;
        ids[l] = (int32_t)l;
    }
}

// sorted (hash, list) -> keep[list] = 0 if its contents equal the run's first
// list (merged into it), else 1; weight[the list it counts for] += 1
__global__ void list_merge_kernel(const int32_t* __restrict__ ids, const int32_t* __restrict__ flag,
                                  const int64_t* __restrict__ pos, const int64_t* __restrict__ start, int64_t n,
                                  const int64_t* __restrict__ poff, const uint32_t* __restrict__ psets,
                                  int32_t* __restrict__ keep, uint32_t* __restrict__ weight) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t hd = start[pos[i] + flag[i] - 1];
        const int32_t l = ids[i], h = ids[hd];
        bool same = false;
        if (i != hd) {
            const int64_t lb = poff[l], le = poff[l + 1], hb = poff[h], he = poff[h + 1];
            same = le - lb == he - hb;
            for (int64_t y = 0; same && y < le - lb; y++) same = psets[lb + y] == psets[hb + y];
        }
        keep[l] = same ? 0 : 1;
        atomicAdd(weight + (same ? h : l), 1u);
    }
}

__global__ void record_keep_kernel(const uint64_t* __restrict__ recs, int64_t n, const int32_t* __restrict__ keep,
                                   int32_t* __restrict__ rk) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t y = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; y < n; y += stride) rk[y] = keep[recs[y] >> 32];
}

// kept lists' records, renumbered: member sets in list order, and the same
// records keyed by set (set << 32 | new list) for the set -> rare CSR
__global__ void list_compact_kernel(const uint64_t* __restrict__ recs, int64_t n, const int32_t* __restrict__ keep,
                                    const int64_t* __restrict__ newid, const int64_t* __restrict__ rpos,
                                    uint32_t* __restrict__ out_sets, uint64_t* __restrict__ out_recs) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t y = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; y < n; y += stride) {
        const int64_t l = (int64_t)(recs[y] >> 32);
        if (!keep[l]) continue;
        const uint32_t set = (uint32_t)recs[y];
        out_sets[rpos[y]] = set;
        out_recs[rpos[y]] = ((uint64_t)set << 32) | (uint64_t)newid[l];
    }
}

__global__ void list_offsets_kernel(const int64_t* __restrict__ poff, int64_t nl, const int32_t* __restrict__ keep,
                                    const int64_t* __restrict__ newid, const int64_t* __restrict__ rpos,
                                    const uint32_t* __restrict__ weight, int64_t* __restrict__ out_off,
                                    uint32_t* __restrict__ out_w) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; l < nl; l += stride)
        if (keep[l]) { out_off[newid[l]] = rpos[poff[l]]; out_w[newid[l]] = weight[l]; }
}

__global__ void narrow_u16_kernel(const uint32_t* __restrict__ in, int64_t n, uint16_t* __restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = (uint16_t)in[i];
}

__global__ void fill_u32_kernel(uint32_t* __restrict__ p, int64_t n, uint32_t v) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = v;
}

// set-side weights: the weight of each entry's list
__global__ void entry_weights_kernel(const uint64_t* __restrict__ keys, int64_t n, const uint32_t* __restrict__ pw,
                                     uint32_t* __restrict__ sw) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) sw[i] = pw[(uint32_t)keys[i]];
}

// the heaviest row of the set side: max over sets of the sum of their
// entries' list weights (a pair's rare count is at most its row's)
__global__ void row_weight_max_kernel(const int64_t* __restrict__ soff, const uint32_t* __restrict__ sw,
                                      int64_t nsets, unsigned long long* __restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    unsigned long long mx = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nsets; i += stride) {
        unsigned long long t = 0;
        for (int64_t x = soff[i]; x < soff[i + 1]; x++) t += sw[x];
        mx = t > mx ? t : mx;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long v = __shfl_xor(mx, o, 64);
        mx = v > mx ? v : mx;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(out, mx);
}

}  // namespace

// rare records (rank << 32 | set) -> posting lists CSR on `s`, identical
// lists merged (GDIST_RARE_DEDUP=0 keeps one list per kmer, A/B)
void build_postings(gdist_ctx* ctx, gdist_sets* s, unsigned long long* recs, int64_t n, int64_t Ur) {
    hipStream_t st = ctx->stream;
    Trace tr(st, ctx->trace());
    s->n_rare = Ur;
    s->rare_kmers = Ur;
    s->rare_records = n;
    s->post_off.alloc((Ur + 1) * 8, st);
    s->post_sets.alloc(n * 4 + 16, st);          // padded: the row walk reads 16 bytes at a time
    s->rare_incs = s->rare_max_list = s->rare_incs_long = 0;
    s->rare_row_wmax = 0;
    if (Ur == 0 || n == 0) {
        GD_HIP(hipMemsetAsync(s->post_off.p, 0, (Ur + 1) * 8, st));
        s->post_w.alloc(Ur * 4 + 4, st);
        s->srare_off.alloc((s->nsets + 1) * 8, st);
        GD_HIP(hipMemsetAsync(s->srare_off.p, 0, (s->nsets + 1) * 8, st));
        s->srare_ent.alloc(8, st);
        s->srare_w.alloc(4, st);
        s->srare_skip.alloc(8, st);
        s->n_rare = 0;
        s->rare_records = 0;
        GD_HIP(hipStreamSynchronize(st));
        return;
    }
    GD_REQUIRE(Ur < (int64_t(1) << 31), "rare tier: too many lists");
    DevBuf alt(n * 8, st);
    uint64_t* keys = reinterpret_cast<uint64_t*>(recs);
    uint64_t* kalt = alt.as<uint64_t>();
    int rbits = 1;
    while ((int64_t(1) << rbits) < Ur) rbits++;
    sort_keys_u64(ctx, keys, kalt, (size_t)n, 0, std::min(64, 32 + rbits));
    posting_offsets_kernel<<<(int)ceil_div(Ur + 1, 256), 256, 0, st>>>(keys, n, Ur, s->post_off.as<int64_t>());
    posting_sets_kernel<<<grid_for(n), 256, 0, st>>>(keys, n, s->post_sets.as<uint32_t>());
    GD_HIP(hipGetLastError());
    tr.mark("postings: lists");
    int64_t nl = Ur, nrec = n;
    if (ctx->option(OPT_RARE_DEDUP, 1) != 0) {
        DevBuf hA(Ur * 8, st), hB(Ur * 8, st), iA(Ur * 4, st), iB(Ur * 4, st);
        list_hash_kernel<<<grid_for(Ur), 256, 0, st>>>(s->post_off.as<int64_t>(), s->post_sets.as<uint32_t>(), Ur,
                                                       hA.as<uint64_t>(), iA.as<int32_t>());
        GD_HIP(hipGetLastError());
        uint64_t* hk = hA.as<uint64_t>(); uint64_t* hkalt = hB.as<uint64_t>();
        int32_t* iv = iA.as<int32_t>(); int32_t* ivalt = iB.as<int32_t>();
        sort_pairs_u64_i32(ctx, hk, hkalt, iv, ivalt, (size_t)Ur, 0, 64);
        DevBuf flag, pos, uniq, start;
        int64_t nruns = 0;
        runs_of(ctx, hk, Ur, flag, pos, uniq, start, nruns);
        DevBuf keep(Ur * 4 + 4, st), weight(Ur * 4 + 4, st), newid(Ur * 8 + 8, st);
        GD_HIP(hipMemsetAsync(weight.p, 0, Ur * 4, st));
        list_merge_kernel<<<grid_for(Ur), 256, 0, st>>>(iv, flag.as<int32_t>(), pos.as<int64_t>(), start.as<int64_t>(),
                                                        Ur, s->post_off.as<int64_t>(), s->post_sets.as<uint32_t>(),
                                                        keep.as<int32_t>(), weight.as<uint32_t>());
        GD_HIP(hipGetLastError());
        exclusive_scan_i32_to_i64(ctx, keep.as<int32_t>(), newid.as<int64_t>(), (size_t)Ur);
        DevBuf rk(n * 4 + 4, st), rpos(n * 8 + 8, st);
        record_keep_kernel<<<grid_for(n), 256, 0, st>>>(keys, n, keep.as<int32_t>(), rk.as<int32_t>());
        GD_HIP(hipGetLastError());
        exclusive_scan_i32_to_i64(ctx, rk.as<int32_t>(), rpos.as<int64_t>(), (size_t)n);
        int64_t h[2];
        int32_t hf[2];
        d2h(&h[0], newid.as<int64_t>() + Ur - 1, 8, st);
        d2h(&h[1], rpos.as<int64_t>() + n - 1, 8, st);
        d2h(&hf[0], keep.as<int32_t>() + Ur - 1, 4, st);
        d2h(&hf[1], rk.as<int32_t>() + n - 1, 4, st);
        nl = h[0] + hf[0];
        nrec = h[1] + hf[1];
        DevBuf noff((nl + 1) * 8, st), nsets(nrec * 4 + 16, st);
        s->post_w.alloc(nl * 4 + 4, st);
        list_offsets_kernel<<<grid_for(Ur), 256, 0, st>>>(s->post_off.as<int64_t>(), Ur, keep.as<int32_t>(),
                                                          newid.as<int64_t>(), rpos.as<int64_t>(),
                                                          weight.as<uint32_t>(), noff.as<int64_t>(),
                                                          s->post_w.as<uint32_t>());
        list_compact_kernel<<<grid_for(n), 256, 0, st>>>(keys, n, keep.as<int32_t>(), newid.as<int64_t>(),
                                                         rpos.as<int64_t>(), nsets.as<uint32_t>(), kalt);
        GD_HIP(hipGetLastError());
        h2d(noff.as<int64_t>() + nl, &nrec, 8, st);
        s->post_off = std::move(noff);
        s->post_sets = std::move(nsets);
        tr.mark("postings: merge identical lists");
    } else {
        s->post_w.alloc(Ur * 4 + 4, st);
        fill_u32_kernel<<<grid_for(Ur), 256, 0, st>>>(s->post_w.as<uint32_t>(), Ur, 1u);
        // the same records keyed by set: set -> rare CSR for the row-major kernels
        swap_halves_kernel<<<grid_for(n), 256, 0, st>>>(keys, n, kalt);
        GD_HIP(hipGetLastError());
    }
    s->n_rare = nl;
    s->rare_records = nrec;
    // kalt: (set << 32 | list) records, sorted by set (into `keys`, then swapped back)
    int sbits = 1;
    while ((int64_t(1) << sbits) < s->nsets) sbits++;
    sort_keys_u64(ctx, kalt, keys, (size_t)nrec, 0, std::min(64, 32 + sbits));
    // packed entries: 40-bit list start, 24-bit length (a rare list has < T <= N + 1 sets)
    GD_REQUIRE(nrec < (int64_t(1) << 40) && s->nsets < (int64_t(1) << 24), "rare tier too large for packed list entries");
    s->srare_off.alloc((s->nsets + 1) * 8, st);
    s->srare_ent.alloc(nrec * 8 + 8, st);
    s->srare_w.alloc(nrec * 4 + 4, st);
    posting_offsets_kernel<<<(int)ceil_div(s->nsets + 1, 256), 256, 0, st>>>(kalt, nrec, s->nsets,
                                                                             s->srare_off.as<int64_t>());
    rare_entries_kernel<<<grid_for(nrec), 256, 0, st>>>(kalt, nrec, s->post_off.as<int64_t>(),
                                                        s->srare_ent.as<uint64_t>());
    entry_weights_kernel<<<grid_for(nrec), 256, 0, st>>>(kalt, nrec, s->post_w.as<uint32_t>(),
                                                         s->srare_w.as<uint32_t>());
    s->srare_skip.alloc(nrec * 2 + 8, st);
    rare_skip_kernel<<<grid_for(nrec), 256, 0, st>>>(kalt, nrec, s->post_off.as<int64_t>(), s->post_sets.as<uint32_t>(),
                                                     s->srare_skip.as<uint16_t>());
    GD_HIP(hipGetLastError());
    // 2-byte members for the row-major walk (collections of <= 65,536 sets;
    // option rare_u16 = 0 keeps the 4-byte ones)
    s->post_sets16.release();
    if (s->nsets <= 65536 && ctx->option(OPT_RARE_U16, 1) != 0) {
        s->post_sets16.alloc(nrec * 2 + 16, st);
        GD_HIP(hipMemsetAsync(s->post_sets16.as<uint16_t>() + nrec, 0, 16, st));
        narrow_u16_kernel<<<grid_for(nrec), 256, 0, st>>>(s->post_sets.as<uint32_t>(), nrec,
                                                          s->post_sets16.as<uint16_t>());
        GD_HIP(hipGetLastError());
    }
    // pair increments of the tier (cost model, kernel choice)
    DevBuf d_incs(24, st);
    GD_HIP(hipMemsetAsync(d_incs.p, 0, 24, st));
    rare_incs_kernel<<<grid_for(nl, 256, 4096), 256, 0, st>>>(s->post_off.as<int64_t>(), nl,
                                                              d_incs.as<unsigned long long>());
    GD_HIP(hipGetLastError());
    unsigned long long hi[3] = {0, 0, 0};
    d2h(hi, d_incs.p, 24, st);
    GD_HIP(hipStreamSynchronize(st));
    s->rare_incs = (int64_t)hi[0];
    s->rare_max_list = (int64_t)hi[1];
    s->rare_incs_long = (int64_t)hi[2];
    {
        DevBuf wm(8, st);
        GD_HIP(hipMemsetAsync(wm.p, 0, 8, st));
        row_weight_max_kernel<<<grid_for(s->nsets, 256, 4096), 256, 0, st>>>(
            s->srare_off.as<int64_t>(), s->srare_w.as<uint32_t>(), s->nsets, wm.as<unsigned long long>());
        GD_HIP(hipGetLastError());
        unsigned long long h = 0;
        d2h(&h, wm.p, 8, st);
        s->rare_row_wmax = (int64_t)h;
    }
    tr.mark("postings: set side");
}

void build_bitsets(gdist_ctx* ctx, gdist_sets* s, unsigned flags, int64_t rare_threshold) {
    const bool keep = (flags & GDIST_BITSET_KEEP_SINGLETONS) != 0;
    int64_t T = keep ? 0 : rare_threshold;     // < 0: cost-optimal from the count histogram
    // a rebuild replaces every tier: the old variant lists, sparse words,
    // plans and FP4 operand must not survive into the new representation
    // (a two-tier rebuild of a variant collection would add its stale
    // variant counts on top of the new bits); synchronises both streams
    free_bitsets(s);
    Trace tr(ctx->stream, ctx->trace());
    const auto t_build = std::chrono::steady_clock::now();
    BuildSplit sp = build_split(ctx, s);
    // the build's wall time and its split stages (gdist_sets_build_timing)
    struct BuildClock {
        gdist_sets* s; BuildSplit& sp; hipStream_t st; std::chrono::steady_clock::time_point t0;
        AllocStats a0;
        bool trace;
        ~BuildClock() {
            (void)hipStreamSynchronize(st);
            if (trace) {
                const AllocStats& a = alloc_stats();
                fprintf(stderr, "gdist: build allocations: %lld fresh blocks, %.2f GB, %.1f ms in hipMalloc; %lld cache trims\n",
                        (long long)(a.fresh - a0.fresh), (a.fresh_bytes - a0.fresh_bytes) / 1e9, a.fresh_ms - a0.fresh_ms,
                        (long long)(a.trims - a0.trims));
            }
            s->build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            s->build_shares = sp.R;
            s->build_split_ms = s->build_share_max_ms = 0;
            for (double v : sp.share_ms) {
                s->build_split_ms += v;
                s->build_share_max_ms = std::max(s->build_share_max_ms, v);
            }
        }
    } clock{s, sp, ctx->stream, t_build, alloc_stats(), ctx->trace()};
    Summary sum;
    // a collection without pack summaries and too many codes for one sort
    // (a gathered 8-GPU collection: C4's 2e10 codes) is counted by code
    // ranges, singletons dropped as they are counted (option range_summary);
    // a split build counts by ranges (its shares are code ranges)
    const int64_t rs_opt = ctx->option(OPT_RANGE_SUMMARY, -1);
    const bool by_range = rs_opt > 0 || (rs_opt < 0 && ((s->pack_sum.empty() && s->total > kRangeSummaryMin) || sp.R > 1));
    if (by_range) range_summary(ctx, s, keep ? 1 : 2, sum, sp);
    else local_summary(ctx, s, sum);
    tr.mark("bitsets: summary");
    DevBuf dict, rare, dcnt;
    int64_t U = 0, Ur = 0, mass = 0;
    const int64_t T_in = T;
    dictionary_from(ctx, {SummaryView{sum.codes.as<uint64_t>(), sum.counts.as<uint32_t>(), sum.n}}, keep, T, s->nsets,
                    dict, U, rare, Ur, mass, &dcnt);
    tr.mark("bitsets: dictionary");
    // the variant tier when kmers held by T .. Dmin - 1 sets dominate the
    // dictionary (variant.hip); its rare threshold is at most kVariantMaxT
    // unless given: kmers shared by a few sets stay posting lists, the rest
    // of the non-dense kmers form the variant words
    if (!keep) {
        // the variant tier's rare threshold: the model's T (which prices the
        // kmers below Dmin as dense words or posting lists only) capped at
        // kVariantMaxT unless given; its share of the summary decides
        const int64_t dmin = variant_dmin(ctx, s->nsets);
        const int64_t Tv = (T_in >= 0 || ctx->has_option(OPT_RARE_T)) ? T : std::min<int64_t>(T, kVariantMaxT);
        const int64_t mid = count_in_range(ctx, sum.counts.as<uint32_t>(), sum.n, Tv, dmin);
        const int64_t ge = count_in_range(ctx, sum.counts.as<uint32_t>(), sum.n, Tv, INT64_MAX);
        if (variant_wanted(ctx, s->nsets, mid, ge)) {
            if (Tv != T) {
                T = Tv;
                dictionary_from(ctx, {SummaryView{sum.codes.as<uint64_t>(), sum.counts.as<uint32_t>(), sum.n}}, false,
                                T, s->nsets, dict, U, rare, Ur, mass, &dcnt);
            }
            sum.codes.release();
            sum.counts.release();
            // 47-kmer words (option variant_bits, default): a substitution's k
            // windows on each strand fit one word when k x strands <= 47, and
            // with < 2^17 sets a list member packs into 8 bytes (C4: 42 kmers
            // a substitution, 100,000 sets); else 64-kmer words of 12-byte members
            const int strands = (s->kind == GDIST_DNA && (s->flags & GDIST_STRAND_MASK) == GDIST_STRAND_BOTH) ? 2 : 1;
            const int64_t vb = ctx->option(OPT_VARIANT_BITS, (s->nsets < (int64_t(1) << 17) &&
                                                              (int64_t)s->k * strands <= 47) ? 47 : 64);
            build_variant_bitsets(ctx, s, dict, dcnt, U, rare, Ur, mass, T, sp, -1, vb == 47 ? 47 : 64);
            return;
        }
        // The grouped rare tier (round 5, option rare_group): the kmers of 2 ..
        // T - 1 sets as variant words of 16 kmers, one substitution a word
        // (its k windows held by nearly the same sets), walked a thread an
        // entry from packed (set | mask << 16) lists. C3: 71.9 M posting
        // records (Σ m(m−1)/2 ≈ 0.5 G increments of 2-byte members, each record
        // a random line) become 22.7 M entries and 0.28 G products. By default
        // for 4,096 .. 65,536 sets with locus guides and many rare records; the
        // dense tier keeps its threshold T (option variant = 0 keeps the two
        // tiers unless rare_group = 1).
        const int64_t rg = ctx->option(OPT_RARE_GROUP, -1);
        const bool group = s->nsets <= 65536 && T > 2 && mass > 0 &&
                           (rg > 0 || (rg < 0 && ctx->option(OPT_VARIANT, -1) != 0 && s->nsets >= kVariantMinSets &&
                                       s->n_guide > 0 && locus_order_enabled(ctx) && mass >= 64 * s->nsets));
        if (group) {
            const int64_t dmin = T;
            T = 2;
            dictionary_from(ctx, {SummaryView{sum.codes.as<uint64_t>(), sum.counts.as<uint32_t>(), sum.n}}, false, T,
                            s->nsets, dict, U, rare, Ur, mass, &dcnt);
            // (probing by default and with rare_group = 2; 1 forces the tier)
            if (build_variant_bitsets(ctx, s, dict, dcnt, U, rare, Ur, mass, T, sp, dmin, 16, rg <= 0 || rg == 2)) {
                sum.codes.release();
                sum.counts.release();
                return;
            }
            // keyless kmers dominate (no substitution structure): the two tiers
            T = dmin;
            dictionary_from(ctx, {SummaryView{sum.codes.as<uint64_t>(), sum.counts.as<uint32_t>(), sum.n}}, false, T,
                            s->nsets, dict, U, rare, Ur, mass, &dcnt);
        }
    }
    const int64_t W = bitset_words(U);
    DevBuf perm;
    if (s->n_guide > 0 && locus_order_enabled(ctx)) {
        DevBuf key;
        locus_keys(ctx, s, dict.as<uint64_t>(), dcnt.as<uint32_t>(), U, 0, key);
        locus_perm(ctx, key, U, perm);
        tr.mark("bitsets: locus order");
    }
    s->fp4.release();                    // the MFMA operand expanded the old bits
    s->fp4_W = 0;
    // rows of R equal shares (split build): slot r of the in-place all-gather
    const int64_t mrows = BuildSplit::ceil_div_h(s->nsets, sp.R);
    s->bits.alloc((size_t)sp.R * mrows * W * 8 + 8, ctx->stream);
    DevBuf recs(mass * 8 + 8, ctx->stream);
    int64_t written = 0;
    tr.mark("bitsets: alloc");
    for (int r = sp.first(); r < sp.last(); r++) {
        ShareClock clk(sp, r, ctx->stream);
        int64_t w = 0;
        fill_bits(ctx, s, dict.as<uint64_t>(), U, W, s->bits.as<unsigned long long>(), rare.as<uint64_t>(), Ur, 0,
                  recs.as<unsigned long long>() + written, mass - written, &w, perm.as<uint32_t>(), FillHook(),
                  sp.set_lo(r, s->nsets), sp.set_hi(r, s->nsets));
        written += w;
    }
    if (sp.real) {
        comm_allgather_inplace(ctx, s->bits.p, (size_t)mrows * W * 8);
        written = allgather_concat(ctx, recs, written, 8);
    }
    tr.mark("bitsets: fill");
    GD_REQUIRE(written == mass, "rare-tier record count mismatch");
    build_postings(ctx, s, recs.as<unsigned long long>(), written, Ur);
    tr.mark("bitsets: postings");
    s->W = W;
    s->dict_size = U;
    s->rare_T = T;
    s->bits_keep_singletons = keep;
    build_sparse_words(ctx, s);
}

RareTier rare_tier(const gdist_sets* s) {
    RareTier t;
    t.incs = (double)s->rare_incs;
    t.incs_long = (double)s->rare_incs_long;
    t.records = (double)s->rare_records;
    t.lists = (double)s->n_rare;
    return t;
}

double block_pairs(int64_t r0, int64_t r1, int64_t c0, int64_t c1, bool upper) {
    if (r1 <= r0 || c1 <= c0) return 0.0;
    if (!upper) return (double)(r1 - r0) * (double)(c1 - c0);
    // row i holds columns max(c0, i + 1) .. c1 - 1: full rows while i + 1 <= c0,
    // then c1 - 1 - i for i in [c0, c1 - 1)
    const int64_t a = std::min(r1, std::max(r0, c0));            // rows [r0, a): all nc columns
    double p = (double)(a - r0) * (double)(c1 - c0);
    const int64_t b0 = a, b1 = std::min(r1, c1 - 1);              // rows [b0, b1): c1 - 1 - i columns
    if (b1 > b0) p += 0.5 * (double)(b1 - b0) * (double)((c1 - 1 - b0) + (c1 - b1));
    return p;
}

// The 128 x 128 tiles bitset_matrix launches on a block (same enumeration:
// upper-triangle blocks tile their columns from corg = r0 mod BT, diagonal
// tiles go to the DIAG launch), counted per row tile in closed form. A
// partial last row tile with RR = ceil(rows / 16) <= kPartialMaxRR runs RR of
// 8 accumulator rows and costs ~RR/8 of a tile (at least 2/8: the column
// fragments are read from LDS whatever RR is); partial columns cost full
// tiles. What the row partition must see.
static void dense_tiles(int64_t r0, int64_t r1, int64_t c0, int64_t c1, bool upper, double* off, double* diag) {
    *off = *diag = 0.0;
    if (r1 <= r0 || c1 <= c0) return;
    const int64_t tr = ceil_div(r1 - r0, BT);
    const int64_t rr = ceil_div(r1 - r0 - (tr - 1) * BT, 16);
    const double last_w = rr <= kPartialMaxRR ? (double)std::max<int64_t>(2, rr) / 8.0 : 1.0;
    auto w = [&](int64_t a) { return a == tr - 1 ? std::min(1.0, last_w) : 1.0; };
    if (!upper) {
        *off = ((double)(tr - 1) + w(tr - 1)) * (double)ceil_div(c1 - c0, BT);
        return;
    }
    const int64_t corg = c0 - (((c0 - r0) % BT) + BT) % BT;
    const int64_t dlt_t = (r0 - corg) / BT, tc2 = ceil_div(c1 - corg, BT);
    for (int64_t a = 0; a < tr; a++) {
        const int64_t x = std::max(c0, r0 + a * BT + 1);   // tile b is launched iff its last column cmax >= x
        if (c1 - 1 < x) break;                            // rows only grow: no later row tile has any
        const int64_t b_lo = std::max<int64_t>(0, ceil_div(x + 1 - corg, BT) - 1);
        if (b_lo >= tc2) continue;
        const bool has_diag = a + dlt_t >= b_lo && a + dlt_t < tc2;
        *diag += (has_diag ? 1.0 : 0.0) * w(a);
        *off += ((double)(tc2 - b_lo) - (has_diag ? 1.0 : 0.0)) * w(a);
    }
}

// the variant tier's row walk: its share of the products, and one list
// search per (entry of the block's rows, column chunk)
static double variant_cost_s(const gdist_sets* s, double f_area, double f_rows, double ncols) {
    if (!s->variant) return 0.0;
    return f_area * s->vw_products / kVariantProductsPerS +
           f_rows * (double)s->vw_entries * std::ceil(ncols / 16384.0) / kVariantVisitsPerS;
}

double bitset_block_cost_s(const gdist_sets* s, int64_t r0, int64_t r1, int64_t c0, int64_t c1, bool upper,
                           bool* rare_row_major) {
    const double n = (double)s->nsets, tot = 0.5 * n * (n - 1.0);
    const double pairs = block_pairs(r0, r1, c0, c1, upper);
    const RareChoice rc = rare_choice(rare_tier(s), tot > 0 ? std::min(1.0, pairs / tot) : 1.0,
                                      n > 0 ? (double)(r1 - r0) / n : 1.0);
    if (rare_row_major) *rare_row_major = rc.row_major;
    double off, diag;
    dense_tiles(r0, r1, c0, c1, upper, &off, &diag);
    const double tW = s->sparse ? (s->sp_fold_dense ? 0.0 : (double)s->Wd) : (double)s->W;
    // sparse tiles: exactly the tiles the block's sparse plan launches (a
    // thin, unaligned row block still visits every word in each of its row
    // blocks' tiles: round-2 G = 8 emulation, balance 0.76 with the area estimate)
    double sp_tiles = 0.0;
    if (s->sparse && r1 > r0 && c1 > c0)
        for (int64_t A = r0 / BT; A <= (r1 - 1) / BT; A++)
            for (int64_t B = c0 / BT; B <= (c1 - 1) / BT; B++) {
                const int64_t rmin = std::max(r0, A * BT);
                const int64_t cmax = std::min(c1, (B + 1) * BT) - 1;
                if (!(upper && cmax <= rmin)) sp_tiles += 1.0;
            }
    // the rare tier's pairs are recounted by the sparse tile launch's rare
    // rows (sparse.hip rare_slab_plan) when the tier is small and its lists
    // short; priced as the list-major kernel beside the tiles
    const bool rare_in_reduce = s->sparse && s->n_rare > 0 && s->rare_max_list <= kLongList &&
                                (double)s->rare_records + (double)s->rare_incs <= double(int64_t(1) << 26);
    return (off + kDiagTileShare * diag) * (double)(BT * BT) * tW / kDenseWordPairsPerS +
           (rare_in_reduce ? rc.list_s * kRareOverlapExposed : rc.cost()) +
           sparse_block_cost_s(s, tot > 0 ? std::min(1.0, pairs / tot) : 1.0, sp_tiles) +
           variant_cost_s(s, tot > 0 ? std::min(1.0, pairs / tot) : 1.0, n > 0 ? (double)(r1 - r0) / n : 1.0,
                          (double)(c1 - c0));
}

double bitset_cost_s(const gdist_sets* s, double pairs) {
    // a region given only by its pair count: its share of the rows taken as its share of the pairs
    const double tot = 0.5 * (double)s->nsets * (double)(s->nsets - 1);
    const double frac = tot > 0 ? std::min(1.0, pairs / tot) : 1.0;
    const double tW = s->sparse ? (s->sp_fold_dense ? 0.0 : (double)s->Wd) : (double)s->W;
    return pairs * tW / kDenseWordPairsPerS + rare_choice(rare_tier(s), frac, frac).cost() +
           sparse_block_cost_s(s, frac, pairs / (double)(BT * BT) + std::sqrt(2.0 * pairs) / BT) +
           variant_cost_s(s, frac, frac, (double)s->nsets);
}

double sorted_cost_s(const gdist_sets* s, double pairs) {
    // streaming hash join: 8(n_i + n_j) bytes per pair at ~6 TB/s (C3)
    const double mean_n = s->nsets ? (double)s->total / (double)s->nsets : 0.0;
    return pairs * 16.0 * mean_n / kSortedBytesPerS;
}

void free_bitsets(gdist_sets* s) {
    free_sparse(s);                      // (synchronises both streams, clears plans and graphs)
    free_variant(s);
    s->fp4.release();
    s->fp4_W = 0;
    s->bits.release();
    s->post_off.release();
    s->post_sets.release();
    s->post_sets16.release();
    s->post_w.release();
    s->srare_off.release();
    s->srare_ent.release();
    s->srare_w.release();
    s->srare_skip.release();
    s->W = s->dict_size = 0;
    s->n_rare = s->rare_T = s->rare_records = s->rare_incs = s->rare_max_list = s->rare_incs_long = 0;
    s->rare_row_wmax = 0;
    s->rare_kmers = 0;
}

// The region's launch plan (tile groups, K-split, the sparse plan's slot),
// built once per region and option set, then reused
static MatrixPlan& matrix_plan(gdist_ctx* ctx, const gdist_sets* s, int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                               bool upper) {
    hipStream_t st = ctx->stream;
    const int64_t nr = r1 - r0;
    const int tr = (int)ceil_div(nr, BT);
    // dense tile operands: every word, or only the dense words when the
    // complement-sparse words run in their own kernel (sparse.hip)
    const int64_t tW = s->sparse ? s->Wd : s->W;
    // Diagonal tiles of an upper-triangle region (row0 == col0) get their
    // own launch of the DIAG variant, which skips the accumulators that
    // only hold pairs with j <= i (option bitset_diag = 0 keeps one launch).
    const bool split_diag = upper && ctx->option(OPT_BITSET_DIAG, 1) != 0;
    // The last row tile of a block whose rows are not a multiple of BT
    // holds nlast rows: its tiles get launches instantiated for
    // RR = ceil(nlast / 16) accumulator rows, skipping the others' work.
    // (option bitset_partial_rr: the largest RR given its own launches, A/B)
    const int max_rr = (int)ctx->option(OPT_BITSET_PARTIAL_RR, kPartialMaxRR);

    // ---- the region's launch plan (built once, then reused)
    // the key holds every option the plan (and the sparse plan in it) reads,
    // so that changing one builds a new plan instead of reusing a stale one
    // the dense tiles on the matrix cores (FP4 MFMA) when there are enough
    // words to amortise a 256 x 256 tile's stages, however few the tiles
    // (C2-realistic: 10 tiles of 1,936 dense words, step 0.317 ms against
    // 0.442 with the AND+popcount tiles, profiles/r05/s12/ab_c2r.txt;
    // option bitset_mfma 0: the AND+popcount tiles)
    const bool use_mfma = tW >= kMfmaMinWords && ctx->option(OPT_BITSET_MFMA, 1) != 0;
    const std::vector<int64_t> key{r0, r1, c0, c1, upper ? 1 : 0, split_diag ? 1 : 0, max_rr, tW, use_mfma ? 1 : 0,
                                   ctx->option(OPT_BITSET_MFMA_GROUP, 0),
                                   ctx->option(OPT_SPARSE_RARE, 1), ctx->option(OPT_SPARSE_CHUNKS, -1),
                                   ctx->option(OPT_SPARSE_PART_BUDGET, -1), ctx->option(OPT_SPARSE_WG_PER_CU, -1),
                                   ctx->option(OPT_SPARSE_XCD, 0)};
    auto it = s->plans.find(key);
    if (it == s->plans.end()) {
        if (s->plans.size() >= 8) {   // row-block loops: keep the cache small
            // launches on either stream may still read the old plans' buffers
            GD_HIP(hipStreamSynchronize(ctx->side));
            GD_HIP(hipStreamSynchronize(ctx->stream));
            s->graphs.clear();        // (captured steps hold the plans' buffers)
            s->plans.clear();
        }
        auto plan = std::make_unique<MatrixPlan>();
        MatrixPlan& p = *plan;
        // Upper-triangle regions tile their columns from an origin corg <= c0
        // with corg = r0 (mod BT), so tiles lie exactly on the diagonal whatever
        // r0 is (row-sharded ranks get exact equal-area row blocks); columns
        // below c0 are loaded clamped and discarded. Diagonal tiles: col0 == row0.
        p.corg = split_diag ? c0 - (((c0 - r0) % BT) + BT) % BT : c0;
        const int64_t dlt_t = (r0 - p.corg) / BT;
        const int64_t nlast = nr - (int64_t)(tr - 1) * BT;
        p.rr = (int)ceil_div(nlast, 16);
        p.part = p.rr <= max_rr;
        std::vector<int2> grp[4];   // off-diagonal, diagonal, partial off-diagonal, partial diagonal
        const int tc2 = (int)ceil_div(c1 - p.corg, BT);
        for (int a = 0; a < tr; a++)
            for (int b = 0; b < tc2; b++) {
                const int64_t rmin = r0 + (int64_t)a * BT;
                const int64_t cmax = std::min<int64_t>(c1, p.corg + (int64_t)(b + 1) * BT) - 1;
                if (cmax < c0 || (upper && cmax <= rmin)) continue;
                const int g = ((split_diag && (int64_t)b - a == dlt_t) ? 1 : 0) + ((p.part && a == tr - 1) ? 2 : 0);
                grp[g].push_back(make_int2(a, b));
            }
        for (int g = 0; g < 4; g++) p.at[g + 1] = p.at[g] + grp[g].size();
        if (use_mfma) {
            // the MFMA tiles: 256 x 256 from (r0, c0), those holding a pair of the region
            // (option bitset_mfma_group G > 0: the tiles in blocks of G row
            // tiles x 2G column tiles, so the ~32 consecutive tiles an XCD runs
            // at once share G row panels and 2G column panels in its L2)
            std::vector<int2> mt;
            const int tm = (int)ceil_div(nr, MT), tn = (int)ceil_div(c1 - c0, MT);
            const int gr = (int)std::max<int64_t>(1, ctx->option(OPT_BITSET_MFMA_GROUP, 0));
            const int gc = ctx->option(OPT_BITSET_MFMA_GROUP, 0) > 0 ? 2 * gr : tn;
            for (int a0 = 0; a0 < tm; a0 += gr)
                for (int b0 = 0; b0 < tn; b0 += gc)
                    for (int a = a0; a < std::min(tm, a0 + gr); a++)
                        for (int b = b0; b < std::min(tn, b0 + gc); b++) {
                            const int64_t rmin = r0 + (int64_t)a * MT;
                            const int64_t cmax = std::min<int64_t>(c1, c0 + (int64_t)(b + 1) * MT) - 1;
                            if (upper && cmax <= rmin) continue;
                            mt.push_back(make_int2(a, b));
                        }
            p.nmt = (int64_t)mt.size();
            p.mtiles.alloc(mt.size() * sizeof(int2) + 8, st);
            if (!mt.empty()) h2d(p.mtiles.p, mt.data(), mt.size() * sizeof(int2), st);
        }
        p.tiles.alloc(p.at[4] * sizeof(int2) + 8, st);
        for (int g = 0; g < 4; g++)
            if (!grp[g].empty()) h2d(p.tiles.as<int2>() + p.at[g], grp[g].data(), grp[g].size() * sizeof(int2), st);
        it = s->plans.emplace(key, std::move(plan)).first;
    }
    return *it->second;
}

void bitset_matrix(gdist_ctx* ctx, const gdist_sets* s, int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                   bool upper, int32_t* d_I, int64_t ldI) {
    hipStream_t st = ctx->stream;
    const int64_t nr = r1 - r0, nc = c1 - c0;
    if (nr <= 0 || nc <= 0) return;
    const unsigned long long* tbits = s->sparse ? s->dbits.as<unsigned long long>() : s->bits.as<unsigned long long>();
    const int64_t tW = s->sparse ? s->Wd : s->W;
    MatrixPlan& p = matrix_plan(ctx, s, r0, r1, c0, c1, upper);
    if (p.at[4] == 0) return;   // no pair in the region

    // Rare kernel per call from the cost model (rare_choice): list-major opens
    // every list and walks the pairs from this block's rows with global
    // atomics (short lists, blocks with few pairs per row: C2, the last rank
    // of a row-sharded triangle); row-major walks each row's lists into LDS
    // counters (lists feeding several increments per record: C3, C4; ranks
    // with many pairs per row). GDIST_RARE_KERNEL=0|1 forces one (A/B). The
    // list-major kernel uses atomics only, like the dense kernel, so it runs
    // beside the dense launch on the side stream (GDIST_RARE_OVERLAP=0 keeps
    // it in line).
    bool row_major = false;
    if (s->n_rare > 0) (void)bitset_block_cost_s(s, r0, r1, c0, c1, upper, &row_major);
    const bool list_major = ctx->has_option(OPT_RARE_KERNEL) ? ctx->option(OPT_RARE_KERNEL, 0) == 0 : !row_major;
    const bool overlap = s->n_rare > 0 && list_major && ctx->option(OPT_RARE_OVERLAP, 1) != 0;
    // The row-major rare kernel too, when it flushes its rows with atomics
    // (round 3, C3: its scattered list reads overlap the VALU-bound tiles)
    const bool rows_side = s->n_rare > 0 && !list_major && !s->sparse && ctx->option(OPT_RARE_OVERLAP, 1) != 0;
    // The sparse words and the list-major rare kernel add atomically, like
    // the dense tiles, so they run on the side stream beside them; so does
    // the variant tier's row walk (variant.hip)
    const bool side = overlap || s->sparse || rows_side || s->variant;
    bool rare_done = false;               // the sparse chunk reduce added the rare pairs
    auto launch_rare_rows = [&](hipStream_t rs, bool atomic_flush) {
        const int nch = (int)ceil_div(nc, RCH);
        // past one LDS chunk of columns every record once, members added to I
        // by atomics (option rare_direct; the LDS kernel re-walks the row's
        // lists once per chunk)
        if (ctx->option(OPT_RARE_DIRECT, nch > 1 ? 1 : 0) != 0) {
            const int dsplit = (int)std::max<int64_t>(1, std::min<int64_t>(64, ceil_div((int64_t)ctx->cus * 8, nr)));
            const int64_t dgrid = nr * dsplit;
            GD_REQUIRE(dgrid < (int64_t(1) << 31), "rare-tier grid too large");
            FamilyTimer ft(ctx, GDIST_KERNEL_RARE, rs);
            if (s->post_sets16.p)
                rare_rows_direct_kernel<uint16_t><<<(unsigned)dgrid, 256, 0, rs>>>(
                    s->srare_off.as<int64_t>(), s->srare_ent.as<uint64_t>(), s->srare_w.as<uint32_t>(),
                    s->srare_skip.as<uint16_t>(), s->post_sets16.as<uint16_t>(), r0, r1, c0, c1, dsplit,
                    upper ? 1 : 0, d_I, ldI);
            else
                rare_rows_direct_kernel<uint32_t><<<(unsigned)dgrid, 256, 0, rs>>>(
                    s->srare_off.as<int64_t>(), s->srare_ent.as<uint64_t>(), s->srare_w.as<uint32_t>(),
                    s->srare_skip.as<uint16_t>(), s->post_sets.as<uint32_t>(), r0, r1, c0, c1, dsplit,
                    upper ? 1 : 0, d_I, ldI);
            GD_HIP(hipGetLastError());
            ft.end();
            return;
        }
        const int64_t units = nr * nch;
        // few rows (C2: 1000): slice each row's rare kmers over several workgroups
        const int nsplit = (int)std::max<int64_t>(1, std::min<int64_t>(16, ceil_div((int64_t)ctx->cus * 8, units)));
        const int64_t rgrid = units * nsplit;
        GD_REQUIRE(rgrid < (int64_t(1) << 31), "rare-tier grid too large");
        // 16-bit counters when no row can reach 2^16 (option rare_c16, default on)
        const bool c16 = s->rare_row_wmax < 65536 && ctx->option(OPT_RARE_C16, 1) != 0;
        const size_t lds = c16 ? (size_t)((std::min<int64_t>(nc, RCH) + 1) / 2) * 4 : (size_t)std::min<int64_t>(nc, RCH) * 4;
        FamilyTimer ft(ctx, GDIST_KERNEL_RARE, rs);
        // threads a workgroup: the LDS counters allow 4 workgroups a CU up to
        // 40 KiB (10,240 columns: C3), 2 beyond (C4's 64 KiB chunks); 32 waves
        // a CU either way (option rare_rows_threads 256 / 512 / 1024)
        const int64_t nt_opt = ctx->option(OPT_RARE_ROWS_THREADS, lds > 40 * 1024 ? 1024 : 512);
        const int rt = nt_opt == 256 ? 256 : nt_opt == 1024 ? 1024 : 512;
        auto go = [&](auto kern, int nt, auto* members) {
            kern<<<(unsigned)rgrid, nt, lds, rs>>>(s->srare_off.as<int64_t>(), s->srare_ent.as<uint64_t>(),
                                                   s->srare_w.as<uint32_t>(), s->srare_skip.as<uint16_t>(), members,
                                                   r0, r1, c0, c1, nch, nsplit, upper ? 1 : 0, atomic_flush ? 1 : 0,
                                                   d_I, ldI);
        };
        if (s->post_sets16.p && c16) {
            if (rt == 1024) go(rare_rows_kernel<uint16_t, 1024, true>, 1024, s->post_sets16.as<uint16_t>());
            else if (rt == 512) go(rare_rows_kernel<uint16_t, 512, true>, 512, s->post_sets16.as<uint16_t>());
            else go(rare_rows_kernel<uint16_t, 256, true>, 256, s->post_sets16.as<uint16_t>());
        } else if (s->post_sets16.p) {
            if (rt == 1024) go(rare_rows_kernel<uint16_t, 1024>, 1024, s->post_sets16.as<uint16_t>());
            else if (rt == 512) go(rare_rows_kernel<uint16_t, 512>, 512, s->post_sets16.as<uint16_t>());
            else go(rare_rows_kernel<uint16_t, 256>, 256, s->post_sets16.as<uint16_t>());
        } else {
            if (rt == 1024) go(rare_rows_kernel<uint32_t, 1024>, 1024, s->post_sets.as<uint32_t>());
            else if (rt == 512) go(rare_rows_kernel<uint32_t, 512>, 512, s->post_sets.as<uint32_t>());
            else go(rare_rows_kernel<uint32_t, 256>, 256, s->post_sets.as<uint32_t>());
        }
        ft.end();
    };
    auto launch_rare_pairs = [&](hipStream_t rs) {
        FamilyTimer ft(ctx, GDIST_KERNEL_RARE, rs);
        rare_pairs_kernel<<<grid_for(s->n_rare, 256, 256 * 64), 256, 0, rs>>>(
            s->post_off.as<int64_t>(), s->post_sets.as<uint32_t>(), s->post_w.as<uint32_t>(), s->n_rare, r0, r1, c0,
            c1, upper ? 1 : 0, d_I, ldI);
        ft.end();
    };
    if (!ctx->capturing) GD_HIP(hipEventRecord(ctx->ev_k0, st));
    // option serial_step = 1: the side stream's families run on the main
    // stream before the dense tiles, one after another (each family's time
    // alone: the C4 slice's MFMA tiles and variant walk otherwise share the
    // CUs); option dense_first: the dense tiles are issued before the side
    // stream's launches (which still wait only for the fork) — by default
    // unless the side stream carries the sparse tiles (C3: step 2.51 vs
    // 2.63 ms, C4 slice 15.8 vs 16.0 ms; C2-realistic's sparse launch first:
    // 0.321 vs 0.353 ms, profiles/r05/s16/)
    const bool serial = ctx->option(OPT_SERIAL_STEP, 0) != 0;
    // option bitset_mfma_store: the MFMA tiles store their counts (one K
    // split; the side families then start after them: the fork is recorded
    // after the dense launch). Off by default: the tiles alone gain (C3 0.71
    // vs 0.76 ms) but the step loses its overlap (C3 1.81 vs 1.67 ms, C4
    // slice span 16.9 vs 14.8 ms; profiles/r05/s26)
    // (only the raw 16-word kernel has the storing form: mstore with another
    // stage layout would give up the overlap without the stores)
    const int64_t tWm = s->sparse ? s->Wd : s->W;
    const bool mraw = ctx->option(OPT_BITSET_MFMA_RAW, 1) != 0;
    const bool mkm2 = ctx->option(OPT_BITSET_MFMA_KM, 4) == 2;
    const int mkm = mraw ? (mkm2 ? 8 : 16) : mkm2 ? 2 : 4;     // words a stage (below)
    const bool mstore = p.nmt > 0 && !s->sparse && mraw && !mkm2 && ctx->option(OPT_BITSET_MFMA_STORE, 0) != 0 &&
                        mfma_min_splits(tWm / mkm, mkm) == 1;
    // raw 16-word stages: the next stage's DMA spread between the MFMAs, one
    // barrier a stage (bitset_mfma_kernel SPREAD; 0: the round-5 schedule.
    // Waves 4-7 at priority 1 as well measured neutral: C4 slice span 14.25-
    // 14.40 vs 14.08-14.63 ms, profiles/r06/s12)
    const bool mspread = ctx->option(OPT_BITSET_MFMA_SCHED, 1) != 0;
    // bit-plane operands (PLANE; tiles alone C3 0.709-0.714 vs 0.715-0.736 ms,
    // C4 slice 7.38-7.50 vs 7.51-7.54, spans unchanged: profiles/r06/s17)
    const bool mplane = ctx->option(OPT_BITSET_MFMA_PLANE, 1) != 0;
    const bool dense_first = side && (mstore || (!serial && ctx->option(OPT_DENSE_FIRST, s->sparse ? 0 : 1) != 0));
    if (side && !mstore) GD_HIP(hipEventRecord(ctx->ev_fork, st));
    auto launch_side = [&]() {
        hipStream_t sd = serial ? st : ctx->side;
        GD_HIP(hipStreamWaitEvent(sd, ctx->ev_fork, 0));
        if (s->sparse) rare_done = sparse_matrix(ctx, s, r0, r1, c0, c1, upper, d_I, ldI, sd, p.sparse);
        // beside the sparse kernel the list-major rare kernel goes to the main
        // stream after the dense tiles (the side stream is busy until the
        // sparse tiles and their reduce end: C2 0.0185 ms in line there)
        if (overlap && !s->sparse) launch_rare_pairs(sd);
        if (rows_side) launch_rare_rows(sd, true);
        if (s->variant) variant_matrix(ctx, s, r0, r1, c0, c1, upper, d_I, ldI, sd);
        GD_HIP(hipGetLastError());
        GD_HIP(hipEventRecord(ctx->ev_join, sd));
    };
    if (side && !dense_first) launch_side();
    if (tW == 0 || (s->sparse && s->sp_fold_dense)) {
        // no dense words, or so few that the sparse flush counts them
    } else {
        const int64_t nch2 = tW / KC2;
        // workgroups per CU the K-split aims for (GDIST_BITSET_WG_PER_CU, A/B)
        const int64_t wg_per_cu = std::max<int64_t>(1, ctx->option(OPT_BITSET_WG_PER_CU, 16));
        // ... but each workgroup streams at least min_kc chunks: a split's
        // prologue and its 16K accumulator atomics amortise over its chunks
        // (launches of few tiles: diagonal, partial; GDIST_BITSET_MIN_CHUNKS, A/B)
        const int64_t min_kc = std::max<int64_t>(1, ctx->option(OPT_BITSET_MIN_CHUNKS, 16));
        const int64_t corg = p.corg;
        auto launch = [&](auto kern, const int2* dtiles, size_t nt) {
            if (nt == 0) return;
            const int64_t target2 = (int64_t)ctx->cus * wg_per_cu;
            const int sp2 = (int)std::max<int64_t>(
                1, std::min<int64_t>(std::max<int64_t>(1, nch2 / min_kc), ceil_div(target2, (int64_t)nt)));
            const int64_t grid2 = (int64_t)nt * sp2;
            GD_REQUIRE(grid2 < (int64_t(1) << 31), "bitset matrix grid too large");
            kern<<<(unsigned)grid2, NT, 0, st>>>(tbits, tW, dtiles, (int)nt, sp2, nch2,
                                                 r0, r1, c0, c1, corg, upper ? 1 : 0, d_I, ldI);
        };
        const int2* dg = p.tiles.as<int2>();
        const size_t* at = p.at;
        FamilyTimer ft(ctx, GDIST_KERNEL_DENSE, st);
        if (p.nmt > 0) {
            // FP4 MFMA tiles: one 128 KiB workgroup per CU; K split so that
            // the grid fills ~4 rounds of the chip, each split >= 8 stages
            // option bitset_mfma_raw (default 1): stages of the bitsets
            // themselves, 16 words a stage, expanded in registers; 0: the FP4
            // nibble operand (KM = 4 or 2 words a stage)
            const bool raw = mraw, km2 = mkm2;
            // words a stage: raw 16 (8 with bitset_mfma_km 2), nibbles 4 (2)
            const int km = mkm;
            const int64_t nst = tW / km;
            // (~2 rounds when side-stream families run beside the tiles: C3's
            // 820 tiles unsplit, step 1.61 vs 1.67 ms with 2 splits, the walk
            // keeping more of the CUs; profiles/r05/s26)
            const int64_t rounds = side ? 2 : 4;
            int msp = (int)std::max<int64_t>(
                1, std::min<int64_t>(std::max<int64_t>(1, nst / 8), ceil_div((int64_t)ctx->cus * rounds, p.nmt)));
            if (ctx->has_option(OPT_BITSET_MFMA_SPLITS))      // A/B: a given K split
                msp = (int)std::max<int64_t>(1, std::min<int64_t>(nst, ctx->option(OPT_BITSET_MFMA_SPLITS, 1)));
            if (mstore) msp = 1;                              // stores: one writer a pair
            // exactness: a split's f32 accumulator sums at most 64 x (its
            // words) bits; f32 holds every integer <= 2^24 exactly, so no
            // split may span more than kMfmaMaxSplitWords words (a pair of
            // ~10 Mbp genomes on both strands shares > 2^24 dense kmers)
            msp = (int)std::max<int64_t>(msp, mfma_min_splits(nst, km));
            GD_REQUIRE(ceil_div(nst, (int64_t)msp) * km <= kMfmaMaxSplitWords, "MFMA K split past the f32 exact bound");
            const int64_t mgrid = p.nmt * msp;
            GD_REQUIRE(mgrid < (int64_t(1) << 31), "MFMA tile grid too large");
            if (!raw && s->fp4_W != tW) {
                // the operand as FP4 nibbles, once per set of bitsets (every
                // rebuild of the bits drops it; a capture replays a call that
                // ran uncaptured first, so the operand exists by then)
                GD_REQUIRE(!ctx->capturing, "FP4 operand built inside a capture");
                gdist_sets* ms = const_cast<gdist_sets*>(s);
                ms->fp4.alloc((size_t)s->nsets * tW * 32 + 64, st);
                fp4_expand_kernel<<<grid_for(s->nsets * tW, 256, 256 * 256), 256, 0, st>>>(
                    tbits, s->nsets * tW, ms->fp4.as<uint4>());
                GD_HIP(hipGetLastError());
                ms->fp4_W = tW;
            }
            // stage ring: KM words a stage x NS stages (option bitset_mfma_ns: 2..4
            // with KM = 2; KM = 4 only double-buffered, 128 KiB either way)
            const int ns = !km2 ? 2 : (int)std::max<int64_t>(2, std::min<int64_t>(4, ctx->option(OPT_BITSET_MFMA_NS, 2)));
            auto mlaunch = [&](auto kern, int lds_bytes) {
                GD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes));
                const unsigned char* op = raw ? reinterpret_cast<const unsigned char*>(tbits) : s->fp4.as<unsigned char>();
                kern<<<(unsigned)mgrid, MNT, lds_bytes, st>>>(op, tW, p.mtiles.as<int2>(), (int)p.nmt, msp, nst, r0,
                                                               r1, c0, c1, upper ? 1 : 0, d_I, ldI);
            };
            if (raw && !km2 && mstore) mlaunch(&bitset_mfma_kernel<4, 2, true, true>, 2 * 2 * mopb<4>());
            else if (raw && !km2 && mspread && mplane)
                mlaunch(&bitset_mfma_kernel<4, 2, true, false, true, true>, 2 * 2 * mopb<4>());
            else if (raw && !km2 && mspread) mlaunch(&bitset_mfma_kernel<4, 2, true, false, true>, 2 * 2 * mopb<4>());
            else if (raw && !km2) mlaunch(&bitset_mfma_kernel<4, 2, true>, 2 * 2 * mopb<4>());
            else if (raw && ns == 4) mlaunch(&bitset_mfma_kernel<2, 4, true>, 4 * 2 * mopb<2>());
            else if (raw && ns == 3) mlaunch(&bitset_mfma_kernel<2, 3, true>, 3 * 2 * mopb<2>());
            else if (raw) mlaunch(&bitset_mfma_kernel<2, 2, true>, 2 * 2 * mopb<2>());
            else if (km == 4) mlaunch(&bitset_mfma_kernel<4, 2>, 2 * 2 * mopb<4>());
            else if (ns == 4) mlaunch(&bitset_mfma_kernel<2, 4>, 4 * 2 * mopb<2>());
            else if (ns == 3) mlaunch(&bitset_mfma_kernel<2, 3>, 3 * 2 * mopb<2>());
            else mlaunch(&bitset_mfma_kernel<2, 2>, 2 * 2 * mopb<2>());
        } else {
            launch(bitset_tile_kernel2<false>, dg, at[1]);
            launch(bitset_tile_kernel2<true>, dg + at[1], at[2] - at[1]);
            auto partial = [&](auto off_k, auto diag_k) {
                launch(off_k, dg + at[2], at[3] - at[2]);
                launch(diag_k, dg + at[3], at[4] - at[3]);
            };
            switch (p.part ? p.rr : 8) {
                case 1: partial(bitset_tile_kernel2<false, 1>, bitset_tile_kernel2<true, 1>); break;
                case 2: partial(bitset_tile_kernel2<false, 2>, bitset_tile_kernel2<true, 2>); break;
                case 3: partial(bitset_tile_kernel2<false, 3>, bitset_tile_kernel2<true, 3>); break;
                case 4: partial(bitset_tile_kernel2<false, 4>, bitset_tile_kernel2<true, 4>); break;
                case 5: partial(bitset_tile_kernel2<false, 5>, bitset_tile_kernel2<true, 5>); break;
                case 6: partial(bitset_tile_kernel2<false, 6>, bitset_tile_kernel2<true, 6>); break;
                case 7: partial(bitset_tile_kernel2<false, 7>, bitset_tile_kernel2<true, 7>); break;
                default: break;   // no partial row tile
            }
        }
        ft.end();
    }
    if (side && mstore) GD_HIP(hipEventRecord(ctx->ev_fork, st));   // after the stored tiles
    if (dense_first) launch_side();
    if (overlap && s->sparse && !rare_done) launch_rare_pairs(st);
    GD_HIP(hipGetLastError());
    ctx->last.launches = 1;
    if (side) GD_HIP(hipStreamWaitEvent(st, ctx->ev_join, 0));
    if (s->n_rare > 0 && !rare_done) {
        if (overlap) {
        } else if (list_major) {
            launch_rare_pairs(st);
        } else if (!rows_side) {
            launch_rare_rows(st, false);
        }
        GD_HIP(hipGetLastError());
        ctx->last.launches = 2;
    }
    if (!ctx->capturing) GD_HIP(hipEventRecord(ctx->ev_k1, st));
    const int64_t lo = std::max(r0, c0), hi = std::min(r1, c1);
    if (!upper && hi > lo) {
        self_pairs_kernel<<<(unsigned)ceil_div(hi - lo, 256), 256, 0, st>>>(s->off.as<int64_t>(), lo, hi, r0, c0, d_I,
                                                                             ldI);
        GD_HIP(hipGetLastError());
    }
}

bool bitset_matrix_fused(gdist_ctx* ctx, const gdist_sets* s, int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                         bool upper, unsigned flags, int32_t* d_I, int64_t ldI, double* d_D, int64_t ldD) {
    // One stream, two launches: the sparse tile kernel (dense words folded
    // in) and its chunk reduce, which adds the rare pairs, STORES I (no
    // zeroing) and writes D (no epilogue launch). Only when every count of
    // the region comes from that reduce: sparse tier, no dense-word launch,
    // chunk partials, the rare pairs in its table (or no rare tier).
    if (!s->sparse || s->variant || !d_D || ctx->option(OPT_SPARSE_FUSED, 1) == 0) return false;
    if (r1 <= r0 || c1 <= c0 || !(s->sp_fold_dense || s->Wd == 0)) return false;
    MatrixPlan& p = matrix_plan(ctx, s, r0, r1, c0, c1, upper);
    sparse_plan(ctx, s, r0, r1, c0, c1, upper, ctx->stream, p.sparse);
    if (p.sparse.ntiles == 0 || !p.sparse.use_part || (s->n_rare > 0 && !p.sparse.rare_in)) return false;
    SparseEpilogue ep;
    ep.D = d_D;
    ep.ldD = ldD;
    ep.off = s->off.as<int64_t>();
    ep.empty_nan = (flags & GDIST_EMPTY_NAN) ? 1 : 0;
    hipStream_t st = ctx->stream;
    if (!ctx->capturing) GD_HIP(hipEventRecord(ctx->ev_k0, st));
    sparse_matrix(ctx, s, r0, r1, c0, c1, upper, d_I, ldI, st, p.sparse, &ep);
    if (!ctx->capturing) GD_HIP(hipEventRecord(ctx->ev_k1, st));
    ctx->last.launches = 1;
    return true;
}

namespace {
// row a of the block: columns j > i zeroed, 16-byte stores from the first
// 16-byte boundary (round 5: 4-byte stores ran at 2.3 TB/s, C3 0.088 ms a step)
__global__ void zero_upper_kernel(int32_t* __restrict__ I, int64_t ldI, int64_t r0, int64_t c0, int64_t nr, int64_t nc) {
    const int64_t a = blockIdx.y;
    const int64_t l0 = r0 + a + 1 - c0;                 // first column position with j > i
    const int64_t lo = l0 > 0 ? l0 : 0;
    if (lo >= nc) return;
    int32_t* row = I + a * ldI;
    const int64_t head = std::min<int64_t>(nc - lo, (int64_t)(((16u - ((uintptr_t)(row + lo) & 15u)) & 15u) >> 2));
    if (blockIdx.x == 0 && threadIdx.x < head) row[lo + threadIdx.x] = 0;
    const int64_t bb = lo + head, n4 = (nc - bb) >> 2;
    int4* body = reinterpret_cast<int4*>(row + bb);
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n4; k += (int64_t)gridDim.x * blockDim.x)
        body[k] = make_int4(0, 0, 0, 0);
    const int64_t t = bb + 4 * n4 + threadIdx.x;
    if (blockIdx.x == 0 && t < nc) row[t] = 0;
}
}  // namespace

void zero_counts(gdist_ctx* ctx, int64_t r0, int64_t r1, int64_t c0, int64_t c1, bool upper, int32_t* d_I,
                 int64_t ldI) {
    const int64_t nr = r1 - r0, nc = c1 - c0;
    if (nr <= 0 || nc <= 0) return;
    if (!upper) {
        GD_HIP(hipMemset2DAsync(d_I, ldI * 4, 0, nc * 4, nr, ctx->stream));
        return;
    }
    for (int64_t a0 = 0; a0 < nr; a0 += 65535) {       // grid.y limit
        const int64_t rows = std::min<int64_t>(65535, nr - a0);
        dim3 grid((unsigned)std::min<int64_t>(16, ceil_div(nc, 1024)), (unsigned)rows);
        zero_upper_kernel<<<grid, 256, 0, ctx->stream>>>(d_I + a0 * ldI, ldI, r0 + a0, c0, rows, nc);
        GD_HIP(hipGetLastError());
    }
}

void distance_epilogue(gdist_ctx* ctx, const gdist_sets* s, int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                       bool upper, unsigned flags, const int32_t* d_I, int64_t ldI, double* d_D, int64_t ldD) {
    const int64_t nr = r1 - r0, nc = c1 - c0;
    if (nr <= 0 || nc <= 0) return;
    // a block row a, its columns strided (round 5: the flat kernel's 64-bit
    // division per element and its skipped lower half ran C3's epilogue at
    // 0.18 ms a step; option epilogue_rows 0 keeps it, A/B)
    if (ctx->option(OPT_EPILOGUE_ROWS, 1) == 0) {
        epilogue_kernel<<<grid_for(nr * nc), 256, 0, ctx->stream>>>(s->off.as<int64_t>(), r0, r1, c0, c1,
                                                                     upper ? 1 : 0, (flags & GDIST_EMPTY_NAN) ? 1 : 0,
                                                                     d_I, ldI, d_D, ldD);
        GD_HIP(hipGetLastError());
        return;
    }
    for (int64_t a0 = 0; a0 < nr; a0 += 65535) {       // grid.y limit
        const int64_t rows = std::min<int64_t>(65535, nr - a0);
        dim3 grid((unsigned)std::min<int64_t>(16, ceil_div(nc, 1024)), (unsigned)rows);
        epilogue_rows_kernel<<<grid, 256, 0, ctx->stream>>>(s->off.as<int64_t>(), r0 + a0, c0, nc, upper ? 1 : 0,
                                                           (flags & GDIST_EMPTY_NAN) ? 1 : 0, d_I + a0 * ldI,
                                                           ldI, d_D + a0 * ldD, ldD);
        GD_HIP(hipGetLastError());
    }
}

}  // namespace gdist
