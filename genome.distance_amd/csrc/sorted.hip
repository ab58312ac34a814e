// sorted.hip — exact |A∩B| over sorted uint64 kmer sets by LDS hash-join tiles.
//
// Same contract as bitset.hip (SequenceKmers.distance over many pairs,
// FastaDistanceProcessor.java:177-186, GenomeProcessor.java:140), for set
// collections whose shared-kmer dictionary would be too wide for bitsets
// (diverse genomes / proteins: SURVEY §8d configs 3 and 4).
//
// Segment index: P-1 global splitters (sampled quantiles of all codes) cut
// every sorted set into P value-range segments, segoff[set][p]. Only
// segment p of A can meet segment p of B.
//
// Kernel (sorted_join_kernel): one 512-thread workgroup per (row set i,
// block of 64 column sets). For each segment p it builds an open-addressing
// hash table of A_i's segment in LDS (8192 × 8 B, ≤ 50 % load; larger
// segments are processed in sub-chunks, which is exact because A's
// sub-chunks are disjoint), then every wave streams its columns' segment p
// from HBM/L2 (coalesced) and probes the table. Per-column counts stay in
// LDS and are stored once at the end: no atomics, every pair written by
// exactly one workgroup. Workgroups are ordered column-block-major and
// remapped so that one XCD runs consecutive units: the ~64 workgroups
// resident on an XCD share the same 64 column sets in its L2.
#include <cstring>
#include <rocprim/rocprim.hpp>

#include <algorithm>

#include "gdist_internal.hpp"

namespace gdist {
namespace {

constexpr int TBL_LOG2 = 13;
constexpr int TBL = 1 << TBL_LOG2;        // 8192 slots = 64 KiB
constexpr int SUB = TBL / 2;              // max keys per table fill
constexpr int CBW = 64;                   // column sets per workgroup
constexpr int NTJ = 512;                  // threads per workgroup (8 waves)
constexpr int SEG_TARGET = 2048;          // mean segment length aimed for
constexpr uint64_t EMPTY = ~0ULL;


__global__ void gather_kernel(const uint64_t* __restrict__ codes, const int64_t* __restrict__ idx, int64_t n,
                              uint64_t* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = codes[idx[i]];
}

// segoff[s][t]: t = 0 -> off[s], t = P -> off[s+1], else lower_bound(splitter[t-1])
__global__ void segoff_kernel(const uint64_t* __restrict__ codes, const int64_t* __restrict__ off, int64_t nsets,
                              const uint64_t* __restrict__ split, int nseg, int64_t* __restrict__ segoff) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per = nseg + 1;
    if (e >= nsets * per) return;
    const int64_t s = e / per;
    const int t = (int)(e - s * per);
    const int64_t b = off[s], en = off[s + 1];
    int64_t r;
    if (t == 0) r = b;
    else if (t == nseg) r = en;
    else {
        const uint64_t v = split[t - 1];
        int64_t lo = b, hi = en;
        while (lo < hi) {
            int64_t mid = (lo + hi) >> 1;
            if (codes[mid] < v) lo = mid + 1; else hi = mid;
        }
        r = lo;
    }
    segoff[e] = r;
}

__device__ __forceinline__ uint32_t slot_of(uint64_t v) {
    return (uint32_t)((v * 0x9E3779B97F4A7C15ull) >> (64 - TBL_LOG2));
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__global__ __launch_bounds__(NTJ, 1) void sorted_join_kernel(
    const uint64_t* __restrict__ codes, const int64_t* __restrict__ segoff, int nseg,
    const int64_t* __restrict__ cb_prefix, int ncb, int64_t u0, int64_t nunits, int64_t r0, int64_t r1, int64_t c0,
    int64_t c1, const int64_t* __restrict__ colidx, int upper, int32_t* __restrict__ I, int64_t ldI) {
    __shared__ unsigned long long table[TBL];
    __shared__ int32_t cnt[CBW];
    __shared__ int has_empty_key;

    // XCD-aware bijective remap of this launch's units [u0, u0 + G): XCD x
    // gets a contiguous range of them
    const int64_t G = gridDim.x;
    const int64_t b = blockIdx.x;
    const int64_t x = b & 7, kq = b >> 3;
    const int64_t q = G >> 3, rem = G & 7;
    const int64_t u = u0 + x * q + (x < rem ? x : rem) + kq;
    if (u >= nunits) return;

    // unit -> (column block, row)
    int lo = 0, hi = ncb;
    while (hi - lo > 1) {
        int mid = (lo + hi) >> 1;
        if (cb_prefix[mid] <= u) lo = mid; else hi = mid;
    }
    const int cb = lo;
    const int64_t i = r0 + (u - cb_prefix[cb]);
    if (i < r0 || i >= r1) return;   // defensive: never address outside the region
    const int64_t cs = c0 + (int64_t)cb * CBW;
    const int64_t ce = cs + CBW < c1 ? cs + CBW : c1;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < CBW) cnt[tid] = 0;

    const int64_t per = nseg + 1;
    const int64_t* arow = segoff + i * per;
    for (int p = 0; p < nseg; p++) {
        const int64_t a0 = arow[p], a1 = arow[p + 1];
        if (a0 == a1) continue;
        for (int64_t sb = a0; sb < a1; sb += SUB) {
            const int64_t se = sb + SUB < a1 ? sb + SUB : a1;
            for (int t = tid; t < TBL; t += NTJ) table[t] = EMPTY;
            if (tid == 0) has_empty_key = 0;
            __syncthreads();
            for (int64_t e = sb + tid; e < se; e += NTJ) {
                const uint64_t v = codes[e];
                if (v == EMPTY) { has_empty_key = 1; continue; }
                uint32_t h = slot_of(v);
                while (true) {
                    unsigned long long old = atomicCAS(&table[h], EMPTY, (unsigned long long)v);
                    if (old == EMPTY) break;
                    h = (h + 1) & (TBL - 1);
                }
            }
            __syncthreads();
            const int hek = has_empty_key;
            for (int64_t t = wave; t < ce - cs; t += NTJ / 64) {
                const int64_t j = colidx ? colidx[cs + t] : cs + t;
                if (upper && j <= i) continue;
                const int64_t* brow = segoff + j * per;
                const int64_t b0 = brow[p], b1 = brow[p + 1];
                int c = 0;
                for (int64_t e = b0 + lane; e < b1; e += 64) {
                    const uint64_t v = codes[e];
                    if (v == EMPTY) { c += hek; continue; }
                    uint32_t h = slot_of(v);
                    while (true) {
                        const unsigned long long tv = table[h];
                        if (tv == v) { c++; break; }
                        if (tv == EMPTY) break;
                        h = (h + 1) & (TBL - 1);
                    }
                }
                c = wave_sum(c);
                if (lane == 0) cnt[t] += c;
            }
            __syncthreads();
        }
    }
    __syncthreads();
    for (int64_t t = tid; t < ce - cs; t += NTJ) {
        const int64_t j = colidx ? colidx[cs + t] : cs + t;
        if (upper && j <= i) continue;
        I[(i - r0) * ldI + (colidx ? (cs + t - c0) : (j - c0))] = cnt[t];
    }
}

}  // namespace

void build_segments(gdist_ctx* ctx, gdist_sets* s) {
    hipStream_t st = ctx->stream;
    int64_t maxn = 0;
    for (int64_t i = 0; i < s->nsets; i++) maxn = std::max(maxn, s->h_off[i + 1] - s->h_off[i]);
    int nseg = (int)std::max<int64_t>(1, std::min<int64_t>(4096, ceil_div(maxn, SEG_TARGET)));
    // splitters: sampled quantiles over all codes
    std::vector<uint64_t> split;
    if (nseg > 1 && s->total > 0) {
        const int64_t want = std::min<int64_t>(s->total, (int64_t)nseg * 64);
        std::vector<int64_t> idx(want);
        for (int64_t t = 0; t < want; t++) idx[t] = (int64_t)((double)(t + 0.5) * (double)s->total / (double)want);
        DevBuf di(want * 8, st), dv(want * 8, st);
        h2d(di.p, idx.data(), want * 8, st);
        gather_kernel<<<(int)ceil_div(want, 256), 256, 0, st>>>(s->codes.as<uint64_t>(), di.as<int64_t>(), want,
                                                                dv.as<uint64_t>());
        GD_HIP(hipGetLastError());
        std::vector<uint64_t> v(want);
        d2h(v.data(), dv.p, want * 8, st);
        GD_HIP(hipStreamSynchronize(st));
        std::sort(v.begin(), v.end());
        for (int t = 1; t < nseg; t++) {
            uint64_t sp = v[(size_t)((double)t * (double)want / (double)nseg)];
            if (split.empty() || sp > split.back()) split.push_back(sp);
        }
        nseg = (int)split.size() + 1;
    } else {
        nseg = 1;
    }
    DevBuf dsplit(split.size() * 8 + 8, st);
    if (!split.empty())
        h2d(dsplit.p, split.data(), split.size() * 8, st);
    const int64_t n = s->nsets * (int64_t)(nseg + 1);
    s->segoff.alloc(n * 8 + 8, st);
    if (n)
        segoff_kernel<<<(int)ceil_div(n, 256), 256, 0, st>>>(s->codes.as<uint64_t>(), s->off.as<int64_t>(), s->nsets,
                                                            dsplit.as<uint64_t>(), nseg, s->segoff.as<int64_t>());
    GD_HIP(hipGetLastError());
    std::vector<int64_t> h(n);
    if (n) d2h(h.data(), s->segoff.p, n * 8, st);
    GD_HIP(hipStreamSynchronize(st));
    int64_t mx = 0;
    for (int64_t e = 0; e < s->nsets; e++)
        for (int t = 0; t < nseg; t++) mx = std::max(mx, h[e * (nseg + 1) + t + 1] - h[e * (nseg + 1) + t]);
    s->nseg = nseg;
    s->max_seg = mx;
    s->seg_split = std::move(dsplit);
}

// Sets appended to an indexed collection (gdist_sets_append: the Java
// methods drop-in's genome cache, one genome at a time) get their rows with
// the collection's splitters; the old rows stay valid (they hold code
// positions, which an append does not move). ADVICE r5: rebuilding the whole
// index after every append cost O(genomes x total codes) over a pair list.
// The splitters were sampled from the old sets only: any splitters give an
// exact join, they only set how evenly the segments split.
void extend_segments(gdist_ctx* ctx, gdist_sets* s, int64_t n_old) {
    hipStream_t st = ctx->stream;
    const int nseg = s->nseg;
    const int64_t per = nseg + 1, nadd = s->nsets - n_old;
    if (nadd <= 0) return;
    DevBuf grown((size_t)(s->nsets * per) * 8 + 8, st);
    if (n_old) GD_HIP(hipMemcpyAsync(grown.p, s->segoff.p, (size_t)(n_old * per) * 8, hipMemcpyDeviceToDevice, st));
    segoff_kernel<<<(int)ceil_div(nadd * per, 256), 256, 0, st>>>(
        s->codes.as<uint64_t>(), s->off.as<int64_t>() + n_old, nadd, s->seg_split.as<uint64_t>(), nseg,
        grown.as<int64_t>() + n_old * per);
    GD_HIP(hipGetLastError());
    std::vector<int64_t> h(nadd * per);
    d2h(h.data(), grown.as<int64_t>() + n_old * per, nadd * per * 8, st);
    GD_HIP(hipStreamSynchronize(st));
    for (int64_t e = 0; e < nadd; e++)
        for (int t = 0; t < nseg; t++) s->max_seg = std::max(s->max_seg, h[e * per + t + 1] - h[e * per + t]);
    s->segoff = std::move(grown);
}

static void launch_join(gdist_ctx* ctx, const gdist_sets* s, int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                        const int64_t* d_colidx, bool upper, int32_t* d_I, int64_t ldI) {
    hipStream_t st = ctx->stream;
    const int64_t nc = c1 - c0;
    const int ncb = (int)ceil_div(nc, CBW);
    std::vector<int64_t> prefix(ncb + 1, 0);
    for (int cb = 0; cb < ncb; cb++) {
        const int64_t ce = std::min<int64_t>(c1, c0 + (int64_t)(cb + 1) * CBW);
        int64_t rows_end = r1;
        if (upper && !d_colidx) rows_end = std::min<int64_t>(r1, ce - 1);   // need some j > i
        prefix[cb + 1] = prefix[cb] + std::max<int64_t>(0, rows_end - r0);
    }
    const int64_t nunits = prefix[ncb];
    if (nunits == 0) return;
    DevBuf dp((ncb + 1) * 8, st);
    h2d(dp.p, prefix.data(), (ncb + 1) * 8, st);
    GD_HIP(hipEventRecord(ctx->ev_k0, st));
    // a dispatch holds < 2^32 work-items: launches of at most 2^31 threads
    // (C4's largest row block is ~55 M units)
    const int64_t per = (int64_t(1) << 31) / NTJ;
    int launches = 0;
    FamilyTimer ft(ctx, GDIST_KERNEL_SORTED, st);
    for (int64_t u0 = 0; u0 < nunits; u0 += per, launches++)
        sorted_join_kernel<<<(unsigned)std::min(per, nunits - u0), NTJ, 0, st>>>(
            s->codes.as<uint64_t>(), s->segoff.as<int64_t>(), s->nseg, dp.as<int64_t>(), ncb, u0, nunits, r0, r1, c0,
            c1, d_colidx, upper ? 1 : 0, d_I, ldI);
    GD_HIP(hipGetLastError());
    ft.end();
    GD_HIP(hipEventRecord(ctx->ev_k1, st));
    ctx->last.launches = launches;
}

void sorted_matrix(gdist_ctx* ctx, const gdist_sets* s, int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                   bool upper, int32_t* d_I, int64_t ldI) {
    launch_join(ctx, s, r0, r1, c0, c1, nullptr, upper, d_I, ldI);
}

// one row against an explicit column list (row queries)
void sorted_row(gdist_ctx* ctx, const gdist_sets* s, int64_t q, const int64_t* d_cols, int64_t ncols,
                int32_t* d_I) {
    launch_join(ctx, s, q, q + 1, 0, ncols, d_cols, false, d_I, ncols);
}

}  // namespace gdist
