// pack.hip — device-side kmer extraction and packing into sorted unique
// uint64 code sets (CSR).  Replaces KmerType.createKmers(seq, K)
// (FastaDistanceProcessor.java:153,184), new GenomeKmers(genome)
// (GenomeProcessor.java:109,139) and new ProteinKmers(seq)
// (ProteinKmerReader.java:101), which build a HashSet<String> per sequence.
//
// Pipeline per chunk of sequences (bounded so keys+values fit comfortably):
//   1. validate   — unencodable chars in keep / 5-bit modes -> EINVAL
//   2. extract    — one thread per window: code (fwd, rc or canonical),
//                   value = set id, or the "invalid" id for skipped windows
//   3. radix sort of code|set keys (the chunk's dictionary summary is the
//      runs of codes), then a stable radix sort on the set bits alone
//   4. unique flags + exclusive scan -> compacted CSR codes, offsets by
//      lower_bound of each set id in the sorted keys
// From host bytes (gdist_sets_pack) a host thread uploads chunk c + 1 while
// the device works on chunk c (ChunkUploader).
// The alphabet maps are order preserving, so code order == Java String order.
#include <cstring>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <atomic>
#include <future>
#include <thread>

#include "gdist_internal.hpp"

namespace gdist {

int code_bits(int kind, int k, unsigned flags) {
    unsigned am = flags & GDIST_AMBIG_MASK;
    if (kind == GDIST_DNA) {
        bool skip = (am != GDIST_AMBIG_KEEP);
        return skip ? 2 * k : 3 * k;
    }
    return k <= 8 ? 8 * k : 5 * k;
}

namespace {

// Symbol table per (kind, flags): sym[c] = code symbol, -1 = unencodable,
// -2 = skip the window (ambiguity skip mode). comp[sym] for DNA.
struct Alphabet {
    int8_t sym[256];
    int8_t comp[8];
    int bits;
    bool fold;
};

Alphabet make_alphabet(int kind, int k, unsigned flags) {
    Alphabet a{};
    unsigned am = flags & GDIST_AMBIG_MASK;
    bool skip = (am == GDIST_AMBIG_SKIP) || (am == GDIST_AMBIG_DEFAULT && kind == GDIST_DNA);
    a.fold = (kind == GDIST_DNA) || !(flags & GDIST_NO_CASE_FOLD);
    for (int c = 0; c < 256; c++) a.sym[c] = -1;
    for (int i = 0; i < 8; i++) a.comp[i] = 0;
    if (kind == GDIST_DNA) {
        if (skip) {
            a.bits = 2;
            const char* al = "ACGT";
            for (int i = 0; i < 4; i++) a.sym[(unsigned char)al[i]] = (int8_t)i;
            for (int c = 0; c < 256; c++) if (a.sym[c] < 0) a.sym[c] = -2;
            a.comp[0] = 3; a.comp[1] = 2; a.comp[2] = 1; a.comp[3] = 0;
        } else {
            a.bits = 3;
            const char* al = "ACGNRTY";
            for (int i = 0; i < 7; i++) a.sym[(unsigned char)al[i]] = (int8_t)i;
            const int8_t cp[7] = {5, 2, 1, 3, 6, 0, 4};
            for (int i = 0; i < 7; i++) a.comp[i] = cp[i];
        }
    } else {
        a.bits = (k <= 8) ? 8 : 5;
        for (int c = 0; c < 256; c++) {
            if (a.bits == 8) a.sym[c] = 0;            // raw byte (value taken from c)
            else if (c == '*') a.sym[c] = 0;
            else if (c >= 'A' && c <= 'Z') a.sym[c] = (int8_t)(1 + c - 'A');
        }
        if (skip) {
            for (int c = 0; c < 256; c++) {
                bool std_aa = c != 0 && std::char_traits<char>::find("ACDEFGHIKLMNPQRSTVWY", 20, (char)c);
                if (!std_aa) a.sym[c] = -2;
            }
        }
    }
    // fold lower case onto upper case entries
    if (a.fold)
        for (int c = 'a'; c <= 'z'; c++) a.sym[c] = a.sym[c - 32];
    a.sym[0] = -2;   // sequence separator: no kmer spans it, in every mode
    return a;
}

struct AlphabetDev {
    int8_t sym[256];
    int8_t comp[8];
};

__global__ void validate_kernel(const unsigned char* __restrict__ seqs, int64_t begin, int64_t end,
                                AlphabetDev al, int* __restrict__ bad) {
    int64_t i = begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int local = 0;
    for (; i < end; i += stride) local |= (al.sym[seqs[i]] == -1);
    if (__any(local) && (threadIdx.x & 63) == 0) atomicOr(bad, 1);
}

// Window w of the chunk -> sequence s (binary search in win_off), position,
// then the k symbols. Emits 1 or 2 (BOTH) entries per window.
// CM: the code-major sort keys code << idbits | id straight away (the
// summary path), no id array; any_invalid (CM) is set to 1 when a window was
// skipped (plain stores, every writer writes 1)
template <bool RAW8, bool CM = false>
__global__ __launch_bounds__(256) void extract_kernel(
    const unsigned char* __restrict__ seqs, const int64_t* __restrict__ seq_off,
    const int64_t* __restrict__ win_off, int nseq, int64_t nwin, int k, int bits, int strand,
    AlphabetDev al, uint64_t* __restrict__ keys, int32_t* __restrict__ vals, int idbits = 0,
    int* __restrict__ any_invalid = nullptr) {
    __shared__ int8_t sym[256];
    __shared__ int8_t comp[8];
    for (int t = threadIdx.x; t < 256; t += blockDim.x) sym[t] = al.sym[t];
    if (threadIdx.x < 8) comp[threadIdx.x] = al.comp[threadIdx.x];
    __syncthreads();
    const uint64_t mask = (k * bits >= 64) ? ~0ULL : ((1ULL << (k * bits)) - 1);
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwin; w += stride) {
        // upper_bound(win_off[0..nseq], w) - 1
        int lo = 0, hi = nseq;
        while (hi - lo > 1) {
            int mid = (lo + hi) >> 1;
            if (win_off[mid] <= w) lo = mid; else hi = mid;
        }
        const int s = lo;
        const unsigned char* p = seqs + seq_off[s] + (w - win_off[s]);
        uint64_t fwd = 0, rc = 0;
        bool valid = true;
        for (int t = 0; t < k; t++) {
            unsigned char c = p[t];
            int sy = sym[c];
            valid &= (sy >= 0);
            // raw 8-bit protein codes take the (pre-folded) byte itself
            uint64_t v = RAW8 ? (uint64_t)c : (uint64_t)(sy < 0 ? 0 : sy);
            fwd = (fwd << bits) | v;
            if (strand != GDIST_STRAND_FWD)
                rc |= (uint64_t)comp[sy < 0 ? 0 : sy] << (bits * t);
        }
        fwd &= mask;
        const int32_t id = valid ? s : nseq;
        if (CM) {
            if (!valid) *any_invalid = 1;
            const uint64_t sid = (uint64_t)(uint32_t)id;
            if (strand == GDIST_STRAND_BOTH) {
                keys[2 * w] = (fwd << idbits) | sid;
                keys[2 * w + 1] = (rc << idbits) | sid;
            } else {
                keys[w] = ((strand == GDIST_STRAND_CANON ? (fwd < rc ? fwd : rc) : fwd) << idbits) | sid;
            }
            continue;
        }
        if (strand == GDIST_STRAND_BOTH) {
            keys[2 * w] = fwd; vals[2 * w] = id;
            keys[2 * w + 1] = rc; vals[2 * w + 1] = id;
        } else if (strand == GDIST_STRAND_CANON) {
            keys[w] = fwd < rc ? fwd : rc; vals[w] = id;
        } else {
            keys[w] = fwd; vals[w] = id;
        }
    }
}

// Raw 8-bit protein codes with case folding need the folded byte value.
__global__ __launch_bounds__(256) void fold_bytes_kernel(unsigned char* __restrict__ dst,
                                                         const unsigned char* __restrict__ src,
                                                         int64_t n) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        unsigned char c = src[i];
        dst[i] = (c >= 'a' && c <= 'z') ? (unsigned char)(c - 32) : c;
    }
}

// After the two sorts: unique & valid flags.
__global__ void unique_flags_kernel(const uint64_t* __restrict__ codes, const int32_t* __restrict__ ids,
                                    int64_t n, int32_t invalid, int32_t* __restrict__ flag) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        int32_t id = ids[i];
        bool f = id != invalid && (i == 0 || codes[i] != codes[i - 1] || id != ids[i - 1]);
        flag[i] = f ? 1 : 0;
    }
}

__global__ void compact_kernel(const uint64_t* __restrict__ codes, const int32_t* __restrict__ flag,
                               const int64_t* __restrict__ pos, int64_t n, uint64_t* __restrict__ out) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        if (flag[i]) out[pos[i]] = codes[i];
}

// (set, code) pairs <-> one key set << cbits | code (cbits + set bits <= 64)
__global__ void pack_keys_kernel(const uint64_t* __restrict__ codes, const int32_t* __restrict__ ids, int64_t n,
                                 int cbits, uint64_t* __restrict__ keys) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        keys[i] = cbits < 64 ? ((uint64_t)(uint32_t)ids[i] << cbits) | codes[i] : codes[i];
}

__global__ void unpack_keys_kernel(const uint64_t* __restrict__ keys, int64_t n, int cbits,
                                   uint64_t* __restrict__ codes, int32_t* __restrict__ ids) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const uint64_t mask = cbits < 64 ? (uint64_t(1) << cbits) - 1 : ~0ull;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t k = keys[i];
        codes[i] = k & mask;
        ids[i] = cbits < 64 ? (int32_t)(k >> cbits) : 0;
    }
}

// off[s] = pos[lower_bound(ids, s)] (or the unique total past the end).
__global__ void set_offsets_kernel(const int32_t* __restrict__ ids, const int64_t* __restrict__ pos,
                                   const int32_t* __restrict__ flag, int64_t n, int nsets,
                                   int64_t base, int64_t* __restrict__ off) {
    int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s > nsets) return;
    int64_t lo = 0, hi = n;   // first index with ids[idx] >= s
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (ids[mid] < s) lo = mid + 1; else hi = mid;
    }
    int64_t total = n ? pos[n - 1] + flag[n - 1] : 0;
    off[s] = base + (lo < n ? pos[lo] : total);
}

// Code-major keys (option pack_summary): code << idbits | set, the set field
// nsets marking an invalid window. Sorted, equal keys are one set's repeats of
// a kmer, and the runs of equal codes (one key per holding set after the
// unique) are the chunk's dictionary summary; a stable sort on the set bits
// alone then gives the set-major CSR with each set's codes still ascending.
__global__ void pack_keys_cm_kernel(const uint64_t* __restrict__ codes, const int32_t* __restrict__ ids, int64_t n,
                                    int idbits, uint64_t* __restrict__ keys) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        keys[i] = (codes[i] << idbits) | (uint32_t)ids[i];
}

// The unique pass in two reads of the sorted keys instead of a flag array,
// its scan and an emit pass over flags + positions (16 B of flags and 16 B
// of positions a key): tiles of kSelTile keys; cm_count_kernel sums each
// tile's flag words, one exclusive scan over the tiles, cm_select_kernel
// recomputes the flags of its tile (staged in LDS with the key before it),
// scans them within the block and writes the unique keys and the run heads.
constexpr int kSelT = 256, kSelPer = 16, kSelTile = kSelT * kSelPer;

__device__ __forceinline__ int64_t cm_flag(uint64_t k, uint64_t p, bool first, uint64_t smask, uint64_t invalid,
                                           int idbits) {
    const bool u = (k & smask) != invalid && (first || k != p);
    const bool h = u && (first || (k >> idbits) != (p >> idbits));
    return (int64_t)u | ((int64_t)h << 32);
}

// int64 sum over the block (every thread gets it) / exclusive prefix of the thread
__device__ __forceinline__ int64_t block_excl_scan_i64(int64_t v, int64_t* red, int64_t* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) red[wv] = x;
    __syncthreads();
    int64_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kSelT / 64; w++) {
        before += w < wv ? red[w] : 0;
        all += red[w];
    }
    __syncthreads();
    *total = all;
    return before + x - v;
}

__global__ __launch_bounds__(kSelT) void cm_count_kernel(const uint64_t* __restrict__ keys, int64_t n, uint64_t smask,
                                                         uint64_t invalid, int idbits, int64_t* __restrict__ bsum) {
    __shared__ int64_t red[kSelT / 64];
    const int64_t t0 = (int64_t)blockIdx.x * kSelTile;
    int64_t acc = 0;
#pragma unroll 4
    for (int j = 0; j < kSelPer; j++) {
        const int64_t i = t0 + j * kSelT + threadIdx.x;
        if (i < n) acc += cm_flag(keys[i], i ? keys[i - 1] : 0, i == 0, smask, invalid, idbits);
    }
    int64_t total;
    block_excl_scan_i64(acc, red, &total);
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(kSelT) void cm_select_kernel(const uint64_t* __restrict__ keys, int64_t n, uint64_t smask,
                                                          uint64_t invalid, int idbits, const int64_t* __restrict__ bpre,
                                                          uint64_t* __restrict__ u, uint64_t* __restrict__ codes,
                                                          int64_t* __restrict__ start) {
    // slot i of the tile (i = 0: the key before it) at i + i / 16: a thread's
    // 16 consecutive keys then sit 17 words from the next thread's (2-way
    // bank conflicts instead of 32-way)
    __shared__ uint64_t sk[kSelTile + 1 + (kSelTile + 1) / 16 + 1];
    __shared__ int64_t red[kSelT / 64];
    const int64_t t0 = (int64_t)blockIdx.x * kSelTile;
    const int m = (int)(n - t0 < kSelTile ? n - t0 : kSelTile);
    for (int j = threadIdx.x; j < m; j += kSelT) sk[(1 + j) + ((1 + j) >> 4)] = keys[t0 + j];
    if (threadIdx.x == 0) sk[0] = t0 ? keys[t0 - 1] : 0;
    __syncthreads();
    const int b = threadIdx.x * kSelPer;
    int64_t f[kSelPer], tot = 0;
    uint64_t kv[kSelPer + 1];
    kv[0] = sk[b + (b >> 4)];
#pragma unroll
    for (int j = 0; j < kSelPer; j++) {
        const int i = b + 1 + j;
        kv[j + 1] = sk[i + (i >> 4)];
    }
#pragma unroll
    for (int j = 0; j < kSelPer; j++) {
        const int x = b + j;
        f[j] = x < m ? cm_flag(kv[j + 1], kv[j], t0 + x == 0, smask, invalid, idbits) : 0;
        tot += f[j];
    }
    int64_t all;
    const int64_t excl = block_excl_scan_i64(tot, red, &all);   // every thread's keys are in registers
    int64_t p = bpre[blockIdx.x] + excl;
    // the tile's unique keys are one contiguous run of u: gathered in LDS (the
    // key tile, free after the scan) and stored coalesced, not 16 keys a
    // thread at 128-byte strides
    int lp = (int)(excl & 0xFFFFFFFFll);
#pragma unroll
    for (int j = 0; j < kSelPer; j++) {
        if (f[j] & 1) {
            const uint64_t k = kv[j + 1];
            sk[lp + (lp >> 4)] = k;
            lp++;
            if (f[j] >> 32) { codes[p >> 32] = k >> idbits; start[p >> 32] = p & 0xFFFFFFFFll; }
        }
        p += f[j];
    }
    __syncthreads();
    const int64_t ub = bpre[blockIdx.x] & 0xFFFFFFFFll;
    const int nu = (int)(all & 0xFFFFFFFFll);
    for (int i = threadIdx.x; i < nu; i += kSelT) u[ub + i] = sk[i + (i >> 4)];
}

__global__ void cm_run_counts_kernel(const int64_t* __restrict__ start, int64_t nruns, int64_t n,
                                     uint32_t* __restrict__ counts) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nruns; r += stride)
        counts[r] = (uint32_t)((r + 1 < nruns ? start[r + 1] : n) - start[r]);
}

__global__ void cm_codes_kernel(const uint64_t* __restrict__ u, int64_t n, int idbits, uint64_t* __restrict__ codes) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) codes[i] = u[i] >> idbits;
}

// off[s] = base + lower_bound(u & smask, s) over the set-major unique keys
__global__ void cm_set_offsets_kernel(const uint64_t* __restrict__ u, int64_t n, uint64_t smask, int nsets,
                                      int64_t base, int64_t* __restrict__ off) {
    int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s > nsets) return;
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if ((int64_t)(u[mid] & smask) < s) lo = mid + 1; else hi = mid;
    }
    off[s] = base + lo;
}

inline int grid_for(int64_t n, int block = 256, int64_t cap = 256 * 32) {
    int64_t g = ceil_div(n, block);
    return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

__global__ void valid_flags_kernel(const int32_t* __restrict__ ids, int64_t n, int32_t invalid,
                                   int32_t* __restrict__ flag) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        flag[i] = ids[i] != invalid ? 1 : 0;
}

// valid extracted entries -> (code, entry index); the index is the locus key
__global__ void guide_compact_kernel(const uint64_t* __restrict__ keys, const int32_t* __restrict__ flag,
                                     const int64_t* __restrict__ pos, int64_t n, uint64_t* __restrict__ codes,
                                     int32_t* __restrict__ idx) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        if (flag[i]) { codes[pos[i]] = keys[i]; idx[pos[i]] = (int32_t)i; }
}

__global__ void code_heads_kernel(const uint64_t* __restrict__ codes, int64_t n, int32_t* __restrict__ flag) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        flag[i] = (i == 0 || codes[i] != codes[i - 1]) ? 1 : 0;
}

__global__ void guide_unique_kernel(const uint64_t* __restrict__ codes, const int32_t* __restrict__ idx,
                                    const int32_t* __restrict__ flag, const int64_t* __restrict__ pos, int64_t n,
                                    uint64_t* __restrict__ ucodes, uint64_t* __restrict__ ukeys) {
    int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        if (flag[i]) { ucodes[pos[i]] = codes[i]; ukeys[pos[i]] = (uint64_t)idx[i]; }
}

}  // namespace

// Locus guides of a collection (sparse.hip): the first n extracted entries
// (the windows of the first kGuides sequences, in window order; with both
// strands entry 2w + strand) -> distinct codes with the index of their first
// valid entry. The radix sort is stable, so the first entry of a code's run
// is its first occurrence.
static void guide_from_extract(gdist_ctx* ctx, const uint64_t* keys, const int32_t* ids, int64_t n, int32_t invalid,
                               int cbits, gdist_sets* out) {
    hipStream_t st = ctx->stream;
    out->n_guide = 0;
    if (n <= 0 || n >= (int64_t(1) << 31)) return;
    DevBuf flag(n * 4 + 4, st), pos(n * 8 + 8, st);
    valid_flags_kernel<<<grid_for(n), 256, 0, st>>>(ids, n, invalid, flag.as<int32_t>());
    GD_HIP(hipGetLastError());
    exclusive_scan_i32_to_i64(ctx, flag.as<int32_t>(), pos.as<int64_t>(), (size_t)n);
    int64_t last = 0;
    int32_t lf = 0;
    d2h(&last, pos.as<int64_t>() + n - 1, 8, st);
    d2h(&lf, flag.as<int32_t>() + n - 1, 4, st);
    const int64_t nv = last + lf;
    if (nv == 0) return;
    DevBuf kA(nv * 8, st), kB(nv * 8, st), vA(nv * 4, st), vB(nv * 4, st);
    guide_compact_kernel<<<grid_for(n), 256, 0, st>>>(keys, flag.as<int32_t>(), pos.as<int64_t>(), n,
                                                      kA.as<uint64_t>(), vA.as<int32_t>());
    GD_HIP(hipGetLastError());
    uint64_t* k = kA.as<uint64_t>(); uint64_t* ka = kB.as<uint64_t>();
    int32_t* v = vA.as<int32_t>(); int32_t* va = vB.as<int32_t>();
    sort_pairs_u64_i32(ctx, k, ka, v, va, (size_t)nv, 0, std::min(64, cbits));
    code_heads_kernel<<<grid_for(nv), 256, 0, st>>>(k, nv, flag.as<int32_t>());
    GD_HIP(hipGetLastError());
    exclusive_scan_i32_to_i64(ctx, flag.as<int32_t>(), pos.as<int64_t>(), (size_t)nv);
    d2h(&last, pos.as<int64_t>() + nv - 1, 8, st);
    d2h(&lf, flag.as<int32_t>() + nv - 1, 4, st);
    const int64_t nu = last + lf;
    out->guide_codes.alloc(nu * 8, st);
    out->guide_keys.alloc(nu * 8, st);
    guide_unique_kernel<<<grid_for(nv), 256, 0, st>>>(k, v, flag.as<int32_t>(), pos.as<int64_t>(), nv,
                                                      out->guide_codes.as<uint64_t>(), out->guide_keys.as<uint64_t>());
    GD_HIP(hipGetLastError());
    GD_HIP(hipStreamSynchronize(st));
    out->n_guide = nu;
}

void sort_pairs_u64_i32(gdist_ctx* ctx, uint64_t*& keys, uint64_t*& keys_alt, int32_t*& vals,
                        int32_t*& vals_alt, size_t n, int begin_bit, int end_bit) {
    if (n == 0) return;
    rocprim::double_buffer<uint64_t> kb(keys, keys_alt);
    rocprim::double_buffer<int32_t> vb(vals, vals_alt);
    size_t tmp = 0;
    GD_HIP(rocprim::radix_sort_pairs(nullptr, tmp, kb, vb, n, begin_bit, end_bit, ctx->stream));
    DevBuf t(tmp, ctx->stream);
    GD_HIP(rocprim::radix_sort_pairs(t.p, tmp, kb, vb, n, begin_bit, end_bit, ctx->stream));
    keys = kb.current(); keys_alt = kb.alternate();
    vals = vb.current(); vals_alt = vb.alternate();
}

static void sort_pairs_i32_u64(gdist_ctx* ctx, int32_t*& keys, int32_t*& keys_alt, uint64_t*& vals,
                               uint64_t*& vals_alt, size_t n, int end_bit) {
    if (n == 0) return;
    // ids are non-negative: sort them as unsigned
    rocprim::double_buffer<uint32_t> kb(reinterpret_cast<uint32_t*>(keys),
                                        reinterpret_cast<uint32_t*>(keys_alt));
    rocprim::double_buffer<uint64_t> vb(vals, vals_alt);
    size_t tmp = 0;
    GD_HIP(rocprim::radix_sort_pairs(nullptr, tmp, kb, vb, n, 0, end_bit, ctx->stream));
    DevBuf t(tmp, ctx->stream);
    GD_HIP(rocprim::radix_sort_pairs(t.p, tmp, kb, vb, n, 0, end_bit, ctx->stream));
    keys = reinterpret_cast<int32_t*>(kb.current());
    keys_alt = reinterpret_cast<int32_t*>(kb.alternate());
    vals = vb.current(); vals_alt = vb.alternate();
}

// option sort_radix 10: onesweep passes of 10 bits (C2's 49-bit pack keys: 5
// passes instead of 7; A/B)
using Onesweep10 = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 12>, rocprim::kernel_config<512, 12>, 10,
                                        rocprim::block_radix_rank_algorithm::match>>;

void sort_keys_u64(gdist_ctx* ctx, uint64_t*& keys, uint64_t*& keys_alt, size_t n, int begin_bit,
                   int end_bit) {
    if (n == 0) return;
    rocprim::double_buffer<uint64_t> kb(keys, keys_alt);
    size_t tmp = 0;
    if (ctx->option(OPT_SORT_RADIX, 8) == 10 && n > (size_t(1) << 22)) {
        GD_HIP(rocprim::radix_sort_keys<Onesweep10>(nullptr, tmp, kb, n, begin_bit, end_bit, ctx->stream));
        DevBuf t(tmp, ctx->stream);
        GD_HIP(rocprim::radix_sort_keys<Onesweep10>(t.p, tmp, kb, n, begin_bit, end_bit, ctx->stream));
    } else {
        GD_HIP(rocprim::radix_sort_keys(nullptr, tmp, kb, n, begin_bit, end_bit, ctx->stream));
        DevBuf t(tmp, ctx->stream);
        GD_HIP(rocprim::radix_sort_keys(t.p, tmp, kb, n, begin_bit, end_bit, ctx->stream));
    }
    keys = kb.current(); keys_alt = kb.alternate();
}

void exclusive_scan_i64(gdist_ctx* ctx, const int64_t* in, int64_t* out, size_t n) {
    if (n == 0) return;
    size_t tmp = 0;
    GD_HIP(rocprim::exclusive_scan(nullptr, tmp, in, out, (int64_t)0, n, rocprim::plus<int64_t>(),
                                   ctx->stream));
    DevBuf t(tmp, ctx->stream);
    GD_HIP(rocprim::exclusive_scan(t.p, tmp, in, out, (int64_t)0, n, rocprim::plus<int64_t>(),
                                   ctx->stream));
}

void exclusive_scan_i32_to_i64(gdist_ctx* ctx, const int32_t* in, int64_t* out, size_t n) {
    if (n == 0) return;
    size_t tmp = 0;
    auto it = rocprim::make_transform_iterator(in, [] __device__(int32_t v) { return (int64_t)v; });
    GD_HIP(rocprim::exclusive_scan(nullptr, tmp, it, out, (int64_t)0, n, rocprim::plus<int64_t>(),
                                   ctx->stream));
    DevBuf t(tmp, ctx->stream);
    GD_HIP(rocprim::exclusive_scan(t.p, tmp, it, out, (int64_t)0, n, rocprim::plus<int64_t>(),
                                   ctx->stream));
}

// Overlapped upload of host sequence bytes: a host thread copies each pack
// chunk's byte range on its own stream in 64 MiB pieces (the runtime's
// pageable path, ~6 GB/s on the box: faster than our own pinned staging with
// a CPU memcpy — one thread, or round 4's eight threads with two pinned 4 MiB
// buffers each (pack 0.38-0.42 s vs 0.32-0.33 s, profiles/r04/s22/abs) — and
// than registering the range, all measured),
// synchronises, then signals the chunk; the
// pack waits for chunk c's signal before its extraction, so chunk c + 1's
// bytes move while chunk c sorts (chunk 0's wait is the part left on the
// clock). Pieces, not one copy per chunk, so that the pack's own small
// read-backs interleave with the upload.
// true when p lies in page-locked host memory (gdist_host_alloc): the
// upload is then one DMA per chunk at the link's rate (~50 GB/s) instead of
// the runtime's staged pageable copies (~6 GB/s, the C2 pack's bound)
static bool host_pinned(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

class ChunkUploader {
  public:
    // mode 1: the runtime's staged pageable copies; 2: register each chunk's
    // host range (page-locked, one DMA); pinned: the caller's buffer is
    // page-locked already (gdist_host_alloc): one DMA per chunk
    ChunkUploader(int device, const char* h, char* d, std::vector<std::pair<int64_t, int64_t>> ranges, int mode,
                  bool pinned)
        : ready_(ranges.size()), pin_(mode == 2 && !pinned), src_pinned_(pinned) {
        for (auto& p : ready_) got_.push_back(p.get_future());
        th_ = std::thread([this, device, h, d, ranges] { run(device, h, d, ranges); });
    }
    ~ChunkUploader() {
        stop_ = true;
        if (th_.joinable()) th_.join();
    }
    void wait(size_t c) { got_[c].get(); }   // rethrows the uploader's error

  private:
    static constexpr int64_t kPiece = int64_t(64) << 20;
    void run(int device, const char* h, char* d, const std::vector<std::pair<int64_t, int64_t>>& ranges) {
        size_t c = 0;
        hipStream_t us = nullptr;
        try {
            GD_HIP(hipSetDevice(device));
            GD_HIP(hipStreamCreateWithFlags(&us, hipStreamNonBlocking));
            for (; c < ranges.size() && !stop_; c++) {
                const int64_t b0 = ranges[c].first, b1 = ranges[c].second;
                // chunks are registered one at a time: adjacent ranges share a page
                bool reg = pin_ && b1 > b0 &&
                           hipHostRegister(const_cast<char*>(h) + b0, (size_t)(b1 - b0), hipHostRegisterDefault) ==
                               hipSuccess;
                if (pin_ && !reg) (void)hipGetLastError();
                if (reg || (src_pinned_ && b1 > b0)) {
                    GD_HIP(hipMemcpyAsync(d + b0, h + b0, (size_t)(b1 - b0), hipMemcpyHostToDevice, us));
                } else {
                    for (int64_t o = b0; o < b1; o += kPiece) {
                        const size_t len = (size_t)std::min(kPiece, b1 - o);
                        GD_HIP(hipMemcpyWithStream(d + o, h + o, len, hipMemcpyHostToDevice, us));
                    }
                }
                GD_HIP(hipStreamSynchronize(us));
                if (reg) GD_HIP(hipHostUnregister(const_cast<char*>(h) + b0));
                ready_[c].set_value();
            }
        } catch (...) {
            for (; c < ranges.size(); c++) ready_[c].set_exception(std::current_exception());
        }
        if (us) {
            (void)hipStreamSynchronize(us);
            (void)hipStreamDestroy(us);
        }
    }
    std::vector<std::promise<void>> ready_;
    std::vector<std::future<void>> got_;
    bool pin_ = false, src_pinned_ = false;
    std::atomic<bool> stop_{false};
    std::thread th_;
};

// Debug hook (diagnostics only): host copies of each stage of the first chunk.
struct PackDebug {
    uint64_t* k_extract; int32_t* v_extract;
    uint64_t* k_sort1; int32_t* v_sort1;
    uint64_t* k_sort2; int32_t* v_sort2;
    int64_t n;
};
static PackDebug* g_pack_debug = nullptr;

// Pack sequences [0, nseq) (device bytes + device/host offsets) into `out`.
void pack_sets(gdist_ctx* ctx, int kind, int k, unsigned flags, const char* d_seqs,
               const int64_t* d_seq_off, const std::vector<int64_t>& h_seq_off, gdist_sets* out,
               const char* h_seqs) {
    const int64_t nseq = (int64_t)h_seq_off.size() - 1;
    GD_REQUIRE(kind == GDIST_DNA || kind == GDIST_PROT, "kind must be GDIST_DNA or GDIST_PROT");
    unsigned am = flags & GDIST_AMBIG_MASK;
    GD_REQUIRE(am != (GDIST_AMBIG_SKIP | GDIST_AMBIG_KEEP), "AMBIG_SKIP and AMBIG_KEEP are exclusive");
    bool dna_keep = kind == GDIST_DNA && am == GDIST_AMBIG_KEEP;
    if (kind == GDIST_DNA)
        GD_REQUIRE(k >= 1 && k <= (dna_keep ? 21 : 32), "DNA kmer size out of range (1..32 skip, 1..21 keep)");
    else
        GD_REQUIRE(k >= 1 && k <= 12, "protein kmer size out of range (1..12)");
    int strand = (kind == GDIST_DNA) ? (int)(flags & GDIST_STRAND_MASK) : (int)GDIST_STRAND_FWD;
    GD_REQUIRE(strand != 3, "invalid strand mode");
    const int mult = (strand == GDIST_STRAND_BOTH) ? 2 : 1;

    Alphabet alh = make_alphabet(kind, k, flags);
    AlphabetDev al{};
    for (int c = 0; c < 256; c++) al.sym[c] = alh.sym[c];
    for (int c = 0; c < 8; c++) al.comp[c] = alh.comp[c];
    const int bits = alh.bits;
    const bool raw8 = (kind == GDIST_PROT && bits == 8);
    const int cbits = code_bits(kind, k, flags);
    hipStream_t st = ctx->stream;

    out->kind = kind; out->k = k; out->flags = flags; out->nsets = nseq;

    const int64_t total_bytes = h_seq_off.back() - h_seq_off.front();
    bool need_validate = dna_keep || (kind == GDIST_PROT && bits == 5);
    // windows per sequence
    std::vector<int64_t> nwin(nseq);
    for (int64_t s = 0; s < nseq; s++) {
        int64_t len = h_seq_off[s + 1] - h_seq_off[s];
        GD_REQUIRE(len >= 0, "sequence offsets must be non-decreasing");
        nwin[s] = std::max<int64_t>(0, len - k + 1);
    }
    // chunks of sequences, at most kChunk entries each (the first sequence of a chunk always fits)
    const int64_t kChunk = std::max<int64_t>(1, ctx->option(OPT_PACK_CHUNK, int64_t(1) << 28));
    std::vector<std::pair<int64_t, int64_t>> chunks;   // [s0, s1)
    for (int64_t s0 = 0, s1; s0 < nseq; s0 = s1) {
        int64_t entries = 0;
        for (s1 = s0; s1 < nseq && (s1 == s0 || entries + nwin[s1] * mult <= kChunk); s1++) entries += nwin[s1] * mult;
        chunks.push_back({s0, s1});
    }
    // host bytes: whole-range passes (validation, folding) need every byte
    // first; otherwise chunk c + 1 uploads while chunk c is packed
    std::unique_ptr<ChunkUploader> up;
    if (h_seqs && total_bytes > 0) {
        char* dst = const_cast<char*>(d_seqs);         // the caller's upload buffer (gdist_sets_pack)
        if (need_validate || (raw8 && alh.fold) || chunks.size() < 2 || ctx->option(OPT_PACK_OVERLAP, 1) == 0) {
            h2d(dst + h_seq_off.front(), h_seqs + h_seq_off.front(), total_bytes, st);
        } else {
            std::vector<std::pair<int64_t, int64_t>> ranges;
            for (auto& c : chunks) ranges.push_back({h_seq_off[c.first], h_seq_off[c.second]});
            up.reset(new ChunkUploader(ctx->device, h_seqs, dst, std::move(ranges), (int)ctx->option(OPT_PACK_OVERLAP, 1),
                                       host_pinned(h_seqs)));
        }
    }

    // 1. validation of the whole byte range (keep modes; 5-bit protein)
    if (need_validate && total_bytes > 0) {
        DevBuf bad(sizeof(int), st);
        GD_HIP(hipMemsetAsync(bad.p, 0, sizeof(int), st));
        validate_kernel<<<grid_for(total_bytes), 256, 0, st>>>(
            reinterpret_cast<const unsigned char*>(d_seqs), h_seq_off.front(), h_seq_off.back(), al,
            bad.as<int>());
        GD_HIP(hipGetLastError());
        int hbad = 0;
        d2h(&hbad, bad.p, sizeof(int), st);
        GD_HIP(hipStreamSynchronize(st));
        GD_REQUIRE(!hbad, "sequence holds a character the kmer code cannot represent "
                          "(DNA keep mode: ACGNRTY; protein k>8: A-Z and '*')");
    }

    // raw 8-bit protein codes take the folded byte value
    DevBuf folded;
    const unsigned char* src = reinterpret_cast<const unsigned char*>(d_seqs);
    if (raw8 && alh.fold && total_bytes > 0) {
        folded.alloc((size_t)h_seq_off.back(), st);
        fold_bytes_kernel<<<grid_for(h_seq_off.back()), 256, 0, st>>>(folded.as<unsigned char>(), src,
                                                                        h_seq_off.back());
        GD_HIP(hipGetLastError());
        src = folded.as<unsigned char>();
    }

    // 2-4. the chunks
    Trace tr(st, ctx->trace());
    tr.mark("pack: validate/fold");
    size_t ci = 0;
    // every chunk compacts its unique codes straight into one buffer. When
    // a buffer for every window (the upper bound `cap`) fits the budget
    // (option pack_codes_budget, default 1/4 of the device memory) it is
    // that; otherwise it is sized after the first chunk from its unique /
    // window ratio and grows (by >= 25 %, re-projected) when a chunk would
    // overflow it, so repetitive input (small k, near-identical sets) needs
    // about its unique codes instead of 8 B per window
    int64_t cap = 0;
    for (int64_t s = 0; s < nseq; s++) cap += nwin[s] * mult;
    int64_t codes_budget = ctx->option(OPT_PACK_CODES_BUDGET, -1);
    if (codes_budget < 0) {
        hipDeviceProp_t prop;
        GD_HIP(hipGetDeviceProperties(&prop, ctx->device));
        codes_budget = (int64_t)(prop.totalGlobalMem / 4);
    }
    int64_t base = 0;                      // unique codes compacted so far
    DevBuf all_codes;
    int64_t all_cap = 0;                   // codes all_codes holds room for
    if (cap * 8 <= codes_budget) {
        all_codes.alloc(cap * 8 + 8, st);
        all_cap = cap;
    }
    // room for `need` codes after `done` of the cap's windows were packed
    auto ensure = [&](int64_t need, int64_t done) {
        if (need <= all_cap) return;
        const double proj = (double)need * (double)cap / (double)std::max<int64_t>(done, 1) * 1.125;
        int64_t want = std::max<int64_t>(need, (int64_t)std::min<double>((double)cap, proj));
        if (all_cap) want = std::max<int64_t>(want, std::min<int64_t>(cap, all_cap + all_cap / 4));
        want = std::max(need, std::min(cap, want));
        DevBuf grown(want * 8 + 8, st);
        if (base) GD_HIP(hipMemcpyAsync(grown.p, all_codes.p, base * 8, hipMemcpyDeviceToDevice, st));
        all_codes = std::move(grown);      // releases the old block after the stream drained
        all_cap = want;
    };
    int64_t done = 0;                      // windows (x strands) of the chunks packed so far
    std::vector<int64_t> h_off(nseq + 1, 0);
    DevBuf d_off((nseq + 1) * sizeof(int64_t), st);
    int64_t s0 = 0;
    bool want_sum = ctx->option(OPT_PACK_SUMMARY, 1) != 0, sum_ok = true;
    std::vector<Summary> pack_sum;
    int64_t sum_runs = 0;
    while (s0 < nseq || (nseq == 0 && s0 == 0)) {
        if (nseq == 0) break;
        int64_t s1 = s0, entries = 0;
        while (s1 < nseq && (s1 == s0 || entries + nwin[s1] * mult <= kChunk)) {
            entries += nwin[s1] * mult;
            s1++;
        }
        GD_REQUIRE(ci < chunks.size() && chunks[ci].first == s0 && chunks[ci].second == s1, "pack: chunk plan");
        if (up) up->wait(ci);                            // this chunk's bytes are on the device
        ci++;
        const int nc = (int)(s1 - s0);
        std::vector<int64_t> hwo(nc + 1, 0);
        for (int i = 0; i < nc; i++) hwo[i + 1] = hwo[i] + nwin[s0 + i];
        const int64_t nw = hwo[nc];
        const int64_t n = nw * mult;
        DevBuf cw((nc + 1) * sizeof(int64_t), st);
        h2d(cw.p, hwo.data(), (nc + 1) * sizeof(int64_t), st);

        int idbits = 1;
        while ((int64_t(1) << idbits) <= nc) idbits++;
        const int64_t nguides = std::min<int64_t>(nc, std::max<int64_t>(0, ctx->option(OPT_GUIDES, kGuides)));
        const bool guides_here = s0 == 0 && nw > 0 && nguides > 0 && locus_order_enabled(ctx);
        PackDebug* dbg = (s0 == 0) ? g_pack_debug : nullptr;
        const bool cm_path = want_sum && !dbg && cbits + idbits <= 64 && n < (int64_t(1) << 31) &&
                             ctx->option(OPT_PACK_SORT, 0) == 0;
        // the summary path's keys come out of the extraction (the guides need
        // the plain code and id arrays: the first chunk extracts those)
        const bool cm_extract = cm_path && !guides_here;
        DevBuf kA(n * 8 + 8, st), kB(n * 8 + 8, st), vA(cm_extract ? 8 : n * 4 + 4, st),
            vB(cm_path ? 8 : n * 4 + 4, st);
        // CM keys: whether a window was skipped (its key's set field is the
        // invalid id nc; see the sort below)
        DevBuf inv(cm_extract ? 4 : 0, st);
        if (cm_extract) GD_HIP(hipMemsetAsync(inv.p, 0, 4, st));
        if (nw > 0 && cm_extract) {
            if (raw8)
                extract_kernel<true, true><<<grid_for(nw, 256, 256 * 64), 256, 0, st>>>(
                    src, d_seq_off + s0, cw.as<int64_t>(), nc, nw, k, bits, strand, al, kA.as<uint64_t>(), nullptr,
                    idbits, inv.as<int>());
            else
                extract_kernel<false, true><<<grid_for(nw, 256, 256 * 64), 256, 0, st>>>(
                    src, d_seq_off + s0, cw.as<int64_t>(), nc, nw, k, bits, strand, al, kA.as<uint64_t>(), nullptr,
                    idbits, inv.as<int>());
            GD_HIP(hipGetLastError());
        } else if (nw > 0) {
            if (raw8)
                extract_kernel<true><<<grid_for(nw, 256, 256 * 64), 256, 0, st>>>(
                    src, d_seq_off + s0, cw.as<int64_t>(), nc, nw, k, bits, strand, al, kA.as<uint64_t>(),
                    vA.as<int32_t>());
            else
                extract_kernel<false><<<grid_for(nw, 256, 256 * 64), 256, 0, st>>>(
                    src, d_seq_off + s0, cw.as<int64_t>(), nc, nw, k, bits, strand, al, kA.as<uint64_t>(),
                    vA.as<int32_t>());
            GD_HIP(hipGetLastError());
        }
        tr.mark("pack: alloc+extract");
        if (guides_here)
            guide_from_extract(ctx, kA.as<uint64_t>(), vA.as<int32_t>(), hwo[nguides] * mult, nc, cbits, out);
        uint64_t* keys = kA.as<uint64_t>(); uint64_t* keys_alt = kB.as<uint64_t>();
        int32_t* ids = vA.as<int32_t>(); int32_t* ids_alt = vB.as<int32_t>();
        if (dbg) { dbg->n = n; d2h(dbg->k_extract, keys, n * 8, st); d2h(dbg->v_extract, ids, n * 4, st); }
        if (cm_path) {
            // code-major keys: the chunk's summary falls out of the same sort
            const uint64_t smask = (uint64_t(1) << idbits) - 1;
            if (n > 0 && !cm_extract) {
                pack_keys_cm_kernel<<<grid_for(n), 256, 0, st>>>(keys, ids, n, idbits, keys_alt);
                GD_HIP(hipGetLastError());
                std::swap(keys, keys_alt);
            }
            // The extraction writes each set's keys after the previous set's
            // (windows in order), so a stable radix sort on the code bits
            // alone leaves equal codes in set order: C2's 42-bit codes sort
            // in 6 passes instead of 7 for code|set. A skipped window's key
            // (set field nc) would sit inside its code's run in input order,
            // not last, so a chunk with skipped windows sorts the set bits too
            int hinv = 1;
            if (cm_extract && n > 0 && ctx->option(OPT_PACK_CODE_SORT, 1) != 0) {
                d2h(&hinv, inv.p, 4, st);
                GD_HIP(hipStreamSynchronize(st));
            }
            sort_keys_u64(ctx, keys, keys_alt, (size_t)n, hinv ? 0 : idbits, cbits + idbits);
            tr.mark("pack: sort by code|set");
            // one flag word per key: bit 0 = first key of its (code, set)
            // (valid), bit 32 = first valid key of its code; their prefix sums
            // are the unique positions (low half) and the run index (high),
            // per tile of keys (cm_count_kernel), then within the tile
            const int64_t ntile = ceil_div(n, (int64_t)kSelTile);
            DevBuf bsum(ntile * 8 + 8, st), bpre(ntile * 8 + 8, st);
            int64_t uniq = 0, nruns = 0;
            if (n > 0) {
                cm_count_kernel<<<(unsigned)ntile, kSelT, 0, st>>>(keys, n, smask, (uint64_t)nc, idbits,
                                                                    bsum.as<int64_t>());
                GD_HIP(hipGetLastError());
                exclusive_scan_i64(ctx, bsum.as<int64_t>(), bpre.as<int64_t>(), (size_t)ntile);
                int64_t last = 0, lf = 0;
                d2h(&last, bpre.as<int64_t>() + ntile - 1, 8, st);
                d2h(&lf, bsum.as<int64_t>() + ntile - 1, 8, st);
                GD_HIP(hipStreamSynchronize(st));
                uniq = (last + lf) & 0xFFFFFFFFll;
                nruns = (last + lf) >> 32;
            }
            Summary sum;
            sum.codes.alloc(nruns * 8 + 8, st);
            sum.counts.alloc(nruns * 4 + 4, st);
            sum.n = nruns;
            if (uniq > 0) {
                DevBuf start(nruns * 8 + 8, st);
                cm_select_kernel<<<(unsigned)ntile, kSelT, 0, st>>>(keys, n, smask, (uint64_t)nc, idbits,
                                                                     bpre.as<int64_t>(), keys_alt,
                                                                     sum.codes.as<uint64_t>(), start.as<int64_t>());
                GD_HIP(hipGetLastError());
                std::swap(keys, keys_alt);                      // keys: the unique code|set keys
                cm_run_counts_kernel<<<grid_for(nruns), 256, 0, st>>>(start.as<int64_t>(), nruns, uniq,
                                                                       sum.counts.as<uint32_t>());
                GD_HIP(hipGetLastError());
                // set-major: a stable sort on the set bits keeps each set's codes ascending
                sort_keys_u64(ctx, keys, keys_alt, (size_t)uniq, 0, idbits);
                GD_HIP(hipStreamSynchronize(st));
            }
            tr.mark("pack: unique+summary+by set");
            done += n;
            ensure(base + uniq, done);
            if (uniq > 0) {
                cm_codes_kernel<<<grid_for(uniq), 256, 0, st>>>(keys, uniq, idbits, all_codes.as<uint64_t>() + base);
                GD_HIP(hipGetLastError());
            }
            cm_set_offsets_kernel<<<(int)ceil_div(nc + 1, 256), 256, 0, st>>>(keys, uniq, smask, nc, base,
                                                                               d_off.as<int64_t>() + s0);
            GD_HIP(hipGetLastError());
            std::vector<int64_t> co(nc + 1);
            d2h(co.data(), d_off.as<int64_t>() + s0, (nc + 1) * sizeof(int64_t), st);
            GD_HIP(hipStreamSynchronize(st));
            GD_REQUIRE(co[nc] - base == uniq, "pack: set offsets disagree with the unique count");
            for (int i = 0; i <= nc; i++) h_off[s0 + i] = co[i];
            tr.mark("pack: codes+offsets");
            // keep the summaries only while they are much smaller than the
            // codes (shared kmers); otherwise the bitset build sorts the codes
            sum_runs += nruns;
            if (sum_runs * 4 > base + uniq) {
                want_sum = false;
                pack_sum.clear();
            } else {
                pack_sum.push_back(std::move(sum));
            }
            base += uniq;
            s0 = s1;
            continue;
        }
        sum_ok = false;                                        // a chunk without a summary
        if (!dbg && cbits + idbits <= 64 && ctx->option(OPT_PACK_SORT, 0) == 0) {
            // one sort of (set << cbits | code) keys: 8-byte records instead of two
            // 12-byte pair sorts (C2: 52-bit keys, 7 digit passes instead of 6 + 2)
            if (n > 0) {
                pack_keys_kernel<<<grid_for(n), 256, 0, st>>>(keys, ids, n, cbits, keys_alt);
                GD_HIP(hipGetLastError());
            }
            std::swap(keys, keys_alt);
            sort_keys_u64(ctx, keys, keys_alt, (size_t)n, 0, cbits + idbits);
            if (n > 0) {
                unpack_keys_kernel<<<grid_for(n), 256, 0, st>>>(keys, n, cbits, keys_alt, ids);
                GD_HIP(hipGetLastError());
            }
            std::swap(keys, keys_alt);
            tr.mark("pack: sort by set|code");
        } else {
            sort_pairs_u64_i32(ctx, keys, keys_alt, ids, ids_alt, (size_t)n, 0, std::min(64, cbits));
            if (dbg) { d2h(dbg->k_sort1, keys, n * 8, st); d2h(dbg->v_sort1, ids, n * 4, st); }
            sort_pairs_i32_u64(ctx, ids, ids_alt, keys, keys_alt, (size_t)n, idbits);
            if (dbg) { d2h(dbg->k_sort2, keys, n * 8, st); d2h(dbg->v_sort2, ids, n * 4, st); }
            tr.mark("pack: sort by code, by set");
        }

        DevBuf flag(n * 4 + 4, st), pos(n * 8 + 8, st);
        if (n > 0) {
            unique_flags_kernel<<<grid_for(n), 256, 0, st>>>(keys, ids, n, nc, flag.as<int32_t>());
            GD_HIP(hipGetLastError());
            exclusive_scan_i32_to_i64(ctx, flag.as<int32_t>(), pos.as<int64_t>(), (size_t)n);
        }
        // chunk offsets straight into the final offsets array
        set_offsets_kernel<<<(int)ceil_div(nc + 1, 256), 256, 0, st>>>(
            ids, pos.as<int64_t>(), flag.as<int32_t>(), n, nc, base, d_off.as<int64_t>() + s0);
        GD_HIP(hipGetLastError());
        std::vector<int64_t> co(nc + 1);
        d2h(co.data(), d_off.as<int64_t>() + s0, (nc + 1) * sizeof(int64_t), st);
        GD_HIP(hipStreamSynchronize(st));
        const int64_t uniq = co[nc] - base;
        done += n;
        ensure(base + uniq, done);
        if (n > 0) {
            compact_kernel<<<grid_for(n), 256, 0, st>>>(keys, flag.as<int32_t>(), pos.as<int64_t>(), n,
                                                         all_codes.as<uint64_t>() + base);
            GD_HIP(hipGetLastError());
        }
        for (int i = 0; i <= nc; i++) h_off[s0 + i] = co[i];
        tr.mark("pack: unique+compact");
        base += uniq;
        s0 = s1;
    }
    out->h_off = h_off;
    out->total = base;
    out->pack_sum.clear();
    if (want_sum && sum_ok && nseq > 0) out->pack_sum = std::move(pack_sum);
    out->off = std::move(d_off);
    if (nseq == 0) {
        out->off.alloc(sizeof(int64_t), st);
        GD_HIP(hipMemsetAsync(out->off.p, 0, sizeof(int64_t), st));
        out->h_off.assign(1, 0);
    }
    if (!all_codes.p) {                   // no window at all
        all_codes.alloc(8, st);
        all_cap = 0;
    }
    if (base < all_cap / 2 && (all_cap - base) * 8 > (int64_t(64) << 20)) {
        // mostly repeated windows: keep an exact-size copy instead of the bound
        out->codes.alloc(base * 8 + 8, st);
        if (base) GD_HIP(hipMemcpyAsync(out->codes.p, all_codes.p, base * 8, hipMemcpyDeviceToDevice, st));
    } else {
        out->codes = std::move(all_codes);
    }
    GD_HIP(hipStreamSynchronize(st));
    tr.mark("pack: codes");
}

}  // namespace gdist

// Not part of include/gdist.h: stage dump for diagnostics (tests/diag_*).
extern "C" int gdist_debug_pack_stages(gdist_ctx* ctx, int kind, int k, unsigned flags, const char* seqs,
                                       const int64_t* seq_off, int64_t nseqs, uint64_t* k_extract,
                                       int32_t* v_extract, uint64_t* k_sort1, int32_t* v_sort1, uint64_t* k_sort2,
                                       int32_t* v_sort2, gdist_sets** out) {
    using namespace gdist;
    try {
        GD_HIP(hipSetDevice(ctx->device));
        PackDebug dbg{k_extract, v_extract, k_sort1, v_sort1, k_sort2, v_sort2, 0};
        g_pack_debug = &dbg;
        std::vector<int64_t> h(seq_off, seq_off + nseqs + 1);
        DevBuf dseq(h[nseqs] + 1, ctx->stream), doff((nseqs + 1) * 8, ctx->stream);
        h2d(dseq.p, seqs, h[nseqs], ctx->stream);
        h2d(doff.p, h.data(), (nseqs + 1) * 8, ctx->stream);
        auto* s = new gdist_sets();
        s->ctx = ctx;
        pack_sets(ctx, kind, k, flags, dseq.as<char>(), doff.as<int64_t>(), h, s);
        g_pack_debug = nullptr;
        *out = s;
        return 0;
    } catch (const Error& e) {
        g_pack_debug = nullptr;
        set_last_error(e.what());
        return e.code;
    }
}
