// sparse.hip — locus order of the dense dictionary and the complement-sparse
// words of the dense tier.
//
// The dense tier holds kmers most sets share (C2: the ancestral kmers, in
// ~98 % of the genomes). A set lacks such a kmer only near its own variants,
// and a substitution removes the k consecutive windows that cover it, on both
// strands. Ranked in code order those absences are scattered over every word
// of the bitset; ranked in LOCUS order (the window position of the kmer in a
// guide sequence, strands interleaved) they fall into 1-2 words per variant.
// The dictionary rank -> bit position map is therefore a permutation that
// sorts the dense kmers by (guide, window, strand); kmers no guide holds keep
// code order at the end. Any bijection gives the same popcounts, so this
// changes only where work can be skipped, never a count.
//
// Then each 64-bit word w of the dense tier is classified by z_w, the number
// of sets whose complement word c_i[w] = ~bits_i[w] & valid(w) is non-zero:
//   * dense words (large z_w) stay bit columns for the AND+popcount tiles;
//   * sparse words contribute, per pair,
//       sum_w popc(a_w & b_w) = U_s - nc_i - nc_j + sum_{w in both lists} popc(c_i[w] & c_j[w])
//     with U_s the valid bits of the sparse words and nc_i the complement
//     bits of set i over them: only the words where BOTH sets lack something
//     cost work. Entries are grouped by (128-set block, sparse word), so a tile
//     of 128 x 128 pairs visits, per word, the few rows and columns that have
//     an entry and adds their products into LDS counters.
// C2 (1000 x 2 Mbp): 62.5 K words of which every one is sparse (z_w ~ 51 of
// 1000), 95 M products per step instead of 31 G word pairs.
#include <algorithm>
#include <map>
#include <cmath>
#include <cstring>

#include "gdist_internal.hpp"

namespace gdist {
namespace {

inline int grid_for(int64_t n, int block = 256, int64_t cap = 256 * 32) {
    int64_t g = ceil_div(n, block);
    return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

constexpr int SB = 128;                  // sets per block of the sparse entry index (tile edge)
constexpr int SNT = 512;                 // threads per workgroup (4 per CU, LDS-limited: 8 waves per SIMD)
constexpr int kBucketShift = 10;         // sparse words per complement-bit bucket: 1024

// ---- locus order -------------------------------------------------------
__global__ void locus_key_kernel(const uint64_t* __restrict__ gcodes, const uint64_t* __restrict__ gkeys, int64_t ng,
                                 const uint64_t* __restrict__ dict, int64_t U, uint64_t tag,
                                 uint64_t* __restrict__ key) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ng; g += stride) {
        const uint64_t c = gcodes[g];
        int64_t lo = 0, hi = U;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (dict[mid] < c) lo = mid + 1; else hi = mid;
        }
        if (lo < U && dict[lo] == c) key[lo] = tag | gkeys[g];   // guide codes are unique: one writer per rank
    }
}

// kmers no guide holds: after every guide key (rank tags < 2^48), ordered by
// the number of sets holding them, so the words they fill are homogeneous:
// rarely held kmers (positive-sparse words) apart from commonly held ones
// (complement-sparse words); the same on every rank (global counts)
__global__ void unkeyed_kernel(uint64_t* __restrict__ p, const uint32_t* __restrict__ cnt, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        p[i] = (0xFFull << 56) | (cnt ? (uint64_t)cnt[i] : 0xFFFFFFFFull);
}

__global__ void iota_i32_kernel(int32_t* __restrict__ p, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = (int32_t)i;
}

__global__ void min_over_ranks_kernel(const uint64_t* __restrict__ all, int64_t U, int64_t stride_r, int R,
                                      uint64_t* __restrict__ key) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < U; r += stride) {
        uint64_t m = all[r];
        for (int q = 1; q < R; q++) m = all[q * stride_r + r] < m ? all[q * stride_r + r] : m;
        key[r] = m;
    }
}

__global__ void invert_perm_kernel(const int32_t* __restrict__ order, int64_t U, uint32_t* __restrict__ perm) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < U; i += stride) perm[order[i]] = (uint32_t)i;
}

// ---- word classification ------------------------------------------------
__device__ __forceinline__ unsigned long long valid_mask(int64_t w, int64_t U) {
    const int64_t full = U >> 6;
    if (w < full) return ~0ull;
    if (w == full && (U & 63)) return (1ull << (U & 63)) - 1ull;
    return 0ull;
}

// z[w] += sets of this block of rows whose complement word is non-zero,
// zp[w] += sets whose word is non-zero
__global__ __launch_bounds__(256) void word_z_kernel(const unsigned long long* __restrict__ bits, int64_t N, int64_t W,
                                                     int64_t U, int64_t rows_per_block, int32_t* __restrict__ z,
                                                     int32_t* __restrict__ zp) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t i0 = (int64_t)blockIdx.y * rows_per_block;
    const int64_t i1 = i0 + rows_per_block < N ? i0 + rows_per_block : N;
    if (w >= W) return;
    const unsigned long long m = valid_mask(w, U);
    int c = 0, p = 0;
    for (int64_t i = i0; i < i1; i++) {
        const unsigned long long b = bits[i * W + w] & m;
        c += b != m;
        p += b != 0;
    }
    if (c) atomicAdd(z + w, c);
    if (p) atomicAdd(zp + w, p);
}

__global__ void gather_words_kernel(const unsigned long long* __restrict__ bits, int64_t W,
                                    const int32_t* __restrict__ dw, int64_t Wd, int64_t Wdp, int64_t N,
                                    unsigned long long* __restrict__ out) {
    const int64_t n = N * Wdp;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
        const int64_t i = e / Wdp, d = e - i * Wdp;
        out[e] = d < Wd ? bits[i * W + dw[d]] : 0ull;
    }
}

// the entry word of set word b: the complement (complement-sparse words) or
// the word itself (positive-sparse words: few sets hold any of its kmers)
__device__ __forceinline__ unsigned long long entry_word(unsigned long long b, unsigned long long m, bool pos) {
    return pos ? (b & m) : (~b & m);
}

// Group tier (below): a factorised word s keeps of each grouped set only
// the residual, the bits of its entry word outside its group's pattern
constexpr int kGroupMax = 64;                    // groups (disjoint sets of sets) per collection
struct GroupWords {
    const int32_t* grp = nullptr;               // [N] group of each set, -1: none
    const int32_t* prow = nullptr;              // [Ws] pattern row of sparse word s (| kRowLack), -1: not factorised
    const unsigned long long* pats = nullptr;   // [rows][m] each group's pattern in the word
    int m = 0;                                  // groups
    int32_t* V = nullptr;                       // [m][N] group x set part (filled with the entries)
    int64_t N = 0;
};
constexpr int32_t kRowLack = 1 << 30;           // pattern row flag: the word's residuals are the lacked bits
__device__ __forceinline__ unsigned long long residual(unsigned long long e, const GroupWords& gw, int r, int64_t i) {
    if (r < 0) return e;
    const int g = gw.grp[i];
    if (g < 0) return e;                        // (0 in a lacked-mode word)
    const unsigned long long P = gw.pats[(int64_t)(r & ~kRowLack) * gw.m + g];
    return (r & kRowLack) ? (P & ~e) : (e & ~P);
}

// entries per (block b, sparse word s): sets of the block whose (residual) entry word is non-zero
__global__ __launch_bounds__(256) void sparse_count_kernel(const unsigned long long* __restrict__ bits, int64_t N,
                                                           int64_t W, int64_t U, const int32_t* __restrict__ sw,
                                                           const uint8_t* __restrict__ spos, int64_t Ws,
                                                           GroupWords gw, int32_t* __restrict__ cnt) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t b = blockIdx.y;
    if (s >= Ws) return;
    const int64_t w = sw[s];
    const bool pos = spos[s] != 0;
    const unsigned long long m = valid_mask(w, U);
    const int r = gw.prow ? gw.prow[s] : -1;
    const int64_t i1 = (b + 1) * SB < N ? (b + 1) * SB : N;
    int c = 0;
    for (int64_t i = b * SB; i < i1; i++) c += residual(entry_word(bits[i * W + w], m, pos), gw, r, i) != 0;
    cnt[b * Ws + s] = c;
}

__global__ __launch_bounds__(256) void sparse_fill_kernel(const unsigned long long* __restrict__ bits, int64_t N,
                                                          int64_t W, int64_t U, const int32_t* __restrict__ sw,
                                                          const uint8_t* __restrict__ spos,
                                                          int64_t Ws, GroupWords gw, const int64_t* __restrict__ off,
                                                          unsigned long long* __restrict__ word,
                                                          uint8_t* __restrict__ set, int32_t* __restrict__ nc,
                                                          int32_t* __restrict__ bucket_bits, int64_t nbk) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t b = blockIdx.y;
    if (s >= Ws) return;
    const int64_t w = sw[s];
    const bool pos = spos[s] != 0;
    const unsigned long long m = valid_mask(w, U);
    const int r = gw.prow ? gw.prow[s] : -1;
    const int64_t i1 = (b + 1) * SB < N ? (b + 1) * SB : N;
    int64_t p = off[b * Ws + s];
    for (int64_t i = b * SB; i < i1; i++) {
        const unsigned long long e = entry_word(bits[i * W + w], m, pos);
        // constant part: the complement words' WHOLE complement bits
        if (!pos && e) atomicAdd(nc + i, (int32_t)__popcll(e));
        const unsigned long long c = residual(e, gw, r, i);
        if (c) {
            word[p] = c;
            set[p] = (uint8_t)(i - b * SB);
            p++;
            atomicAdd(bucket_bits + i * nbk + (s >> kBucketShift), (int32_t)__popcll(c));
            if (r >= 0) {                  // V[G][i] += popc(P_G & a_i), -= popc(P_G & b_i) (group tier)
                const unsigned long long* P = gw.pats + (int64_t)(r & ~kRowLack) * gw.m;
                const int sg = (r & kRowLack) ? -1 : 1;
                for (int g = 0; g < gw.m; g++) {
                    const int v = __popcll(P[g] & c);
                    if (v) atomicAdd(gw.V + (int64_t)g * gw.N + i, sg * v);
                }
            }
        }
    }
}

// ---- group tier -----------------------------------------------------------
// Structured collections (clades: C2-realistic) hold words whose entry word
// carries, in every member of a group of sets, that group's pattern (the
// clade's variant lacked, or held, by all its members), plus each set's own
// few bits. The groups partition (part of) the sets. In a factorised word,
// group G's pattern P_G is the AND of its members' entry words, so a member's
// e_i = P_G ∪ a_i with P_G ∩ a_i = ∅ (a_i, the residual) and an ungrouped
// set has P = ∅, a_i = e_i. Per pair the four parts are disjoint:
//   popc(e_i & e_j) = popc(P_gi & P_gj) + popc(P_gi & a_j) + popc(a_i & P_gj) + popc(a_i & a_j)
// Summed over the factorised words:
//   T[G][H] = Σ_w popc(P_G & P_H),  V[G][j] = Σ_w popc(P_G & a_j)  (0 for members of G)
//   X[i][j] = T[gi][gj] + V[gi][j] + V[gj][i]
// and the residuals are ordinary sparse entries; the reduce / flush adds
// X[i][j] (int32, [N][N]). Lacked mode, for words whose members mostly
// hold the group's bits (a clade's variant kmers on the positive side, where
// one member's own substitution would drop a bit from the AND): P_G is the OR
// of the members' entry words and the residual is b_i = P_G \ e_i, so
//   popc(e_i & e_j) = popc(P_gi & P_gj) - popc(P_gi & b_j) - popc(b_i & P_gj) + popc(b_i & b_j)
// (the V terms enter with a minus; allowed only when no ungrouped set has an
// entry in the word). Any choice of groups is exact; the choice only decides
// how much work leaves the products. Groups are found from the data: per heavy word, the most
// frequent non-zero entry value v and its members {i : e_i ⊇ v}; member
// lists recurring over many words (hash of the bitmap) are taken greedily,
// most words first, keeping them disjoint.
constexpr int kGroupSample = 4096;               // sets sampled for a word's modal entry value
constexpr int kGroupMinSize = 16;                // smallest group worth a pattern
constexpr int kGroupMinWords = 8;                // ... and the fewest words it must recur in
constexpr int kGroupMinZ = 32;                   // candidate words: at least this many entries
constexpr int64_t kGroupMaxN = 16384;            // discovery keeps an N-bit member bitmap per heavy word

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Per candidate word c: the most frequent non-zero entry value v among the
// first kGroupSample sets (bitonic sort in LDS, longest run), then its
// members {i : e_i ⊇ v} over all sets as a bitmap, their number and a hash
// of the bitmap.
__global__ __launch_bounds__(256) void group_modal_kernel(const unsigned long long* __restrict__ bits, int64_t N,
                                                          int64_t W, int64_t U, const int32_t* __restrict__ cw,
                                                          const uint8_t* __restrict__ cpos, int64_t nwb,
                                                          unsigned long long* __restrict__ mbits,
                                                          int32_t* __restrict__ msize,
                                                          unsigned long long* __restrict__ mhash) {
    __shared__ unsigned long long v[kGroupSample];
    __shared__ unsigned long long rv[256];
    __shared__ int rn[256];
    const int64_t c = blockIdx.x;
    const int64_t w = cw[c];
    const bool pos = cpos[c] != 0;
    const unsigned long long m = valid_mask(w, U);
    const int n = (int)(N < kGroupSample ? N : kGroupSample);
    int np = 1;
    while (np < n) np <<= 1;
    for (int t = threadIdx.x; t < np; t += 256) v[t] = t < n ? entry_word(bits[(int64_t)t * W + w], m, pos) : ~0ull;
    __syncthreads();
    for (int k = 2; k <= np; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = threadIdx.x; t < np; t += 256) {
                const int x = t ^ j;
                if (x > t) {
                    const unsigned long long a = v[t], b = v[x];
                    if ((a > b) == ((t & k) == 0)) { v[t] = b; v[x] = a; }
                }
            }
            __syncthreads();
        }
    int bn = 0;
    unsigned long long bv = 0;
    for (int p = threadIdx.x; p < n; p += 256) {
        const unsigned long long x = v[p];
        if (x == 0 || (p > 0 && v[p - 1] == x)) continue;
        int e = p + 1;
        while (e < n && v[e] == x) e++;
        if (e - p > bn || (e - p == bn && x < bv)) { bn = e - p; bv = x; }
    }
    rv[threadIdx.x] = bv;
    rn[threadIdx.x] = bn;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            const int a = rn[threadIdx.x], b = rn[threadIdx.x + o];
            const unsigned long long x = rv[threadIdx.x], y = rv[threadIdx.x + o];
            if (b > a || (b == a && y < x)) { rn[threadIdx.x] = b; rv[threadIdx.x] = y; }
        }
        __syncthreads();
    }
    const unsigned long long v0 = rn[0] >= 2 ? rv[0] : 0ull;
    __syncthreads();
    int cnt = 0;
    unsigned long long h = 0;
    for (int64_t q = threadIdx.x; q < nwb; q += 256) {
        unsigned long long word = 0;
        for (int b = 0; b < 64; b++) {
            const int64_t i = q * 64 + b;
            if (i >= N) break;
            const unsigned long long e = entry_word(bits[i * W + w], m, pos);
            if (v0 && (e & v0) == v0) word |= 1ull << b;
        }
        mbits[c * nwb + q] = word;
        cnt += __popcll(word);
        h += mix64(word ^ (0x632BE59BD9B4E019ull * (unsigned long long)(q + 1)));
    }
    rn[threadIdx.x] = cnt;
    rv[threadIdx.x] = h;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) { rn[threadIdx.x] += rn[threadIdx.x + o]; rv[threadIdx.x] += rv[threadIdx.x + o]; }
        __syncthreads();
    }
    if (threadIdx.x == 0) { msize[c] = v0 ? rn[0] : 0; mhash[c] = rv[0]; }
}

// Every group's patterns in candidate word c (AND and OR of its members'
// entry words, LDS atomics) and the word's residual entry count in either mode
__global__ __launch_bounds__(256) void group_pattern_kernel(const unsigned long long* __restrict__ bits, int64_t N,
                                                            int64_t W, int64_t U, const int32_t* __restrict__ cw,
                                                            const uint8_t* __restrict__ cpos,
                                                            const int32_t* __restrict__ grp, int mg,
                                                            unsigned long long* __restrict__ cpat,
                                                            int32_t* __restrict__ zres) {
    __shared__ unsigned long long pat[kGroupMax], por[kGroupMax];
    __shared__ int rz[256], ro[256];
    const int64_t c = blockIdx.x;
    const int64_t w = cw[c];
    const bool pos = cpos[c] != 0;
    const unsigned long long m = valid_mask(w, U);
    for (int g = threadIdx.x; g < mg; g += 256) { pat[g] = ~0ull; por[g] = 0ull; }
    __syncthreads();
    for (int64_t i = threadIdx.x; i < N; i += 256) {
        const int g = grp[i];
        const unsigned long long e = entry_word(bits[i * W + w], m, pos);
        if (g >= 0) { atomicAnd(&pat[g], e); if (e) atomicOr(&por[g], e); }
    }
    __syncthreads();
    int z = 0, zo = 0;
    for (int64_t i = threadIdx.x; i < N; i += 256) {
        const int g = grp[i];
        const unsigned long long e = entry_word(bits[i * W + w], m, pos);
        z += (g >= 0 ? (e & ~pat[g]) : e) != 0;
        zo += g >= 0 ? ((por[g] & ~e) != 0) : (e ? 1 << 20 : 0);     // an ungrouped entry rules lacked mode out
    }
    rz[threadIdx.x] = z;
    ro[threadIdx.x] = zo;
    for (int g = threadIdx.x; g < mg; g += 256) {
        cpat[(2 * c) * mg + g] = pat[g];
        cpat[(2 * c + 1) * mg + g] = por[g];
    }
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            rz[threadIdx.x] += rz[threadIdx.x + o];
            ro[threadIdx.x] = min(ro[threadIdx.x] + ro[threadIdx.x + o], 1 << 20);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) { zres[2 * c] = rz[0]; zres[2 * c + 1] = ro[0]; }
}

// T[G][H] += popc(P_G & P_H) per factorised word (pattern row r)
__global__ void group_t_kernel(const unsigned long long* __restrict__ pats, int64_t rows, int mg,
                               int32_t* __restrict__ T) {
    const int64_t r = blockIdx.x;
    if (r >= rows) return;
    for (int e = threadIdx.x; e < mg * mg; e += blockDim.x) {
        const int G = e / mg, H = e - G * mg;
        const int v = __popcll(pats[r * mg + G] & pats[r * mg + H]);
        if (v) atomicAdd(T + e, v);
    }
}

// The group part of pair (i, j): T[gi][gj] + V[gi][j] + V[gj][i] (0 without
// groups), evaluated per pair by the tile kernel's flush and the chunk
// reduce from the small tables
struct GroupPart {
    const int32_t* grp = nullptr;               // [N] group of each set, -1: none (null: no group tier)
    const int32_t* V = nullptr;                 // [m][N]
    const int32_t* T = nullptr;                 // [m][m]
    int m = 0;
    int64_t N = 0;
    __device__ __forceinline__ int at(int64_t i, int64_t j) const {
        if (!grp) return 0;
        const int gi = grp[i], gj = grp[j];
        int x = 0;
        if (gi >= 0) x += V[(int64_t)gi * N + j];
        if (gj >= 0) x += V[(int64_t)gj * N + i];
        if (gi >= 0 && gj >= 0) x += T[gi * m + gj];
        return x;
    }
};

// LDS counter of local pair (row a, column b), as a 16-bit slot t (dword
// t >> 1, half t & 1): row a owns dwords [64 a, 64 a + 64); column b sits in
// dword (b >> 1) ^ (a & 63) of it, half b & 1. The XOR rotation by the row
// spreads the products of one word (its rows x its columns) over the banks.
// The records carry the two halves of the address precomputed (entry_codes):
// a row entry's byte base with its rotation key, a column entry's byte offset
// and half shift, so a product's counter costs one XOR and one shift.
__host__ __device__ __forceinline__ int cnt_index(int a, int b) {
    return ((a * 64 + ((b >> 1) ^ (a & 63))) << 1) | (b & 1);
}
__host__ __device__ __forceinline__ void cnt_pair(int t, int& a, int& b) {
    const int d = t >> 1;
    a = d >> 6;
    b = (((d & 63) ^ (a & 63)) << 1) | (t & 1);
}
// record codes of set s (0..127): row role = byte address of its row with the
// rotation key in bits 2-7 (row bytes 256 s, keys < 256); column role = shift
// (s & 1) << 4 in bits 0-4 and its dword's byte offset (s >> 1) << 2 in bits 16+
__host__ __device__ __forceinline__ uint32_t row_code(int s) { return ((uint32_t)s << 8) | ((uint32_t)(s & 63) << 2); }
__host__ __device__ __forceinline__ uint32_t col_code(int s) {
    return ((uint32_t)(s & 1) << 4) | (((uint32_t)(s >> 1) << 2) << 16);
}
constexpr uint32_t kLastOfList = 32;     // column code bit 5 (above the shift, below the offset): the entry ends its (block, word) list
constexpr int kSentinelRecs = 512;       // zero records after the entries (the virtual word's)
// the counter add of a product of row code r and column code c (byte address r ^ c >> 16)
__device__ __forceinline__ void cnt_add(uint32_t* cnt, uint32_t r, uint32_t c, uint32_t v) {
    atomicAdd(reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(cnt) + (r ^ (c >> 16))), v << (c & 31));
}

// 16-byte records of the entries (E16 / v5 / v6 tile kernels), as four
// dwords {row_code(set), word lo, word hi, col_code(set)}: a row needs the
// first 12 bytes, a column the last 12, so v6 loads 12 per entry
// (global_load_dwordx3) instead of 16
struct Rec3 {
    uint32_t a, b, c;
};
__device__ __forceinline__ unsigned long long rec_word(const ulonglong2& r) { return (r.x >> 32) | (r.y << 32); }
__device__ __forceinline__ uint32_t rec_row(const ulonglong2& r) { return (uint32_t)r.x; }
__device__ __forceinline__ uint32_t rec_col(const ulonglong2& r) { return (uint32_t)(r.y >> 32); }
__global__ void sparse_records_kernel(const unsigned long long* __restrict__ word, const uint8_t* __restrict__ set,
                                      int64_t n, ulonglong2* __restrict__ ent) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
        const int st = set[e];
        const unsigned long long w = word[e];
        ent[e] = make_ulonglong2((unsigned long long)row_code(st) | (w << 32),
                                 (w >> 32) | ((unsigned long long)col_code(st) << 32));
    }
}

// column code bit 5 of each (block, word) list's last entry (the walk's
// second column of an odd list's last pair is then dropped)
__global__ void sparse_last_kernel(const int64_t* __restrict__ off, int64_t nlists, ulonglong2* __restrict__ ent) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nlists; t += stride) {
        const int64_t b = off[t], e = off[t + 1];
        if (e > b) ent[e - 1].y |= (unsigned long long)kLastOfList << 32;
    }
}

// the rare tier's set -> list CSR (bitset.hip build_postings), walked in every step
struct RareRows {
    const int64_t* soff = nullptr;        // [N + 1] (null: no walk)
    const uint64_t* sent = nullptr;       // (list start << 24 | list length) per (set, list) record
    const uint32_t* sw = nullptr;         // the list's weight
    const uint16_t* sskip = nullptr;      // 1 + the set's position in its list (0: none)
    const uint32_t* psets = nullptr;      // list members, ascending
};
inline RareRows rare_rows_of(const gdist_sets* s) {
    return RareRows{s->srare_off.as<int64_t>(), s->srare_ent.as<uint64_t>(), s->srare_w.as<uint32_t>(),
                    s->srare_skip.as<uint16_t>(), s->post_sets.as<uint32_t>()};
}

// The rare tier's pairs, recounted in every step by workgroups of the tile
// launch itself (its last nrare workgroups; no per-pair state survives
// between steps, no extra launch, no second stream): one workgroup per (row
// i, chunk of 8192 columns) walks the row's (set, list) records, adds each
// list member in the chunk (upper triangle: from the row's own position on,
// members after i) into LDS counters, and STORES the row into every tile
// slab of the region's tiles it meets (kRareSlab layout = cnt_index, 0 where
// no rare kmer is shared), so the chunk reduce adds them coalesced. These
// latency-bound walks run beside the tile workgroups of the same launch.
constexpr int kRareChunkCols = SB * SB / 2;       // the tile kernel's 32 KiB of LDS counters, one per column
struct RareSlab {
    RareRows rr;
    int nrare = 0;                        // trailing workgroups doing rare rows (0: none)
    int nch = 1;                          // column chunks per row
    uint32_t* slab = nullptr;             // uint32 [ntiles][128 x 128]
    const int32_t* tile_of = nullptr;     // [row blocks of the region][column blocks]: tile index or -1
    int64_t ab0 = 0, nbc = 0;             // first row block of the region, column blocks
};
__device__ __forceinline__ void rare_slab_row(const RareSlab& rs, int unit, int64_t r0, int64_t c0, int64_t c1,
                                              int upper, uint32_t* __restrict__ cnt) {
    const int64_t i = r0 + unit / rs.nch;
    const int64_t cb = c0 + (int64_t)(unit % rs.nch) * kRareChunkCols;
    const int64_t ce = cb + kRareChunkCols < c1 ? cb + kRareChunkCols : c1;
    const int n = (int)(ce - cb);
    for (int t = threadIdx.x; t < n; t += SNT) cnt[t] = 0;
    __syncthreads();
    const int64_t xb = rs.rr.soff[i], xe = rs.rr.soff[i + 1];
    for (int64_t x = xb + threadIdx.x; x < xe; x += SNT) {
        const uint64_t ent = rs.rr.sent[x];
        const uint32_t w = rs.rr.sw[x];
        const int64_t b0 = (int64_t)(ent >> 24), e = b0 + (int64_t)(ent & 0xFFFFFFu);
        const int sk = upper ? (int)rs.rr.sskip[x] : 0;
        for (int64_t y = b0 + sk; y < e; y++) {
            const int64_t t = rs.rr.psets[y];
            if (t >= ce) break;                                     // members ascend
            if (t < cb || t == i || (upper && t < i)) continue;     // (skip 0: from the list's start)
            atomicAdd(&cnt[t - cb], w);
        }
    }
    __syncthreads();
    // the row's slots of every tile it meets: 128 columns per column block
    const int64_t A = i / SB;
    const int a = (int)(i - A * SB);
    const int64_t B0 = cb / SB, B1 = (ce - 1) / SB;
    for (int64_t e = threadIdx.x; e < (B1 - B0 + 1) * SB; e += SNT) {
        const int64_t B = B0 + e / SB;
        const int b = (int)(e % SB);
        const int32_t tl = rs.tile_of[(A - rs.ab0) * rs.nbc + B];
        if (tl < 0) continue;
        const int64_t j = B * SB + b;
        // a block straddling two chunks gets each column from its own chunk;
        // slots outside the region are never read by the reduce
        if (j < cb || j >= ce) continue;
        rs.slab[(int64_t)tl * (SB * SB) + cnt_index(a, b)] = cnt[j - cb];
    }
}

// ---- the sparse tile kernel ---------------------------------------------
// One workgroup per (128 x 128 tile of absolute set blocks (A, B), chunk of
// the sparse words). Each wave takes 64 sparse words at a time: lane l loads
// the (A, s) and (B, s) entry ranges of word s = base + l, the wave
// prefix-sums the word's product slots, parks the walk fields in LDS, and the
// 64 lanes then walk the flattened slots, SUN per lane in flight so their
// loads overlap, adding popc(c_i & c_j) to LDS counters. A diagonal tile
// (A == B) walks each word's pairs x < y of its one entry list (mirrored
// when the region is not an upper triangle). With one chunk per tile the
// counters go to I directly (atomics) with the constant part
// U_s - nc_i - nc_j; with several, each chunk stores its counters to `part`
// and sparse_reduce_kernel sums them.
//
// The instruction stream per slot (round 4; ~26 VALU per 1 x 2 slot, r3: ~47):
//   * the walk records of a batch's words sit in LDS in slot order, words
//     without slots left out, so the word of slot f is the number of words
//     whose last slot is below f: per group of 64 slots one ballot counts the
//     words ending before the group and a 64-bit mask of the last slots inside
//     it (built per window of kWinGroups groups with LDS ORs) gives the rest
//     through mbcnt — two VALU per slot instead of a ballot + readlane search;
//   * an off-diagonal slot is a 1 x 2 micro-tile: one row entry and a PAIR of
//     adjacent column entries of one word; the row is q / ncp by a float
//     reciprocal whose low 8 mantissa bits carry 2 ncp (exact: the quotient
//     (2q + 1) / (2 ncp) stays >= 1/128 from an integer, the packed
//     reciprocal's error is < 2^-15 relative; checked exhaustively), and the
//     record offsets are byte offsets, so a slot's quotient and both load
//     addresses are eight VALU;
//   * an odd column list's last pair reads the next record as its second
//     column: that record's product is dropped by the FIRST column's
//     last-of-list flag (column code bit 5, set at build time), not by a
//     compare against the list length;
//   * slots past the batch's last word fall on a virtual word whose records
//     are zero (the sentinel run after the entries), so no slot is masked;
//   * an entry is one 16-byte record {row code, word, column code}: a row
//     loads its first 12 bytes, a column its last 12 (global_load_dwordx3);
//   * the counter add is unconditional (a zero product adds 0).
// Counters are 16-bit, two to an LDS dword: a chunk holds at most kChunkWords
// sparse words, so a pair's count in one chunk is at most 64 x 1023 < 2^16
// and a packed ds_add_u32 never carries into the neighbour (32 KiB per tile)
constexpr int kChunkWords = 1023;
// dense words per in-kernel fold slab: a pair gains at most 64 x 8 in the
// chunk that folds a slab, so such chunks hold at most kChunkWords -
// kFoldSlabWords sparse words
constexpr int kFoldSlabWords = 8;
constexpr int SNW = SNT / 64;
// a wave's LDS (1 KiB of the 8 KiB record area): kBatchWords walk records +
// the virtual word's, then the window's last-slot masks
constexpr int kBatchWords = 48;
constexpr int kWinGroups = 16;
static_assert((kBatchWords + 1) * 16 + kWinGroups * 8 <= 1024 - 16, "a wave's walk LDS (its last 16 bytes spare: wave 0's hold the batch counter)");

struct SparseWalk {
    const char* eA;                       // the chunk's row-side records (bytes)
    const char* eB;                       // ... and column-side records
};

// the word (compacted record index) of slot gb + lane: words ending before
// the group + last slots of the group below this lane
__device__ __forceinline__ int slot_rec(int last, int gb, unsigned long long m) {
    const int before = __popcll(__ballot(last < gb));
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, (uint32_t)before));
}

// Diagonal tiles: slot q of a word is its pair (y, x), y < x, q = x(x-1)/2 +
// y; rec = {-first slot, row start (entries), -, -}
template <int SU>
__device__ __forceinline__ void sparse_diag_slots(const int4* __restrict__ rec,
                                                  const unsigned long long* __restrict__ masks, int W0, int last,
                                                  int fb, int lane, const SparseWalk& e, uint32_t* __restrict__ cnt,
                                                  bool mirror) {
    int4 r[SU];
    unsigned long long m[SU];
    const unsigned long long* mk = masks + ((fb - W0) >> 6);
#pragma unroll
    for (int u = 0; u < SU; u++) m[u] = mk[u];
#pragma unroll
    for (int u = 0; u < SU; u++) r[u] = rec[slot_rec(last, fb + 64 * u, m[u])];
    uint32_t ri[SU], ci[SU];
#pragma unroll
    for (int u = 0; u < SU; u++) {
        const int q = fb + 64 * u + lane + r[u].x;
        int x = (int)((1.0f + __builtin_amdgcn_sqrtf(1.0f + 8.0f * (float)q)) * 0.5f);
        const int t = (int)(__umul24(x, x - 1) >> 1);
        // x -= 1 when t > q, x += 1 when (x + 1) x / 2 <= q: arithmetic, not branches
        const int dn = (int)(t > q), up = (int)(t + x <= q);
        const int xc = x + up - dn;
        const int tc = t + __mul24(up, x) - __mul24(dn, x - 1);
        ri[u] = (uint32_t)(r[u].y + (q - tc)) << 4;
        ci[u] = (uint32_t)(r[u].y + xc) << 4;
    }
    ulonglong2 a[SU], b[SU];
#pragma unroll
    for (int u = 0; u < SU; u++) {
        a[u] = *reinterpret_cast<const ulonglong2*>(e.eA + ri[u]);
        b[u] = *reinterpret_cast<const ulonglong2*>(e.eA + ci[u]);
    }
#pragma unroll
    for (int u = 0; u < SU; u++) {
        const uint32_t v = (uint32_t)__popcll(rec_word(a[u]) & rec_word(b[u]));
        cnt_add(cnt, rec_row(a[u]), rec_col(b[u]), v);
        if (mirror) cnt_add(cnt, rec_row(b[u]), rec_col(a[u]), v);
    }
}

// Off-diagonal tiles: 1 x 2 micro-tiles, ncp = ceil(ncol / 2) slots per row
// entry; rec = {-2 first slot, row start (bytes), column start (bytes),
// 1 / (2 ncp) with 2 ncp in its low byte}
template <int SU>
__device__ __forceinline__ void sparse_off_slots(const int4* __restrict__ rec,
                                                 const unsigned long long* __restrict__ masks, int W0, int last,
                                                 int fb, int lane, const SparseWalk& e, uint32_t* __restrict__ cnt) {
    int4 r[SU];
    unsigned long long m[SU];
    const unsigned long long* mk = masks + ((fb - W0) >> 6);
#pragma unroll
    for (int u = 0; u < SU; u++) m[u] = mk[u];
#pragma unroll
    for (int u = 0; u < SU; u++) r[u] = rec[slot_rec(last, fb + 64 * u, m[u])];
    uint32_t ri[SU], ci[SU];
#pragma unroll
    for (int u = 0; u < SU; u++) {
        const int q2 = 2 * (fb + 64 * u) + 2 * lane + r[u].x;
        const float rcp = __int_as_float(r[u].w);
        const int xc = (int)__builtin_fmaf((float)q2, rcp, rcp);
        const int yc2 = q2 - (int)__umul24((uint32_t)xc, (uint32_t)r[u].w & 0xFFu);
        ri[u] = (uint32_t)r[u].y + ((uint32_t)xc << 4);
        ci[u] = (uint32_t)r[u].z + ((uint32_t)yc2 << 4);
    }
    Rec3 a[SU], b0[SU], b1[SU];                   // row {row code, word}, columns {word, column code}
#pragma unroll
    for (int u = 0; u < SU; u++) {
        const char* pb = e.eB + ci[u] + 4;
        a[u] = *reinterpret_cast<const Rec3*>(e.eA + ri[u]);
        b0[u] = *reinterpret_cast<const Rec3*>(pb);
        b1[u] = *reinterpret_cast<const Rec3*>(pb + 16);
    }
#pragma unroll
    for (int u = 0; u < SU; u++) {
        const uint32_t rc = a[u].a;
        const uint32_t v0 = (uint32_t)(__popc(a[u].b & b0[u].a) + __popc(a[u].c & b0[u].b));
        uint32_t v1 = (uint32_t)(__popc(a[u].b & b1[u].a) + __popc(a[u].c & b1[u].b));
        v1 &= ~(uint32_t)__builtin_amdgcn_sbfe((int)b0[u].c, 5, 1);      // kLastOfList: bit 5
        cnt_add(cnt, rc, b0[u].c, v0);
        cnt_add(cnt, rc, b1[u].c, v1);
    }
}

// Off-diagonal 2 x 2 micro-tiles (option sparse_mt 2): ceil(nrow / 2) row
// pairs x ncp column pairs per word, the same records and quotient as above
// with the row pair's byte offset at xc << 5. Four products a slot from four
// record loads (1 x 2: two from three), so the walk issues a third fewer
// scattered loads per product (the texture address unit is its busiest unit:
// TA ~63 % busy, VALU ~28 % of its issue rate, profiles/r04/s13). The row
// pair's second row past an odd list is the next record: its products are
// dropped by the first row's last-of-list flag (the column code, read with
// the first row's 16 bytes). Not for row-trimmed tiles (rpart: a trimmed
// list's last row is not its list's last).
template <int SU>
__device__ __forceinline__ void sparse_off22_slots(const int4* __restrict__ rec,
                                                   const unsigned long long* __restrict__ masks, int W0, int last,
                                                   int fb, int lane, const SparseWalk& e, uint32_t* __restrict__ cnt) {
    int4 r[SU];
    unsigned long long m[SU];
    const unsigned long long* mk = masks + ((fb - W0) >> 6);
#pragma unroll
    for (int u = 0; u < SU; u++) m[u] = mk[u];
#pragma unroll
    for (int u = 0; u < SU; u++) r[u] = rec[slot_rec(last, fb + 64 * u, m[u])];
    uint32_t ri[SU], ci[SU];
#pragma unroll
    for (int u = 0; u < SU; u++) {
        const int q2 = 2 * (fb + 64 * u) + 2 * lane + r[u].x;
        const float rcp = __int_as_float(r[u].w);
        const int xc = (int)__builtin_fmaf((float)q2, rcp, rcp);
        const int yc2 = q2 - (int)__umul24((uint32_t)xc, (uint32_t)r[u].w & 0xFFu);
        ri[u] = (uint32_t)r[u].y + ((uint32_t)xc << 5);
        ci[u] = (uint32_t)r[u].z + ((uint32_t)yc2 << 4);
    }
    uint4 a0[SU];
    Rec3 a1[SU], b0[SU], b1[SU];                   // rows {row code, word (, column code)}, columns {word, column code}
#pragma unroll
    for (int u = 0; u < SU; u++) {
        const char* pa = e.eA + ri[u];
        const char* pb = e.eB + ci[u] + 4;
        a0[u] = *reinterpret_cast<const uint4*>(pa);
        a1[u] = *reinterpret_cast<const Rec3*>(pa + 16);
        b0[u] = *reinterpret_cast<const Rec3*>(pb);
        b1[u] = *reinterpret_cast<const Rec3*>(pb + 16);
    }
#pragma unroll
    for (int u = 0; u < SU; u++) {
        const uint32_t la = ~(uint32_t)__builtin_amdgcn_sbfe((int)a0[u].w, 5, 1);    // kLastOfList: bit 5
        const uint32_t lb = ~(uint32_t)__builtin_amdgcn_sbfe((int)b0[u].c, 5, 1);
        const uint32_t v00 = (uint32_t)(__popc(a0[u].y & b0[u].a) + __popc(a0[u].z & b0[u].b));
        const uint32_t v01 = (uint32_t)(__popc(a0[u].y & b1[u].a) + __popc(a0[u].z & b1[u].b)) & lb;
        const uint32_t v10 = (uint32_t)(__popc(a1[u].b & b0[u].a) + __popc(a1[u].c & b0[u].b)) & la;
        const uint32_t v11 = (uint32_t)(__popc(a1[u].b & b1[u].a) + __popc(a1[u].c & b1[u].b)) & (la & lb);
        cnt_add(cnt, a0[u].x, b0[u].c, v00);
        cnt_add(cnt, a0[u].x, b1[u].c, v01);
        cnt_add(cnt, a1[u].a, b0[u].c, v10);
        cnt_add(cnt, a1[u].a, b1[u].c, v11);
    }
}

// Diagonal tiles in 2 x 2 micro-tiles (with sparse_mt 2): the word's n
// entries as m = ceil(n / 2) pairs; slot q is the pair of pairs (Y, X), Y <=
// X, q = X (X + 1) / 2 + Y. X > Y: all four products are pairs y < x (the
// column pair's second entry past an odd list dropped by the first's
// last-of-list flag); X == Y: only (2Y, 2Y + 1). Three products a slot on
// average instead of one, from four loads instead of two; rec as
// sparse_diag_slots.
template <int SU>
__device__ __forceinline__ void sparse_diag22_slots(const int4* __restrict__ rec,
                                                    const unsigned long long* __restrict__ masks, int W0, int last,
                                                    int fb, int lane, const SparseWalk& e, uint32_t* __restrict__ cnt,
                                                    bool mirror) {
    int4 r[SU];
    unsigned long long m[SU];
    const unsigned long long* mk = masks + ((fb - W0) >> 6);
#pragma unroll
    for (int u = 0; u < SU; u++) m[u] = mk[u];
#pragma unroll
    for (int u = 0; u < SU; u++) r[u] = rec[slot_rec(last, fb + 64 * u, m[u])];
    uint32_t ri[SU], ci[SU], ne[SU];
#pragma unroll
    for (int u = 0; u < SU; u++) {
        const int q = fb + 64 * u + lane + r[u].x;
        int x = (int)((__builtin_amdgcn_sqrtf(1.0f + 8.0f * (float)q) - 1.0f) * 0.5f);
        const int t = (int)(__umul24(x, x + 1) >> 1);
        // x -= 1 when t > q, x += 1 when (x + 1)(x + 2) / 2 <= q
        const int dn = (int)(t > q), up = (int)(t + x + 1 <= q);
        const int xc = x + up - dn;
        const int tc = t + __mul24(up, x + 1) - __mul24(dn, x);
        const int yc = q - tc;
        ri[u] = (uint32_t)(r[u].y + 2 * yc) << 4;
        ci[u] = (uint32_t)(r[u].y + 2 * xc) << 4;
        ne[u] = xc != yc ? ~0u : 0u;
    }
    uint4 a0[SU], a1[SU], b0[SU], b1[SU];         // {row code, word lo, word hi, column code}
#pragma unroll
    for (int u = 0; u < SU; u++) {
        a0[u] = *reinterpret_cast<const uint4*>(e.eA + ri[u]);
        a1[u] = *reinterpret_cast<const uint4*>(e.eA + ri[u] + 16);
        b0[u] = *reinterpret_cast<const uint4*>(e.eA + ci[u]);
        b1[u] = *reinterpret_cast<const uint4*>(e.eA + ci[u] + 16);
    }
#pragma unroll
    for (int u = 0; u < SU; u++) {
        const uint32_t lb = ~(uint32_t)__builtin_amdgcn_sbfe((int)b0[u].w, 5, 1);    // kLastOfList: bit 5
        const uint32_t v00 = (uint32_t)(__popc(a0[u].y & b0[u].y) + __popc(a0[u].z & b0[u].z)) & ne[u];
        const uint32_t v01 = (uint32_t)(__popc(a0[u].y & b1[u].y) + __popc(a0[u].z & b1[u].z)) & lb;
        const uint32_t v10 = (uint32_t)(__popc(a1[u].y & b0[u].y) + __popc(a1[u].z & b0[u].z)) & ne[u];
        const uint32_t v11 = (uint32_t)(__popc(a1[u].y & b1[u].y) + __popc(a1[u].z & b1[u].z)) & (ne[u] & lb);
        cnt_add(cnt, a0[u].x, b0[u].w, v00);
        cnt_add(cnt, a0[u].x, b1[u].w, v01);
        cnt_add(cnt, a1[u].x, b0[u].w, v10);
        cnt_add(cnt, a1[u].x, b1[u].w, v11);
        if (mirror) {
            cnt_add(cnt, b0[u].x, a0[u].w, v00);
            cnt_add(cnt, b1[u].x, a0[u].w, v01);
            cnt_add(cnt, b0[u].x, a1[u].w, v10);
            cnt_add(cnt, b1[u].x, a1[u].w, v11);
        }
    }
}

// A batch's walk: windows of G groups of 64 slots (G a multiple of SUN):
// the window's last-slot masks, then SUN groups per step while whole steps
// remain, one group at a time after
template <int SUN, int MODE>
__device__ __forceinline__ void sparse_walk(const int4* __restrict__ rec, unsigned long long* __restrict__ masks,
                                            int last, int total, int lane, const SparseWalk& e,
                                            uint32_t* __restrict__ cnt, bool mirror) {
    constexpr int G = kWinGroups / SUN * SUN;
    for (int W0 = 0; W0 < total; W0 += 64 * G) {
        if (lane < G) masks[lane] = 0ull;
        __builtin_amdgcn_wave_barrier();
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        const uint32_t rel = (uint32_t)(last - W0);
        if (rel < 64u * G) atomicOr(&masks[rel >> 6], 1ull << (rel & 63));
        __builtin_amdgcn_wave_barrier();
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        const int wend = total < W0 + 64 * G ? total : W0 + 64 * G;
        int fb = W0;
        for (; fb + 64 * SUN <= wend; fb += 64 * SUN) {
            if (MODE == 0) sparse_diag_slots<SUN>(rec, masks, W0, last, fb, lane, e, cnt, mirror);
            else if (MODE == 1) sparse_off_slots<SUN>(rec, masks, W0, last, fb, lane, e, cnt);
            else if (MODE == 2) sparse_off22_slots<SUN>(rec, masks, W0, last, fb, lane, e, cnt);
            else sparse_diag22_slots<SUN>(rec, masks, W0, last, fb, lane, e, cnt, mirror);
        }
        for (; fb < wend; fb += 64) {
            if (MODE == 0) sparse_diag_slots<1>(rec, masks, W0, last, fb, lane, e, cnt, mirror);
            else if (MODE == 1) sparse_off_slots<1>(rec, masks, W0, last, fb, lane, e, cnt);
            else if (MODE == 2) sparse_off22_slots<1>(rec, masks, W0, last, fb, lane, e, cnt);
            else sparse_diag22_slots<1>(rec, masks, W0, last, fb, lane, e, cnt, mirror);
        }
        __builtin_amdgcn_wave_barrier();
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
    }
}

// The tile being walked (sparse_tile_kernel): its blocks' (block, word)
// offsets, bases of the chunk's records, row trimming, shape flags.
struct TileWalk {
    const int64_t* offA;
    const int64_t* offB;
    const ulonglong2* ent;
    int64_t ra0, cb0;                     // chunk bases (entries < 2^28 in all: byte offsets)
    uint32_t zA, zB;                      // the sentinel run from those bases
    SparseWalk e;
    int rlo, rhi;
    bool rpart, diag, mirror, r22;
    bool d22;                             // diagonal tiles in 2 x 2 micro-tiles (MT 2, option sparse_diag22)
};

// One batch of up to kBatchWords words [s0, we) walked over global memory
// (only >= 0: that lane's word alone)
template <int SUN, int MT>
__device__ __forceinline__ void global_batch(const TileWalk& tc, int64_t s0, int64_t we, int only, int lane,
                                             int4* __restrict__ wrec, unsigned long long* __restrict__ masks,
                                             uint32_t* __restrict__ cnt) {
    const int64_t* offA = tc.offA;
    const int64_t* offB = tc.offB;
    const ulonglong2* ent = tc.ent;
    const int64_t ra0 = tc.ra0, cb0 = tc.cb0;
    const uint32_t zA = tc.zA, zB = tc.zB;
    const SparseWalk& e = tc.e;
    const int rlo = tc.rlo, rhi = tc.rhi;
    const bool rpart = tc.rpart, diag = tc.diag, mirror = tc.mirror, r22 = tc.r22;
    const bool d22 = MT == 2 && tc.d22;
    const int64_t s = s0 + lane;
    int64_t rb = ra0, cb = cb0;
    int nr = 0, ncl = 0;
    if (lane < kBatchWords && s < we && (only < 0 || lane == only)) {
        rb = offA[s]; nr = (int)(offA[s + 1] - rb);
        cb = offB[s]; ncl = (int)(offB[s + 1] - cb);
        if (rpart) {                               // lists are sorted by set: trim both ends
            int a = 0, en = nr;
            for (int t = 0; t < nr; t++) {
                const int st = (int)((uint32_t)ent[rb + t].x >> 8);   // row code: set << 8 | rotation key
                a += st < rlo;
                en -= st >= rhi;
            }
            rb += a;
            nr = en > a ? en - a : 0;
        }
    }
    const int ncd = diag ? ncl : (ncl + 1) >> 1;   // column pairs per row (pair) (off-diagonal micro-tiles)
    const int hp = (nr + 1) >> 1;                 // 2 x 2 diagonal: pairs of entries
    const int P = diag ? (d22 ? (nr >= 2 ? hp * (hp + 1) / 2 : 0) : nr * (nr - 1) / 2)
                       : (r22 ? hp : nr) * ncd;
    int incl = P;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    const int total = __builtin_amdgcn_readlane(incl, 63);      // uniform: the walk's loop stays scalar
    // the records of the words with slots, compacted in slot order, and the
    // virtual word after them (its records: the zero sentinel run)
    const unsigned long long nz = __ballot(P > 0);
    const int k = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(nz >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)nz, 0u));
    if (P > 0) {
        if (diag) {
            wrec[k] = make_int4(-(incl - P), (int32_t)(rb - ra0), 0, 0);
        } else {
            const uint32_t rcp = (uint32_t)__float_as_int(__builtin_amdgcn_rcpf(2.0f * (float)ncd));
            wrec[k] = make_int4(-2 * (incl - P), (int32_t)((rb - ra0) << 4), (int32_t)((cb - cb0) << 4),
                                (int32_t)((rcp & 0xFFFFFF00u) | (uint32_t)(2 * ncd)));
        }
    }
    if (lane == 0) {
        const int nw = __popcll(nz);
        wrec[nw] = diag ? make_int4(-total, (int32_t)zA, 0, 0)
                        : make_int4(-2 * total, (int32_t)(zA << 4), (int32_t)(zB << 4), 0);
    }
    const int last = P > 0 ? incl - 1 : 0x7FFFFFFF;
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (MT == 2 && diag && d22) sparse_walk<2, 3>(wrec, masks, last, total, lane, e, cnt, mirror);
    else if (diag) sparse_walk<SUN, 0>(wrec, masks, last, total, lane, e, cnt, mirror);
    else if (MT == 2 && r22) sparse_walk<MT == 2 ? SUN : 1, 2>(wrec, masks, last, total, lane, e, cnt, false);
    else sparse_walk<SUN, 1>(wrec, masks, last, total, lane, e, cnt, false);
}

template <int SUN, int MT>
__global__ __launch_bounds__(SNT, 8) void sparse_tile_kernel(
    const int64_t* __restrict__ off, const ulonglong2* __restrict__ ent, const int32_t* __restrict__ nc, int64_t Us,
    int64_t Ws, const int2* __restrict__ tiles, const int32_t* __restrict__ cbnd, int nchunks, int64_t r0, int64_t r1,
    int64_t c0, int64_t c1, int upper, int32_t* __restrict__ I, int64_t ldI, int32_t* __restrict__ part, int64_t Wdp,
    int64_t N, const unsigned long long* __restrict__ slab_bits, int slabs, GroupPart gp, int xmap, int ntiles,
    RareSlab rs, int dyn, int diag22, int rpart22) {
    // gp: the group tier's part of every pair, added with the constant part
    // slab_bits / slabs: the in-kernel fold's dense words (set-major [N][Wdp])
    __shared__ uint32_t cnt[SB * SB / 2];                  // 32 KiB, 16-bit counters (cnt_index layout)
    __shared__ int4 rec[SNW][64];                          // 8 KiB: the batch's walk records
    // dyn: the chunk's next unclaimed batch, in wave 0's unused last record
    // (an LDS variable of its own would take the workgroup past 40 KiB: 3
    // workgroups a CU instead of 4, and the compiler then spends 80 VGPRs)
    int& next_batch = rec[0][63].w;
    // the rare rows of this step (above) are the launch's LAST workgroups:
    // they fill the CUs the tile workgroups' last round leaves idle
    const unsigned ntw = gridDim.x - (unsigned)rs.nrare;
    if (blockIdx.x >= ntw) {
        rare_slab_row(rs, (int)(blockIdx.x - ntw), r0, c0, c1, upper, cnt);
        return;
    }
    const unsigned bid = blockIdx.x;
    int tile, ch;
    if (xmap) {
        // option sparse_xcd: workgroup b = 8 (t + ntiles g) + x runs chunk
        // 8 g + x of tile t. Workgroups are dealt to the 8 XCDs round-robin,
        // so chunk c of every tile runs on XCD c mod 8, the tiles of one
        // chunk back to back: that XCD's L2 serves the chunk's records
        // (~0.85 MB on C2) to all the tiles reading them
        const int x = (int)(bid & 7), k = (int)(bid >> 3);
        tile = k % ntiles;
        ch = 8 * (k / ntiles) + x;
        if (ch >= nchunks) return;
    } else {
        tile = (int)(bid / (unsigned)nchunks);
        ch = (int)(bid % (unsigned)nchunks);
    }
    const int64_t A = tiles[tile].x, B = tiles[tile].y;
    const int rlo = (int)(r0 - A * SB > 0 ? r0 - A * SB : 0);
    const int rhi = (int)(r1 - A * SB < SB ? r1 - A * SB : SB);
    // rows trimmed only where the region cuts a block's existing rows: the
    // collection's last, partial block ending at r1 = N needs no trimming
    const bool rpart = rlo > 0 || (rhi < SB && r1 < N);
    const bool diag = A == B && !rpart, mirror = diag && !upper;
    // 2 x 2 micro-tiles, row-trimmed tiles too (option sparse_rpart22): a
    // trimmed list's odd last pair reads the entry after the range as its
    // second row — a row outside the region, whose counters no store reads
    const bool r22 = MT == 2 && !diag && (!rpart || rpart22);
    for (int t = threadIdx.x; t < SB * SB / 2; t += SNT) cnt[t] = 0;
    if (threadIdx.x == 0) next_batch = SNW;
    __syncthreads();
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int64_t sb = cbnd[ch], se = cbnd[ch + 1];          // the chunk's sparse words
    const int64_t* offA = off + A * Ws;
    const int64_t* offB = off + B * Ws;
    const int64_t ra0 = offA[sb], cb0 = offB[sb];           // chunk bases (entries < 2^28 in all: byte offsets)
    const int64_t ntot = off[(int64_t)ceil_div(N, SB) * Ws];         // entries of every block: the sentinel run
    const uint32_t zA = (uint32_t)(ntot - ra0), zB = (uint32_t)(ntot - cb0);
    const TileWalk tc{offA, offB, ent, ra0, cb0, zA, zB,
                      SparseWalk{reinterpret_cast<const char*>(ent + ra0), reinterpret_cast<const char*>(ent + cb0)},
                      rlo, rhi, rpart, diag, mirror, r22, diag22 != 0};
    int4* wrec = &rec[wv][0];
    unsigned long long* masks = reinterpret_cast<unsigned long long*>(&rec[wv][kBatchWords + 1]);
    // the wave's share of the chunk's words, in batches of kBatchWords: an
    // equal run of words per wave, or (dyn, default) batch wv first and then
    // the next unclaimed one (an LDS counter), so that a wave that drew light
    // words takes more of them instead of idling until the heaviest wave ends
    const int64_t per = ceil_div(se - sb, (int64_t)SNW);
    const int64_t wb = dyn ? sb + (int64_t)wv * kBatchWords : sb + (int64_t)wv * per;
    const int64_t we = dyn ? se : (wb + per < se ? wb + per : se);
    for (int64_t s0 = wb; s0 < we;) {
        global_batch<SUN, MT>(tc, s0, we, -1, lane, wrec, masks, cnt);
        if (dyn) {
            int nb = 0;
            if (lane == 0) nb = atomicAdd(&next_batch, 1);
            s0 = sb + (int64_t)__builtin_amdgcn_readfirstlane(__shfl(nb, 0, 64)) * kBatchWords;
        } else {
            s0 += kBatchWords;
        }
    }
    if (ch < slabs) {
        // dense words [8 ch, 8 ch + 8) of the tile's 128 x 128 pairs: the
        // rows' words staged in the record area (8 KiB), a thread holds one
        // column's 8 words and walks 32 rows (broadcast LDS reads)
        __syncthreads();                                   // every wave is done with its records
        unsigned long long* As = reinterpret_cast<unsigned long long*>(&rec[0][0]);
        const int64_t w0 = (int64_t)ch * kFoldSlabWords;
        for (int t = threadIdx.x; t < SB * kFoldSlabWords; t += SNT) {
            const int64_t i = A * SB + (t >> 3);
            As[t] = i < N ? slab_bits[i * Wdp + w0 + (t & 7)] : 0ull;
        }
        __syncthreads();
        const int b = threadIdx.x & (SB - 1), rg = threadIdx.x >> 7;
        const int64_t j = B * SB + b;
        if (j < N) {
            unsigned long long bw[kFoldSlabWords];
#pragma unroll
            for (int k = 0; k < kFoldSlabWords; k++) bw[k] = slab_bits[j * Wdp + w0 + k];
            for (int a = rg * (SB / 4); a < (rg + 1) * (SB / 4); a++) {
                const ulonglong2* ar = reinterpret_cast<const ulonglong2*>(As + a * kFoldSlabWords);
                uint32_t v = 0;
#pragma unroll
                for (int k = 0; k < kFoldSlabWords / 2; k++) {
                    const ulonglong2 x = ar[k];
                    v += (uint32_t)__popcll(x.x & bw[2 * k]) + (uint32_t)__popcll(x.y & bw[2 * k + 1]);
                }
                const int t0 = cnt_index(a, b);
                atomicAdd(&cnt[t0 >> 1], v << ((t0 & 1) << 4));
            }
        }
    }
    __syncthreads();
    if (part) {
        uint32_t* dst = reinterpret_cast<uint32_t*>(part) + ((int64_t)tile * nchunks + ch) * (SB * SB / 2);
        for (int t = threadIdx.x; t < SB * SB / 2; t += SNT) dst[t] = cnt[t];
        return;
    }
    for (int t = threadIdx.x; t < SB * SB; t += SNT) {
        int a, b;
        cnt_pair(t, a, b);
        const int64_t i = A * SB + a, j = B * SB + b;
        if (i < r0 || i >= r1 || j < c0 || j >= c1 || (upper && j <= i)) continue;
        // the constant part once per pair: by chunk 0 (chunks flush with atomics)
        const int v = (int)((cnt[t >> 1] >> ((t & 1) << 4)) & 0xFFFFu) +
                      (ch == 0 ? (int)Us - nc[i] - nc[j] + gp.at(i, j) : 0);
        if (v) atomicAdd(I + (i - r0) * ldI + (j - c0), v);
    }
}

// the chunks' counters of each tile + the constant part, into I. A lane
// owns 8 counters (one 16-byte word of a chunk's partial); the four waves of
// a workgroup take every fourth chunk of the same 64 words (independent
// 16-byte loads, several in flight per lane), sum through LDS, and wave 0
// adds the 512 counters into I. 32 workgroups per tile: the loads of the
// whole grid in flight cover the latency of the partials' read (round 2: one
// workgroup per CU, 62 loads per lane in a chain, ran at ~2 TB/s).
constexpr int kReduceCnt = 8;
constexpr int kReduceGroups = 64;                            // 16-byte groups per workgroup
__global__ __launch_bounds__(256) void sparse_reduce_kernel(const int32_t* __restrict__ part, int nchunks,
                                                            const int2* __restrict__ tiles,
                                                            const int32_t* __restrict__ nc, int64_t Us, int64_t r0,
                                                            int64_t r1, int64_t c0, int64_t c1, int upper,
                                                            int32_t* __restrict__ I, int64_t ldI,
                                                            const uint32_t* __restrict__ rslab,
                                                            double* __restrict__ D, int64_t ldD,
                                                            const int64_t* __restrict__ soff, int empty_nan,
                                                            GroupPart gp) {
#pragma clang fp contract(off)
    constexpr int per_tile = SB * SB / kReduceCnt / kReduceGroups;       // workgroups per tile
    __shared__ uint32_t sum[4][kReduceCnt][kReduceGroups];               // 8 KiB
    const int tile = blockIdx.x / per_tile;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = (blockIdx.x % per_tile) * kReduceGroups + lane;        // 16-byte group of the tile's counters
    const uint4* p = reinterpret_cast<const uint4*>(part) + (int64_t)tile * nchunks * (SB * SB / 8) + g;
    uint32_t acc[kReduceCnt] = {0, 0, 0, 0, 0, 0, 0, 0};
    auto add = [&](const uint4& v) {
        acc[0] += v.x & 0xFFFFu; acc[1] += v.x >> 16;
        acc[2] += v.y & 0xFFFFu; acc[3] += v.y >> 16;
        acc[4] += v.z & 0xFFFFu; acc[5] += v.z >> 16;
        acc[6] += v.w & 0xFFFFu; acc[7] += v.w >> 16;
    };
    // 8 independent 16-byte loads in flight per lane (4 in round 2/3: the
    // partials sit in L2 / the Infinity Cache right after the tile kernel,
    // and the read is latency-bound at 4 per lane)
    int c = wv;
    for (; c + 28 < nchunks; c += 32) {
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = p[(int64_t)(c + 4 * k) * (SB * SB / 8)];
#pragma unroll
        for (int k = 0; k < 8; k++) add(v[k]);
    }
    for (; c + 12 < nchunks; c += 16) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = p[(int64_t)(c + 4 * k) * (SB * SB / 8)];
#pragma unroll
        for (int k = 0; k < 4; k++) add(v[k]);
    }
    for (; c < nchunks; c += 4) add(p[(int64_t)c * (SB * SB / 8)]);
#pragma unroll
    for (int k = 0; k < kReduceCnt; k++) sum[wv][k][lane] = acc[k];
    __syncthreads();
    // 512 counters per workgroup: each thread finalizes two
    for (int e = threadIdx.x; e < kReduceCnt * kReduceGroups; e += 256) {
        const int gl = e / kReduceCnt, k = e % kReduceCnt;               // consecutive threads: consecutive counters
        const int t = ((blockIdx.x % per_tile) * kReduceGroups + gl) * kReduceCnt + k;   // cnt_index layout
        // + the rare tier's pairs of this step (the tile launch's rare rows
        // wrote every slot of the region's rows: same layout, coalesced)
        const uint32_t tot = sum[0][k][gl] + sum[1][k][gl] + sum[2][k][gl] + sum[3][k][gl] +
                             (rslab ? rslab[(int64_t)tile * (SB * SB) + t] : 0u);
        int a, b;
        cnt_pair(t, a, b);
        const int64_t i = (int64_t)tiles[tile].x * SB + a, j = (int64_t)tiles[tile].y * SB + b;
        if (i < r0 || i >= r1 || j < c0 || j >= c1 || (upper && j <= i)) continue;
        int v = (int)Us - nc[i] - nc[j] + (int)tot + gp.at(i, j);
        if (D && i == j) v = (int)(soff[i + 1] - soff[i]);        // a set with itself (self_pairs_kernel)
        if (D) {                             // fused: the only writer of I over the region, then D
            I[(i - r0) * ldI + (j - c0)] = v;
            const int64_t na = soff[i + 1] - soff[i], nb = soff[j + 1] - soff[j];
            double d;
            if (v > 0) d = 1.0 - (double)v / (double)(na + nb - v);      // as epilogue_kernel (bitset.hip)
            else d = (empty_nan && na + nb == 0) ? __builtin_nan("") : 1.0;
            D[(i - r0) * ldD + (j - c0)] = d;
        } else if (v) {
            atomicAdd(I + (i - r0) * ldI + (j - c0), v);
        }
    }
}

}  // namespace

// ---- host side ------------------------------------------------------------

void locus_keys(gdist_ctx* ctx, const gdist_sets* s, const uint64_t* dict, const uint32_t* dcounts, int64_t U,
                uint64_t tag, DevBuf& key) {
    hipStream_t st = ctx->stream;
    key.alloc(U * 8 + 8, st);
    if (U == 0) return;
    unkeyed_kernel<<<grid_for(U), 256, 0, st>>>(key.as<uint64_t>(), dcounts, U);
    if (s->n_guide > 0)
        locus_key_kernel<<<grid_for(s->n_guide), 256, 0, st>>>(s->guide_codes.as<uint64_t>(),
                                                               s->guide_keys.as<uint64_t>(), s->n_guide, dict, U, tag,
                                                               key.as<uint64_t>());
    GD_HIP(hipGetLastError());
}

void locus_keys_min(gdist_ctx* ctx, const uint64_t* all, int64_t U, int64_t stride_r, int R, DevBuf& key) {
    hipStream_t st = ctx->stream;
    key.alloc(U * 8 + 8, st);
    if (U == 0) return;
    min_over_ranks_kernel<<<grid_for(U), 256, 0, st>>>(all, U, stride_r, R, key.as<uint64_t>());
    GD_HIP(hipGetLastError());
}

void locus_perm(gdist_ctx* ctx, DevBuf& key, int64_t U, DevBuf& perm) {
    hipStream_t st = ctx->stream;
    GD_REQUIRE(U < (int64_t(1) << 31), "dense dictionary too large for the locus order");
    perm.alloc(U * 4 + 4, st);
    if (U == 0) return;
    DevBuf kB(U * 8, st), vA(U * 4, st), vB(U * 4, st);
    iota_i32_kernel<<<grid_for(U), 256, 0, st>>>(vA.as<int32_t>(), U);
    GD_HIP(hipGetLastError());
    uint64_t* k = key.as<uint64_t>(); uint64_t* ka = kB.as<uint64_t>();
    int32_t* v = vA.as<int32_t>(); int32_t* va = vB.as<int32_t>();
    sort_pairs_u64_i32(ctx, k, ka, v, va, (size_t)U, 0, 64);   // stable: unkeyed ranks keep code order
    invert_perm_kernel<<<grid_for(U), 256, 0, st>>>(v, U, perm.as<uint32_t>());
    GD_HIP(hipGetLastError());
    GD_HIP(hipStreamSynchronize(st));
}

bool locus_order_enabled(const gdist_ctx* ctx) { return ctx->option(OPT_LOCUS_ORDER, 1) != 0; }

void free_sparse(gdist_sets* s) {
    if (s->ctx) {                        // launches on the side stream may still read these buffers
        (void)hipStreamSynchronize(s->ctx->side);
        (void)hipStreamSynchronize(s->ctx->stream);
    }
    s->fp4.release();                     // the MFMA operand expands the dense words
    s->fp4_W = 0;
    s->graphs.clear();
    s->plans.clear();
    s->dbits.release();
    s->sp_off.release();
    s->sp_ent.release();
    s->sp_nc.release();
    s->sparse = false;
    s->Wd = s->Ws = s->sp_entries = s->sp_U = 0;
    s->sp_bucket_bits.clear();
    s->sp_nbk = 0;
    s->sp_pos_words = 0;
    s->sp_fold_dense = false;
    s->sp_fold_slabs = 0;
    s->sp_products = s->sp_items = s->sp_pairs = 0.0;
    s->sp_grp.release();
    s->sp_V.release();
    s->sp_T.release();
    s->sp_groups = s->sp_group_words = 0;
}

// Modelled seconds of the sparse words over a block: products (each pair's
// common sparse words) and the (tile, word) visits of every launched tile.
double sparse_block_cost_s(const gdist_sets* s, double f_area, double tiles) {
    if (!s->sparse) return 0.0;
    const double nb = (double)ceil_div(s->nsets, SB);
    const double all_tiles = nb * (nb + 1) / 2;
    return f_area * s->sp_products / kSparseProductsPerS + tiles / all_tiles * s->sp_items / kSparseItemsPerS;
}

void build_sparse_words(gdist_ctx* ctx, gdist_sets* s) {
    free_sparse(s);
    if (ctx->option(OPT_SPARSE, 1) == 0 || s->W == 0 || s->nsets < 2) return;
    hipStream_t st = ctx->stream;
    Trace tr(st, ctx->trace());
    const int64_t N = s->nsets, W = s->W, U = s->dict_size;
    const int64_t Wv = ceil_div(U, 64);   // words holding dictionary bits
    if (Wv == 0) return;
    const unsigned long long* bits = s->bits.as<unsigned long long>();
    DevBuf dz(W * 8, st);
    GD_HIP(hipMemsetAsync(dz.p, 0, W * 8, st));
    const int64_t rpb = 64;
    dim3 g((unsigned)ceil_div(W, 256), (unsigned)ceil_div(N, rpb));
    word_z_kernel<<<g, 256, 0, st>>>(bits, N, W, U, rpb, dz.as<int32_t>(), dz.as<int32_t>() + W);
    GD_HIP(hipGetLastError());
    std::vector<int32_t> zc(W), zp(W), z(W);
    d2h(zc.data(), dz.p, W * 4, st);
    d2h(zp.data(), dz.as<int32_t>() + W, W * 4, st);
    // each word is counted from the side fewer sets have entries on: the
    // complement (sets lacking a common kmer) or the word itself (sets
    // holding a rare one); the option sparse_zmax forces the complement side
    std::vector<uint8_t> wpos(W, 0);
    for (int64_t w = 0; w < W; w++) {
        wpos[w] = !ctx->has_option(OPT_SPARSE_ZMAX) && zp[w] < zc[w];
        z[w] = wpos[w] ? zp[w] : zc[w];
    }
    tr.mark("sparse: word classes");
    // ---- group tier: heavy words whose entries are the groups' patterns
    const bool zm = ctx->has_option(OPT_SPARSE_ZMAX);
    const int64_t nwb = ceil_div(N, 64);
    std::vector<int32_t> wrow(W, -1);                     // factorised word -> pattern row
    std::vector<unsigned long long> prow_pats;            // rows x mg patterns
    std::vector<int32_t> grp;                             // set -> group
    int mg = 0;
    int64_t lacked_words = 0;
    if (ctx->option(OPT_SPARSE_GROUPS, 1) != 0 && !zm && N >= 2 * kGroupMinSize && N <= kGroupMaxN) {
        std::vector<int32_t> cw;
        std::vector<uint8_t> cp;
        for (int64_t w = 0; w < Wv; w++)
            if (z[w] >= kGroupMinZ) { cw.push_back((int32_t)w); cp.push_back(wpos[w]); }
        const int64_t nc = (int64_t)cw.size();
        if (nc > 0) {
            DevBuf dcw(nc * 4, st), dcp(nc + 8, st), ms(nc * 4, st), mh(nc * 8, st);
            h2d(dcw.p, cw.data(), nc * 4, st);
            h2d(dcp.p, cp.data(), nc, st);
            std::vector<int32_t> hs(nc);
            std::vector<unsigned long long> hh(nc);
            // 1. discovery: each heavy word's modal pattern and its members
            std::map<std::pair<unsigned long long, int32_t>, std::vector<int64_t>> by;
            std::vector<std::pair<int64_t, std::vector<unsigned long long>>> cands;   // (words, member bitmap)
            {
                DevBuf mb((size_t)nc * nwb * 8, st);
                group_modal_kernel<<<(unsigned)nc, 256, 0, st>>>(bits, N, W, U, dcw.as<int32_t>(), dcp.as<uint8_t>(),
                                                                  nwb, mb.as<unsigned long long>(), ms.as<int32_t>(),
                                                                  mh.as<unsigned long long>());
                GD_HIP(hipGetLastError());
                d2h(hs.data(), ms.p, nc * 4, st);
                d2h(hh.data(), mh.p, nc * 8, st);
                for (int64_t c = 0; c < nc; c++)
                    if (hs[c] >= kGroupMinSize && hs[c] < N) by[{hh[c], hs[c]}].push_back(c);
                std::vector<const std::vector<int64_t>*> order;
                for (auto& kv : by)
                    if ((int64_t)kv.second.size() >= kGroupMinWords) order.push_back(&kv.second);
                std::stable_sort(order.begin(), order.end(), [](const std::vector<int64_t>* a,
                                                                const std::vector<int64_t>* b) {
                    return a->size() > b->size();
                });
                if (order.size() > 256) order.resize(256);   // the 256 most recurring lists
                for (auto* o : order) {
                    std::vector<unsigned long long> bm(nwb);
                    d2h(bm.data(), mb.as<unsigned long long>() + (*o)[0] * nwb, nwb * 8, st);
                    cands.push_back({(int64_t)o->size(), std::move(bm)});
                }
            }
            // 2. the groups: the atoms of the recurring member lists (sets in
            //    exactly the same lists form one group), so that a list which is
            //    a union of groups (clades sharing a pattern) is expressed by
            //    its groups, each with that pattern. Lists refine the partition
            //    most recurring first, and a list that would split off a part
            //    smaller than a group (a clade less a member) is passed over.
            grp.assign(N, -1);
            {
                std::vector<unsigned long long> sig(N, 0);
                std::vector<unsigned char> in(N);
                for (size_t k = 0; k < cands.size(); k++) {
                    for (int64_t i = 0; i < N; i++) in[i] = (cands[k].second[i >> 6] >> (i & 63)) & 1;
                    std::map<unsigned long long, std::pair<int64_t, int64_t>> split;   // atom -> (in, out)
                    for (int64_t i = 0; i < N; i++) (in[i] ? split[sig[i]].first : split[sig[i]].second)++;
                    bool ok = true;
                    for (auto& kv : split)
                        if ((kv.second.first && kv.second.first < kGroupMinSize) ||
                            (kv.second.second && kv.second.second < kGroupMinSize && kv.first != 0)) ok = false;
                    if (!ok) continue;
                    const unsigned long long key = 0x9E3779B97F4A7C15ull * (unsigned long long)(k + 1);
                    for (int64_t i = 0; i < N; i++)
                        if (in[i]) sig[i] = (sig[i] ^ key) * 0xBF58476D1CE4E5B9ull + 1;
                }
                std::map<unsigned long long, std::vector<int64_t>> atoms;
                for (int64_t i = 0; i < N; i++)
                    if (sig[i]) atoms[sig[i]].push_back(i);
                std::vector<const std::vector<int64_t>*> order;
                for (auto& kv : atoms)
                    if ((int64_t)kv.second.size() >= kGroupMinSize) order.push_back(&kv.second);
                std::stable_sort(order.begin(), order.end(), [](const std::vector<int64_t>* a,
                                                                const std::vector<int64_t>* b) {
                    return a->size() > b->size();
                });
                for (auto* o : order) {
                    if (mg >= kGroupMax) break;
                    for (int64_t i : *o) grp[i] = mg;
                    mg++;
                }
            }
            // 3. every group's pattern per candidate word; factorise the words
            //    whose residual entries are fewer
            if (mg > 0) {
                DevBuf dgrp(N * 4, st), cpat((size_t)nc * 2 * mg * 8, st), zres(nc * 2 * 4, st);
                h2d(dgrp.p, grp.data(), N * 4, st);
                group_pattern_kernel<<<(unsigned)nc, 256, 0, st>>>(bits, N, W, U, dcw.as<int32_t>(), dcp.as<uint8_t>(),
                                                                    dgrp.as<int32_t>(), mg,
                                                                    cpat.as<unsigned long long>(), zres.as<int32_t>());
                GD_HIP(hipGetLastError());
                std::vector<unsigned long long> hp((size_t)nc * 2 * mg);
                std::vector<int32_t> hz(nc * 2);
                d2h(hp.data(), cpat.p, hp.size() * 8, st);
                d2h(hz.data(), zres.p, nc * 2 * 4, st);
                for (int64_t c = 0; c < nc; c++) {
                    const int64_t w = cw[c];
                    const int lack = hz[2 * c + 1] < hz[2 * c] ? 1 : 0;
                    if (hz[2 * c + lack] >= z[w]) continue;
                    wrow[w] = (int32_t)(prow_pats.size() / mg) | (lack ? kRowLack : 0);
                    prow_pats.insert(prow_pats.end(), hp.begin() + (2 * c + lack) * mg, hp.begin() + (2 * c + lack + 1) * mg);
                    z[w] = hz[2 * c + lack];      // the residual entries decide the word's class
                    lacked_words += lack;
                }
            }
            if (ctx->trace()) {
                int64_t grouped_sets = 0;
                for (int32_t g : grp) grouped_sets += g >= 0;
                fprintf(stderr, "gdist: group tier: %lld candidate words, %zu recurring member lists, %d groups "
                                "(%lld sets), %zu words factorised (%lld in lacked mode)\n",
                        (long long)nc, cands.size(), mg, (long long)grouped_sets, mg ? prow_pats.size() / mg : 0,
                        (long long)lacked_words);
            }
        }
        tr.mark("sparse: group tier");
    }
    // A word is sparse when its products + visits cost less than its column
    // of word pairs in the dense tiles (option sparse_zmax overrides).
    const double n = (double)N, pairs = 0.5 * n * (n - 1.0);
    const double nb = (double)ceil_div(N, SB), tiles = nb * (nb + 1) / 2;
    const double dense_word_s = pairs / kDenseWordPairsPerS;
    const int64_t zmax = ctx->option(OPT_SPARSE_ZMAX, 0);
    std::vector<int32_t> sw, dw;
    double products = 0.0, zpairs = 0.0;
    for (int64_t w = 0; w < Wv; w++) {
        const double zz = (double)z[w];
        const bool sparse = zm ? z[w] <= zmax
                               : 0.5 * zz * zz / kSparseProductsPerS + tiles / kSparseItemsPerS < dense_word_s;
        if (sparse) { sw.push_back((int32_t)w); products += 0.5 * zz * zz; zpairs += 0.5 * zz * (zz - 1.0); }
        else dw.push_back((int32_t)w);
    }
    const int64_t Ws = (int64_t)sw.size(), Wd = (int64_t)dw.size();
    if (ctx->trace() && Wd) {
        std::vector<int32_t> zd;
        for (int32_t w : dw) zd.push_back(z[w]);
        std::sort(zd.begin(), zd.end());
        fprintf(stderr, "gdist: %lld dense words, z min %d median %d max %d (of %lld sets), word indices %d..%d of %lld; "
                        "words past the valid bits %lld\n",
                (long long)Wd, zd.front(), zd[zd.size() / 2], zd.back(), (long long)N, dw.front(), dw.back(),
                (long long)Wv, (long long)(W - Wv));
    }
    const int64_t Wdp = Wd ? ceil_div(Wd, 16) * 16 : 0;
    // whole-triangle estimates: keep the split only if it beats the plain tiles
    const double t_plain = pairs * (double)W / kDenseWordPairsPerS;
    const double t_split = pairs * (double)Wdp / kDenseWordPairsPerS + products / kSparseProductsPerS +
                           tiles * (double)Ws / kSparseItemsPerS;
    if (ctx->trace())
        fprintf(stderr, "gdist: sparse split model: plain tiles %.3f ms, split %.3f ms (%lld sparse words, %.3g products)\n",
                t_plain * 1e3, t_split * 1e3, (long long)Ws, products);
    if (Ws == 0 || !(zm || t_split < 0.8 * t_plain)) return;
    const int64_t nblk = ceil_div(N, SB);
    GD_REQUIRE((double)nblk * (double)Ws < 2e9, "sparse word index too large");
    std::vector<uint8_t> spos(Ws);
    for (int64_t k = 0; k < Ws; k++) spos[k] = wpos[sw[k]];
    DevBuf dsw(Ws * 4, st), dsp(Ws + 8, st), cnt(nblk * Ws * 4 + 4, st);
    h2d(dsw.p, sw.data(), Ws * 4, st);
    h2d(dsp.p, spos.data(), Ws, st);
    // the sparse words' pattern rows (group tier)
    std::vector<int32_t> sprow(Ws, -1);
    std::vector<unsigned long long> spats;
    int64_t grouped = 0;
    for (int64_t k = 0; k < Ws; k++)
        if (wrow[sw[k]] >= 0) {
            const int64_t row = wrow[sw[k]] & ~kRowLack;
            sprow[k] = (int32_t)grouped++ | (wrow[sw[k]] & kRowLack);
            spats.insert(spats.end(), prow_pats.begin() + row * mg, prow_pats.begin() + (row + 1) * mg);
        }
    DevBuf dgrp, dprow, dpats, dV;
    GroupWords gw;
    if (grouped) {
        dgrp.alloc(N * 4, st);
        dprow.alloc(Ws * 4, st);
        dpats.alloc(spats.size() * 8, st);
        dV.alloc((size_t)mg * N * 4, st);
        h2d(dgrp.p, grp.data(), N * 4, st);
        h2d(dprow.p, sprow.data(), Ws * 4, st);
        h2d(dpats.p, spats.data(), spats.size() * 8, st);
        GD_HIP(hipMemsetAsync(dV.p, 0, (size_t)mg * N * 4, st));
        gw.grp = dgrp.as<int32_t>();
        gw.prow = dprow.as<int32_t>();
        gw.pats = dpats.as<unsigned long long>();
        gw.m = mg;
        gw.V = dV.as<int32_t>();
        gw.N = N;
    }
    dim3 gs((unsigned)ceil_div(Ws, 256), (unsigned)nblk);
    sparse_count_kernel<<<gs, 256, 0, st>>>(bits, N, W, U, dsw.as<int32_t>(), dsp.as<uint8_t>(), Ws, gw,
                                            cnt.as<int32_t>());
    GD_HIP(hipGetLastError());
    GD_HIP(hipMemsetAsync(cnt.as<int32_t>() + nblk * Ws, 0, 4, st));
    s->sp_off.alloc((nblk * Ws + 1) * 8, st);
    exclusive_scan_i32_to_i64(ctx, cnt.as<int32_t>(), s->sp_off.as<int64_t>(), (size_t)(nblk * Ws + 1));
    int64_t total = 0;
    d2h(&total, s->sp_off.as<int64_t>() + nblk * Ws, 8, st);
    // the tile kernel addresses a chunk's records by 32-bit byte offsets from
    // its base, the sentinel run after the last entry included
    if (total + kSentinelRecs >= (int64_t(1) << 28)) {
        if (ctx->trace())
            fprintf(stderr, "gdist: %lld sparse entries exceed the tile kernel's 2^28: no sparse split\n",
                    (long long)total);
        free_sparse(s);
        return;
    }
    // the entries' words and set bytes, turned into the kernel's records below
    DevBuf sp_word(total * 8 + 8, st), sp_set(total + 8, st);
    s->sp_nc.alloc(N * 4, st);
    GD_HIP(hipMemsetAsync(s->sp_nc.p, 0, N * 4, st));
    const int64_t nbk = ceil_div(Ws, int64_t(1) << kBucketShift);
    DevBuf dbb((size_t)N * nbk * 4, st);
    GD_HIP(hipMemsetAsync(dbb.p, 0, (size_t)N * nbk * 4, st));
    sparse_fill_kernel<<<gs, 256, 0, st>>>(bits, N, W, U, dsw.as<int32_t>(), dsp.as<uint8_t>(), Ws, gw,
                                           s->sp_off.as<int64_t>(),
                                           sp_word.as<unsigned long long>(), sp_set.as<uint8_t>(),
                                           s->sp_nc.as<int32_t>(), dbb.as<int32_t>(), nbk);
    GD_HIP(hipGetLastError());
    {   // complement bits of every set per bucket of 1024 sparse words, kept
        // on the host for the chunk bound of sparse_matrix
        s->sp_nbk = nbk;
        s->sp_bucket_bits.assign((size_t)N * nbk, 0);
        d2h(s->sp_bucket_bits.data(), dbb.p, (size_t)N * nbk * 4, st);
    }
    GD_HIP(hipGetLastError());
    s->sp_ent.alloc((total + kSentinelRecs) * 16, st);
    GD_HIP(hipMemsetAsync(s->sp_ent.as<ulonglong2>() + total, 0, kSentinelRecs * 16, st));   // the sentinel run
    if (total) {
        sparse_records_kernel<<<grid_for(total), 256, 0, st>>>(sp_word.as<unsigned long long>(),
                                                                sp_set.as<uint8_t>(), total,
                                                                s->sp_ent.as<ulonglong2>());
        GD_HIP(hipGetLastError());
        sparse_last_kernel<<<grid_for(nblk * Ws), 256, 0, st>>>(s->sp_off.as<int64_t>(), nblk * Ws,
                                                                s->sp_ent.as<ulonglong2>());
    }
    GD_HIP(hipGetLastError());
    if (grouped) {
        // the group part of every pair: T from the pattern rows, V came with
        // the entries (sparse_fill_kernel); the set -> group map stays
        DevBuf T((size_t)mg * mg * 4, st);
        GD_HIP(hipMemsetAsync(T.p, 0, (size_t)mg * mg * 4, st));
        group_t_kernel<<<(unsigned)grouped, 256, 0, st>>>(dpats.as<unsigned long long>(), grouped, mg,
                                                           T.as<int32_t>());
        GD_HIP(hipGetLastError());
        GD_HIP(hipStreamSynchronize(st));
        s->sp_grp = std::move(dgrp);
        s->sp_V = std::move(dV);
        s->sp_T = std::move(T);
        s->sp_groups = mg;
        s->sp_group_words = grouped;
    }
    if (Wdp) {
        DevBuf ddw(Wd * 4, st);
        h2d(ddw.p, dw.data(), Wd * 4, st);
        s->dbits.alloc((size_t)N * Wdp * 8, st);
        gather_words_kernel<<<grid_for(N * Wdp), 256, 0, st>>>(bits, W, ddw.as<int32_t>(), Wd, Wdp, N,
                                                               s->dbits.as<unsigned long long>());
        GD_HIP(hipGetLastError());
    }
    int64_t Us = 0;                       // valid bits of the complement-sparse words
    int64_t npos = 0;
    for (int32_t w : sw) {
        if (wpos[w]) { npos++; continue; }
        Us += (w + 1) * 64 <= U ? 64 : U - (int64_t)w * 64;
    }
    s->sp_pos_words = npos;
    // The dense words counted inside the tile kernel (option sparse_fold,
    // default up to 64 words): chunk c < Wdp / 8 of every tile adds words
    // [8c, 8c + 8) of its 128 x 128 pairs into its LDS counters (~2 us per
    // such workgroup), so no dense-word tile launch shares the CUs with the
    // sparse kernel (C2: 0.09 + 0.04 ms of tiles beside it); past the option
    // the dense words get their own tile launch (bitset_matrix)
    if (Wdp > 0 && Wdp <= ctx->option(OPT_SPARSE_FOLD, 64)) {
        s->sp_fold_dense = true;
        s->sp_fold_slabs = (int)(Wdp / kFoldSlabWords);
    }
    GD_HIP(hipStreamSynchronize(st));
    s->sparse = true;
    s->Ws = Ws;
    s->Wd = Wdp;
    s->sp_entries = total;
    s->sp_U = Us;
    s->sp_products = products;
    s->sp_pairs = zpairs;
    s->sp_items = tiles * (double)Ws;
    tr.mark("sparse: entries + dense words");
}

// The rare tier's pairs of a region are recounted in every step by the
// trailing workgroups of the sparse tile launch (rare_slab_row above) into a
// per-tile slab the chunk reduce adds. The plan keeps only geometry: the
// region's (row block, column block) -> tile map and the slab's allocation.
// Taken when the tier is small and its lists short (a row's thread walks a
// list serially); otherwise the rare kernels of bitset_matrix count them.
constexpr double kRareSlabWorkMax = double(int64_t(1) << 26);

static void rare_slab_plan(gdist_ctx* ctx, const gdist_sets* s, int64_t r0, int64_t r1,
                           const std::vector<int2>& tiles, SparseScratch& sc) {
    hipStream_t st = ctx->stream;
    sc.rare_in = false;
    if (s->n_rare == 0) return;
    if (ctx->option(OPT_SPARSE_RARE, 1) == 0 || tiles.empty()) return;
    if ((double)s->rare_records + (double)s->rare_incs > kRareSlabWorkMax || s->rare_max_list > kLongList) return;
    const int64_t nbc = ceil_div(s->nsets, SB), ab0 = r0 / SB, nrb = (r1 - 1) / SB - ab0 + 1;
    std::vector<int32_t> tile_of((size_t)(nrb * nbc), -1);
    for (size_t t = 0; t < tiles.size(); t++) tile_of[(size_t)((tiles[t].x - ab0) * nbc + tiles[t].y)] = (int32_t)t;
    sc.rare_tile.alloc(tile_of.size() * 4, st);
    h2d(sc.rare_tile.p, tile_of.data(), tile_of.size() * 4, st);
    sc.rare_slab.alloc(tiles.size() * (size_t)(SB * SB) * 4, st);
    sc.rare_ab0 = ab0;
    sc.rare_nbc = nbc;
    sc.rare_in = true;
}

void sparse_plan(gdist_ctx* ctx, const gdist_sets* s, int64_t r0, int64_t r1, int64_t c0, int64_t c1, bool upper,
                 hipStream_t st, SparseScratch& sc) {
    if (!s->sparse || r1 <= r0 || c1 <= c0) return;
    if (!sc.ready) {
        std::vector<int2> tiles;
        for (int64_t A = r0 / SB; A <= (r1 - 1) / SB; A++)
            for (int64_t B = c0 / SB; B <= (c1 - 1) / SB; B++) {
                const int64_t rmin = std::max(r0, A * SB);
                const int64_t cmax = std::min(c1, (B + 1) * SB) - 1;
                if (upper && cmax <= rmin) continue;
                tiles.push_back(make_int2((int)A, (int)B));
            }
        sc.ntiles = (int64_t)tiles.size();
        // enough workgroups to fill the chip, each over >= 512 sparse words
        const int64_t target = (int64_t)ctx->cus * std::max<int64_t>(1, ctx->option(OPT_SPARSE_WG_PER_CU, 4));
        const int64_t budget = ctx->option(OPT_SPARSE_PART_BUDGET, int64_t(1) << 30);
        const int64_t tile_bytes = SB * SB * 2;
        // chunks that fold a dense-word slab (the first sp_fold_slabs) hold
        // at most kChunkWords - kFoldSlabWords words: every chunk does
        const int64_t cap = s->sp_fold_slabs ? kChunkWords - kFoldSlabWords : kChunkWords;
        // chunk bounds at equal word counts (n chunks)
        auto make_bounds = [&](int64_t n) {
            std::vector<int32_t> b;
            for (int64_t c = 0; c <= n; c++) b.push_back((int32_t)(s->Ws * c / n));
            return b;
        };
        // A chunk is exact when it holds <= kChunkWords words (64 x 1023 <
        // 2^16 whatever the sets) or when the SECOND largest set total of
        // complement bits over the buckets covering it is <= 65535 (one set
        // may hold more: a guide lacks every kmer the later guides key, C2's
        // sets 0-3); sp_bucket_bits holds the totals per set and bucket of
        // 1024 sparse words.
        auto bounds_ok = [&](const std::vector<int32_t>& b) {
            const int64_t N = s->nsets, nbk = s->sp_nbk;
            if ((int64_t)b.size() - 1 < s->sp_fold_slabs) return false;    // a chunk per slab
            for (size_t c = 0; c + 1 < b.size(); c++) {
                const int64_t b0 = b[c], b1 = b[c + 1];
                const int64_t fold = (int64_t)c < s->sp_fold_slabs ? 64 * kFoldSlabWords : 0;
                if (b1 - b0 <= cap) continue;
                if ((int64_t)s->sp_bucket_bits.size() != N * nbk) return false;
                int64_t m1 = 0, m2 = 0;
                for (int64_t i = 0; i < N; i++) {
                    int64_t t = 0;
                    for (int64_t k = b0 >> kBucketShift; k <= (b1 - 1) >> kBucketShift; k++)
                        t += s->sp_bucket_bits[i * nbk + k];
                    if (t > m1) { m2 = m1; m1 = t; } else if (t > m2) m2 = t;
                }
                if (m2 + fold > 65535) return false;
            }
            return true;
        };
        std::vector<int32_t> bnd;
        if (sc.ntiles) {
            int64_t n0 = std::max<int64_t>(std::max<int64_t>(ceil_div(s->Ws, cap), s->sp_fold_slabs),
                                           std::min<int64_t>(ceil_div(s->Ws, 512), ceil_div(target, sc.ntiles)));
            bnd = make_bounds(n0);
            // Past the partial budget (many tiles: N >> 1000), fewer and
            // longer chunks where the complement bits allow it (bounds_ok), so
            // that the partials fit; otherwise the chunks flush with atomics.
            const int64_t nb0 = (int64_t)bnd.size() - 1;
            if (sc.ntiles * nb0 * tile_bytes > budget) {
                for (int64_t fewer = std::max<int64_t>(1, budget / (sc.ntiles * tile_bytes)); fewer < nb0; fewer *= 2) {
                    auto b = make_bounds(fewer);
                    if (bounds_ok(b)) { bnd = b; break; }
                }
            }
            // XCD-mapped order (option sparse_xcd): whole groups of 8 chunks, so
            // every XCD gets the same number of chunks of every tile
            const int64_t nb1 = (int64_t)bnd.size() - 1;
            if (ctx->option(OPT_SPARSE_XCD, 0) != 0 && nb1 > 8 && nb1 % 8) {
                auto b = make_bounds(ceil_div(nb1, 8) * 8);
                if (bounds_ok(b)) bnd = b;
            }
            if (ctx->has_option(OPT_SPARSE_CHUNKS))   // tests: a given chunk count (exactness still checked)
                bnd = make_bounds(std::max<int64_t>(s->sp_fold_slabs,
                                                    std::max<int64_t>(1, std::min<int64_t>(s->Ws, ctx->option(OPT_SPARSE_CHUNKS, 1)))));
            GD_REQUIRE(bounds_ok(bnd), "sparse chunks exceed the 16-bit counter bound");
        }
        const int64_t nch = sc.ntiles ? (int64_t)bnd.size() - 1 : 0;
        sc.nchunks = (int)nch;
        if (sc.ntiles) {
            sc.tiles.alloc(sc.ntiles * sizeof(int2), st);
            h2d(sc.tiles.p, tiles.data(), sc.ntiles * sizeof(int2), st);
            sc.bounds.alloc(bnd.size() * 4, st);
            h2d(sc.bounds.p, bnd.data(), bnd.size() * 4, st);
        }
        // chunk partials (16-bit counters, 32 KiB per tile and chunk) within a
        // byte budget (option sparse_part_budget, default 1 GiB); past it the
        // chunks flush their counters with global atomics instead
        const int64_t part_bytes = sc.ntiles * sc.nchunks * tile_bytes;
        sc.use_part = sc.nchunks > 1 && part_bytes <= budget;
        if (sc.use_part) sc.part.alloc((size_t)part_bytes, st);
        if (ctx->trace())
            fprintf(stderr, "gdist: sparse plan rows [%lld,%lld) cols [%lld,%lld): %lld tiles x %d chunks, %s, "
                            "%lld of %lld sparse words positive\n",
                    (long long)r0, (long long)r1, (long long)c0, (long long)c1, (long long)sc.ntiles, sc.nchunks,
                    sc.use_part ? "partials" : "atomic flush", (long long)s->sp_pos_words,
                    (long long)s->Ws);
        GD_REQUIRE(sc.ntiles * sc.nchunks < (int64_t(1) << 31), "sparse grid too large");
        if (sc.use_part) rare_slab_plan(ctx, s, r0, r1, tiles, sc);
        sc.ready = true;
    }
}

GroupPart group_part(const gdist_sets* s) {
    GroupPart g;
    if (s->sp_groups > 0) {
        g.grp = s->sp_grp.as<int32_t>();
        g.V = s->sp_V.as<int32_t>();
        g.T = s->sp_T.as<int32_t>();
        g.m = (int)s->sp_groups;
        g.N = s->nsets;
    }
    return g;
}

bool sparse_matrix(gdist_ctx* ctx, const gdist_sets* s, int64_t r0, int64_t r1, int64_t c0, int64_t c1, bool upper,
                   int32_t* d_I, int64_t ldI, hipStream_t st, SparseScratch& sc, const SparseEpilogue* ep) {
    if (!s->sparse || r1 <= r0 || c1 <= c0) return false;
    sparse_plan(ctx, s, r0, r1, c0, c1, upper, st, sc);
    GD_REQUIRE(!ep || (sc.use_part && (s->n_rare == 0 || sc.rare_in)), "fused sparse epilogue without its plan");
    if (sc.ntiles == 0) return false;
    const int nchunks = sc.nchunks;
    const int64_t nt = sc.ntiles;
    // __launch_bounds__'s second argument is the minimum waves per SIMD: 8
    // holds the registers under the 8-wave budget (4 workgroups per CU,
    // LDS-limited; profiles/r01/sparse/occ_{3,8}.json)
    // 2 x 2 micro-tiles, 3 slots (12 products) per lane in flight; 1 x 2 with
    // 4 (C2 A/B, profiles/r04/s21/ab, r04/s13/ab_sun: 2 x 2 with 4 spills)
    const int mt = (int)ctx->option(OPT_SPARSE_MT, 2);
    const int sun = (int)ctx->option(OPT_SPARSE_SUN, mt == 2 ? 3 : 4);
    GD_REQUIRE(sun >= 2 && sun <= 4, "sparse_sun: 2, 3 or 4");
    GD_REQUIRE(mt == 1 || mt == 2, "sparse_mt: 1 (1 x 2 micro-tiles) or 2 (2 x 2)");
    auto kern = mt == 2 ? (sun == 2 ? sparse_tile_kernel<2, 2> : sun == 4 ? sparse_tile_kernel<4, 2> : sparse_tile_kernel<3, 2>)
                        : (sun == 2 ? sparse_tile_kernel<2, 1> : sun == 4 ? sparse_tile_kernel<4, 1> : sparse_tile_kernel<3, 1>);
    // the rare tier's pairs of this step: the launch's trailing workgroups
    const bool rare = sc.use_part && sc.rare_in;
    FamilyTimer ft(ctx, GDIST_KERNEL_SPARSE, st);
    const bool xmap = ctx->option(OPT_SPARSE_XCD, 0) != 0;
    RareSlab rs;
    if (rare) {
        rs.rr = rare_rows_of(s);
        rs.nch = (int)ceil_div(c1 - c0, kRareChunkCols);
        const int64_t nrare = (r1 - r0) * rs.nch;
        GD_REQUIRE(nrare < (int64_t(1) << 30), "too many rare rows");
        rs.nrare = (int)nrare;
        rs.slab = sc.rare_slab.as<uint32_t>();
        rs.tile_of = sc.rare_tile.as<int32_t>();
        rs.ab0 = sc.rare_ab0;
        rs.nbc = sc.rare_nbc;
    }
    const int64_t grid = (xmap ? ceil_div(nchunks, 8) * 8 * nt : nt * nchunks) + rs.nrare;
    GD_REQUIRE(grid < (int64_t(1) << 31), "sparse grid too large");
    kern<<<(unsigned)grid, SNT, 0, st>>>(s->sp_off.as<int64_t>(), s->sp_ent.as<ulonglong2>(), s->sp_nc.as<int32_t>(),
                                         s->sp_U, s->Ws, sc.tiles.as<int2>(), sc.bounds.as<int32_t>(), nchunks, r0, r1,
                                         c0, c1, upper ? 1 : 0, d_I, ldI, sc.use_part ? sc.part.as<int32_t>() : nullptr,
                                         s->Wd, s->nsets, s->dbits.as<unsigned long long>(), s->sp_fold_slabs,
                                         group_part(s), xmap ? 1 : 0, (int)nt, rs,
                                         (int)ctx->option(OPT_SPARSE_DYN, 1), (int)ctx->option(OPT_SPARSE_DIAG22, 1),
                                         (int)ctx->option(OPT_SPARSE_RPART22, 1));
    GD_HIP(hipGetLastError());
    ft.end();
    if (sc.use_part) {
        sparse_reduce_kernel<<<(unsigned)(nt * (SB * SB / kReduceCnt / kReduceGroups)), 256, 0, st>>>(
            sc.part.as<int32_t>(), nchunks, sc.tiles.as<int2>(), s->sp_nc.as<int32_t>(), s->sp_U, r0, r1, c0, c1,
            upper ? 1 : 0, d_I, ldI,
            rare ? sc.rare_slab.as<uint32_t>() : nullptr, ep ? ep->D : nullptr, ep ? ep->ldD : 0,
            ep ? ep->off : nullptr, ep ? ep->empty_nan : 0, group_part(s));
        GD_HIP(hipGetLastError());
    }
    return sc.use_part && sc.rare_in;
}

}  // namespace gdist
