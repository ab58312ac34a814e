/*
 * gdist_oracle.c — CPU restatement of the SEEDtk genome.distance kmer-distance
 * path (TEST INFRASTRUCTURE: checker and CPU baseline only, never the product).
 *
 * PARITY UNPINNED: the reference arithmetic is in the absent
 * org.theseed:sequence module; this file follows the call-site contracts cited
 * below and the packing spec of include/gdist.h, and is pinned against the
 * independent Python string-set restatement oracle/pyref.py via tests/golden/.
 */
#include "gdist_oracle.h"
#include "../include/gdist.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ */
/* alphabet                                                             */

static inline unsigned char fold_upper(unsigned char c) {
    return (c >= 'a' && c <= 'z') ? (unsigned char)(c - 32) : c;
}

/* 2-bit DNA (ASCII order A<C<G<T). */
static inline int dna2_sym(unsigned char c) {
    switch (c) { case 'A': return 0; case 'C': return 1; case 'G': return 2; case 'T': return 3; }
    return -1;
}
/* 3-bit DNA keep alphabet in ASCII order: A0 C1 G2 N3 R4 T5 Y6. */
static inline int dna3_sym(unsigned char c) {
    switch (c) {
    case 'A': return 0; case 'C': return 1; case 'G': return 2; case 'N': return 3;
    case 'R': return 4; case 'T': return 5; case 'Y': return 6;
    }
    return -1;
}
static const int dna3_comp[7] = {5, 2, 1, 3, 6, 0, 4};
static const char dna2_chr[4] = {'A', 'C', 'G', 'T'};
static const char dna3_chr[7] = {'A', 'C', 'G', 'N', 'R', 'T', 'Y'};

static inline int prot5_sym(unsigned char c) {
    if (c == '*') return 0;
    if (c >= 'A' && c <= 'Z') return 1 + (c - 'A');
    return -1;
}
static inline int prot_standard(unsigned char c) {
    return strchr("ACDEFGHIKLMNPQRSTVWY", c) != NULL && c != 0;
}

static int cmp_u64(const void* a, const void* b) {
    uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return (x > y) - (x < y);
}
static int cmp_i32(const void* a, const void* b) {
    int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
    return (x > y) - (x < y);
}

/* LSD radix sort of u64 keys, 8 bits a pass; passes whose byte is the same
 * in every key are skipped (DNA k=21 codes: 6 of 8). Any correct sort gives
 * the same set; this one only makes the checker's full-size columns fast
 * (qsort's comparator calls were ~10 ms a 200 K-kmer genome). */
static void radix_sort_u64(uint64_t* v, int64_t n) {
    /* the scratch is per thread and kept (a fresh 1.6 MB block a call is an
     * mmap + page faults, serialised across the checker's threads) */
    static __thread uint64_t* tmp = NULL;
    static __thread int64_t cap = 0;
    if (n > cap) {
        free(tmp);
        cap = n + n / 4;
        tmp = (uint64_t*)malloc((size_t)cap * sizeof(uint64_t));
        if (!tmp) { cap = 0; qsort(v, (size_t)n, sizeof(uint64_t), cmp_u64); return; }
    }
    uint64_t* src = v;
    uint64_t* dst = tmp;
    for (int sh = 0; sh < 64; sh += 8) {
        int64_t cnt[256];
        memset(cnt, 0, sizeof(cnt));
        for (int64_t i = 0; i < n; i++) cnt[(src[i] >> sh) & 255]++;
        if (cnt[(src[0] >> sh) & 255] == n) continue;     /* one byte value: nothing moves */
        int64_t sum = 0;
        for (int b = 0; b < 256; b++) { int64_t c = cnt[b]; cnt[b] = sum; sum += c; }
        for (int64_t i = 0; i < n; i++) dst[cnt[(src[i] >> sh) & 255]++] = src[i];
        uint64_t* t = src; src = dst; dst = t;
    }
    if (src != v) memcpy(v, src, (size_t)n * sizeof(uint64_t));
}

static int64_t sort_unique(uint64_t* v, int64_t n) {
    if (n <= 1) return n;
    if (n >= 4096) radix_sort_u64(v, n);
    else qsort(v, (size_t)n, sizeof(uint64_t), cmp_u64);
    int64_t w = 1;
    for (int64_t i = 1; i < n; i++)
        if (v[i] != v[w - 1]) v[w++] = v[i];
    return w;
}

/* Effective ambiguity mode per kind (gdist.h: DNA default skip, PROT keep). */
static int ambig_skip(int kind, unsigned flags) {
    unsigned m = flags & GDIST_AMBIG_MASK;
    if (m == GDIST_AMBIG_SKIP) return 1;
    if (m == GDIST_AMBIG_KEEP) return 0;
    return kind == GDIST_DNA;
}

/* ------------------------------------------------------------------ */
/* kmer codes — KmerType.createKmers(seq, K) (FastaDistanceProcessor.java:153,184),
 * new GenomeKmers(genome) (GenomeProcessor.java:109), new ProteinKmers(seq)
 * (ProteinKmerReader.java:101). Set semantics: every length-k substring, once. */

int64_t or_kmer_codes(int kind, int k, unsigned flags, const char* seq, int64_t len, uint64_t* out) {
    if (k < 1) return -1;
    int64_t n = 0;
    if (kind == GDIST_DNA) {
        int skip = ambig_skip(kind, flags);
        unsigned strand = flags & GDIST_STRAND_MASK;
        int bits = skip ? 2 : 3;
        if ((skip && k > 32) || (!skip && k > 21)) return -1;
        uint64_t mask = (k * bits >= 64) ? ~0ULL : ((1ULL << (k * bits)) - 1);
        uint64_t fwd = 0, rc = 0;
        int64_t valid_run = 0;   /* consecutive encodable chars ending here */
        for (int64_t i = 0; i < len; i++) {
            unsigned char c = fold_upper((unsigned char)seq[i]);
            if (c == 0) { valid_run = 0; fwd = 0; rc = 0; continue; }   /* separator */
            int s = skip ? dna2_sym(c) : dna3_sym(c);
            if (s < 0) {
                if (!skip) return -1;   /* keep mode: unencodable char */
                valid_run = 0; fwd = 0; rc = 0;
                continue;
            }
            int cs = skip ? (3 - s) : dna3_comp[s];
            fwd = ((fwd << bits) | (uint64_t)s) & mask;
            rc = (rc >> bits) | ((uint64_t)cs << (bits * (k - 1)));
            valid_run++;
            if (valid_run >= k) {
                if (strand == GDIST_STRAND_FWD) out[n++] = fwd;
                else if (strand == GDIST_STRAND_CANON) out[n++] = fwd < rc ? fwd : rc;
                else { out[n++] = fwd; out[n++] = rc; }
            }
        }
    } else if (kind == GDIST_PROT) {
        if (k > 12) return -1;
        int skip = ambig_skip(kind, flags);
        int fold = !(flags & GDIST_NO_CASE_FOLD);
        int bits = (k <= 8) ? 8 : 5;
        uint64_t mask = (k * bits >= 64) ? ~0ULL : ((1ULL << (k * bits)) - 1);
        uint64_t code = 0;
        int64_t run = 0;
        for (int64_t i = 0; i < len; i++) {
            unsigned char c = (unsigned char)seq[i];
            if (fold) c = fold_upper(c);
            if (c == 0) { run = 0; code = 0; continue; }                  /* separator */
            if (skip && !prot_standard(c)) { run = 0; code = 0; continue; }
            int s;
            if (bits == 8) s = c;
            else { s = prot5_sym(c); if (s < 0) return -1; }
            code = ((code << bits) | (uint64_t)s) & mask;
            run++;
            if (run >= k) out[n++] = code;
        }
    } else {
        return -1;
    }
    return sort_unique(out, n);
}

int or_decode_kmer(int kind, int k, unsigned flags, uint64_t code, char* out) {
    if (kind == GDIST_DNA) {
        int skip = ambig_skip(kind, flags);
        int bits = skip ? 2 : 3;
        for (int i = 0; i < k; i++) {
            unsigned s = (unsigned)((code >> (bits * (k - 1 - i))) & ((1u << bits) - 1));
            out[i] = skip ? dna2_chr[s] : dna3_chr[s < 7 ? s : 3];
        }
    } else {
        int bits = (k <= 8) ? 8 : 5;
        for (int i = 0; i < k; i++) {
            unsigned s = (unsigned)((code >> (bits * (k - 1 - i))) & ((1u << bits) - 1));
            out[i] = (bits == 8) ? (char)s : (s == 0 ? '*' : (char)('A' + s - 1));
        }
    }
    out[k] = 0;
    return k;
}

/* ------------------------------------------------------------------ */
/* SequenceKmers.similarity / distance (inferred) */

int64_t or_intersect(const uint64_t* a, int64_t na, const uint64_t* b, int64_t nb) {
    int64_t i = 0, j = 0, c = 0;
    while (i < na && j < nb) {
        if (a[i] < b[j]) i++;
        else if (b[j] < a[i]) j++;
        else { c++; i++; j++; }
    }
    return c;
}

double or_distance(int64_t inter, int64_t na, int64_t nb, unsigned flags) {
    if (inter > 0) {
        double uni = (double)(na + nb - inter);
        return 1.0 - (double)inter / uni;
    }
    if (na + nb == 0 && (flags & GDIST_EMPTY_NAN)) return NAN;
    return 1.0;
}

/* ------------------------------------------------------------------ */
/* Java Double.toString (JDK 21): shortest decimal that rounds to d, closest
 * to d; when that is one digit long, the closest two-digit decimal.
 * Layout: plain for 1e-3 <= |d| < 1e7 (at least one fraction digit), else
 * d.dddE[-]n. Used at FastaDistanceProcessor.java:189-190,
 * GenomeProcessor.java:144, DistanceRepsProcessor.java:250-251. */
int or_java_dtoa(double d, char* buf) {
    if (isnan(d)) return sprintf(buf, "NaN");
    if (isinf(d)) return sprintf(buf, d > 0 ? "Infinity" : "-Infinity");
    if (d == 0.0) return sprintf(buf, signbit(d) ? "-0.0" : "0.0");
    char tmp[64];
    int p;
    for (p = 1; p <= 17; p++) {
        snprintf(tmp, sizeof tmp, "%.*e", p - 1, d);
        if (strtod(tmp, NULL) == d) break;
    }
    if (p == 1) snprintf(tmp, sizeof tmp, "%.1e", d);
    /* parse [-]D[.DDD]e[+-]XX */
    const char* s = tmp;
    int neg = 0;
    if (*s == '-') { neg = 1; s++; }
    char dig[32];
    int nd = 0;
    while (*s && *s != 'e') { if (*s != '.') dig[nd++] = *s; s++; }
    int e = atoi(s + 1);
    while (nd > 1 && dig[nd - 1] == '0') nd--;
    dig[nd] = 0;
    char* o = buf;
    if (neg) *o++ = '-';
    double a = fabs(d);
    if (a >= 1e-3 && a < 1e7) {
        if (e >= 0) {
            for (int i = 0; i <= e; i++) *o++ = (i < nd) ? dig[i] : '0';
            *o++ = '.';
            if (nd > e + 1) for (int i = e + 1; i < nd; i++) *o++ = dig[i];
            else *o++ = '0';
        } else {
            *o++ = '0'; *o++ = '.';
            for (int i = 0; i < -e - 1; i++) *o++ = '0';
            for (int i = 0; i < nd; i++) *o++ = dig[i];
        }
    } else {
        *o++ = dig[0]; *o++ = '.';
        if (nd > 1) for (int i = 1; i < nd; i++) *o++ = dig[i];
        else *o++ = '0';
        o += sprintf(o, "E%d", e);
    }
    *o = 0;
    return (int)(o - buf);
}

/* ------------------------------------------------------------------ */
/* MinHash sketches — SequenceKmers.hashSet(width) (SketchProcessor.java:88,
 * WidthProcessor.java:178) and Sketch.distance (WidthProcessor.java:185).
 * Hash function and distance formula are unpinned. */

static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

uint32_t or_murmur3_32(const uint8_t* data, int len, uint32_t seed) {
    const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
    uint32_t h = seed;
    int nblocks = len / 4;
    for (int i = 0; i < nblocks; i++) {
        uint32_t k = (uint32_t)data[4 * i] | ((uint32_t)data[4 * i + 1] << 8) |
                     ((uint32_t)data[4 * i + 2] << 16) | ((uint32_t)data[4 * i + 3] << 24);
        k *= c1; k = rotl32(k, 15); k *= c2;
        h ^= k; h = rotl32(h, 13); h = h * 5 + 0xe6546b64u;
    }
    const uint8_t* tail = data + 4 * nblocks;
    uint32_t k1 = 0;
    switch (len & 3) {
    case 3: k1 ^= (uint32_t)tail[2] << 16; /* fallthrough */
    case 2: k1 ^= (uint32_t)tail[1] << 8;  /* fallthrough */
    case 1: k1 ^= tail[0];
            k1 *= c1; k1 = rotl32(k1, 15); k1 *= c2; h ^= k1;
    }
    h ^= (uint32_t)len;
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}

int64_t or_sketch(int kind, int k, unsigned flags, const uint64_t* codes, int64_t n, int width, int32_t* out) {
    if (width <= 0) return 0;
    int32_t* h = (int32_t*)malloc((size_t)(n > 0 ? n : 1) * sizeof(int32_t));
    char kmer[40];
    for (int64_t i = 0; i < n; i++) {
        or_decode_kmer(kind, k, flags, codes[i], kmer);
        h[i] = (int32_t)or_murmur3_32((const uint8_t*)kmer, k, 0);
    }
    qsort(h, (size_t)n, sizeof(int32_t), cmp_i32);
    int64_t m = 0;
    for (int64_t i = 0; i < n && m < width; i++)
        if (m == 0 || h[i] != out[m - 1]) out[m++] = h[i];
    free(h);
    return m;
}

double or_sketch_distance(const int32_t* a, int64_t na, const int32_t* b, int64_t nb,
                          int width, unsigned flags, int64_t* common_out) {
    int64_t i = 0, j = 0, common = 0;
    if (flags & GDIST_SKETCH_JACCARD) {
        while (i < na && j < nb) {
            if (a[i] < b[j]) i++;
            else if (b[j] < a[i]) j++;
            else { common++; i++; j++; }
        }
        if (common_out) *common_out = common;
        return or_distance(common, na, nb, flags);
    }
    int64_t taken = 0;
    while (taken < width && (i < na || j < nb)) {
        if (j >= nb || (i < na && a[i] < b[j])) i++;
        else if (i >= na || b[j] < a[i]) j++;
        else { common++; i++; j++; }
        taken++;
    }
    if (common_out) *common_out = common;
    if (common > 0) return 1.0 - (double)common / (double)taken;
    if (taken == 0 && (flags & GDIST_EMPTY_NAN)) return NAN;
    return 1.0;
}

/* ------------------------------------------------------------------ */
/* optimised CPU all-pairs (sorted merge, OpenMP over rows) */

void or_matrix(const int64_t* off, const uint64_t* codes,
               int64_t r0, int64_t r1, int64_t c0, int64_t c1, unsigned flags,
               int32_t* I_out, double* D_out, int64_t ld, int nthreads) {
    int upper = (flags & GDIST_UPPER_TRIANGLE) != 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int64_t i = r0; i < r1; i++) {
        const uint64_t* a = codes + off[i];
        int64_t na = off[i + 1] - off[i];
        for (int64_t j = c0; j < c1; j++) {
            if (upper && j <= i) continue;
            const uint64_t* b = codes + off[j];
            int64_t nb = off[j + 1] - off[j];
            int64_t I = or_intersect(a, na, b, nb);
            int64_t idx = (i - r0) * ld + (j - c0);
            if (I_out) I_out[idx] = (int32_t)I;
            if (D_out) D_out[idx] = or_distance(I, na, nb, flags);
        }
    }
    (void)nthreads;
}

/* Rows of a collection too large to pack on the host (C4: 100,000 x 100 kbp
 * = 160 GB of codes) against every column: column j's codes are extracted
 * from blob[coff[j], coff[j+1]) by or_kmer_codes, counted (sizes[j]) and
 * intersected with each of the nrows row sets (CSR roff / rcodes), OpenMP
 * over columns; inter[r * ncols + j]. Returns 0, or -1 on unencodable
 * input. The pair loop of FastaDistanceProcessor.java:157-186 for a few
 * rows, the columns streamed. */
int or_rows_vs_columns(int kind, int k, unsigned flags, const char* blob, const int64_t* coff, int64_t ncols,
                       const int64_t* roff, const uint64_t* rcodes, int64_t nrows, int64_t* inter,
                       int64_t* sizes, int nthreads) {
    int bad = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
    {
        int64_t cap = 0;
        uint64_t* buf = NULL;
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 16)
#endif
        for (int64_t j = 0; j < ncols; j++) {
            const int64_t len = coff[j + 1] - coff[j];
            if (2 * len + 1 > cap) {
                free(buf);
                cap = 2 * len + 1;
                buf = (uint64_t*)malloc((size_t)cap * sizeof(uint64_t));
            }
            const int64_t nb = buf ? or_kmer_codes(kind, k, flags, blob + coff[j], len, buf) : -1;
            if (nb < 0) { bad = 1; continue; }
            sizes[j] = nb;
            for (int64_t r = 0; r < nrows; r++)
                inter[r * ncols + j] = or_intersect(rcodes + roff[r], roff[r + 1] - roff[r], buf, nb);
        }
        free(buf);
    }
    (void)nthreads;
    return bad ? -1 : 0;
}

/* ------------------------------------------------------------------ */
/* Java-faithful path: HashSet<String> of substring kmers.
 * String.hashCode = s[0]*31^(n-1) + ... (int arithmetic); HashMap spreads
 * h ^ (h >>> 16), power-of-two table, load factor 0.75, chained buckets. */

typedef struct { int32_t hash; int32_t next; int64_t off; } jnode;
typedef struct {
    int32_t* table; int32_t cap;
    jnode* nodes; int32_t n, ncap;
    char* arena; int64_t asz, acap;
    int k;
} jset;

static int32_t jstring_hash(const char* s, int k) {
    int32_t h = 0;
    for (int i = 0; i < k; i++) h = (int32_t)((uint32_t)h * 31u + (uint32_t)(unsigned char)s[i]);
    return h;
}
static inline int32_t jspread(int32_t h) { return h ^ (int32_t)((uint32_t)h >> 16); }

static void jset_init(jset* s, int k) {
    s->cap = 16; s->table = (int32_t*)malloc(16 * sizeof(int32_t));
    for (int i = 0; i < 16; i++) s->table[i] = -1;
    s->ncap = 1024; s->n = 0; s->nodes = (jnode*)malloc(1024 * sizeof(jnode));
    s->acap = 1024 * (int64_t)k; s->asz = 0; s->arena = (char*)malloc((size_t)s->acap);
    s->k = k;
}
static void jset_free(jset* s) { free(s->table); free(s->nodes); free(s->arena); }

static void jset_resize(jset* s) {
    int32_t ncap = s->cap * 2;
    int32_t* t = (int32_t*)malloc((size_t)ncap * sizeof(int32_t));
    for (int32_t i = 0; i < ncap; i++) t[i] = -1;
    /* re-link in insertion order (tail insertion keeps Java's bucket order) */
    int32_t* tail = (int32_t*)malloc((size_t)ncap * sizeof(int32_t));
    for (int32_t i = 0; i < ncap; i++) tail[i] = -1;
    for (int32_t x = 0; x < s->n; x++) {
        int32_t b = jspread(s->nodes[x].hash) & (ncap - 1);
        s->nodes[x].next = -1;
        if (tail[b] < 0) t[b] = x; else s->nodes[tail[b]].next = x;
        tail[b] = x;
    }
    free(tail); free(s->table);
    s->table = t; s->cap = ncap;
}

static int jset_contains(const jset* s, const char* kmer, int32_t h) {
    int32_t b = jspread(h) & (s->cap - 1);
    for (int32_t x = s->table[b]; x >= 0; x = s->nodes[x].next)
        if (s->nodes[x].hash == h && memcmp(s->arena + s->nodes[x].off, kmer, (size_t)s->k) == 0) return 1;
    return 0;
}

static void jset_add(jset* s, const char* sub) {
    /* Java: new String(substring) is allocated before the probe */
    char kmer[64];
    memcpy(kmer, sub, (size_t)s->k);
    int32_t h = jstring_hash(kmer, s->k);
    int32_t b = jspread(h) & (s->cap - 1);
    int32_t last = -1;
    for (int32_t x = s->table[b]; x >= 0; x = s->nodes[x].next) {
        if (s->nodes[x].hash == h && memcmp(s->arena + s->nodes[x].off, kmer, (size_t)s->k) == 0) return;
        last = x;
    }
    if (s->n == s->ncap) { s->ncap *= 2; s->nodes = (jnode*)realloc(s->nodes, (size_t)s->ncap * sizeof(jnode)); }
    if (s->asz + s->k > s->acap) { s->acap *= 2; s->arena = (char*)realloc(s->arena, (size_t)s->acap); }
    memcpy(s->arena + s->asz, kmer, (size_t)s->k);
    jnode* nd = &s->nodes[s->n];
    nd->hash = h; nd->next = -1; nd->off = s->asz;
    s->asz += s->k;
    if (last < 0) s->table[b] = s->n; else s->nodes[last].next = s->n;
    s->n++;
    if (s->n > (int32_t)(0.75 * s->cap)) jset_resize(s);
}

static int dna_valid(unsigned char c, int skip) { return skip ? dna2_sym(c) >= 0 : 1; }
static char dna_comp_chr(char c) {
    switch (c) { case 'A': return 'T'; case 'T': return 'A'; case 'C': return 'G'; case 'G': return 'C';
                 case 'R': return 'Y'; case 'Y': return 'R'; }
    return c;
}

/* KmerType.createKmers restated on Strings */
static void jset_build(jset* s, int kind, int k, unsigned flags, const char* seq, int64_t len) {
    jset_init(s, k);
    if (len < k) return;
    char* f = (char*)malloc((size_t)len + 1);
    int fold = kind == GDIST_DNA || !(flags & GDIST_NO_CASE_FOLD);
    for (int64_t i = 0; i < len; i++) f[i] = fold ? (char)fold_upper((unsigned char)seq[i]) : seq[i];
    int skip = ambig_skip(kind, flags);
    unsigned strand = flags & GDIST_STRAND_MASK;
    char rc[64];
    for (int64_t i = 0; i + k <= len; i++) {
        const char* w = f + i;
        int ok = 1;
        if (memchr(w, 0, (size_t)k)) continue;                            /* separator */
        if (skip) for (int t = 0; t < k; t++) {
            unsigned char c = (unsigned char)w[t];
            if (kind == GDIST_DNA ? !dna_valid(c, 1) : !prot_standard(c)) { ok = 0; break; }
        }
        if (!ok) continue;
        if (kind == GDIST_DNA && strand != GDIST_STRAND_FWD) {
            for (int t = 0; t < k; t++) rc[t] = dna_comp_chr(w[k - 1 - t]);
            if (strand == GDIST_STRAND_CANON) jset_add(s, memcmp(w, rc, (size_t)k) <= 0 ? w : rc);
            else { jset_add(s, w); jset_add(s, rc); }
        } else {
            jset_add(s, w);
        }
    }
    free(f);
}

static double jset_distance(const jset* a, const jset* b, unsigned flags) {
    int64_t sim = 0;
    for (int32_t x = 0; x < b->n; x++)
        if (jset_contains(a, b->arena + b->nodes[x].off, b->nodes[x].hash)) sim++;
    return or_distance(sim, a->n, b->n, flags);
}

int64_t or_faithful_fasta_dist(int kind, int k, unsigned flags,
                               const char* seqs, const int64_t* seq_off, int64_t n,
                               int batch, int64_t max_rows, double* D_out, int nthreads) {
    if (batch < 1) batch = 1;
    if (max_rows <= 0 || max_rows > n) max_rows = n;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    int64_t pairs = 0;
    int64_t first = 0;             /* list = [first, n) — FastaDistanceProcessor.java:141,161 */
    jset* cache = (jset*)calloc((size_t)batch, sizeof(jset));
    while (first < n && first < max_rows) {
        int64_t remaining = n - first;
        int64_t bsize = batch < remaining ? batch : remaining;   /* :146-149 */
        int64_t rows = bsize;                                     /* bounded sample */
        if (first + rows > max_rows) rows = max_rows - first;
        for (int64_t i = 0; i < bsize; i++)                       /* :151-155 */
            jset_build(&cache[i], kind, k, flags, seqs + seq_off[first + i],
                       seq_off[first + i + 1] - seq_off[first + i]);
        int64_t batch_pairs = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) reduction(+:batch_pairs)
#endif
        for (int64_t i = 0; i < rows; i++) {                      /* :157-158 */
            for (int64_t jdx = i + 1; jdx < remaining; jdx++) {   /* :177 */
                int64_t j = first + jdx;
                jset tmp;
                const jset* s2;
                if (jdx < batch) s2 = &cache[jdx];                /* :181-182 */
                else {                                            /* :184 rebuilt per pair */
                    jset_build(&tmp, kind, k, flags, seqs + seq_off[j], seq_off[j + 1] - seq_off[j]);
                    s2 = &tmp;
                }
                double d = jset_distance(&cache[i], s2, flags);   /* :186 */
                if (D_out) D_out[(first + i) * n + j] = d;
                if (s2 == &tmp) jset_free(&tmp);
                batch_pairs++;
            }
        }
        pairs += batch_pairs;
        for (int64_t i = 0; i < bsize; i++) jset_free(&cache[i]);
        first += bsize;                                           /* :161 */
    }
    free(cache);
    return pairs;
}
