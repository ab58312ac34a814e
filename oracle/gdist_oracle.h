/*
 * gdist_oracle.h — CPU restatement of the reference's kmer-distance path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load liboracle.so, and only as the checker
 * or the timed CPU baseline — never as the product path.
 *
 * PARITY UNPINNED: the arithmetic of the reference path lives in the
 * un-vendored org.theseed:sequence:1.0.0 module (pom.xml:46-49) and no JVM
 * exists in this container, so neither the reference nor any reference test
 * vector can pin this restatement. It follows the in-repo call
 * sites cited per function, the packing spec in include/gdist.h, and is
 * cross-checked bit-for-bit against an independent pure-Python string-set
 * restatement (oracle/pyref.py) on the committed fixtures in tests/golden/.
 */
#ifndef GDIST_ORACLE_H
#define GDIST_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Kmer codes of one sequence, sorted ascending and unique.
 * out must hold 2*len codes. Returns the count, or -1 (unencodable input,
 * bad k) — mirrors KmerType.createKmers (FastaDistanceProcessor.java:153). */
int64_t or_kmer_codes(int kind, int k, unsigned flags, const char* seq, int64_t len, uint64_t* out);

/* |A ∩ B| of two sorted unique code arrays (SequenceKmers.similarity, inferred). */
int64_t or_intersect(const uint64_t* a, int64_t na, const uint64_t* b, int64_t nb);

/* Java expression of SequenceKmers.distance (FastaDistanceProcessor.java:186). */
double or_distance(int64_t inter, int64_t na, int64_t nb, unsigned flags);

/* Java Double.toString (JDK 19+ shortest-uniquely-identifying; JDK 21 per pom.xml:17).
 * Returns the length written into buf (>= 32 bytes). */
int or_java_dtoa(double d, char* buf);

/* MurmurHash3_x86_32 (Appleby, public domain algorithm). */
uint32_t or_murmur3_32(const uint8_t* data, int len, uint32_t seed);

/* Decode a code back to its k-char kmer string (folded case). */
int or_decode_kmer(int kind, int k, unsigned flags, uint64_t code, char* out);

/* SequenceKmers.hashSet(width) restatement: bottom-width distinct signed
 * murmur3 hashes of the kmer strings, ascending. Returns the count. */
int64_t or_sketch(int kind, int k, unsigned flags, const uint64_t* codes, int64_t n, int width, int32_t* out);

/* Sketch.distance restatement (default Mash bottom-s of the union,
 * GDIST_SKETCH_JACCARD for plain signature Jaccard). */
double or_sketch_distance(const int32_t* a, int64_t na, const int32_t* b, int64_t nb,
                          int width, unsigned flags, int64_t* common_out);

/* All-pairs over a CSR collection: I and D for rows [r0,r1) x cols [c0,c1),
 * optional upper triangle; sorted-merge, OpenMP over rows (optimised CPU). */
void or_matrix(const int64_t* off, const uint64_t* codes,
               int64_t r0, int64_t r1, int64_t c0, int64_t c1, unsigned flags,
               int32_t* I_out, double* D_out, int64_t ld, int nthreads);

/* A few row sets against every column of a byte collection, the columns'
 * codes extracted on the fly (a collection too large to pack on the host):
 * inter[r * ncols + j] = |row r ∩ codes(column j)|, sizes[j] = |codes(j)|. */
int or_rows_vs_columns(int kind, int k, unsigned flags, const char* blob, const int64_t* coff, int64_t ncols,
                       const int64_t* roff, const uint64_t* rcodes, int64_t nrows, int64_t* inter,
                       int64_t* sizes, int nthreads);

/* Java-faithful CPU path: HashSet<String> kmer sets (String.hashCode,
 * HashMap spreading/resizing) and the FastaDistanceProcessor loop
 * (FastaDistanceProcessor.java:141-194): batches of `batch` cached sets,
 * rows of a batch in parallel, sets beyond the cache rebuilt per pair.
 * Runs only rows [0, max_rows) of the first batches. D_out is n x n
 * row-major (upper triangle written). Returns the number of pairs. */
int64_t or_faithful_fasta_dist(int kind, int k, unsigned flags,
                               const char* seqs, const int64_t* seq_off, int64_t n,
                               int batch, int64_t max_rows, double* D_out, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
