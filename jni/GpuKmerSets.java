package org.theseed.genome.distance.gpu;

/**
 * Java side of jni/gdist_jni.c: a collection of kmer sets resident on one
 * MI355X (libgdist.so, include/gdist.h). What it replaces in the reference:
 * KmerType.createKmers / new GenomeKmers / new ProteinKmers (pack),
 * SequenceKmers.distance over row blocks (distances: FastaDistanceProcessor
 * and GenomeProcessor loops), anyMatch / argmin row queries
 * (DistanceRepsProcessor), hashSet(width) + Sketch.distance (WidthProcessor).
 * Callers batch: one call per row block, group or matrix, never per pair.
 */
public final class GpuKmerSets implements AutoCloseable {
    static { System.loadLibrary("gdist_jni"); }

    public static final int DNA = 0, PROT = 1;
    public static final int METHOD_AUTO = 0, METHOD_SORTED = 1, METHOD_BITSET = 2;
    public static final int UPPER_TRIANGLE = 0x100;

    static native long nCtxCreate(int device);
    static native void nCtxDestroy(long ctx);
    static native void nSetOption(long ctx, String name, long value);
    static native long nPack(long ctx, int kind, int k, int flags, byte[][] seqs);
    static native long nAppend(long ctx, long sets, byte[][] seqs);
    static native long nConcat(long a, long b);
    static native void nFree(long sets);
    static native long nSize(long sets);
    static native void nSizes(long sets, long[] out);
    static native void nBuildBitsets(long sets, int flags);
    static native int nPrepare(long ctx, long sets, int method, double pairs);
    static native void nMatrix(long ctx, long sets, long r0, long r1, long c0, long c1, int method, int flags,
                               double[] out, int ld);
    static native boolean nAnyLe(long ctx, long sets, long q, long[] cols, double t);
    static native int nArgmin(long ctx, long sets, long q, long[] cols, double[] bestD);
    static native void nRow(long ctx, long sets, long q, long[] cols, double[] out);
    static native long nGreedyReps(long ctx, long sets, double t, long[] tieRank, int[] isRep, long[] repOf,
                                   double[] repDist);
    static native long nSketch(long ctx, long sets, int width);
    static native long nTotal(long sets);
    static native void nSketchDownload(long sk, long[] off, int[] sigs);
    static native long nSketchUpload(long ctx, int width, long[] off, int[] sigs);
    static native void nSketchMatrix(long ctx, long sk, long r0, long r1, long c0, long c1, int flags,
                                     double[] out, int ld);

    /** One device context (gdist_ctx): serialises its calls, shared by threads. */
    public static final class Context implements AutoCloseable {
        final long h;
        public Context(int device) { this.h = nCtxCreate(device); }
        /** a tuning option (gdist_ctx_set_option); results never change */
        public void setOption(String name, long value) { nSetOption(h, name, value); }
        @Override public void close() { nCtxDestroy(h); }
    }

    private final long ctx;
    private long handle;

    /** kmer sets of `seqs` (KmerType.createKmers(seq, k) for each), packed on the device. */
    public GpuKmerSets(long ctx, int kind, int k, byte[][] seqs) {
        this.ctx = ctx;
        this.handle = nPack(ctx, kind, k, 0, seqs);
    }

    public GpuKmerSets(Context ctx, int kind, int k, byte[][] seqs) { this(ctx.h, kind, k, seqs); }

    private GpuKmerSets(long ctx, long handle) {
        this.ctx = ctx;
        this.handle = handle;
    }

    /** kmer sets of `seqs` packed with this collection's spec and appended
     *  (gdist_sets_append); returns the index of the first new set */
    public long append(byte[][] seqs) { return nAppend(ctx, handle, seqs); }

    /** a new collection: this one's sets, then other's (gdist_sets_concat; codes
     *  copied on the device, nothing re-packed) */
    public GpuKmerSets concat(GpuKmerSets other) { return new GpuKmerSets(ctx, nConcat(handle, other.handle)); }

    /** the number of sets */
    public long size() { return nSize(handle); }

    /** SequenceKmers.size() of every set */
    public long[] sizes() {
        long[] out = new long[(int) size()];
        nSizes(handle, out);
        return out;
    }

    /** the two-tier bitsets now (otherwise the first distance call decides, METHOD_AUTO) */
    public void buildBitsets() { nBuildBitsets(handle, 0); }

    /** the representation METHOD_AUTO picks for `pairs` pairs (METHOD_BITSET / METHOD_SORTED) */
    public int prepare(double pairs) { return nPrepare(ctx, handle, METHOD_AUTO, pairs); }

    /** distances of rows [r0, r1) x columns [c0, c1), row-major with stride ld */
    public void distances(long r0, long r1, long c0, long c1, boolean upperTriangle, double[] out, int ld) {
        nMatrix(ctx, handle, r0, r1, c0, c1, METHOD_AUTO, upperTriangle ? UPPER_TRIANGLE : 0, out, ld);
    }

    /** anyMatch(d <= maxDist) of set q against cols (DistanceRepsProcessor.java:190) */
    public boolean anyWithin(long q, long[] cols, double maxDist) { return nAnyLe(ctx, handle, q, cols, maxDist); }

    /** the distances of set q to cols */
    public void row(long q, long[] cols, double[] out) { nRow(ctx, handle, q, cols, out); }

    /** argmin over cols (DistanceRepsProcessor.java:238-239): the position in cols,
     *  -1 when none is below 1.0; bestD[0] = its distance */
    public int closest(long q, long[] cols, double[] bestD) { return nArgmin(ctx, handle, q, cols, bestD); }

    /** Both passes of DistanceRepsProcessor.java:185-262 in one call: isRep[i] = 1
     *  for representatives (in set order, greedy); repOf / repDist = each set's
     *  closest representative. tieRank (optional) = repMap's iteration order of
     *  the representatives, which breaks argmin ties as the reference's reduce does.
     *  Every array holds one element per set. Returns the number of representatives. */
    public long greedyReps(double maxDist, long[] tieRank, int[] isRep, long[] repOf, double[] repDist) {
        return nGreedyReps(ctx, handle, maxDist, tieRank, isRep, repOf, repDist);
    }

    /** hashSet(width) of every set, as a sketch collection (WidthProcessor.java:178) */
    public GpuKmerSets sketches(int width) { return new GpuKmerSets(ctx, nSketch(ctx, handle, width)); }

    /** Sketch.distance of rows [r0, r1) x columns [c0, c1) of a sketch collection
     *  (WidthProcessor.java:183-185), row-major with stride ld */
    public void sketchDistances(long r0, long r1, long c0, long c1, boolean upperTriangle, double[] out, int ld) {
        nSketchMatrix(ctx, handle, r0, r1, c0, c1, upperTriangle ? UPPER_TRIANGLE : 0, out, ld);
    }

    /** a sketch collection of given signatures (each ascending; Sketch.getSignature
     *  of a Bucket's sketches, TuningProcessor.java:114-131), width = the sketch size */
    public static GpuKmerSets fromSignatures(Context ctx, int width, int[][] sigs) {
        long[] off = new long[sigs.length + 1];
        for (int i = 0; i < sigs.length; i++)
            off[i + 1] = off[i] + sigs[i].length;
        int[] all = new int[(int) off[sigs.length]];
        for (int i = 0; i < sigs.length; i++)
            System.arraycopy(sigs[i], 0, all, (int) off[i], sigs[i].length);
        return new GpuKmerSets(ctx.h, nSketchUpload(ctx.h, width, off, all));
    }

    /** the signatures of a sketch collection (hashSet(width) of each set,
     *  ascending ints; shorter than the width for a small set: a "dwarf") */
    public int[][] signatures() {
        final int n = (int) size();
        long[] off = new long[n + 1];
        int[] sigs = new int[(int) nTotal(handle)];
        nSketchDownload(handle, off, sigs);
        int[][] out = new int[n][];
        for (int i = 0; i < n; i++)
            out[i] = java.util.Arrays.copyOfRange(sigs, (int) off[i], (int) off[i + 1]);
        return out;
    }

    @Override
    public synchronized void close() {
        if (handle != 0) {
            nFree(handle);
            handle = 0;
        }
    }
}
