package org.theseed.genome.distance.gpu;

import java.io.File;
import java.io.FileNotFoundException;
import java.io.IOException;
import java.util.Set;

import org.kohsuke.args4j.Argument;
import org.kohsuke.args4j.Option;
import org.slf4j.Logger;
import org.slf4j.LoggerFactory;
import org.theseed.basic.BaseProcessor;
import org.theseed.basic.ParseFailureException;
import org.theseed.sequence.hash.Bucket;
import org.theseed.sequence.hash.LSHMemSeqHash;
import org.theseed.sequence.hash.Sketch;
import org.theseed.utils.SizeList;

/**
 * The `tune` command with its all-pairs sketch count on one MI355X
 * (TuningProcessor.java:43-166: the same options, defaults, validation
 * messages, header and report lines).
 *
 * What moves to the device is the pair count of :125-139 — for every sketch
 * i the sketches after it (Bucket.after(i)) closer than the target,
 * sketch1.distance(sketch2) < target — which is an upper-triangle
 * Sketch.distance matrix and a threshold: the Bucket's signatures are
 * uploaded once (gdist_sketch_upload) and the triangle is computed in row
 * blocks (gdist_sketch_matrix, the ring kernel) and counted per row. The
 * sketch width passed is the longest signature (the width the sketches were
 * made with; shorter ones are dwarves). The stage-size loop (:145-163) runs
 * the reference's LSHMemSeqHash on the CPU unchanged: the LSH tables are out
 * of scope (SURVEY §2).
 *
 * Registered in App next to "tune" (e.g. "tuneGpu").
 */
public class GpuTuningProcessor extends BaseProcessor {

    protected static Logger log = LoggerFactory.getLogger(GpuTuningProcessor.class);
    /** cells of one row block of the device matrix (2^24 doubles, 128 MB) */
    private static final long ROW_BLOCK_CELLS = 1L << 24;
    private int[] stageSizes;

    @Option(name = "-b", aliases = { "--buckets" }, metaVar = "200", usage = "number of buckets per stage")
    private int bucketCount;

    @Option(name = "-s", aliases = { "--step", "--incr" }, metaVar = "5", usage = "increment for stage count search")
    private int stepSize;

    @Option(name = "-w", aliases = { "--width", "--sketch" }, metaVar = "200", usage = "number of values per protein sketch")
    private int width;

    @Option(name = "-t", aliases = { "--target", "--minDist" }, metaVar = "0.50", usage = "target sketch distance")
    private double target;

    @Option(name = "--device", metaVar = "0", usage = "GPU device index")
    private int device;

    @Argument(index = 0, metaVar = "sketchesIn.ser", usage = "input file containing protein sketches", required = true)
    private File inFile;

    @Argument(index = 1, metaVar = "10", usage = "starting (minimum) stage count", required = true)
    private int minStageCount;

    @Argument(index = 2, metaVar = "100", usage = "ending (maximum) stage count", required = true)
    private int maxStageCount;

    @Override
    protected void setDefaults() {
        this.bucketCount = 300;
        this.stepSize = 5;
        this.width = 360;
        this.target = 0.7;
        this.device = 0;
    }

    @Override
    protected boolean validateParms() throws IOException, ParseFailureException {
        if (! this.inFile.canRead())
            throw new FileNotFoundException("Input file " + this.inFile + " not found or unreadable.");
        if (this.minStageCount < 1)
            throw new ParseFailureException("Minimum stage count must be at least 1.");
        if (this.maxStageCount < this.minStageCount)
            throw new ParseFailureException("Maximum stage count must be no less than minimum.");
        if (this.stepSize < 1)
            throw new ParseFailureException("Step size must be at least 1.");
        if (this.bucketCount < 10)
            throw new ParseFailureException("Bucket count must be at least 10.");
        if (this.target <= 0.0 || this.target >= 1.0)
            throw new ParseFailureException("Target distance must be between 0 and 1 (exclusive).");
        this.stageSizes = SizeList.getSizes(this.minStageCount, this.maxStageCount, this.stepSize);
        return true;
    }

    /**
     * expected[i] = #{ j > i : distance(i, j) < target } over the sketches'
     * signatures: one upload, the upper triangle in row blocks on the device.
     */
    static int[] closeCounts(GpuKmerSets.Context ctx, int[][] sigs, double target) {
        final int n = sigs.length;
        int[] expected = new int[n];
        if (n < 2)
            return expected;
        int width = 1;
        for (int[] s : sigs)
            width = Math.max(width, s.length);
        try (GpuKmerSets sk = GpuKmerSets.fromSignatures(ctx, width, sigs)) {
            final int rows = (int) Math.max(1, Math.min(n, ROW_BLOCK_CELLS / n));
            double[] d = new double[rows * n];
            for (int r0 = 0; r0 < n; r0 += rows) {
                int r1 = Math.min(n, r0 + rows);
                sk.sketchDistances(r0, r1, 0, n, true, d, n);
                for (int i = r0; i < r1; i++) {
                    int base = (i - r0) * n, count = 0;
                    for (int j = i + 1; j < n; j++)
                        if (d[base + j] < target)
                            count++;
                    expected[i] = count;
                }
            }
        }
        return expected;
    }

    @Override
    public void runCommand() throws Exception {
        System.out.println("Stages\tFound\tFailed\tQuality");
        log.info("Reading sketches from {}.", this.inFile);
        Bucket testSketches = Bucket.load(this.inFile);
        int n = testSketches.size();
        log.info("{} proteins found in file.", n);
        int idx = 1;
        int[][] sigs = new int[n][];
        for (Sketch sketch : testSketches) {
            sketch.setName(String.format("p%d", idx));
            sigs[idx - 1] = sketch.getSignature();
            idx++;
        }
        Bucket goodSketches = new Bucket();
        int totalPairs = 0;
        try (GpuKmerSets.Context ctx = new GpuKmerSets.Context(this.device)) {
            int[] expected = closeCounts(ctx, sigs, this.target);
            for (int i = 0; i < n; i++) {
                if (expected[i] > 0) {
                    totalPairs += expected[i];
                    goodSketches.add(testSketches.get(i));
                }
            }
        }
        log.info("{} close pairs found in protein list. {} sequences have neighbors.", totalPairs, goodSketches.size());
        totalPairs += totalPairs;
        for (int stageSize : this.stageSizes) {
            log.info("Testing {} stages.", stageSize);
            LSHMemSeqHash hash = new LSHMemSeqHash(200, stageSize, this.bucketCount);
            for (Sketch sketch : testSketches)
                hash.add(sketch);
            log.info("Hash loaded with {} proteins.", testSketches.size());
            int found = 0;
            int failed = 0;
            for (Sketch sketch : goodSketches) {
                Set<Bucket.Result> results = hash.getClose(sketch, this.target);
                found += results.size() - 1;
                if (results.size() <= 1)
                    failed++;
            }
            System.out.format("%8d\t%8d\t%8d\t%8.4f%n", stageSize, found, failed,
                    ((double) found) / totalPairs);
        }
    }
}
