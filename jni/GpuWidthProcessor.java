package org.theseed.genome.distance.gpu;

import java.io.IOException;
import java.util.ArrayList;
import java.util.List;

import org.kohsuke.args4j.Argument;
import org.kohsuke.args4j.Option;
import org.slf4j.Logger;
import org.slf4j.LoggerFactory;
import org.theseed.basic.ParseFailureException;
import org.theseed.io.TabbedLineReader;
import org.theseed.utils.SizeList;

/**
 * The `width` command on one MI355X: WidthProcessor's options, defaults,
 * validation messages and report (WidthProcessor.java:62-106, :111-208),
 * with each group's two all-pairs loops on the device: the exact distances
 * (:159-165) are one upper-triangle matrix call over the group's packed
 * proteins, and per sketch size the sketches (hashSet(size), :178) and their
 * all-pairs Sketch.distance (:183-185) are one sketch build and one sketch
 * matrix call. The error sums run on the host in the reference's i-major
 * order (`total += error`, :186-191), so the printed means are the same
 * doubles; dwarves (:179) are the sketches shorter than the size.
 *
 * Registered in App next to "width" (e.g. "widthGpu").
 */
public class GpuWidthProcessor extends GpuProteinKmerReader {

    protected static Logger log = LoggerFactory.getLogger(GpuWidthProcessor.class);
    private static final int INVALID_TARGET_SIZE = Integer.MAX_VALUE;
    private int[] sizes;
    private int targetSize;

    @Option(name = "-s", aliases = { "--step", "--incr" }, metaVar = "5", usage = "increment for sketch size search")
    private int stepSize;

    @Option(name = "-M", aliases = { "--limit", "--maxGroup" }, metaVar = "500", usage = "maximum permissible group size")
    private int maxGroup;

    @Option(name = "-e", aliases = { "--error", "--target" }, metaVar = "0.001", usage = "target value for mean error")
    private double targetError;

    @Argument(index = 0, metaVar = "50", usage = "starting (minimum) sketch size", required = true)
    private int minSize;

    @Argument(index = 1, metaVar = "300", usage = "ending (maximum) sketch size", required = true)
    private int maxSize;

    private GpuKmerSets.Context ctx;

    @Override
    protected void setDefaults() {
        this.stepSize = 10;
        this.initProteinParms();
        this.maxGroup = 1000;
        this.targetError = 0.001;
    }

    @Override
    protected boolean validateParms() throws IOException, ParseFailureException {
        this.validateProteinParms();
        if (this.minSize > this.maxSize)
            throw new ParseFailureException("Minimum sketch size cannot be larger than maximum.");
        if (this.stepSize <= 0)
            throw new ParseFailureException("Step size must be greater than 0.");
        if (this.maxGroup < 10)
            throw new ParseFailureException("Maximum group size must be 10 or greater.");
        if (this.targetError > 0.1 || this.targetError <= 0.0)
            throw new ParseFailureException("Target error must be > 0 and < 0.1.");
        this.sizes = SizeList.getSizes(this.minSize, this.maxSize, this.stepSize);
        return true;
    }

    @Override
    protected void processProteins() {
        String groupId = "";
        List<byte[]> proteins = new ArrayList<byte[]>();
        this.targetSize = this.minSize;
        System.out.println("Group\tSize\tPairs\tDwarves\tMean E\tMax E");
        try (GpuKmerSets.Context c = new GpuKmerSets.Context(this.device())) {
            this.ctx = c;
            for (TabbedLineReader.Line line : this.input()) {
                String group = this.getGroupId(line);
                if (! group.contentEquals(groupId) || proteins.size() >= this.maxGroup) {
                    if (proteins.size() > 0)
                        this.processGroup(groupId, proteins);
                    log.info("Reading group {}.", group);
                    groupId = group;
                    proteins.clear();
                }
                proteins.add(this.getProtein(line));
            }
            if (proteins.size() > 0)
                this.processGroup(groupId, proteins);
        } finally {
            this.ctx = null;
        }
        if (this.targetSize == INVALID_TARGET_SIZE)
            log.warn("Target sketch size is larger than maxmimum.");
        else
            log.info("Target sketch size is {}.", this.targetSize);
    }

    /** WidthProcessor.ProcessGroup (:153-208) with the pair loops on the device */
    private void processGroup(String groupId, List<byte[]> proteins) {
        final int n = proteins.size();
        log.info("Processing group {} with {} sequences.", groupId, n);
        try (GpuKmerSets sets = new GpuKmerSets(this.ctx, GpuKmerSets.PROT, this.kmerSize(),
                                                proteins.toArray(new byte[0][]))) {
            double[] real = new double[n * n];
            sets.distances(0, n, 0, n, true, real, n);
            int pairs = 0;
            for (int i = 0; i < n; i++)
                for (int j = i + 1; j < n; j++)
                    if (real[i * n + j] < 1.0) pairs++;
            if (pairs == 0) {
                log.warn("Group {} has no usable distance pairs.", groupId);
                return;
            }
            log.info("Group {} has {} usable distance pairs.", groupId, pairs);
            int minGoodSize = INVALID_TARGET_SIZE;
            double[] sk = new double[n * n];
            for (int size : this.sizes) {
                long dwarves = 0;
                try (GpuKmerSets sketches = sets.sketches(size)) {
                    for (long len : sketches.sizes())
                        if (len < size) dwarves++;
                    sketches.sketchDistances(0, n, 0, n, true, sk, n);
                }
                double total = 0.0;
                double maxErr = 0.0;
                for (int i = 0; i < n; i++)
                    for (int j = i + 1; j < n; j++) {
                        double sketchDist = sk[i * n + j];
                        double realDist = real[i * n + j];
                        if (realDist != sketchDist) {
                            double error = Math.abs(realDist - sketchDist) * 2.0 / (realDist + sketchDist);
                            if (error > maxErr) maxErr = error;
                            total += error;
                        }
                    }
                double meanError = total / pairs;
                System.out.format("%s\t%8d\t%8d\t%8d\t%8.4f\t%8.4f%n", groupId, size, pairs, dwarves,
                        meanError, maxErr);
                if (size < minGoodSize && meanError <= this.targetError)
                    minGoodSize = size;
            }
            if (minGoodSize > this.targetSize) this.targetSize = minGoodSize;
            if (minGoodSize == INVALID_TARGET_SIZE)
                log.warn("{} has no acceptable sketch size in range.", groupId);
            else
                log.info("Minimum acceptable size for {} is {}.", groupId, minGoodSize);
        }
    }
}
