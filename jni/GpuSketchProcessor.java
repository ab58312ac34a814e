package org.theseed.genome.distance.gpu;

import java.io.File;
import java.io.FileNotFoundException;
import java.io.IOException;
import java.util.ArrayList;
import java.util.List;

import org.kohsuke.args4j.Argument;
import org.kohsuke.args4j.Option;
import org.slf4j.Logger;
import org.slf4j.LoggerFactory;
import org.theseed.basic.ParseFailureException;
import org.theseed.io.TabbedLineReader;
import org.theseed.sequence.hash.Bucket;
import org.theseed.sequence.hash.Sketch;

/**
 * The `sketches` command on one MI355X: SketchProcessor's options, defaults,
 * validation messages and output (SketchProcessor.java:51-99). The proteins
 * are packed in batches of BATCH and their hashSet(width) signatures
 * (:88) computed on the device (gdist_sketch_build) and downloaded; each
 * becomes `new Sketch(signature, group)` in input order, and the Bucket is
 * saved as the reference saves it.
 *
 * Registered in App next to "sketches" (e.g. "sketchesGpu").
 */
public class GpuSketchProcessor extends GpuProteinKmerReader {

    protected static Logger log = LoggerFactory.getLogger(GpuSketchProcessor.class);
    /** proteins per device pack */
    private static final int BATCH = 50000;

    @Option(name = "-w", aliases = { "--width", "--sketchSize" }, metaVar = "400", usage = "sketch size for each protein")
    private int width;

    @Argument(index = 0, metaVar = "outFile.ser", usage = "output file name", required = true)
    private File outFile;

    @Override
    protected void setDefaults() {
        this.initProteinParms();
        this.width = 360;
    }

    @Override
    protected boolean validateParms() throws IOException, ParseFailureException {
        this.validateProteinParms();
        if (! this.outFile.exists()) {
            this.outFile.createNewFile();
        } else if (! this.outFile.canWrite())
            throw new FileNotFoundException("Cannot write to output file " + this.outFile + ".");
        if (this.width < 10)
            throw new ParseFailureException("Sketch width cannot be less than 10.");
        return true;
    }

    @Override
    protected void processProteins() throws IOException {
        Bucket outBucket = new Bucket();
        int protCount = 0;
        List<byte[]> prots = new ArrayList<byte[]>();
        List<String> groups = new ArrayList<String>();
        try (GpuKmerSets.Context ctx = new GpuKmerSets.Context(this.device())) {
            for (TabbedLineReader.Line line : this.input()) {
                prots.add(this.getProtein(line));
                groups.add(this.getGroupId(line));
                if (prots.size() >= BATCH) {
                    protCount += this.flush(ctx, prots, groups, outBucket);
                    log.info("{} proteins processed.", protCount);
                }
            }
            protCount += this.flush(ctx, prots, groups, outBucket);
        }
        log.info("Writing {} sketches to {}.", protCount, this.outFile);
        outBucket.save(this.outFile);
        log.info("All done.");
    }

    private int flush(GpuKmerSets.Context ctx, List<byte[]> prots, List<String> groups, Bucket out) {
        final int n = prots.size();
        if (n == 0)
            return 0;
        try (GpuKmerSets sets = new GpuKmerSets(ctx, GpuKmerSets.PROT, this.kmerSize(), prots.toArray(new byte[0][]));
             GpuKmerSets sk = sets.sketches(this.width)) {
            int[][] sigs = sk.signatures();
            for (int i = 0; i < n; i++)
                out.add(new Sketch(sigs[i], groups.get(i)));
        }
        prots.clear();
        groups.clear();
        return n;
    }
}
