package org.theseed.genome.distance.gpu;

import java.io.File;
import java.io.FileNotFoundException;
import java.io.IOException;
import java.io.PrintWriter;
import java.nio.charset.StandardCharsets;
import java.util.ArrayList;
import java.util.List;

import org.kohsuke.args4j.Option;
import org.slf4j.Logger;
import org.slf4j.LoggerFactory;
import org.theseed.basic.BaseReportProcessor;
import org.theseed.basic.ParseFailureException;
import org.theseed.sequence.FastaInputStream;
import org.theseed.sequence.KmerType;
import org.theseed.sequence.Sequence;

/**
 * The `fastaDist` command on one MI355X: the same options, defaults,
 * validation messages and report as FastaDistanceProcessor
 * (FastaDistanceProcessor.java:73-112, :134-194), the pair loop replaced by
 * libgdist.so. Every sequence is packed once (KmerType.createKmers for all of
 * them, on the device) instead of once per batch plus once per pair outside
 * the batch (:150-155, :181-184); the N x N upper triangle is computed a
 * block of `--batch` rows at a time (gdist_intersect_matrix with
 * GDIST_UPPER_TRIANGLE) and printed row by row, pairs (i, j > i), with
 * "" + distance (Double.toString), as :188-191 prints them. The reference's
 * line order is the nondeterministic interleaving of its parallel rows; this
 * one is row-major, a valid ordering of the same lines.
 *
 * Registered in App next to "fastaDist" (e.g. "fastaDistGpu"); needs
 * libgdist_jni.so (jni/Makefile) on java.library.path.
 */
public class GpuFastaDistanceProcessor extends BaseReportProcessor {

    protected static Logger log = LoggerFactory.getLogger(GpuFastaDistanceProcessor.class);

    private List<Sequence> sequences;

    @Option(name = "--input", aliases = { "-i" }, usage = "input FASTA file (if not STDIN)")
    private File inFile;

    @Option(name = "--kSize", aliases = { "--kmerSize", "-K" }, usage = "kmer size to use; 0 for sequence type default")
    private int kmerSize;

    @Option(name = "--batch", aliases = { "-b" }, usage = "rows per device call")
    private int batchSize;

    @Option(name = "--type", usage = "input sequence type")
    private KmerType seqType;

    @Option(name = "--device", usage = "GPU ordinal")
    private int device;

    @Override
    protected void setReporterDefaults() {
        this.inFile = null;
        this.kmerSize = 0;
        this.batchSize = 20;
        this.seqType = KmerType.DNA;
        this.device = 0;
    }

    @Override
    protected void validateReporterParms() throws IOException, ParseFailureException {
        if (this.kmerSize == 0)
            this.kmerSize = this.seqType.getKmerSize();
        if (this.kmerSize < 2)
            throw new ParseFailureException("Kmer size must be at least 2.");
        if (this.batchSize < 1)
            throw new ParseFailureException("Batch size must be at least 1.");
        FastaInputStream in;
        if (this.inFile == null)
            in = new FastaInputStream(System.in);
        else if (! this.inFile.canRead())
            throw new FileNotFoundException("Input file " + this.inFile + " is not found or unreadable.");
        else
            in = new FastaInputStream(this.inFile);
        try (FastaInputStream stream = in) {
            this.sequences = new ArrayList<Sequence>();
            for (Sequence seq : stream)
                this.sequences.add(seq);
        }
        log.info("{} sequences read from input.", this.sequences.size());
    }

    @Override
    protected void runReporter(PrintWriter writer) throws Exception {
        writer.println("seq1\tname1\tseq2\tname2\tdistance");
        final int n = this.sequences.size();
        if (n < 2)
            return;
        byte[][] seqs = new byte[n][];
        for (int i = 0; i < n; i++)
            seqs[i] = this.sequences.get(i).getSequence().getBytes(StandardCharsets.US_ASCII);
        final int kind = this.seqType == KmerType.DNA ? GpuKmerSets.DNA : GpuKmerSets.PROT;
        try (GpuKmerSets.Context ctx = new GpuKmerSets.Context(this.device);
             GpuKmerSets sets = new GpuKmerSets(ctx, kind, this.kmerSize, seqs)) {
            seqs = null;
            // the pair loop's representation (two-tier bitsets or the sorted join), chosen once
            sets.prepare(0.5 * n * (double) (n - 1));
            final int rows = Math.max(1, Math.min(this.batchSize, Integer.MAX_VALUE / n));
            double[] d = new double[rows * n];
            long pairs = 0;
            for (int r0 = 0; r0 < n - 1; r0 += rows) {
                final int r1 = Math.min(n - 1, r0 + rows);
                sets.distances(r0, r1, 0, n, true, d, n);
                for (int i = r0; i < r1; i++) {
                    Sequence s1 = this.sequences.get(i);
                    String head = s1.getLabel() + "\t" + s1.getComment() + "\t";
                    for (int j = i + 1; j < n; j++) {
                        Sequence s2 = this.sequences.get(j);
                        writer.println(head + s2.getLabel() + "\t" + s2.getComment() + "\t" + d[(i - r0) * n + j]);
                    }
                    pairs += n - 1 - i;
                }
            }
            log.info("{} pairs computed.", pairs);
        }
    }
}
