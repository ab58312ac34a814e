package org.theseed.genome.distance.gpu;

import java.io.File;
import java.io.FileNotFoundException;
import java.io.IOException;
import java.io.PrintWriter;
import java.nio.charset.StandardCharsets;
import java.util.ArrayList;
import java.util.HashMap;
import java.util.HashSet;
import java.util.List;
import java.util.Map;

import org.kohsuke.args4j.Option;
import org.slf4j.Logger;
import org.slf4j.LoggerFactory;
import org.theseed.basic.BaseReportProcessor;
import org.theseed.basic.ParseFailureException;
import org.theseed.sequence.FastaInputStream;
import org.theseed.sequence.KmerType;
import org.theseed.sequence.Sequence;

/**
 * The `fastaReps` command on one MI355X: FastaDistanceRepsProcessor's
 * options, defaults, validation messages and report
 * (FastaDistanceRepsProcessor.java:54-92, :111-149). The sequences are
 * packed once; a sequence becomes a representative when no representative so
 * far is within maxDist (the early-exit loop of :122-136 decides a boolean,
 * so its HashMap order does not matter): one gdist_greedy_reps call when the
 * labels are unique, else one anyWithin row query per sequence with the
 * reference's repMap.put replacement. Each new representative prints
 * `label \t comment` in input order (:141-144).
 *
 * Registered in App next to "fastaReps" (e.g. "fastaRepsGpu").
 */
public class GpuFastaDistanceRepsProcessor extends BaseReportProcessor {

    protected static Logger log = LoggerFactory.getLogger(GpuFastaDistanceRepsProcessor.class);

    @Option(name = "--input", aliases = { "-i" }, usage = "input FASTA file (if not STDIN)")
    private File inFile;

    @Option(name = "--kSize", aliases = {"--kmerSize", "-K" }, usage = "kmer size to use; 0 for sequence type default")
    private int kmerSize;

    @Option(name = "--dist", aliases = { "--maxDist", "-d" }, usage = "maximum distance a neighbor can be from a representative")
    private double maxDist;

    @Option(name = "--type", usage = "input sequence type")
    private KmerType seqType;

    @Option(name = "--device", usage = "GPU ordinal")
    private int device;

    @Override
    protected void setReporterDefaults() {
        this.inFile = null;
        this.kmerSize = 0;
        this.seqType = KmerType.DNA;
        this.maxDist = 0.97;
        this.device = 0;
    }

    @Override
    protected void validateReporterParms() throws IOException, ParseFailureException {
        if (this.kmerSize == 0)
            this.kmerSize = this.seqType.getKmerSize();
        if (this.kmerSize < 2)
            throw new ParseFailureException("Kmer size must be at least 2.");
        if (this.inFile != null && ! this.inFile.canRead())
            throw new FileNotFoundException("Input file " + this.inFile + " is not found or invalid.");
    }

    @Override
    protected void runReporter(PrintWriter writer) throws Exception {
        writer.println("seq\tname");
        List<Sequence> seqs = new ArrayList<Sequence>();
        try (FastaInputStream in = this.inFile == null ? new FastaInputStream(System.in)
                                                       : new FastaInputStream(this.inFile)) {
            for (Sequence seq : in)
                seqs.add(seq);
        }
        final int n = seqs.size();
        if (n == 0)
            return;
        byte[][] bytes = new byte[n][];
        List<String> labels = new ArrayList<String>(n);
        for (int i = 0; i < n; i++) {
            bytes[i] = seqs.get(i).getSequence().getBytes(StandardCharsets.US_ASCII);
            labels.add(seqs.get(i).getLabel());
        }
        final int kind = this.seqType == KmerType.DNA ? GpuKmerSets.DNA : GpuKmerSets.PROT;
        int reps = 0;
        try (GpuKmerSets.Context ctx = new GpuKmerSets.Context(this.device);
             GpuKmerSets sets = new GpuKmerSets(ctx, kind, this.kmerSize, bytes)) {
            bytes = null;
            if (new HashSet<String>(labels).size() == n) {
                int[] isRep = new int[n];
                sets.greedyReps(this.maxDist, null, isRep, null, null);
                for (int i = 0; i < n; i++)
                    if (isRep[i] != 0) {
                        writer.println(seqs.get(i).getLabel() + "\t" + seqs.get(i).getComment());
                        reps++;
                    }
            } else {
                Map<String, Integer> repMap = new HashMap<String, Integer>(100);
                for (int i = 0; i < n; i++) {
                    long[] cur = new long[repMap.size()];
                    int k = 0;
                    for (Integer x : repMap.values())
                        cur[k++] = x;
                    if (cur.length == 0 || ! sets.anyWithin(i, cur, this.maxDist)) {
                        writer.println(seqs.get(i).getLabel() + "\t" + seqs.get(i).getComment());
                        repMap.put(labels.get(i), i);
                    }
                }
                reps = repMap.size();
            }
        }
        log.info("{} representatives found for {} sequences.", reps, n);
    }
}
