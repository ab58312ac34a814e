package org.theseed.genome.distance.gpu;

import java.io.File;
import java.io.FileNotFoundException;
import java.io.IOException;
import java.io.PrintWriter;
import java.io.ByteArrayOutputStream;
import java.nio.charset.StandardCharsets;
import java.util.ArrayList;
import java.util.List;

import org.kohsuke.args4j.Argument;
import org.kohsuke.args4j.Option;
import org.slf4j.Logger;
import org.slf4j.LoggerFactory;
import org.theseed.basic.BaseReportProcessor;
import org.theseed.basic.ParseFailureException;
import org.theseed.genome.Contig;
import org.theseed.genome.Genome;
import org.theseed.genome.iterator.GenomeSource;

/**
 * The `genomes` command on one MI355X (GenomeProcessor.java:53-150): base
 * genomes packed once as GenomeKmers sets (contigs joined by a 0x00 byte no
 * kmer spans, the build's reading of GenomeKmers(Genome), SURVEY App. B Q7),
 * then every comparison genome of every directory packed with them and one
 * gdist_intersect_matrix per directory (rows = the directory's genomes,
 * columns = the base genomes) replacing the parallel
 * kmers.distance(mainKmers[i]) loop (:140); output
 * "genome1 \t genome2 \t distance" in the reference's order (:143-146).
 * --maxDist is validated and unused, as in the reference (:89-90).
 */
public class GpuGenomeProcessor extends BaseReportProcessor {

    protected static Logger log = LoggerFactory.getLogger(GpuGenomeProcessor.class);

    @Option(name = "--kmerSize", aliases = { "-K", "--kmer" }, metaVar = "12", usage = "DNA kmer size")
    private int kmerSize;

    @Option(name = "--maxDist", aliases = { "-m", "--max", "--distance" }, metaVar = "0.75",
            usage = "maximum acceptable distance for a neighboring genome")
    private double maxDist;

    @Option(name = "--type", aliases = { "-t" }, usage = "type of genome source")
    private GenomeSource.Type sourceType;

    @Option(name = "--device", usage = "GPU ordinal")
    private int device;

    @Argument(index = 0, metaVar = "gtoDir", required = true, usage = "base genome source")
    private File baseDir;

    @Argument(index = 1, metaVar = "gtoDir1 gtoDir2 ...", required = true, usage = "directory of input GTOs")
    private List<File> genomeDirs;

    private List<String> baseIds;
    private List<byte[]> baseSeqs;

    @Override
    protected void setReporterDefaults() {
        this.kmerSize = 21;
        this.maxDist = 0.9;
        this.sourceType = GenomeSource.Type.DIR;
        this.device = 0;
    }

    /** the genome's contigs joined by 0x00 (no kmer spans a contig boundary) */
    static byte[] contigBytes(Genome genome) {
        ByteArrayOutputStream out = new ByteArrayOutputStream();
        boolean first = true;
        for (Contig c : genome.getContigs()) {
            if (! first)
                out.write(0);
            byte[] b = c.getSequence().getBytes(StandardCharsets.US_ASCII);
            out.write(b, 0, b.length);
            first = false;
        }
        return out.toByteArray();
    }

    @Override
    protected void validateReporterParms() throws IOException, ParseFailureException {
        if (this.kmerSize < 4)
            throw new ParseFailureException("Kmer size cannot be less than 4.");
        if (this.maxDist <= 0.0 || this.maxDist > 1.0)
            throw new ParseFailureException("Maximum distance must be > 0 and <= 1.");
        if (! this.baseDir.exists())
            throw new FileNotFoundException("Main genome source \"" + this.baseDir + "\" is not found.");
        for (File genomeDir : this.genomeDirs) {
            if (! genomeDir.exists())
                throw new FileNotFoundException("Genome source \"" + genomeDir + "\" is not found.");
        }
        GenomeSource base = this.sourceType.create(this.baseDir);
        this.baseIds = new ArrayList<String>(base.size());
        this.baseSeqs = new ArrayList<byte[]>(base.size());
        for (Genome genome : base) {
            this.baseIds.add(genome.getId());
            this.baseSeqs.add(contigBytes(genome));
        }
        log.info("{} base genomes loaded from {}.", this.baseIds.size(), this.baseDir);
    }

    @Override
    protected void runReporter(PrintWriter writer) throws Exception {
        writer.println("genome1\tgenome2\tdistance");
        final int nMain = this.baseIds.size();
        long compares = 0;
        try (GpuKmerSets.Context ctx = new GpuKmerSets.Context(this.device);
             GpuKmerSets base = new GpuKmerSets(ctx, GpuKmerSets.DNA, this.kmerSize,
                                                this.baseSeqs.toArray(new byte[0][]))) {
            // the base genomes are packed once (mainKmers, GenomeProcessor.java:100-111)
            for (File dir : this.genomeDirs) {
                GenomeSource genomes = this.sourceType.create(dir);
                List<String> ids = new ArrayList<String>(genomes.size());
                List<byte[]> seqs = new ArrayList<byte[]>(genomes.size());
                for (Genome genome : genomes) {
                    ids.add(genome.getId());
                    seqs.add(contigBytes(genome));
                }
                final int m = ids.size();
                if (m == 0)
                    continue;
                // rows 0..m-1: this directory's genomes; columns m..m+nMain-1: the
                // base genomes' sets, copied on the device (gdist_sets_concat), not re-packed
                try (GpuKmerSets dirSets = new GpuKmerSets(ctx, GpuKmerSets.DNA, this.kmerSize,
                                                           seqs.toArray(new byte[0][]));
                     GpuKmerSets sets = dirSets.concat(base)) {
                    // row blocks of at most ROW_BLOCK_CELLS distances (no int overflow
                    // of m * nMain, bounded host memory)
                    final int rows = (int) Math.max(1, Math.min(m, ROW_BLOCK_CELLS / Math.max(1, nMain)));
                    double[] d = new double[rows * nMain];
                    for (int r0 = 0; r0 < m; r0 += rows) {
                        final int r1 = Math.min(m, r0 + rows);
                        sets.distances(r0, r1, m, m + nMain, false, d, nMain);
                        for (int r = r0; r < r1; r++)
                            for (int i = 0; i < nMain; i++) {
                                writer.println(ids.get(r) + "\t" + this.baseIds.get(i) + "\t" + d[(r - r0) * nMain + i]);
                                compares++;
                            }
                    }
                }
            }
        }
        log.info("{} comparisons output.", compares);
    }

    /** distances per device call (and host buffer): 2^24 doubles = 128 MiB */
    private static final long ROW_BLOCK_CELLS = 1L << 24;
}
