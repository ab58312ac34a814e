package org.theseed.genome.distance.gpu;

import java.io.File;
import java.io.FileNotFoundException;
import java.io.IOException;
import java.nio.charset.StandardCharsets;

import org.kohsuke.args4j.Option;
import org.slf4j.Logger;
import org.slf4j.LoggerFactory;
import org.theseed.io.TabbedLineReader;
import org.theseed.basic.BaseProcessor;

/**
 * The protein input of the GPU `width` and `sketches` commands: the options,
 * defaults and messages of ProteinKmerReader (ProteinKmerReader.java:44-101;
 * its column indexes and kmer size are private there, so a subclass outside
 * its package cannot read the protein column) — `-K` 8, `-i` (STDIN), `-c`
 * "1", `-p` "aa_sequence" — and a `--device` option. Proteins are handed to
 * the device as bytes; `new ProteinKmers(seq)` (:101) is the pack of the
 * whole group or file in one call (GpuKmerSets, kind PROT).
 */
public abstract class GpuProteinKmerReader extends BaseProcessor {

    protected static Logger log = LoggerFactory.getLogger(GpuProteinKmerReader.class);

    private TabbedLineReader inStream;
    private int idIdx;
    private int protIdx;

    @Option(name = "-K", aliases = { "--kmer", "--kmerSize" }, metaVar = "12", usage = "protein kmer size")
    private int kmerSize;

    @Option(name = "-i", aliases = { "--input" }, metaVar = "families.tbl", usage = "input file (if not STDIN)")
    private File inFile;

    @Option(name = "-c", aliases = { "--col", "--groupCol" }, metaVar = "pgfam_id", usage = "group ID column index (1-based) or name")
    private String idColumn;

    @Option(name = "-p", aliases = { "--prot", "--protCol" }, metaVar = "0", usage = "protein sequence column index (1-based) or name")
    private String protColumn;

    @Option(name = "--device", usage = "GPU ordinal")
    private int device;

    protected void initProteinParms() {
        this.kmerSize = 8;
        this.inFile = null;
        this.idColumn = "1";
        this.protColumn = "aa_sequence";
        this.device = 0;
    }

    protected void validateProteinParms() throws IOException, FileNotFoundException {
        if (this.inFile == null) {
            log.info("Proteins will be read from standard input.");
            this.inStream = new TabbedLineReader(System.in);
        } else if (! this.inFile.canRead()) {
            throw new FileNotFoundException("Input file " + this.inFile + " is not found or invalid.");
        } else {
            log.info("Proteins will be read from {}.", this.inFile);
            this.inStream = new TabbedLineReader(this.inFile);
        }
        this.idIdx = this.inStream.findField(this.idColumn);
        this.protIdx = this.inStream.findField(this.protColumn);
    }

    protected int kmerSize() { return this.kmerSize; }

    protected int device() { return this.device; }

    /** the protein on the current line, as bytes for the device pack */
    protected byte[] getProtein(TabbedLineReader.Line line) {
        return line.get(this.protIdx).getBytes(StandardCharsets.US_ASCII);
    }

    protected String getGroupId(TabbedLineReader.Line line) {
        return line.get(this.idIdx);
    }

    protected TabbedLineReader input() {
        return this.inStream;
    }

    protected abstract void processProteins() throws IOException;

    @Override
    public void runCommand() throws Exception {
        try {
            this.processProteins();
        } finally {
            this.inStream.close();
        }
    }
}
