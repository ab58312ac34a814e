package org.theseed.genome.distance.gpu;

import java.io.File;
import java.io.FileNotFoundException;
import java.io.IOException;
import java.io.PrintWriter;
import java.util.ArrayList;
import java.util.HashMap;
import java.util.HashSet;
import java.util.List;
import java.util.Map;
import java.util.Set;

import org.kohsuke.args4j.Argument;
import org.kohsuke.args4j.Option;
import org.slf4j.Logger;
import org.slf4j.LoggerFactory;
import org.theseed.basic.ParseFailureException;
import org.theseed.counters.CountMap;
import org.theseed.genome.Genome;
import org.theseed.genome.iterator.GenomeSource;
import org.theseed.utils.BaseMultiReportProcessor;

/**
 * The `distReps` command on one MI355X: DistanceRepsProcessor's options,
 * defaults, validation messages and reports (DistanceRepsProcessor.java:
 * 66-77, :141-161, :178-275), the kmer loops on the device.
 *
 * Every genome of every source is packed once (GpuKmerSets, batches of
 * BATCH genomes appended to one collection; contigs joined by 0x00 as
 * GpuGenomeProcessor does). Pass 1 (:185-201, `anyMatch(d <= maxDist)`
 * against the representatives so far, sequential over genomes) and pass 2
 * (:215-262, the closest representative of every other genome) are one
 * device call each (gdist_greedy_reps). Pass 2's reduce breaks ties towards
 * the representative met first in repMap's HashMap iteration (Result.merge,
 * :120-122): that order is read from a java.util.HashMap built exactly as
 * the reference builds repMap (capacity 500, puts in pass-1 order) and handed
 * to the device as tieRank. Genome ids repeated across sources (a put that
 * replaces a representative) run pass 1 as row queries on the host side
 * instead, with the reference's replacement semantics.
 *
 * Registered in App next to "distReps" (e.g. "distRepsGpu").
 */
public class GpuDistanceRepsProcessor extends BaseMultiReportProcessor {

    protected static Logger log = LoggerFactory.getLogger(GpuDistanceRepsProcessor.class);
    /** genomes per device pack */
    private static final int BATCH = 256;

    private List<GenomeSource> genomeSources;
    private int gTotal;

    @Option(name = "--kmerSize", aliases = { "-K", "--kmer" }, metaVar = "20",
            usage = "kmer size to use for distance computation")
    private int kmerSize;

    @Option(name = "--sourceType", aliases = { "--type", "-t" }, usage = "type of genome sources")
    private GenomeSource.Type sourceType;

    @Option(name = "--dist", metaVar = "0.9", usage = "maximum distance for a representative neighborhood")
    private double maxDist;

    @Option(name = "--device", usage = "GPU ordinal")
    private int device;

    @Argument(index = 0, metaVar = "inDir1 inDir2 ...", usage = "file or directory names of the genome sources",
            required = true)
    private List<File> inDirs;

    @Override
    protected File setDefaultOutputDir(File curDir) {
        return new File(curDir, "repDb");
    }

    @Override
    protected void setMultiReportDefaults() {
        this.inDirs = new ArrayList<File>();
        this.maxDist = 0.97;
        this.kmerSize = 9;
        this.sourceType = GenomeSource.Type.DIR;
        this.device = 0;
    }

    @Override
    protected void validateMultiReportParms() throws IOException, ParseFailureException {
        if (this.kmerSize < 4)
            throw new ParseFailureException("Kmer size must be at least 4.");
        if (this.maxDist <= 0.0 || this.maxDist >= 1.0)
            throw new ParseFailureException("Distance must be strictly between 0 and 1.");
        this.gTotal = 0;
        this.genomeSources = new ArrayList<GenomeSource>(this.inDirs.size());
        for (File inDir : this.inDirs) {
            if (! inDir.exists())
                throw new FileNotFoundException("Genome source " + inDir + " is not found.");
            GenomeSource genomes = this.sourceType.create(inDir);
            this.gTotal += genomes.size();
            log.info("{} genomes found in {}.", genomes.size(), inDir);
            this.genomeSources.add(genomes);
        }
        log.info("{} total genomes found in all sources.", this.gTotal);
    }

    @Override
    protected void runMultiReports() throws Exception {
        // every genome once, in pass-1 order (sources in order, each source's iteration)
        final List<String> ids = new ArrayList<String>(this.gTotal);
        final List<String> names = new ArrayList<String>(this.gTotal);
        final List<Map<String, Integer>> setOf = new ArrayList<Map<String, Integer>>();
        try (GpuKmerSets.Context ctx = new GpuKmerSets.Context(this.device)) {
            GpuKmerSets sets = null;
            try {
                List<byte[]> batch = new ArrayList<byte[]>(BATCH);
                for (GenomeSource genomes : this.genomeSources) {
                    Map<String, Integer> idx = new HashMap<String, Integer>();
                    for (Genome genome : genomes) {
                        idx.put(genome.getId(), ids.size());
                        ids.add(genome.getId());
                        names.add(genome.getName());
                        batch.add(GpuGenomeProcessor.contigBytes(genome));
                        if (batch.size() >= BATCH)
                            sets = this.flush(ctx, sets, batch);
                    }
                    setOf.add(idx);
                }
                sets = this.flush(ctx, sets, batch);
                if (sets == null)
                    return;
                this.reports(sets, ids, names, setOf);
            } finally {
                if (sets != null) sets.close();
            }
        }
    }

    private GpuKmerSets flush(GpuKmerSets.Context ctx, GpuKmerSets sets, List<byte[]> batch) {
        if (batch.isEmpty())
            return sets;
        byte[][] seqs = batch.toArray(new byte[0][]);
        batch.clear();
        if (sets == null)
            return new GpuKmerSets(ctx, GpuKmerSets.DNA, this.kmerSize, seqs);
        sets.append(seqs);
        return sets;
    }

    private void reports(GpuKmerSets sets, List<String> ids, List<String> names, List<Map<String, Integer>> setOf)
            throws IOException {
        final int n = ids.size();
        final boolean unique = new HashSet<String>(ids).size() == n;
        // pass 1: repMap (genome id -> set), built as the reference builds it
        Map<String, Integer> repMap = new HashMap<String, Integer>(500);
        int[] isRep = new int[n];
        long[] repOf = new long[n];
        double[] repDist = new double[n];
        if (unique) {
            sets.greedyReps(this.maxDist, null, isRep, repOf, repDist);
            for (int i = 0; i < n; i++)
                if (isRep[i] != 0) repMap.put(ids.get(i), i);
        } else {
            for (int i = 0; i < n; i++) {
                long[] cur = toLongs(repMap.values());
                if (cur.length == 0 || ! sets.anyWithin(i, cur, this.maxDist))
                    repMap.put(ids.get(i), i);
            }
        }
        log.info("{} total representatives found for {} genomes.", repMap.size(), n);
        // the representatives in repMap's iteration order (the reduce's encounter order)
        long[] ordered = toLongs(repMap.values());
        if (unique) {
            long[] tieRank = new long[n];
            java.util.Arrays.fill(tieRank, n);
            for (int p = 0; p < ordered.length; p++)
                tieRank[(int) ordered[p]] = p;
            sets.greedyReps(this.maxDist, tieRank, isRep, repOf, repDist);
        }
        CountMap<String> neighborCounts = new CountMap<String>();
        String namePrefix = String.format("rep%.4f_K%d", this.maxDist, this.kmerSize);
        File listFile = this.getOutFile(namePrefix + ".list.tbl");
        try (PrintWriter writer = new PrintWriter(listFile)) {
            writer.println("genome_id\tgenome_name\trep_id\trep_name\tdistance");
            int gCount = 0;
            double[] best = new double[1];
            for (int s = 0; s < this.genomeSources.size(); s++) {
                GenomeSource genomeSource = this.genomeSources.get(s);
                for (String genomeID : genomeSource.getIDs()) {
                    gCount++;
                    final int i = setOf.get(s).get(genomeID);
                    Integer rep = repMap.get(genomeID);
                    String genomeName;
                    double dist;
                    if (rep != null) {
                        genomeName = names.get(rep);
                        dist = 0.0;
                    } else {
                        genomeName = names.get(i);
                        if (unique) {
                            rep = (int) repOf[i];
                            dist = repDist[i];
                        } else {
                            int pos = sets.closest(i, ordered, best);
                            rep = (int) ordered[pos];
                            dist = best[0];
                        }
                    }
                    final String repID = ids.get(rep);
                    writer.println(genomeID + "\t" + genomeName + "\t" + repID + "\t" + names.get(rep) + "\t" + dist);
                    neighborCounts.count(repID);
                }
            }
            log.info("{} total genomes placed.", gCount);
        }
        File statFile = this.getOutFile(namePrefix + ".stats.tbl");
        try (PrintWriter writer = new PrintWriter(statFile)) {
            writer.println("rep_id\trep_name\tsize");
            for (var count : neighborCounts.sortedCounts()) {
                String repID = count.getKey();
                writer.println(repID + "\t" + names.get(repMap.get(repID)) + "\t" + count.getCount());
            }
        }
    }

    private static long[] toLongs(java.util.Collection<Integer> v) {
        long[] out = new long[v.size()];
        int k = 0;
        for (Integer x : v)
            out[k++] = x;
        return out;
    }
}
