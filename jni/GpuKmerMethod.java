package org.theseed.genome.distance.gpu;

import java.util.HashMap;
import java.util.Map;

import org.theseed.genome.Genome;
import org.theseed.genome.distance.methods.DistanceMethod;
import org.theseed.genome.distance.methods.Measurer;

/**
 * A `methods` distance method (org.theseed.genome.distance.methods
 * .DistanceMethod) computing the kmer Jaccard distance on the GPU: the
 * drop-in for MethodTableProcessor's per-pair call
 * `methods.get(i).getDistance(measurer, genome2)` (MethodTableProcessor.java:275)
 * and its measurer cache per first genome (:261-265, getMeasurers :397-407).
 *
 * Registered where DistanceMethod.create(type) maps type names to classes
 * (MethodTableProcessor.java:178 calls it with the method file's first
 * column), e.g. type "kmer_gpu". Parameters (second column,
 * parseParmString, :179): "K=21" (kmer size), "type=DNA|PROT", "device=0".
 * toString() is the column header (:243) and must be stable for --previous
 * (:200-203): "KMER_GPU_K21".
 *
 * getDistance is called from the ForkJoin pool (one thread per method of a
 * pair); the context serialises device calls. The method keeps ONE genome
 * cache for the run: a device collection to which each genome is appended
 * the first time it is seen (gdist_sets_append, keyed by genome id), so a
 * genome is packed once however many pairs name it; GenomePairList.prepare
 * groups the pairs by id1 (:240), whose measurer holds id1's set. getDistance
 * is then one row query of id1's set against id2's cached set
 * (gdist_row_query): exact, the Java expression 1 - I / (|A| + |B| - I) in
 * fp64 on the device.
 */
public class GpuKmerMethod extends DistanceMethod {

    private int k = 21;
    private int kind = GpuKmerSets.DNA;
    private int device = 0;
    private GpuKmerSets.Context ctx;
    // the genome cache: one collection, genome id -> set index
    private GpuKmerSets cache;
    private final Map<String, Integer> setIndex = new HashMap<String, Integer>();

    @Override
    public void parseParmString(String parms) {
        Map<String, String> p = new HashMap<String, String>();
        if (parms != null)
            for (String kv : parms.split("[,\\s]+")) {
                int eq = kv.indexOf('=');
                if (eq > 0)
                    p.put(kv.substring(0, eq).trim(), kv.substring(eq + 1).trim());
            }
        if (p.containsKey("K"))
            this.k = Integer.parseInt(p.get("K"));
        if (p.containsKey("type"))
            this.kind = p.get("type").equalsIgnoreCase("PROT") ? GpuKmerSets.PROT : GpuKmerSets.DNA;
        if (p.containsKey("device"))
            this.device = Integer.parseInt(p.get("device"));
        if (this.k < 2)
            throw new IllegalArgumentException("Kmer size must be at least 2.");
    }

    synchronized GpuKmerSets.Context context() {
        if (this.ctx == null)
            this.ctx = new GpuKmerSets.Context(this.device);
        return this.ctx;
    }

    int kmerSize() { return this.k; }

    int kind() { return this.kind; }

    /** the set of a genome in the cache, packed and appended on first sight */
    synchronized int setOf(Genome genome) {
        Integer i = this.setIndex.get(genome.getId());
        if (i == null) {
            byte[][] seq = { GpuGenomeProcessor.contigBytes(genome) };
            if (this.cache == null) {
                this.cache = new GpuKmerSets(this.context(), this.kind, this.k, seq);
                i = 0;
            } else {
                i = (int) this.cache.append(seq);
            }
            this.setIndex.put(genome.getId(), i);
        }
        return i;
    }

    /** the distance of cached sets i and j (one device row query) */
    synchronized double distance(int i, int j) {
        double[] d = new double[1];
        this.cache.row(i, new long[] { j }, d);
        return d[0];
    }

    @Override
    public Measurer getMeasurer(Genome genome) {
        return new GpuMeasurer(this, genome);
    }

    @Override
    public double getDistance(Measurer measurer, Genome genome2) {
        return ((GpuMeasurer) measurer).distanceTo(genome2);
    }

    @Override
    public String toString() {
        return "KMER_GPU_K" + this.k + (this.kind == GpuKmerSets.PROT ? "_PROT" : "");
    }

    @Override
    public synchronized void close() {
        if (this.cache != null) {
            this.cache.close();
            this.cache = null;
            this.setIndex.clear();
        }
        if (this.ctx != null) {
            this.ctx.close();
            this.ctx = null;
        }
    }
}
