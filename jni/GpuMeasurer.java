package org.theseed.genome.distance.gpu;

import org.theseed.genome.Genome;
import org.theseed.genome.distance.methods.Measurer;

/**
 * The measurer of GpuKmerMethod for one first genome (MethodTableProcessor
 * .getMeasurers, :397-407): it keeps the genome's contig bytes (joined by a
 * 0x00 byte, GpuGenomeProcessor.contigBytes) and answers distanceTo(genome2)
 * with one two-set pack and matrix call on the method's context.
 */
public class GpuMeasurer extends Measurer {

    private final GpuKmerMethod method;
    private final byte[] seq1;

    GpuMeasurer(GpuKmerMethod method, Genome genome) {
        super(genome);
        this.method = method;
        this.seq1 = GpuGenomeProcessor.contigBytes(genome);
    }

    double distanceTo(Genome genome2) {
        byte[][] both = { this.seq1, GpuGenomeProcessor.contigBytes(genome2) };
        double[] d = new double[2];
        try (GpuKmerSets pair = new GpuKmerSets(this.method.context(), this.method.kind(), this.method.kmerSize(),
                                                both)) {
            pair.distances(0, 1, 1, 2, false, d, 1);
        }
        return d[0];
    }
}
