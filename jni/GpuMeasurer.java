package org.theseed.genome.distance.gpu;

import org.theseed.genome.Genome;
import org.theseed.genome.distance.methods.Measurer;

/**
 * The measurer of GpuKmerMethod for one first genome (MethodTableProcessor
 * .getMeasurers, :397-407): the genome's index in the method's genome cache
 * (packed there once, whatever the number of pairs it appears in).
 * distanceTo(genome2) is one row query of that set against genome2's cached
 * set (gdist_row_query): no packing per pair.
 */
public class GpuMeasurer extends Measurer {

    private final GpuKmerMethod method;
    private final int set1;

    GpuMeasurer(GpuKmerMethod method, Genome genome) {
        super(genome);
        this.method = method;
        this.set1 = method.setOf(genome);
    }

    double distanceTo(Genome genome2) {
        return this.method.distance(this.set1, this.method.setOf(genome2));
    }
}
