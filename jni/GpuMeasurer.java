package org.theseed.genome.distance.gpu;

import org.theseed.genome.Genome;
import org.theseed.genome.distance.methods.Measurer;

/**
 * The measurer of GpuKmerMethod for one first genome (MethodTableProcessor
 * .getMeasurers, :397-407): the genome's index in the method's genome cache
 * (packed there once, whatever the number of pairs it appears in) and, once
 * asked, its distances to every genome of the cache (one device call). A
 * later getDistance reads that row; a second genome appended to the cache
 * after the row was taken (its index past the row) takes the row again, and
 * a cache restarted since (GpuKmerMethod's bound) re-adds the first genome.
 */
public class GpuMeasurer extends Measurer {

    private final GpuKmerMethod method;
    private final Genome genome1;
    private int set1;
    private int gen;
    private double[] row;

    GpuMeasurer(GpuKmerMethod method, Genome genome) {
        super(genome);
        this.method = method;
        this.genome1 = genome;
        this.set1 = method.setOf(genome);
        this.gen = method.generation();
    }

    synchronized double distanceTo(Genome genome2) {
        if (this.gen != this.method.generation()) {
            this.set1 = this.method.setOf(this.genome1);
            this.gen = this.method.generation();
            this.row = null;
        }
        int j = this.method.setOf(genome2);
        if (this.row == null || j >= this.row.length)
            this.row = this.method.row(this.set1);
        return this.row[j];
    }
}
