package org.dma.sketchml.hip;

import org.dma.sketchml.sketch.base.BinaryEncoder;

/**
 * Same surface as binary/DeltaAdaptiveEncoder.java:13-189 (a BinaryEncoder over strictly
 * increasing int keys): the delta histogram, calOptimalIntervals, and the flag / delta bit
 * streams (BitSet.toLongArray words) computed on the GPU.  A non-increasing key raises
 * SketchMLException("Log for ...") as Maths.log2nlz does.
 */
public class HipDeltaAdaptiveEncoder implements BinaryEncoder {
    private int size;
    private int numIntervals;
    private boolean flagKind;
    private long[] flagWords = new long[0];
    private long[] deltaWords = new long[0];

    @Override
    public void encode(int[] values) {
        size = values.length;
        long[] r = HipCodec.deltaEncode(HipCodec.ctx(), values);
        numIntervals = (int) r[0];
        flagKind = r[1] != 0;
        int nf = (int) r[4], nd = (int) r[5];
        flagWords = new long[nf];
        deltaWords = new long[nd];
        System.arraycopy(r, 6, flagWords, 0, nf);
        System.arraycopy(r, 6 + nf, deltaWords, 0, nd);
    }

    @Override
    public int[] decode() {
        return HipCodec.deltaDecode(HipCodec.ctx(), size, numIntervals, flagKind, flagWords, deltaWords);
    }

    public int getNumIntervals() {
        return numIntervals;
    }

    public boolean getFlagKind() {
        return flagKind;
    }
}
