package org.dma.sketchml.hip;

import org.dma.sketchml.sketch.base.Quantizer;
import org.dma.sketchml.sketch.common.Constants;

/**
 * Drop-in for quantization/QuantileQuantizer.java: the same Quantizer fields are filled
 * (binNum, n, splits, zeroIdx, min, max, bins), so Quantizer's own getValues / indexOf /
 * writeObject / readObject work unchanged; the sketch and the bins are computed on the GPU.
 * The compaction RNG is java.util.Random(seed) (the reference's static Random is unseeded).
 */
public class HipQuantileQuantizer extends Quantizer {
    private final long seed;

    public HipQuantileQuantizer(int binNum) {
        this(binNum, 0L);
    }

    public HipQuantileQuantizer(int binNum, long seed) {
        super(binNum);
        this.seed = seed;
    }

    @Override
    public void quantize(double[] values) {
        fill(HipCodec.encodeDenseF64(HipCodec.ctx(), values, binNum, true, seed, 1));  // with Maths.unique
    }

    @Override
    public void parallelQuantize(double[] values) {
        int threads = Constants.Parallel.getParallelism();  // "Parallelism is not set yet"
        fill(HipCodec.encodeDenseF64(HipCodec.ctx(), values, binNum, false, seed, threads));  // no dedup
    }

    private void fill(byte[] payload) {
        double[] info = HipCodec.info(payload);
        binNum = (int) info[0];
        n = (int) info[1];
        zeroIdx = (int) info[2];
        min = info[3];
        max = info[4];
        splits = new double[binNum - 1];
        System.arraycopy(info, 5, splits, 0, binNum - 1);
        bins = new int[n];
        HipCodec.getBins(payload, bins);
    }

    @Override
    public QuantizationType quantizationType() {
        return QuantizationType.QUANTILE;
    }
}
